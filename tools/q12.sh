# count mode: tests + C5 timing quad vs wave (dev tool)
timeout -k 10 400 python -u -m pytest tests/test_gpu_solve.py tests/test_gpu_node.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
for s in quad wave; do timeout -k 10 120 python tools/c5_profile.py $s || exit 1; done
