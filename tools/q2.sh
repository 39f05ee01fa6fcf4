# quick solver check on the GPU box: quad parity tests + timing (dev tool)
mkdir -p gpurun_out/q2
timeout -k 10 300 python -u -m pytest tests/test_gpu_solve.py -x -q --timeout 120 --timeout-method thread -k "quad or identical" > gpurun_out/q2/pytest.log 2>&1; tail -3 gpurun_out/q2/pytest.log
for s in quad halfwave; do timeout -k 10 120 python tools/solve_profile.py --solver $s --n 4000000 --reps 3; done
for v in ${VARIANTS:-}; do SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad --n 4000000 --reps 3 2>&1 | sed "s/^/$v /"; done
for o in ${ORDERS:-}; do for w in solve17 minimal; do timeout -k 10 120 python tools/solve_profile.py --solver quad --order $o --workload $w --n 4000000 --reps 3 --stats; done; done
