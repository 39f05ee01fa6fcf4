# solver tests + default vs variants timing (dev tool)
mkdir -p gpurun_out/q5
timeout -k 10 400 python -u -m pytest tests/test_gpu_solve.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q5/pytest.log 2>&1 || { tail -30 gpurun_out/q5/pytest.log; exit 1; }
tail -2 gpurun_out/q5/pytest.log
for w in solve17 minimal; do
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n 4000000 --reps 3 || exit 1
  for v in ${VARIANTS:-}; do SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n 4000000 --reps 3 2>&1 | sed "s/^/$v /" || exit 1; done
done
