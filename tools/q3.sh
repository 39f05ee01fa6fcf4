# quick solver check on the GPU box: solver tests + LC on/off timing and stats (dev tool)
mkdir -p gpurun_out/q3
timeout -k 10 400 python -u -m pytest tests/test_gpu_solve.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q3/pytest.log 2>&1 || { tail -30 gpurun_out/q3/pytest.log; exit 1; }
tail -3 gpurun_out/q3/pytest.log
for lc in 1 0; do
  for w in solve17 minimal; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --locked $lc --workload $w --n 4000000 --reps 3 --stats || exit 1
  done
done
