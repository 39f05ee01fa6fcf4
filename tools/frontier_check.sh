# Frontier GPU tests and build timing (dev tool)
set -o pipefail
out=gpurun_out/frontier2; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_solve.py -x -q --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for s in quad halfwave; do
  timeout -k 10 120 python3 tools/frontier_levels.py $s > $out/levels_$s.log 2>&1 || { tail -5 $out/levels_$s.log; exit 1; }
  cat $out/levels_$s.log
done
