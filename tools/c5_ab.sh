# C5 count legs, in-tree library against build/variants/lib_prev.so (dev tool), plus the count tests
set -o pipefail
out=gpurun_out/c5ab; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_solve.py tests/test_gpu_frontier.py -x -q --timeout 120 \
  --timeout-method thread -k "count or frontier" > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
OFF="--batch 1024 --check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0"
for rep in 1 2; do
  for v in base prev; do
    lib=""; [ $v != base ] && lib=$PWD/build/variants/lib_$v.so
    env ${lib:+SDK_LIB_PATH=$lib} timeout -k 10 300 python3 bench.py $OFF > $out/bench_$v.json 2> $out/bench_$v.err || { tail -5 $out/bench_$v.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$out/bench_$v.json').read())
print('$v', 'c5', round(d['c5_count']['wall_ms'],2), 'ms', round(d['c5_count']['value']/1e6), 'M/s', 'rebal', round(d['c5_count_rebalanced']['wall_ms'],2), 'ms build', round(d['c5_count_rebalanced']['frontier_1m']['build_ms'],2), d['c5_count']['ok'], d['c5_count_rebalanced']['ok'])
"
  done
done
