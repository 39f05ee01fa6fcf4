# A/B of the in-tree library against build/variants/lib_prev.so (the previous commit), plus the
# solver GPU tests and the launch timeline of the in-tree build (build/variants/lib_tl.so).
set -o pipefail
mkdir -p gpurun_out/abprev
timeout -k 10 300 python -u -m pytest tests/test_gpu_solve.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/abprev/pytest.log 2>&1 || { tail -20 gpurun_out/abprev/pytest.log; exit 1; }
tail -1 gpurun_out/abprev/pytest.log
rm -f gpurun_out/static/sweep.log
VARIANTS="${VARIANTS:-prev}" WORKLOADS="${WORKLOADS:-solve17:1250000 solve17:10000000 solve30:1000000 minimal:1048576 hard:100000}" \
  bash tools/sweep_static.sh > /dev/null || exit 1
cp gpurun_out/static/sweep.log gpurun_out/abprev/sweep.log
cat gpurun_out/abprev/sweep.log
SDK_LIB_PATH=$PWD/build/variants/lib_tl.so timeout -k 10 180 python3 tools/timeline.py --sizes 1250000 \
  --json gpurun_out/abprev/timeline.json > gpurun_out/abprev/timeline.log 2>&1 || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/abprev/timeline.json'))
for n, r in d.items():
    print(n, 'span', round(r['span_us']), 'first', {k: round(v) for k, v in r['first_boards_us'].items()}, 'exit', {k: round(v) for k, v in r['exit_us'].items()})
"
