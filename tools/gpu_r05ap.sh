#!/bin/bash
# round 5 box pass 44: the final tree -- GPU suite, smoke, rocprof stats of the C3/C4 commands, default
# bench; then the headline with three passes in flight for comparison
set -o pipefail
bash tools/gpu_round.sh r05ap tests prof_c3 prof_c4 bench > gpurun_out/r05ap.log 2>&1 || { tail -30 gpurun_out/r05ap.log; exit 1; }
tail -2 gpurun_out/r05ap/pytest_gpu.log
timeout -k 10 300 python -u bench.py --inflight 3 --check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 \
  --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 > gpurun_out/r05ap/bench_inflight3.json 2> gpurun_out/r05ap/bench_inflight3.err || { tail -20 gpurun_out/r05ap/bench_inflight3.err; exit 1; }
python3 -c "
import json
for f in ('bench.json','bench_inflight3.json'):
    r=json.loads(open('gpurun_out/r05ap/'+f).read().strip().splitlines()[-1])
    print(f, round(r['value']/1e9,3), round(r['single_stream']['value']/1e9,3), r['single_stream']['avg_kernel_ms'], r['roofline']['traffic'], r.get('checker_summary',{}).get('frac'))
"
