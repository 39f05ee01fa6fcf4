#!/bin/bash
# round 5 box pass 43: C4 traffic of the no-scratch prop32 build, and the headline with two vs three
# passes in flight, alternated
set -o pipefail
bash tools/pmc_c4.sh gpurun_out/r05an/c4 > gpurun_out/r05an_pmc_c4.log 2>&1 || { tail -20 gpurun_out/r05an_pmc_c4.log; exit 1; }
grep "^sdk::prop32" gpurun_out/r05an_pmc_c4.log | cut -c1-400
for rep in 1 2 3; do
for k in 2 3; do
timeout -k 10 300 python -u bench.py --inflight $k --check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 \
  --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 > gpurun_out/r05an/b.json 2> gpurun_out/r05an/b.err || { tail -20 gpurun_out/r05an/b.err; exit 1; }
python3 -c "
import json; r=json.loads(open('gpurun_out/r05an/b.json').read().strip().splitlines()[-1]); print('inflight $k', round(r['value']/1e9,3), round(r['single_stream']['value']/1e9,3))" | tee -a gpurun_out/r05an/inflight.log
done
done
