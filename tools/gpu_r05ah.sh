#!/bin/bash
# round 5 box pass 37: hard legs in flight -- split budget and passes in flight
set -o pipefail
out=gpurun_out/r05ah
mkdir -p $out
i=0
for opts in "--hard-inflight 3" "--hard-inflight 3 --hard-split-inflight 512" "--hard-inflight 4 --hard-split-inflight 512" "--hard-inflight 3 --hard-split-inflight 1024" "--hard-inflight 4"; do
i=$((i+1))
timeout -k 10 600 python -u bench.py --check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 --count-leg 0 --lane-puzzles 0 \
  --cpu-seconds 0 --http-requests 0 $opts > $out/bench_$i.json 2> $out/bench_$i.err || { tail -20 $out/bench_$i.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$out/bench_$i.json').read().strip().splitlines()[-1])
h=r['hard_search']
for k in ('hard_100k','heaviest_1000','hard_1m'): print('$opts', k, {m: round(h[k][m]['value']/1e6,2) for m in ('donation','donation_in_flight') if m in h[k]}, h['parity']['mismatched_boards'])
"
done
