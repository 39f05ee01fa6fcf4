#!/bin/bash
# round 5 box pass 29: hard legs in flight (3) under prop32 / search knobs
set -o pipefail
out=gpurun_out/r05z
mkdir -p $out
for opts in "" "--opt PROP32_TAIL=1028" "--opt PROP32_LC=3" "--opt PROP32_TAIL=2060"; do
timeout -k 10 600 python -u bench.py --check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 --count-leg 0 --lane-puzzles 0 \
  --cpu-seconds 0 --http-requests 0 $opts > $out/bench_hard.json 2> $out/bench_hard.err || { tail -20 $out/bench_hard.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$out/bench_hard.json').read().strip().splitlines()[-1])
h=r['hard_search']
for k in ('hard_100k','hard_1m'): print('$opts', k, {m: round(h[k][m]['value']/1e6,1) for m in ('donation','donation_in_flight') if m in h[k]}, h['parity'])
"
done
