#!/bin/bash
# Headline C4 leg alone at 1 / 2 / 3 passes in flight, alternating (dev tool; run on the GPU box).
# usage: [BATCH=10000000] bash tools/ab_inflight.sh [reps]   -> one line per run: inflight, value, single-stream value
set -o pipefail
OFF="--check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --first-boards="
for rep in $(seq ${1:-2}); do
  for k in 1 2 3; do
    timeout -k 10 180 python bench.py $OFF --batch ${BATCH:-10000000} --steps ${STEPS:-3} --inflight $k > /tmp/abif.json 2>/tmp/abif.err || { tail -5 /tmp/abif.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('/tmp/abif.json').read().strip().splitlines()[-1])
print('batch', ${BATCH:-10000000}, 'inflight', $k, 'value %.4f G/s' % (d['value']/1e9), 'single %.4f G/s' % (d['single_stream']['value']/1e9), 'kernel %.4f ms' % d['single_stream']['avg_kernel_ms'], 'ms_per_step %.4f' % d['ms_per_step'])"
  done
done
