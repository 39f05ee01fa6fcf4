#!/bin/bash
# Checker leg alone, in-tree library against build/variants/lib_<v>.so, alternating (dev tool; GPU box).
# usage: VARIANTS="head" bash tools/ab_checker.sh [reps]   -> per run: library, timed kernel ms, fraction of 8 TB/s
set -o pipefail
OFF="--batch 1024 --c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --first-boards="
for rep in $(seq ${1:-3}); do
  for v in intree ${VARIANTS:-}; do
    if [ $v = intree ]; then unset SDK_LIB_PATH; else export SDK_LIB_PATH=$PWD/build/variants/lib_$v.so; fi
    timeout -k 10 180 python bench.py $OFF > /tmp/abck.json 2>/tmp/abck.err || { tail -5 /tmp/abck.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('/tmp/abck.json').read().strip().splitlines()[-1]); c=d['checker_summary']
print('$v', 'kernel %.4f ms' % c['avg_kernel_ms'], 'frac %.4f' % c['frac'], 'mismatched', c['mismatched_boards'])"
  done
done
