#!/bin/bash
# round 4 box pass: the shared dequeue tail's chunk (SDK_SOLVE4_TAIL_CHUNK_DIV) and size
# (SDK_SOLVE4_TAIL_DIV) -- the boards handed out last set the launch drain; C4 at 10M / 5M /
# 2.5M / 1.25M, 30-clue, minimal, hard; the timeline of the 2-board tail build
set -o pipefail
out=gpurun_out/r04r
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for v in tc8 tc2 tc1 tc2d64 tc1d256; do
  for wl in "solve17 10000000" "solve17 5000000" "solve17 2500000" "solve17 1250000" "solve30 1000000" "minimal 1048576" "hard 100000"; do
    set -- $wl
    SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/solve_profile.py --workload $1 \
      --n $2 --reps 5 --solver quad --donate 0 2>&1 | grep rate | sed "s/^/$v /" >> $out/ab.log || exit 1
  done
done
done
python3 tools/ab_table.py $out/ab.log
SDK_LIB_PATH=$PWD/build/variants/lib_tltc2.so timeout -k 10 180 python -u tools/timeline.py --sizes 1250000,10000000 \
  --json $out/timeline_tc2.json > $out/timeline_tc2.log 2>&1 || { tail -20 $out/timeline_tc2.log; exit 1; }
python3 -c "
import json
for l in open('$out/timeline_tc2.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['boards'], d['kernel_ms_hip_events'], 'lastdq', d['last_dequeue_us']['p50'], d['last_dequeue_us']['max'], 'exit', d['exit_us']['p50'], d['exit_us']['max'], 'drain', d['drain_us'])
"
