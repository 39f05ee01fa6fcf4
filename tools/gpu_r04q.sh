#!/bin/bash
# round 4 box pass: ticket-mapped segment dequeue (SDK_SOLVE4_TICKETS: 8-board chunks, then 4, then
# 2 at each segment's end) vs fixed chunks -- C4 10M / 1.25M / 2.5M / 5M, 30-clue, minimal, hard;
# the timeline of the ticket build; the solver GPU tests on it
set -o pipefail
out=gpurun_out/r04q
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for v in tk notk; do
  for wl in "solve17 10000000" "solve17 5000000" "solve17 2500000" "solve17 1250000" "solve30 1000000" "minimal 1048576" "hard 100000"; do
    set -- $wl
    SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/solve_profile.py --workload $1 \
      --n $2 --reps 5 --solver quad --donate 0 2>&1 | grep rate | sed "s/^/$v /" | tee -a $out/ab.log || exit 1
  done
done
done
SDK_LIB_PATH=$PWD/build/variants/lib_tltk.so timeout -k 10 180 python -u tools/timeline.py --sizes 1250000,10000000 \
  --json $out/timeline_tk.json > $out/timeline_tk.log 2>&1 || { tail -20 $out/timeline_tk.log; exit 1; }
python3 -c "
import json
for l in open('$out/timeline_tk.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['boards'], d['kernel_ms_hip_events'], 'lastdq', d['last_dequeue_us']['p50'], d['last_dequeue_us']['max'], 'exit', d['exit_us']['p50'], d['exit_us']['max'], 'drain', d['drain_us'])
"
SDK_LIB_PATH=$PWD/build/variants/lib_tk.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_solve.py > $out/pytest_tk.log 2>&1 || { tail -30 $out/pytest_tk.log; exit 1; }
tail -1 $out/pytest_tk.log
