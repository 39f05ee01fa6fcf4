#!/bin/bash
# round 5 box pass 12: prop32 handover of propagated grids and tail handoff -- parity and timing
set -o pipefail
out=gpurun_out/r05l
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/prop32_check.py --quick --variants default,nohandover,tail4x12,tail8x12 > $out/prop32_check_quick.log 2>&1; rc=$?
cat $out/prop32_check_quick.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for wl in solve17:10000000 minimal:1048576 hard:1000000; do
  w=${wl%%:*}; n=${wl##*:}
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 >> $out/ab.log 2>&1 || exit 1
  [ $w = solve17 ] && continue
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32 0 >> $out/ab.log 2>&1 || exit 1
  for t in 1028 2060 3084; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32-tail $t >> $out/ab.log 2>&1 || exit 1
  done
done
done
cat $out/ab.log
