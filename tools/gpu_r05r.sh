#!/bin/bash
# round 5 box pass 18: byte-parallel scatter (parity), phased solves above 2^19 boards (DONATE_MAX 0 vs default)
set -o pipefail
out=gpurun_out/r05r
mkdir -p $out
timeout -k 10 300 python -u tools/prop32_check.py --quick > $out/prop32_check_quick.log 2>&1; rc=$?
grep -E "MISMATCH|hard|minimal" $out/prop32_check_quick.log | head -8
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for wl in hard:1000000 minimal:1048576 solve17:10000000 solve30:1000000 hard:100000; do
  w=${wl%%:*}; n=${wl##*:}
  for dm in -1 0; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --donate-max $dm >> $out/ab.log 2>&1 || { tail -3 $out/ab.log; exit 1; }
  done
done
done
cat $out/ab.log
