#!/bin/bash
# round 5 box pass 21: split budget picked on the device from the searched-board count -- parity, timing
set -o pipefail
out=gpurun_out/r05u
mkdir -p $out
timeout -k 10 300 python -u tools/prop32_check.py --quick > $out/prop32_check_quick.log 2>&1; rc=$?
grep -E "MISMATCH" $out/prop32_check_quick.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for wl in hard:1000000 minimal:1048576 hard:100000 solve17:10000000; do
  w=${wl%%:*}; n=${wl##*:}
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 >> $out/ab.log 2>&1 || { tail -3 $out/ab.log; exit 1; }
done
done
cat $out/ab.log
