#!/bin/bash
# round 5 box pass 22-23: prop32 step changes -- parity, timing, LDS counters
set -o pipefail
out=gpurun_out/r05v
mkdir -p $out
timeout -k 10 300 python -u tools/prop32_check.py --quick > $out/prop32_check_quick.log 2>&1; rc=$?
grep -E "MISMATCH" $out/prop32_check_quick.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for wl in solve17:10000000 solve17:1250000 solve30:1000000 minimal:1048576; do
  w=${wl%%:*}; n=${wl##*:}
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 >> $out/ab.log 2>&1 || { tail -3 $out/ab.log; exit 1; }
done
done
cat $out/ab.log
timeout -k 10 600 bash tools/pmc_r04.sh $out/pmc c4 > $out/pmc.log 2>&1 || { tail -30 $out/pmc.log; exit 1; }
tail -2 $out/pmc.log
