#!/bin/bash
# round 5 box pass 20: prop32 step statistics for longer LC intervals, and timing of each
set -o pipefail
out=gpurun_out/r05t
mkdir -p $out
for wl in solve17:1000000 solve30:1000000 minimal:262144 hard:65536; do
  w=${wl%%:*}; n=${wl##*:}
  for lc in 4 6 8 12; do
    SDK_LIB_PATH=$PWD/build/variants/lib_p32stats.so timeout -k 10 120 python tools/prop32_stats.py --workload $w --n $n --lc $lc >> $out/stats.log 2>&1 || { cat $out/stats.log; exit 1; }
  done
done
for wl in solve17:10000000 solve30:1000000 minimal:1048576; do
  w=${wl%%:*}; n=${wl##*:}
  for lc in 4 6 8; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32-lc $lc >> $out/ab.log 2>&1 || exit 1
  done
done
grep -E "^\S|steps  |lc_pass" $out/stats.log
cat $out/ab.log
