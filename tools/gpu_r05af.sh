#!/bin/bash
# (experiment record: SDK_OPT_PROP32_DEFER was measured and reverted -- see DESIGN.md "Regrouping, measured and dropped")
# round 5 box pass 36: regrouping step statistics (SDK_PROP32_STATS build)
set -o pipefail
out=gpurun_out/r05af
mkdir -p $out
for wl in solve17:1000000 solve30:1000000; do
  w=${wl%%:*}; n=${wl##*:}
  for d in 0 10259 10248; do
    SDK_LIB_PATH=$PWD/build/variants/lib_p32stats.so timeout -k 10 120 python tools/prop32_stats.py --workload $w --n $n --defer $d >> $out/stats.log 2>&1 || { tail $out/stats.log; exit 1; }
  done
done
for d in 0 10259 5139 2581; do
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload solve17 --n 10000000 --reps 3 --prop32-defer $d >> $out/ab.log 2>&1 || exit 1
done
cat $out/stats.log; grep -o "d[0-9]* [a-z0-9]* n=[0-9]* solve=[0-9.]* ms" $out/ab.log
