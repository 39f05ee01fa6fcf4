#!/bin/bash
# round 5 box pass 9: prop32 without spills -- parity (quick) and A/B of 4 (in-tree) vs 5 waves per
# SIMD, LC every 3 / 4 steps, against prop32 off
set -o pipefail
out=gpurun_out/r05i
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prop32_check.py --quick > $out/prop32_check_quick.log 2>&1; rc=$?
cat $out/prop32_check_quick.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for wl in solve17:10000000 solve17:1250000 solve30:1000000 minimal:1048576; do
  w=${wl%%:*}; n=${wl##*:}
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 >> $out/ab.log 2>&1 || exit 1
  SDK_LIB_PATH=$PWD/build/variants/lib_p32w5.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 2>&1 | sed "s/^/w5 /" >> $out/ab.log || exit 1
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32-lc 3 >> $out/ab.log 2>&1 || exit 1
  SDK_LIB_PATH=$PWD/build/variants/lib_p32w5.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32-lc 3 2>&1 | sed "s/^/w5 /" >> $out/ab.log || exit 1
  [ $rep = 1 ] && { timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32 0 >> $out/ab.log 2>&1 || exit 1; }
done
done
cat $out/ab.log
