#!/bin/bash
# round 5 box pass 8: prop32 step algebra in asm, change bits before LC only -- parity (quick) and A/B
# of 5 (in-tree) vs 4 waves per SIMD, LC every 3/4/5 steps
set -o pipefail
out=gpurun_out/r05h
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prop32_check.py --quick > $out/prop32_check_quick.log 2>&1; rc=$?
cat $out/prop32_check_quick.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for wl in solve17:10000000 solve17:1250000 minimal:1048576; do
  w=${wl%%:*}; n=${wl##*:}
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 >> $out/ab.log 2>&1 || exit 1
  SDK_LIB_PATH=$PWD/build/variants/lib_p32w4.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 2>&1 | sed "s/^/w4 /" >> $out/ab.log || exit 1
  for lc in 3 5; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32-lc $lc >> $out/ab.log 2>&1 || exit 1
  done
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32 0 >> $out/ab.log 2>&1 || exit 1
done
done
cat $out/ab.log
