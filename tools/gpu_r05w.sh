#!/bin/bash
# round 5 box pass 24: prop32 at 3 / 4 (in-tree) / 5 waves per SIMD
set -o pipefail
out=gpurun_out/r05w
mkdir -p $out
for rep in 1 2; do
for wl in solve17:10000000 solve30:1000000 minimal:1048576; do
  w=${wl%%:*}; n=${wl##*:}
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 >> $out/ab.log 2>&1 || exit 1
  for v in p32w5 p32w3; do
    SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 2>&1 | sed "s/^/$v /" >> $out/ab.log || exit 1
  done
done
done
cat $out/ab.log
