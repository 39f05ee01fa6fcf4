#!/bin/bash
# Two-phase solve sweep on the GPU box (dev tool): split budget (SDK_OPT_DONATE value) per
# workload, for the in-tree library and the kDnEvery variants built with
#   tools/build_variant.sh dnev<K> -DSDK_DN_EVERY=<K>
# usage: VARIANTS="dnev16 dnev32" bash tools/sweep_split.sh [workload:n ...]
set -o pipefail
for wl in ${*:-hard:100000 hard:1000000 minimal:2000000}; do
  w=${wl%%:*}; n=${wl##*:}
  for dn in 0 16 32 64 128 256; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --donate $dn || exit 1
    for v in ${VARIANTS:-}; do
      [ $dn = 0 ] && continue
      SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad \
        --workload $w --n $n --reps 3 --donate $dn 2>&1 | sed "s/^/$v /" || exit 1
    done
  done
done
