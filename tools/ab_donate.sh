#!/bin/bash
# A/B of subtree donation (SDK_OPT_DONATE) on the GPU box (dev tool): solve_profile.py rates with
# donation on and off, per workload.   usage: bash tools/ab_donate.sh [workload:n ...]
set -o pipefail
for wl in ${*:-hard:1000000 hard:100000 minimal:2000000 solve17:10000000}; do
  w=${wl%%:*}; n=${wl##*:}
  for dn in 1 0; do
    timeout -k 10 180 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --donate $dn || exit 1
  done
done
