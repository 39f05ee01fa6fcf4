#!/bin/bash
# Phased solve with donation vs one launch on the hard workloads (dev tool): split budget x
# donation mode.   usage: bash tools/sweep_heavy.sh [workload:n ...]
set -o pipefail
for wl in ${*:-heavy:1000 heavy:10000 hard:100000 hard:1000000 minimal:2000000}; do w=${wl%%:*}; n=${wl##*:}
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --donate 0 || exit 1
  for dn in 16 64 256; do for mode in 1 0; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --donate $dn --donate-mode $mode || exit 1
  done; done
done
