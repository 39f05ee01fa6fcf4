#!/bin/bash
# round 4 box pass: the size-dependent QUAD chunk rule (default) against chunk 8 (round 3's) on
# every solve workload of the bench
set -o pipefail
out=gpurun_out/r04v
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2 3; do
for ch in 0 8; do
  for wl in "solve17 10000000" "solve17 5000000" "solve17 2500000" "solve17 1250000" "solve30 1000000" "minimal 1048576" "hard 100000"; do
    set -- $wl
    timeout -k 10 120 python -u tools/solve_profile.py --workload $1 --n $2 --reps 5 --solver quad --donate 0 \
      --chunk $ch 2>&1 | grep rate | sed "s/^/ch$ch /" >> $out/ab.log || exit 1
  done
done
done
python3 tools/ab_table.py $out/ab.log
