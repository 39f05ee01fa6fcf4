#!/bin/bash
# round 5 box pass 40: locked-candidates interval after the triad layout (3 / 4 / 5 / 6)
set -o pipefail
out=gpurun_out/r05ak
mkdir -p $out
for rep in 1 2; do
for wl in solve17:10000000 solve30:1000000 minimal:1048576; do
  w=${wl%%:*}; n=${wl##*:}
  for lc in 3 4 5 6; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32-lc $lc >> $out/ab.log 2>&1 || exit 1
  done
done
done
grep -o "p32=.*solve=[0-9.]* ms" $out/ab.log
