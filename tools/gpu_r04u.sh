#!/bin/bash
# round 4 box pass: dequeue chunk (SDK_OPT_SOLVE_CHUNK) by batch size on the default build --
# a size rule for small shards
set -o pipefail
out=gpurun_out/r04u
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for ch in 2 3 4 6 8; do
  for n in 1250000 2500000 5000000 10000000; do
    timeout -k 10 120 python -u tools/solve_profile.py --workload solve17 --n $n --reps 5 --solver quad --donate 0 \
      --chunk $ch 2>&1 | grep rate | sed "s/^/ch$ch /" >> $out/ab.log || exit 1
  done
done
done
python3 tools/ab_table.py $out/ab.log
