#!/bin/bash
# round 4 box pass: LEX vs MRV-unique as the default order, every solve workload of the bench
# (one launch), two runs
set -o pipefail
out=gpurun_out/r04ab
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for o in lex mrv_unique; do
  for wl in "solve17 10000000" "solve17 1250000" "solve30 1000000" "minimal 1048576" "hard 100000" "hard 1000000"; do
    set -- $wl
    timeout -k 10 120 python -u tools/solve_profile.py --workload $1 --n $2 --reps 5 --solver quad --order $o \
      --donate 0 2>&1 | grep rate | sed "s/^/$o /" >> $out/ab.log || exit 1
  done
done
done
python3 tools/ab_table.py $out/ab.log
