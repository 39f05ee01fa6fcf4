#!/bin/bash
# round 4 box pass: donation-launch helpers per board (SDK_OPT_DONATE_HELPERS) on the bench's
# phased workloads: heavy 1000 (split 16), hard 100k (split 128), LEX and MRV-unique, two runs
set -o pipefail
out=gpurun_out/r04y
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for h in 1 2 4 8 16; do
  for o in lex mrv_unique; do
    for wl in "heavy 1000 16" "hard 100000 1"; do
      set -- $wl
      timeout -k 10 120 python -u tools/solve_profile.py --workload $1 --n $2 --reps 5 --solver quad --order $o \
        --donate $3 --donate-max 0 --helpers $h 2>&1 | grep rate | sed "s/^/h$h-$o /" >> $out/ab.log || exit 1
    done
  done
done
done
python3 tools/ab_table.py $out/ab.log
