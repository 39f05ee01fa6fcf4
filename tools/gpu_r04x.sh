#!/bin/bash
# round 4 box pass: donation-launch helpers per board (SDK_OPT_DONATE_HELPERS) at split budgets
# 16..128 on the hard 100k batch -- is the donation launch slowed by its idle waves?
set -o pipefail
out=gpurun_out/r04x
mkdir -p $out
export TMPDIR=/tmp
for sp in 16 32 64 128; do
  for h in 16 4 1; do
    timeout -k 10 120 python -u tools/solve_profile.py --workload hard --n 100000 --reps 5 --solver quad \
      --donate $sp --donate-max 0 --helpers $h 2>&1 | grep rate | sed "s/^/sp$sp-h$h /" >> $out/ab.log || exit 1
  done
done
cat $out/ab.log | sed 's/quad lex lc=1 xh=-1 //'
