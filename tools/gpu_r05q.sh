#!/bin/bash
# round 5 box pass 17: split-budget sweep of the phased solve on the hard sets, prop32 in front
set -o pipefail
out=gpurun_out/r05q
mkdir -p $out
for rep in 1 2; do
for n in 100000 1000000; do
  for dn in 0 16 32 64 128; do
    for o in lex mrv_unique; do
      timeout -k 10 120 python tools/solve_profile.py --solver quad --workload hard --n $n --reps 2 --donate $dn --donate-max 0 --order $o >> $out/sweep.log 2>&1 || { tail -3 $out/sweep.log; exit 1; }
    done
  done
done
done
cat $out/sweep.log
