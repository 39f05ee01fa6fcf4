#!/bin/bash
# round 5 box pass 19: phased-solve settings on the hard sets (prop32 fallback phased at any size)
set -o pipefail
out=gpurun_out/r05s
mkdir -p $out
for n in 100000 1000000; do
  for cfg in "lex 128 1" "lex 192 1" "lex 256 1" "lex 384 1" "mrv_unique 128 1" "mrv_unique 128 0" "mrv_unique 256 1" "mrv_unique 256 0" "mrv_unique 512 0" "mrv_unique 0 1"; do
    set -- $cfg
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload hard --n $n --reps 3 --order $1 --donate $2 --resume $3 >> $out/sweep.log 2>&1 || { tail -3 $out/sweep.log; exit 1; }
  done
done
cat $out/sweep.log
