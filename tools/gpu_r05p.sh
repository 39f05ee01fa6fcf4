#!/bin/bash
# round 5 box pass 16: kernel traces of the hard-search legs (phased LEX with donation, one launch, MRV)
set -o pipefail
out=gpurun_out/r05p
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
for cfg in "hard 100000 -1 lex" "hard 100000 0 lex" "hard 1000000 0 lex" "hard 1000000 0 mrv_unique" "hard 100000 -1 mrv_unique"; do
  set -- $cfg
  tag=$1_$2_dn$3_$4
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $root/$out/$tag -o run -- python3 $root/tools/solve_profile.py --solver quad --workload $1 --n $2 --reps 2 --donate $3 --order $4 > $root/$out/$tag.log 2>&1) || { tail -5 $out/$tag.log; exit 1; }
  tail -1 $out/$tag.log
done
