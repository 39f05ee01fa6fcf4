#!/bin/bash
# round 4 box pass: donation check interval (SDK_DN_EVERY: search nodes between a part's
# donation checks) on the phased heavy / hard solves, LEX and MRV-unique
set -o pipefail
out=gpurun_out/r04t
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for v in base every4 every8 every32; do
  for o in lex mrv_unique; do
    for wl in "heavy 1000 16" "hard 100000 1"; do
      set -- $wl
      SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/solve_profile.py --workload $1 \
        --n $2 --reps 5 --solver quad --order $o --donate $3 --donate-max 0 2>&1 | grep rate | sed "s/^/$v-$o /" >> $out/ab.log || exit 1
    done
  done
done
done
python3 tools/ab_table.py $out/ab.log
