#!/bin/bash
# round 4 box pass: split budget x helpers (1, 2) on hard 100k / heavy 1000 / hard 1M phased,
# LEX and MRV-unique, against one launch
set -o pipefail
out=gpurun_out/r04z
mkdir -p $out
export TMPDIR=/tmp
for o in lex mrv_unique; do
  timeout -k 10 120 python -u tools/solve_profile.py --workload hard --n 100000 --reps 5 --solver quad --order $o \
    --donate 0 2>&1 | grep rate | sed "s/^/one-$o /" >> $out/ab.log || exit 1
  timeout -k 10 120 python -u tools/solve_profile.py --workload hard --n 1000000 --reps 5 --solver quad --order $o \
    --donate 0 2>&1 | grep rate | sed "s/^/one-$o /" >> $out/ab.log || exit 1
  for h in 1 2; do
    for sp in 32 64 128 256; do
      for n in 100000 1000000; do
        timeout -k 10 120 python -u tools/solve_profile.py --workload hard --n $n --reps 5 --solver quad --order $o \
          --donate $sp --donate-max 0 --helpers $h 2>&1 | grep rate | sed "s/^/sp$sp-h$h-$o /" >> $out/ab.log || exit 1
      done
    done
    for sp in 8 16 32; do
      timeout -k 10 120 python -u tools/solve_profile.py --workload heavy --n 1000 --reps 5 --solver quad --order $o \
        --donate $sp --donate-max 0 --helpers $h 2>&1 | grep rate | sed "s/^/sp$sp-h$h-$o /" >> $out/ab.log || exit 1
    done
  done
done
awk '{for(i=1;i<=NF;i++){if($i ~ /^solve=/) ms=$i; if($i ~ /^n=/) n=$i}; print $1, n, ms}' $out/ab.log
