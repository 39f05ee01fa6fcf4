#!/bin/bash
# round 4 box pass: donation-launch grid = boards / 4 + 64 + helpers x min(boards, cap), cap
# 64 / 256 / none, at split budgets 32 / 64 / 128 on hard 100k and heavy 1000 (LEX), two runs
set -o pipefail
out=gpurun_out/r04ad
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for v in cap64 cap256 cap100000; do
  for sp in 32 64 128; do
    SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/solve_profile.py --workload hard \
      --n 100000 --reps 5 --solver quad --donate $sp --donate-max 0 2>&1 | grep rate | sed "s/^/$v-sp$sp /" >> $out/ab.log || exit 1
  done
  SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/solve_profile.py --workload heavy \
    --n 1000 --reps 5 --solver quad --donate 16 --donate-max 0 2>&1 | grep rate | sed "s/^/$v-sp16 /" >> $out/ab.log || exit 1
done
done
awk '{for(i=1;i<=NF;i++){if($i ~ /^solve=/) ms=$i; if($i ~ /^n=/) n=$i}; print $1, n, ms}' $out/ab.log | sort
