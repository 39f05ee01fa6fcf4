#!/bin/bash
# round 4 box pass: the plain kernel after removing the measured-and-dropped dequeue variants
# (clean) against the build before (base): every solve workload, two runs; solver GPU tests on it
set -o pipefail
out=gpurun_out/r04ae
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for v in base clean; do
  for wl in "solve17 10000000" "solve17 1250000" "solve30 1000000" "minimal 1048576" "hard 100000"; do
    set -- $wl
    SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/solve_profile.py --workload $1 \
      --n $2 --reps 5 --solver quad --donate 0 2>&1 | grep rate | sed "s/^/$v /" >> $out/ab.log || exit 1
  done
done
done
python3 tools/ab_table.py $out/ab.log
