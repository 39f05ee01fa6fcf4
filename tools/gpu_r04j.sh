#!/bin/bash
# round 4 box pass: donation diagnostics (per-launch times, participating grid) of the current
# kernel's ticket modes (SDK_DN_CAS 1 / 0 / 2) beside round 3's, twice.
set -o pipefail
out=gpurun_out/r04j
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for v in base cas0 cas2 r03; do
  for wl in "heavy 1000 16" "hard 100000 1"; do
    set -- $wl
    SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/dn_diag.py --workload $1 --n $2 \
      --budgets 0 --splits $3 2>&1 | sed "s/^/$v /" >> $out/dn_diag.log || { tail -20 $out/dn_diag.log; exit 1; }
  done
done
done
grep " n=" $out/dn_diag.log | grep -v "donate=0"
