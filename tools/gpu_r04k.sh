#!/bin/bash
# round 4 box pass: the phased heavy-1000 solve, three times per build (ticket give-back, the same
# without the donor's error-word read, the same without first-round statics, round 3), then one
# kernel trace each of the give-back build and round 3's (per-phase launch times)
set -o pipefail
out=gpurun_out/r04k
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2 3; do
for v in cas2 cas2e0 cas2nofresh r03; do
  SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/dn_diag.py --workload heavy --n 1000 \
    --budgets 0 --splits 16 2>&1 | sed "s/^/$v /" >> $out/dn_diag.log || { tail -20 $out/dn_diag.log; exit 1; }
done
done
grep " n=" $out/dn_diag.log | grep -v "donate=0"
for v in cas2 r03; do
  SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace -d $out/$v -o run -- \
    python3 -u tools/dn_diag.py --workload heavy --n 1000 --budgets 0 --splits 16 > $out/trace_$v.log 2>&1 \
    || { tail -20 $out/trace_$v.log; exit 1; }
done
