#!/bin/bash
# round 4 box pass: donation diagnostics (per-launch times, participating grid) of the current
# kernel beside round 3's, then the whole -m gpu suite on the new default build.
set -o pipefail
out=gpurun_out/r04i
mkdir -p $out
export TMPDIR=/tmp
for v in base r03; do
  for wl in "heavy 1000 16" "hard 100000 1"; do
    set -- $wl
    SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/dn_diag.py --workload $1 --n $2 \
      --budgets 0 --splits $3 2>&1 | sed "s/^/$v /" >> $out/dn_diag.log || { tail -20 $out/dn_diag.log; exit 1; }
  done
done
grep -v "^.*nodes/\|rounds/" $out/dn_diag.log | head -60
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $out/pytest_gpu.log 2>&1 \
  || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
