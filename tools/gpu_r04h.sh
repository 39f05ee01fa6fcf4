#!/bin/bash
# round 4 box pass: per-kernel trace of the phased heavy solve (split / collect / donation / LEX /
# scatter launches) for the current build, the same without first-round statics, and round 3's;
# then the whole -m gpu suite on the default build.
set -o pipefail
out=gpurun_out/r04h
mkdir -p $out
export TMPDIR=/tmp
for v in base nofresh r03; do
  SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/$v -o run -- \
    python3 -u tools/dn_diag.py --workload heavy --n 1000 --budgets 0 --splits 16 > $out/diag_$v.log 2>&1 \
    || { tail -20 $out/diag_$v.log; exit 1; }
  grep -v "nodes/\|rounds/" $out/diag_$v.log | sed "s/^/$v /"
done
python3 tools/trace_phases.py $out base nofresh r03 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $out/pytest_gpu.log 2>&1 \
  || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
