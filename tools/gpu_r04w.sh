#!/bin/bash
# round 4 box pass: where a phased hard-100k solve spends its time at split budgets 16..128
# (per-launch kernel trace: split phase, collect, donation launch, LEX re-solve, scatter)
set -o pipefail
out=gpurun_out/r04w
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- \
  python3 -u tools/dn_diag.py --workload hard --n 100000 --budgets 0 --splits 16,32,64,128 > $out/diag.log 2>&1 \
  || { tail -20 $out/diag.log; exit 1; }
grep " n=\|ctl" $out/diag.log
python3 tools/trace_phases.py $out trace
