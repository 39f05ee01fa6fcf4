#!/bin/bash
# round 5 box pass 5: prop32 bring-up -- parity against the plain solver on every workload, timings
set -o pipefail
out=gpurun_out/r05e
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prop32_check.py --quick > $out/prop32_check_quick.log 2>&1; rc=$?
cat $out/prop32_check_quick.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/prop32_check.py > $out/prop32_check.log 2>&1; rc=$?
cat $out/prop32_check.log
exit $rc
