#!/bin/bash
# round 5 box pass 10: prop32 with bit-transposed input conversion and digit extraction -- parity and timing
set -o pipefail
out=gpurun_out/r05j
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prop32_check.py --quick > $out/prop32_check_quick.log 2>&1; rc=$?
cat $out/prop32_check_quick.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for wl in solve17:10000000 solve17:1250000 solve30:1000000 minimal:1048576; do
  w=${wl%%:*}; n=${wl##*:}
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 >> $out/ab.log 2>&1 || exit 1
done
done
cat $out/ab.log
