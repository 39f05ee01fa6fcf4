#!/bin/bash
# (experiment record: SDK_OPT_PROP32_DEFER was measured and reverted -- see DESIGN.md "Regrouping, measured and dropped")
# round 5 box pass 35: regrouping (SDK_OPT_PROP32_DEFER) -- parity, then timing against no regrouping
set -o pipefail
out=gpurun_out/r05ae
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prop32.py -x -q --timeout 120 --timeout-method thread > $out/pytest_prop32.log 2>&1 || { tail -30 $out/pytest_prop32.log; exit 1; }
tail -1 $out/pytest_prop32.log
timeout -k 10 400 python -u tools/prop32_check.py --quick --variants default,nodefer,defer19x40,defer1x64 > $out/prop32_check_quick.log 2>&1 || { tail -20 $out/prop32_check_quick.log; exit 1; }
tail -1 $out/prop32_check_quick.log
for rep in 1 2; do
for wl in solve17:10000000 solve30:1000000 minimal:1048576 hard:1000000; do
  w=${wl%%:*}; n=${wl##*:}
  for d in 0 2056 10248 4872 5128; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --prop32-defer $d >> $out/ab.log 2>&1 || exit 1
  done
done
done
grep -o "d[0-9]* [a-z0-9]* n=[0-9]* solve=[0-9.]* ms" $out/ab.log
