#!/bin/bash
# round 4, third box pass: the statics-in-first-round variant (SDK_SOLVE4_FRESH_ROUND=1) --
# parity of the solver tests on that library, then an A/B against the in-tree build.
set -o pipefail
out=gpurun_out/r04c
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
SDK_LIB_PATH=$PWD/build/variants/lib_fresh.so timeout -k 10 600 $T tests/test_gpu_solve.py tests/test_gpu_donate.py tests/test_gpu_frontier.py \
  > $out/pytest_fresh.log 2>&1 || { tail -30 $out/pytest_fresh.log; exit 1; }
tail -2 $out/pytest_fresh.log
VARIANTS="fresh" WORKLOADS="solve17:10000000 solve17:1250000 solve30:1000000 minimal:1048576 hard:100000" REPS=3 EXTRA="--donate 0" \
  timeout -k 10 700 bash tools/ab.sh > $out/ab_fresh.log 2>&1 || { tail -30 $out/ab_fresh.log; exit 1; }
cat $out/ab_fresh.log
# phase breakdown of the phased solve on the hard sets (kernel trace: split phase, collect,
# donation launches, scatter)
for wl in "hard 100000 1" "heavy 1000 16"; do
  set -- $wl
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OLDPWD/$out/trace_$1 -o run --output-format csv -- \
     python3 $OLDPWD/tools/solve_profile.py --workload $1 --n $2 --reps 5 --donate $3 --solver quad --donate-max 0 \
     > $OLDPWD/$out/trace_$1.log 2>&1) || { tail -20 $out/trace_$1.log; exit 1; }
  cat $out/trace_$1.log | tail -2
done
# split budget x donation mode on the hard sets (phased solve at any size)
for n in 100000 1000000; do
  for dn in 0 32 64 128; do
    for mode in 1 0; do
      [ $dn = 0 ] && [ $mode = 0 ] && continue
      timeout -k 10 120 python tools/solve_profile.py --solver quad --workload hard --n $n --reps 5 --donate $dn \
        --donate-mode $mode --donate-max 0 >> $out/sweep_hard.log 2>&1 || { tail -5 $out/sweep_hard.log; exit 1; }
    done
  done
done
cat $out/sweep_hard.log
# donation-launch waves per tail board (SDK_OPT_DONATE_HELPERS)
for wl in "hard 100000 128" "heavy 1000 16"; do
  set -- $wl
  for h in 16 48 128; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $1 --n $2 --reps 5 --donate $3 \
      --donate-max 0 --helpers $h >> $out/sweep_helpers.log 2>&1 || { tail -5 $out/sweep_helpers.log; exit 1; }
  done
done
cat $out/sweep_helpers.log
