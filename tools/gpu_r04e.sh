#!/bin/bash
# round 4 box pass: the hard sets (phase breakdown traces, split x mode and helper sweeps), the
# per-SIMD PMC of hard_1m and minimal, and the donation kernel on a GPU shared by two ranks.
set -o pipefail
out=gpurun_out/r04e
mkdir -p $out
export TMPDIR=/tmp
# the donation launch after the fence-free busy accounting, against round 3's kernel (lib_r03)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_donate.py > $out/pytest_donate.log 2>&1 \
  || { tail -30 $out/pytest_donate.log; exit 1; }
tail -1 $out/pytest_donate.log
for rep in 1 2 3; do
  for wl in "hard 100000 1" "heavy 1000 16"; do
    set -- $wl
    for v in base r03; do
      SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $1 \
        --n $2 --reps 5 --donate $3 --donate-max 0 2>&1 | sed "s/^/$v /" >> $out/ab_donate.log || { tail -5 $out/ab_donate.log; exit 1; }
      SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $1 \
        --n $2 --reps 5 --donate 0 2>&1 | sed "s/^/$v /" >> $out/ab_donate.log || { tail -5 $out/ab_donate.log; exit 1; }
    done
  done
done
cat $out/ab_donate.log
for wl in "hard 100000 1" "heavy 1000 16"; do
  set -- $wl
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OLDPWD/$out/trace_$1 -o run --output-format csv -- \
     python3 $OLDPWD/tools/solve_profile.py --workload $1 --n $2 --reps 5 --donate $3 --solver quad --donate-max 0 \
     > $OLDPWD/$out/trace_$1.log 2>&1) || { tail -20 $out/trace_$1.log; exit 1; }
  tail -1 $out/trace_$1.log
done
for n in 100000 1000000; do
  for dn in 0 32 64 128; do
    for mode in 1 0; do
      [ $dn = 0 ] && [ $mode = 0 ] && continue
      timeout -k 10 120 python tools/solve_profile.py --solver quad --workload hard --n $n --reps 5 --donate $dn \
        --donate-mode $mode --donate-max 0 >> $out/sweep_hard.log 2>&1 || { tail -5 $out/sweep_hard.log; exit 1; }
    done
  done
done
for n in 100000 1000000; do
  for order in lex mrv_unique; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload hard --n $n --reps 5 --donate 0       --order $order --stats >> $out/sweep_hard.log 2>&1 || { tail -5 $out/sweep_hard.log; exit 1; }
  done
done
cat $out/sweep_hard.log
for wl in "hard 100000 128" "heavy 1000 16"; do
  set -- $wl
  for h in 16 48 128; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $1 --n $2 --reps 5 --donate $3 \
      --donate-max 0 --helpers $h >> $out/sweep_helpers.log 2>&1 || { tail -5 $out/sweep_helpers.log; exit 1; }
  done
done
cat $out/sweep_helpers.log
timeout -k 10 400 bash tools/pmc_r04.sh $out/pmc hard1m min > $out/pmc.log 2>&1 || { tail -30 $out/pmc.log; exit 1; }
tail -4 $out/pmc.log
timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 \
  --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --hard-reps 1 > $out/bench_2rank_shared.json 2> $out/bench_2rank_shared.err \
  || { tail -30 $out/bench_2rank_shared.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench_2rank_shared.json'));print(json.dumps(d.get('hard_search'))[:1200])"
