#!/bin/bash
# (experiment record: the unaligned-read conversion was measured 8 % slower on C4 and reverted)
# round 5 box pass 39: prop32 triad conversion from one 4-byte read per board
out=gpurun_out/r05ar
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prop32.py -x -q --timeout 120 --timeout-method thread > $out/pytest_prop32.log 2>&1 || { tail -30 $out/pytest_prop32.log; exit 1; }
tail -1 $out/pytest_prop32.log
timeout -k 10 300 python -u tools/prop32_check.py --quick > $out/prop32_check_quick.log 2>&1 || { tail -20 $out/prop32_check_quick.log; exit 1; }
tail -1 $out/prop32_check_quick.log
for rep in 1 2; do
for wl in solve17:10000000 solve30:1000000 minimal:1048576 hard:1000000; do
  w=${wl%%:*}; n=${wl##*:}
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 >> $out/ab.log 2>&1 || exit 1
  SDK_LIB_PATH=$PWD/build/variants/lib_p32base.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 2>&1 | sed "s/^/base /" >> $out/ab.log || exit 1
done
done
grep -o "^\(base \)\?quad.*solve=[0-9.]* ms" $out/ab.log | sed 's/quad lex lc=1 xh=-1 dn=-1.-1.h0 chunk=0//'
