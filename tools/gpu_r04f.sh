#!/bin/bash
# round 4 box pass: which round-4 change slowed the donation launch (one macro off at a time),
# LEX vs MRV-unique order across the workloads, and the statics-in-first-round build again.
set -o pipefail
out=gpurun_out/r04f
mkdir -p $out
export TMPDIR=/tmp
P="python tools/solve_profile.py --solver quad"
for rep in 1 2; do
  for wl in "heavy 1000 16" "hard 100000 1"; do
    set -- $wl
    for v in base cas0 err0 wait0 all0 r03; do
      SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 $P --workload $1 --n $2 --reps 5 --donate $3 \
        --donate-max 0 2>&1 | sed "s/^/$v /" >> $out/bisect.log || { tail -5 $out/bisect.log; exit 1; }
    done
  done
done
cat $out/bisect.log
for rep in 1 2; do
  for wl in solve17:10000000 solve17:1250000 minimal:1048576 hard:100000 hard:1000000; do
    w=${wl%%:*}; n=${wl##*:}
    for order in lex mrv_unique; do
      timeout -k 10 120 $P --workload $w --n $n --reps 3 --order $order >> $out/order.log 2>&1 || { tail -5 $out/order.log; exit 1; }
    done
    SDK_LIB_PATH=$PWD/build/variants/lib_fresh.so timeout -k 10 120 $P --workload $w --n $n --reps 3 2>&1 | sed "s/^/fresh /" \
      >> $out/order.log || { tail -5 $out/order.log; exit 1; }
  done
done
cat $out/order.log
