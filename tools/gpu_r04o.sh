#!/bin/bash
# round 4 box pass: wave-level dequeue pool (SDK_SOLVE4_WAVE_POOL) vs per-slot chunks, C4 at
# 10M / 1.25M, 30-clue 1M, minimal 1M, hard 100k; pool chunk sizes; then the solver GPU tests
set -o pipefail
out=gpurun_out/r04o
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for v in f1p0 f0p1 f1p1; do
  for wl in "solve17 10000000" "solve17 1250000" "solve30 1000000" "minimal 1048576" "hard 100000"; do
    set -- $wl
    SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/solve_profile.py --workload $1 \
      --n $2 --reps 5 --solver quad --donate 0 2>&1 | grep rate | sed "s/^/$v /" | tee -a $out/ab.log || exit 1
  done
done
done
for ch in 4 8 16; do
  for wl in "solve17 10000000" "solve17 1250000"; do
    set -- $wl
    SDK_LIB_PATH=$PWD/build/variants/lib_f0p1.so timeout -k 10 120 python -u tools/solve_profile.py --workload $1 \
      --n $2 --reps 5 --solver quad --donate 0 --chunk $ch 2>&1 | grep rate | sed "s/^/f0p1-ch$ch /" | tee -a $out/ab.log || exit 1
  done
done
SDK_LIB_PATH=$PWD/build/variants/lib_f0p1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_solve.py > $out/pytest_pool.log 2>&1 || { tail -30 $out/pytest_pool.log; exit 1; }
tail -1 $out/pytest_pool.log
