#!/bin/bash
# round 4 box pass: resumed split boards (SDK_OPT_DONATE_RESUME) -- the donation tests, the
# phased solves resumed vs restarted (heavy 1000, hard 100k, hard 1M; LEX and MRV-unique), and
# the plain kernel with and without the split-phase save compiled in (C4 10M, two pairs)
set -o pipefail
out=gpurun_out/r04m
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_donate.py \
  > $out/pytest_donate.log 2>&1 || { tail -40 $out/pytest_donate.log; exit 1; }
tail -1 $out/pytest_donate.log
for wl in "heavy 1000 16" "hard 100000 1" "hard 1000000 1"; do
  set -- $wl
  timeout -k 10 180 python -u tools/dn_diag.py --workload $1 --n $2 --budgets 0 --splits $3 --resume 1,0,1,0 \
    > $out/diag_$1_$2.log 2>&1 || { tail -20 $out/diag_$1_$2.log; exit 1; }
  grep " n=" $out/diag_$1_$2.log
done
for v in base nosave base nosave; do
  SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/solve_profile.py --workload solve17 \
    --n 10000000 --reps 5 --solver quad 2>&1 | grep rate | sed "s/^/$v /"
done
for o in lex mrv_unique; do
  for rs in 1 0; do
    timeout -k 10 120 python -u tools/solve_profile.py --workload hard --n 100000 --reps 5 --solver quad --order $o \
      --donate 1 --donate-max 0 --resume $rs 2>&1 | grep rate | sed "s/^/resume=$rs /"
  done
done
