#!/bin/bash
# round 5 box pass 2: A/B of the round's register shapes (in-place cell update, fresh round on/off)
# against round 4's kernel, then the solver GPU tests on the in-tree build.
set -o pipefail
out=gpurun_out/r05b
mkdir -p $out
export TMPDIR=/tmp
REPS=2 VARIANTS="head ip st0 ipnf ip0" WORKLOADS="solve17:10000000 solve17:1250000 minimal:1048576 hard:100000" \
  timeout -k 10 900 bash tools/ab.sh > $out/ab_round_regs.log 2>&1 || { tail -20 $out/ab_round_regs.log; exit 1; }
sed -i 's/^quad /st quad /' $out/ab_round_regs.log
python3 tools/ab_table.py $out/ab_round_regs.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solve.py tests/test_gpu_donate.py \
  tests/test_gpu_frontier.py > $out/pytest_solve.log 2>&1 || { tail -30 $out/pytest_solve.log; exit 1; }
tail -3 $out/pytest_solve.log
