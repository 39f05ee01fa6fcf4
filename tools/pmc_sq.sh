#!/bin/bash
# One rocprofv3 PMC pass (<= 8 SQ counters) over tools/solve_profile.py's 4M 17-clue solve4 launches
# (dev tool).  usage: tools/pmc_sq.sh <outdir> "<counters>"   then: python3 tools/pmc_sq_sum.py <outdir>
set -o pipefail
out=$1; ctr=$2; root=$(pwd); mkdir -p "$out"; export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$root/$out" -o run -- \
   python3 "$root/tools/solve_profile.py" --solver quad --n 4000000 --reps 2 > "$root/$out/pass.log" 2>&1) \
  || { echo "pass failed"; tail -5 "$out/pass.log"; exit 1; }
python3 "$root/tools/pmc_sq_sum.py" "$out"
