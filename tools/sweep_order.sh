#!/bin/bash
# LEX vs MRV_UNIQUE order on the hard workloads (dev tool): rate, nodes and rounds per board.
set -o pipefail
for wl in ${*:-heavy:1000 heavy:10000 hard:100000 hard:1000000 minimal:2000000}; do w=${wl%%:*}; n=${wl##*:}
  for o in lex mrv_unique; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 --donate 0 --order $o --stats || exit 1
  done
done
