#!/bin/bash
# round 5 box pass 32: kernel breakdown of the hard 1M solve (prop32 pass + phased search), one pass at a time
set -o pipefail
out=gpurun_out/r05ab
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/$out/hard1m -o run -- python3 $root/tools/solve_profile.py --solver quad --workload hard --n 1000000 --reps 5 --donate 1 --donate-max 0 > $root/$out/hard1m.log 2>&1) || { tail -20 $out/hard1m.log; exit 1; }
tail -3 $out/hard1m.log
f=$(find $out/hard1m -name "*kernel_stats.csv" | head -1)
cp $f $out/hard1m_kernel_stats.csv
python3 - "$out/hard1m_kernel_stats.csv" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms total', r['Percentage'])
PY
