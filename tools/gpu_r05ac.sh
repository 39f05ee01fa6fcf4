#!/bin/bash
# round 5 box pass 33: the whole GPU suite, smoke, the hard 1M kernel breakdown, and the default bench
set -o pipefail
out=gpurun_out/r05ac
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/hard1m -o run -- python3 $root/tools/solve_profile.py --solver quad --workload hard --n 1000000 --reps 5 --donate 1 --donate-max 0 > $root/$out/hard1m.log 2>&1) || { tail -20 $out/hard1m.log; exit 1; }
grep "rate=" $out/hard1m.log
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
h=r['hard_search']
print('value', round(r['value']/1e9,3), 'single', round(r['single_stream']['value']/1e9,3), 'kernel_ms', round(r['roofline']['avg_kernel_ms'],3), 'c2', round(r['c2_30clue']['value']/1e9,3), 'min', round(r['minimal_puzzles']['value']/1e6,1), 'checker', r['checker_summary']['frac'])
for k in ('hard_100k','hard_1m'): print('   ', k, {m: round(h[k][m]['value']/1e6,1) for m in ('donation','donation_in_flight') if m in h[k]})
"
