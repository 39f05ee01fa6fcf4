#!/bin/bash
# round 5 box pass 14: the prop32 roofline evidence -- PMC pipe/LDS and traffic passes of the bench's C4
# launch, kernel trace + stats, then the default bench with them in place
set -o pipefail
out=gpurun_out/r05n
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
timeout -k 10 600 bash tools/pmc_r04.sh $out/pmc c4 > $out/pmc.log 2>&1 || { tail -30 $out/pmc.log; exit 1; }
tail -3 $out/pmc.log
timeout -k 10 900 bash tools/pmc_c4.sh $out/traffic > $out/traffic.log 2>&1 || { tail -30 $out/traffic.log; exit 1; }
grep -E "^sdk::prop32|^sdk::check" $out/traffic.log | cut -c1-400
mkdir -p profiles/r05
cp $out/pmc/pmc_pipe.json profiles/r05/pmc_pipe.json
cp $out/traffic/pmc_c4.json profiles/r05/pmc_c4.json
OFF="--c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --check-boards 0"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/prof_c4 -o run -- python3 $root/bench.py --steps 3 --warmup 1 --inflight 1 $OFF > $root/$out/prof_c4.log 2>&1) || { tail -20 $out/prof_c4.log; exit 1; }
f=$(find $out/prof_c4 -name "*kernel_stats.csv" | head -1); cp $f $out/prof_c4_kernel_stats.csv; head -4 $out/prof_c4_kernel_stats.csv
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
print('value', r['value'], 'single', r['single_stream']['value'], r['single_stream']['avg_kernel_ms'])
rf=r['roofline']; print({k: rf.get(k) for k in ('achieved','frac','traffic','kernel')})
v=rf.get('valu',{}); print({k: v.get(k) for k in ('frac','valu_per_quad','issue_busy_frac','valu_insts_per_puzzle')}, (v.get('mix_ceiling') or {}).get('frac'))
for k in ('c2_30clue','minimal_puzzles'): print(k, r.get(k,{}).get('value'))
print('hard', json.dumps(r.get('hard_search',{}))[:600])
print('checker', r.get('checker_summary'))
"
