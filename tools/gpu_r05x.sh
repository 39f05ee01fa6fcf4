#!/bin/bash
# round 5 box pass 25: evidence for the current prop32 build -- PMC pipe/LDS + traffic passes, rocprof kernel
# stats of the C3 and C4 bench commands, then the default bench with the fresh PMC records in place
set -o pipefail
out=gpurun_out/r05x
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
timeout -k 10 600 bash tools/pmc_r04.sh $out/pmc c4 > $out/pmc.log 2>&1 || { tail -30 $out/pmc.log; exit 1; }
tail -2 $out/pmc.log
timeout -k 10 900 bash tools/pmc_c4.sh $out/traffic > $out/traffic.log 2>&1 || { tail -30 $out/traffic.log; exit 1; }
grep -E "^sdk::prop32|^sdk::check" $out/traffic.log | cut -c1-300
cp $out/pmc/pmc_pipe.json profiles/r05/pmc_pipe.json
cp $out/traffic/pmc_c4.json profiles/r05/pmc_c4.json
bash tools/gpu_round.sh r05x prof_c3 prof_c4 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
grep -E "check_kernel|prop32_kernel" $out/prof.log | cut -c1-160
python3 tools/trace_avg.py $(find $out/prof_c3 -name "*kernel_trace.csv" | head -1) check_kernel 10 8200000000
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
print('value', r['value'], 'single', r['single_stream']['value'], r['single_stream']['avg_kernel_ms'])
rf=r['roofline']; print({k: rf.get(k) for k in ('achieved','frac','traffic','kernel')})
v=rf.get('valu',{}); print({k: v.get(k) for k in ('frac','valu_per_quad','issue_busy_frac','valu_insts_per_puzzle','lds_insts_per_puzzle')}, (v.get('mix_ceiling') or {}).get('frac'))
for k in ('c2_30clue','minimal_puzzles'): print(k, r.get(k,{}).get('value'))
h=r.get('hard_search',{})
for k in ('hard_100k','heaviest_1000','hard_1m'): print(k, {m: round(h.get(k,{}).get(m,{}).get('value',0)/1e6,1) for m in ('one_launch','donation','mrv_one_launch','mrv_donation')})
print('checker', r.get('checker_summary'))
"
