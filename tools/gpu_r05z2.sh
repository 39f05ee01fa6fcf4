#!/bin/bash
# round 5 box pass 30: PROP32_LC 3 vs 4 on the whole default bench (C4 headline + hard legs), alternated
set -o pipefail
out=gpurun_out/r05z2
mkdir -p $out
i=0
for opts in "" "--opt PROP32_LC=3" "" "--opt PROP32_LC=3 --opt PROP32_TAIL=2060"; do
i=$((i+1))
timeout -k 10 600 python -u bench.py --cpu-seconds 0 --http-requests 0 $opts > $out/bench_$i.json 2> $out/bench_$i.err || { tail -20 $out/bench_$i.err; exit 1; }
python3 -c "
import json; r=json.loads(open('$out/bench_$i.json').read().strip().splitlines()[-1])
h=r['hard_search']
print('$opts', 'value', round(r['value']/1e9,3), 'kernel_ms', r['roofline']['avg_kernel_ms'], 'frac', r['roofline']['frac'])
for k in ('c2_30clue','minimal_puzzles'):
    v=r[k]
    print('   ', k, v if not isinstance(v,dict) else {kk: vv for kk, vv in v.items() if kk in ('value','ms_per_solve')})
for k in ('hard_100k','hard_1m'): print('   ', k, {m: round(h[k][m]['value']/1e6,1) for m in ('donation','donation_in_flight') if m in h[k]})
"
done
