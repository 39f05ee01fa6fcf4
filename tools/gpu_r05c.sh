#!/bin/bash
# round 5 box pass 3: intra-half stealing at the queue's end (A/B vs round 4's kernel), launch
# timelines of the search-heavy batches, node slices with kernel time, and a bench line.
set -o pipefail
out=gpurun_out/r05c
mkdir -p $out
export TMPDIR=/tmp
REPS=3 VARIANTS="head" WORKLOADS="solve17:10000000 solve17:1250000 minimal:1048576 hard:1000000" \
  timeout -k 10 600 bash tools/ab.sh > $out/ab_steal.log 2>&1 || { tail -20 $out/ab_steal.log; exit 1; }
sed -i 's/^quad /steal quad /' $out/ab_steal.log
python3 tools/ab_table.py $out/ab_steal.log
for wl in "hard 100000,1000000 lex" "hard 1000000 mrv_unique" "minimal 1048576 lex"; do
  set -- $wl
  SDK_LIB_PATH=$PWD/build/variants/lib_tl.so timeout -k 10 180 python tools/timeline.py --workload $1 --sizes $2 --order $3 \
    > $out/timeline_$1_$3.log 2>&1 || { tail -20 $out/timeline_$1_$3.log; exit 1; }
  python3 -c "
import json,sys
for l in open('$out/timeline_$1_$3.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$1 $3', d['boards'], 'kernel_ms', round(d['kernel_ms_hip_events'],3), 'last_deq p50/max', round(d['last_dequeue_us']['p50']), round(d['last_dequeue_us']['max']), 'exit p50/max', round(d['exit_us']['p50']), round(d['exit_us']['max']))
"
done
timeout -k 10 300 python -u tools/slice_probe.py --node --fork --timing --slices 150 > $out/slice_probe_timing.log 2>&1 \
  || { tail -20 $out/slice_probe_timing.log; exit 1; }
sort -t= -k7 -g $out/slice_probe_timing.log | tail -3
timeout -k 10 420 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print('value', d['value']/1e6, 'single', d['single_stream']['value']/1e6, 'valu', json.dumps({k: d['roofline']['valu'].get(k) for k in ('frac','valu_per_quad')}), 'mix', d['roofline']['valu']['mix_ceiling']['frac'] if d['roofline']['valu'].get('mix_ceiling') else None)
print('checker', json.dumps(d['checker_summary']))
print('hard', json.dumps({k: {m: round(v['value']/1e6,1) for m, v in d['hard_search'][k].items() if isinstance(v, dict) and 'value' in v} for k in ('hard_100k','heaviest_1000','hard_1m')}))
"
