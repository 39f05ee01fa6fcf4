# Dequeue-stage A/B (dev tool): in-tree library against build/variants/lib_deq1/deq2.so, and
# their launch timelines (lib_tl*.so) at the small shard.
set -o pipefail
rm -f gpurun_out/static/sweep.log
VARIANTS="deq1 deq2" WORKLOADS="solve17:1250000 solve17:10000000 solve30:1000000 minimal:1048576 hard:100000" \
  bash tools/sweep_static.sh > /dev/null || exit 1
cat gpurun_out/static/sweep.log
out=gpurun_out/deq; mkdir -p $out
for v in tl tldeq1 tldeq2; do
  SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 180 python3 tools/timeline.py --sizes 1250000 --json $out/timeline_$v.json \
    > $out/timeline_$v.log 2>&1 || { tail -5 $out/timeline_$v.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/timeline_$v.json'))
for n, r in d.items():
    print('$v', n, 'ms', round(r['kernel_ms_hip_events'],3), 'span', round(r['span_us']), 'drain', round(r['drain_us']), 'lastdeq', {k: round(v) for k, v in r['last_dequeue_us'].items()}, 'exit', {k: round(v) for k, v in r['exit_us'].items()})
"
done
