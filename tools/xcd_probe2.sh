set -o pipefail
out=gpurun_out/xcd2; mkdir -p $out
for v in tl tlst; do
  SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 180 python3 tools/timeline.py --sizes 1250000 --json $out/timeline_$v.json \
    > $out/timeline_$v.log 2>&1 || { tail -5 $out/timeline_$v.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/timeline_$v.json'))
for n, r in d.items():
    print('$v', n, 'ms', round(r['kernel_ms_hip_events'],3), 'span', round(r['span_us']), 'drain', round(r['drain_us']), 'lastdeq', {k: round(v) for k, v in r['last_dequeue_us'].items()}, 'exit', {k: round(v) for k, v in r['exit_us'].items()}, 'first', {k: round(v) for k, v in r['first_boards_us'].items()})
"
done
