# XCD balance probe (dev tool): one shared dequeue head against per-XCD heads, and the
# per-XCD launch timeline (build/variants/lib_tl.so), 17-clue at 1.25M and 10M boards.
set -o pipefail
out=gpurun_out/xcd; mkdir -p $out
for n in 1250000 10000000; do
  for xh in 1 0; do
    timeout -k 10 120 python3 tools/solve_profile.py --solver quad --n $n --reps 5 --xcd-heads $xh --donate 0 \
      >> $out/heads.log 2>&1 || exit 1
  done
done
cat $out/heads.log
SDK_LIB_PATH=$PWD/build/variants/lib_tl.so timeout -k 10 180 python3 tools/timeline.py --json $out/timeline.json \
  > $out/timeline.log 2>&1 || { tail -5 $out/timeline.log; exit 1; }
python3 -c "
import json; d=json.load(open('$out/timeline.json'))
for n, r in d.items():
    print(n, 'span', round(r['span_us']), 'drain', round(r['drain_us']))
    for k, x in r['per_xcd'].items(): print('  xcd', k, {a: round(b) for a, b in x.items()})
"
