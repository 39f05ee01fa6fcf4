#!/bin/bash
# round 4, second box pass: slice diagnostics, per-SIMD PMC passes, the output-write A/B,
# the bench, and the donation kernel on a GPU shared by two ranks.
set -o pipefail
out=gpurun_out/r04b
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/slice_probe.py --node --fork --slices 300 > $out/slice_probe_node.log 2>&1 || { tail -30 $out/slice_probe_node.log; exit 1; }
tail -2 $out/slice_probe_node.log
timeout -k 10 900 bash tools/pmc_r04.sh $out/pmc c4 hard1m min > $out/pmc.log 2>&1 || { tail -30 $out/pmc.log; exit 1; }
tail -8 $out/pmc.log
VARIANTS="noout base" WORKLOADS="solve17:10000000 solve17:1250000" REPS=3 timeout -k 10 600 bash tools/ab.sh > $out/ab_noout.log 2>&1 || { tail -30 $out/ab_noout.log; exit 1; }
cat $out/ab_noout.log
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json | head -c 3000
timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 \
  --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 > $out/bench_2rank_shared.json 2> $out/bench_2rank_shared.err \
  || { tail -30 $out/bench_2rank_shared.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench_2rank_shared.json'));print(json.dumps(d.get('hard_search'),indent=0)[:1500])"
