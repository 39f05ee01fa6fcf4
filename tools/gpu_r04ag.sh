#!/bin/bash
# round 4 box pass: the bench's pipelined C4 figure at 10M and at an 8-GPU shard (1.25M)
set -o pipefail
out=gpurun_out/r04ag
mkdir -p $out
export TMPDIR=/tmp
OFF="--check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0"
timeout -k 10 300 python -u bench.py $OFF > $out/b10m.json 2> $out/b10m.err || { tail -20 $out/b10m.err; exit 1; }
timeout -k 10 300 python -u bench.py $OFF --batch 1250000 > $out/b125.json 2> $out/b125.err || { tail -20 $out/b125.err; exit 1; }
python3 - <<'PY'
import json
for f in ("b10m", "b125"):
    d = json.loads(open("gpurun_out/r04ag/%s.json" % f).read().strip().splitlines()[-1])
    print(f, round(d["value"] / 1e6, 1), round(d["ms_per_step"], 3), json.dumps(d.get("pipelined")))
PY
