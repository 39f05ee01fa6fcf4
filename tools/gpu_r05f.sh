#!/bin/bash
# round 5 box pass 6: the bench with prop32 (default run) and a kernel-trace profile of its C4 leg
set -o pipefail
out=gpurun_out/r05f
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -c 3000 $out/bench.json
OFF="--c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --check-boards 0"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/prof_c4 -o run -- python3 $root/bench.py --steps 3 --warmup 1 $OFF > $root/$out/prof_c4.log 2>&1) || { tail -20 $out/prof_c4.log; exit 1; }
find $out/prof_c4 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/prof_c4_kernel_stats.csv
head -12 $out/prof_c4_kernel_stats.csv
