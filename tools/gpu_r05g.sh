#!/bin/bash
# round 5 box pass 7: prop32 C4 profile -- kernel trace + stats, per-SIMD pipe and LDS counters
set -o pipefail
out=gpurun_out/r05g
mkdir -p $out
export TMPDIR=/tmp
root=$(pwd)
OFF="--c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --check-boards 0 --pmc-summary="
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/$out/prof_c4 -o run -- python3 $root/bench.py --steps 3 --warmup 1 $OFF > $root/$out/prof_c4.log 2>&1) || { tail -20 $out/prof_c4.log; exit 1; }
f=$(find $out/prof_c4 -name "*kernel_stats.csv" | head -1); cp $f $out/prof_c4_kernel_stats.csv; head -8 $out/prof_c4_kernel_stats.csv
timeout -k 10 600 bash tools/pmc_r04.sh $out/pmc c4 > $out/pmc.log 2>&1 || { tail -30 $out/pmc.log; exit 1; }
tail -4 $out/pmc.log
