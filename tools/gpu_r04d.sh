#!/bin/bash
# round 4 box pass (combined): parity of the statics-in-first-round build, its A/B and the
# output-write A/B, the node's slice diagnostics, the per-SIMD PMC passes of C4, the bench.
set -o pipefail
out=gpurun_out/r04d
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
SDK_LIB_PATH=$PWD/build/variants/lib_fresh.so timeout -k 10 400 $T tests/test_gpu_solve.py tests/test_gpu_donate.py \
  > $out/pytest_fresh.log 2>&1 || { tail -30 $out/pytest_fresh.log; exit 1; }
tail -1 $out/pytest_fresh.log
VARIANTS="fresh noout" WORKLOADS="solve17:10000000 solve17:1250000 minimal:1048576 hard:100000" REPS=2 EXTRA="--donate 0" \
  timeout -k 10 500 bash tools/ab.sh > $out/ab.log 2>&1 || { tail -30 $out/ab.log; exit 1; }
cat $out/ab.log
timeout -k 10 120 python -u tools/slice_probe.py --node --fork --slices 150 > $out/slice_probe_node.log 2>&1 || { tail -30 $out/slice_probe_node.log; exit 1; }
tail -1 $out/slice_probe_node.log
timeout -k 10 300 bash tools/pmc_r04.sh $out/pmc c4 > $out/pmc.log 2>&1 || { tail -30 $out/pmc.log; exit 1; }
tail -3 $out/pmc.log
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
head -c 1500 $out/bench.json
