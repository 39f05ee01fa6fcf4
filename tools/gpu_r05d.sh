#!/bin/bash
# round 5 box pass 4: node slices with the pinned host staging; GPU tests of the node, search and
# solver paths.
set -o pipefail
out=gpurun_out/r05d
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/slice_probe.py --node --fork --timing --slices 200 > $out/slice_probe_timing.log 2>&1 \
  || { tail -20 $out/slice_probe_timing.log; exit 1; }
grep worst $out/slice_probe_timing.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $out/pytest_gpu.log 2>&1 \
  || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
