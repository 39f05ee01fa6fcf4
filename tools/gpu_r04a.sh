#!/bin/bash
# round 4, first box pass: the reworked donation kernel's tests first (bounded), then the
# slice probe, then the node / search tests, then the whole -m gpu suite.
set -o pipefail
out=gpurun_out/r04a
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
(cd /tmp && timeout -k 5 60 rocprofv3 --list-avail > $OLDPWD/$out/list_avail.txt 2>&1) || echo "list-avail failed"
timeout -k 10 400 $T tests/test_gpu_donate.py > $out/donate.log 2>&1 || { tail -30 $out/donate.log; exit 1; }
tail -2 $out/donate.log
timeout -k 10 120 python -u tools/slice_probe.py --slices 30 > $out/slice_probe.log 2>&1 || { tail -30 $out/slice_probe.log; exit 1; }
tail -4 $out/slice_probe.log
timeout -k 10 400 $T tests/test_gpu_search.py tests/test_gpu_node.py > $out/node_search.log 2>&1 || { tail -40 $out/node_search.log; exit 1; }
tail -2 $out/node_search.log
timeout -k 10 900 $T -m gpu tests > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
