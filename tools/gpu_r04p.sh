#!/bin/bash
# round 4 box pass: per-workgroup launch timelines (1.25M / 10M 17-clue) of the default build and
# the wave-pool build
set -o pipefail
out=gpurun_out/r04p
mkdir -p $out
export TMPDIR=/tmp
for v in tl tlp; do
  SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 180 python -u tools/timeline.py --sizes 1250000,10000000 \
    --json $out/timeline_$v.json > $out/timeline_$v.log 2>&1 || { tail -20 $out/timeline_$v.log; exit 1; }
  cat $out/timeline_$v.log
done
