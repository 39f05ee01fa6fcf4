#!/bin/bash
# round 5 box pass 11: prop32 step statistics (SDK_PROP32_STATS build)
set -o pipefail
out=gpurun_out/r05k
mkdir -p $out
export SDK_LIB_PATH=$PWD/build/variants/lib_p32stats.so
for wl in solve17:1000000 solve30:1000000 minimal:262144 hard:65536; do
  w=${wl%%:*}; n=${wl##*:}
  for lc in 4 3; do
    timeout -k 10 120 python tools/prop32_stats.py --workload $w --n $n --lc $lc >> $out/stats.log 2>&1 || { cat $out/stats.log; exit 1; }
  done
done
cat $out/stats.log
