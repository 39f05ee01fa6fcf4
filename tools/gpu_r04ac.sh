#!/bin/bash
# round 4 box pass: adaptive order (SDK_OPT_ADAPT: LEX boards switch to MRV-unique after K nodes)
# -- the headline kernel with the switch compiled in (K = 0) against the build without it, then K
# = 24 / 48 / 96 on every solve workload, one launch; parity of the switched boards by the tests
set -o pipefail
out=gpurun_out/r04ac
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "noadapt 0" "adapt 0" "adapt 24" "adapt 48" "adapt 96"; do
  set -- $cfg
  v=$1; k=$2
  for wl in "solve17 10000000" "solve17 1250000" "solve30 1000000" "minimal 1048576" "hard 100000" "hard 1000000"; do
    set -- $wl
    SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python -u tools/solve_profile.py --workload $1 \
      --n $2 --reps 5 --solver quad --donate 0 --adapt $k 2>&1 | grep rate | sed "s/^/$v-k$k /" >> $out/ab.log || exit 1
  done
done
done
python3 tools/ab_table.py $out/ab.log
