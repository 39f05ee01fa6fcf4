# Dequeue heads x chunk sweep (dev tool): in-tree library (8 heads) and build/variants/lib_h32/h64.so
# (tools/build_variant.sh h32 -DSDK_HEADS=32), 17-clue at a small-shard and the headline size.
set -o pipefail
mkdir -p gpurun_out/heads
log=gpurun_out/heads/sweep.log
for n in 1250000 10000000; do
  for ch in 16 8 4; do
    for v in base ${VARIANTS:-h32 h64}; do
      lib=""; [ $v != base ] && lib=$PWD/build/variants/lib_$v.so
      env ${lib:+SDK_LIB_PATH=$lib} timeout -k 10 120 python3 tools/solve_profile.py --solver quad --n $n --reps 5 --chunk $ch \
        --donate 0 2>&1 | sed "s/^/$v /" >> $log || exit 1
    done
  done
done
cat $log
