# Static round-robin board assignment (build/variants/lib_static.so) against the dequeue (dev tool)
set -o pipefail
mkdir -p gpurun_out/static
log=gpurun_out/static/sweep.log
for wl in ${WORKLOADS:-solve17:1250000 solve17:2500000 solve17:10000000 solve30:1000000 minimal:1048576}; do
  w=${wl%%:*}; n=${wl##*:}
  for v in base ${VARIANTS:-static}; do
    lib=""; [ $v != base ] && lib=$PWD/build/variants/lib_$v.so
    env ${lib:+SDK_LIB_PATH=$lib} timeout -k 10 120 python3 tools/solve_profile.py --solver quad --workload $w --n $n \
      --reps 5 --donate 0 2>&1 | sed "s/^/$v /" >> $log || exit 1
  done
done
cat $log
