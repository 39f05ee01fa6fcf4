# A/B with a waves-per-CU sweep (dev tool)
for w in solve17 minimal; do
  for wpc in 28 32; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n 4000000 --reps 3 --waves-per-cu $wpc | sed "s/^/wpc=$wpc /" || exit 1
    for v in ${VARIANTS:-}; do SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n 4000000 --reps 3 --waves-per-cu $wpc 2>&1 | sed "s/^/$v wpc=$wpc /" || exit 1; done
  done
done
