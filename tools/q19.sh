# tail variants A/B at shard sizes (dev tool)
for wl in "solve17 1250000" "solve17 10000000" "solve30 1000000"; do set -- $wl
  for rep in 1 2; do
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $1 --n $2 --reps 5 || exit 1
  for v in ${VARIANTS:-}; do SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $1 --n $2 --reps 5 2>&1 | sed "s/^/$v /" || exit 1; done
  done
done
