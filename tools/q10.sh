# A/B: default vs variants, XCD heads on (dev tool)
for rep in 1 2; do for w in solve17 minimal solve30; do
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n 4000000 --reps 3 || exit 1
  for v in ${VARIANTS:-}; do SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n 4000000 --reps 3 2>&1 | sed "s/^/$v /" || exit 1; done
done; done
