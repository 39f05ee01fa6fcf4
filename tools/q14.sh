# A/B at the bench size (10M 17-clue) and 4M: HEAD vs variants, interleaved (dev tool)
for rep in 1 2; do
  for n in 10000000; do
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload solve17 --n $n --reps 3 || exit 1
    for v in ${VARIANTS:-}; do SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload solve17 --n $n --reps 3 2>&1 | sed "s/^/$v /" || exit 1; done
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload solve17 --n $n --reps 3 --waves-per-cu 32 | sed "s/^/wpc32 /" || exit 1
  done
done
