# A/B: default (6 waves) vs w7 (7 waves, 28-wave grid) vs c885, at 10M and 4M 17-clue, 4M 30-clue (dev tool)
for rep in 1 2; do
  for wl in "solve17 10000000" "solve17 4000000" "solve30 4000000" "minimal 4000000"; do set -- $wl
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $1 --n $2 --reps 3 || exit 1
    SDK_LIB_PATH=$PWD/build/variants/lib_w7.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $1 --n $2 --reps 3 --waves-per-cu 28 2>&1 | sed "s/^/w7 /" || exit 1
    SDK_LIB_PATH=$PWD/build/variants/lib_c885.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $1 --n $2 --reps 3 2>&1 | sed "s/^/c885 /" || exit 1
  done
done
