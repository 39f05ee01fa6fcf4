# A/B: XCD dequeue heads on/off vs the previous build (dev tool)
for rep in 1 2; do for w in solve17 minimal solve30; do
  for xh in 1 0; do timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n 4000000 --reps 3 --xcd-heads $xh || exit 1; done
  SDK_LIB_PATH=$PWD/build/variants/lib_prev.so timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n 4000000 --reps 3 2>&1 | sed "s/^/prev /" || exit 1
done; done
