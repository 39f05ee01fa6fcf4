# quad: grid sweep 24/32 waves per CU (dev tool)
for w in solve17 minimal solve30; do for wpc in 24 32; do
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n 4000000 --reps 3 --waves-per-cu $wpc | sed "s/^/wpc=$wpc /" || exit 1
done; done
