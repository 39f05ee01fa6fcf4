# kernel rate vs per-GPU batch (strong-scaling shards of 10M: 1.25M, 2.5M, 5M) (dev tool)
for n in 1250000 2500000 5000000 10000000; do
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload solve17 --n $n --reps 5 || exit 1
done
