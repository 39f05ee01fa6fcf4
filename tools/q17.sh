# dequeue chunk sweep at shard sizes (dev tool)
for n in 1250000 10000000; do for ch in 2 4 8 16; do
  timeout -k 10 120 python tools/solve_profile.py --solver quad --workload solve17 --n $n --reps 5 --chunk $ch || exit 1
done; done
for ch in 4 16; do timeout -k 10 120 python tools/solve_profile.py --solver quad --workload solve30 --n 1000000 --reps 5 --chunk $ch || exit 1; done
