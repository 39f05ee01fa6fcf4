set -o pipefail
mkdir -p gpurun_out/chunk
for n in 1250000 10000000; do
  for ch in 16 8 4 2; do
    timeout -k 10 120 python3 tools/solve_profile.py --solver quad --n $n --reps 5 --chunk $ch --donate 0 >> gpurun_out/chunk/sweep.log 2>&1 || exit 1
  done
done
cat gpurun_out/chunk/sweep.log
