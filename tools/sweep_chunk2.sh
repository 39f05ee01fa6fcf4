# Dequeue chunk per shard size (dev tool): 17-clue at the 8/4/2/1-GPU shard sizes and 30-clue 1M.
set -o pipefail
out=gpurun_out/chunk2; mkdir -p $out; log=$out/sweep.log; rm -f $log
for wl in solve17:1250000 solve17:2500000 solve17:5000000 solve17:10000000 solve30:1000000 minimal:1048576; do
  w=${wl%%:*}; n=${wl##*:}
  for ch in 0 6 8 10 12; do
    timeout -k 10 120 python3 tools/solve_profile.py --solver quad --workload $w --n $n --reps 5 --donate 0 --chunk $ch \
      >> $log 2>&1 || exit 1
  done
done
cat $log
