# Split budget sweep of the phased solve (dev tool)
set -o pipefail
out=gpurun_out/split2; mkdir -p $out; log=$out/sweep.log; rm -f $log
for wl in hard:100000 heavy:1000 heavy:10000 minimal:262144; do
  w=${wl%%:*}; n=${wl##*:}
  for dn in 0 128 256 512 1024; do
    timeout -k 10 120 python3 tools/solve_profile.py --solver quad --workload $w --n $n --reps 5 --donate $dn >> $log 2>&1 || exit 1
  done
done
cat $log
