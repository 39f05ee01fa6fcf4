# Tail-only split budget sweep (dev tool): one launch (donate 0) against the phased solve at
# several split budgets, phased at every batch size (SDK_OPT_DONATE_MAX 0).
set -o pipefail
mkdir -p gpurun_out/tailsplit
log=gpurun_out/tailsplit/sweep.log
for wl in ${WORKLOADS:-heavy:1000 hard:100000 heavy:10000 hard:1000000 minimal:1048576 solve17:10000000 solve17:1250000}; do
  w=${wl%%:*}; n=${wl##*:}
  for dn in 0 ${SPLITS:-16 64 256}; do
    timeout -k 10 120 python3 tools/solve_profile.py --solver quad --workload $w --n $n --reps 5 --donate $dn \
      --donate-max 0 >> $log 2>&1 || exit 1
  done
done
cat $log
