# A/B timing of option settings (and library variants) on one GPU box (dev tool).
#   SETTINGS="default|--prop32-lc 773|..."  solve_profile.py argument sets, '|'-separated
#   VARIANTS="r05 ..."    build/variants/lib_<name>.so timed at the default setting beside them
#   WORKLOADS="solve17:10000000 solve30:1000000 minimal:1000000 hard:1000000"   REPS=2
# usage: SETTINGS="default|--prop32-lc 773" bash tools/ab_opts.sh
set -o pipefail
IFS='|' read -ra SETS <<< "${SETTINGS:-default}"
for rep in $(seq ${REPS:-2}); do
  for wl in ${WORKLOADS:-solve17:10000000 solve30:1000000 minimal:1000000 hard:1000000}; do
    w=${wl%%:*}; n=${wl##*:}
    for st in "${SETS[@]}"; do
      a=""; [ "$st" != "default" ] && a="$st"
      timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 5 $a \
        | sed "s/^/[$st] /" || exit 1
    done
    for v in ${VARIANTS:-}; do
      SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad \
        --workload $w --n $n --reps 5 | sed "s/^/[$v] /" || exit 1
    done
  done
done
