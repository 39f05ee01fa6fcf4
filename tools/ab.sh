# A/B timing of the solve kernels on the GPU box (dev tool).
#   VARIANTS="name ..."  libraries build/variants/lib_<name>.so (tools/build_variant.sh,
#                        tools/build_variant_commit.sh) timed beside the in-tree library
#   WORKLOADS="solve17:10000000 solve30:1000000 minimal:2000000"  (workload:boards)
#   REPS=2  EXTRA="--locked 1 ..."  (extra tools/solve_profile.py arguments)
# e.g. VARIANTS=head bash tools/ab.sh
set -o pipefail
for rep in $(seq ${REPS:-2}); do
  for wl in ${WORKLOADS:-solve17:10000000 solve17:4000000 solve30:1000000 minimal:2000000}; do
    w=${wl%%:*}; n=${wl##*:}
    timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --n $n --reps 3 ${EXTRA:-} || exit 1
    for v in ${VARIANTS:-}; do
      SDK_LIB_PATH=$PWD/build/variants/lib_$v.so timeout -k 10 120 python tools/solve_profile.py --solver quad \
        --workload $w --n $n --reps 3 ${EXTRA:-} 2>&1 | sed "s/^/$v /" || exit 1
    done
  done
done
