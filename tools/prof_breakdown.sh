# Cycle breakdown of solve4 per loop part (profiling build: tools/build_variant.sh prof -DSDK_SOLVE4_PROFILE=1), then LC-mode timings (dev tool)
export SDK_LIB_PATH=$PWD/build/variants/lib_prof.so
for w in solve17 minimal; do for lc in 0 1 2; do
timeout -k 10 120 python tools/solve4_prof.py --workload $w --locked $lc --n 2000000 || exit 1
done; done
unset SDK_LIB_PATH
for w in solve17 minimal; do for lc in 0 1 2; do
timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --locked $lc --n 4000000 --reps 3 || exit 1
done; done
