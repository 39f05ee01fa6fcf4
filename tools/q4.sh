# solver parity tests + timings (LC modes) + cycle breakdown (dev tool)
mkdir -p gpurun_out/q4
timeout -k 10 400 python -u -m pytest tests/test_gpu_solve.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q4/pytest.log 2>&1 || { tail -30 gpurun_out/q4/pytest.log; exit 1; }
tail -2 gpurun_out/q4/pytest.log
for w in solve17 minimal; do for lc in 0 1 2; do
timeout -k 10 120 python tools/solve_profile.py --solver quad --workload $w --locked $lc --n 4000000 --reps 3 || exit 1
done; done
export SDK_LIB_PATH=$PWD/build/variants/lib_prof.so
for w in solve17 minimal; do for lc in 0 1; do
timeout -k 10 120 python tools/solve4_prof.py --workload $w --locked $lc --n 2000000 || exit 1
done; done
