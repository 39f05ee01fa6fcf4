# lane solver: tests + C2 timing vs quad + C4 sample with a validation budget (dev tool)
mkdir -p gpurun_out/q8
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q8/pytest.log 2>&1 || { tail -40 gpurun_out/q8/pytest.log; exit 1; }
tail -2 gpurun_out/q8/pytest.log
timeout -k 10 120 python tools/solve_profile.py --solver lane --workload solve30 --n 1000000 --reps 2 || exit 1
timeout -k 10 120 python tools/solve_profile.py --solver quad --workload solve30 --n 1000000 --reps 2 || exit 1
timeout -k 10 120 python tools/solve_profile.py --solver lane --workload solve17 --n 20000 --reps 1 --budget 2000000 || exit 1
