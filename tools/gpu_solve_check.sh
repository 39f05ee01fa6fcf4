set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 120 python3 tools/solve_profile.py --solver halfwave --sweep --stats > gpurun_out/s2/prof_half.txt 2>&1; rc=$?; cat gpurun_out/s2/prof_half.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/solve_profile.py --solver wave --sweep > gpurun_out/s2/prof_wave.txt 2>&1; rc=$?; cat gpurun_out/s2/prof_wave.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_solve.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s2/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/s2/pytest.log; exit $rc
