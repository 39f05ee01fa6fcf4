#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, rocprof kernel stats, HBM PMC passes.
# usage (from the repo root on the box): tools/gpu_round.sh <tag> [tests|bench|prof|pmc ...]
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
tag=${1:-r01}; shift
steps=${*:-tests bench prof pmc}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)

for s in $steps; do
  case $s in
  tests)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$out/pytest_gpu.log"; exit 1; }
    tail -3 "$out/pytest_gpu.log"
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
      || { echo "smoke failed"; tail -20 "$out/smoke.log"; exit 1; }
    cat "$out/smoke.log" ;;
  bench)
    timeout -k 10 420 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" \
      || { echo "bench failed"; tail -20 "$out/bench.err"; exit 1; }
    cat "$out/bench.json" ;;
  prof)
    (cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$root/$out/prof" -o run \
      --output-format csv -- python3 "$root/bench.py" --cpu-seconds 0 --http-requests 0 \
      > "$root/$out/prof_bench.json" 2> "$root/$out/prof.err") \
      || { echo "rocprof failed"; tail -20 "$out/prof.err"; exit 1; }
    find "$out/prof" -name '*kernel_stats.csv' -exec cat {} \; ;;
  prof_c4)   # the headline launch alone: solve4_kernel's average = the C4 launch the bench line times
             # (single stream: --inflight 1, one context, per-launch HIP events)
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$root/$out/prof_c4" -o run \
      --output-format csv -- python3 "$root/bench.py" --check-boards 0 --c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 \
      --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 --inflight 1 > "$root/$out/prof_c4_bench.json" 2> "$root/$out/prof_c4.err") \
      || { echo "rocprof c4 failed"; tail -20 "$out/prof_c4.err"; exit 1; }
    find "$out/prof_c4" -name '*kernel_stats.csv' -exec cat {} \; ;;
  prof_c3)   # the checker launch alone (C4 shrunk to 1024 puzzles)
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$root/$out/prof_c3" -o run \
      --output-format csv -- python3 "$root/bench.py" --batch 1024 --c2-puzzles 0 --minimal-puzzles 0 --hard-leg 0 \
      --count-leg 0 --lane-puzzles 0 --cpu-seconds 0 --http-requests 0 > "$root/$out/prof_c3_bench.json" 2> "$root/$out/prof_c3.err") \
      || { echo "rocprof c3 failed"; tail -20 "$out/prof_c3.err"; exit 1; }
    find "$out/prof_c3" -name '*kernel_stats.csv' -exec cat {} \; ;;
  pmc)
    for c in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$root/$out/pmc_$c" -o run -- \
        python3 "$root/bench.py" --steps 2 --warmup 0 --check-steps 2 --cpu-seconds 0 --http-requests 0 \
        > "$root/$out/pmc_$c.json" 2> "$root/$out/pmc_$c.err") \
        || { echo "pmc $c failed"; tail -20 "$out/pmc_$c.err"; exit 1; }
    done
    python3 tools/pmc_summary.py "$out" | tee "$out/pmc_summary.txt" ;;
  hard_trace)   # the hard-search passes' dispatch sequence (prop32, split phase, donation, scatters)
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$root/$out/hard_trace" -o run --output-format csv \
      -- python3 "$root/tools/hard_phases.py" ${HARD_ARGS:-} > "$root/$out/hard_phases.json" 2> "$root/$out/hard_phases.err") \
      || { echo "hard trace failed"; tail -20 "$out/hard_phases.err"; exit 1; }
    cat "$out/hard_phases.json"
    python3 tools/hard_phases_summary.py "$out/hard_trace" > "$out/hard_phases_summary.txt"
    head -3 "$out/hard_phases_summary.txt" ;;
  ab)   # option settings / library variants (tools/ab_opts.sh; SETTINGS, VARIANTS, WORKLOADS, REPS from the env)
    bash tools/ab_opts.sh > "$out/ab.log" 2>&1 || { echo "ab failed"; tail -20 "$out/ab.log"; exit 1; }
    cat "$out/ab.log" ;;
  read_ceiling)   # HBM read ceiling for the checker's access pattern (tools/read_ceiling.hip)
    timeout -k 10 120 tools/read_ceiling > "$out/read_ceiling.txt" 2>&1 || { echo "read ceiling failed"; tail -5 "$out/read_ceiling.txt"; exit 1; }
    cat "$out/read_ceiling.txt" ;;
  pmc_pipe)   # per-SIMD pipe and LDS counters of the C4 launch and the hard_1m one-launch solve
    bash tools/pmc_r04.sh "$out/pmc_pipe" c4 hard1m > "$out/pmc_pipe.log" 2>&1 || { echo "pmc pipe failed"; tail -10 "$out/pmc_pipe.log"; exit 1; }
    tail -5 "$out/pmc_pipe.log" ;;
  pmc_c4)   # FETCH/WRITE/SQ passes of the C4 and C3 launches (tools/pmc_c4.sh)
    bash tools/pmc_c4.sh "$out/pmc_c4" > "$out/pmc_c4.log" 2>&1 || { echo "pmc c4 failed"; tail -10 "$out/pmc_c4.log"; exit 1; }
    tail -5 "$out/pmc_c4.log" ;;
  clock_ramp)   # per-pass kernel time and in-kernel clock of C4 from a cold GPU (tools/clock_ramp.py)
    timeout -k 10 180 python -u tools/clock_ramp.py > "$out/clock_ramp.jsonl" 2> "$out/clock_ramp.err" \
      || { echo "clock ramp failed"; tail -10 "$out/clock_ramp.err"; exit 1; }
    cat "$out/clock_ramp.jsonl" ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
