"""Frontier build timing per level (dev tool): builds the 1M-board C5 frontier of the 14-clue board
(bench leg c5_count_rebalanced's probe) a few times; run under
  rocprofv3 --kernel-trace --stats -d <dir> -o run --output-format csv -- python3 tools/frontier_levels.py
to get every expand/scan/emit dispatch in order (the per-level durations).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402

b15 = synth.SEEDS17["S1"][:-9] + "0" * 9
b14 = synth.parse(b15[:63] + "000100000" + "0" * 9)     # bench.py c5_board("14")
solver = sys.argv[1] if len(sys.argv) > 1 else "quad"   # quad: expand4_kernel; halfwave: expand_kernel
with SudokuEngine(0) as eng:
    eng.set_option(L.SDK_OPT_SOLVER, L.SDK_SOLVER_QUAD if solver == "quad" else L.SDK_SOLVER_HALFWAVE)
    for target in (1_000_000, 1_000_000, 1_000_000):
        t0 = time.perf_counter()
        size, leaves = eng.frontier_build(b14, target=target)
        print(f"{solver} target {target}: {size} boards, {leaves} leaves, {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
