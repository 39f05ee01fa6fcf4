"""C5 count timing (dev tool): the 15-clue board's exhaustive count through shard.sharded_count on
one GPU, repeated, for a rocprofv3 --kernel-trace --stats split between frontier build and count."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402
from distributed_sudoku_solver_amd.shard import sharded_count  # noqa: E402

solver = sys.argv[1] if len(sys.argv) > 1 else ""
opts = dict(a.split("=") for a in sys.argv[2:])   # e.g. locked=0 wpc=16
board = synth.parse(synth.SEEDS17["S1"][:-9] + "0" * 9)
with SudokuEngine(0) as eng:
    if solver:
        eng.set_option(L.SDK_OPT_SOLVER, {"quad": L.SDK_SOLVER_QUAD, "wave": L.SDK_SOLVER_WAVE,
                                          "halfwave": L.SDK_SOLVER_HALFWAVE}[solver])
    if "locked" in opts:
        eng.set_option(L.SDK_OPT_LOCKED, int(opts["locked"]))
    if "wpc" in opts:      # the frontier target is CUs x this x 8
        eng.set_option(L.SDK_OPT_WAVES_PER_CU, int(opts["wpc"]))
    sharded_count(eng, board, 0, 1)
    for _ in range(3):
        t0 = time.perf_counter()
        total, st, size = sharded_count(eng, board, 0, 1)
        print(f"{solver or 'default'} {opts} count {total} status {st} frontier {size} wall {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
