"""Time sharded_solve (frontier first-solution scan) per golden solve case at the default frontier
target (dev tool): frontier size, build and scan time per case."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from distributed_sudoku_solver_amd import SudokuEngine, _lib as L  # noqa: E402
from distributed_sudoku_solver_amd.shard import sharded_solve, default_target  # noqa: E402
from oracle import oracle as O  # noqa: E402

cases = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "solve_cases.json")))["cases"]
with SudokuEngine(0) as eng:
    print("default target", default_target(eng, 1))
    for c in cases[:40]:
        board = np.array(c["puzzle"], np.uint8)
        m = O.range_mask(*c["range"])
        t0 = time.perf_counter()
        size, _ = eng.frontier_build(board, mask=m, mode=L.SDK_FRONTIER_FIRST, target=default_target(eng, 1))
        t1 = time.perf_counter()
        out, st = sharded_solve(eng, board, 0, 1, mask=m)
        t2 = time.perf_counter()
        print(f"{c['name'][:40]:40s} size={size:8d} build={1e3 * (t1 - t0):8.2f} ms solve={1e3 * (t2 - t1):8.2f} ms st={st}",
              flush=True)
