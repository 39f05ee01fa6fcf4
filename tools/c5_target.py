"""Count wall time against the frontier target (dev tool): sharded_count and
sharded_count_rebalanced at world 1 on bench.py's C5 boards (15 and 14 clues)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth  # noqa: E402
from distributed_sudoku_solver_amd.shard import sharded_count, sharded_count_rebalanced  # noqa: E402
import bench  # noqa: E402

with SudokuEngine(0) as eng:
    for clues, fn in (("15", sharded_count), ("14", sharded_count_rebalanced)):
        board, expected, _ = bench.c5_board(synth, clues)
        for target in (65536, 131072, 262144, 524288, 1048576):
            fn(eng, board, 0, 1, target=target)
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                total, st, size = fn(eng, board, 0, 1, target=target)
            ms = (time.perf_counter() - t0) / reps * 1e3
            print(f"{clues}-clue {fn.__name__} target={target}: frontier {size} total {total} ok={total == expected} {ms:.2f} ms", flush=True)
