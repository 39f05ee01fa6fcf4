"""Host-pointer API throughput (dev tool): sdk_solve_batch / sdk_check_batch on host arrays,
PCIe included (the pipelined path above 2M boards)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
p, s = synth.make_17clue(n, seed=3)
b, exp = synth.make_check_boards(n * 4, seed=4)
with SudokuEngine(0) as eng:
    eng.solve_batch(p[:100000])
    for _ in range(2):
        t0 = time.perf_counter()
        out, st, _ = eng.solve_batch(p)
        t = time.perf_counter() - t0
        print(f"solve_batch host {n}: {t * 1e3:.1f} ms = {n / t / 1e6:.1f} M puzzles/s ok={(out == s).all()}", flush=True)
    for _ in range(2):
        t0 = time.perf_counter()
        v = eng.check_batch(b)
        t = time.perf_counter() - t0
        print(f"check_batch host {4 * n}: {t * 1e3:.1f} ms = {4 * n / t / 1e6:.1f} M boards/s = "
              f"{4 * n * 81 / t / 1e9:.1f} GB/s ok={(v == exp).all()}", flush=True)
