"""Solver sweep: boards per dequeue x grid waves per CU on the C4 batch (10M 17-clue), interleaved repeats (dev tool)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
eng = SudokuEngine(0)
p, s = synth.make_17clue(n, seed=20250614)
d_in, d_out, d_st = eng.alloc(n * 81), eng.alloc(n * 81), eng.alloc(n)
d_in.upload(p)
res = {}
for rnd in range(2):
    for wpc in (24, 32):
        for chunk in (0, 8, 16, 24, 32, 48, 64):
            eng.set_option(L.SDK_OPT_WAVES_PER_CU2, wpc)
            eng.set_option(L.SDK_OPT_SOLVE_CHUNK, chunk)
            eng.solve_batch_dev(d_in, d_out, d_st, n); eng.synchronize()
            if rnd == 0:
                out = np.empty((n, 81), np.uint8); d_out.download(out)
                assert (out == s).all(), (wpc, chunk)
            eng.timer_reset()
            for _ in range(3): eng.solve_batch_dev(d_in, d_out, d_st, n)
            eng.synchronize(); ms, nl = eng.timer_read()
            res.setdefault((wpc, chunk), []).append(ms / nl)
    print(f"round {rnd} done", flush=True)
for (wpc, chunk), t in sorted(res.items(), key=lambda kv: min(kv[1])):
    print(f"waves/CU={wpc} chunk={chunk or 'auto'}: {min(t):.3f} ms  {n / min(t) / 1e3:.1f} M puzzles/s", flush=True)
