"""Solver sweep: residency x order on resident batches, interleaved rounds (dev tool)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L
eng = SudokuEngine(0)
work = {}
for name, gen, n in (("17clue", synth.make_17clue, 4_000_000), ("30clue", synth.make_30clue, 4_000_000)):
    p, s = gen(n, seed=3)
    d_in, d_out, d_st = eng.alloc(n * 81), eng.alloc(n * 81), eng.alloc(n)
    d_in.upload(p)
    res = {}
    for rnd in range(3):
        for order in ("mrv", "lex"):
            eng.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX if order == "lex" else L.SDK_ORDER_MRV_UNIQUE)
            for wpc in (8, 16, 24, 32):
                eng.set_option(L.SDK_OPT_WAVES_PER_CU, wpc)
                eng.timer_reset()
                eng.solve_batch_dev(d_in, d_out, d_st, n); eng.synchronize()
                ms, _ = eng.timer_read()
                res.setdefault((order, wpc), []).append(ms)
    out = np.empty((n, 81), np.uint8); d_out.download(out)
    print(name, "exact:", bool((out == s).all()), flush=True)
    for k, v in sorted(res.items()):
        print(f"  {name} order={k[0]} waves/CU={k[1]:2d} min={min(v):.2f}ms  {n/min(v)*1e3/1e6:.1f} M puzzles/s", flush=True)
    for b in (d_in, d_out, d_st): b.free()
eng.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_MRV_UNIQUE); eng.set_option(L.SDK_OPT_WAVES_PER_CU, 16)
p, s = synth.make_17clue(200000, seed=4)
out, st, wk = eng.solve_batch(p, want_work=True)
print("nodes per 17-clue puzzle: mean %.2f p99 %d max %d" % (wk.mean(), np.percentile(wk, 99), wk.max()))
import time
s1 = synth.SEEDS17["S1"]
for name, b in (("16clue", s1[:-9] + "000800000"), ("15clue", s1[:-9] + "0" * 9), ("14clue", s1[:-18] + "000100000" + "0" * 9)):
    eng.timer_reset(); t = time.time(); c = eng.count_solutions(synth.parse(b)); dt = time.time() - t
    ms, nl = eng.timer_read()
    print(f"count {name}: {c} wall {dt*1e3:.1f} ms kernels {ms:.1f} ms ({nl} launches)", flush=True)
