"""Ad-hoc GPU exploration: timings and search-node statistics (dev tool, not a test)."""
import sys, time, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L

eng = SudokuEngine(0)
for n in (1000, 100000):
    p, s = synth.make_17clue(n, seed=5)
    for order in (L.SDK_ORDER_MRV_UNIQUE, L.SDK_ORDER_LEX):
        eng.set_option(L.SDK_OPT_ORDER, order)
        eng.solve_batch(p[:100])
        eng.timer_reset()
        t = time.time(); out, st, work = eng.solve_batch(p, want_work=True); dt = time.time() - t
        ms, nl = eng.timer_read()
        print(f"17clue n={n} order={order} wall={dt:.3f}s kernel={ms:.1f}ms rate={n/(ms/1e3):.0f}/s ok={(out==s).all()} "
              f"work mean={work.mean():.1f} p50={np.median(work):.0f} p99={np.percentile(work,99):.0f} max={work.max()}", flush=True)
eng.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_MRV_UNIQUE)
p, s = synth.make_30clue(100000, seed=5)
eng.timer_reset(); out, st, work = eng.solve_batch(p, want_work=True); ms, nl = eng.timer_read()
print(f"30clue kernel={ms:.1f}ms rate={100000/(ms/1e3):.0f}/s ok={(out==s).all()} work mean={work.mean():.2f} max={work.max()}", flush=True)
for wpc in (4, 8, 16, 32):
    eng.set_option(L.SDK_OPT_WAVES_PER_CU, wpc)
    p, s = synth.make_17clue(100000, seed=6)
    eng.timer_reset(); out, st, work = eng.solve_batch(p); ms, nl = eng.timer_read()
    print(f"waves/cu={wpc} 17clue kernel={ms:.1f}ms rate={100000/(ms/1e3):.0f}/s", flush=True)
eng.set_option(L.SDK_OPT_WAVES_PER_CU, 16)
eng.set_option(L.SDK_OPT_NODE_BUDGET, 2_000_000)
b = np.zeros(81, np.uint8); b[0] = b[1] = 5
eng.timer_reset(); out, st, work = eng.solve_batch(b[None], want_work=True); ms, _ = eng.timer_read()
print("55-board status", st, "work", work, "ms", ms, flush=True)
eng.set_option(L.SDK_OPT_NODE_BUDGET, 0)
b, exp = synth.make_check_boards(1 << 20, seed=1)
nb = 20 * (1 << 20)
d_b = eng.alloc(nb * 81); d_v = eng.alloc(nb)
import ctypes
for k in range(20):
    L.check(eng.lib.sdk_memcpy_h2d(eng.ctx, ctypes.c_void_p(d_b.ptr.value + k * (1 << 20) * 81), ctypes.c_void_p(b.ctypes.data), b.nbytes), "h2d")
eng.check_batch_dev(d_b, d_v, nb); eng.synchronize()
eng.timer_reset()
for _ in range(5): eng.check_batch_dev(d_b, d_v, nb)
eng.synchronize(); ms, nl = eng.timer_read()
per = ms / nl
print(f"check n={nb} kernel={per:.3f}ms  {82*nb/per/1e6:.0f} GB/s  {nb/per*1e3/1e9:.2f} Gboards/s", flush=True)
v = np.empty(nb, np.uint8); d_v.download(v); print("check ok", (v == np.tile(exp, 20)).all())
