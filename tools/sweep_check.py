"""Checker sweep: grid size (blocks per CU) x repeats, interleaved in one process (dev tool)."""
import sys, os, ctypes
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L
eng = SudokuEngine(0)
pool_n = 1 << 20
b, exp = synth.make_check_boards(pool_n, seed=1)
nb = 100_000_000
d_b = eng.alloc(nb * 81); d_v = eng.alloc(nb)
for s in range(0, nb, pool_n):
    m = min(pool_n, nb - s)
    L.check(eng.lib.sdk_memcpy_h2d(eng.ctx, ctypes.c_void_p(d_b.ptr.value + s * 81), ctypes.c_void_p(b.ctypes.data), m * 81), "h2d")
res = {}
for rnd in range(3):
    for bpc in (2, 3, 4, 6, 8, 12, 16):
        eng.set_option(L.SDK_OPT_CHECK_BLOCKS_PER_CU, bpc)
        eng.check_batch_dev(d_b, d_v, nb); eng.synchronize()
        eng.timer_reset()
        for _ in range(5): eng.check_batch_dev(d_b, d_v, nb)
        eng.synchronize(); ms, nl = eng.timer_read()
        res.setdefault(bpc, []).append(ms / nl)
for bpc, v in res.items():
    per = min(v)
    print(f"blocks/CU={bpc:2d} min={per:.3f}ms med={sorted(v)[1]:.3f}ms  {82*nb/per/1e6:.0f} GB/s  frac={82*nb/per/1e6/8000:.3f}", flush=True)
v = np.empty(nb, np.uint8); d_v.download(v); print("check ok", (v == np.tile(exp, nb // pool_n + 1)[:nb]).all())
