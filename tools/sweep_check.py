"""Checker sweep: tile pipeline variant x grid size (blocks per CU), interleaved repeats in one process (dev tool).
Prints min / median launch time per (variant, blocks/CU) over 100M resident boards and the verdict parity."""
import sys, os, ctypes
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L
eng = SudokuEngine(0)
pool_n = 1 << 20
b, exp = synth.make_check_boards(pool_n, seed=int(os.environ.get("SWEEP_SEED", "1")))
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
if os.environ.get("SWEEP_PREALLOC"):   # mimic a preceding leg: 10M-puzzle solve buffers, freed
    tmp = [eng.alloc(10_000_000 * 81), eng.alloc(10_000_000 * 81), eng.alloc(10_000_000)]
    for x in tmp: x.free()
d_b = eng.alloc(nb * 81); d_v = eng.alloc(nb)
for s in range(0, nb, pool_n):
    m = min(pool_n, nb - s)
    L.check(eng.lib.sdk_memcpy_h2d(eng.ctx, ctypes.c_void_p(d_b.ptr.value + s * 81), ctypes.c_void_p(b.ctypes.data), m * 81), "h2d")
expect = np.tile(exp, nb // pool_n + 1)[:nb]
names = {L.SDK_CHECK_REG1: "reg1", L.SDK_CHECK_REG2: "reg2", L.SDK_CHECK_GLDS2: "glds2",
         L.SDK_CHECK_GLDS3: "glds3", L.SDK_CHECK_GLDS4: "glds4", L.SDK_CHECK_WAVE1: "wave1",
         L.SDK_CHECK_WAVE2: "wave2"}
grid = {L.SDK_CHECK_REG1: (2, 3, 4), L.SDK_CHECK_REG2: (2, 3), L.SDK_CHECK_GLDS2: (2, 3),
        L.SDK_CHECK_GLDS3: (1, 2), L.SDK_CHECK_GLDS4: (1,), L.SDK_CHECK_WAVE1: (2, 3, 4),
        L.SDK_CHECK_WAVE2: (2, 3, 4)}
only = os.environ.get("SWEEP_VARIANTS")          # e.g. "reg1,wave1,wave2"
if only:
    grid = {k: v for k, v in grid.items() if names[k] in only.split(",")}
res = {}
v = np.empty(nb, np.uint8)
for rnd in range(3):
    for var, bpcs in grid.items():
        eng.set_option(L.SDK_OPT_CHECK_VARIANT, var)
        for bpc in bpcs:
            eng.set_option(L.SDK_OPT_CHECK_BLOCKS_PER_CU, bpc)
            eng.check_batch_dev(d_b, d_v, nb); eng.synchronize()
            if rnd == 0:
                d_v.download(v)
                assert (v == expect).all(), (names[var], bpc)
            eng.timer_reset()
            for _ in range(int(os.environ.get("SWEEP_LAUNCHES", "5"))): eng.check_batch_dev(d_b, d_v, nb)
            eng.synchronize(); ms, nl = eng.timer_read()
            res.setdefault((var, bpc), []).append(ms / nl)
    print(f"round {rnd} done", flush=True)
for (var, bpc), t in sorted(res.items(), key=lambda kv: min(kv[1])):
    per = min(t)
    print(f"{names[var]:6s} blocks/CU={bpc:2d} min={per:.3f}ms med={sorted(t)[1]:.3f}ms  "
          f"{82*nb/per/1e6:.0f} GB/s  frac={82*nb/per/1e6/8000:.3f}", flush=True)
print("check ok (all variants bit-exact vs expected verdicts)")
