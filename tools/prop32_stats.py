"""prop32 step statistics (dev tool, GPU; needs a SDK_PROP32_STATS build, e.g.
`tools/build_variant.sh p32stats -DSDK_PROP32_STATS=1` and SDK_LIB_PATH=build/variants/lib_p32stats.so):
per 64-board group, the steps it ran, the step at which at most 4 / 1 boards were still live, and its
locked-candidates passes.

usage: python tools/prop32_stats.py [--workload solve17|solve30|minimal|hard] [--n N] [--lc K]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="solve17")
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--lc", type=int, default=0)
args = ap.parse_args()
gen = {"solve17": lambda n: synth.make_17clue(n, seed=11), "solve30": lambda n: synth.make_30clue(n),
       "minimal": lambda n: synth.make_minimal_sym(n, threads=16), "hard": lambda n: synth.make_hard_sym(n, threads=16)}
p, s = gen[args.workload](args.n)
with SudokuEngine(0) as eng:
    if args.lc:
        eng.set_option(L.SDK_OPT_PROP32_LC, args.lc)
    h = (ctypes.c_ulonglong * 512)()
    eng.solve_batch(p[:100_000])
    eng.lib.sdk_debug_p32_stats(h)
    out, st, _ = eng.solve_batch(p)
    eng.lib.sdk_debug_p32_stats(h)
    und = eng.get_option(L.SDK_OPT_PROP32_UNDECIDED)
    a = np.array(h[:], dtype=np.float64).reshape(4, 128)
    names = ["steps", "step_live<=4", "step_live<=1", "lc_passes"]
    print(f"{args.workload} n={args.n} lc={args.lc or 'default'} undecided={und} ok={(out == s).all()}")
    for k in range(4):
        hist = a[k]
        tot = hist.sum()
        idx = np.arange(128)
        mean = (hist * idx).sum() / max(tot, 1)
        cum = np.cumsum(hist) / max(tot, 1)
        pct = [int(np.searchsorted(cum, q)) for q in (0.1, 0.5, 0.9, 0.99)]
        print(f"  {names[k]:14s} groups={int(tot)} mean={mean:.2f} p10/p50/p90/p99={pct} max={int(idx[hist > 0].max()) if tot else 0}")
