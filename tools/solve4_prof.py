"""Cycle breakdown of solve4_kernel (dev tool): load the profiling build
(tools/build_variant.sh prof -DSDK_SOLVE4_PROFILE=1) through SDK_LIB_PATH and print where
the waves' shader-clock cycles go per solved puzzle.

usage: SDK_LIB_PATH=build/variants/lib_prof.so python tools/solve4_prof.py [--n N] [--workload ..] [--locked 0|1]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=2_000_000)
ap.add_argument("--workload", default="solve17")
ap.add_argument("--locked", type=int, default=1)
args = ap.parse_args()
if args.workload == "minimal":
    p, s = synth.make_minimal_sym(args.n, threads=16)
else:
    gen = synth.make_17clue if args.workload == "solve17" else synth.make_30clue
    p, s = gen(args.n, seed=11)
NAMES = ["round4", "step slot0", "step slot1", "finish+next board", "locked cands", "backtrack", "branch", "-",
         "whole loop", "iterations"]
with SudokuEngine(0) as eng:
    lib = L.load()
    fn = lib.sdk_debug_prof4
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 10)()
    eng.set_option(L.SDK_OPT_LOCKED, args.locked)
    out, st, _ = eng.solve_batch(p)
    assert (out == s).all()
    fn(buf, 1)
    out, st, _ = eng.solve_batch(p)
    fn(buf, 1)
    v = np.array(list(buf), dtype=np.float64)
    print(f"{args.workload} n={args.n} locked={args.locked}: per puzzle (wave cycles), iterations/puzzle "
          f"{v[9] / args.n * 4:.2f} (x4 boards per wave)")
    for k in range(9):
        if NAMES[k] != "-":
            print(f"  {NAMES[k]:>18}: {v[k] / args.n:10.1f}   ({v[k] / v[8] * 100:5.1f} % of loop)")
