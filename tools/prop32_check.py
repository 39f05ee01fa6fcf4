"""prop32 bring-up check (dev tool, GPU): the same batches solved with SDK_OPT_PROP32 on and off must
give byte-identical outputs and statuses; prints the boards the propagation pass left to the search
and the timed solve span (SDK_OPT_TIMING) of both.

usage: python tools/prop32_check.py [--quick]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import _lib as L  # noqa: E402
from distributed_sudoku_solver_amd import synth  # noqa: E402
from distributed_sudoku_solver_amd.engine import SudokuEngine  # noqa: E402


def edge_boards(n, seed=5):
    """A mix of the cases the pass must leave alone or decide exactly: out-of-domain and duplicated
    givens, contradictions, complete grids (valid and not), the empty board -- built on 37-clue
    boards so the plain solver's search stays short on the broken ones."""
    rng = np.random.default_rng(seed)
    base, _ = synth.make_30clue(n, seed=seed, extra=20)
    sol, _ = synth.make_30clue(n, seed=seed + 1, extra=64)   # complete grids
    out = base.copy()
    kind = rng.integers(0, 8, n)
    for i in range(n):
        k = kind[i]
        if k == 1:                      # an out-of-domain given
            c = rng.integers(0, 81)
            out[i, c] = rng.integers(10, 256)
        elif k == 2:                    # a duplicated given in a row
            r = rng.integers(0, 9)
            row = out[i, 9 * r:9 * r + 9]
            nz = np.flatnonzero(row)
            z = np.flatnonzero(row == 0)
            if len(nz) and len(z):
                out[i, 9 * r + z[0]] = row[nz[0]]
        elif k == 3:                    # a complete grid
            out[i] = sol[i]
        elif k == 4:                    # a complete grid with one wrong digit: contradiction
            out[i] = sol[i]
            c = rng.integers(0, 81)
            out[i, c] = out[i, c] % 9 + 1
        elif k == 5:
            out[i] = 0                  # the empty board: many completions
        elif k == 6:                    # a complete grid with holes and one wrong given
            out[i] = sol[i]
            out[i, rng.choice(81, 40, replace=False)] = 0
            nz = np.flatnonzero(out[i])
            c = nz[rng.integers(0, len(nz))]
            out[i, c] = out[i, c] % 9 + 1
    return out


def run(e, boards, prop, order, opts=()):
    e.set_option(L.SDK_OPT_PROP32, prop)
    e.set_option(L.SDK_OPT_ORDER, order)
    for k, v in opts:
        e.set_option(k, v)
    e.solve_batch(boards[:8192])
    e.timer_reset()
    t = time.perf_counter()
    out, st, _ = e.solve_batch(boards)
    wall = time.perf_counter() - t
    ms, nt = e.timer_read()
    e.timer_stop()
    und = e.get_option(L.SDK_OPT_PROP32_UNDECIDED) if prop else -1
    return out, st, ms, wall, und


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--variants", default="default",
                    help="comma list of prop32 settings to check: default, nohandover, tail<live>x<step>")
    args = ap.parse_args()
    variants = []
    for v in args.variants.split(","):
        if v == "default":
            variants.append((v, ((L.SDK_OPT_PROP32_HANDOVER, 1), (L.SDK_OPT_PROP32_TAIL, 0))))
        elif v == "nohandover":
            variants.append((v, ((L.SDK_OPT_PROP32_HANDOVER, 0), (L.SDK_OPT_PROP32_TAIL, 0))))
        elif v.startswith("tail"):
            live, step = (int(t) for t in v[4:].split("x"))
            variants.append((v, ((L.SDK_OPT_PROP32_HANDOVER, 1), (L.SDK_OPT_PROP32_TAIL, live | step << 8))))
    e = SudokuEngine(0)
    q = args.quick
    work = [
        ("c4_17clue", synth.make_17clue(200_000 if q else 1_000_000, seed=11)[0]),
        ("30clue", synth.make_30clue(100_000 if q else 500_000)[0]),
        ("minimal", synth.make_minimal_sym(65536 if q else 262144, threads=8)[0]),
        ("hard", synth.make_hard_sym(16384 if q else 65536)[0]),
        ("edge_4133", edge_boards(4096 + 37)),
        ("edge_20000", edge_boards(20000, seed=9)),
    ]
    bad = 0
    for name, boards in work:
        for order, oname in ((L.SDK_ORDER_LEX, "lex"), (L.SDK_ORDER_MRV_UNIQUE, "mrv")):
          o0, s0, ms0, w0, _ = run(e, boards, 0, order)
          for vname, opts in variants:
            o1, s1, ms1, w1, und = run(e, boards, 1, order, opts)
            mo = int(np.count_nonzero((o0 != o1).any(axis=1)))
            ms_ = int(np.count_nonzero(s0 != s1))
            bad += mo + ms_
            stc = {int(k): int(v) for k, v in zip(*np.unique(s1, return_counts=True))}
            print(f"{name:12s} {oname} {vname:10s} n={len(boards):8d} undecided={und:8d} out_mismatch={mo} "
                  f"status_mismatch={ms_} solve_ms off={ms0:8.3f} on={ms1:8.3f} speedup={ms0 / max(ms1, 1e-9):5.2f} "
                  f"statuses={stc}", flush=True)
            if mo or ms_:
                i = int(np.flatnonzero((o0 != o1).any(axis=1) | (s0 != s1))[0])
                print("  first mismatch", i, "status", s0[i], s1[i])
                print("  in ", boards[i].tolist())
                print("  off", o0[i].tolist())
                print("  on ", o1[i].tolist())
    print("MISMATCHES", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
