"""Phase structure of the hard-search passes (dev tool; run under rocprofv3 --kernel-trace).

Times `--reps` single-context passes of each hard batch in the bench's default mode (prop32 pass,
then the phased solve: split phase, donation, LEX re-solve, scatters), one synchronize per pass, and
prints each pass's wall time.  Under `rocprofv3 --kernel-trace` every dispatch of every pass is in
the trace: `tools/hard_phases_summary.py <dir>` splits it into passes and reports, per kernel, its
span and the gaps between kernels (the GPU idle inside a pass).

usage: python tools/hard_phases.py [--sets hard_1m,hard_100k,heaviest_1000,minimal_1m] [--reps 5] [--order lex|mrv]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", default="hard_1m,hard_100k")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--order", default="lex", choices=["lex", "mrv"])
    ap.add_argument("--donate", type=int, default=1)
    ap.add_argument("--opt", action="append", default=[], help="NAME=VALUE SDK_OPT_* option")
    args = ap.parse_args()
    with SudokuEngine(0) as eng:
        eng.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX if args.order == "lex" else L.SDK_ORDER_MRV_UNIQUE)
        eng.set_option(L.SDK_OPT_DONATE, args.donate)
        eng.set_option(L.SDK_OPT_DONATE_MAX, 0)
        for kv in args.opt:
            k, v = kv.split("=", 1)
            eng.set_option(getattr(L, "SDK_OPT_" + k), int(v))
        for name in args.sets.split(","):
            if name == "hard_1m":
                p, s = synth.make_hard_sym(1_000_000, threads=16)
            elif name == "hard_100k":
                p, s, _ = synth.load_hard(threads=16)
            elif name == "heaviest_1000":
                p, s = synth.make_hard_heaviest(1000, threads=16)
            elif name == "minimal_1m":    # the bench's minimal leg
                p, s = synth.make_minimal_sym(1_048_576, base=65536, threads=16)
            else:
                raise SystemExit(f"unknown set {name}")
            n = len(p)
            d_in, d_out, d_st = eng.alloc(n * 81), eng.alloc(n * 81), eng.alloc(n)
            d_in.upload(p)
            eng.solve_batch_dev(d_in, d_out, d_st, n)
            eng.synchronize()
            walls = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                eng.solve_batch_dev(d_in, d_out, d_st, n)
                eng.synchronize()
                walls.append(1000 * (time.perf_counter() - t0))
                time.sleep(0.002)          # a visible gap between passes in the trace
            out = np.empty((n, 81), np.uint8)
            d_out.download(out)
            bad = int((out != s).any(axis=1).sum())
            print(json.dumps({"set": name, "boards": n, "wall_ms": walls, "min_ms": min(walls),
                              "split_boards": eng.get_option(L.SDK_OPT_SPLIT_BOARDS),
                              "undecided_by_prop32": eng.get_option(L.SDK_OPT_PROP32_UNDECIDED),
                              "mismatched": bad}), flush=True)
            for b in (d_in, d_out, d_st):
                b.free()
            if bad:
                return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
