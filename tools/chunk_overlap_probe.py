"""Would one pass gain from splitting its batch over two streams? (dev tool)

Times, on the same resident boards: one solve_batch_dev pass of the whole batch on one context, and
the batch cut in two parts issued back to back on two engine contexts (own HIP streams: the second
part's kernels fill what the first part's drain and donation launch leave idle), both synchronised.
Every output is checked.  Prints ms per pass for each cut fraction.

usage: python tools/chunk_overlap_probe.py [--sets hard_1m,hard_100k,c4] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402


class _View:
    """A device pointer at an offset into a DeviceBuffer (what solve_batch_dev reads: .ptr)."""

    def __init__(self, buf, off):
        self.ptr = ctypes.c_void_p(buf.ptr.value + int(off))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", default="hard_1m,hard_100k,c4")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cuts", default="0.5,0.65,0.8")
    args = ap.parse_args()
    with SudokuEngine(0) as eng:
        eng.set_option(L.SDK_OPT_DONATE_MAX, 0)
        twin = eng.fork()
        for name in args.sets.split(","):
            if name == "hard_1m":
                p, s = synth.make_hard_sym(1_000_000, threads=16)
            elif name == "hard_100k":
                p, s, _ = synth.load_hard(threads=16)
            else:
                p, s = synth.make_17clue(10_000_000)
            n = len(p)
            d_in, d_out, d_st = eng.alloc(n * 81), eng.alloc(n * 81), eng.alloc(n)
            d_in.upload(p)
            res = {"set": name, "boards": n}

            def one():
                eng.solve_batch_dev(d_in, d_out, d_st, n)
                eng.synchronize()

            def two(k):
                # part 2 through offset views of the same buffers
                eng.solve_batch_dev(d_in, d_out, d_st, k)
                twin.solve_batch_dev(_View(d_in, k * 81), _View(d_out, k * 81), _View(d_st, k), n - k)
                eng.synchronize()
                twin.synchronize()

            for _ in range(20):          # warm the clock
                one()
            for label, fn in [("one", one)] + [(f"two@{c}", (lambda c=c: two(int(n * float(c)) // 64 * 64)))
                                             for c in args.cuts.split(",")]:
                walls = []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    fn()
                    walls.append(1000 * (time.perf_counter() - t0))
                out = np.empty((n, 81), np.uint8)
                d_out.download(out)
                res[label] = {"min_ms": round(min(walls), 3), "median_ms": round(sorted(walls)[len(walls) // 2], 3),
                              "ok": bool((out == s).all())}
            print(json.dumps(res), flush=True)
            for b in (d_in, d_out, d_st):
                b.free()
        twin.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
