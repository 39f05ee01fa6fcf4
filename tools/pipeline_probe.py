"""Batches in flight on one GPU (dev tool): K back-to-back C4 solve passes over one resident batch,
issued on P engine contexts in turn (each its own HIP stream, dequeue state and DFS stacks; its own
output buffer), so that one launch's drain overlaps the next launch's start.  Prints ms per pass
and puzzles/s for every size and P, and checks every output buffer against the known solutions.

usage: python tools/pipeline_probe.py [--sizes 1250000,10000000] [--contexts 1,2,3] [--steps 6]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from distributed_sudoku_solver_amd import SudokuEngine, synth  # noqa: E402


def run(eng, puzzles, expected, contexts, steps, reps):
    n = len(puzzles)
    engines = [eng] + [eng.fork() for _ in range(contexts - 1)]
    d_in = eng.alloc(n * 81)
    d_in.upload(puzzles)
    outs = [(e.alloc(n * 81), e.alloc(n)) for e in engines]
    for e, (o, st) in zip(engines, outs):
        e.solve_batch_dev(d_in, o, st, n)
    for e in engines:
        e.synchronize()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        for i in range(steps):
            o, st = outs[i % contexts]
            engines[i % contexts].solve_batch_dev(d_in, o, st, n)
        for e in engines:
            e.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    bad = 0
    for o, st in outs:
        out = np.empty((n, 81), np.uint8)
        s = np.empty(n, np.int8)
        o.download(out)
        st.download(s)
        bad += int(((out != expected).any(axis=1) | (s != 1)).sum())
    for o, st in outs:
        o.free()
        st.free()
    d_in.free()
    for e in engines[1:]:
        e.close()
    return best / steps, bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1250000,2500000,10000000")
    ap.add_argument("--contexts", default="1,2,3")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    with SudokuEngine(0) as eng:
        for n in [int(x) for x in args.sizes.split(",")]:
            p, s = synth.make_17clue(n, seed=11)
            for c in [int(x) for x in args.contexts.split(",")]:
                per, bad = run(eng, p, s, c, args.steps, args.reps)
                print(f"n={n} contexts={c} steps={args.steps}: {per * 1e3:.3f} ms per pass, "
                      f"{n / per / 1e6:.1f} M puzzles/s, bad={bad}", flush=True)


if __name__ == "__main__":
    main()
