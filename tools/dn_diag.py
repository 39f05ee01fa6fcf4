"""Subtree-donation diagnostics on the GPU (dev tool): launch time, items donated and summed
search nodes with SDK_OPT_DONATE on and off, per workload and node budget.

    python tools/dn_diag.py [--n 100000] [--workload hard|minimal|solve17]
"""
import argparse
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--workload", default="hard")
    ap.add_argument("--budgets", default="0,100000,1000")
    ap.add_argument("--splits", default="1")
    ap.add_argument("--resume", default="1", help="SDK_OPT_DONATE_RESUME values to run, e.g. 1,0")
    args = ap.parse_args()
    if args.workload == "hard":
        p, s = synth.make_hard_sym(args.n, threads=16)
    elif args.workload == "heavy":
        p, s = synth.make_hard_heaviest(args.n, threads=16)
    elif args.workload == "minimal":
        p, s = synth.make_minimal_sym(args.n, threads=16)
    else:
        p, s = synth.make_17clue(args.n, seed=11)
    with SudokuEngine(0) as eng:
        eng.set_option(L.SDK_OPT_TIMING, 1)
        for budget, dn, rs in [(b, d, r) for b in [int(x) for x in args.budgets.split(",")]
                               for d in [0] + [int(x) for x in args.splits.split(",")]
                               for r in ([1] if d == 0 else [int(x) for x in args.resume.split(",")])]:
            if True:
                eng.set_option(L.SDK_OPT_DONATE, dn)
                eng.set_option(L.SDK_OPT_DONATE_RESUME, rs)
                eng.solve_batch(p[:1024], want_work=True, budget=budget)
                eng.timer_reset()
                t0 = time.time()
                out, st, work = eng.solve_batch(p, want_work=True, budget=budget)
                wall = time.time() - t0
                ms, nl = eng.timer_read()
                lst = (ctypes.c_double * 16)()
                cnt = ctypes.c_int64()
                eng.lib.sdk_debug_timer_list(eng.ctx, lst, ctypes.c_int64(16), ctypes.byref(cnt))
                print(f"  launches: {[round(lst[i], 3) for i in range(min(cnt.value, 16))]}", flush=True)
                donated = eng.get_option(L.SDK_OPT_DONATED) if dn else 0
                if dn:
                    ctl = (ctypes.c_uint32 * 16)()
                    eng.lib.sdk_debug_dn_ctl(eng.ctx, ctl)
                    c = list(ctl)
                    print(f"  ctl: epoch={c[0]} delivered={c[1]} items={c[2]} nrec={c[3]} exit_all={c[4]} "
                          f"parts_ended={c[5]} finalized={c[6]} err={c[8]} grid={c[10]} helpers={c[11]} "
                          f"split_boards={eng.get_option(L.SDK_OPT_SPLIT_BOARDS)}",
                          flush=True)
                ok = (out[st == 1] == s[st == 1]).all()
                resumed = eng.get_option(L.SDK_OPT_RESUMED) if dn else 0
                print(f"{args.workload} n={args.n} budget={budget} donate={dn} resume={rs} resumed={resumed}: "
                      f"kernels {ms:.2f} ms "
                      f"wall {wall * 1e3:.1f} ms donated={donated} solved={int((st == 1).sum())} "
                      f"hit={int((st == -2).sum())} nodes sum={int(work.sum())} max={int(work.max())} ok={ok}",
                      flush=True)
        eng.set_option(L.SDK_OPT_DONATE, 0)
        for kind, name in ((L.SDK_WORK_NODES, "nodes"), (L.SDK_WORK_ROUNDS, "rounds")):
            eng.set_option(L.SDK_OPT_WORK_COUNTER, kind)
            _, _, w = eng.solve_batch(p, want_work=True)
            w = w.astype(np.int64)
            print(f"{name}/board: mean={w.mean():.1f} p50={np.median(w):.0f} p90={np.percentile(w, 90):.0f} "
                  f"p99={np.percentile(w, 99):.0f} p99.9={np.percentile(w, 99.9):.0f} max={w.max()} sum={w.sum()}",
                  flush=True)
        eng.set_option(L.SDK_OPT_WORK_COUNTER, L.SDK_WORK_NODES)
        eng.set_option(L.SDK_OPT_DONATE, 1)
        # a few heavy boards alone (the whole grid idle): donation at its most
        eng.set_option(L.SDK_OPT_DONATE, 0)
        _, _, w = eng.solve_batch(p[:20000], want_work=True)
        idx = np.argsort(-w.astype(np.int64))[:64]
        for dn in (0, 1, 16):
            eng.set_option(L.SDK_OPT_DONATE, dn)
            eng.timer_reset()
            out, st, work = eng.solve_batch(p[idx], want_work=True)
            ms, nl = eng.timer_read()
            lst = (ctypes.c_double * 16)()
            cnt = ctypes.c_int64()
            eng.lib.sdk_debug_timer_list(eng.ctx, lst, ctypes.c_int64(16), ctypes.byref(cnt))
            print(f"  launches: {[round(lst[i], 3) for i in range(min(cnt.value, 16))]}", flush=True)
            donated = eng.get_option(L.SDK_OPT_DONATED) if dn else 0
            print(f"64 heaviest: donate={dn} kernel {ms:.3f} ms donated={donated} nodes={work.tolist()[:8]} "
                  f"ok={(out == s[idx]).all()}", flush=True)
        eng.set_option(L.SDK_OPT_DONATE, 1)


if __name__ == "__main__":
    main()
