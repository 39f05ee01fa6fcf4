"""Solve-kernel profiling driver (dev tool, not a test): timing, search nodes and propagation
rounds per puzzle, and a fixed workload for rocprofv3 --pmc passes.

usage: python tools/solve_profile.py [--n N] [--workload solve17|solve30] [--reps R] [--stats]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=2_000_000)
ap.add_argument("--workload", default="solve17")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--stats", action="store_true")
ap.add_argument("--waves-per-cu", type=int, default=0)
ap.add_argument("--solver", default="halfwave", choices=["halfwave", "wave", "quad", "lane"])
ap.add_argument("--sweep", action="store_true", help="time waves-per-CU settings")
ap.add_argument("--budget", type=int, default=0, help="SDK_OPT_NODE_BUDGET (LANE: reference validations)")
ap.add_argument("--xcd-heads", type=int, default=-1, help="QUAD: SDK_OPT_XCD_HEADS (default: library default)")
ap.add_argument("--chunk", type=int, default=0, help="SDK_OPT_SOLVE_CHUNK (0: automatic)")
ap.add_argument("--order", default="lex", choices=["mrv_unique", "lex"])
ap.add_argument("--locked", type=int, default=1, help="QUAD: locked-candidates pass (SDK_OPT_LOCKED: 0 off, 1 root, 2 all nodes)")
ap.add_argument("--donate", type=int, default=-1, help="QUAD: SDK_OPT_DONATE (default: library default)")
ap.add_argument("--donate-mode", type=int, default=-1, help="QUAD: SDK_OPT_DONATE_MODE (1 exhaustive, 0 LEX)")
ap.add_argument("--donate-max", type=int, default=-1, help="QUAD: SDK_OPT_DONATE_MAX (0: phased at any size)")
ap.add_argument("--helpers", type=int, default=0, help="QUAD: SDK_OPT_DONATE_HELPERS (waves per tail board)")
ap.add_argument("--resume", type=int, default=-1, help="QUAD: SDK_OPT_DONATE_RESUME (default: library default)")
ap.add_argument("--prop32", type=int, default=-1, help="QUAD: SDK_OPT_PROP32 (default: library default)")
ap.add_argument("--prop32-lc", type=int, default=0, help="QUAD: SDK_OPT_PROP32_LC (0: library default)")
ap.add_argument("--prop32-tail", type=int, default=-1, help="QUAD: SDK_OPT_PROP32_TAIL (live | step << 8)")
args = ap.parse_args()

if args.workload == "minimal":
    p, s = synth.make_minimal_sym(args.n, threads=16)
elif args.workload == "hard":
    p, s = synth.make_hard_sym(args.n, threads=16)
elif args.workload == "heavy":
    p, s = synth.make_hard_heaviest(args.n, threads=16)
else:
    gen = synth.make_17clue if args.workload == "solve17" else synth.make_30clue
    p, s = gen(args.n, seed=11)
with SudokuEngine(0) as eng:
    eng.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX if args.order == "lex" else L.SDK_ORDER_MRV_UNIQUE)
    eng.set_option(L.SDK_OPT_LOCKED, args.locked)
    eng.set_option(L.SDK_OPT_SOLVER, {"halfwave": L.SDK_SOLVER_HALFWAVE, "wave": L.SDK_SOLVER_WAVE,
                                      "quad": L.SDK_SOLVER_QUAD, "lane": L.SDK_SOLVER_LANE}[args.solver])
    wopt = L.SDK_OPT_WAVES_PER_CU if args.solver == "wave" else L.SDK_OPT_WAVES_PER_CU2
    if args.budget:
        eng.set_option(L.SDK_OPT_NODE_BUDGET, args.budget)
    if args.chunk:
        eng.set_option(L.SDK_OPT_SOLVE_CHUNK, args.chunk)
    if args.xcd_heads >= 0:
        eng.set_option(L.SDK_OPT_XCD_HEADS, args.xcd_heads)
    if args.donate >= 0:
        eng.set_option(L.SDK_OPT_DONATE, args.donate)
    if args.donate_mode >= 0:
        eng.set_option(L.SDK_OPT_DONATE_MODE, args.donate_mode)
    if args.donate_max >= 0:
        eng.set_option(L.SDK_OPT_DONATE_MAX, args.donate_max)
    if args.helpers:
        eng.set_option(L.SDK_OPT_DONATE_HELPERS, args.helpers)
    if args.resume >= 0:
        eng.set_option(L.SDK_OPT_DONATE_RESUME, args.resume)
    if args.waves_per_cu:
        eng.set_option(wopt, args.waves_per_cu)
    if args.prop32 >= 0 and hasattr(L, "SDK_OPT_PROP32"):
        eng.set_option(L.SDK_OPT_PROP32, args.prop32)
    if args.prop32_lc and hasattr(L, "SDK_OPT_PROP32_LC"):
        eng.set_option(L.SDK_OPT_PROP32_LC, args.prop32_lc)
    if args.prop32_tail >= 0:
        eng.set_option(L.SDK_OPT_PROP32_TAIL, args.prop32_tail)
    d_in, d_out, d_st = eng.alloc(args.n * 81), eng.alloc(args.n * 81), eng.alloc(args.n)
    d_in.upload(p)
    eng.solve_batch_dev(d_in, d_out, d_st, args.n)
    eng.synchronize()
    eng.timer_reset()
    for _ in range(args.reps):
        eng.solve_batch_dev(d_in, d_out, d_st, args.n)
    eng.synchronize()
    ms, nl = eng.timer_read()
    out = np.empty((args.n, 81), np.uint8)
    d_out.download(out)
    per = ms / args.reps       # one solve: one launch, or both launches of a two-phase solve
    p32 = (f" p32={args.prop32}/{args.prop32_lc}/t{args.prop32_tail}"
           if args.prop32 >= 0 or args.prop32_lc or args.prop32_tail >= 0 else "")
    print(f"{args.solver} {args.order} lc={args.locked} xh={args.xcd_heads} dn={args.donate}/{args.donate_mode}/h{args.helpers} chunk={args.chunk}{p32} {args.workload} n={args.n} solve={per:.3f} ms "
          f"({nl // args.reps} launches) rate={args.n / per * 1e3 / 1e6:.1f} M/s ok={(out == s).all()}", flush=True)
    if args.sweep:
        for wpc in (8, 12, 16, 20, 24, 32):
            eng.set_option(wopt, wpc)
            eng.solve_batch_dev(d_in, d_out, d_st, args.n)
            eng.synchronize()
            eng.timer_reset()
            eng.solve_batch_dev(d_in, d_out, d_st, args.n)
            eng.synchronize()
            ms, _ = eng.timer_read()
            print(f"  {args.solver} waves/CU={wpc}: {ms:.3f} ms  {args.n / ms * 1e3 / 1e6:.1f} M/s", flush=True)
    if args.stats:
        m = min(args.n, 200_000)
        for kind, name in ((L.SDK_WORK_NODES, "nodes"), (L.SDK_WORK_ROUNDS, "rounds")):
            eng.set_option(L.SDK_OPT_WORK_COUNTER, kind)
            _, _, w = eng.solve_batch(p[:m], want_work=True)
            print(f"{name}/puzzle: mean={w.mean():.2f} p50={np.median(w):.0f} p90={np.percentile(w, 90):.0f} "
                  f"p99={np.percentile(w, 99):.0f} max={w.max()}", flush=True)
        eng.set_option(L.SDK_OPT_WORK_COUNTER, L.SDK_WORK_NODES)
    for b in (d_in, d_out, d_st):
        b.free()
