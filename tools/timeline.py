"""Per-workgroup launch timeline of solve4_kernel (dev tool): load the timeline build
(tools/build_variant.sh tl -DSDK_SOLVE4_TIMELINE=1) through SDK_LIB_PATH; for each shard size,
one C4 launch split into dispatch ramp (workgroup start times), start-up (first boards held),
steady work and drain (last dequeue -> exit), in microseconds from the first workgroup's start.

usage: SDK_LIB_PATH=$PWD/build/variants/lib_tl.so python tools/timeline.py [--sizes 1250000,10000000]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402


def pct(x):
    return {k: float(np.percentile(x, q)) for k, q in (("min", 0), ("p10", 10), ("p50", 50), ("p90", 90),
                                                         ("p99", 99), ("max", 100))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1250000,10000000")
    ap.add_argument("--workload", default="solve17")
    ap.add_argument("--json", default="")
    ap.add_argument("--order", default="lex", choices=["lex", "mrv_unique"])
    args = ap.parse_args()
    lib = L.load()
    fn = lib.sdk_debug_tl4
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    res = {}
    with SudokuEngine(0) as eng:
        cus = eng.get_option(L.SDK_OPT_DEVICE_CUS)
        grid_max = cus * eng.get_option(L.SDK_OPT_WAVES_PER_CU2)
        eng.set_option(L.SDK_OPT_DONATE, 0)          # one launch: the timeline of that launch
        eng.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX if args.order == "lex" else L.SDK_ORDER_MRV_UNIQUE)
        for n in [int(x) for x in args.sizes.split(",")]:
            if args.workload == "hard":
                p, s = synth.make_hard_sym(n, threads=16)
            elif args.workload == "minimal":
                p, s = synth.make_minimal_sym(n, threads=16)
            else:
                gen = synth.make_17clue if args.workload == "solve17" else synth.make_30clue
                p, s = gen(n, seed=11)
            d_in, d_out, d_st = eng.alloc(n * 81), eng.alloc(n * 81), eng.alloc(n)
            d_in.upload(p)
            buf = (ctypes.c_ulonglong * (16384 * 4))()
            for rep in range(3):
                eng.timer_reset()
                eng.solve_batch_dev(d_in, d_out, d_st, n)
                eng.synchronize()
                ms, _ = eng.timer_read()
                assert fn(buf, 16384) == 0
            t = np.array(list(buf), dtype=np.float64).reshape(16384, 4)
            g = int((t[:, 0] > 0).sum())
            t = t[:g]
            t0 = t[:, 0].min()
            us = (t - t0) / 100.0          # 100 MHz ticks -> us
            last_deq = us[:, 2][us[:, 2] > 0]
            r = {"boards": n, "kernel_ms_hip_events": ms, "workgroups": g, "grid_max": grid_max,
                 "start_us": pct(us[:, 0]), "first_boards_us": pct(us[:, 1] - us[:, 0]),
                 "last_dequeue_us": pct(last_deq), "exit_us": pct(us[:, 3]),
                 "drain_us": float(us[:, 3].max() - np.median(last_deq)),
                 "span_us": float(us[:, 3].max())}
            # per XCD (workgroup % 8: the dispatch's round robin): when its segment work ends
            xcd = np.arange(g) % 8
            r["per_xcd"] = {int(k): {"last_dequeue_p50": float(np.median(us[xcd == k, 2])),
                                     "last_dequeue_max": float(us[xcd == k, 2].max()),
                                     "exit_p50": float(np.median(us[xcd == k, 3])),
                                     "exit_max": float(us[xcd == k, 3].max())} for k in range(8)}
            res[str(n)] = r
            print(json.dumps(r), flush=True)
            out = np.empty((n, 81), np.uint8)
            d_out.download(out)
            assert (out == s).all()
            for b in (d_in, d_out, d_st):
                b.free()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
