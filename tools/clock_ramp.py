"""Clock ramp of the C4 launch from a cold GPU (dev tool): back-to-back prop32 passes over 10M resident
17-clue puzzles with the stamped twin of the kernel (sdk_debug_clock_arm), each pass synchronised and
timed by its HIP events, printing per pass: the kernel's duration and its workgroups' median in-kernel
clock (s_memtime / s_memrealtime, MI355X_MICROARCH.md "DVFS give-back" item 6).  Shows whether the
first passes' extra time is the clock.

usage: python tools/clock_ramp.py [--n 10000000] [--passes 40] [--idle-ms 0]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--passes", type=int, default=40)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep between passes")
    args = ap.parse_args()
    p, s = synth.make_17clue(args.n)
    with SudokuEngine(0) as eng:
        lib = eng.lib
        d_in, d_out, d_st = eng.alloc(args.n * 81), eng.alloc(args.n * 81), eng.alloc(args.n)
        d_in.upload(p)
        eng.synchronize()
        time.sleep(1.0)                      # let the GPU drop to idle first
        L.check(lib.sdk_debug_clock_arm(eng.ctx, 1), "arm")
        eng.timer_reset()
        out4 = (ctypes.c_double * 4)()
        wgs = ctypes.c_int64()
        rows = []
        t0 = time.perf_counter()
        for i in range(args.passes):
            eng.solve_batch_dev(d_in, d_out, d_st, args.n)
            L.check(lib.sdk_debug_clock_read(eng.ctx, out4, ctypes.byref(wgs)), "read")
            rows.append({"pass": i, "t_ms": 1000 * (time.perf_counter() - t0), "ghz": round(out4[0], 4),
                         "ghz_p10": round(out4[1], 4), "ghz_p90": round(out4[2], 4)})
            if args.idle_ms:
                time.sleep(args.idle_ms / 1000)
        cap = 1 << 10
        arr = (ctypes.c_double * cap)()
        cnt = ctypes.c_int64()
        L.check(lib.sdk_debug_timer_list(eng.ctx, arr, ctypes.c_int64(cap), ctypes.byref(cnt)), "timer")
        spans = list(arr[:cnt.value])
        for r in rows:                       # two spans per prop32 solve: the pass, then its fallback
            r["kernel_ms"] = round(spans[2 * r["pass"]], 4) if 2 * r["pass"] < len(spans) else None
            print(json.dumps(r), flush=True)
        lib.sdk_debug_clock_arm(eng.ctx, 0)
        for b in (d_in, d_out, d_st):
            b.free()
    return 0


if __name__ == "__main__":
    sys.exit(main())
