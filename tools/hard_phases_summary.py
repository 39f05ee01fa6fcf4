"""Summary of a rocprofv3 --kernel-trace of tools/hard_phases.py (dev tool).

Splits the dispatches into passes at gaps > 1 ms, and for the last passes of each batch prints
every dispatch (start and end relative to the pass's first dispatch, duration, grid) and the pass's
busy and idle time (sum of gaps between consecutive dispatches).

usage: python3 tools/hard_phases_summary.py <trace dir> [--last 3]
"""
import csv
import glob
import os
import sys


def main(d, last=3):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ds = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sdk::", ""),
           int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Grid_Size", r.get("Grid_Size_X", "")))
          for r in rows]
    passes, cur = [], []
    for k in ds:
        if cur and k[1] - max(e for _, _, e, _ in cur) > 1_000_000:
            passes.append(cur)
            cur = []
        cur.append(k)
    if cur:
        passes.append(cur)
    print(f"{len(ds)} dispatches, {len(passes)} passes")
    for i, p in enumerate(passes):
        t0 = p[0][1]
        end = max(e for _, _, e, _ in p)
        busy, idle, prev = 0, 0, t0
        for _, s, e, _ in p:
            if s > prev:
                idle += s - prev
            busy += e - s
            prev = max(prev, e)
        print(f"pass {i}: span {(end - t0) / 1e3:.1f} us, idle {idle / 1e3:.1f} us, {len(p)} dispatches")
        if i >= len(passes) - last or len(passes) <= last:
            for name, s, e, grid in p:
                print(f"    {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f} {grid:>9} {name}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3))
