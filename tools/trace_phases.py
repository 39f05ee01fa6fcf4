"""Per-dispatch kernel sequence of rocprofv3 kernel traces (dev tool; rocprofv3 --kernel-trace runs of tools/gpu_round.sh).

usage: python3 tools/trace_phases.py <dir> <variant>...   (reads <dir>/<variant>/**/*kernel_trace.csv)
Writes <dir>/phases_<variant>.txt (every dispatch: name, duration us, grid) and prints the
donation-kernel dispatches (solve4_kernel<true>) and the plain ones above 50 us, in order.
"""
import csv
import glob
import os
import sys


def dispatches(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sdk::", "")
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        out.append((name, us, r.get("Grid_Size", r.get("Grid_Size_X", "")), int(r["Start_Timestamp"])))
    return out


def main(d, variants):
    for v in variants:
        ds = dispatches(os.path.join(d, v))
        if not ds:
            print(f"{v}: no trace")
            return 1
        t0 = ds[0][3]
        with open(os.path.join(d, f"phases_{v}.txt"), "w") as fh:
            for name, us, grid, ts in ds:
                fh.write(f"{(ts - t0) / 1e3:12.1f} {us:9.1f} {grid:>9} {name}\n")
        sel = [f"{name[:22]}:{us:.0f}" for name, us, _, _ in ds
               if "solve4_kernel<true>" in name and us > 5 or ("solve4_kernel<false>" in name and us > 50)]
        print(v, " ".join(sel))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2:]))
