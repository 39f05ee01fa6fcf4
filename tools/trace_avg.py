"""Average duration of the last K dispatches of a kernel in a rocprofv3 kernel trace (dev tool):
the timed launches of a bench leg, without its warm-up launches.
usage: python3 tools/trace_avg.py <run_kernel_trace.csv> <kernel-substring> <K> [bytes-per-launch]
"""
import csv
import sys

path, name, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
nbytes = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        if name in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rows.sort()
last = rows[-k:]
d = [(e - s) / 1e6 for s, e in last]
avg = sum(d) / len(d)
print(f"{name}: {len(rows)} dispatches, last {len(d)}: avg {avg:.4f} ms, min {min(d):.4f}, max {max(d):.4f}")
if nbytes:
    print(f"  {nbytes / (avg / 1e3) / 1e12:.3f} TB/s = {nbytes / (avg / 1e3) / 8e12 * 100:.1f} % of 8 TB/s")
