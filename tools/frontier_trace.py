"""Per-level durations of a frontier build from a rocprofv3 kernel trace (dev tool): every
expand / scan / emit dispatch of tools/frontier_levels.py's last build, in order.
usage: python3 tools/frontier_trace.py <run_kernel_trace.csv>
"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
# the last build: dispatches after the last host gap of more than 0.5 ms
cut = 0
for i in range(1, len(rows)):
    if rows[i][0] - rows[i - 1][1] > 500_000:
        cut = i
build = rows[cut:]
t0 = build[0][0]
total = {}
for s, e, n in build:
    total[n] = total.get(n, 0) + (e - s)
    if "expand" in n:
        print(f"{(s - t0) / 1e3:9.1f} us  {n:40s} {(e - s) / 1e3:8.1f} us")
print("per kernel (us):", {k: round(v / 1e3, 1) for k, v in sorted(total.items(), key=lambda x: -x[1])})
print(f"build span {(build[-1][1] - t0) / 1e3:.1f} us")
