"""Summarise solve_profile A/B logs (dev tool): mean ms per launch and M puzzles/s per build and
workload, from lines '<build> quad ... <workload> n=<n> solve=<ms> ms ... rate=<r> M/s ...'.

usage: python3 tools/ab_table.py <log>
"""
import re
import sys
from collections import defaultdict


def main(path):
    rows = defaultdict(list)
    order_b, order_w = [], []
    for line in open(path):
        m = re.match(r"(\S+) .*? (\w+) n=(\d+) solve=([\d.]+) ms .*rate=([\d.]+) M/s", line)
        if not m:
            continue
        b, wl, n, ms, rate = m.group(1), f"{m.group(2)}:{m.group(3)}", m.group(3), float(m.group(4)), float(m.group(5))
        rows[(b, wl)].append(rate)
        if b not in order_b:
            order_b.append(b)
        if wl not in order_w:
            order_w.append(wl)
    print("build".ljust(12) + "".join(w.ljust(18) for w in order_w))
    for b in order_b:
        cells = []
        for w in order_w:
            r = rows.get((b, w))
            cells.append((f"{sum(r) / len(r):.1f}" + (f" ({min(r):.0f}-{max(r):.0f})" if len(r) > 1 else "")) if r else "-")
        print(b.ljust(12) + "".join(c.ljust(18) for c in cells))


if __name__ == "__main__":
    main(sys.argv[1])
