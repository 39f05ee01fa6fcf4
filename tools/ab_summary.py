"""Table of tools/ab_opts.sh logs: per workload and setting, the solve times (ms) of every repeat."""
import collections
import re
import sys

d = collections.defaultdict(list)
for path in sys.argv[1:]:
    for line in open(path):
        m = re.match(r'\[(.*?)\].* (\w+) n=(\d+) solve=([\d.]+) ms.*ok=(\w+)', line)
        if m:
            d[(m.group(2), m.group(3), m.group(1))].append(float(m.group(4)) if m.group(5) == "True" else float("nan"))
for w in sorted(set(k[:2] for k in d)):
    print(f"{w[0]} n={w[1]}")
    for k, v in d.items():
        if k[:2] == w:
            print(f"   {k[2]:22s} " + " ".join(f"{x:.3f}" for x in v) + f"   min {min(v):.3f}")
