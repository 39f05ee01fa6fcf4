"""Per-dispatch sums of every counter of tools/pmc_sq.sh's pass, for the solve kernels (dev tool)."""
import csv, glob, os, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].strip()
        if "solve" in k:
            per[(k, row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
for (k, d), cs in sorted(per.items()):
    print(k, d, " ".join(f"{c}={v:.4g}" for c, v in sorted(cs.items())))
