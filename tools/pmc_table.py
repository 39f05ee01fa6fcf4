"""Per-kernel table of every PMC counter found under <dir>/pass*/ (rocprofv3 --pmc csv output).

Values are summed over the dispatches of each kernel (last run of the script wins per pass).
usage: python tools/pmc_table.py <dir>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, all_kernels=False):
    vals = defaultdict(lambda: defaultdict(float))
    ndisp = defaultdict(set)
    for f in sorted(glob.glob(os.path.join(d, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0]
                if not all_kernels and not k.startswith("sdk::"):
                    continue
                vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
                ndisp[k].add((f, row["Dispatch_Id"]))
    for k, cs in vals.items():
        print(f"== {k}")
        for c in sorted(cs):
            print(f"  {c:28s} {cs[c]:.6g}")
        v = cs
        if v.get("SQ_WAVE_CYCLES") and v.get("SQ_ACTIVE_INST_VALU") is not None:
            print(f"  VALU active / wave cycles   {v['SQ_ACTIVE_INST_VALU'] / v['SQ_WAVE_CYCLES']:.3f}")
        if v.get("SQ_WAVE_CYCLES") and v.get("SQ_WAIT_ANY") is not None:
            print(f"  wait_any / wave cycles      {v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES']:.3f}")
            if v.get("SQ_WAIT_INST_ANY") is not None:
                print(f"  wait_inst_any / wave cycles {v['SQ_WAIT_INST_ANY'] / v['SQ_WAVE_CYCLES']:.3f}")
            if v.get("SQ_ACTIVE_INST_ANY") is not None:
                print(f"  active_any / wave cycles    {v['SQ_ACTIVE_INST_ANY'] / v['SQ_WAVE_CYCLES']:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], "--all" in sys.argv[2:])
