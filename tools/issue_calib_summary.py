"""Summarise rocprofv3 --pmc passes over tools/issue_calib: VALU issue per SIMD quad-cycle of each
calibration kernel at 7 and 8 waves per SIMD (the instruction-mix ceilings of solve4_kernel's
compute roofline).

issue_calib launches every kernel 6 times per occupancy (one warm-up, five timed), occupancies 7
then 8 waves per SIMD; dispatches of one kernel are therefore split in order into the two
occupancies and the warm-up of each is dropped.  Units as tools/pmc_pipe_summary.py.
usage: python3 tools/issue_calib_summary.py <dir> [tag ...]   -> <dir>/issue_calib.json
"""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_pipe_summary import _rows, _name, summarize  # noqa: E402

KERNELS = ("k_int2", "k_or3", "k_b3", "k_pk", "k_mix2", "k_mix", "k_round<true>", "k_round<false>")


def kernel_of(name):
    n = _name(name)
    for k in KERNELS:
        if n.startswith(k):
            return k
    return None


def main(d, tags):
    out = {}
    for tag in tags:
        ctr = defaultdict(lambda: defaultdict(float))
        kname = {}
        for r in _rows(d, tag, "*counter_collection.csv"):
            k = kernel_of(r["Kernel_Name"])
            if k:
                ctr[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                kname[r["Dispatch_Id"]] = k
        wall = {}
        for r in _rows(d, tag, "*kernel_trace.csv"):
            if kernel_of(r["Kernel_Name"]):
                wall[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        by_k = defaultdict(list)
        for i in sorted(ctr, key=int):
            by_k[kname[i]].append(i)
        for k, ids in by_k.items():
            half = len(ids) // 2
            for wps, part in ((7, ids[:half]), (8, ids[half:])):
                rec = summarize({i: ctr[i] for i in part}, {i: wall[i] for i in part if i in wall})
                if rec:
                    rec.pop("counters", None) if tag != tags[0] else None
                    out.setdefault(f"{k}@{wps}", {})[tag] = rec
    with open(os.path.join(d, "issue_calib.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for key, recs in out.items():
        for tag, s in recs.items():
            brief = {x: (round(v, 4) if isinstance(v, float) else v) for x, v in s.items()
                     if x in ("kernel_ms", "clock_ghz", "valu_per_quad", "valu_busy_frac", "valu_dual_frac",
                              "waves_per_simd", "lds_busy_frac", "salu_per_cu_cycle")}
            print(f"{key:18s} {tag:6s} {json.dumps(brief)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:] or ["pipe"])
