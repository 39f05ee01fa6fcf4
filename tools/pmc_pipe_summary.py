"""Summarise tools/pmc_r04.sh: what bounds solve4_kernel per SIMD.

Per pass (c4 / hard1m / min), for the plain solve4_kernel dispatches (the first dispatch of
each run is a warm-up and is dropped when there are more):
  clock_ghz           GRBM_GUI_ACTIVE / 8 / kernel wall (MI355X_MICROARCH.md "DVFS give-back":
                      rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs)
  simd_cycles         SQ_CYCLES (clock cycles, summed over every SIMD)
  valu_issue_frac     SQ_INSTS_VALU / (simd_cycles / 2): VALU issue against the SIMD's peak of one
                      wave64 VALU instruction per 2 cycles (two per quad-cycle, SQ_ACTIVE_INST_VALU2)
  valu_dual_frac      SQ_ACTIVE_INST_VALU2 / (simd_cycles / 4): quad-cycles in which the SIMD
                      issued two VALU instructions
  valu_any_frac       from SQ_ACTIVE_INST_VALU ... reported raw (per-wave quad-cycles, summed over waves)
  salu_per_cu_cycle   SQ_INSTS_SALU / (simd_cycles / 4): SALU instructions per CU-cycle
  lds_busy_frac       SQ_LDS_IDX_ACTIVE / (simd_cycles / 4): cycles the CU's LDS was busy with
                      indexed accesses per CU-cycle (4 SIMDs per CU)
  lds_latency_cycles  SQ_INST_LEVEL_LDS / SQ_INSTS_LDS (in-flight LDS instructions per cycle over the
                      instruction count: the mean LDS instruction latency)
  waves_per_simd      SQ_WAVE_CYCLES * 4 / simd_cycles (mean resident waves)
usage: python3 tools/pmc_pipe_summary.py <dir>      -> <dir>/pmc_pipe.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(d, tag, pattern):
    out = []
    for f in glob.glob(os.path.join(d, tag, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def _name(k):
    k = k.split("(")[0].strip()
    if k.startswith("void "):
        k = k[5:]
    return k


def load(d, tag, kernel="solve4_kernel<false>"):
    """{dispatch: {counter: value}} and {dispatch: wall ns} of `kernel` in one pass."""
    ctr = defaultdict(lambda: defaultdict(float))
    for r in _rows(d, tag, "*counter_collection.csv"):
        if kernel in r["Kernel_Name"]:
            ctr[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    wall = {}
    for r in _rows(d, tag, "*kernel_trace.csv"):
        if kernel in r["Kernel_Name"]:
            wall[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return ctr, wall


def summarize(ctr, wall):
    ids = sorted(ctr, key=int)
    if len(ids) > 1:
        ids = ids[1:]                      # the first dispatch warms up
    if not ids:
        return None
    g = defaultdict(float)
    for i in ids:
        for k, v in ctr[i].items():
            g[k] += v / len(ids)
    walls = [wall[i] for i in ids if i in wall]
    ns = sum(walls) / len(walls) if walls else None
    rec = {"dispatches": len(ids), "kernel_ms": ns / 1e6 if ns else None, "counters": dict(g)}
    cyc = g.get("SQ_CYCLES")
    if ns and g.get("GRBM_GUI_ACTIVE"):
        rec["clock_ghz"] = g["GRBM_GUI_ACTIVE"] / 8 / ns
    if cyc:
        rec["simd_cycles"] = cyc
        if ns:
            rec["simds_x_clock_ghz"] = cyc / ns
        for key, num, den in (("valu_issue_frac", "SQ_INSTS_VALU", cyc / 2),
                              ("valu_dual_frac", "SQ_ACTIVE_INST_VALU2", cyc / 4),
                              ("salu_per_cu_cycle", "SQ_INSTS_SALU", cyc / 4),
                              ("lds_busy_frac", "SQ_LDS_IDX_ACTIVE", cyc / 4),
                              ("lds_bank_conflict_frac", "SQ_LDS_BANK_CONFLICT", cyc / 4),
                              ("lds_data_fifo_full_frac", "SQ_LDS_DATA_FIFO_FULL", cyc / 4),
                              ("lds_cmd_fifo_full_frac", "SQ_LDS_CMD_FIFO_FULL", cyc / 4),
                              ("waves_per_simd", "SQ_WAVE_CYCLES", cyc / 4)):
            if g.get(num) is not None:
                rec[key] = g[num] / den
    if g.get("SQ_INSTS_LDS") and g.get("SQ_INST_LEVEL_LDS"):
        rec["lds_latency_cycles"] = g["SQ_INST_LEVEL_LDS"] / g["SQ_INSTS_LDS"]
    return rec


def main(d):
    out = {}
    units = {"c4": 10_000_000, "hard1m": 1_000_000, "min": 1_048_576}
    for run in ("c4", "hard1m", "min"):
        rec = {"units_per_launch": units[run]}
        for part in ("pipe", "lds"):
            ctr, wall = load(d, f"{run}_{part}")
            s = summarize(ctr, wall)
            if s:
                rec[part] = s
        if len(rec) > 1:
            out[run] = rec
    with open(os.path.join(d, "pmc_pipe.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for run, rec in out.items():
        for part, s in rec.items():
            if not isinstance(s, dict):
                continue
            brief = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in s.items() if k != "counters"}
            print(run, part, json.dumps(brief))


if __name__ == "__main__":
    main(sys.argv[1])
