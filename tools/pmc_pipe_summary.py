"""Summarise tools/pmc_r04.sh: what bounds solve4_kernel per SIMD.

Per pass (c4 / hard1m / min), for the plain solve4_kernel dispatches (the first dispatch of
each run is a warm-up and is dropped when there are more).  Units, from the counters' own
descriptions (rocprofv3 --list-avail) and checked against the kernel wall time:
  * SQ_CYCLES is summed over the shader engines (32 on MI355X: SQ_CYCLES / (wall x clock) = 32);
    an SE holds 8 CUs = 32 SIMDs, so SIMD quad-cycles = SQ_CYCLES / 4 x 32 and CU-cycles =
    SQ_CYCLES x 8;
  * a wave64 VALU instruction issues over 2 cycles on a SIMD-32 (MI355X_MICROARCH.md:54), so the
    issue peak is 2 per SIMD quad-cycle.  SQ_ACTIVE_INST_VALU2 counts the quad-cycles in which a
    SIMD issued TWO VALU instructions, so the quad-cycles with any VALU issue are
    INSTS_VALU - VALU2, and
      valu_per_quad    = SQ_INSTS_VALU / SIMD quad-cycles (the peak: 2.0)
      valu_busy_frac   = (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) / SIMD quad-cycles
      valu_dual_frac   = SQ_ACTIVE_INST_VALU2 / SIMD quad-cycles
    How much of the peak a kernel can use depends on its instruction mix: tools/issue_calib.hip
    measures that (round 5: 2-operand VOP2 ops dual-issue in 78 % of quad-cycles, 3-source VOP3
    and packed VOP3P ops in ~7 % and 0 %, so solve4's mix tops out near 1.05 per quad-cycle);
  * salu_per_cu_cycle = SQ_INSTS_SALU / CU-cycles; lds_busy_frac = SQ_LDS_IDX_ACTIVE / CU-cycles;
    lds_*_fifo_full_frac likewise; waves_per_simd = SQ_WAVE_CYCLES / SIMD quad-cycles;
  * clock_ghz = GRBM_GUI_ACTIVE / 8 / kernel wall (MI355X_MICROARCH.md "DVFS give-back").
usage: python3 tools/pmc_pipe_summary.py <dir>      -> <dir>/pmc_pipe.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CUS = 256                 # MI355X compute units (4 SIMDs each)


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


def load(d, tag, kernel="solve4_kernel<false"):
    """{dispatch: {counter: value}} and {dispatch: wall ns} of `kernel` in one pass (a name prefix:
    the plain instance is solve4_kernel<false> to round 4's split-save instance, <false, false> after)."""
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
    if cyc and rec.get("clock_ghz"):
        n_se = max(1, round(cyc / (ns * rec["clock_ghz"])))
        simd_quads = cyc / 4 * (CUS * 4 / n_se)
        cu_cycles = cyc * (CUS / n_se)
        rec.update(shader_engines=n_se, simd_quad_cycles=simd_quads, cu_cycles=cu_cycles)
        if g.get("SQ_INSTS_VALU") is not None:
            v2 = g.get("SQ_ACTIVE_INST_VALU2", 0.0)
            rec["valu_per_quad"] = g["SQ_INSTS_VALU"] / simd_quads
            rec["valu_busy_frac"] = (g["SQ_INSTS_VALU"] - v2) / simd_quads
            rec["valu_dual_frac"] = v2 / simd_quads
        for key, num, den in (("salu_per_cu_cycle", "SQ_INSTS_SALU", cu_cycles),
                              ("lds_busy_frac", "SQ_LDS_IDX_ACTIVE", cu_cycles),
                              ("lds_bank_conflict_frac", "SQ_LDS_BANK_CONFLICT", cu_cycles),
                              ("lds_data_fifo_full_frac", "SQ_LDS_DATA_FIFO_FULL", cu_cycles),
                              ("lds_cmd_fifo_full_frac", "SQ_LDS_CMD_FIFO_FULL", cu_cycles),
                              ("waves_per_simd", "SQ_WAVE_CYCLES", simd_quads)):
            if g.get(num) is not None:
                rec[key] = g[num] / den
        if g.get("SQ_INSTS_LDS") is not None:
            rec["lds_insts_per_cu_cycle"] = g["SQ_INSTS_LDS"] / cu_cycles
    return rec


def main(d):
    out = {}
    units = {"c4": 10_000_000, "hard1m": 1_000_000, "min": 1_048_576}
    # the kernel each run is summarised for: C4's boards are all decided by the prop32 pass (round 5);
    # the search workloads' time is solve4's (PMC_C4_KERNEL / PMC_SEARCH_KERNEL override)
    kern = {"c4": os.environ.get("PMC_C4_KERNEL", "prop32_kernel"),
            "hard1m": os.environ.get("PMC_SEARCH_KERNEL", "solve4_kernel<false"),
            "min": os.environ.get("PMC_SEARCH_KERNEL", "solve4_kernel<false")}
    for run in ("c4", "hard1m", "min"):
        rec = {"units_per_launch": units[run], "kernel": kern[run]}
        for part in ("pipe", "lds"):
            ctr, wall = load(d, f"{run}_{part}", kern[run])
            s = summarize(ctr, wall)
            if s:
                rec[part] = s
        if len(rec) > 2:
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
