"""Summarise tools/pmc_c4.sh: per-launch PMC figures of the bench's headline solve kernel (C4) and
its checker (C3), written to <dir>/pmc_c4.json in the form bench.py's `--pmc-summary` reads.

Per kernel, every counter is summed over the rows of one dispatch and averaged over the
dispatches of that kernel in its own run (all of them the same launch configuration).

HBM traffic (FETCH_SIZE / WRITE_SIZE, KiB per dispatch):
  * check_kernel reads with 16-B-per-lane streaming loads: on gfx950 FETCH_SIZE reports half of
    those bytes (MI355X_MICROARCH.md, HBM section), so its read side is doubled.
  * the solve kernels load and store single bytes (3 per lane per board, csrc/solve4_kernel.h);
    no correction is assumed for that pattern: tools/fetch_calib moves 10M records with exactly
    that pattern and known byte counts, and the ratio (algorithmic / counter) it measures,
    read and write side separately, is applied to the solve kernel's counters.
usage: python3 tools/pmc_c4_summary.py <dir>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CAL_RECORDS = 10_000_000
C4_PUZZLES = 10_000_000
C3_BOARDS = 100_000_000
MIN_PUZZLES = 1_048_576
HARD_PUZZLES = 100_000


def load(d, tag):
    """{kernel: {counter: [per-dispatch value, ...]}} of one pass directory."""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(d, tag, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0].strip()
                if k.startswith("void "):
                    k = k[5:]
                k = k.replace("solve4_kernel<false>", "solve4_kernel").replace("solve4_kernel<true>",
                                                                              "solve4_kernel_donate")
                per[k][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in per.items()}


def avg(xs):
    return sum(xs) / len(xs) if xs else None


def kernel_like(table, prefix):
    for k in table:
        if k.startswith(prefix) or k.split("::")[-1].startswith(prefix.split("::")[-1]):
            return k
    return None


SQW_FIELDS = ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS",
              "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM")


def stall_breakdown(g):
    """SQ_WAIT_* / SQ_ACTIVE_INST_* per wave-cycle (all in quad-cycles; WAIT_ANY + WAIT_INST_ANY +
    ACTIVE_INST_ANY ~= WAVE_CYCLES, MI355X_MICROARCH.md rocprofv3 PMC slots)."""
    wc = g.get("SQ_WAVE_CYCLES")
    if not wc:
        return None
    return {c.lower().replace("sq_", "") + "_per_wave_cycle": g[c] / wc for c in SQW_FIELDS if g.get(c) is not None}


def sq_fields(rec, s, sw):
    if s:
        g = {c: avg(v) for c, v in s.items()}
        rec.update(valu_insts=g.get("SQ_INSTS_VALU"), salu_insts=g.get("SQ_INSTS_SALU"),
                   lds_insts=g.get("SQ_INSTS_LDS"), lds_bank_conflict=g.get("SQ_LDS_BANK_CONFLICT"),
                   lds_idx_active=g.get("SQ_LDS_IDX_ACTIVE"), waves=g.get("SQ_WAVES"),
                   valu_active_per_wave_cycle=(g["SQ_ACTIVE_INST_VALU"] / g["SQ_WAVE_CYCLES"]
                                               if g.get("SQ_WAVE_CYCLES") else None))
        u = rec["units_per_launch"]
        rec.update(valu_insts_per_unit=g.get("SQ_INSTS_VALU", 0) / u, lds_insts_per_unit=g.get("SQ_INSTS_LDS", 0) / u)
    if sw:
        rec["stalls"] = stall_breakdown({c: avg(v) for c, v in sw.items()})


def calibration(d, tag, records):
    f, w = load(d, f"{tag}_fetch"), load(d, f"{tag}_write")
    kf, kw = kernel_like(f, "fetch_kernel"), kernel_like(w, "fetch_kernel")
    if not kf or not kw:
        return {}
    fb = avg(f[kf]["FETCH_SIZE"]) * 1024
    wb = avg(w[kw]["WRITE_SIZE"]) * 1024
    return {"records": records, "kernel": kf, "fetch_size_bytes": fb, "write_size_bytes": wb,
            "read_correction": records * 81 / fb, "write_correction": records * 82 / wb}


def main(d):
    out = {}
    cal = calibration(d, "cal", CAL_RECORDS)
    if cal:
        out["calibration"] = cal
    calw = calibration(d, "calw", CAL_RECORDS)
    if calw:
        calw["note"] = ("the same 10M records and bytes, output written 16 records (1296 B, 16-B aligned) at a "
                        "time with 16-B stores")
        out["calibration_wide_stores"] = calw
    for tag, units, prefix, read_corr, write_corr, note, algo in (
            ("c4", C4_PUZZLES, "sdk::solve", cal.get("read_correction"), cal.get("write_correction"),
             "FETCH/WRITE_SIZE scaled by tools/fetch_calib's algorithmic/counter ratios for the solvers' "
             "byte-load/byte-store pattern", (81, 82)),
            # round 5: the C4 boards are decided by the propagation pass, which moves whole groups
            # (5184 B) with 16-B loads and stores, the checker's access pattern
            ("c4", C4_PUZZLES, "sdk::prop32", 2.0, 1.0,
             "2 x FETCH_SIZE (gfx950: FETCH_SIZE reports half of a 16-B/lane read, as for the checker) + "
             "WRITE_SIZE (16-B stores)", (81, 82)),
            ("c3", C3_BOARDS, "sdk::check_kernel", 2.0, 1.0,
             "2 x FETCH_SIZE (gfx950: FETCH_SIZE reports half of a 16-B/lane streaming read) + WRITE_SIZE", (81, 1)),
            ("min", MIN_PUZZLES, "sdk::solve4_kernel", None, None, None, None),
            ("hard", HARD_PUZZLES, "sdk::solve4_kernel", None, None, None, None)):
        f, w = load(d, f"{tag}_fetch"), load(d, f"{tag}_write")
        sq, sqw = load(d, f"{tag}_sq"), load(d, f"{tag}_sqw")
        for k in sorted(set(f) | set(sq) | set(sqw)):
            if not k.startswith(prefix) or k.endswith("_donate"):
                continue
            if tag == "c3" and k != "sdk::check_kernel":
                continue
            rec = {"units_per_launch": units, "run": tag}
            fb = avg(f.get(k, {}).get("FETCH_SIZE", []))
            wb = avg(w.get(k, {}).get("WRITE_SIZE", []))
            if fb is not None and wb is not None and read_corr and write_corr:
                rec.update(dispatches=len(f[k]["FETCH_SIZE"]), fetch_size_bytes=fb * 1024,
                           write_size_bytes=wb * 1024, read_correction=read_corr, write_correction=write_corr,
                           traffic_bytes=fb * 1024 * read_corr + wb * 1024 * write_corr, traffic_note=note,
                           traffic_raw={"fetch_size_bytes": fb * 1024, "write_size_bytes": wb * 1024,
                                        "algorithmic_read_bytes": algo[0] * units,
                                        "algorithmic_write_bytes": algo[1] * units,
                                        "raw_write_over_algorithmic": wb * 1024 / (algo[1] * units)})
            sq_fields(rec, sq.get(k, {}), sqw.get(k, {}))
            key = k if tag in ("c4", "c3") else f"{k}@{tag}"
            out[key] = rec
    with open(os.path.join(d, "pmc_c4.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in out.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main(sys.argv[1])
