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


def load(d, tag):
    """{kernel: {counter: [per-dispatch value, ...]}} of one pass directory."""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(d, tag, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0].strip()
                per[k][row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in per.items()}


def avg(xs):
    return sum(xs) / len(xs) if xs else None


def kernel_like(table, prefix):
    for k in table:
        if k.startswith(prefix) or k.split("::")[-1].startswith(prefix.split("::")[-1]):
            return k
    return None


def main(d):
    out = {}
    cal_f, cal_w = load(d, "cal_fetch"), load(d, "cal_write")
    kc = kernel_like(cal_f, "fetch_kernel")
    cal = {}
    if kc:
        fb = avg(cal_f[kc]["FETCH_SIZE"]) * 1024
        wb = avg(cal_w[kernel_like(cal_w, "fetch_kernel")]["WRITE_SIZE"]) * 1024
        cal = {"records": CAL_RECORDS, "fetch_size_bytes": fb, "write_size_bytes": wb,
               "read_correction": CAL_RECORDS * 81 / fb, "write_correction": CAL_RECORDS * 82 / wb}
        out["calibration"] = cal
    for tag, units, prefix, read_corr, write_corr, note in (
            ("c4", C4_PUZZLES, "sdk::solve", cal.get("read_correction"), cal.get("write_correction"),
             "FETCH/WRITE_SIZE scaled by tools/fetch_calib's algorithmic/counter ratios for the solvers' "
             "byte-load/byte-store pattern"),
            ("c3", C3_BOARDS, "sdk::check_kernel", 2.0, 1.0,
             "2 x FETCH_SIZE (gfx950: FETCH_SIZE reports half of a 16-B/lane streaming read) + WRITE_SIZE")):
        f, w, sq = load(d, f"{tag}_fetch"), load(d, f"{tag}_write"), load(d, f"{tag}_sq")
        for k in sorted(set(f) | set(sq)):
            if not k.startswith(prefix):
                continue
            if tag == "c3" and k != "sdk::check_kernel":
                continue
            rec = {"units_per_launch": units, "run": tag}
            fb = avg(f.get(k, {}).get("FETCH_SIZE", []))
            wb = avg(w.get(k, {}).get("WRITE_SIZE", []))
            if fb is not None and wb is not None and read_corr and write_corr:
                rec.update(dispatches=len(f[k]["FETCH_SIZE"]), fetch_size_bytes=fb * 1024,
                           write_size_bytes=wb * 1024, read_correction=read_corr, write_correction=write_corr,
                           traffic_bytes=fb * 1024 * read_corr + wb * 1024 * write_corr, traffic_note=note)
            s = sq.get(k, {})
            if s:
                g = {c: avg(v) for c, v in s.items()}
                rec.update(valu_insts=g.get("SQ_INSTS_VALU"), salu_insts=g.get("SQ_INSTS_SALU"),
                           lds_insts=g.get("SQ_INSTS_LDS"), lds_bank_conflict=g.get("SQ_LDS_BANK_CONFLICT"),
                           lds_idx_active=g.get("SQ_LDS_IDX_ACTIVE"), waves=g.get("SQ_WAVES"),
                           valu_active_per_wave_cycle=(g["SQ_ACTIVE_INST_VALU"] / g["SQ_WAVE_CYCLES"]
                                                       if g.get("SQ_WAVE_CYCLES") else None))
            out[k] = rec
    with open(os.path.join(d, "pmc_c4.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in out.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main(sys.argv[1])
