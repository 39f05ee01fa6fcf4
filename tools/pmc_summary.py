"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel (per dispatch, in bytes).

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch. Per MI355X_MICROARCH.md (HBM section), on gfx950
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so the
"corrected" read column doubles it; WRITE_SIZE is exact for 16-B/lane streaming stores.
usage: python tools/pmc_summary.py <dir containing pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/>
"""
import csv
import json
import glob
import os
import sys
from collections import defaultdict


def load(d, counter):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter:
                    per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def main(d):
    fetch = load(d, "FETCH_SIZE")
    write = load(d, "WRITE_SIZE")
    summary = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("sdk::"):
            continue
        f = fetch.get(k, [])
        w = write.get(k, [])
        fmax = max(f) * 1024 if f else float("nan")
        wmax = max(w) * 1024 if w else float("nan")
        name = k.split("(")[0]
        summary[name] = {"dispatches": len(f), "fetch_size_bytes": fmax, "read_bytes_corrected": 2 * fmax,
                         "write_size_bytes": wmax, "traffic_bytes": 2 * fmax + wmax}
        print(f"{k[:60]:60s} dispatches={len(f)} FETCH_SIZE(max)={fmax/1e9:.4f} GB "
              f"corrected_read={2*fmax/1e9:.4f} GB WRITE_SIZE(max)={wmax/1e9:.4f} GB")
    with open(os.path.join(d, "pmc_summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
