#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output for the avdb kernels.

    prof_summary.py stats  <dir>                  kernel-trace --stats summary
    prof_summary.py pmc    <fetch_dir> <write_dir> <kernel-substring> <bytes_per_launch> [out.json]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE come from separate passes (TCC slot limits), are in KiB, and on
gfx950 FETCH_SIZE reads exactly 1/2 of the bytes of a wide coalesced streaming
read, so it is doubled (WRITE_SIZE is exact for 16-B-per-lane stores).
"""

import csv
import glob
import json
import os
import re
import sys


def short(name: str) -> str:
    m = re.search(r"(avdb::k_[a-z0-9_]+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:80]


def stats(d):
    f = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
    rows = list(csv.DictReader(open(f)))
    out = []
    for r in rows:
        if "avdb" in r["Name"]:
            out.append({"kernel": short(r["Name"]), "calls": int(r["Calls"]),
                        "avg_us": float(r["AverageNs"]) / 1e3, "min_us": float(r["MinNs"]) / 1e3,
                        "max_us": float(r["MaxNs"]) / 1e3})
    return out


def pmc_values(d, counter, kern):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    vals = []
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    mode = sys.argv[1]
    if mode == "stats":
        for s in stats(sys.argv[2]):
            print(json.dumps(s))
        return
    fetch_dir, write_dir, kern, alg = sys.argv[2], sys.argv[3], sys.argv[4], float(sys.argv[5])
    fv = pmc_values(fetch_dir, "FETCH_SIZE", kern)
    wv = pmc_values(write_dir, "WRITE_SIZE", kern)
    # skip the first (cold) dispatch when several are present
    fv2 = fv[1:] if len(fv) > 1 else fv
    wv2 = wv[1:] if len(wv) > 1 else wv
    fetch = 2 * 1024 * sum(fv2) / len(fv2)
    write = 1024 * sum(wv2) / len(wv2)
    res = {"kernel": kern, "dispatches": [len(fv), len(wv)],
           "fetch_size_kib_raw": sum(fv2) / len(fv2), "write_size_kib_raw": sum(wv2) / len(wv2),
           "fetch_bytes_corrected": fetch, "write_bytes": write,
           "hbm_bytes_per_launch": fetch + write, "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": (fetch + write) / alg,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB->B; separate --pmc passes"}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 6:
        json.dump(res, open(sys.argv[6], "w"), indent=1)


if __name__ == "__main__":
    main()
