#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output for the avdb kernels.

    prof_summary.py stats  <dir>                  kernel-trace --stats summary
    prof_summary.py pmc    <fetch_dir> <write_dir> <kernel-substring> <bytes_per_launch> [out.json]
    prof_summary.py traffic <rd_dir> <wr_dir>      per-kernel bytes from request-size counters

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


def per_kernel(d):
    """{short kernel name: {counter: mean over dispatches (the first, cold one skipped)}}"""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = {}
    for r in csv.DictReader(open(f)):
        if "avdb" not in r["Kernel_Name"]:
            continue
        acc.setdefault(short(r["Kernel_Name"]), {}).setdefault(r["Counter_Name"], []).append(
            float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: (sum(v[1:]) / len(v[1:]) if len(v) > 1 else v[0]) for c, v in cs.items()}
    return out


def traffic(rd_dir, wr_dir):
    """Bytes between L2 and the fabric per launch, from request-size counters:
    reads 32/64/128-B requests, writes 32/64-B requests (exact sizes, so no
    FETCH_SIZE-style width correction is needed), plus the DRAM-bound share."""
    rd, wr = per_kernel(rd_dir), per_kernel(wr_dir)
    res = {}
    for k in sorted(set(rd) | set(wr)):
        r, w = rd.get(k, {}), wr.get(k, {})
        read = 32 * r.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * r.get("TCC_EA0_RDREQ_64B_sum", 0) + \
            128 * r.get("TCC_EA0_RDREQ_128B_sum", 0)
        n64 = w.get("TCC_EA0_WRREQ_64B_sum", 0)
        write = 32 * (w.get("TCC_EA0_WRREQ_sum", 0) - n64) + 64 * n64
        res[k] = {"read_bytes": read, "write_bytes": write, "bytes": read + write,
                  "read_dram_bytes": 32 * r.get("TCC_EA0_RDREQ_DRAM_32B_sum", 0),
                  "write_dram_bytes": 32 * w.get("TCC_EA0_WRREQ_WRITE_DRAM_32B_sum", 0)}
    return res


def main():
    mode = sys.argv[1]
    if mode == "stats":
        for s in stats(sys.argv[2]):
            print(json.dumps(s))
        return
    if mode == "traffic":
        print(json.dumps(traffic(sys.argv[2], sys.argv[3]), indent=1))
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
