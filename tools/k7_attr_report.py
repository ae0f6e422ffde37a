"""Summarise tools/k7_attr.sh: per library variant, the C4k keys + paths time
and the SQ counters of k_record_keys_v2 per 64-record tile.

    python tools/k7_attr_report.py gpurun_out/TAG [> profiles/...json]
"""
import csv
import glob
import json
import os
import sys

N = 125_000_000
TILES = N / 64

KNOBS = {1: "no key render", 2: "no path render", 4: "no ':'/ASCII check", 8: "no allele ranges",
         16: "no ':rs' suffix", 32: "no label:pos: prefix", 64: "no flushes", 128: "no window loads"}


def counters(d):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "k_record_keys_v2" not in row.get("Kernel_Name", ""):
                    continue
                key = (row["Dispatch_Id"], row["Counter_Name"])
                acc[key] = acc.get(key, 0.0) + float(row["Counter_Value"])
    per = {}
    for (disp, name), v in acc.items():
        per.setdefault(name, []).append(v)
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    d = sys.argv[1]
    out = []
    for f in sorted(glob.glob(os.path.join(d, "probe_x*.json"))):
        v = os.path.basename(f)[len("probe_"):-len(".json")]
        bits = int(v[1:]) if v[1:].isdigit() else 0
        try:
            probe = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            probe = {}
        c = counters(os.path.join(d, "pmc_" + v))
        row = {"variant": v, "drops": ([KNOBS[b] for b in KNOBS if bits & b] or ["nothing"]) if v[1:].isdigit() else [],
               "keys_paths_ms": probe.get("keys_paths_ms")}
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_INSTS_BRANCH"):
            if k in c:
                row[k.replace("SQ_INSTS_", "").lower() + "_per_tile"] = round(c[k] / TILES, 1)
        out.append(row)
    base = next((r for r in out if r["variant"] in ("x0", "xbase")), None)
    if base:
        for r in out:
            if r is not base and r.get("keys_paths_ms") and base.get("keys_paths_ms"):
                r["saves_ms"] = round(base["keys_paths_ms"] - r["keys_paths_ms"], 3)
            if r is not base and "valu_per_tile" in r and "valu_per_tile" in base:
                r["saves_valu_per_tile"] = round(base["valu_per_tile"] - r["valu_per_tile"], 1)
    print(json.dumps({"what": "k_record_keys_v2 attribution on C4k (1.25e8 records, keys + paths): each "
                      "variant drops the parts named (wrong text; timing only)", "rows": out}, indent=1))


if __name__ == "__main__":
    main()
