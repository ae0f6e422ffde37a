#!/usr/bin/env python3
"""Write the profiles/pmc_*.json files bench.py reads its `traffic` field from.

    pmc_files.py step  WORKLOAD <traffic.json> <bench line .json|.log>   (c4k, vcf, load)
    pmc_files.py k7    <k7_counters dir>                                   (pmc_k7.json)

`traffic.json` is tools/traffic_counters.sh's per-kernel L2<->fabric bytes
(request-size counters, two --pmc passes).  For c4k the step's kernels are
summed (the bench's first step is unkeyed; its kernels are listed apart), for
vcf every K0 kernel, for load the K5 write pass the bench line's roofline
names.  The algorithmic bytes come from the bench line measured beside it.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import per_kernel  # noqa: E402

C4K_STEP = ("k_record_prep4<true, 1, 1>", "k_dedup_resolve_list", "k_long_hist_codes", "k_long_scan",
            "k_long_scatter_codes", "k_vrs_digest", "k_key_group_scan", "k_record_keys_v2")
# (the vcf step tokenizes without the public line table, count-free: the window parse
# <true>, the two window scans and the per-window emit; the line-table forms
# k_vcf_parse_windows<false> / k_vcf_emit<false> run only in the bench's setup)
VCF_STEP = ("k_vcf_parse_windows<true>", "k_vcf_local_tiles", "k_vcf_local_top", "k_vcf_emit_local")


def bench_line(path):
    lines = [l for l in open(path) if l.startswith("{")]
    return json.loads(lines[-1])


def step(workload, traffic_path, bench_path):
    t = json.load(open(traffic_path))
    b = bench_line(bench_path)
    alg = b["roofline"]["algorithmic_bytes_per_launch"] if "algorithmic_bytes_per_launch" in b["roofline"] \
        else b["roofline"].get("algorithmic_bytes")
    if workload == "load":
        k = next(n for n in t if "k_vcf_format<true>" in n)
        v = t[k]
        return {"kernel": "k_vcf_format<true>", "hbm_bytes_per_launch": v["bytes"], "read_bytes": v["read_bytes"],
                "write_bytes": v["write_bytes"], "algorithmic_bytes_per_launch": alg,
                "traffic_over_algorithmic": v["bytes"] / alg,
                "note": "K5 write pass, L2<->fabric bytes from request-size counters (tools/traffic_counters.sh "
                        "load); algorithmic = the bench line's roofline bytes"}
    names = C4K_STEP if workload == "c4k" else VCF_STEP
    inside = {n: v for n, v in t.items() if any(s in n for s in names)}
    outside = {n: v for n, v in t.items() if n not in inside}
    total = sum(v["bytes"] for v in inside.values())
    return {"workload": workload, "hbm_bytes_per_launch": total, "algorithmic_bytes_per_launch": alg,
            "traffic_over_algorithmic": total / alg,
            "note": ("sum over the kernels of one steady-state step of L2<->fabric bytes from request-size "
                     "counters (tools/traffic_counters.sh %s, two --pmc passes); kernels of the bench's other "
                     "launches (the unkeyed first step, text tiling) under 'not_in_step'" % workload),
            "kernels": inside, "not_in_step": outside}


def k7(d):
    pm = {}
    for sub in ("pmc1", "pmc2", "rd", "wr"):
        for k, cs in per_kernel(os.path.join(d, sub)).items():
            if "k_record_keys_v2" in k:
                pm.update(cs)
    n = 125_000_000
    tiles = n / 64
    read = 32 * pm.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * pm.get("TCC_EA0_RDREQ_64B_sum", 0) + \
        128 * pm.get("TCC_EA0_RDREQ_128B_sum", 0)
    n64 = pm.get("TCC_EA0_WRREQ_64B_sum", 0)
    write = 32 * (pm.get("TCC_EA0_WRREQ_sum", 0) - n64) + 64 * n64
    return {"kernel": "k_record_keys_v2 (K7 one-pass write pass)",
            "source": "tools/k7_counters.sh: rocprofv3 --pmc passes over tools/k7_probe.py (C4k keyed batch, "
                      "1.25e8 records, keys + paths), averaged over the launches of k_record_keys_v2",
            "per_launch": pm, "records": n,
            "valu_wave_instr_per_64_records": pm.get("SQ_INSTS_VALU", 0) / tiles,
            "salu_wave_instr_per_64_records": pm.get("SQ_INSTS_SALU", 0) / tiles,
            "hbm_read_bytes": read, "hbm_write_bytes": write, "hbm_bytes_per_launch": read + write}


def main():
    if sys.argv[1] == "step":
        print(json.dumps(step(sys.argv[2], sys.argv[3], sys.argv[4]), indent=1))
    elif sys.argv[1] == "k7":
        print(json.dumps(k7(sys.argv[2]), indent=1))
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main()
