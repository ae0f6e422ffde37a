#!/usr/bin/env python3
"""A/B sweep of K1 launch geometry / memory policy on one GPU (all variants in
one process, interleaved rounds, median of repeated launches).  Every variant's
codes/histogram/counters are checked equal to the first variant's.
Writes one JSON line per (variant, workload)."""

import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from annotatedvdb_amd import synth
from annotatedvdb_amd.engine import Engine


def main():
    n = int(os.environ.get("N", 100_000_000))
    reps = int(os.environ.get("REPS", 12))
    dev = torch.device("cuda", 0)
    chrom, start = synth.point_snvs(n, seed=2, device=dev)
    c3, s3, end = synth.spans(n, seed=3, device=dev)
    code = torch.empty(n, dtype=torch.int32, device=dev)
    variants = []
    grid = [(256, b) for b in (4, 6, 8)] + [(512, b) for b in (2, 3, 4)]
    for (blk, bpc), unroll, flags in itertools.product(grid, [2, 4], [0, 1, 2, 3]):
        os.environ["AVDB_K1_BLOCK"] = str(blk)
        os.environ["AVDB_K1_BLOCKS_PER_CU"] = str(bpc)
        os.environ["AVDB_K1_UNROLL"] = str(unroll)
        os.environ["AVDB_K1_FLAGS"] = str(flags)
        variants.append(((blk, bpc, unroll, flags), Engine(0)))
    hist = variants[0][1].new_histogram()
    ctr = variants[0][1].new_counters()
    wls = (("c2", True), ("c2", False), ("c3", True))
    # correctness: every variant agrees with variant 0
    ref = {}
    for key, eng in variants:
        for wl, use_hist in wls:
            hist.zero_(); ctr.zero_()
            cc, ss, ee = (chrom, start, None) if wl == "c2" else (c3, s3, end)
            eng.bin_assign(cc, ss, ee, want_status=False, hist=hist if use_hist else None,
                           counters=ctr if use_hist else None, out_code=code)
            sig = (int(code.sum()), int((code.long() * torch.arange(n, device=dev) % 1000003).sum()),
                   hist.cpu().numpy().tobytes() if use_hist else b"", ctr.cpu().numpy().tobytes() if use_hist else b"")
            if (wl, use_hist) not in ref:
                ref[(wl, use_hist)] = sig
            elif ref[(wl, use_hist)] != sig:
                print(json.dumps({"MISMATCH": key, "workload": wl, "hist": use_hist}), flush=True)
    results = {}
    for rnd in range(reps):
        for key, eng in variants:
            for wl, use_hist in wls:
                cc, ss, ee = (chrom, start, None) if wl == "c2" else (c3, s3, end)
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                eng.bin_assign(cc, ss, ee, want_status=False, hist=hist if use_hist else None,
                               counters=ctr if use_hist else None, out_code=code)
                ev1.record()
                ev1.synchronize()
                if rnd >= 2:
                    results.setdefault(key + (wl, use_hist), []).append(ev0.elapsed_time(ev1))
    for k, ts in sorted(results.items()):
        blk, bpc, unroll, flags, wl, use_hist = k
        ms = float(np.median(ts))
        bpr = 9 if wl == "c2" else 13
        print(json.dumps({"block": blk, "blocks_per_cu": bpc, "unroll": unroll, "flags": flags,
                          "workload": wl, "hist": use_hist, "ms": round(ms, 4),
                          "GBps": round(n * bpr / ms / 1e6, 1)}))


if __name__ == "__main__":
    main()
