#!/usr/bin/env python3
"""Probe K1 cost components: histogram / counters on-off per workload, plus a
torch copy of the same byte volume as an achievable-bandwidth reference."""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from annotatedvdb_amd import synth
from annotatedvdb_amd.engine import Engine


def timeit(fn, reps=12):
    ts = []
    for r in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    n = int(os.environ.get("N", 100_000_000))
    dev = torch.device("cuda", 0)
    chrom, start = synth.point_snvs(n, seed=2, device=dev)
    c3, s3, end = synth.spans(n, seed=3, device=dev)
    code = torch.empty(n, dtype=torch.int32, device=dev)
    eng = Engine(0)
    hist = eng.new_histogram()
    ctr = eng.new_counters()
    for wl in ("c2", "c3"):
        cc, ss, ee = (chrom, start, None) if wl == "c2" else (c3, s3, end)
        bpr = 9 if wl == "c2" else 13
        for h, c in ((0, 0), (1, 0), (0, 1), (1, 1)):
            ms = timeit(lambda: eng.bin_assign(cc, ss, ee, want_status=False, hist=hist if h else None,
                                               counters=ctr if c else None, out_code=code))
            print(json.dumps({"workload": wl, "hist": h, "ctrs": c, "ms": round(ms, 4),
                              "GBps": round(n * bpr / ms / 1e6, 1)}), flush=True)
    # achievable references: torch copies
    src = torch.empty(n * 2, dtype=torch.int32, device=dev)
    dst = torch.empty(n * 2, dtype=torch.int32, device=dev)
    ms = timeit(lambda: dst.copy_(src))
    print(json.dumps({"ref": "torch copy int32 (read+write)", "bytes": n * 16, "ms": round(ms, 4),
                      "GBps": round(n * 16 / ms / 1e6, 1)}))
    ms = timeit(lambda: src.sum())
    print(json.dumps({"ref": "torch sum int32 (read only)", "bytes": n * 8, "ms": round(ms, 4),
                      "GBps": round(n * 8 / ms / 1e6, 1)}))
    ms = timeit(lambda: dst.fill_(1))
    print(json.dumps({"ref": "torch fill int32 (write only)", "bytes": n * 8, "ms": round(ms, 4),
                      "GBps": round(n * 8 / ms / 1e6, 1)}))


if __name__ == "__main__":
    main()
