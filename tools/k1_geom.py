#!/usr/bin/env python3
"""Interleaved A/B of a few K1 variants (env-configured engines) after a warm-up."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from annotatedvdb_amd import synth
from annotatedvdb_amd.engine import Engine

VARIANTS = [dict(AVDB_K1_VARIANT=v, AVDB_K1_BLOCK=b, AVDB_K1_BLOCKS_PER_CU=p)
            for (v, b, p) in [tuple(int(x) for x in t.split(",")) for t in os.environ.get(
                "K1_VARIANTS", "0,512,4;1,512,4;1,512,3;2,512,3;3,512,3;3,512,2;5,512,4;0,256,8;4,512,4").split(";")]]

def main():
    n = int(os.environ.get("N", 100_000_000)); reps = int(os.environ.get("REPS", 20))
    dev = torch.device("cuda", 0)
    chrom, start = synth.point_snvs(n, seed=2, device=dev)
    c3, s3, end = synth.spans(n, seed=3, device=dev)
    code = torch.empty(n, dtype=torch.int32, device=dev)
    engs = []
    for v in VARIANTS:
        for k, x in v.items(): os.environ[k] = str(x)
        engs.append(Engine(0))
    hist = engs[0].new_histogram(); ctr = engs[0].new_counters()
    # warm-up ~2 s of back-to-back launches
    t0 = time.time()
    while time.time() - t0 < 2.0:
        engs[0].bin_assign(chrom, start, None, want_status=False, hist=hist, counters=ctr, out_code=code)
        torch.cuda.synchronize()
    res = {}
    # BACK2BACK=k: time k back-to-back launches per sample (the bench's steady
    # state: each launch also pays for the previous one's write-back), else one
    # launch per sample with a host sync in between
    b2b = int(os.environ.get("BACK2BACK", "1"))
    for r in range(reps):
        for i, e in enumerate(engs):
            for wl in ("c2", "c3"):
                cc, ss, ee = (chrom, start, None) if wl == "c2" else (c3, s3, end)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(b2b):
                    e.bin_assign(cc, ss, ee, want_status=False, hist=hist, counters=ctr, out_code=code)
                b.record()
                b.synchronize()
                res.setdefault((i, wl), []).append(a.elapsed_time(b) / b2b)
    for (i, wl), ts in sorted(res.items()):
        ms = float(np.median(ts[2:])); bpr = 9 if wl == "c2" else 13
        print(json.dumps({**VARIANTS[i], "workload": wl, "ms": round(ms, 4), "GBps": round(n * bpr / ms / 1e6, 1),
                          "p10_ms": round(float(np.percentile(ts[2:], 10)), 4)}))

main()
