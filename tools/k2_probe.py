"""K2 probe: record prep (end + bin + status + L8 histogram) on the C5 batch.
Prints the HIP-event time of avdb_record_prep for the ctx options in the
environment (AVDB_K2_UNROLL, AVDB_K2_BLOCKS_PER_CU, AVDB_K2_VECTOR).

    python tools/k2_probe.py [N] [REPS]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from annotatedvdb_amd import synth  # noqa: E402
from annotatedvdb_amd.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    eng = Engine(0)
    batch = synth.alleles(n, seed=5, device=eng.device)
    hist = eng.new_histogram()
    ts = []
    for r in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        eng.record_prep(batch, want_lcp=False, hist=hist)
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    env = {k: os.environ.get(k) for k in ("AVDB_K2_UNROLL", "AVDB_K2_BLOCKS_PER_CU", "AVDB_K2_VECTOR")}
    print(json.dumps({"env": env, "records": n, "ms_min": min(ts), "ms_median": sorted(ts)[len(ts) // 2]}))


if __name__ == "__main__":
    main()
