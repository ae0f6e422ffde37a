"""K4 beside K7: the C4k keyed batch's digest kernel (VALU-bound SHA-512) on a
second stream while the key/path write pass (HBM/store-bound) runs on the first.
Times each alone and both together (HIP events around both streams), so the
gain of running them concurrently is measured before the pipeline is split.
The write pass reads the previous launch's digests (timing only).

    AVDB_K4_BLOCKS_PER_CU=1 python tools/overlap_probe.py [N] [REPS]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from annotatedvdb_amd import synth  # noqa: E402
from annotatedvdb_amd.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    eng = Engine(0)
    eng.set_sequence_digests(["%032d" % i for i in range(25)])
    b = synth.dbsnp_alleles(n, seed=4)
    _, code, _, _ = eng.record_prep(b, want_lcp=False)
    import ctypes
    sz = ctypes.c_size_t()
    eng.lib.avdb_vrs_digest_workspace_size(n, ctypes.byref(sz))
    ws4 = torch.empty(int(sz.value), dtype=torch.uint8, device="cuda")
    dig, _ = eng.vrs_digest(b, 50, workspace=ws4)
    kt = eng.primary_keys(b, code=code, digest=dig)
    torch.cuda.synchronize()
    sa = torch.cuda.current_stream()
    sb = torch.cuda.Stream()

    def run(k4, k7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(sa)
        sb.wait_event(e0)
        if k4:
            with torch.cuda.stream(sb):
                eng.vrs_digest(b, 50, workspace=ws4)
        if k7:
            eng.primary_keys(b, code=code, digest=dig, out=kt)
        eb = torch.cuda.Event()
        eb.record(sb)
        sa.wait_event(eb)
        e1.record(sa)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    res = {}
    for name, k4, k7 in (("k4", 1, 0), ("k7", 0, 1), ("both", 1, 1)):
        ts = [run(k4, k7) for _ in range(reps)]
        res[name] = min(ts[1:]) if len(ts) > 1 else ts[0]
    res["sum"] = res["k4"] + res["k7"]
    res["k4_blocks_per_cu"] = os.environ.get("AVDB_K4_BLOCKS_PER_CU", "3")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
