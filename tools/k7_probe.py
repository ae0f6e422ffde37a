"""K7 probe: primary-key + ltree-path text of the keyed C4 batch (1.25e8
dbSNP-mix records per GPU, synth.dbsnp_alleles).  Times the write pass alone
(buffers reused, so no host sync) for keys only and for keys + paths, with HIP
events, so rocprofv3 passes over this script attribute SQ / TCC counters to
k_record_keys<true>.

    python tools/k7_probe.py [N] [REPS]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from annotatedvdb_amd import synth  # noqa: E402
from annotatedvdb_amd.engine import Engine  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts[1:]) if len(ts) > 1 else ts[0], ts


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    eng = Engine(0)
    eng.set_sequence_digests(["%032d" % i for i in range(25)])
    b = synth.dbsnp_alleles(n, seed=4)
    _, code, _, _ = eng.record_prep(b, want_lcp=False)
    dig, _ = eng.vrs_digest(b, 50)
    mode = os.environ.get("AVDB_K7_PROBE_MODE", "all")  # all | both (keys + paths only, for counter passes)
    # (narrow offsets by default, as the bench's serial keyed step writes them; AVDB_K7_PROBE_NARROW=0: u64)
    narrow = os.environ.get("AVDB_K7_PROBE_NARROW", "1") == "1"
    kt = eng.primary_keys(b, code=code, digest=dig,
                          out=eng.new_key_text(n, int(b.heap.numel()), paths=True, off32=True) if narrow else None)
    # (mode both launches no keys-only pass at all, so per-launch counter averages
    # describe keys + paths launches only)
    ko = eng.primary_keys(b, digest=dig) if mode == "all" else None
    torch.cuda.synchronize()
    kb, pb = int(kt.key_offsets(n)[n].item()), int(kt.path_offsets(n)[n].item())
    t_both, all_both = timed(lambda: eng.primary_keys(b, code=code, digest=dig, out=kt), reps)
    t_keys, all_keys = (timed(lambda: eng.primary_keys(b, digest=dig, out=ko), reps) if mode == "all"
                        else (None, []))
    print(json.dumps({"n": n, "key_bytes": kb, "path_bytes": pb, "keys_paths_ms": t_both, "keys_only_ms": t_keys,
                      "all_both": all_both, "all_keys": all_keys,
                      "text_TBps_both": (kb + pb) / (t_both * 1e-3) / 1e12}))


if __name__ == "__main__":
    main()
