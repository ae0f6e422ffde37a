"""K4 probe: VRS long-allele digest on the C5 batch (25 M ADSP-style records).

Prints the HIP-event time of ``avdb_vrs_digest`` (compaction + digest), the
number of long records and the SHA-512 compressions one launch performs (from
the allele lengths: 2 SequenceLocation blocks + the Allele message blocks per
long record), so SQ counter passes over this script can be turned into
VALU instructions per compression.

    python tools/k4_probe.py [N] [REPS]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from annotatedvdb_amd import synth  # noqa: E402
from annotatedvdb_amd.engine import Engine  # noqa: E402

AL_PREFIX, AL_SUFFIX = 68, 54  # VRS Allele blob: prefix bytes before ALT, suffix after


def sha_blocks(t):
    return (t + 17 + 127) // 128


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    eng = Engine(0)
    eng.set_sequence_digests(["%032d" % i for i in range(25)])
    b = synth.alleles(n, seed=5)
    rl, al = b.ref_len.long(), b.alt_len.long()
    lng = (rl + al) > 50
    n_long = int(lng.sum().item())
    blocks_allele = int(sha_blocks(AL_PREFIX + al[lng] + AL_SUFFIX).sum().item())
    blocks = 2 * n_long + blocks_allele
    ws = torch.empty(0, dtype=torch.uint8, device=b.device)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.vrs_digest(b, 50, workspace=ws if ws.numel() else None)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    best = min(ts[1:]) if len(ts) > 1 else ts[0]
    print(json.dumps({"n": n, "n_long": n_long, "sha_blocks": blocks, "blocks_per_long": blocks / max(1, n_long),
                      "k4_ms_best": best, "k4_ms_all": ts,
                      "compressions_per_s": blocks / (best * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
