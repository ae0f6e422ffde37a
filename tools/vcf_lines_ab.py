"""K0 A/B: vcf_tokenize with the public 80-byte line table (the load path) and
without it (want_lines=False: 32-byte emit records in the parse workspace), the
bench's vcf workload (8.39 M dbSNP-shaped lines tiled on the device), alternating,
HIP-event times.

    python tools/vcf_lines_ab.py [REPS]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from annotatedvdb_amd import synth  # noqa: E402
from annotatedvdb_amd.engine import Engine  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    eng = Engine(0)
    tile = synth.vcf_text(1 << 19, seed=6)
    text = torch.frombuffer(bytearray(tile), dtype=torch.uint8).to("cuda").repeat(16)
    res = {"with_lines": [], "without_lines": []}
    for _ in range(3):
        eng.vcf_tokenize(text)
        eng.vcf_tokenize(text, want_lines=False)
    for _ in range(reps):
        for key, wl in (("with_lines", True), ("without_lines", False)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.vcf_tokenize(text, want_lines=wl)
            e1.record()
            torch.cuda.synchronize()
            res[key].append(e0.elapsed_time(e1))
    out = {k: {"min_ms": min(v), "median_ms": sorted(v)[len(v) // 2]} for k, v in res.items()}
    out["text_bytes"] = int(text.numel())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
