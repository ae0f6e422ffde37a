"""K0 one-pass tokenizer probe: the bench's 8.4 M-line text through
avdb_vcf_tokenize, timed with HIP events, and the per-chunk s_memrealtime
stamps the kernel leaves in its workspace (aggregate published -> prefix
published = the look-back wait) summarised.

    python tools/k0_onepass_probe.py [LINES] [REPS]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from annotatedvdb_amd import synth  # noqa: E402
from annotatedvdb_amd.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8_388_608
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    eng = Engine(0)
    tile = synth.vcf_text(min(131072, n), seed=6)
    reps_t = -(-n // 131072)
    text = torch.frombuffer(bytearray(tile), dtype=torch.uint8).to(eng.device).repeat(reps_t)
    res = {"text_bytes": int(text.numel())}
    for fused in (False, True):
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.vcf_tokenize(text, fused=fused)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res["fused" if fused else "four"] = ts
    nb = int(text.numel())
    nc = -(-nb // 16384)
    ws = eng._tok_ws
    t0 = 256 + 8 * nc + 48 * nc
    c0 = t0 + 4 * ((nc + 1) & ~1)
    clk = ws[c0:c0 + 16 * nc].view(torch.int64).cpu().numpy().reshape(nc, 2).astype(np.float64) / 100.0  # us
    wait = clk[1:, 1] - clk[1:, 0]
    res["chunks"] = nc
    res["lookback_wait_us"] = {q: float(np.percentile(wait, q)) for q in (50, 90, 99, 100)}
    res["span_us"] = float(clk[:, 1].max() - clk[:, 0][clk[:, 0] > 0].min())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
