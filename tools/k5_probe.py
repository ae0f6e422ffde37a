"""K5 probe: time the format size / write passes on a dbSNP-shaped batch."""
import sys, time
sys.path.insert(0, ".")
import torch
from annotatedvdb_amd import synth
from annotatedvdb_amd.engine import Engine

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
eng = Engine(0)
tile = synth.vcf_text(min(1 << 19, n), seed=6)
text = torch.frombuffer(bytearray(tile), dtype=torch.uint8).cuda().repeat(n // min(1 << 19, n))
vb = eng.vcf_tokenize(text)
end, code, status, _ = eng.record_prep(vb.records, want_lcp=False)
for it in range(4):
    ev = {}
    fr = eng.vcf_format(vb, end, code, status, alg_id="1", events=ev)
    torch.cuda.synchronize()
    t = {k: v[0][0].elapsed_time(v[0][1]) for k, v in ev.items()}
    out = fr.copy.numel() + fr.mapping.numel()
    print("lines %d  size %.3f ms  write %.3f ms  out %.0f MB  write-rate %.1f GB/s  host_lines %d" % (
        vb.n_lines, t["format_size"], t["format_write"], out / 1e6, out / t["format_write"] / 1e6,
        int(fr.counters[27])), flush=True)
def cks(t):
    t = t.to(torch.int64)
    w = torch.arange(t.numel(), device=t.device, dtype=torch.int64) % 251 + 1
    return int(t.sum()), int((t * w).sum())
print("checksum copy", cks(fr.copy), "mapping", cks(fr.mapping), flush=True)
