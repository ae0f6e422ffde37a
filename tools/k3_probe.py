"""K3 probe: grouped dedup time vs duplicate density (25 M ADSP-style records)."""
import sys
sys.path.insert(0, ".")
import torch
from annotatedvdb_amd import synth
from annotatedvdb_amd.engine import Engine

eng = Engine(0)
for dup, lf in ((0.0, 0.05), (0.02, 0.0), (0.02, 0.05), (0.1, 0.05)):
    b = synth.alleles(25_000_000, seed=5, dup_frac=dup, long_frac=lf)
    ts = []
    for it in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.pk_dedup(b, grouped=True)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print("dup_frac %.2f long_frac %.2f  k3 %.3f ms" % (dup, lf, min(ts[1:])), flush=True)
    del b
