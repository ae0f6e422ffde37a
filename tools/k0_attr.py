"""K0 attribution driver: the bench's vcf text (8.39 M dbSNP-shaped lines tiled on
the device) tokenized REPS times without the public line table, for a
rocprofv3 --kernel-trace --stats run per library (tools/k0_attr.sh).

    python tools/k0_attr.py [REPS]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from annotatedvdb_amd import synth  # noqa: E402
from annotatedvdb_amd.engine import Engine  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    eng = Engine(0)
    tile = synth.vcf_text(1 << 19, seed=6)
    text = torch.frombuffer(bytearray(tile), dtype=torch.uint8).to("cuda").repeat(16)
    for _ in range(reps):
        eng.vcf_tokenize(text, want_lines=False)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
