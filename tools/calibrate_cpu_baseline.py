#!/usr/bin/env python3
"""Calibrate the CPU-baseline port (oracle.avdb_oracle.PortBinIndex) against the
reference's own BinIndex (imported verbatim from /root/reference with the stub
DB of tests/golden/make_golden.py).  Build container only — the reference does
not travel to the GPU box.  Prints both per-call costs on the same sample."""

import os
import sys
import time

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import make_golden as MG  # noqa: E402
from annotatedvdb_amd import synth  # noqa: E402
from annotatedvdb_amd.chromosomes import CHROM_NAMES, GRCH38_LENGTHS  # noqa: E402
from oracle import avdb_oracle as O  # noqa: E402


def run(bi, names, pos, ends):
    t0 = time.perf_counter()
    if ends is None:
        for c, p in zip(names, pos):
            bi.find_bin_index(c, p)
    else:
        for c, p, e in zip(names, pos, ends):
            bi.find_bin_index(c, p, e)
    return time.perf_counter() - t0


def main():
    n = int(os.environ.get("N", 1_000_000))
    MG.install_stubs()
    MG.build_binindexref()
    from AnnotatedVDB.BinIndex.bin_index import BinIndex
    table = O.BinTable(GRCH38_LENGTHS)
    for wl in ("c2", "c3"):
        if wl == "c2":
            chrom, pos = synth.np_point_snvs(n, seed=2)
            ends = None
        else:
            chrom, pos, ends = synth.np_spans(n, seed=3)
            ends = ends.tolist()
        names = [CHROM_NAMES[c] for c in chrom.tolist()]
        pos = pos.tolist()
        tr = run(BinIndex(None, verbose=False), names, pos, ends)
        tp = run(O.PortBinIndex(table), names, pos, ends)
        print(f"{wl}: reference {tr / n * 1e6:.3f} us/call ({n / tr:,.0f}/s), "
              f"port {tp / n * 1e6:.3f} us/call ({n / tp:,.0f}/s), port/ref time = {tp / tr:.3f}")


if __name__ == "__main__":
    main()
