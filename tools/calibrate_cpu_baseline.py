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


def calibrate_load(n_lines):
    """Load path: the verbatim reference loader (parse_variant + the driver's
    mapping print) vs oracle.load_line with the PortBinIndex, per line."""
    import io
    from AnnotatedVDB.Util.loaders import VCFVariantLoader
    from annotatedvdb_amd.chromosomes import length_table
    lines = synth.vcf_text(n_lines, seed=6).decode().splitlines()
    ld = VCFVariantLoader("dbSNP")
    ld.initialize_pk_generator("GRCh38", "/nonexistent")
    ld.initialize_bin_indexer(None)
    ld._alg_invocation_id = "1"
    ld.initialize_copy_sql()
    out = io.StringIO()
    t0 = time.perf_counter()
    for ln in lines:
        for k, v in ld.parse_variant(ln).items():
            print(k, v, sep="\t", file=out)
    tr = time.perf_counter() - t0
    bi = O.PortBinIndex(O.BinTable(GRCH38_LENGTHS))
    lens = length_table()
    t0 = time.perf_counter()
    for ln in lines:
        O.load_line(ln, lens, bin_index=bi)
    tp = time.perf_counter() - t0
    print(f"load: reference {tr / n_lines * 1e6:.2f} us/line ({n_lines / tr:,.0f} lines/s), "
          f"port {tp / n_lines * 1e6:.2f} us/line ({n_lines / tp:,.0f} lines/s), port/ref time = {tp / tr:.3f}")


def c1_records(n):
    d = synth.np_c1(n, seed=1)
    heap = d["heap"].tobytes()
    o, r, a = d["allele_off"].tolist(), d["ref_len"].tolist(), d["alt_len"].tolist()
    refs = [heap[x:x + y].decode() for x, y in zip(o, r)]
    alts = [heap[x + y:x + y + z].decode() for x, y, z in zip(o, r, a)]
    exts = ["rs%d" % e if e else None for e in d["ext_id"].tolist()]
    return ["22"] * n, d["pos"].tolist(), refs, alts, exts


def calibrate_c1(n):
    """C1 per-record path: the verbatim reference (VariantAnnotator
    + VariantPKGenerator.generate_primary_key + get_normalized_alleles (loader
    :309) + infer_variant_end_location on a second annotator, as
    vcf_parser.py:225-231 does + BinIndex.find_bin_index) vs
    oracle.c1_port_loop, on the C1 records."""
    from AnnotatedVDB.BinIndex.bin_index import BinIndex
    from AnnotatedVDB.Util.primary_key_generator import VariantPKGenerator
    from AnnotatedVDB.Util.variant_annotator import VariantAnnotator
    names, pos, refs, alts, exts = c1_records(n)
    pkg = VariantPKGenerator("GRCh38", "/nonexistent")
    bi = BinIndex(None, verbose=False)
    t0 = time.perf_counter()
    for c, p, r, a, e in zip(names, pos, refs, alts, exts):
        va = VariantAnnotator(r, a, c, p)
        pkg.generate_primary_key(va.get_metaseq_id(), e)
        va.get_normalized_alleles()  # vcf_variant_loader.py:309
        end = VariantAnnotator(r, a, c, p).infer_variant_end_location()
        bi.find_bin_index(c, p, end)
    tr = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.c1_port_loop(names, pos, refs, alts, exts, O.PortBinIndex(O.BinTable(GRCH38_LENGTHS)))
    tp = time.perf_counter() - t0
    print(f"c1: reference {tr / n * 1e6:.3f} us/record ({n / tr:,.0f}/s), port {tp / n * 1e6:.3f} us/record "
          f"({n / tp:,.0f}/s), port/ref time = {tp / tr:.3f}")


def main():
    n = int(os.environ.get("N", 1_000_000))
    MG.install_stubs()
    MG.build_binindexref()
    calibrate_c1(int(os.environ.get("N_C1", 1_100_000)))
    if os.environ.get("C1_ONLY"):
        return
    calibrate_load(int(os.environ.get("N_LINES", 100_000)))
    if os.environ.get("LOAD_ONLY"):
        return
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
