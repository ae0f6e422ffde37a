"""Drop-in classes (BinIndex, VariantAnnotator, VariantPKGenerator,
VCFVariantLoader) on the GPU vs the reference's own outputs (golden files)."""

import gzip
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import avdb_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def read_tsv(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as fh:
        header = fh.readline().rstrip("\n").split("\t")
        return [dict(zip(header, line.rstrip("\n").split("\t"))) for line in fh]


def golden_lines():
    with gzip.open(os.path.join(GOLDEN, "vcf_lines.tsv.gz"), "rt") as fh:
        fh.readline()
        return [(r.replace("\\t", "\t"), json.loads(m), json.loads(c), json.loads(e))
                for r, m, c, e in (line.rstrip("\n").split("\t") for line in fh)]


@pytest.fixture(scope="module")
def loader():
    from annotatedvdb_amd.loaders import VCFVariantLoader
    ld = VCFVariantLoader("dbSNP")
    ld.initialize_pk_generator("GRCh38", None)
    ld.initialize_bin_indexer(None)
    ld.set_algorithm_invocation_id(1)
    ld.initialize_copy_sql()
    return ld


def _check(lines, outs, copy_rows):
    ci = 0
    for (raw, mapping, copy5, _), out in zip(lines, outs):
        if "__error__" in mapping:
            assert isinstance(out, Exception) and type(out).__name__ == mapping["__error__"], (raw, out)
            ci += len(copy5)  # rows the reference wrote before raising (none in these fixtures)
            continue
        assert out == mapping, raw
        for row in copy5:
            assert "#".join(copy_rows[ci].split("#")[:5]) == row
            ci += 1


def test_loader_batch_matches_reference(loader):
    lines = golden_lines()
    loader.reset_copy_buffer()
    outs = loader.parse_variants([l[0] for l in lines], errors="record")
    rows = loader.copy_buffer().getvalue().splitlines()
    _check(lines, outs, rows)
    assert loader.get_count("variant") == len(rows)


def test_loader_per_line_matches_reference(loader):
    lines = golden_lines()[:400]
    outs = []
    rows = []
    for raw, mapping, copy5, _ in lines:
        loader.reset_copy_buffer()
        try:
            outs.append(loader.parse_variant(raw))
        except Exception as err:  # noqa: BLE001
            outs.append(err)
        rows += loader.copy_buffer().getvalue().splitlines()
    _check(lines, outs, rows)


def test_loader_dedup_batch(loader):
    lines = [l[0] for l in golden_lines() if "__error__" not in l[1]][:2000]
    loader.reset_copy_buffer()
    before = loader.get_count("duplicates")
    outs = loader.parse_variants(lines, dedup=True)
    rows = loader.copy_buffer().getvalue().splitlines()
    pks = [r.split("#")[1] for r in rows]
    assert len(pks) == len(set(pks))
    all_pks = [m["primary_key"] for o in outs for v in o.values() for m in v]
    assert loader.get_count("duplicates") - before == len(all_pks) - len(set(all_pks)) > 0


def test_bin_index_per_record_and_batch():
    from annotatedvdb_amd.bin_index import BinIndex
    rows = read_tsv("bin_queries.tsv.gz")
    bi = BinIndex(None, verbose=False)
    for r in rows[:1500] + rows[-600:]:
        end = int(r["end"]) if r["end"] else None
        try:
            got = bi.find_bin_index(r["chrom"], int(r["start"]), end)
        except TypeError:
            got = "TypeError"
        assert got == r["bin_index"], r
    paths = bi.find_bin_indices([r["chrom"] for r in rows], [int(r["start"]) for r in rows],
                                [int(r["end"]) if r["end"] else None for r in rows])
    for r, p in zip(rows, paths):
        assert (p or "TypeError") == r["bin_index"], r
    with pytest.raises(TypeError):
        bi.find_bin_indices(["chrUn"], [5], errors="raise")


def test_variant_annotator_matches_reference():
    from annotatedvdb_amd.variant_annotator import VariantAnnotator
    rows = read_tsv("end_infer.tsv.gz")[:300]
    for r in rows:
        va = VariantAnnotator(r["ref"], r["alt"], "1", int(r["pos"]))
        assert va.infer_variant_end_location() == int(r["end"])
        nr, na = va.get_normalized_alleles()
        lcp = int(r["lcp"])
        if len(r["ref"]) == 1 and len(r["alt"]) == 1 or lcp == 0:
            assert (nr, na) == (r["ref"], r["alt"])
        else:
            assert (nr, na) == (r["ref"][lcp:], r["alt"][lcp:])
        assert va.get_metaseq_id() == r["metaseq_id"]


def test_pk_generator_short_and_long():
    from annotatedvdb_amd.primary_key_generator import VariantPKGenerator
    from annotatedvdb_amd.chromosomes import CHROM_NAMES
    digs = {c: "%032d" % i for i, c in enumerate(CHROM_NAMES)}
    g = VariantPKGenerator("GRCh38", None, sequence_digests=digs)
    assert g.generate_primary_key("1:148893911:TGGCCAACA:TAGCCAACG", "rs71261250") == \
        "1:148893911:TGGCCAACA:TAGCCAACG:rs71261250"
    rows = read_tsv("long_alleles.tsv.gz")[:200]
    items = [("%s:%s:%s:%s" % (r["chrom"], r["pos"], r["ref"], r["alt"]), None) for r in rows]
    keys = g.generate_primary_keys(items)
    for r, k in zip(rows, keys):
        d = O.vrs_allele_digest(digs[r["chrom"]], int(r["pos"]), r["ref"], r["alt"])
        assert k == "%s:%s:%s" % (r["chrom"], r["pos"], d)
    assert g.generate_primary_key(items[0][0], "rs1").endswith(":rs1")
    nodig = VariantPKGenerator("GRCh38", None)
    with pytest.raises(ValueError, match="Sequence mismatch"):
        nodig.generate_primary_key(items[0][0])
    with pytest.raises(ValueError):
        g.generate_primary_key("1:5:A:<DUP:TANDEM>")
