"""ADSP datasource (vcf_variant_loader.py:303-307,336-337) and load-driver
failure semantics, vs the reference's own driver output.

tests/golden/adsp_load.tsv.gz was produced by running the reference loader
verbatim as VCFVariantLoader('ADSP') with --skipExisting over a stub validator
whose answers come from tests/golden/adsp_existing.json (make_golden.py --only
adsp; map_variants itself is external SQL, so that lookup model is the
unpinned part).  Both the per-line path (parse_variant) and the whole-batch GPU
path (load_vcf_text: K7 keys -> K6 text probe -> K5 with the ADSP column) must
reproduce every COPY row, .mapping line, is_adsp_variant update and counter."""

import gzip
import io
import json
import os

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

KEYS = ("line", "variant", "skipped", "duplicates", "update")


def adsp_rows():
    with gzip.open(os.path.join(GOLDEN, "adsp_load.tsv.gz"), "rt") as fh:
        fh.readline()
        out = []
        for line in fh:
            raw, err, mapping, copy, upd, delta = line.rstrip("\n").split("\t")
            out.append((raw.replace("\\t", "\t"), err or None, json.loads(mapping), json.loads(copy),
                        [tuple(u) for u in json.loads(upd)], json.loads(delta)))
        return out


def existing(engine):
    from annotatedvdb_amd.existing import ExistingVariants
    ex = json.load(open(os.path.join(GOLDEN, "adsp_existing.json")))
    return ExistingVariants(list(ex["metaseq"].items()), engine=engine, primary_keys=list(ex["primary_key"]))


def adsp_loader(engine, with_existing=True):
    from annotatedvdb_amd.loaders import VCFVariantLoader
    ld = VCFVariantLoader("ADSP")
    ld.initialize_pk_generator("GRCh38", None)
    ld.initialize_bin_indexer(None)
    ld.set_algorithm_invocation_id(1)
    ld.initialize_copy_sql()
    if with_existing:
        ld.set_skip_existing(True, existing=existing(engine))
    return ld


def test_adsp_per_line_matches_reference(engine):
    rows = adsp_rows()
    ld = adsp_loader(engine)
    assert "is_adsp_variant" in ld._copy_sql
    for raw, err, mapping, copy, upd, delta in rows:
        ld.reset_copy_buffer()
        ld.reset_update_buffer()
        before = [ld.get_count(k) for k in KEYS]
        try:
            res = ld.parse_variant(raw)
            got_map, got_err = ["%s\t%s" % kv for kv in res.items()], None
        except Exception as e:  # noqa: BLE001
            got_map, got_err = [], type(e).__name__
        assert got_err == err, raw
        assert got_map == mapping, raw
        assert ld.copy_buffer().getvalue().splitlines() == copy, raw
        assert [tuple(u) for u in ld.update_buffer()] == upd, raw
        assert [ld.get_count(k) - b for k, b in zip(KEYS, before)] == delta, raw


def test_adsp_gpu_batch_matches_reference(engine):
    rows = adsp_rows()
    ld = adsp_loader(engine)
    text = ("\n".join(r[0] for r in rows) + "\n").encode()
    mapping = ld.load_vcf_text(text, errors="record")
    assert ld.copy_buffer().getvalue().splitlines() == [c for r in rows for c in r[3]]
    assert mapping.splitlines() == [m for r in rows if r[1] is None for m in r[2]]
    assert [tuple(u) for u in ld.update_buffer()] == [u for r in rows for u in r[4]]
    assert sum(1 for r in rows for _ in r[4]) > 100
    st = ld.last_load_stats
    assert st["gpu_lines"] > 0.75 * len(rows), st
    # GPU lines: counters as the reference's (host lines count themselves)
    tot = [sum(r[5][i] for r in rows) for i in range(len(KEYS))]
    assert [ld.get_count(k) for k in KEYS] == tot


def test_adsp_without_validator_raises_like_reference(engine):
    """The reference's ADSP branch calls is_duplicate on a validator that only
    set_skip_existing creates: without it, AttributeError at the first alt."""
    ld = adsp_loader(engine, with_existing=False)
    line = "1\t100\trs5\tA\tG\t.\t.\tRS=5"
    with pytest.raises(AttributeError):
        ld.parse_variant(line)
    with pytest.raises(AttributeError):
        ld.load_vcf_text((line + "\n").encode())


def test_load_raise_keeps_earlier_output_and_counters(engine):
    """errors='raise' on line k of the second device batch: the COPY rows, the
    .mapping text and the counters of every earlier line are exactly what a
    loop of parse_variant produced before the failing line."""
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.loaders import VCFVariantLoader
    lines = synth.vcf_text(3000, seed=21).decode().splitlines()
    bad = 2200
    lines[bad] = lines[bad].split("\t")[0] + "\t123\trs1\tA:C\tA\t.\t.\tRS=1"  # ':' -> ValueError
    text = ("\n".join(lines) + "\n").encode()

    def fresh():
        ld = VCFVariantLoader("dbSNP")
        ld.initialize_pk_generator("GRCh38", None)
        ld.initialize_bin_indexer(None)
        ld.set_algorithm_invocation_id(1)
        ld.initialize_copy_sql()
        return ld

    ref = fresh()
    exp_map = []
    with pytest.raises(ValueError):
        for ln in lines:
            exp_map += ["%s\t%s" % kv for kv in ref.parse_variant(ln).items()]
    ld = fresh()
    sink = io.StringIO()
    with pytest.raises(ValueError) as ei:
        ld.load_vcf_text(text, batch_bytes=len(text) // 3, mapping_out=sink)
    assert sink.getvalue().splitlines() == exp_map
    assert ei.value.avdb_partial_mapping.splitlines() == exp_map
    assert ld.copy_buffer().getvalue() == ref.copy_buffer().getvalue()
    assert [ld.get_count(k) for k in KEYS] == [ref.get_count(k) for k in KEYS]


def test_grch37_positions_past_grch38_lengths(engine):
    """genomeBuild GRCh37: the bin indexer takes the PK generator's build, so a
    chr1 position past GRCh38's length (248,956,422) still has a bin."""
    from annotatedvdb_amd.loaders import VCFVariantLoader
    ld = VCFVariantLoader("dbSNP")
    ld.initialize_pk_generator("GRCh37", None)
    ld.initialize_bin_indexer(None)
    ld.set_algorithm_invocation_id(1)
    ld.initialize_copy_sql()
    res = ld.parse_variant("1\t249000000\trs7\tA\tG\t.\t.\tRS=7")
    (vid, m), = res.items()
    assert m[0]["primary_key"] == "1:249000000:A:G:rs7"
    assert m[0]["bin_index"].startswith("chr1.L1.B4.")
    ld38 = VCFVariantLoader("dbSNP")
    ld38.initialize_pk_generator("GRCh38", None)
    ld38.initialize_bin_indexer(None)
    with pytest.raises(TypeError):
        ld38.parse_variant("1\t249000000\trs7\tA\tG\t.\t.\tRS=7")
