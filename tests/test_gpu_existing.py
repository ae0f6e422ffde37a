"""K6 (--skipExisting key set) on the GPU vs the oracle's lookup semantics, and
the loader's skip path (vcf_variant_loader.py:284-291) vs the oracle loader.
map_variants itself is external SQL: the lookup order (exact, then switched
alleles) and the first-hit rule are the documented contract (parity unpinned)."""

import numpy as np
import pytest

from annotatedvdb_amd.chromosomes import CHROM_NAMES, length_table
from oracle import avdb_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _lines(n, seed):
    from annotatedvdb_amd import synth
    return synth.vcf_text(n, seed=seed).decode().splitlines()


def _metaseqs(lines):
    out = []
    for ln in lines:
        f = ln.split("\t")
        for a in f[4].split(","):
            if a != ".":
                out.append("%s:%s:%s:%s" % (f[0], f[1], f[3], a))
    return out


def test_k6_probe_vs_oracle(engine):
    from annotatedvdb_amd.engine import pack_records
    from annotatedvdb_amd.existing import ExistingVariants
    rng = np.random.default_rng(3)
    ms = _metaseqs(_lines(20000, 31))
    # existing rows: a third of the records as-is, a sixth with switched alleles,
    # duplicates (first wins), plus unrelated keys
    keys = []
    for m in ms:
        u = rng.random()
        if u < 0.33:
            keys.append(m)
        elif u < 0.5:
            c, p, r, a = m.split(":")
            keys.append(":".join((c, p, a, r)))
        if rng.random() < 0.02:
            keys.append(m)
    keys += ["%d:%d:A:G" % (rng.integers(1, 23), rng.integers(1, 10**8)) for _ in range(5000)]
    ex = ExistingVariants([(k, [{"primary_key": "pk%d" % i, "bin_index": "b"}]) for i, k in enumerate(keys)],
                          engine=engine)
    first = {}
    for i, k in enumerate(keys):
        first.setdefault(k, i)
    recs = [m.split(":") for m in ms]
    b = pack_records([CHROM_NAMES.index(r[0]) for r in recs], [int(r[1]) for r in recs],
                     [r[2].encode() for r in recs], [r[3].encode() for r in recs])
    ctr = engine.new_counters()
    match, kind = engine.keyset_probe(ex.table, ex.keys, ex.key_off, b, True, ctr)
    match, kind = match.cpu().numpy(), kind.cpu().numpy()
    exp = np.array([O.existing_match(first, m) for m in ms])
    assert np.array_equal(match, exp)
    exact = np.array([first.get(m, -1) >= 0 for m in ms])
    assert np.array_equal(kind == 1, exact)
    assert np.array_equal(kind == 2, (exp >= 0) & ~exact)
    assert int(ctr[28]) == int((exp >= 0).sum()) and int(ctr[22]) == 0
    # without checkAltVariants only exact matches
    m2, _ = engine.keyset_probe(ex.table, ex.keys, ex.key_off, b, False)
    assert np.array_equal(m2.cpu().numpy(), np.where(exact, exp, -1))


def test_loader_skip_existing_matches_oracle(engine):
    from annotatedvdb_amd.existing import ExistingVariants
    from annotatedvdb_amd.loaders import VCFVariantLoader
    lines = _lines(6000, 32)
    ms = _metaseqs(lines)
    rng = np.random.default_rng(4)
    keys = [m for m in ms if rng.random() < 0.4]
    payloads = [[{"primary_key": "old:%d" % i, "bin_index": "chrX.L1.B1"}] for i in range(len(keys))]
    ex = ExistingVariants(list(zip(keys, payloads)), engine=engine)
    first = {}
    for i, k in enumerate(keys):
        first.setdefault(k, i)
    ld = VCFVariantLoader("dbSNP")
    ld.initialize_pk_generator("GRCh38", None)
    ld.initialize_bin_indexer(None)
    ld.set_algorithm_invocation_id(1)
    ld.initialize_copy_sql()
    ld.set_skip_existing(True, existing=ex)
    exp_copy, exp_map = [], []
    for ln in lines:
        err, m, c = O.load_line(ln, length_table(), existing=first, payloads=payloads)
        assert err is None
        exp_copy += c
        exp_map += m
    # whole-batch GPU path (K6 consumed by K5)
    ld.reset_copy_buffer()
    mapping = ld.load_vcf_text(("\n".join(lines) + "\n").encode())
    assert ld.last_load_stats["host_lines"] == 0
    assert ld.copy_buffer().getvalue().splitlines() == exp_copy
    assert mapping.splitlines() == exp_map
    # per-line path
    ld.reset_copy_buffer()
    outs = ld.parse_variants(lines[:500])
    n_map = sum(1 for _ in outs)
    assert ["%s\t%s" % kv for o in outs for kv in o.items()] == exp_map[:n_map]
    # per-record API
    hit = keys[0]
    assert ld.is_duplicate(hit) is True
    assert ld.is_duplicate(hit, returnMatch=True) == payloads[first[hit]]
    assert ld.is_duplicate("1:1:A:C", returnMatch=True) is None
