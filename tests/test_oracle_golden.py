"""Pin the CPU oracle to the golden vectors produced by the reference itself
(tests/golden/make_golden.py ran the reference's Python verbatim)."""

import gzip
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from annotatedvdb_amd.chromosomes import CHROM_NAMES, GRCH38_LENGTHS, bin_index_chrom_code, length_table
from oracle import avdb_oracle as O


def read_tsv(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as fh:
        header = fh.readline().rstrip("\n").split("\t")
        return [dict(zip(header, line.rstrip("\n").split("\t"))) for line in fh]


LENS = {"chr" + c: GRCH38_LENGTHS[c] for c in CHROM_NAMES}


def oracle_path(chrom, start, end):
    code = bin_index_chrom_code(chrom)
    L = length_table()[code] if code < len(CHROM_NAMES) else None
    c, st = O.bin_code(L, start, end)
    if c == O.BIN_NONE:
        return "TypeError"
    return O.format_bin_path(CHROM_NAMES[code], c)


def test_binindexref_table_matches_generator():
    """The restated BinIndexRef rows equal the reference generator's rows
    (count, per-level counts and sha256 over every row)."""
    summ = json.load(open(os.path.join(GOLDEN, "binindexref_summary.json")))
    h = hashlib.sha256()
    gbin = 0
    counts = {}
    for c in CHROM_NAMES:
        for level, path, lo, hi in O.generate_binindexref(c, GRCH38_LENGTHS[c]):
            gbin += 1
            counts.setdefault("chr" + c, [0] * 14)[level] += 1
            h.update(("\t".join(str(x) for x in ("chr" + c, level, gbin, path, lo, hi)) + "\n").encode())
    assert gbin == summ["n_rows"] == 395448
    assert counts == summ["per_chrom_level_counts"]
    assert h.hexdigest() == summ["rows_sha256"]


def test_bin_queries_golden():
    rows = read_tsv("bin_queries.tsv.gz")
    assert len(rows) > 1000
    bad = []
    for r in rows:
        start = int(r["start"])
        end = int(r["end"]) if r["end"] else None
        got = oracle_path(r["chrom"], start, end)
        if got != r["bin_index"]:
            bad.append((r, got))
    assert not bad, bad[:5]


def test_bin_queries_numpy_matches_scalar():
    rows = [r for r in read_tsv("bin_queries.tsv.gz")]
    chrom = np.array([min(bin_index_chrom_code(r["chrom"]), 255) for r in rows], dtype=np.uint8)
    start = np.array([int(r["start"]) for r in rows], dtype=np.int64)
    end = np.array([int(r["end"]) if r["end"] else int(r["start"]) for r in rows], dtype=np.int64)
    codes, status = O.bin_codes_np(chrom, start, end, length_table())
    for i, r in enumerate(rows):
        L = length_table()[chrom[i]] if chrom[i] < 25 else None
        c, s = O.bin_code(L, int(start[i]), int(end[i]))
        assert codes[i] == c and status[i] == s, (r, codes[i], c)


def test_table_search_equals_closed_form():
    """Independent cross-check: deepest-containing table search over the
    restated BinIndexRef (the SQL's semantics) == closed form."""
    t = O.BinTable({"21": GRCH38_LENGTHS["21"], "M": GRCH38_LENGTHS["M"]})
    rng = np.random.default_rng(11)
    for c in ("21", "M"):
        L = GRCH38_LENGTHS[c]
        for _ in range(3000):
            s = int(rng.integers(1, L + 1))
            e = min(L, s + int(10 ** rng.uniform(0, 6.5)))
            row = t.find("chr" + c, s, e)
            code, _ = O.bin_code(L, s, e)
            assert row["global_bin_path"] == O.format_bin_path(c, code)


def test_end_inference_golden():
    rows = read_tsv("end_infer.tsv.gz")
    for r in rows:
        end, lcp = O.infer_end(int(r["pos"]), r["ref"], r["alt"])
        assert (end, lcp) == (int(r["end"]), int(r["lcp"])), r
        assert O.metaseq_id("1", int(r["pos"]), r["ref"], r["alt"]) == r["metaseq_id"]


def test_long_alleles_golden():
    rows = read_tsv("long_alleles.tsv.gz")
    for r in rows:
        end, lcp = O.infer_end(int(r["pos"]), r["ref"], r["alt"])
        assert (end, lcp) == (int(r["end"]), int(r["lcp"]))
        assert oracle_path(r["chrom"], int(r["pos"]), end) == r["bin_index"]
        assert O.is_long(r["ref"], r["alt"])


def test_kat():
    for k in json.load(open(os.path.join(GOLDEN, "kat.json"))):
        if "source" in k:  # in-repo known answer, GRCh37 DB; position far from any chromosome end
            end, _ = O.infer_end(k["pos"], k["ref"], k["alt"])
            assert oracle_path(k["chrom"], k["pos"], end) == k["bin_index_expected"]
            continue
        end, _ = O.infer_end(k["pos"], k["ref"], k["alt"])
        assert end == k["end"]
        got = oracle_path(k["chrom"], k["pos"], end)
        assert got == (k["bin_index"] or "TypeError")
        if k["primary_key"]:
            assert O.primary_key(k["chrom"], k["pos"], k["ref"], k["alt"], k["rsid"]) == k["primary_key"]


def test_port_bin_index_cache_matches_golden():
    """The reference-structured port (one-bin L13 cache + table search), used as
    the CPU baseline, answers the golden queries in their recorded order."""
    rows = read_tsv("bin_queries.tsv.gz")
    t = O.BinTable(GRCH38_LENGTHS)
    bi = O.PortBinIndex(t)
    for r in rows[:8000]:
        end = int(r["end"]) if r["end"] else None
        try:
            got = bi.find_bin_index(r["chrom"], int(r["start"]), end)
        except TypeError:
            got = "TypeError"
        assert got == r["bin_index"], r


def test_bin_queries_wide_golden():
    """200,000 reference answers in random order over all 25 contigs, spans to 1 Mb
    (make_golden.py --only scale): the numpy closed form the kernels restate."""
    rows = read_tsv("bin_queries_wide.tsv.gz")
    assert len(rows) == 200000
    assert {bin_index_chrom_code(r["chrom"]) for r in rows} == set(range(25))
    chrom = np.array([min(bin_index_chrom_code(r["chrom"]), 255) for r in rows], dtype=np.uint8)
    start = np.array([int(r["start"]) for r in rows], dtype=np.int64)
    end = np.array([int(r["end"]) if r["end"] else int(r["start"]) for r in rows], dtype=np.int64)
    codes, status = O.bin_codes_np(chrom, start, end, length_table())
    bad = []
    for i, r in enumerate(rows):
        got = "TypeError" if status[i] else O.format_bin_path(CHROM_NAMES[chrom[i]], int(codes[i]))
        if got != r["bin_index"]:
            bad.append((r, got))
    assert not bad, bad[:5]
    assert sum(r["bin_index"] == "TypeError" for r in rows) > 300  # spans past the contig end


def test_port_bin_index_replays_sequence():
    """The loader-order sequence (make_golden.py --only scale) through the port's one
    BinIndex: every answer, TypeErrors included, in order — and the fixture does
    what it is for: end < start records answered from the cached L13 leaf."""
    rows = read_tsv("bin_sequence.tsv.gz")
    bi = O.PortBinIndex(O.BinTable(GRCH38_LENGTHS))
    served_swapped = 0
    for r in rows:
        end = int(r["end"]) if r["end"] else None
        before = bi._currentBin
        try:
            got = bi.find_bin_index(r["chrom"], int(r["start"]), end)
        except TypeError:
            got = "TypeError"
        assert got == r["bin_index"], r
        if end is not None and end < int(r["start"]) and before and bi._currentBin is before:
            served_swapped += 1
    assert served_swapped > 5000


def test_sha512t24u_primitive():
    # published GA4GH example: sha512t24u(b"") == "z4PhNX7vuL3xVChQ1m2AB9Yg5AULVxXc"
    assert O.sha512t24u(b"") == "z4PhNX7vuL3xVChQ1m2AB9Yg5AULVxXc"
    assert O.sha512t24u(b"ACGT") == "aKF498dAxcJAqme6QYQ7EZ07-fiw8Kw2"


def test_vrs_published_example_pins_serialization_rules():
    """The digest serialisation K4 restates (sorted keys, compact JSON, nested
    objects and ga4gh CURIEs as bare digests, sha512t24u) reproduces vrs-python's
    published VRS 1.1 example — APOE rs7412, NC_000019.10 (ga4gh:SQ.IIB53T8CNeJJdUqzn9V_JnRtQadwWCbl)
    interbase 44908821-44908822, state T: SequenceLocation
    ga4gh:VSL.u5fspwVbQ79QkX6GHLF8tXPCAXFJqRPx, Allele ga4gh:VA.EgHPXXhULTwoP4-ACfs-YCXaeUQJBjH_ —
    digit for digit, with only that schema's type names (SimpleInterval,
    SequenceState).  The VRS 1.2/1.3 type names K4 uses (SequenceInterval of
    Number, LiteralSequenceExpression; vrs-python 0.7-0.8, the
    ``_from_gnomad(..., require_validation=)`` / ``.for_json()`` API that
    primary_key_generator.py:137,142 calls) come from that schema; no published
    1.2/1.3 digest is at hand here, so they stay unpinned."""
    seq = "IIB53T8CNeJJdUqzn9V_JnRtQadwWCbl"
    loc = O.sha512t24u(O.vrs_location_blob(seq, 44908821, 44908822, schema="1.1"))
    assert loc == "u5fspwVbQ79QkX6GHLF8tXPCAXFJqRPx"
    assert O.sha512t24u(O.vrs_allele_blob(loc, b"T", schema="1.1")) == "EgHPXXhULTwoP4-ACfs-YCXaeUQJBjH_"
    assert O.vrs_allele_digest(seq, 44908822, "C", "T", schema="1.1") == "EgHPXXhULTwoP4-ACfs-YCXaeUQJBjH_"
    # (the CURIE written whole instead of as its digest gives another identifier)
    assert O.sha512t24u(O.vrs_location_blob("ga4gh:SQ." + seq, 44908821, 44908822, schema="1.1")) != loc


def test_display_attributes_golden():
    """variant_annotator.py:134-241 restated == the reference's dicts (key order too)."""
    rows = read_tsv("display_attrs.tsv.gz")
    assert len(rows) > 500
    for r in rows:
        got = O.display_attributes(r["chrom"], int(r["pos"]), r["ref"], r["alt"])
        assert json.dumps(got) == r["attributes"], r


def load_rows():
    with gzip.open(os.path.join(GOLDEN, "vcf_load.tsv.gz"), "rt") as fh:
        fh.readline()
        for line in fh:
            raw, err, mapping, copy = line.rstrip("\n").split("\t")
            yield raw.replace("\\t", "\t"), err or None, json.loads(mapping), json.loads(copy)


def test_load_driver_golden():
    """The whole load-driver output per line (COPY rows with every column,
    .mapping line, or the exception) restated == the reference's."""
    n = 0
    for raw, err, mapping, copy in load_rows():
        e, m, c = O.load_line(raw, length_table())
        assert (e, c) == (err, copy), raw
        if err is None:
            assert m == mapping, raw
        n += 1
    assert n > 400


def test_float_repr_subset():
    """The FREQ numbers the GPU formats itself follow Python's float repr."""
    for s in ["0.9990", "0.0010", "0.00001", "0.0001", "12.50", "5.", ".5", "100.0", "0.0", "00.000",
              "123456789012345.0", "1234567890123456.0", "0.000123456789012345", "99999999999999.9"]:
        assert O.xstr_json({"x": O.to_numeric(s)}) == '{"x": %r}' % float(s)


def test_dedup_semantics():
    keys = ["1:5:A:G", "1:5:A:T", "1:5:A:G", "1:5:A:G:rs1", "1:5:A:G"]
    assert O.dedup_keep(keys) == [1, 1, 0, 1, 0]


def test_c_oracle_vrs_digest_and_keys_match_python_oracle():
    """The C oracle's long-key digest and primary-key text (used to check whole
    GPU batches) equal the Python restatement record by record."""
    import oracle
    from annotatedvdb_amd import synth
    d = synth.np_c1(3000, seed=11)
    rng = np.random.default_rng(3)
    # splice in long records (ref + alt > 50) so both key forms occur
    n = len(d["pos"])
    heap = bytearray(d["heap"].tobytes())
    off, rl, al = d["allele_off"].copy(), d["ref_len"].copy(), d["alt_len"].copy()
    for i in rng.choice(n, 300, replace=False):
        r, a = int(rng.integers(1, 400)), int(rng.integers(51, 700))
        off[i] = len(heap)
        heap += bytes(rng.choice(list(b"ACGT"), r + a).astype(np.uint8))
        rl[i], al[i] = r, a
    heap_np = np.frombuffer(bytes(heap), dtype=np.uint8)
    chrom = rng.integers(0, 25, n).astype(np.uint8)
    digs = "".join("%032d" % (7 * i) for i in range(25))
    lib = oracle.c_oracle()
    dig = np.zeros(n * 32, dtype=np.uint8)
    buf = np.zeros(4096, dtype=np.uint8)
    lib.avdb_oracle_vrs_digest(chrom.ctypes.data, d["pos"].ctypes.data, off.ctypes.data, rl.ctypes.data,
                               al.ctypes.data, heap_np.ctypes.data, n, 50, digs.encode(), 25, buf.ctypes.data,
                               dig.ctypes.data)
    keys = np.zeros(n * 200, dtype=np.uint8)
    koff = np.zeros(n + 1, dtype=np.uint64)
    lib.avdb_oracle_primary_keys(chrom.ctypes.data, d["pos"].ctypes.data, off.ctypes.data, rl.ctypes.data,
                                 al.ctypes.data, heap_np.ctypes.data, d["ext_id"].ctypes.data, dig.ctypes.data,
                                 n, 50, keys.ctypes.data, koff.ctypes.data)
    kb = keys.tobytes()
    for i in range(n):
        o, r, a = int(off[i]), int(rl[i]), int(al[i])
        ref, alt = bytes(heap[o:o + r]), bytes(heap[o + r:o + r + a])
        label = CHROM_NAMES[chrom[i]]
        dg = None
        if r + a > 50:
            c = int(chrom[i])
            dg = O.vrs_allele_digest(digs[32 * c:32 * c + 32], int(d["pos"][i]), ref, alt)
            assert dig[32 * i:32 * i + 32].tobytes().decode() == dg
        e = int(d["ext_id"][i])
        exp = O.primary_key(label, int(d["pos"][i]), ref.decode(), alt.decode(), "rs%d" % e if e else None, digest=dg)
        assert kb[int(koff[i]):int(koff[i + 1])].decode() == exp


def test_c_oracle_bin_paths_match_python_oracle_and_golden():
    """The C oracle's ltree path formatter (the checker of K7's path text over
    whole keyed-C4 shards) equals the Python restatement on spans of every
    level and contig, gives empty text for unmappable codes, and reproduces the
    reference-generated C1 prefix paths."""
    import oracle
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.chromosomes import length_table
    c, s, e = synth.np_spans(30000, seed=19)
    code, _ = O.bin_codes_np(c, s, e, length_table())
    code = code.astype(np.uint32)
    code[::97] = O.BIN_NONE
    c = c.astype(np.uint8)
    out = np.zeros(96 * len(c), dtype=np.uint8)
    off = np.zeros(len(c) + 1, dtype=np.uint64)
    lib = oracle.c_oracle()
    lib.avdb_oracle_bin_paths(c.ctypes.data, code.ctypes.data, len(c), out.ctypes.data, off.ctypes.data)
    b = out.tobytes()
    levels = set()
    for i in range(len(c)):
        exp = "" if code[i] == O.BIN_NONE else O.format_bin_path(CHROM_NAMES[c[i]], int(code[i]))
        assert b[off[i]:off[i + 1]].decode() == exp, i
        levels.add(int(code[i]) >> 28)
    assert len(levels) >= 12
    # against the reference's own paths (tests/golden/c1_prefix.tsv.gz, make_golden.py)
    with gzip.open(os.path.join(GOLDEN, "c1_prefix.tsv.gz"), "rt") as fh:
        fh.readline()
        rows = [ln.rstrip("\n").split("\t") for ln in fh][:20000]
    d = synth.np_c1(seed=1)  # the golden rows are the prefix of the whole C1 set
    d = {k: v[:len(rows)] for k, v in d.items() if k in ("chrom", "pos")}
    end = np.array([int(r[1]) for r in rows], dtype=np.uint32)
    code, _ = O.bin_codes_np(d["chrom"], d["pos"], end, length_table())
    code = code.astype(np.uint32)
    ch = d["chrom"].astype(np.uint8)
    out = np.zeros(96 * len(rows), dtype=np.uint8)
    off = np.zeros(len(rows) + 1, dtype=np.uint64)
    lib.avdb_oracle_bin_paths(ch.ctypes.data, code.ctypes.data, len(rows), out.ctypes.data, off.ctypes.data)
    b = out.tobytes()
    assert all(b[off[i]:off[i + 1]].decode() == rows[i][2] for i in range(len(rows)))


def test_c1_prefix_golden():
    """BASELINE config C1 (synth.np_c1, seed 1): the oracle's end, bin path and
    primary key for the first 100,000 records equal what the reference computed
    (tests/golden/c1_prefix.tsv.gz, make_golden.py --only c1)."""
    from annotatedvdb_amd import synth
    rows = read_tsv("c1_prefix.tsv.gz")
    d = synth.np_c1(synth.C1_N, seed=1)
    heap = d["heap"].tobytes()
    L = GRCH38_LENGTHS["22"]
    bi = O.PortBinIndex(O.BinTable(GRCH38_LENGTHS))
    assert len(rows) == 100000
    for i, row in enumerate(rows):
        o, r, a = int(d["allele_off"][i]), int(d["ref_len"][i]), int(d["alt_len"][i])
        ref, alt = heap[o:o + r].decode(), heap[o + r:o + r + a].decode()
        pos, ext = int(d["pos"][i]), int(d["ext_id"][i])
        end, _ = O.infer_end(pos, ref, alt)
        assert str(end) == row["end"], i
        assert O.primary_key("22", pos, ref, alt, "rs%d" % ext if ext else None) == row["primary_key"], i
        c, st = O.bin_code(L, pos, end)
        assert O.format_bin_path("22", c) == row["bin_index"], i
        if i % 50 == 0:  # the reference-structured cached lookup agrees too
            assert bi.find_bin_index("22", pos, end) == row["bin_index"]
