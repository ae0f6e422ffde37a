"""GPU parity: every kernel through the C ABI vs the CPU oracle and the golden
vectors the reference produced.  Integer/byte work: bit-exact everywhere."""

import gzip
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN
from annotatedvdb_amd.chromosomes import CHROM_NAMES, GRCH38_LENGTHS, bin_index_chrom_code, length_table
from oracle import avdb_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LENGTHS = length_table()


def read_tsv(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as fh:
        header = fh.readline().rstrip("\n").split("\t")
        return [dict(zip(header, line.rstrip("\n").split("\t"))) for line in fh]


def u32(t):
    return t.cpu().numpy().view(np.uint32)


# ---------------------------------------------------------------------------
# K1 bin assignment
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["bin_queries.tsv.gz", "bin_queries_wide.tsv.gz"])
def test_k1_golden_bin_queries(engine, name):
    rows = read_tsv(name)
    chrom = np.array([min(bin_index_chrom_code(r["chrom"]), 255) for r in rows], dtype=np.uint8)
    start = np.array([int(r["start"]) for r in rows], dtype=np.int32)
    end = np.array([int(r["end"]) if r["end"] else int(r["start"]) for r in rows], dtype=np.int32)
    code, status = engine.bin_assign(torch.from_numpy(chrom), torch.from_numpy(start), torch.from_numpy(end))
    paths = engine.format_paths(chrom, u32(code))
    st = status.cpu().numpy()
    for i, r in enumerate(rows):
        exp = r["bin_index"]
        got = paths[i] if paths[i] is not None else "TypeError"
        assert got == exp, (r, got, st[i])


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 63, 64, 65, 1000, 4099, 1 << 20])
def test_k1_random_spans_vs_oracle(engine, n):
    chrom, start, end = __import__("annotatedvdb_amd.synth", fromlist=["x"]).np_spans(n, seed=n)
    if n > 10:
        chrom[::97] = 25 + (np.arange(chrom[::97].size) % 200)   # unknown contigs
        start[::89] = 0                                           # start < 1
        end[::83] = np.asarray(LENGTHS, dtype=np.int64)[np.minimum(chrom[::83], 24)] + 1
        sw = slice(5, None, 71)
        start[sw], end[sw] = end[sw].copy(), start[sw].copy()     # end < start
    code, status = engine.bin_assign(torch.from_numpy(chrom), torch.from_numpy(start), torch.from_numpy(end))
    rc, rs = O.bin_codes_np(chrom, start, end, LENGTHS)
    assert np.array_equal(u32(code), rc)
    assert np.array_equal(status.cpu().numpy(), rs)
    # points (end=NULL)
    code, status = engine.bin_assign(torch.from_numpy(chrom), torch.from_numpy(start))
    rc, rs = O.bin_codes_np(chrom, start, None, LENGTHS)
    assert np.array_equal(u32(code), rc)
    assert np.array_equal(status.cpu().numpy(), rs)


def test_k1_misaligned_scalar_path(engine):
    chrom, start, end = __import__("annotatedvdb_amd.synth", fromlist=["x"]).np_spans(10001, seed=3)
    dc = torch.from_numpy(chrom).cuda()[1:]
    ds = torch.from_numpy(start).cuda()[1:]
    de = torch.from_numpy(end).cuda()[1:]
    code, status = engine.bin_assign(dc, ds, de)
    rc, rs = O.bin_codes_np(chrom[1:], start[1:], end[1:], LENGTHS)
    assert np.array_equal(u32(code), rc)
    assert np.array_equal(status.cpu().numpy(), rs)


@pytest.mark.parametrize("sort", [True, False])
def test_k1_histogram_and_counters(engine, sort):
    from annotatedvdb_amd import synth
    chrom, start, end = synth.np_spans(300001, seed=9)
    if not sort:
        p = np.random.default_rng(1).permutation(len(chrom))
        chrom, start, end = chrom[p], start[p], end[p]
    chrom[::1001] = 77
    hist = engine.new_histogram()
    ctr = engine.new_counters()
    code, status = engine.bin_assign(torch.from_numpy(chrom), torch.from_numpy(start), torch.from_numpy(end),
                                     hist=hist, counters=ctr)
    rc, rs = O.bin_codes_np(chrom, start, end, LENGTHS)
    exp_hist = O.l8_histogram_np(chrom, start, rs, LENGTHS)
    assert np.array_equal(hist.cpu().numpy().view(np.uint32), exp_hist)
    c = ctr.cpu().numpy()
    assert np.array_equal(c[16:20], np.bincount(rs, minlength=4))
    assert c[20] == len(chrom)
    # scalar path (misaligned) accumulates identically
    hist2 = engine.new_histogram()
    ctr2 = engine.new_counters()
    engine.bin_assign(torch.from_numpy(chrom).cuda()[1:], torch.from_numpy(start).cuda()[1:],
                      torch.from_numpy(end).cuda()[1:], hist=hist2, counters=ctr2)
    exp2 = O.l8_histogram_np(chrom[1:], start[1:], rs[1:], LENGTHS)
    assert np.array_equal(hist2.cpu().numpy().view(np.uint32), exp2)
    assert int(ctr2[20]) == len(chrom) - 1


@pytest.mark.slow
def test_k1_full_size_c2_properties(engine):
    """BASELINE config 2 at full size (1e8 points): properties + sampled oracle."""
    from annotatedvdb_amd import synth
    n = 100_000_000
    chrom, start = synth.point_snvs(n, seed=2)
    hist = engine.new_histogram()
    ctr = engine.new_counters()
    code, _ = engine.bin_assign(chrom, start, None, want_status=False, hist=hist, counters=ctr)
    torch.cuda.synchronize()
    c = ctr.cpu().numpy()
    assert c[20] == n and c[16] == n                         # every point mappable, status OK
    assert int(hist.sum()) == n
    # leaf index == (start-1) // 15625 for every record (checked on device)
    idx = (code & 0x0FFFFFFF).long()
    assert bool(torch.equal(idx, ((start.long() - 1) // 15625)))
    assert bool((code.long() >> 28 & 0xF).eq(13).all())
    # sampled rows vs the oracle
    sel = torch.randint(0, n, (200_000,), device="cuda")
    rc, _ = O.bin_codes_np(chrom[sel].cpu().numpy(), start[sel].cpu().numpy(), None, LENGTHS)
    assert np.array_equal(u32(code[sel]), rc)


@pytest.mark.slow
def test_k1_full_size_c3_vs_c_oracle(engine):
    """BASELINE config 3 at full size (1e8 spans) vs the C oracle, bit-exact."""
    import ctypes
    import oracle
    from annotatedvdb_amd import synth
    n = 100_000_000
    chrom, start, end = synth.spans(n, seed=3)
    code, status = engine.bin_assign(chrom, start, end)
    hc, hs, he = chrom.cpu().numpy(), start.cpu().numpy(), end.cpu().numpy()
    rc = np.empty(n, dtype=np.uint32)
    rs = np.empty(n, dtype=np.uint8)
    lens = np.asarray(LENGTHS, dtype=np.uint32)
    oracle.c_oracle().avdb_oracle_bin_assign(hc.ctypes.data, hs.ctypes.data, he.ctypes.data, n,
                                            lens.ctypes.data, len(lens), rc.ctypes.data, rs.ctypes.data)
    assert np.array_equal(u32(code), rc)
    assert np.array_equal(status.cpu().numpy(), rs)


@pytest.mark.slow
def test_k1_c4_one_billion_vs_c_oracle(engine):
    """BASELINE config 4's whole job on one GPU, shard by shard: the 8 ranks'
    length-balanced pieces x 1.25e8 mixed records (1e9 in all, the bench's own
    generator and seeds), every bin code and status bit-exact vs the C oracle."""
    import oracle
    from annotatedvdb_amd import shard, synth
    n = 125_000_000
    lens = np.asarray(LENGTHS, dtype=np.uint32)
    plan = shard.plan(8)
    total = 0
    for rank in range(8):
        chrom, start, end = synth.spans(n, seed=4 + 1000 * rank, pieces=plan[rank], mix="c4")
        code, status = engine.bin_assign(chrom, start, end)
        hc, hs, he = chrom.cpu().numpy(), start.cpu().numpy(), end.cpu().numpy()
        rc = np.empty(n, dtype=np.uint32)
        rs = np.empty(n, dtype=np.uint8)
        oracle.c_oracle().avdb_oracle_bin_assign(hc.ctypes.data, hs.ctypes.data, he.ctypes.data, n,
                                                lens.ctypes.data, len(lens), rc.ctypes.data, rs.ctypes.data)
        assert np.array_equal(u32(code), rc), rank
        assert np.array_equal(status.cpu().numpy(), rs), rank
        total += n
        del chrom, start, end, code, status, hc, hs, he, rc, rs
    assert total == 1_000_000_000


# ---------------------------------------------------------------------------
# K2 record prep (end inference + bin)
# ---------------------------------------------------------------------------
def _prep_rows(engine, chroms, pos, refs, alts):
    from annotatedvdb_amd.engine import pack_records
    b = pack_records(chroms, pos, [r.encode() for r in refs], [a.encode() for a in alts])
    return engine.record_prep(b)


def test_k2_golden_end_infer(engine):
    rows = read_tsv("end_infer.tsv.gz")
    end, code, status, lcp = _prep_rows(engine, [0] * len(rows), [int(r["pos"]) for r in rows],
                                        [r["ref"] for r in rows], [r["alt"] for r in rows])
    e = end.cpu().numpy()
    l = lcp.cpu().numpy()
    for i, r in enumerate(rows):
        assert (int(e[i]), int(l[i])) == (int(r["end"]), int(r["lcp"])), r


def test_k2_golden_long_alleles(engine):
    rows = read_tsv("long_alleles.tsv.gz")
    chroms = [bin_index_chrom_code(r["chrom"]) for r in rows]
    end, code, status, lcp = _prep_rows(engine, chroms, [int(r["pos"]) for r in rows],
                                        [r["ref"] for r in rows], [r["alt"] for r in rows])
    paths = engine.format_paths(np.asarray(chroms, dtype=np.uint8), u32(code))
    for i, r in enumerate(rows):
        assert int(end[i]) == int(r["end"])
        assert (paths[i] or "TypeError") == r["bin_index"]


def test_k2_random_vs_c_oracle(engine):
    """1e6 synthetic C5-shaped records vs the C oracle (end, code, status, lcp)."""
    import oracle
    from annotatedvdb_amd import synth
    b = synth.alleles(1_000_000, seed=21)
    end, code, status, lcp = engine.record_prep(b)
    h = {k: getattr(b, k).cpu().numpy() for k in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "heap")}
    n = b.n
    re_, rc, rl = (np.empty(n, dtype=np.uint32) for _ in range(3))
    rs = np.empty(n, dtype=np.uint8)
    lens = np.asarray(LENGTHS, dtype=np.uint32)
    oracle.c_oracle().avdb_oracle_record_prep(
        h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data, h["ref_len"].ctypes.data,
        h["alt_len"].ctypes.data, h["heap"].ctypes.data, n, lens.ctypes.data, len(lens),
        re_.ctypes.data, rc.ctypes.data, rs.ctypes.data, rl.ctypes.data)
    assert np.array_equal(u32(end), re_)
    assert np.array_equal(u32(code), rc)
    assert np.array_equal(status.cpu().numpy(), rs)
    assert np.array_equal(u32(lcp), rl)


# ---------------------------------------------------------------------------
# K3 dedup
# ---------------------------------------------------------------------------
def _oracle_keep(b):
    import oracle
    h = {k: getattr(b, k).cpu().numpy() for k in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "heap", "ext_id")}
    keep = np.empty(b.n, dtype=np.uint8)
    d = oracle.c_oracle().avdb_oracle_dedup_grouped(
        h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data, h["ref_len"].ctypes.data,
        h["alt_len"].ctypes.data, h["heap"].ctypes.data, h["ext_id"].ctypes.data, b.n, keep.ctypes.data)
    return keep, d


def test_k3_dedup_grouped_and_hash(engine):
    from annotatedvdb_amd import synth
    b = synth.alleles(500_000, seed=33, dup_frac=0.05)
    exp, ndup = _oracle_keep(b)
    assert ndup > 1000
    ctr = engine.new_counters()
    keep = engine.pk_dedup(b, grouped=True, counters=ctr)
    assert np.array_equal(keep.cpu().numpy(), exp)
    assert int(ctr[21]) == ndup
    ctr = engine.new_counters()
    keep = engine.pk_dedup(b, grouped=False, counters=ctr)
    assert np.array_equal(keep.cpu().numpy(), exp)
    assert int(ctr[21]) == ndup and int(ctr[22]) == 0


def test_k3_dedup_ragged_long_and_unaligned(engine):
    """Grouped dedup at sizes ending inside a 4-record group, with long duplicate
    alleles (wave-cooperative compares) and dense duplicate runs crossing lane,
    wave and workgroup boundaries; then the same records through unaligned array
    views (the one-record-per-lane kernel)."""
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.engine import RecordBatch
    for n in (1, 2, 5, 255, 257, 1031, 70001):
        b = synth.alleles(n, seed=60 + n, long_frac=0.3, dup_frac=0.3)
        exp, ndup = _oracle_keep(b)
        ctr = engine.new_counters()
        keep = engine.pk_dedup(b, grouped=True, counters=ctr)
        assert np.array_equal(keep.cpu().numpy(), exp), n
        assert int(ctr[21]) == ndup
    # views starting one record in: pos / chrom / keep lose their 16- and 4-byte alignment
    b = synth.alleles(20001, seed=71, long_frac=0.3, dup_frac=0.3)
    v = RecordBatch(**{f: (getattr(b, f)[1:] if f != "heap" else b.heap)
                       for f in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "heap", "ext_id")})
    exp, _ = _oracle_keep(v)
    assert np.array_equal(engine.pk_dedup(v, grouped=True).cpu().numpy(), exp)


def test_k3_dedup_small_cases(engine):
    from annotatedvdb_amd.engine import pack_records
    recs = [(0, 5, "A", "G", 0), (0, 5, "A", "T", 0), (0, 5, "A", "G", 0), (0, 5, "A", "G", 7),
            (0, 5, "A", "G", 0), (0, 6, "A", "G", 0), (1, 6, "A", "G", 0), (1, 6, "AC", "G", 0),
            (1, 6, "A", "CG", 0), (1, 6, "A", "G", 0)]
    b = pack_records([r[0] for r in recs], [r[1] for r in recs], [r[2].encode() for r in recs],
                     [r[3].encode() for r in recs], [r[4] for r in recs])
    exp = O.dedup_keep([(r[0], r[1], r[2], r[3], r[4]) for r in recs])
    for grouped in (True, False):
        keep = engine.pk_dedup(b, grouped=grouped)
        assert keep.cpu().tolist() == exp
    # unsorted input through the hash path: first occurrence wins
    perm = [9, 3, 0, 7, 2, 5, 1, 8, 4, 6]
    rp = [recs[i] for i in perm]
    b = pack_records([r[0] for r in rp], [r[1] for r in rp], [r[2].encode() for r in rp],
                     [r[3].encode() for r in rp], [r[4] for r in rp])
    keep = engine.pk_dedup(b, grouped=False)
    assert keep.cpu().tolist() == O.dedup_keep([(r[0], r[1], r[2], r[3], r[4]) for r in rp])


# ---------------------------------------------------------------------------
# K4 digests
# ---------------------------------------------------------------------------
def test_k4_sha512t24u_vs_hashlib(engine):
    rng = np.random.default_rng(4)
    blobs = [b"", b"ACGT", b"a" * 111, b"b" * 112, b"c" * 127, b"d" * 128, b"e" * 129, b"f" * 240]
    blobs += [bytes(rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8)) for _ in range(500)]
    got = engine.sha512t24u(blobs)
    assert got == [O.sha512t24u(x) for x in blobs]
    assert got[0] == "z4PhNX7vuL3xVChQ1m2AB9Yg5AULVxXc"
    # vrs-python's published VRS 1.1 example (tests/test_oracle_golden.py): the
    # SequenceLocation and Allele digests of APOE rs7412 through the GPU's SHA-512
    seq = "IIB53T8CNeJJdUqzn9V_JnRtQadwWCbl"
    loc_blob = O.vrs_location_blob(seq, 44908821, 44908822, schema="1.1")
    assert engine.sha512t24u([loc_blob]) == ["u5fspwVbQ79QkX6GHLF8tXPCAXFJqRPx"]
    assert engine.sha512t24u([O.vrs_allele_blob("u5fspwVbQ79QkX6GHLF8tXPCAXFJqRPx", b"T", schema="1.1")]) == \
        ["EgHPXXhULTwoP4-ACfs-YCXaeUQJBjH_"]


def test_k4_vrs_digest_vs_oracle_serialisation(engine):
    """Long-allele key digest == the oracle's VRS-1.x serialisation + sha512t24u.
    (Parity vs vrs-python itself is UNPINNED: not available offline.)"""
    from annotatedvdb_amd import synth
    digs = ["%032d" % i for i in range(25)]
    eng2 = type(engine)(0, sequence_digests=digs)
    b = synth.alleles(20000, seed=44, long_frac=0.2)
    d, is_long = eng2.vrs_digest(b, 50)
    h = {k: getattr(b, k).cpu().numpy() for k in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "heap")}
    il = is_long.cpu().numpy()
    raw = d.cpu().numpy()
    assert il.sum() > 1000
    for i in range(b.n):
        r, a = int(h["ref_len"][i]), int(h["alt_len"][i])
        assert il[i] == (r + a > 50)
        if not il[i]:
            continue
        o = int(h["allele_off"][i])
        ref = h["heap"][o:o + r].tobytes()
        alt = h["heap"][o + r:o + r + a].tobytes()
        exp = O.vrs_allele_digest(digs[h["chrom"][i]], int(h["pos"][i]), ref, alt)
        assert raw[i].tobytes().decode() == exp


def test_k4_is_long_ragged_batch(engine):
    """is_long / digests for batch sizes that end inside a 4-record group (the
    compaction kernels' 16-byte-load path stores is_long 4 bytes at a time)."""
    from annotatedvdb_amd import synth
    digs = ["%032d" % i for i in range(25)]
    eng2 = type(engine)(0, sequence_digests=digs)
    for n in (1, 3, 4097, 20003):
        b = synth.alleles(n, seed=45 + n, long_frac=0.3)
        d, is_long = eng2.vrs_digest(b, 50)
        r, a = b.ref_len.cpu().numpy().astype(np.int64), b.alt_len.cpu().numpy()
        assert np.array_equal(is_long.cpu().numpy(), (r + a > 50).astype(np.uint8)), n


@pytest.mark.slow
def test_c5_all_shards_vs_c_oracle(engine):
    """BASELINE config 5's whole job (8 ranks x 2.5e7 ADSP-style records, the
    bench's generator, seeds and pieces) on one GPU through ``pipeline.PrepStep``,
    the object the bench times (K2 with K4's codes and K3's marks, K3 resolving the
    listed runs, K4 from the codes), on sentinel-filled buffers: end / bin / status
    (K2) and keep-first (K3) bit-exact vs the C oracle for all 2e8 records; the
    digests and long flags equal K4 run alone (classifying from the lengths)."""
    import oracle
    from annotatedvdb_amd import shard, synth
    from annotatedvdb_amd.pipeline import PrepStep
    n = 25_000_000
    lens = np.asarray(LENGTHS, dtype=np.uint32)
    plan = shard.plan(8)
    digs = ["%032d" % (11 * i) for i in range(25)]
    eng = type(engine)(0, sequence_digests=digs)
    eng.poison = 0xA5
    for rank in range(8):
        b = synth.alleles(n, seed=5 + 1000 * rank, pieces=plan[rank])
        o = PrepStep(eng, b).run()
        end, code, status, keep = o["end"], o["code"], o["status"], o["keep"]
        if rank == 0:
            d0, l0 = eng.vrs_digest(b, 50)  # (no codes pending: K4's own length pass)
            assert torch.equal(o["is_long"], l0)
            sel = l0.bool()
            assert int(sel.sum()) > 0 and torch.equal(o["digest"][sel], d0[sel])
        h = {k: getattr(b, k).cpu().numpy() for k in ("chrom", "pos", "allele_off", "ref_len", "alt_len",
                                                      "heap", "ext_id")}
        re_, rc, rl = (np.empty(n, dtype=np.uint32) for _ in range(3))
        rs = np.empty(n, dtype=np.uint8)
        oracle.c_oracle().avdb_oracle_record_prep(
            h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data, h["ref_len"].ctypes.data,
            h["alt_len"].ctypes.data, h["heap"].ctypes.data, n, lens.ctypes.data, len(lens),
            re_.ctypes.data, rc.ctypes.data, rs.ctypes.data, rl.ctypes.data)
        assert np.array_equal(u32(end), re_), rank
        assert np.array_equal(u32(code), rc), rank
        assert np.array_equal(status.cpu().numpy(), rs), rank
        ek = np.empty(n, dtype=np.uint8)
        oracle.c_oracle().avdb_oracle_dedup_grouped(
            h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data, h["ref_len"].ctypes.data,
            h["alt_len"].ctypes.data, h["heap"].ctypes.data, h["ext_id"].ctypes.data, n, ek.ctypes.data)
        assert np.array_equal(keep[:n].cpu().numpy(), ek), rank
        del b, o, end, code, status, keep, h
    eng.poison = None


@pytest.mark.slow
def test_c5_full_size_vs_c_oracle(engine):
    """BASELINE config 5 at full per-GPU size (2.5e7 ADSP-style records): K2 end /
    bin / status and K3 keep-first bit-exact vs the C oracle; the hash-path dedup
    equals the grouped path; long-key digests on a sample vs the oracle's
    serialisation (VRS layout itself unpinned)."""
    import oracle
    from annotatedvdb_amd import synth
    n = 25_000_000
    b = synth.alleles(n, seed=5)
    end, code, status, _ = engine.record_prep(b, want_lcp=False)
    h = {k: getattr(b, k).cpu().numpy() for k in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "heap",
                                                  "ext_id")}
    re_, rc, rl = (np.empty(n, dtype=np.uint32) for _ in range(3))
    rs = np.empty(n, dtype=np.uint8)
    lens = np.asarray(LENGTHS, dtype=np.uint32)
    oracle.c_oracle().avdb_oracle_record_prep(
        h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data, h["ref_len"].ctypes.data,
        h["alt_len"].ctypes.data, h["heap"].ctypes.data, n, lens.ctypes.data, len(lens),
        re_.ctypes.data, rc.ctypes.data, rs.ctypes.data, rl.ctypes.data)
    assert np.array_equal(u32(end), re_)
    assert np.array_equal(u32(code), rc)
    assert np.array_equal(status.cpu().numpy(), rs)
    keep = np.empty(n, dtype=np.uint8)
    ndup = oracle.c_oracle().avdb_oracle_dedup_grouped(
        h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data, h["ref_len"].ctypes.data,
        h["alt_len"].ctypes.data, h["heap"].ctypes.data, h["ext_id"].ctypes.data, n, keep.ctypes.data)
    kg = engine.pk_dedup(b, grouped=True)
    assert np.array_equal(kg.cpu().numpy(), keep) and ndup > 0
    kh = engine.pk_dedup(b, grouped=False)
    assert torch.equal(kg, kh)
    digs = ["%032d" % i for i in range(25)]
    eng2 = type(engine)(0, sequence_digests=digs)
    d, is_long = eng2.vrs_digest(b, 50)
    il = is_long.cpu().numpy()
    assert np.array_equal(il, (h["ref_len"].astype(np.int64) + h["alt_len"] > 50).astype(np.uint8))
    # every long record's digest vs the C oracle's serialisation + SHA-512
    exp = np.zeros(n * 32, dtype=np.uint8)
    buf = np.zeros(8192, dtype=np.uint8)
    oracle.c_oracle().avdb_oracle_vrs_digest(
        h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data, h["ref_len"].ctypes.data,
        h["alt_len"].ctypes.data, h["heap"].ctypes.data, n, 50, "".join(digs).encode(), 25, buf.ctypes.data,
        exp.ctypes.data)
    got = d.cpu().numpy().reshape(n, 32)
    rows = np.nonzero(il)[0]
    assert len(rows) > 1_000_000
    assert np.array_equal(got[rows], exp.reshape(n, 32)[rows])
    # and a sample through the Python restatement
    sel = rows[np.random.default_rng(5).choice(len(rows), 100, replace=False)]
    for i in sel:
        o, r, a = int(h["allele_off"][i]), int(h["ref_len"][i]), int(h["alt_len"][i])
        e = O.vrs_allele_digest(digs[h["chrom"][i]], int(h["pos"][i]), h["heap"][o:o + r].tobytes(),
                                h["heap"][o + r:o + r + a].tobytes())
        assert got[i].tobytes().decode() == e


# ---------------------------------------------------------------------------
# launch-shape knobs: the same kernels on other grids give the same results
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("knob,value", [("AVDB_K1_BLOCKS_PER_CU", "1"), ("AVDB_K2_BLOCKS_PER_CU", "16"),
                                        ("AVDB_K4_BLOCKS_PER_CU", "1"), ("AVDB_K7_RAW_BLOCKS", "0")])
def test_grid_knobs_parity(engine, knob, value):
    """Every environment knob the library reads (``grep getenv csrc/``) at a
    non-default value: K1 spans + histogram, the keyed step (K2, K3, K4, K7) and
    its outputs equal the default context's; and ``AVDB_OPT_K4_GRID`` /
    ``AVDB_OPT_K7_GRID`` (K4's persistent grid and K7's write-pass grid, what the
    overlap layout shrinks) the same way, in the serial and the overlap layout."""
    from annotatedvdb_amd import _native as N
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.engine import Engine
    from annotatedvdb_amd.pipeline import KeyedStep
    digs = ["%032d" % (13 * i) for i in range(25)]
    os.environ[knob] = value
    try:
        alt = Engine(0, sequence_digests=digs)
    finally:
        del os.environ[knob]
    ref = Engine(0, sequence_digests=digs)
    chrom, start, end = synth.np_spans(1 << 20, seed=4)
    outs = []
    for e in (ref, alt):
        h = e.new_histogram()
        code, status = e.bin_assign(torch.from_numpy(chrom), torch.from_numpy(start), torch.from_numpy(end), hist=h)
        outs.append((code, status, h))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
    n = 3 * 4096 * 64 + 77  # several K7 scan blocks
    b = synth.alleles(n, seed=6, long_frac=0.04, dup_frac=0.05, device="cuda")
    res = []
    for e, grid, layout in ((ref, 0, "serial"), (alt, 0, "serial"), (alt, 37, "serial"), (alt, 37, "overlap")):
        o = KeyedStep(e, b, digests=True, layout=layout, k4_grid=grid, k7_grid=grid).run()
        kt = o["kt"]
        sel = o["is_long"].bool()
        res.append((o["end"], o["code"], o["status"], o["keep"][:n], o["is_long"], o["digest"][sel],
                    kt.key_offsets(n), kt.path_offsets(n), kt.state[:n], kt.keys[: int(kt.key_offsets(n)[n])],
                    kt.paths[: int(kt.path_offsets(n)[n])]))
    for r in res[1:]:
        for x, y in zip(res[0], r):
            assert torch.equal(x, y)
    with pytest.raises(N.NativeError):
        alt.set_option(N.OPT_K4_GRID, -1)
    with pytest.raises(N.NativeError):
        alt.set_option(N.OPT_K7_GRID, -1)
    with pytest.raises(N.NativeError):
        alt.set_option(99, 1)


@pytest.mark.parametrize("n", [1, 3, 4, 5, 257, 1000, 300001])
def test_prep_step_equals_plain_chain(engine, n):
    """pipeline.PrepStep (the C5 step: keyed K2 without K7 totals, so it classifies
    long records for K4 and runs K3's mark phase; below 4 records or unaligned it is
    the plain K2) gives the plain K2 -> K3 -> K4 chain's outputs at sizes around the
    vector form's edges, with duplicates and long alleles, two steps over the same
    buffers."""
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.pipeline import PrepStep
    digs = ["%032d" % (3 * i) for i in range(25)]
    eng = type(engine)(0, sequence_digests=digs)
    b = synth.alleles(n, seed=40 + n % 13, long_frac=0.05, dup_frac=0.05, device="cuda")
    end, code, status, _ = eng.record_prep(b, want_lcp=False)
    keep = eng.pk_dedup(b, grouped=True)
    dig, is_long = eng.vrs_digest(b, 50)
    ps = PrepStep(eng, b)
    for _ in range(2):
        o = ps.run()
        for k, v in (("end", end), ("code", code), ("status", status)):
            assert torch.equal(o[k][:n], v[:n]), k
        assert torch.equal(o["keep"][:n], keep[:n])
        assert torch.equal(o["is_long"][:n], is_long[:n])
        sel = is_long[:n].bool()
        assert torch.equal(o["digest"][:n][sel], dig[:n][sel])
