"""GPU parity for BASELINE config C1 (chr22, 1.1 M records) and K7 (primary
keys + bin paths as text): the whole C1 batch through K2 / K3 / K7 vs the C
oracle, and its 100,000-record prefix vs what the reference itself computed
(tests/golden/c1_prefix.tsv.gz)."""

import gzip
import os

import numpy as np
import pytest

from conftest import GOLDEN
from annotatedvdb_amd.chromosomes import CHROM_NAMES, length_table
from oracle import avdb_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LENGTHS = np.asarray(length_table(), dtype=np.uint32)
FIELDS = ("chrom", "pos", "allele_off", "ref_len", "alt_len", "heap", "ext_id")


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def host(b):
    return {k: getattr(b, k).cpu().numpy() for k in FIELDS}


def oracle_keys(h, digest=None, max_len=50):
    import oracle
    n = len(h["pos"])
    cap = int(h["ref_len"].astype(np.int64).sum() + h["alt_len"].sum()) + 80 * n + 8
    out = np.zeros(cap, dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.uint64)
    dg = None if digest is None else digest.ctypes.data
    oracle.c_oracle().avdb_oracle_primary_keys(
        h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data, h["ref_len"].ctypes.data,
        h["alt_len"].ctypes.data, h["heap"].ctypes.data, h["ext_id"].ctypes.data, dg, n, max_len,
        out.ctypes.data, off.ctypes.data)
    return out[: int(off[n])].tobytes(), off


def oracle_prep(h):
    import oracle
    n = len(h["pos"])
    end, code, lcp = (np.empty(n, dtype=np.uint32) for _ in range(3))
    status = np.empty(n, dtype=np.uint8)
    keep = np.empty(n, dtype=np.uint8)
    lib = oracle.c_oracle()
    lib.avdb_oracle_record_prep(h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data,
                                h["ref_len"].ctypes.data, h["alt_len"].ctypes.data, h["heap"].ctypes.data, n,
                                LENGTHS.ctypes.data, len(LENGTHS), end.ctypes.data, code.ctypes.data,
                                status.ctypes.data, lcp.ctypes.data)
    lib.avdb_oracle_dedup_grouped(h["chrom"].ctypes.data, h["pos"].ctypes.data, h["allele_off"].ctypes.data,
                                  h["ref_len"].ctypes.data, h["alt_len"].ctypes.data, h["heap"].ctypes.data,
                                  h["ext_id"].ctypes.data, n, keep.ctypes.data)
    return end, code, status, keep


def paths_of(chrom, code):
    """ltree text per record via the Python oracle (one format per distinct code)."""
    memo = {}
    out = []
    for c, k in zip(chrom.tolist(), code.tolist()):
        if k == O.BIN_NONE:
            out.append(None)
            continue
        p = memo.get((c, k))
        if p is None:
            p = memo[(c, k)] = O.format_bin_path(CHROM_NAMES[c], k)
        out.append(p)
    return out


def test_c1_whole_batch_vs_c_oracle(engine):
    """All 1.1 M C1 records: end / bin / status (K2), keep (K3), key and path
    text (K7) bit-exact vs the C oracle."""
    from annotatedvdb_amd import synth
    b = synth.c1_batch(device="cuda")
    n = b.n
    end, code, status, _ = engine.record_prep(b, want_lcp=False)
    keep = engine.pk_dedup(b, grouped=True)
    kt = engine.primary_keys(b, code=code)
    h = host(b)
    re_, rc, rs, rk = oracle_prep(h)
    assert np.array_equal(u32(end), re_)
    assert np.array_equal(u32(code), rc)
    assert np.array_equal(status.cpu().numpy(), rs) and not rs.any()
    assert np.array_equal(keep.cpu().numpy(), rk)
    assert not kt.state[:n].cpu().numpy().any()
    kb, ko = oracle_keys(h)
    assert np.array_equal(kt.key_off.cpu().numpy().astype(np.uint64), ko)
    # (array compares: a failing bytes == bytes assert makes pytest diff 26 MB)
    assert np.array_equal(kt.keys[: len(kb)].cpu().numpy(), np.frombuffer(kb, dtype=np.uint8))
    po = kt.path_off.cpu().numpy()
    pb = kt.paths[: int(po[n])].cpu().numpy().tobytes().decode()
    exp = paths_of(h["chrom"], rc)
    assert all(pb[po[i]:po[i + 1]] == exp[i] for i in range(n))


def test_c1_prefix_vs_reference_golden(engine):
    """The first 100,000 C1 records: GPU end, bin path and primary key equal the
    reference's own VariantAnnotator / BinIndex / VariantPKGenerator output."""
    from annotatedvdb_amd import synth
    with gzip.open(os.path.join(GOLDEN, "c1_prefix.tsv.gz"), "rt") as fh:
        fh.readline()
        rows = [ln.rstrip("\n").split("\t") for ln in fh]
    b = synth.c1_batch(device="cuda")
    end, code, status, _ = engine.record_prep(b, want_lcp=False)
    kt = engine.primary_keys(b, code=code)
    keys, paths = kt.host(len(rows))
    e = u32(end)
    for i, (pk, ee, path) in enumerate(rows):
        assert keys[i] == pk, i
        assert str(e[i]) == ee, i
        assert paths[i] == path, i


def test_k7_keys_long_digests_and_ragged_batches(engine):
    """K7 on ADSP-style batches (long alleles keyed by the K4 digest, rsids)
    vs the C oracle, at batch sizes that end off every alignment."""
    from annotatedvdb_amd import synth
    digs = ["%032d" % (3 * i) for i in range(25)]
    eng2 = type(engine)(0, sequence_digests=digs)
    for n in (1, 7, 4099, 60001):
        b = synth.alleles(n, seed=70 + n, long_frac=0.1)
        dig, _ = eng2.vrs_digest(b, 50)
        end, code, status, _ = eng2.record_prep(b, want_lcp=False)
        kt = eng2.primary_keys(b, code=code, digest=dig)
        h = host(b)
        hd = dig.cpu().numpy().reshape(-1).copy()
        kb, ko = oracle_keys(h, digest=hd)
        assert not kt.state[:n].cpu().numpy().any(), n
        assert np.array_equal(kt.key_off.cpu().numpy().astype(np.uint64), ko), n
        assert np.array_equal(kt.keys[: len(kb)].cpu().numpy(), np.frombuffer(kb, dtype=np.uint8)), n
        _, paths = kt.host(n)
        assert paths == paths_of(h["chrom"], u32(code)), n


def test_k7_states_and_edge_records(engine):
    """':' in an allele (the reference's ValueError), interned external ids,
    long records without digests, unlabelled contigs and unmappable bins."""
    from annotatedvdb_amd.engine import pack_records
    from annotatedvdb_amd import _native as N
    recs = [(0, 100, b"A", b"G", 0), (1, 5, b"A:C", b"A", 0), (2, 9, b"C", b"T", (1 << 63) | 4),
            (3, 11, b"A" * 30, b"C" * 30, 7), (30, 12, b"A", b"C", 0), (24, 16569, b"T", b"TAA", 12),
            (21, 50818468, b"G", b"GT", 0), (22, 1, b"", b"A", 5)]
    b = pack_records([r[0] for r in recs], [r[1] for r in recs], [r[2] for r in recs], [r[3] for r in recs],
                     [r[4] for r in recs])
    b = b.to("cuda")
    end, code, status, _ = engine.record_prep(b, want_lcp=False)
    kt = engine.primary_keys(b, code=code)
    st = kt.state[: b.n].cpu().tolist()
    keys, paths = kt.host(b.n)
    assert st == [N.KEY_OK, N.KEY_HOST, N.KEY_HOST, N.KEY_NEED_DIGEST, N.KEY_HOST, N.KEY_OK, N.KEY_OK, N.KEY_OK]
    assert keys[0] == "1:100:A:G"
    assert keys[5] == "M:16569:T:TAA:rs12" and paths[5] is None  # end 16570 > chrM
    assert keys[6] == "22:50818468:G:GT"
    assert keys[7] == "X:1::A:rs5"
    c = u32(code)
    assert paths[4] is None and c[4] == O.BIN_NONE            # contig 30: unknown
    assert paths[6] is None and c[6] == O.BIN_NONE            # end past chr22's length
    assert paths[0] == O.format_bin_path("1", int(c[0]))
    # empty batch
    e = pack_records([], [], [], []).to("cuda")
    kt0 = engine.primary_keys(e)
    assert int(kt0.key_off[0]) == 0
    # ... and in the narrow layout (one u32 word and one u64 base)
    k32 = engine.primary_keys(e, out=engine.new_key_text(0, 1, off32=True))
    assert k32.off32 and k32.key_offsets(0).tolist() == [0]


@pytest.mark.parametrize("mode", ["gpu", "host"])
def test_k8_small_batch_equals_multi_kernel_path(engine, mode):
    """K8 (one launch, host-mapped memory) and K8h (the same record arithmetic in
    the library's host code: the per-call drop-in path) give the same end / bin /
    status, key text, ltree path and display-attribute JSON as K2 + K7 + K5a on
    the same records, across allele classes and edge records."""
    from annotatedvdb_amd import _native as N
    sp = engine.small()
    old_mode = sp.mode
    sp.mode = mode
    try:
        _k8_vs_kernels(engine, N, sp)
        assert sp.last_path == mode
    finally:
        sp.mode = old_mode


def _k8_vs_kernels(engine, N, sp):
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.engine import pack_records
    b = synth.alleles(3000, seed=81, long_frac=0.05)
    h = host(b)
    n = b.n
    refs = [h["heap"][o:o + r].tobytes() for o, r in zip(h["allele_off"], h["ref_len"])]
    alts = [h["heap"][o + r:o + r + a].tobytes() for o, r, a in zip(h["allele_off"], h["ref_len"], h["alt_len"])]
    extra = [(0, 100, b"A:C", b"A", 0), (24, 16569, b"T", b"TAA", 12), (30, 5, b"A", b"G", 0),
             (21, 50818468, b"G", b"GT", 0), (0, 7, b"AT", b"AT", 5), (2, 9, b"C", b"T", (1 << 63) | 4)]
    chrom = list(h["chrom"]) + [e[0] for e in extra]
    pos = list(h["pos"]) + [e[1] for e in extra]
    refs += [e[2] for e in extra]
    alts += [e[3] for e in extra]
    ext = [int(x) for x in h["ext_id"]] + [e[4] for e in extra]
    res = sp.run(chrom, pos, refs=refs, alts=alts, ext=ext,
                             want=N.SMALL_PATH | N.SMALL_KEY | N.SMALL_DISPLAY)
    assert res is not None
    db = pack_records(chrom, pos, refs, alts, ext).to("cuda")
    end, code, status, _ = engine.record_prep(db, want_lcp=False)
    assert np.array_equal(res["end"], u32(end))
    assert np.array_equal(res["code"], u32(code))
    assert np.array_equal(res["status"], status.cpu().numpy())
    kt = engine.primary_keys(db, code=code)
    keys, paths = kt.host(db.n)
    ks = kt.state[: db.n].cpu().numpy()
    # K7 without digests: long records are NEED_DIGEST in both
    assert np.array_equal(res["key_state"], ks)
    assert [k if s == N.KEY_OK else None for k, s in zip(res["key"], res["key_state"])] == keys
    assert res["path"] == paths
    text, off, st = engine.display_attributes(db, end)
    raw = text.cpu().numpy().tobytes().decode()
    o = off.cpu().numpy()
    assert np.array_equal(res["disp_state"], st.cpu().numpy())
    exp_disp = [raw[o[i]:o[i + 1]] if st[i] == 0 else None for i in range(db.n)]
    assert res["display"] == exp_disp
    # bins of explicit intervals (the find_bin_index miss path)
    r2 = sp.run([0, 0, 21, 99], [15625, 1, 50818468, 5], ends=[15626, 248956422, 50818469, 5],
                            want=N.SMALL_PATH)
    assert r2["path"][0] == O.format_bin_path("1", int(r2["code"][0])) and r2["path"][1] == "chr1"
    assert r2["path"][2] is None and r2["path"][3] is None
    assert list(r2["status"]) == [0, 0, 2, 1]


@pytest.mark.parametrize("onepass", [False, True])
def test_k7_reused_buffers_flag_overflow(engine, onepass):
    """A KeyText reused for a batch whose keys and paths are longer: the texts
    that do not fit are not written and their records say so (KEY_OVERFLOW,
    PATH_OVERFLOW); KeyText.host refuses the batch instead of returning stale text."""
    from annotatedvdb_amd import _native as N
    from annotatedvdb_amd.engine import pack_records
    a = pack_records([0] * 64, [100] * 64, [b"A"] * 64, [b"G"] * 64).to("cuda")
    _, code, _, _ = engine.record_prep(a, want_lcp=False)
    kt = engine.primary_keys(a, code=code, onepass=onepass)
    assert kt.host(64)[0][0] == "1:100:A:G"
    if onepass:  # buffers sized by avdb_primary_keys_bound: shrink them to the first batch's text
        kt.keys, kt.paths = kt.keys[: int(kt.key_off[64])], kt.paths[: int(kt.path_off[64])]
    b = pack_records([9] * 64, [100000] * 64, [b"ACGTACGTAC"] * 64, [b"G"] * 64).to("cuda")  # leaf bins: 87-byte paths
    _, code2, _, _ = engine.record_prep(b, want_lcp=False)
    kt2 = engine.primary_keys(b, code=code2, out=kt, onepass=onepass)
    st = kt2.state[:64].cpu().numpy()
    assert ((st & 0x0F) == N.KEY_OVERFLOW).sum() > 0 and ((st & N.PATH_OVERFLOW) != 0).sum() > 0
    assert ((st & 0x0F) == N.KEY_OK).sum() > 0  # the keys that fit were written
    with pytest.raises(ValueError):
        kt2.host(64)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 257, 4097, 300001, 1048577 + 300, (4 << 20) - 1, (4 << 20) + 4097])
def test_k7_onepass_equals_two_pass(engine, n):
    """K7 with group offsets (group totals + two scans + a write pass that writes
    the offsets) == the size pass + hipCUB scans + write pass: offsets, states, key
    and path text, at sizes that end off every tile, group and scan-block boundary,
    with one-tile groups (below 4 M records) and four-tile groups (from 4 M on)."""
    from annotatedvdb_amd import synth
    digs = ["%032d" % (7 * i) for i in range(25)]
    engine.set_sequence_digests(digs)
    b = synth.alleles(n, seed=90 + n % 7, long_frac=0.05, device="cuda")
    end, code, status, _ = engine.record_prep(b, want_lcp=False)
    dig, _ = engine.vrs_digest(b, 50)
    one = engine.primary_keys(b, code=code, digest=dig)
    two = engine.primary_keys(b, code=code, digest=dig, onepass=False)
    for a, c in ((one.key_off, two.key_off), (one.path_off, two.path_off)):
        assert torch.equal(a[: n + 1], c[: n + 1])
    assert torch.equal(one.state[:n], two.state[:n])
    kn, pn = int(two.key_off[n]), int(two.path_off[n])
    assert torch.equal(one.keys[:kn], two.keys[:kn]) and torch.equal(one.paths[:pn], two.paths[:pn])
    # and reused buffers: a second launch over the same KeyText
    again = engine.primary_keys(b, code=code, digest=dig, out=one)
    assert torch.equal(again.keys[:kn], two.keys[:kn]) and torch.equal(again.key_off[: n + 1], two.key_off[: n + 1])


@pytest.mark.parametrize("n", [(4 << 20) + 4099, (4 << 20) + 256 * 7, 1100000, 300001, 4097, 130, 64, 5, 3])
def test_keyed_record_prep_feeds_k7(engine, n):
    """K2 writing K7's group totals (avdb_record_prep_keyed, the C4k and C1
    pipelines) then K7 without its totals pass == plain K2 + K7: end / bin / status
    and every key, path, offset and state — 256-record groups from 4 Mi records on,
    64-record groups (four per K2 wave step) below; under 4 records the keyed call
    is plain K2 and K7 sums the totals itself.  The keyed pair writes into a fresh
    KeyText whose workspace, offsets, states and text are all sentinel bytes."""
    from annotatedvdb_amd import synth
    digs = ["%032d" % (5 * i) for i in range(25)]
    engine.set_sequence_digests(digs)
    b = synth.alleles(n, seed=11 + n % 5, long_frac=0.03, device="cuda")
    end, code, status, _ = engine.record_prep(b, want_lcp=False)
    dig, _ = engine.vrs_digest(b, 50)
    ref = engine.primary_keys(b, code=code, digest=dig)
    kt = engine.new_key_text(n, b.heap.numel())  # fresh buffers, every byte a sentinel
    for t in (kt.ws, kt.key_off, kt.path_off, kt.state, kt.keys, kt.paths):
        t.view(torch.uint8).fill_(0xA5)
    end2, code2, status2, _ = engine.record_prep(b, want_lcp=False, keys=kt, key_digest=True)
    assert ("totals" in engine._pending) == (n >= 4)
    assert torch.equal(end, end2) and torch.equal(code, code2) and torch.equal(status, status2)
    out = engine.primary_keys(b, code=code2, digest=dig, out=kt)
    assert "totals" not in engine._pending
    assert torch.equal(out.key_off[: n + 1], ref.key_off[: n + 1])
    assert torch.equal(out.path_off[: n + 1], ref.path_off[: n + 1])
    assert torch.equal(out.state[:n], ref.state[:n])
    kn, pn = int(ref.key_off[n]), int(ref.path_off[n])
    assert torch.equal(out.keys[:kn], ref.keys[:kn]) and torch.equal(out.paths[:pn], ref.paths[:pn])


def test_keyed_totals_not_reused_for_another_batch(engine):
    """Group totals a keyed K2 left for batch A are not taken for batch B of the
    same size: B's keys and offsets are B's own."""
    from annotatedvdb_amd import synth
    n = (4 << 20) + 17
    engine.set_sequence_digests(["%032d" % (3 * i) for i in range(25)])
    a = synth.alleles(n, seed=21, long_frac=0.02, device="cuda")
    b = synth.alleles(n, seed=22, long_frac=0.02, device="cuda")
    _, ca, _, _ = engine.record_prep(a, want_lcp=False)
    _, cb, _, _ = engine.record_prep(b, want_lcp=False)
    da, _ = engine.vrs_digest(a, 50)
    db, _ = engine.vrs_digest(b, 50)
    ref = engine.primary_keys(b, code=cb, digest=db)
    kt = engine.primary_keys(a, code=ca, digest=da)
    engine.record_prep(a, want_lcp=False, keys=kt, key_digest=True)
    assert "totals" in engine._pending
    out = engine.primary_keys(b, code=cb, digest=db, out=kt)
    assert torch.equal(out.key_off[: n + 1], ref.key_off[: n + 1])
    assert torch.equal(out.path_off[: n + 1], ref.path_off[: n + 1])


def test_keyed_handoffs_not_taken_after_realloc_or_inplace_edit(engine):
    """a keyed K2's hand-offs are tied to the tensors themselves, not
    to their addresses.  (1) The batch is freed and a same-size batch is
    allocated (the caching allocator hands back the same blocks): K7 / K4 / K3
    compute the new batch's own results.  (2) The batch is edited in place
    between K2 and K7 (refSNP ids removed, so key sizes change): K7 recomputes."""
    from annotatedvdb_amd import synth
    n = (4 << 20) + 17
    engine.set_sequence_digests(["%032d" % (7 * i) for i in range(25)])
    a = synth.alleles(n, seed=31, long_frac=0.02, dup_frac=0.05, device="cuda")
    _, ca, _, _ = engine.record_prep(a, want_lcp=False)
    kt = engine.primary_keys(a, code=ca)
    sz = __import__("ctypes").c_size_t()
    engine.lib.avdb_vrs_digest_workspace_size(n, __import__("ctypes").byref(sz))
    ws4 = torch.zeros(int(sz.value), dtype=torch.uint8, device="cuda")
    ws3 = torch.empty(16384 + 4 * (((n + 3) & ~3) + (1 << 22)), dtype=torch.uint8, device="cuda")
    engine.record_prep(a, want_lcp=False, keys=kt, key_digest=True, digest_workspace=ws4, dedup_workspace=ws3)
    assert set(engine._pending) == {"totals", "codes", "marks"}
    ptrs = (a.chrom.data_ptr(), a.pos.data_ptr(), a.ref_len.data_ptr())
    del a, ca
    b = synth.alleles(n, seed=32, long_frac=0.02, dup_frac=0.05, device="cuda")
    _, cb, _, _ = engine.record_prep(b, want_lcp=False)  # (clears the pending entries too)
    engine._pending.clear()
    ref_keep = engine.pk_dedup(b, grouped=True)
    ref_dig, ref_long = engine.vrs_digest(b, 50)
    ref = engine.primary_keys(b, code=cb, digest=ref_dig)
    # re-create the stale entries as a skipped consumer would have left them
    a2 = synth.alleles(n, seed=31, long_frac=0.02, dup_frac=0.05, device="cuda")
    _, ca2, _, _ = engine.record_prep(a2, want_lcp=False)
    engine.record_prep(a2, want_lcp=False, keys=kt, key_digest=True, digest_workspace=ws4, dedup_workspace=ws3)
    stale = dict(engine._pending)
    del a2, ca2
    b2 = synth.alleles(n, seed=32, long_frac=0.02, dup_frac=0.05, device="cuda")
    engine._pending.update(stale)  # as if nothing had run since
    keep = engine.pk_dedup(b2, grouped=True, workspace=ws3)
    dig, is_long = engine.vrs_digest(b2, 50, workspace=ws4)
    _, cb2, _, _ = engine.record_prep(b2, want_lcp=False)
    engine._pending.update(stale)
    out = engine.primary_keys(b2, code=cb2, digest=dig, out=kt)
    assert torch.equal(keep[:n], ref_keep[:n]) and torch.equal(is_long[:n], ref_long[:n])
    assert torch.equal(out.key_off[: n + 1], ref.key_off[: n + 1])
    assert torch.equal(out.path_off[: n + 1], ref.path_off[: n + 1])
    del ptrs
    # (2) in-place edit between the keyed K2 and K7
    _, cb3, _, _ = engine.record_prep(b2, want_lcp=False, keys=kt, key_digest=True)
    assert "totals" in engine._pending
    b2.ext_id[::3] = 0
    ref2 = engine.primary_keys(b2, code=cb3, digest=dig)
    engine._pending.clear()
    engine.record_prep(b2, want_lcp=False, keys=kt, key_digest=True)
    b2.ext_id[1::3] = 0
    out2 = engine.primary_keys(b2, code=cb3, digest=dig, out=kt)
    ref3 = engine.primary_keys(b2, code=cb3, digest=dig)
    assert torch.equal(out2.key_off[: n + 1], ref3.key_off[: n + 1])
    kn = int(ref3.key_off[n])
    assert torch.equal(out2.keys[:kn], ref3.keys[:kn])
    del ref2


def test_k7_block_scan_launch_equals_raw_block_sums(engine):
    """Past ctx->k7_raw_blocks blocks of 4,096 groups K7 scans the block totals in
    a launch of its own; below, the write pass sums them.  Both give the same
    offsets and text (forced here with AVDB_K7_RAW_BLOCKS=0 on a second context)."""
    import os
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.engine import Engine
    n = 3 * 4096 * 64 + 77  # four blocks of 64-record groups
    b = synth.alleles(n, seed=5, long_frac=0.0, device="cuda")
    _, code, _, _ = engine.record_prep(b, want_lcp=False)
    raw = engine.primary_keys(b, code=code)
    os.environ["AVDB_K7_RAW_BLOCKS"] = "0"
    try:
        e2 = Engine(0)
    finally:
        del os.environ["AVDB_K7_RAW_BLOCKS"]
    scanned = e2.primary_keys(b, code=code)
    assert torch.equal(raw.key_off[: n + 1], scanned.key_off[: n + 1])
    assert torch.equal(raw.path_off[: n + 1], scanned.path_off[: n + 1])
    assert torch.equal(raw.state[:n], scanned.state[:n])
    kn, pn = int(raw.key_off[n]), int(raw.path_off[n])
    assert torch.equal(raw.keys[:kn], scanned.keys[:kn]) and torch.equal(raw.paths[:pn], scanned.paths[:pn])


@pytest.mark.parametrize("n,long_frac", [((4 << 20) + 4099, 0.03), (1100000, 0.02), (4097, 0.5), (130, 1.0), (5, 0.4),
                                         (3, 1.0)])
def test_keyed_record_prep_classifies_for_k4(engine, n, long_frac):
    """The keyed K2 with a K4 workspace writes each record's long-record bucket
    (avdb_record_prep_keyed + AVDB_DIGEST_CODES_READY): K4 then skips its pass over
    both length arrays and gives the same digests and is_long flags as on its own;
    the workspace is not taken for another batch or another max_seq_len."""
    from annotatedvdb_amd import synth
    digs = ["%032d" % (11 * i) for i in range(25)]
    engine.set_sequence_digests(digs)
    b = synth.alleles(n, seed=13 + n % 7, long_frac=long_frac, device="cuda")
    ref_dig, ref_long = engine.vrs_digest(b, 50)
    sel = ref_long.bool()
    kt = engine.primary_keys(b, code=engine.record_prep(b, want_lcp=False)[1], digest=ref_dig)
    sz = __import__("ctypes").c_size_t()
    engine.lib.avdb_vrs_digest_workspace_size(n, __import__("ctypes").byref(sz))
    ws = torch.zeros(int(sz.value), dtype=torch.uint8, device="cuda")
    engine.record_prep(b, want_lcp=False, keys=kt, key_digest=True, digest_workspace=ws)
    assert ("codes" in engine._pending) == (n >= 4)
    dig, is_long = engine.vrs_digest(b, 50, workspace=ws)
    assert "codes" not in engine._pending
    assert torch.equal(is_long[:n], ref_long[:n])
    assert torch.equal(dig[sel], ref_dig[sel])
    # another max_seq_len: the codes are not used
    engine.record_prep(b, want_lcp=False, keys=kt, key_digest=True, digest_workspace=ws)
    dig2, is_long2 = engine.vrs_digest(b, 20, workspace=ws)
    ref2_dig, ref2_long = engine.vrs_digest(b, 20)
    assert torch.equal(is_long2[:n], ref2_long[:n])
    sel2 = ref2_long.bool()
    assert torch.equal(dig2[sel2], ref2_dig[sel2])


@pytest.mark.parametrize("n,dup", [((4 << 20) + 4099, 0.01), (1100000, 0.05), (300001, 0.3), (4097, 0.5), (130, 0.5),
                                   (7, 0.5), (5, 0.0)])
def test_keyed_record_prep_marks_for_k3(engine, n, dup):
    """The keyed K2 with a K3 workspace runs K3's first phase (keep = 1, the records
    sharing their predecessor's position listed per K2 workgroup; avdb_pk_dedup_ex +
    AVDB_DEDUP_MARKED resolves them): the same keep flags and duplicate count as
    K3 on its own; a workspace marked for one batch is not taken for another."""
    from annotatedvdb_amd import _native as N
    from annotatedvdb_amd import synth
    b = synth.alleles(n, seed=17 + n % 5, long_frac=0.02, dup_frac=dup, device="cuda")
    ctr0 = torch.zeros(N.N_COUNTERS, dtype=torch.int64, device="cuda")
    ref_keep = engine.pk_dedup(b, grouped=True, counters=ctr0)
    kt = engine.primary_keys(b, code=engine.record_prep(b, want_lcp=False)[1])
    ws = torch.empty(16384 + 4 * (((n + 3) & ~3) + (1 << 22)), dtype=torch.uint8, device="cuda")
    engine.record_prep(b, want_lcp=False, keys=kt, dedup_workspace=ws)
    assert ("marks" in engine._pending) == (n >= 4)
    ctr1 = torch.zeros(N.N_COUNTERS, dtype=torch.int64, device="cuda")
    keep = engine.pk_dedup(b, grouped=True, counters=ctr1, workspace=ws)
    assert "marks" not in engine._pending
    assert torch.equal(keep[:n], ref_keep[:n])
    assert torch.equal(ctr0, ctr1)
    if dup:
        assert int((keep[:n] == 0).sum()) > 0
    # marked for batch b, then asked for batch c of the same size: c's own result
    c = synth.alleles(n, seed=99 + n % 5, long_frac=0.02, dup_frac=dup, device="cuda")
    engine.record_prep(b, want_lcp=False, keys=kt, dedup_workspace=ws)
    assert torch.equal(engine.pk_dedup(c, grouped=True, workspace=ws)[:n], engine.pk_dedup(c, grouped=True)[:n])


def _run_batch(n, seed, long_every=0):
    """Position runs of 1-6 records (lane and wave boundaries fall everywhere in them)
    whose alleles come from a small set and whose refSNP ids from {0, 7, 9}, so equal
    primary keys are frequent, also third-or-later in a run and behind a differing
    record; every `long_every`-th allele is long (> 50 bases).  Returns the batch
    (host numpy) and keep-first per (chrom, pos, ref, alt, rsid) — the primary key
    the dedup compares (removeDuplicates.sql:2-24)."""
    rng = np.random.default_rng(seed)
    runs = rng.choice([1, 2, 3, 4, 5, 6], size=n, p=[0.3, 0.3, 0.15, 0.12, 0.08, 0.05])
    pos = np.repeat(np.cumsum(rng.integers(1, 4, runs.size)) + 1_000_000, runs)[:n].astype(np.int32)
    alle = [b"A", b"C", b"G", b"AC", b"ACG", b"ACGTACGTA", b"AAAAAAAAAAAAAAAAAA"]
    refs = [alle[k] for k in rng.integers(0, len(alle), n)]
    alts = [alle[k] for k in rng.integers(0, 3, n)]
    if long_every:
        for i in range(0, n, long_every):
            refs[i] = b"T" * 60
    ext = rng.choice(np.array([0, 7, 9], dtype=np.int64), size=n, p=[0.2, 0.6, 0.2])
    rl = np.array([len(r) for r in refs], dtype=np.int32)
    al = np.array([len(a) for a in alts], dtype=np.int32)
    heap = b"".join(r + a for r, a in zip(refs, alts))
    off = np.concatenate([[0], np.cumsum(rl.astype(np.int64) + al)[:-1]]).astype(np.int64)
    seen, keep = set(), np.ones(n, dtype=np.uint8)
    for i in range(n):
        k = (int(pos[i]), refs[i], alts[i], int(ext[i]))
        if k in seen:
            keep[i] = 0
        seen.add(k)
    d = dict(chrom=np.full(n, 21, dtype=np.uint8), pos=pos, allele_off=off, ref_len=rl, alt_len=al,
             heap=np.frombuffer(heap, dtype=np.uint8).copy(), ext_id=ext)
    return d, keep


@pytest.mark.parametrize("n,seed,long_every", [(4097, 1, 0), (70001, 2, 0), (262147, 3, 97), (1027, 4, 5),
                                               (4_200_001, 5, 0)])
def test_keyed_marks_list_only_possible_repeats(engine, n, seed, long_every):
    """The keyed K2 lists for K3 only the same-position records that could repeat an
    earlier primary key (the predecessor's lengths and refSNP id, or third or later at
    the position); keep after the resolve equals keep-first per primary key computed
    here in Python, and K3 on its own, on runs built to hit the unlisted cases (4.2 M
    records: the C4k form of the keyed K2, 256-record groups)."""
    from annotatedvdb_amd import _native as N
    from annotatedvdb_amd.engine import RecordBatch
    d, want = _run_batch(n, seed, long_every)
    b = RecordBatch(**{k: torch.from_numpy(v).cuda() for k, v in d.items()})
    kt = engine.primary_keys(b, code=engine.record_prep(b, want_lcp=False)[1])
    ws = torch.empty(16384 + 4 * (((n + 3) & ~3) + (1 << 22)), dtype=torch.uint8, device="cuda")
    engine.record_prep(b, want_lcp=False, keys=kt, dedup_workspace=ws)
    assert "marks" in engine._pending
    ctr = torch.zeros(N.N_COUNTERS, dtype=torch.int64, device="cuda")
    keep = engine.pk_dedup(b, grouped=True, counters=ctr, workspace=ws)
    np.testing.assert_array_equal(keep[:n].cpu().numpy(), want)
    assert torch.equal(keep[:n], engine.pk_dedup(b, grouped=True)[:n])
    assert int((want == 0).sum()) > n // 100


@pytest.mark.parametrize("layout", ["onepass", "serial", "fork"])
def test_c1_graph_replay_vs_c_oracle(engine, layout):
    """The step bench.py times for C1, as it times it: ``pipeline.KeyedStep`` in
    the bench's layout (``pipeline.C1_LAYOUT``; and "fork": K3 on a second stream
    beside K7) captured once as a HIP graph and replayed.  Every buffer is a sentinel before the capture, and the
    text buffers and outputs are poisoned again between replays; after each
    replay end / bin / status / keep and every key, path, offset and state are
    bit-exact vs the C oracle."""
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.pipeline import KeyedStep
    b = synth.c1_batch(device="cuda")
    n = b.n
    h = host(b)
    re_, rc, rs, rk = oracle_prep(h)
    kb, ko = oracle_keys(h)
    exp_paths = paths_of(h["chrom"], rc)
    engine.poison = 0xA5
    try:
        ks = KeyedStep(engine, b, digests=False, layout=layout, hist=engine.new_histogram(),
                       counters=engine.new_counters())
        ks.run()  # warm-up step (the bench's warmup)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ks.run()
    finally:
        engine.poison = None
    for rep in range(2):
        out = ks.out
        for t in (out["end"], out["code"], out["status"], out["keep"], ks.kt.keys, ks.kt.paths, ks.kt.key_off,
                  ks.kt.path_off, ks.kt.state):
            t.view(torch.uint8).fill_(0x5A + rep)
        g.replay()
        torch.cuda.synchronize()
        kt = out["kt"]
        assert np.array_equal(u32(out["end"]), re_)
        assert np.array_equal(u32(out["code"]), rc)
        assert np.array_equal(out["status"].cpu().numpy(), rs)
        assert np.array_equal(out["keep"][:n].cpu().numpy(), rk)
        assert not kt.state[:n].cpu().numpy().any()
        assert np.array_equal(kt.key_offsets(n).cpu().numpy().astype(np.uint64), ko)
        assert np.array_equal(kt.keys[: len(kb)].cpu().numpy(), np.frombuffer(kb, dtype=np.uint8))
        po = kt.path_offsets(n).cpu().numpy()
        pb = kt.paths[: int(po[n])].cpu().numpy().tobytes().decode()
        assert all(pb[po[i]:po[i + 1]] == exp_paths[i] for i in range(n))


@pytest.mark.parametrize("n", [1, 5, 63, 64, 65, 4097, 300001, (4 << 20) + 4099])
def test_k7_deferred_digests_then_fill(engine, n):
    """K7 with AVDB_KEYS_DIGEST_DEFERRED (no digests yet: long keys laid out with
    their digest characters pending, state KEY_DIGEST_PENDING) then
    avdb_primary_keys_fill_digests == K7 given the digests: offsets, states,
    key and path text; and the pending states before the fill are exactly the
    long records with a labelled contig.  Keyed (K2 totals) and plain forms."""
    from annotatedvdb_amd import _native as N
    from annotatedvdb_amd import synth
    digs = ["%032d" % (17 * i) for i in range(25)]
    engine.set_sequence_digests(digs)
    b = synth.alleles(n, seed=41 + n % 9, long_frac=0.2, device="cuda")
    end, code, status, _ = engine.record_prep(b, want_lcp=False)
    dig, is_long = engine.vrs_digest(b, 50)
    ref = engine.primary_keys(b, code=code, digest=dig)
    for keyed in (False, True):
        kt = engine.new_key_text(n, b.heap.numel())
        for t in (kt.ws, kt.key_off, kt.path_off, kt.state, kt.keys, kt.paths):
            t.view(torch.uint8).fill_(0xA5)
        if keyed:
            engine.record_prep(b, want_lcp=False, keys=kt, key_digest=True)
        out = engine.primary_keys(b, code=code, out=kt, defer_digest=True)
        st = out.state[:n].cpu().numpy()
        chrom = b.chrom.cpu().numpy()
        assert np.array_equal(st == N.KEY_DIGEST_PENDING, is_long[:n].cpu().numpy().astype(bool) & (chrom < 25))
        if keyed:  # K4 writing the pending keys itself (avdb_vrs_digest_keys) instead of the fill pass
            dig2, _ = engine.vrs_digest(b, 50, keys=out)
            lm = is_long[:n].bool()
            assert torch.equal(dig2[:n][lm], dig[:n][lm])
        else:
            engine.fill_digests(b, dig, out)
        assert torch.equal(out.key_off[: n + 1], ref.key_off[: n + 1])
        assert torch.equal(out.path_off[: n + 1], ref.path_off[: n + 1])
        assert torch.equal(out.state[:n], ref.state[:n])
        kn, pn = int(ref.key_off[n]), int(ref.path_off[n])
        assert torch.equal(out.keys[:kn], ref.keys[:kn]) and torch.equal(out.paths[:pn], ref.paths[:pn])


@pytest.mark.parametrize("n", [1, 2, 4095, 4096, 4097, 8192, 8193, 300001])
def test_k7_narrow_offsets_equal_wide(engine, n):
    """K7 with AVDB_KEYS_OFF32 (u32 low words + a u64 base per 4,096 records):
    the widened offsets, states, key and path text equal the u64 form's, at sizes
    around every base boundary (the C4k shards cross 4 GB of path text: the
    wrap of the low words is covered there)."""
    from annotatedvdb_amd import synth
    digs = ["%032d" % (5 * i) for i in range(25)]
    eng2 = type(engine)(0, sequence_digests=digs)
    b = synth.alleles(n, seed=300 + n % 7, long_frac=0.05, device="cuda")
    end, code, status, _ = eng2.record_prep(b, want_lcp=False)
    dig, _ = eng2.vrs_digest(b, 50)
    ref = eng2.primary_keys(b, code=code, digest=dig)
    kt = eng2.new_key_text(n, b.heap.numel(), off32=True)
    for t in (kt.ws, kt.key_off, kt.path_off, kt.state, kt.keys, kt.paths):
        t.view(torch.uint8).fill_(0xA5)
    out = eng2.primary_keys(b, code=code, digest=dig, out=kt)
    assert out.off32 and out.key_off.dtype == torch.uint8
    assert torch.equal(out.key_offsets(n), ref.key_off[: n + 1])
    assert torch.equal(out.path_offsets(n), ref.path_off[: n + 1])
    assert torch.equal(out.state[:n], ref.state[:n])
    kn, pn = int(ref.key_off[n]), int(ref.path_off[n])
    assert torch.equal(out.keys[:kn], ref.keys[:kn]) and torch.equal(out.paths[:pn], ref.paths[:pn])
    assert out.host(n) == ref.host(n)
