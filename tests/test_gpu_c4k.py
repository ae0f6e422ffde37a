"""north_star's target on BASELINE config C4: "bit-exact bin paths and primary
keys for 1B synthetic variants".  The keyed C4 job (``synth.dbsnp_alleles``,
the bench's own generator and seeds: 8 ranks' length-balanced pieces x 1.25e8
records = 1e9) runs shard by shard on one GPU through K2 (end, bin), K3
(keep-first dedup), K4 (VRS digests of the long records) and K7 (primary-key and
ltree-path text), in the keyed form bench.py times (K2 also writing K7's group
totals, K4's long-record codes and K3's first phase); every output of every
record is compared with the C oracle.
The oracle runs in chunks on a thread pool (ctypes releases the GIL).

The long-record digests are checked against the oracle's restatement of the
VRS 1.x serialisation; that restatement itself is unpinned against vrs-python
(absent here)."""

import ctypes
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from annotatedvdb_amd.chromosomes import length_table

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

torch = pytest.importorskip("torch")

LENGTHS = np.asarray(length_table(), dtype=np.uint32)
N_PER_RANK = 125_000_000
CHUNK = 4_000_000
DIGS = ["%032d" % i for i in range(25)]  # the bench's synthetic refget ids


def _p(a, k=0):
    return a.ctypes.data + k * a.itemsize


def _check_shard(engine, n, seed, pieces):
    import oracle
    from annotatedvdb_amd import synth
    lib = oracle.c_oracle()
    b = synth.dbsnp_alleles(n, seed=seed, device="cuda", pieces=pieces)
    sz = ctypes.c_size_t()
    engine.lib.avdb_vrs_digest_workspace_size(n, ctypes.byref(sz))
    ws4 = torch.empty(int(sz.value), dtype=torch.uint8, device="cuda")
    ws3 = torch.empty(16384 + 4 * (((n + 3) & ~3) + (1 << 22)), dtype=torch.uint8, device="cuda")
    end, code, status, _ = engine.record_prep(b, want_lcp=False)
    keep = engine.pk_dedup(b, grouped=True)
    dig, is_long = engine.vrs_digest(b, 50, workspace=ws4)
    kt = engine.primary_keys(b, code=code, digest=dig)
    del end, code, status, keep, dig, is_long
    # then the bench's keyed step on the same batch, reusing the key text buffers:
    # K2 writes K7's group totals, K4's long-record codes and K3's first phase, and
    # K7, K4 and K3 skip their own passes over the SoA (what bench.py --workload c4k times)
    end, code, status, _ = engine.record_prep(b, want_lcp=False, keys=kt, key_digest=True, digest_workspace=ws4,
                                              dedup_workspace=ws3)
    assert set(engine._pending) == {"totals", "codes", "marks"}
    keep = engine.pk_dedup(b, grouped=True, workspace=ws3)
    dig, is_long = engine.vrs_digest(b, 50, workspace=ws4)
    kt = engine.primary_keys(b, code=code, digest=dig, out=kt)
    torch.cuda.synchronize()
    del ws4, ws3
    assert not kt.state[:n].cpu().numpy().any()
    h = {k: getattr(b, k).cpu().numpy() for k in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "heap",
                                                  "ext_id")}
    chrom, pos = h["chrom"], h["pos"].view(np.uint32)
    off, rl, al = h["allele_off"].view(np.uint64), h["ref_len"].view(np.uint32), h["alt_len"].view(np.uint32)
    heap, ext = h["heap"], h["ext_id"].view(np.uint64)
    g_end, g_code = end.cpu().numpy().view(np.uint32), code.cpu().numpy().view(np.uint32)
    g_status, g_keep = status.cpu().numpy(), keep.cpu().numpy()
    g_long = is_long.cpu().numpy().astype(bool)
    g_dig = dig.cpu().numpy()
    del end, code, status, keep, dig, is_long
    g_ko = kt.key_off[: n + 1].cpu().numpy().view(np.uint64)
    g_po = kt.path_off[: n + 1].cpu().numpy().view(np.uint64)
    g_keys = kt.keys[: int(g_ko[n])].cpu().numpy()
    g_paths = kt.paths[: int(g_po[n])].cpu().numpy()
    del kt, b
    torch.cuda.empty_cache()
    seqd = "".join(DIGS).encode()
    long_ = (rl.astype(np.int64) + al) > 50
    assert np.array_equal(g_long, long_)

    def chunk(a):
        z = min(n, a + CHUNK)
        m = z - a
        o_end, o_code = np.empty(m, np.uint32), np.empty(m, np.uint32)
        o_st = np.empty(m, np.uint8)
        lib.avdb_oracle_record_prep(_p(chrom, a), _p(pos, a), _p(off, a), _p(rl, a), _p(al, a), _p(heap), m,
                                    _p(LENGTHS), len(LENGTHS), _p(o_end), _p(o_code), _p(o_st), None)
        if not (np.array_equal(o_end, g_end[a:z]) and np.array_equal(o_code, g_code[a:z])
                and np.array_equal(o_st, g_status[a:z])):
            return "record_prep", a
        o_dig = np.zeros((m, 32), np.uint8)
        buf = np.empty(8192, np.uint8)
        lib.avdb_oracle_vrs_digest(_p(chrom, a), _p(pos, a), _p(off, a), _p(rl, a), _p(al, a), _p(heap), m, 50,
                                   seqd, 25, _p(buf), _p(o_dig))
        lm = long_[a:z]
        if not np.array_equal(o_dig[lm], g_dig[a:z][lm]):
            return "digest", a
        cap = int(rl[a:z].astype(np.int64).sum() + al[a:z].sum()) + 64 * m + 8
        o_keys = np.empty(cap, np.uint8)
        o_ko = np.empty(m + 1, np.uint64)
        kb = lib.avdb_oracle_primary_keys(_p(chrom, a), _p(pos, a), _p(off, a), _p(rl, a), _p(al, a), _p(heap),
                                          _p(ext, a), _p(o_dig), m, 50, _p(o_keys), _p(o_ko))
        if not (np.array_equal(o_ko + g_ko[a], g_ko[a:z + 1])
                and np.array_equal(o_keys[:kb], g_keys[int(g_ko[a]):int(g_ko[z])])):
            return "keys", a
        o_paths = np.empty(96 * m + 8, np.uint8)
        o_po = np.empty(m + 1, np.uint64)
        pb = lib.avdb_oracle_bin_paths(_p(chrom, a), _p(o_code), m, _p(o_paths), _p(o_po))
        if not (np.array_equal(o_po + g_po[a], g_po[a:z + 1])
                and np.array_equal(o_paths[:pb], g_paths[int(g_po[a]):int(g_po[z])])):
            return "paths", a
        return None

    def dedup():
        o_keep = np.empty(n, np.uint8)
        lib.avdb_oracle_dedup_grouped(_p(chrom), _p(pos), _p(off), _p(rl), _p(al), _p(heap), _p(ext), n,
                                      _p(o_keep))
        return None if np.array_equal(o_keep, g_keep) else ("dedup", 0)

    with ThreadPoolExecutor(16) as ex:
        futs = [ex.submit(dedup)] + [ex.submit(chunk, a) for a in range(0, n, CHUNK)]
        bad = [f.result() for f in futs]
    bad = [x for x in bad if x is not None]
    assert not bad, bad[:4]
    return int(long_.sum()), int(g_ko[n]), int(g_po[n])


@pytest.mark.parametrize("rank", range(8))
def test_c4k_shard_vs_c_oracle(engine, rank):
    """Rank ``rank``'s whole shard of the keyed C4 job (1.25e8 records): end,
    bin code, status, keep, long-record digests, primary-key text and ltree-path
    text (with their offsets) bit-exact vs the C oracle."""
    from annotatedvdb_amd import shard
    eng = type(engine)(0, sequence_digests=DIGS)
    plan = shard.plan(8)
    n_long, kbytes, pbytes = _check_shard(eng, N_PER_RANK, 4 + 1000 * rank, plan[rank])
    assert n_long > 0.015 * N_PER_RANK and kbytes > 20 * N_PER_RANK and pbytes > 50 * N_PER_RANK


def test_c4k_small_vs_c_oracle(engine):
    """The same check at a size the oracle finishes instantly (every code path,
    one chunk boundary)."""
    eng = type(engine)(0, sequence_digests=DIGS)
    _check_shard(eng, CHUNK + 12345, 77, None)
