"""north_star's target on BASELINE config C4: "bit-exact bin paths and primary
keys for 1B synthetic variants".  The keyed C4 job (``synth.dbsnp_alleles``,
the bench's own generator and seeds: 8 ranks' length-balanced pieces x 1.25e8
records = 1e9) runs shard by shard on one GPU through the step bench.py times —
``pipeline.KeyedStep`` in the bench's layout (``pipeline.C4K_LAYOUT``): K2 (end,
bin, and K7's group totals, K4's long-record codes, K3's first phase), K3
(keep-first dedup), K4 (VRS digests of the long records) and K7 (primary-key and
ltree-path text).  Nothing runs before it on the shard: every buffer the engine
and the step allocate — text buffers, offsets, states, workspaces, every output
— is filled with a sentinel byte first (``Engine.poison``), so what is compared
is only what the benched kernels wrote.  Every output of every record is
compared with the C oracle, which runs in chunks on a thread pool (ctypes
releases the GIL).

The long-record digests are checked against the oracle's restatement of the
VRS 1.x serialisation; that restatement itself is unpinned against vrs-python
(absent here)."""

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
POISON = 0xA5


def _p(a, k=0):
    return a.ctypes.data + k * a.itemsize


def _check_shard(engine, n, seed, pieces, layout=None, steps=1):
    import oracle
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.pipeline import C4K_LAYOUT, KeyedStep
    lib = oracle.c_oracle()
    b = synth.dbsnp_alleles(n, seed=seed, device="cuda", pieces=pieces)
    engine.poison = POISON
    try:
        ks = KeyedStep(engine, b, digests=True, layout=layout or C4K_LAYOUT)
        for k in range(steps):
            if k:  # the text buffers the previous step wrote: poisoned again
                for t in (ks.kt.keys, ks.kt.paths, ks.kt.key_off, ks.kt.path_off, ks.kt.state):
                    t.view(torch.uint8).fill_(POISON)
            out = ks.run()
    finally:
        engine.poison = None
    torch.cuda.synchronize()
    kt = out["kt"]
    assert not kt.state[:n].cpu().numpy().any()
    h = {k: getattr(b, k).cpu().numpy() for k in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "heap",
                                                  "ext_id")}
    chrom, pos = h["chrom"], h["pos"].view(np.uint32)
    off, rl, al = h["allele_off"].view(np.uint64), h["ref_len"].view(np.uint32), h["alt_len"].view(np.uint32)
    heap, ext = h["heap"], h["ext_id"].view(np.uint64)
    g_end, g_code = out["end"].cpu().numpy().view(np.uint32), out["code"].cpu().numpy().view(np.uint32)
    g_status, g_keep = out["status"].cpu().numpy(), out["keep"][:n].cpu().numpy()
    g_long = out["is_long"].cpu().numpy().astype(bool)
    g_dig = out["digest"].cpu().numpy()
    g_ko = kt.key_offsets(n).cpu().numpy().view(np.uint64)  # (the narrow layout widened: KeyText.off32)
    g_po = kt.path_offsets(n).cpu().numpy().view(np.uint64)
    g_keys = kt.keys[: int(g_ko[n])].cpu().numpy()
    g_paths = kt.paths[: int(g_po[n])].cpu().numpy()
    del out, kt, ks, b
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
    """Rank ``rank``'s whole shard of the keyed C4 job (1.25e8 records), the
    bench's step on sentinel-filled buffers: end, bin code, status, keep,
    long-record digests, primary-key text and ltree-path text (with their
    offsets) bit-exact vs the C oracle."""
    from annotatedvdb_amd import shard
    eng = type(engine)(0, sequence_digests=DIGS)
    plan = shard.plan(8)
    n_long, kbytes, pbytes = _check_shard(eng, N_PER_RANK, 4 + 1000 * rank, plan[rank])
    assert n_long > 0.015 * N_PER_RANK and kbytes > 20 * N_PER_RANK and pbytes > 50 * N_PER_RANK


@pytest.mark.parametrize("layout", ["onepass", "serial", "fork", "overlap"])
def test_c4k_small_vs_c_oracle(engine, layout):
    """Every stream layout of the step at a size the oracle finishes instantly
    (every code path, one chunk boundary), twice over the same buffers (the
    bench's steady state: the second step's K2 hands over into the workspaces the
    first step used; its text buffers are poisoned again in between)."""
    eng = type(engine)(0, sequence_digests=DIGS)
    _check_shard(eng, CHUNK + 12345, 77, None, layout=layout, steps=2)
