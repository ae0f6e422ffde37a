"""The one-pass keyed prep (``avdb_keyed_prep``; ``pipeline.KeyedStep`` layout
"onepass"): K2 and K7 in one launch over the SoA, the text offsets from a
decoupled look-back over 256-record groups.  Its outputs must be the two-kernel
step's, bit for bit — the serial layout that tests/test_gpu_c4k.py and
test_gpu_c1.py pin to the C oracle — at every size where groups, tiles and
waves break differently, on sorted, unsorted and adversarial batches, with the
L8 histogram and counters; every buffer the one-pass step reads back is a
sentinel before it runs."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

DIGS = ["%032d" % (7 * i) for i in range(25)]
POISON = 0xA5


def _run(engine, b, layout, digests, steps=1):
    from annotatedvdb_amd.pipeline import KeyedStep
    hist, ctr = engine.new_histogram(), engine.new_counters()
    engine.poison = POISON if layout == "onepass" else None
    try:
        ks = KeyedStep(engine, b, digests=digests, layout=layout, hist=hist, counters=ctr)
        for k in range(steps):
            if k:
                hist.zero_()
                ctr.zero_()
                for t in (ks.kt.keys, ks.kt.paths, ks.kt.key_off, ks.kt.path_off, ks.kt.state):
                    t.view(torch.uint8).fill_(POISON)
            out = ks.run()
    finally:
        engine.poison = None
    torch.cuda.synchronize()
    if layout == "onepass":
        assert engine.keyed_prep_lookback_errors(ks.ws_op) == 0
    return ks, out, hist, ctr


def _same(engine, b, digests=True, steps=1):
    n = b.n
    ks0, o0, h0, c0 = _run(engine, b, "serial", digests)
    ks1, o1, h1, c1 = _run(engine, b, "onepass", digests, steps=steps)
    for k in ("end", "code", "status"):
        assert torch.equal(o0[k][:n], o1[k][:n]), k
    assert torch.equal(o0["keep"][:n], o1["keep"][:n])
    if digests:
        assert torch.equal(o0["is_long"][:n], o1["is_long"][:n])
        lm = o0["is_long"][:n].bool()
        assert torch.equal(o0["digest"][:n][lm], o1["digest"][:n][lm])
    k0, k1 = ks0.kt, ks1.kt
    assert torch.equal(k0.key_offsets(n), k1.key_offsets(n))
    assert torch.equal(k0.path_offsets(n), k1.path_offsets(n))
    assert torch.equal(k0.state[:n], k1.state[:n])
    kn, pn = int(k0.key_offsets(n)[n]), int(k0.path_offsets(n)[n])
    assert torch.equal(k0.keys[:kn], k1.keys[:kn])
    assert torch.equal(k0.paths[:pn], k1.paths[:pn])
    assert torch.equal(h0, h1)
    assert torch.equal(c0, c1)
    return o1, ks1


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 255, 256, 257, 511, 1000, 4095, 65537, 1_000_003])
def test_onepass_equals_serial_sizes(engine, n):
    """ADSP-style batches (long alleles, adjacent duplicates, rsids) at sizes
    around every wave / group edge."""
    from annotatedvdb_amd import synth
    engine.set_sequence_digests(DIGS)
    b = synth.alleles(n, seed=90 + n % 11, long_frac=0.05, device="cuda")
    _same(engine, b)


def test_onepass_dbsnp_two_steps(engine):
    """The C4k mix (the bench's generator) over 4 Mi + records, two steps over the
    same buffers, the text poisoned in between (the bench's steady state)."""
    from annotatedvdb_amd import synth
    engine.set_sequence_digests(DIGS)
    b = synth.dbsnp_alleles((4 << 20) + 12345, seed=9, device="cuda")
    _same(engine, b, steps=2)


def test_onepass_unsorted(engine):
    """Records in random order: waves of mixed L8 keys (the histogram's direct
    adds), duplicates no longer adjacent (nothing listed that the run scan would
    not list)."""
    from annotatedvdb_amd import synth
    from annotatedvdb_amd.engine import RecordBatch
    engine.set_sequence_digests(DIGS)
    b = synth.alleles(200_003, seed=17, long_frac=0.05, device="cuda")
    perm = torch.randperm(b.n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    u = RecordBatch(chrom=b.chrom[perm].contiguous(), pos=b.pos[perm].contiguous(),
                    allele_off=b.allele_off[perm].contiguous(), ref_len=b.ref_len[perm].contiguous(),
                    alt_len=b.alt_len[perm].contiguous(), heap=b.heap, ext_id=b.ext_id[perm].contiguous())
    _same(engine, u)


def test_onepass_adversarial(engine):
    """Unknown contigs, positions 0 and past the contig end, end < start
    (identical alleles), ':' and non-ASCII bytes in alleles (HOST keys), interned
    external ids, unlabelled contigs of a longer table; without digests long
    records are NEED_DIGEST and carry no key bytes."""
    from annotatedvdb_amd.engine import pack_records
    from annotatedvdb_amd.chromosomes import length_table
    rng = np.random.default_rng(5)
    L = length_table()
    chrom, pos, refs, alts, ext = [], [], [], [], []
    for i in range(3000):
        c = int(rng.integers(0, 25))
        p = int(rng.integers(1, L[c]))
        kind = i % 12
        r, a = b"A", b"G"
        if kind == 1:
            c = 30  # unknown contig
        elif kind == 2:
            p = 0
        elif kind == 3:
            p = L[c] + 5
        elif kind == 4:
            r, a = b"AT", b"AT"  # end = pos - 1
        elif kind == 5:
            r, a = b"A:C", b"G"
        elif kind == 6:
            r, a = b"A", "é".encode()
        elif kind == 7:
            r, a = b"A" * 30, b"C" * 40  # long
        elif kind == 8:
            r, a = b"ACGTACGT" * 3, b"A"
        chrom.append(c)
        pos.append(p)
        refs.append(r)
        alts.append(a)
        ext.append((1 << 63) | i if kind == 9 else (int(rng.integers(1, 1 << 40)) if kind % 2 else 0))
    # sort by (chrom, pos) so the grouped dedup applies; duplicate every 50th record next to itself
    order = sorted(range(len(pos)), key=lambda k: (chrom[k], pos[k]))
    cols = [[x[k] for k in order] for x in (chrom, pos, refs, alts, ext)]
    for k in range(len(order) - 1, 0, -50):
        for col in cols:
            col.insert(k, col[k])
    b = pack_records(*cols).to(engine.device)
    for digests in (False, True):
        engine.set_sequence_digests(DIGS)
        _same(engine, b, digests=digests)
