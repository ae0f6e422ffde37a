"""Synthetic GRCh38-shaped variant batches for the benchmark configs
(BASELINE.json ``configs``; generator shapes from SURVEY.md §8d).

Generation happens on the device with a seeded ``torch.Generator`` so a
100 M-record batch is ready in well under a second; it is never timed.  The
same shapes are produced on the CPU (numpy PCG64) for oracle-sized tests.

C2  point SNVs: chrom ∝ length, pos ~ U[1, len], sorted by (chrom, pos)
C3  spans: 0 w.p. 0.5, geometric(1/8) w.p. 0.3, log-uniform[50, 1e6] w.p. 0.2,
    end = min(pos + span, len)
C4  dbSNP-scale mix: 90 % SNV / 8 % indel <= 50 bp / 2 % log-uniform <= 1 Mb
C5  ADSP-style alleles: SNV / short indel / MNV / 5 % long (ref+alt in (50, 2000]),
    2 % exact duplicate records injected adjacent, 60 % with an rsid
"""

from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from .chromosomes import length_table
from .shard import Piece, pieces as all_pieces


def _piece_counts(ps: Sequence[Piece], n: int) -> np.ndarray:
    w = np.array([p.length for p in ps], dtype=np.float64)
    c = np.floor(n * w / w.sum()).astype(np.int64)
    c[np.argmax(w)] += n - c.sum()
    return c


def _positions(ps: Sequence[Piece], n: int, g: torch.Generator, device) -> tuple:
    """Sorted (chrom u8, pos i32) over the given pieces, density ∝ length."""
    counts = _piece_counts(ps, n)
    cnt_t = torch.from_numpy(counts).to(device)
    chrom = torch.repeat_interleave(torch.tensor([p.chrom for p in ps], dtype=torch.uint8, device=device),
                                    cnt_t)
    lo = torch.repeat_interleave(torch.tensor([p.lo for p in ps], dtype=torch.int64, device=device), cnt_t)
    ln = torch.repeat_interleave(torch.tensor([p.length for p in ps], dtype=torch.int64, device=device), cnt_t)
    u = torch.rand(n, generator=g, device=device, dtype=torch.float64)
    pos = lo + 1 + (u * ln).long().clamp_(max=ln - 1)
    # pieces are in (chrom, lo) order, so sorting positions inside each piece
    # sorts the batch: sort the global key once
    key = chrom.long() << 32 | pos
    key, _ = torch.sort(key)
    return (key >> 32).to(torch.uint8), (key & 0xFFFFFFFF).to(torch.int32)


def point_snvs(n: int, seed: int = 2, device="cuda", pieces: Optional[Sequence[Piece]] = None):
    """C2: returns (chrom u8, start i32) device tensors, sorted."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return _positions(pieces or all_pieces(), n, g, device)


def spans(n: int, seed: int = 3, device="cuda", pieces: Optional[Sequence[Piece]] = None,
          mix: str = "c3"):
    """C3 (or C4 with mix='c4'): (chrom u8, start i32, end i32), sorted by start."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    chrom, start = _positions(pieces or all_pieces(), n, g, device)
    lens = torch.tensor(length_table(), dtype=torch.int64, device=device)
    u = torch.rand(n, generator=g, device=device, dtype=torch.float64)
    geo = torch.floor(torch.log(torch.rand(n, generator=g, device=device, dtype=torch.float64).clamp_min(1e-300))
                      / np.log(1 - 1 / 8)).long()
    logu = torch.pow(10.0, torch.rand(n, generator=g, device=device, dtype=torch.float64)
                     * (6 - np.log10(50)) + np.log10(50)).long()
    if mix == "c3":
        span = torch.where(u < 0.5, torch.zeros_like(geo), torch.where(u < 0.8, geo, logu))
    else:  # c4: 90% SNV / 8% indel <= 50 / 2% log-uniform <= 1 Mb
        ind = (torch.rand(n, generator=g, device=device) * 50).long()
        span = torch.where(u < 0.9, torch.zeros_like(geo), torch.where(u < 0.98, ind, logu))
    end = torch.minimum(start.long() + span, lens[chrom.long()]).to(torch.int32)
    return chrom, start, end


def alleles(n: int, seed: int = 5, device="cuda", pieces: Optional[Sequence[Piece]] = None,
            long_frac: float = 0.05, dup_frac: float = 0.02, rs_frac: float = 0.6,
            classes=(0.80, 0.85, 0.90), indel_max: int = 20):
    """C5: a RecordBatch (device) of ADSP-style records, position-sorted, with
    exact duplicates injected adjacent (so the grouped dedup path applies).
    ``classes`` are the cumulative SNV / insertion / deletion thresholds (MNV up
    to ``1 - long_frac``, long above); indels add 1..``indel_max`` bases."""
    from .engine import RecordBatch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    chrom, pos = _positions(pieces or all_pieces(), n, g, device)
    u = torch.rand(n, generator=g, device=device)
    r1 = torch.randint(1, indel_max + 1, (n,), generator=g, device=device)
    r2 = torch.randint(1, 21, (n,), generator=g, device=device)
    L = torch.randint(51, 2001, (n,), generator=g, device=device)
    split = (torch.rand(n, generator=g, device=device) * (L - 1).float()).long() + 1
    one = torch.ones(n, dtype=torch.long, device=device)
    # classes: SNV 80 %, insertion 5 %, deletion 5 %, MNV 5 %, long 5 % (by long_frac)
    c_snv, c_ins, c_del = classes
    snv = u < c_snv
    ins = (u >= c_snv) & (u < c_ins)
    dele = (u >= c_ins) & (u < c_del)
    mnv = (u >= c_del) & (u < 1.0 - long_frac)
    lng = u >= 1.0 - long_frac
    rl = torch.where(snv, one, torch.where(ins, one, torch.where(dele, r1 + 1, torch.where(mnv, r2 + 1, split))))
    al = torch.where(snv, one, torch.where(ins, r1 + 1, torch.where(dele, one, torch.where(mnv, r2 + 1, L - split))))
    # duplicates: record i copies record i-1 (same chrom/pos/alleles/rsid)
    dup = torch.rand(n, generator=g, device=device) < dup_frac
    dup[0] = False
    src = torch.arange(n, device=device)
    src = torch.where(dup, src - 1, src)
    # chains of duplicates resolve to their first record
    src = torch.cummax(torch.where(dup, torch.zeros_like(src), src), 0).values
    rl = rl[src]
    al = al[src]
    chrom = chrom[src]
    pos = pos[src]
    tot = rl + al
    off = torch.cumsum(tot, 0) - tot
    H = int(tot.sum().item())
    acgt = torch.tensor([65, 67, 71, 84], dtype=torch.uint8, device=device)
    heap = acgt[torch.randint(0, 4, (H,), generator=g, device=device)]
    # indel anchors: alt[0] = ref[0]
    anchor = (ins | dele)[src] & ~dup
    a_idx = off[anchor]
    heap[a_idx + rl[anchor]] = heap[a_idx]
    # copy duplicate bytes from their source record
    if bool(dup.any()):
        d_rows = torch.nonzero(dup).squeeze(1)
        first = src[d_rows]
        dl = tot[d_rows]
        rep = torch.repeat_interleave(torch.arange(d_rows.numel(), device=device), dl)
        within = torch.arange(int(dl.sum().item()), device=device) - torch.repeat_interleave(
            torch.cumsum(dl, 0) - dl, dl)
        heap[off[d_rows][rep] + within] = heap[off[first][rep] + within]
    ext = torch.where(torch.rand(n, generator=g, device=device) < rs_frac,
                      torch.randint(1, 10 ** 9, (n,), generator=g, device=device), torch.zeros_like(pos, dtype=torch.long))
    ext = ext[src]
    return RecordBatch(chrom=chrom, pos=pos, allele_off=off, ref_len=rl.to(torch.int32),
                       alt_len=al.to(torch.int32), heap=heap, ext_id=ext)


def dbsnp_alleles(n: int, seed: int = 4, device="cuda", pieces: Optional[Sequence[Piece]] = None):
    """C4 with alleles (the keyed form of BASELINE configs[3]): SURVEY §8d's
    dbSNP mix as VCF records — 90 % SNV, 8 % anchored indels (4 % insertions,
    4 % deletions of 1-48 bases, so ref+alt <= 50 and the key stays short), 2 %
    long alleles (ref+alt in (50, 2000], keyed by the VRS digest); every record
    carries an rsid; 0.5 % exact duplicates injected adjacent.  The 2 % of
    SURVEY's spans up to 1 Mb are binned by K1 in C3/C4; as literal alleles
    they are capped at 2 kb here to bound the heap."""
    return alleles(n, seed=seed, device=device, pieces=pieces, long_frac=0.02, dup_frac=0.005,
                   rs_frac=1.0, classes=(0.90, 0.94, 0.98), indel_max=48)


C1_N = 1_100_000
C1_LO, C1_HI = 16_050_000, 50_800_000  # chr22 region a 1000 Genomes VCF covers


def np_c1(n: int = C1_N, seed: int = 1, rs_frac: float = 0.6):
    """C1 (BASELINE configs[0]): ``n`` chr22 records with
    positions uniform in [16,050,000, 50,800,000], position-sorted; 88 % SNVs,
    6 % insertions of 1-20 bp and 6 % deletions of 1-30 bp (both VCF-anchored:
    alt[0] == ref[0]); ``rs_frac`` of the records carry an rsid.  numpy PCG64,
    host-side, so tests and bench use byte-identical records.

    Returns a dict of numpy arrays in the ``RecordBatch`` layout (``chrom`` u8,
    ``pos`` i32, ``allele_off`` i64, ``ref_len``/``alt_len`` i32, ``heap`` u8,
    ``ext_id`` i64: rsid number or 0)."""
    from .chromosomes import CHROM_NAMES
    rng = np.random.Generator(np.random.PCG64(seed))
    pos = np.sort(rng.integers(C1_LO, C1_HI + 1, n)).astype(np.int32)
    u = rng.random(n)
    ins = (u >= 0.88) & (u < 0.94)
    dele = u >= 0.94
    k_ins = rng.integers(1, 21, n)
    k_del = rng.integers(1, 31, n)
    rl = np.where(dele, 1 + k_del, 1).astype(np.int64)
    al = np.where(ins, 1 + k_ins, 1).astype(np.int64)
    tot = rl + al
    off = np.zeros(n, dtype=np.int64)
    if n:
        np.cumsum(tot[:-1], out=off[1:])
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    code = rng.integers(0, 4, int(tot.sum()))
    ref0 = code[off]
    # SNV alt: one of the three other bases; indel alt/ref anchor = ref[0]
    snv = ~(ins | dele)
    code[(off + 1)[snv]] = (ref0[snv] + rng.integers(1, 4, int(snv.sum()))) % 4
    code[(off + rl)[~snv]] = ref0[~snv]
    heap = acgt[code]
    ext = np.where(rng.random(n) < rs_frac, rng.integers(1, 2 * 10 ** 9, n), 0).astype(np.int64)
    return dict(chrom=np.full(n, CHROM_NAMES.index("22"), dtype=np.uint8), pos=pos, allele_off=off,
                ref_len=rl.astype(np.int32), alt_len=al.astype(np.int32),
                heap=heap if heap.size else np.zeros(1, dtype=np.uint8), ext_id=ext)


def c1_batch(n: int = C1_N, seed: int = 1, device="cpu"):
    """C1 as a ``RecordBatch`` (numpy-generated, then moved to ``device``)."""
    from .engine import RecordBatch
    d = np_c1(n, seed)
    return RecordBatch(**{k: torch.from_numpy(v).to(device) for k, v in d.items()})


# ---- numpy (CPU) versions, oracle-sized ------------------------------------
def np_point_snvs(n: int, seed: int = 2, lengths=None):
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = np.asarray(lengths if lengths is not None else length_table(), dtype=np.int64)
    chrom = rng.choice(len(lengths), size=n, p=lengths / lengths.sum()).astype(np.uint8)
    pos = (rng.random(n) * lengths[chrom]).astype(np.int64) + 1
    order = np.lexsort((pos, chrom))
    return chrom[order], pos[order].astype(np.int32)


def np_spans(n: int, seed: int = 3, lengths=None, mix: str = "c3"):
    """C3 spans (or the C4 mix: 90 % SNV / 8 % indel <= 50 bp / 2 % log-uniform
    <= 1 Mb) on the host, numpy PCG64 (the CPU baselines' sample)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = np.asarray(lengths if lengths is not None else length_table(), dtype=np.int64)
    chrom, start = np_point_snvs(n, seed, lengths)
    u = rng.random(n)
    geo = rng.geometric(1 / 8, n) - 1
    logu = (10 ** rng.uniform(np.log10(50), 6, n)).astype(np.int64)
    if mix == "c4":
        span = np.where(u < 0.9, 0, np.where(u < 0.98, rng.integers(1, 51, n), logu))
    else:
        span = np.where(u < 0.5, 0, np.where(u < 0.8, geo, logu))
    end = np.minimum(start.astype(np.int64) + span, lengths[chrom]).astype(np.int32)
    return chrom, start, end


def vcf_text(n_lines: int, seed: int = 6, lengths=None, multi_frac: float = 0.1,
             rs_frac: float = 0.6, info: bool = True) -> bytes:
    """dbSNP-shaped VCF data lines (no header): sorted (chrom, pos); 80 % SNV,
    10 % short indels, 10 % MNV; ``multi_frac`` of lines carry two ALTs; the ID
    column holds an rsid for ``rs_frac`` of lines, otherwise '.', with RS= in
    INFO; INFO mimics dbSNP (RS, dbSNPBuildID, SSR, VC, FREQ).  Host-side
    (numpy PCG64 + one formatting pass), never timed."""
    from .chromosomes import CHROM_NAMES
    rng = np.random.Generator(np.random.PCG64(seed))
    chrom, pos = np_point_snvs(n_lines, seed, lengths)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    u = rng.random(n_lines)
    klen = np.where(u < 0.8, 1, rng.integers(2, 12, n_lines))
    rbytes = acgt[rng.integers(0, 4, (n_lines, 12))]
    abytes = acgt[rng.integers(0, 4, (n_lines, 2, 12))]
    multi = rng.random(n_lines) < multi_frac
    has_rs = rng.random(n_lines) < rs_frac
    rsn = rng.integers(1, 2 * 10 ** 9, n_lines)
    fq = rng.integers(1, 9999, n_lines)
    out = []
    for i in range(n_lines):
        k = int(klen[i])
        if u[i] < 0.8:
            ref, alts = rbytes[i, :1].tobytes(), [abytes[i, 0, :1].tobytes()]
            if alts[0] == ref:
                alts[0] = b"T" if ref != b"T" else b"A"
        elif u[i] < 0.85:      # insertion, anchored
            ref = rbytes[i, :1].tobytes()
            alts = [ref + abytes[i, 0, :k].tobytes()]
        elif u[i] < 0.9:       # deletion, anchored
            ref = rbytes[i, :k].tobytes()
            alts = [ref[:1]]
        else:                  # MNV
            ref = rbytes[i, :k].tobytes()
            alts = [abytes[i, 0, :k].tobytes()]
        if multi[i]:
            alts.append(abytes[i, 1, :max(1, k - 1)].tobytes())
        alt = b",".join(alts).decode()
        rid = "rs%d" % rsn[i] if has_rs[i] else "."
        vc = "SNV" if u[i] < 0.8 else ("INDEL" if u[i] < 0.9 else "MNV")
        # FREQ: one value for REF and one per ALT (vcf_parser.py:213-220 indexes by ALT)
        fr = "1000Genomes:0.%04d,0.%04d" % (10000 - fq[i], fq[i]) + (",." if multi[i] else "")
        if fq[i] % 3 == 0:
            fr += "|GnomAD:0.%04d,0.%04d" % (10000 - fq[i] // 2, fq[i] // 2) + (",0.0001" if multi[i] else "")
        inf = ("RS=%d;dbSNPBuildID=151;SSR=0;VC=%s;FREQ=%s" % (rsn[i], vc, fr)) if info else "."
        out.append("%s\t%d\t%s\t%s\t%s\t.\t.\t%s" % (CHROM_NAMES[chrom[i]], pos[i], rid,
                                                    ref.decode(), alt, inf))
    return ("\n".join(out) + "\n").encode()
