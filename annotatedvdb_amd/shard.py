"""Length-balanced sharding of the genome across GPUs.

The reference parallelises one OS process per chromosome file
(``Load/bin/load_vcf_file.py:307-313``).  A bin is a pure function of
(chrom, start, end, chrom_len) and every duplicate primary key shares
(chrom, pos), so any partition by contiguous (chrom, position) ranges needs no
data exchange for correctness.  Whole-chromosome LPT balances 8 GPUs to 1.036
max/mean on GRCh38; cutting chromosomes at 64 Mb (L1 bin) boundaries gives 61
pieces and 1.012.  A record belongs to the piece holding its ``start``; the bin
arithmetic still uses full-chromosome coordinates, so spanning variants get L0
exactly as in the reference.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

from .chromosomes import CHROM_NAMES, length_table

PIECE = 64_000_000  # L1 bin width (generate_bin_index_references.py:93)


@dataclass(frozen=True)
class Piece:
    chrom: int        # u8 code
    lo: int           # positions lo+1 .. hi (a (lo,hi] range, like BinIndexRef)
    hi: int

    @property
    def length(self) -> int:
        return self.hi - self.lo


def pieces(lengths: Sequence[int] | None = None, cut: int = PIECE) -> List[Piece]:
    lengths = list(lengths) if lengths is not None else length_table()
    out = []
    for c, L in enumerate(lengths):
        lo = 0
        while lo < L:
            hi = min(lo + cut, L)
            out.append(Piece(c, lo, hi))
            lo = hi
    return out


def plan(world_size: int, lengths: Sequence[int] | None = None, cut: int = PIECE) -> List[List[Piece]]:
    """LPT (longest processing time first) assignment of pieces to ranks.
    Deterministic: ties broken by piece order, then rank index."""
    ps = pieces(lengths, cut)
    order = sorted(range(len(ps)), key=lambda i: (-ps[i].length, i))
    load = [0] * world_size
    out: List[List[Piece]] = [[] for _ in range(world_size)]
    for i in order:
        r = min(range(world_size), key=lambda k: (load[k], k))
        out[r].append(ps[i])
        load[r] += ps[i].length
    for r in range(world_size):
        out[r].sort(key=lambda p: (p.chrom, p.lo))
    return out


def imbalance(assignment: List[List[Piece]]) -> float:
    loads = [sum(p.length for p in a) for a in assignment]
    mean = sum(loads) / len(loads)
    return max(loads) / mean if mean else 1.0


def piece_table(assignment: List[List[Piece]], lengths: Sequence[int] | None = None, cut: int = PIECE):
    """The plan as the flat tables K9 (``avdb_vcf_select_lines``) stages in LDS:
    ``(piece_base[n_chrom], piece_count[n_chrom], piece_rank[n_pieces])`` over
    ``pieces(lengths, cut)`` order (numpy arrays)."""
    import numpy as np
    ps = pieces(lengths, cut)
    owner = {}
    for r, a in enumerate(assignment):
        for p in a:
            owner[(p.chrom, p.lo)] = r
    n_chrom = len(list(lengths) if lengths is not None else length_table())
    base = np.zeros(n_chrom, dtype=np.uint32)
    count = np.zeros(n_chrom, dtype=np.uint32)
    rank = np.zeros(len(ps), dtype=np.uint8)
    for i, p in enumerate(ps):
        if count[p.chrom] == 0:
            base[p.chrom] = i
        count[p.chrom] += 1
        rank[i] = owner[(p.chrom, p.lo)]
    return base, count, rank


def owner_of_lines(assignment: List[List[Piece]], chrom, pos, flags, n_chrom: int = 25,
                   lengths: Sequence[int] | None = None, cut: int = PIECE):
    """Host restatement of K9's line placement (the test checker): -1 for
    comment lines, 0 for lines K0 could not place, else the piece owner."""
    import numpy as np
    base, count, rank = piece_table(assignment, lengths, cut)
    chrom = np.asarray(chrom, dtype=np.int64)
    pos = np.asarray(pos, dtype=np.int64)
    flags = np.asarray(flags, dtype=np.int64)
    out = np.zeros(len(chrom), dtype=np.int64)
    ok = (chrom < n_chrom) & ((flags & (0x004 | 0x080 | 0x100 | 0x002)) == 0)
    c = np.where(ok, chrom, 0)
    k = np.where(pos > 0, (pos - 1) // cut, 0)
    k = np.minimum(k, count[c].astype(np.int64) - 1)
    out[ok] = rank[(base[c].astype(np.int64) + k)[ok]]
    out[(flags & 0x001) != 0] = -1
    return out


def shard_of(assignment: List[List[Piece]], chrom: int, start: int) -> int:
    for r, ps in enumerate(assignment):
        for p in ps:
            if p.chrom == chrom and p.lo < start <= p.hi:
                return r
    return -1


def describe(assignment: List[List[Piece]]) -> List[Tuple[int, List[str]]]:
    return [(sum(p.length for p in a), ["chr%s:%d-%d" % (CHROM_NAMES[p.chrom], p.lo + 1, p.hi) for p in a])
            for a in assignment]
