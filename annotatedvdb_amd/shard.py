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


def shard_of(assignment: List[List[Piece]], chrom: int, start: int) -> int:
    for r, ps in enumerate(assignment):
        for p in ps:
            if p.chrom == chrom and p.lo < start <= p.hi:
                return r
    return -1


def describe(assignment: List[List[Piece]]) -> List[Tuple[int, List[str]]]:
    return [(sum(p.length for p in a), ["chr%s:%d-%d" % (CHROM_NAMES[p.chrom], p.lo + 1, p.hi) for p in a])
            for a in assignment]
