"""Drop-in ``BinIndex`` — same constructor, ``find_bin_index`` and ``close`` as
``AnnotatedVDB.BinIndex.bin_index.BinIndex`` (BinIndex/lib/python/bin_index.py:16-75),
plus a batch entry point.

The reference answers a cache miss with a synchronous Postgres round trip to the
external SQL ``find_bin_index(chr,start,end)`` over ``BinIndexRef``
(:9-14, :43-56).  Here the lookup is the K1 kernel (``avdb_bin_assign``) on the
GPU; there is no database and no CPU fallback.  The per-record API keeps the
reference's observable behaviour, including its one-bin cache (served only for
L13 bins, :66-71) and ``TypeError`` for unmappable locations (``None[...]`` at
:75).  ``find_bin_indices`` is the batched form the loaders use.
"""

from __future__ import annotations

import sys
from ctypes import string_at as ctypes_string_at
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .chromosomes import CHROM_NAMES, N_CHROM, UNKNOWN_CHROM, bin_index_chrom_code, length_table

INC = [0] + [64000000 >> (lvl - 1) for lvl in range(1, 14)]
_CODES = {}  # chromosome argument -> contig code (bin_index_chrom_code), memoised
_LABELS = ["chr" + c for c in CHROM_NAMES]


def bin_location(code: int, chrom_len: int) -> Tuple[int, int]:
    """``(lo, hi)`` of the BinIndexRef row ``(lo,hi]`` a bin code names
    (generate_bin_index_references.py:55-65: aligned, clipped at the length)."""
    level, g = code >> 28, code & 0x0FFFFFFF
    if level == 0:
        return 0, chrom_len
    lo = g * INC[level]
    return lo, min(lo + INC[level], chrom_len)


class _K1h:
    """``avdb_bin_path_host`` with its ctypes arguments allocated once."""

    def __init__(self, engine):
        import ctypes
        from . import _native as N
        self.eng, self.N = engine, N
        self.code, self.status = ctypes.c_uint32(), ctypes.c_uint8()
        self._buf = ctypes.create_string_buffer(N.MAX_PATH)
        self._args = (ctypes.byref(self.code), ctypes.byref(self.status), self._buf, N.MAX_PATH)
        self._addr = ctypes.addressof(self._buf)
        self._fn = engine.lib.avdb_bin_path_host

    def path(self, chrom: int, start: int, end: int) -> Optional[str]:
        k = self._fn(self.eng.ctx, chrom, start, end, *self._args)
        if k <= 0:
            self.N.check("avdb_bin_path_host", k)
            return None
        return ctypes_string_at(self._addr, k).decode("ascii")


class BinIndex(object):
    """GPU-backed drop-in for the reference ``BinIndex``."""

    def __init__(self, gusConfigFile=None, verbose=True, assembly: str = "GRCh38",
                 chromosome_lengths: Optional[Sequence[int]] = None, device=None):
        # gusConfigFile is accepted for signature compatibility: no DB is used
        self._gusConfigFile = gusConfigFile
        self._verbose = verbose
        self._currentBin = {}
        from .engine import Engine, default_engine
        if chromosome_lengths is None and assembly == "GRCh38" and device is None:
            self._engine = default_engine()
        else:
            self._engine = Engine(device, lengths=chromosome_lengths, assembly=assembly)
        self._lengths = self._engine.lengths
        self._k1h = None

    # ---- reference API ----------------------------------------------------
    def close(self):
        """Nothing to close (the reference closes its DB cursor, :38-41)."""
        self._currentBin = {}

    def _lookup_one(self, chrm: str, start: int, end: int) -> Optional[dict]:
        """The reference's SQL round trip for one record: K1h
        (``avdb_bin_path_host``, K1's closed form in the library's host code) —
        a miss costs one library call, not a GPU launch + stream sync."""
        code = _CODES.get(chrm)
        if code is None:
            code = _CODES[chrm] = min(bin_index_chrom_code(chrm), 255)
        lo, hi = (start, end) if end >= start else (end, start)
        if lo < 1 or hi >= 4294967296:  # outside any bin (and outside the kernels' u32 positions)
            return None
        k1h = self._k1h
        if k1h is None:
            k1h = self._k1h = _K1h(self._engine)
        path = k1h.path(code, int(start), int(end))
        if path is None:
            return None
        bcode = k1h.code.value
        level = bcode >> 28
        if level:
            lo = (bcode & 0x0FFFFFFF) * INC[level]
            hi = min(lo + INC[level], self._lengths[code])
        else:
            lo, hi = 0, self._lengths[code]
        return {"chromosome": _LABELS[code], "global_bin_path": path, "location": (lo, hi),
                "bin_level": 1 + 2 * level}

    def _update_current_bin_index(self, chrm, start, end):
        if self._verbose:
            print("Updating current bin", file=sys.stderr)
        self._currentBin = self._lookup_one(chrm, start, end)
        if self._verbose:
            print(self._currentBin, file=sys.stderr)
        return None

    def find_bin_index(self, chrm, start, end=None):
        """Smallest enclosing bin path of ``[start, end]`` (bin_index.py:59-75)."""
        if end is None:
            end = start
        if "chr" not in chrm:  # TypeError for a non-string, as in the reference
            chrm = "chr" + str(chrm)
        cur = self._currentBin
        if cur:  # one-bin cache, L13 bins only (nlevel >= 27)
            if cur["bin_level"] >= 27:
                lo, hi = cur["location"]
                if cur["chromosome"] == chrm and lo < start <= hi and lo < end <= hi:
                    return cur["global_bin_path"]
        self._update_current_bin_index(chrm, start, end)
        return self._currentBin["global_bin_path"]

    # ---- batch API --------------------------------------------------------
    def find_bin_codes(self, chroms: Sequence, starts, ends=None):
        """Batch lookup on the GPU.  Returns ``(chrom_codes u8, bin_codes u32,
        status u8)`` numpy arrays; chromosome labels resolve exactly as
        ``find_bin_index`` does (``'chr'`` prepended when absent)."""
        import torch
        cc = np.fromiter((min(bin_index_chrom_code(c), 255) for c in chroms), dtype=np.uint8,
                         count=len(chroms))
        s = np.asarray(starts, dtype=np.int64).astype(np.int32)
        e = None if ends is None else np.asarray(
            [st if en is None else en for st, en in zip(starts, ends)], dtype=np.int64).astype(np.int32)
        code, status = self._engine.bin_assign(torch.from_numpy(cc), torch.from_numpy(s),
                                               None if e is None else torch.from_numpy(e))
        return cc, code.cpu().numpy().view(np.uint32), status.cpu().numpy()

    def find_bin_indices(self, chroms: Sequence, starts, ends=None, errors: str = "none") -> List[Optional[str]]:
        """Batch ``find_bin_index``: list of paths (``None`` where unmappable, or
        ``errors='raise'`` to raise ``TypeError`` like the per-record API)."""
        cc, codes, status = self.find_bin_codes(chroms, starts, ends)
        paths = self._engine.format_paths(cc, codes)
        if errors == "raise":
            for i, p in enumerate(paths):
                if p is None:
                    raise TypeError("'NoneType' object is not subscriptable (unmappable: %s:%s-%s)"
                                    % (chroms[i], starts[i], starts[i] if ends is None else ends[i]))
        return paths
