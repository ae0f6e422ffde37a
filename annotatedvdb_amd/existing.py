"""Variants already in ``AnnotatedVDB.Variant`` — the ``--skipExisting`` check
(SURVEY.md §8f rank 4).

The reference asks the database once per alt allele:
``VCFVariantLoader.__parse_alt_alleles`` → ``is_duplicate(metaseq_id,
returnMatch=True)`` (``Util/lib/python/loaders/vcf_variant_loader.py:284-291``,
``variant_loader.py:173-174``) → ``VariantRecord.exists`` → SQL
``map_variants(id, firstHitOnly=True, checkAltVariants=True)``
(``Util/lib/python/database/variant.py:41,287-309``).  Here the existing rows are
exported once (their metaseq ids plus what a match contributes to the
``.mapping`` line) and the whole batch is a hash join on the GPU (K6,
``avdb_keyset_build`` / ``avdb_keyset_probe``): exact ``chrom:pos:ref:alt``
first, then — as ``checkAltVariants`` — the switched ``chrom:pos:alt:ref``;
the first of equal keys wins (``firstHitOnly``).

``map_variants`` itself is external SQL (GenomicsDBData, not in the reference):
its ranking and its result shape are **unpinned**.  A match here contributes a
list of mapping entries (default ``[{'primary_key': pk, 'bin_index': bin}]`` of
the existing row), which the loader appends exactly as the reference's
``primaryKeyMapping += matchedVariant`` does.
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch


class ExistingVariants(object):
    """Device key set over the metaseq ids of variants already loaded."""

    def __init__(self, entries: Iterable[Tuple[str, Sequence[dict]]], engine=None, check_alt: bool = True):
        from .engine import default_engine
        self._engine = engine or default_engine()
        self.check_alt = check_alt
        ids: List[str] = []
        self._payload: List[List[dict]] = []
        for metaseq, match in entries:
            ids.append(metaseq)
            self._payload.append(list(match) if not isinstance(match, dict) else [match])
        self._ids = ids
        self._index: Optional[Dict[str, int]] = None
        kb = [x.encode("utf-8") for x in ids]
        lens = np.fromiter((len(x) for x in kb), dtype=np.int64, count=len(kb))
        off = np.zeros(len(kb) + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        blob = b"".join(kb)
        dev = self._engine.device
        self.keys = torch.from_numpy(np.frombuffer(blob or b"\0", dtype=np.uint8).copy()).to(dev)
        self.key_off = torch.from_numpy(off).to(dev)
        self.table = self._engine.keyset_build(self.keys, self.key_off)
        # .mapping text each key contributes: ', '.join(repr(entry)) — what
        # print(id, primaryKeyMapping) renders for the appended entries
        frags = [", ".join(repr(d) for d in p).encode("utf-8") for p in self._payload]
        flen = np.fromiter((len(x) for x in frags), dtype=np.int64, count=len(frags))
        foff = np.zeros(len(frags) + 1, dtype=np.int64)
        np.cumsum(flen, out=foff[1:])
        self.frag = torch.from_numpy(np.frombuffer(b"".join(frags) or b"\0", dtype=np.uint8).copy()).to(dev)
        self.frag_off = torch.from_numpy(foff).to(dev)

    def __len__(self):
        return len(self._ids)

    @classmethod
    def from_tsv(cls, path: str, **kw) -> "ExistingVariants":
        """``metaseq_id<TAB>record_primary_key<TAB>bin_index`` lines (an export of
        AnnotatedVDB.Variant, e.g. ``COPY (SELECT metaseq_id, record_primary_key,
        bin_index FROM AnnotatedVDB.Variant) TO STDOUT``)."""
        entries = []
        with open(path) as fh:
            for line in fh:
                f = line.rstrip("\n").split("\t")
                if len(f) < 3 or f[0] == "metaseq_id":
                    continue
                entries.append((f[0], [{"primary_key": f[1], "bin_index": f[2]}]))
        return cls(entries, **kw)

    def payload(self, k: int) -> List[dict]:
        return self._payload[k]

    def probe(self, batch, counters=None):
        """K6 over a device record batch: ``(match int32, kind uint8)`` tensors."""
        return self._engine.keyset_probe(self.table, self.keys, self.key_off, batch, self.check_alt, counters)

    def resolve_host(self, metaseq: str) -> int:
        """Records on contigs without a canonical label (``AVDB_MATCH_HOST``): the
        same lookup on the host over the exported ids."""
        if self._index is None:
            self._index = {}
            for i, x in enumerate(self._ids):
                self._index.setdefault(x, i)
        k = self._index.get(metaseq, -1)
        if k < 0 and self.check_alt:
            c, p, r, a = metaseq.split(":")
            k = self._index.get(":".join((c, p, a, r)), -1)
        return k

    def format_args(self, match, kind):
        return (match, kind, self.frag, self.frag_off)
