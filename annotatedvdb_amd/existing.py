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

ADSP loads additionally ask ``is_duplicate(recordPK)`` for every alt that was
not skipped (``vcf_variant_loader.py:303-307``): the export's
``record_primary_key`` column forms a second key set, probed with the primary
keys K7 rendered (``avdb_keyset_probe_text``).  A primary key without an external
id equals the metaseq id, which the ``--skipExisting`` check already looked up,
so a key set over the exported primary keys answers the same as a
``map_variants`` lookup would on a consistent export (unpinned, as above).
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch


class ExistingVariants(object):
    """Device key set over the metaseq ids of variants already loaded."""

    def __init__(self, entries: Iterable[Tuple[str, Sequence[dict]]], engine=None, check_alt: bool = True,
                 primary_keys: Optional[Iterable[str]] = None):
        from .engine import default_engine
        self._engine = engine or default_engine()
        self.check_alt = check_alt
        self._pks: List[str] = list(primary_keys) if primary_keys is not None else []
        self._pk_set = None
        self._pk_dev = None
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
        entries, pks = [], []
        with open(path) as fh:
            for line in fh:
                f = line.rstrip("\n").split("\t")
                if len(f) < 3 or f[0] == "metaseq_id":
                    continue
                entries.append((f[0], [{"primary_key": f[1], "bin_index": f[2]}]))
                pks.append(f[1])
        return cls(entries, primary_keys=pks, **kw)

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

    # ---- primary keys (ADSP is_duplicate(recordPK)) ---------------------------
    def has_primary_key(self, pk: str) -> bool:
        if self._pk_set is None:
            self._pk_set = set(self._pks)
        return pk in self._pk_set

    def _pk_table(self):
        if self._pk_dev is None:
            kb = [x.encode("utf-8") for x in self._pks]
            off = np.zeros(len(kb) + 1, dtype=np.int64)
            np.cumsum(np.fromiter((len(x) for x in kb), dtype=np.int64, count=len(kb)), out=off[1:])
            dev = self._engine.device
            keys = torch.from_numpy(np.frombuffer(b"".join(kb) or b"\0", dtype=np.uint8).copy()).to(dev)
            key_off = torch.from_numpy(off).to(dev)
            self._pk_dev = (keys, key_off, self._engine.keyset_build(keys, key_off))
        return self._pk_dev

    def probe_primary_keys(self, text: torch.Tensor, text_off: torch.Tensor, n: int,
                           skip: Optional[torch.Tensor] = None, counters=None) -> torch.Tensor:
        """K6 over strings: ``match int32[n]`` (-1: not loaded) for the keys
        ``text[text_off[i]:text_off[i+1]]`` (rows with ``skip[i]`` not probed)."""
        keys, key_off, table = self._pk_table()
        return self._engine.keyset_probe_text(table, keys, key_off, text, text_off, n, skip, counters)
