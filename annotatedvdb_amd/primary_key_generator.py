"""Drop-in ``VariantPKGenerator`` (Util/lib/python/primary_key_generator.py:33-165).

Keys follow the reference rules (:99-122): ``chr:pos:ref:alt[:externalId]``
when ``len(ref)+len(alt) <= maxSequenceLength`` (default 50, :53), otherwise
``chr:pos:<digest>[:externalId]`` where the digest is the GA4GH computed
identifier of the VRS Allele with its ``ga4gh:VA.`` prefix dropped
(:147-165).  The digest is computed on the GPU (K4, ``avdb_vrs_digest``).

The reference obtains the Allele from ``vrs-python``'s
``Translator._from_gnomad`` against a local SeqRepo, which is not available
here: the refget sequence digest of every contig must be supplied
(``sequence_digests``, or a ``chrom<TAB>digest`` / JSON file given as
``seqrepoProxyPath``), reference-sequence validation is not performed, and
parity of the digest with vrs-python is **unpinned** (DESIGN.md).  Without
digests a long allele raises ``ValueError('Sequence mismatch for ...')`` — the
same exception the reference raises when VRS translation fails (:116-117).
"""

from __future__ import annotations

import json
import os
import warnings
from typing import Dict, List, Optional, Sequence, Tuple

from .chromosomes import CHROM_NAMES, UNKNOWN_CHROM, chrom_code


def load_sequence_digests(path: str) -> Dict[str, str]:
    """``chrom -> 32-char refget digest`` from a JSON object or a TSV file."""
    if path.endswith(".json"):
        d = json.load(open(path))
    else:
        d = {}
        for line in open(path):
            line = line.strip()
            if line and not line.startswith("#"):
                k, v = line.split("\t")[:2]
                d[k] = v
    out = {}
    for k, v in d.items():
        v = v.split("SQ.", 1)[1] if "SQ." in v else v
        code = chrom_code(k)
        if code != UNKNOWN_CHROM:
            out[CHROM_NAMES[code]] = v
    return out


class VariantPKGenerator(object):
    """GPU-backed drop-in for the reference ``VariantPKGenerator``."""

    def __init__(self, genomeBuild, seqrepoProxyPath=None, maxSequenceLength=50, normalize=False,
                 verbose=False, debug=False, sequence_digests: Optional[Dict[str, str]] = None,
                 device=None):
        self._verbose = verbose
        self._debug = debug
        self._genomeBuild = genomeBuild
        self._maxSequenceLength = maxSequenceLength
        self._normalize = normalize
        self._ga4gh_sequence_map = {}
        self._device = device
        self._engine = None
        digs = dict(sequence_digests or {})
        if not digs and seqrepoProxyPath:
            if os.path.isfile(str(seqrepoProxyPath)):
                digs = load_sequence_digests(str(seqrepoProxyPath))
            else:
                # the reference CLI passes a SeqRepo directory (primary_key_generator.py:74-83);
                # without vrs-python/SeqRepo only a chrom->refget-digest file can be used,
                # so say now that long alleles (> maxSequenceLength) will fail
                warnings.warn("seqrepoProxyPath %r is not a chrom<TAB>refget-digest (or JSON) file: long-allele "
                              "primary keys (len(ref)+len(alt) > %d) will raise ValueError('Sequence mismatch "
                              "...'); pass sequence_digests or a digest file" % (seqrepoProxyPath,
                                                                                maxSequenceLength),
                              RuntimeWarning, stacklevel=2)
        self._ga4gh_sequence_map = digs
        if normalize:
            raise NotImplementedError("VRS normalisation needs vrs-python/SeqRepo (absent)")

    def max_sequence_length(self) -> int:
        return self._maxSequenceLength

    def genome_build(self):
        return self._genomeBuild

    def has_sequence_digests(self) -> bool:
        return all(c in self._ga4gh_sequence_map for c in CHROM_NAMES)

    def _eng(self):
        if self._engine is None:
            from .engine import Engine
            if not self.has_sequence_digests():
                raise ValueError("no refget sequence digests configured")
            self._engine = Engine(self._device, assembly=self._genomeBuild if self._genomeBuild in
                                  ("GRCh37", "GRCh38") else "GRCh38",
                                  sequence_digests=[self._ga4gh_sequence_map[c] for c in CHROM_NAMES])
        return self._engine

    # ---- reference API ----------------------------------------------------
    def translate_vrs(self, vrsDict, formatSpec="spdi"):
        raise NotImplementedError("VRS translation needs vrs-python/SeqRepo (absent)")

    def get_vrs_allele_dict(self, metaseqId, serialize=False, toJson=False, requireValidation=True):
        raise NotImplementedError("VRS allele objects need vrs-python (absent); see compute_vrs_identifier")

    def compute_vrs_identifier(self, metaseqId, requireValidation=True):
        """Digest of the VRS Allele for ``chr:pos:ref:alt`` (K4 on the GPU)."""
        return self.compute_vrs_identifiers([metaseqId])[0]

    def generate_primary_key(self, metaseqId, externalId=None, requireValidation=True):
        """Primary key per primary_key_generator.py:99-122."""
        chrm, position, ref, alt = metaseqId.split(":")
        pk = [chrm, position]
        if len(ref) + len(alt) <= self._maxSequenceLength:
            pk.extend([ref, alt])
        else:
            try:
                pk.append(self.compute_vrs_identifier(metaseqId, requireValidation))
            except Exception as err:
                raise ValueError(f"Sequence mismatch for {metaseqId}: {err}")
        if externalId is not None:
            pk.append(externalId)
        return ":".join(pk)

    # ---- batch API --------------------------------------------------------
    def compute_vrs_identifiers(self, metaseqIds: Sequence[str]) -> List[str]:
        from .engine import pack_records
        eng = self._eng()
        codes, pos, refs, alts = [], [], [], []
        for m in metaseqIds:
            chrm, position, ref, alt = m.split(":")
            c = chrom_code(chrm)
            if c == UNKNOWN_CHROM:
                raise ValueError(f"unknown chromosome {chrm}")
            codes.append(c)
            pos.append(int(position))
            refs.append(ref.encode())
            alts.append(alt.encode())
        b = pack_records(codes, pos, refs, alts)
        dig, _ = eng.vrs_digest(b, max_seq_len=0)  # every row is hashed
        raw = dig.cpu().numpy()
        return [raw[i].tobytes().decode("ascii") for i in range(len(metaseqIds))]

    def generate_primary_keys(self, items: Sequence[Tuple[str, Optional[str]]]) -> List[str]:
        """Batch ``generate_primary_key`` over ``(metaseqId, externalId)`` pairs;
        long alleles are digested in one GPU launch."""
        out: List[Optional[str]] = [None] * len(items)
        longs = []
        for i, (m, ext) in enumerate(items):
            chrm, position, ref, alt = m.split(":")
            if len(ref) + len(alt) <= self._maxSequenceLength:
                out[i] = ":".join([chrm, position, ref, alt] + ([ext] if ext is not None else []))
            else:
                longs.append(i)
        if longs:
            try:
                digs = self.compute_vrs_identifiers([items[i][0] for i in longs])
            except Exception as err:
                raise ValueError(f"Sequence mismatch for {items[longs[0]][0]}: {err}")
            for i, d in zip(longs, digs):
                m, ext = items[i]
                chrm, position = m.split(":")[:2]
                out[i] = ":".join([chrm, position, d] + ([ext] if ext is not None else []))
        return out
