"""Drop-in ``VariantAnnotator`` for the hot-path methods of
``Util/lib/python/variant_annotator.py:18-131``: allele normalisation
(common-prefix trim), end-location inference and the metaseq id.

End inference and the common prefix come from the K2 kernel
(``avdb_record_prep``) — one launch per annotator, evaluated lazily and cached
on the instance.  Batched use goes through ``engine.Engine.record_prep`` (what
the loaders do).  ``get_display_attributes`` (:134-241) comes from K5a
(``avdb_display_attributes``).
"""

from __future__ import annotations


def _xstr(v) -> str:
    return "" if v is None else str(v)


class VariantAnnotator(object):
    """GPU-backed drop-in for the reference ``VariantAnnotator``."""

    def __init__(self, refAllele, altAllele, chrom, position):
        self.__ref = refAllele
        self.__alt = altAllele
        self.__chrom = chrom
        self.__position = position
        self.__metaseqId = None
        self.__prep = None  # (end, lcp) from the kernel
        self.__set_metaseq_id()

    # -- kernel evaluation ---------------------------------------------------
    def __evaluate(self):
        if self.__prep is None:
            from .engine import default_engine, pack_records
            eng = default_engine()
            ref = self.__ref.encode("utf-8") if isinstance(self.__ref, str) else bytes(self.__ref)
            alt = self.__alt.encode("utf-8") if isinstance(self.__alt, str) else bytes(self.__alt)
            b = pack_records([0], [int(self.__position)], [ref], [alt])
            end, _, _, lcp = eng.record_prep(b)
            self.__prep = (int(end.cpu()[0]), int(lcp.cpu()[0]))
        return self.__prep

    # -- reference API ---------------------------------------------------------
    def get_normalized_alleles(self, snvDivMinus=False):
        """Left-normalised alleles (variant_annotator.py:82-121)."""
        ref, alt = self.__ref, self.__alt
        if len(ref) == 1 and len(alt) == 1:  # SNV: untouched (:97-98)
            return ref, alt
        _, lcp = self.__evaluate()
        if lcp > 0:
            normAlt = alt[lcp:]
            if not normAlt and snvDivMinus:
                normAlt = "-"
            normRef = ref[lcp:]
            if not normRef and snvDivMinus:
                normRef = "-"
            return normRef, normAlt
        return ref, alt  # no common prefix: unchanged (:120-121)

    def infer_variant_end_location(self, rsPosition=None):
        """End coordinate inferred from the alleles (variant_annotator.py:36-79)."""
        int(self.__position)  # same ValueError as the reference for a bad position
        end, _ = self.__evaluate()
        return end

    def __set_metaseq_id(self):
        self.__metaseqId = ":".join((_xstr(self.__chrom), _xstr(self.__position), self.__ref, self.__alt))

    def get_metaseq_id(self):
        return self.__metaseqId

    def get_display_attributes(self, rsPosition=None):
        """Display attributes (variant_annotator.py:134-241), computed by K5a
        (``avdb_display_attributes``) on the GPU; the dict keeps the
        reference's key order.  Alleles must be ASCII; the position an int (as
        every caller passes it)."""
        import json
        from .chromosomes import CHROM_NAMES
        from .engine import default_engine, pack_records
        eng = default_engine()
        label = _xstr(self.__chrom)
        code = CHROM_NAMES.index(label) if label in CHROM_NAMES else 255
        ref = self.__ref.encode("utf-8") if isinstance(self.__ref, str) else bytes(self.__ref)
        alt = self.__alt.encode("utf-8") if isinstance(self.__alt, str) else bytes(self.__alt)
        b = pack_records([code], [int(self.__position)], [ref], [alt])
        end, _, _, lcp = eng.record_prep(b)
        self.__prep = (int(end.cpu()[0]), int(lcp.cpu()[0]))
        text, off, state = eng.display_attributes(b, end)
        if int(state[0]) != 0:
            raise ValueError("non-ASCII allele: outside the GPU path's contract")
        attrs = json.loads(text.cpu().numpy().tobytes().decode("ascii"))
        nm = attrs.get("normalized_metaseq_id")
        if nm is not None and code == 255:  # the kernel leaves unknown contig labels to the host
            attrs["normalized_metaseq_id"] = label + nm
        return attrs
