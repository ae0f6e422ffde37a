"""Drop-in ``VariantAnnotator`` for ``Util/lib/python/variant_annotator.py:18-241``:
allele normalisation (common-prefix trim), end-location inference, the metaseq
id and the display attributes.

The reference constructs one annotator per alt allele and calls one method on
it (``vcf_parser.py:225-231``, ``vcf_variant_loader.py:309-311``), so this class
is a per-call API: each instance makes ONE call of K8a (``avdb_annotate_host``),
which runs the kernels' own record arithmetic — K2's ``infer_end`` and K5a's
``display_json``, the ``AVDB_HD`` definitions the GPU kernels compile — in the
library's host code.  No launch, no device copy, no stream sync: a GPU launch
costs more than the reference's whole call.  Batches of records go through
``engine.Engine.record_prep`` / ``display_attributes`` on the GPU (what the
loaders do).  Alleles must be ASCII (VCF 4.x REF/ALT): the kernels work on
bytes, the reference on code points, so anything else raises ``ValueError``.
"""

from __future__ import annotations

from .chromosomes import CHROM_NAMES

_CODES = {name: i for i, name in enumerate(CHROM_NAMES)}
_PC = None  # the avdb_percall binding, initialised with avdb_annotate_host + a host context


def _xstr(v) -> str:
    return "" if v is None else str(v)


def _percall():
    """``avdb_percall`` (CPython binding of K8a, built in-tree by
    ``build_native.build_percall``), bound to the library's entry."""
    global _PC
    if _PC is None:
        import ctypes
        from . import _native as N
        try:
            from . import avdb_percall as pc
        except ImportError as err:
            raise N.NativeUnavailable("avdb_percall extension not built: run "
                                      "`python -c 'import __graft_entry__ as g; g.build()'`") from err
        lib = N.load_library()
        pc.init(ctypes.cast(lib.avdb_annotate_host, ctypes.c_void_p).value, N.host_ctx().value)
        _PC = pc
    return _PC


class VariantAnnotator(object):
    """Drop-in for the reference ``VariantAnnotator`` (one K8a call per instance)."""

    __prep = None  # (end - position, lcp) from K8a, set on the instance at first use

    def __init__(self, refAllele, altAllele, chrom, position):
        self.__ref = refAllele
        self.__alt = altAllele
        self.__chrom = chrom
        self.__position = position
        # __set_metaseq_id, inline (the constructor is most of a per-call figure)
        self.__metaseqId = ":".join(("" if chrom is None else str(chrom), "" if position is None else str(position),
                                     refAllele, altAllele))

    # -- K8a ------------------------------------------------------------------
    def __evaluate(self):
        if self.__prep is None:
            self.__prep = (_PC or _percall()).end_lcp(self.__ref, self.__alt)
        return self.__prep

    # -- reference API ---------------------------------------------------------
    def get_normalized_alleles(self, snvDivMinus=False):
        """Left-normalised alleles (variant_annotator.py:30-33,82-121)."""
        ref, alt = self.__ref, self.__alt
        if len(ref) == 1 and len(alt) == 1:  # SNV: untouched (:97-98)
            return ref, alt
        lcp = self.__evaluate()[1]
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
        position = int(self.__position)  # same ValueError as the reference for a bad position
        if len(self.__ref) == 1 and len(self.__alt) == 1:  # SNV (:56-57): no call needed
            return position
        return position + self.__evaluate()[0]

    def __set_metaseq_id(self):
        c, p = self.__chrom, self.__position
        self.__metaseqId = ":".join(("" if c is None else str(c), "" if p is None else str(p), self.__ref, self.__alt))

    def get_metaseq_id(self):
        return self.__metaseqId

    def get_display_attributes(self, rsPosition=None):
        """Display attributes (variant_annotator.py:134-241): K8a's fields, the
        dict built by the binding in the reference's key order."""
        pos = int(self.__position)
        if not 0 <= pos < 4294967296:
            raise ValueError("position outside the kernels' u32 coordinates")
        attrs, rel, lcp = (_PC or _percall()).display(self.__ref, self.__alt, _xstr(self.__chrom), pos)
        self.__prep = (rel, lcp)
        if attrs is None:
            raise ValueError("display coordinates outside u32: outside the kernels' contract")
        return attrs
