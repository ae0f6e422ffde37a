"""CPU oracle for the AnnotatedVDB bin/key hot path — TEST INFRASTRUCTURE ONLY.

This module is the *checker*.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product path
(``annotatedvdb_amd``) never does, and never falls back to it.

It restates, from the reference's behaviour (not its code), every function on
the path.  Each function cites the reference ``file:line`` it follows; paths are
relative to the NIAGADS/AnnotatedVDB repository root.  Parity is pinned by the
golden vectors under ``tests/golden/`` that ``tests/golden/make_golden.py``
produced by running the reference itself (see ``tests/test_oracle_golden.py``);
the long-allele VRS digest is the exception: **parity unpinned** (vrs-python and
SeqRepo are absent; only the ``sha512t24u`` primitive is pinned, to hashlib).
"""

from __future__ import annotations

import base64
import bisect
import hashlib
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

# ---------------------------------------------------------------------------
# constants — BinIndex/bin/generate_bin_index_references.py:93
#   increments = [-1, 64e6, 32e6, ..., 15625]; level l>=1 bin width 64e6>>(l-1)
# ---------------------------------------------------------------------------
N_LEVELS = 14
LEAF_WIDTH = 15625
INC = [0] + [64000000 >> (lvl - 1) for lvl in range(1, N_LEVELS)]
assert INC[13] == LEAF_WIDTH

STATUS_OK = 0
STATUS_UNKNOWN_CHROM = 1
STATUS_OUT_OF_RANGE = 2
STATUS_END_BEFORE_START = 3  # bin of the swapped interval; reference is history-dependent
BIN_NONE = 0xFFFFFFFF

CHROM_NAMES = [str(i) for i in range(1, 23)] + ["X", "Y", "M"]


def make_code(level: int, index: int) -> int:
    return (level << 28) | index


def code_level(code: int) -> int:
    return code >> 28


def code_index(code: int) -> int:
    return code & 0x0FFFFFFF


# ---------------------------------------------------------------------------
# a2/a3: smallest enclosing bin
#   bin_index.py:59-75 (find_bin_index; end defaults to start :63) and the
#   BinIndexRef rows of generate_bin_index_references.py:46-83, ranges (lo,hi]
#   (:83), clipped at the chromosome length (:62-65).  The deepest row whose
#   (lo,hi] holds both start and end is the answer (cache test bin_index.py:70).
# ---------------------------------------------------------------------------
def bin_code(chrom_len: Optional[int], start: int, end: Optional[int] = None) -> Tuple[int, int]:
    """Return ``(code, status)`` for one interval (closed, 1-based)."""
    if end is None:
        end = start
    if chrom_len is None:
        return BIN_NONE, STATUS_UNKNOWN_CHROM
    status = STATUS_OK
    if end < start:
        start, end = end, start
        status = STATUS_END_BEFORE_START
    if start < 1 or end > chrom_len:
        return BIN_NONE, STATUS_OUT_OF_RANGE
    qs = (start - 1) // LEAF_WIDTH
    qe = (end - 1) // LEAF_WIDTH
    blen = (qs ^ qe).bit_length()
    level = 13 - blen if blen <= 12 else 0
    index = qs >> (13 - level) if level > 0 else 0
    return make_code(level, index), status


def format_bin_path(chrom_name: str, code: int) -> str:
    """ltree path ``chrN.L1.Bk...`` — labels per generate_bin_index_references.py:54,60-61,74
    (``B`` restarts at 1 under every parent; L0 is the bare chromosome)."""
    level, g = code_level(code), code_index(code)
    parts = ["chr" + chrom_name]
    for lvl in range(1, level + 1):
        gl = g >> (level - lvl)
        b = gl + 1 if lvl == 1 else (gl & 1) + 1
        parts.append("L%d.B%d" % (lvl, b))
    return ".".join(parts)


def bin_codes_np(chrom: np.ndarray, start: np.ndarray, end: Optional[np.ndarray],
                 lengths: Sequence[int]) -> Tuple[np.ndarray, np.ndarray]:
    """Vectorised :func:`bin_code` (numpy, int64 arithmetic)."""
    chrom = np.asarray(chrom, dtype=np.int64)
    s = np.asarray(start, dtype=np.int64)
    e = s.copy() if end is None else np.asarray(end, dtype=np.int64)
    lens = np.asarray(list(lengths) + [0] * (256 - len(lengths)), dtype=np.int64)
    known = chrom < len(lengths)
    L = lens[np.clip(chrom, 0, 255)]
    swapped = e < s
    lo = np.minimum(s, e)
    hi = np.maximum(s, e)
    inrange = (lo >= 1) & (hi <= L)
    qs = (np.maximum(lo, 1) - 1) // LEAF_WIDTH
    qe = (np.maximum(hi, 1) - 1) // LEAF_WIDTH
    x = qs ^ qe
    blen = np.zeros_like(x)
    nz = x > 0
    blen[nz] = np.floor(np.log2(x[nz])).astype(np.int64) + 1
    level = np.where(blen <= 12, 13 - blen, 0)
    index = np.where(level > 0, qs >> np.clip(13 - level, 0, 13), 0)
    code = (level << 28) | index
    status = np.where(swapped, STATUS_END_BEFORE_START, STATUS_OK)
    status = np.where(inrange, status, STATUS_OUT_OF_RANGE)
    status = np.where(known, status, STATUS_UNKNOWN_CHROM)
    code = np.where((status == STATUS_OK) | (status == STATUS_END_BEFORE_START), code, BIN_NONE)
    return code.astype(np.uint32), status.astype(np.uint8)


# ---------------------------------------------------------------------------
# a3: BinIndexRef table restated (for the reference-structured CPU baseline and
# for table-search cross-checks).  Rows (chrom, level, path, lo, hi) in the
# generator's depth-first order, generate_bin_index_references.py:46-77.
# ---------------------------------------------------------------------------
def generate_binindexref(chrom_name: str, length: int) -> List[Tuple[int, str, int, int]]:
    rows: List[Tuple[int, str, int, int]] = []

    def rec(prefix: str, lo: int, hi: int, level: int):
        # children of the bin (lo,hi] at `level`, clipped to hi
        if level >= N_LEVELS:
            return
        k = 0
        b = lo
        while b < hi:
            k += 1
            top = min(b + INC[level], hi, length)
            path = prefix + ".B%d" % k
            rows.append((level, path, b, top))
            rec(path + ".L%d" % (level + 1), b, top, level + 1)
            b = top

    root = "chr" + chrom_name
    rows.append((0, root, 0, length))
    rec(root + ".L1", 0, length, 1)
    return rows


class LeftOpenRange:
    """``(lo, hi]`` containment with the published control flow of psycopg2's
    ``Range.__contains__`` (bounds string checked per call) — the object
    ``NumericRange(lo, hi, '(]')`` the cache test at bin_index.py:70 calls."""

    __slots__ = ("_lower", "_upper", "_bounds")

    def __init__(self, lower, upper, bounds="(]"):
        self._lower = lower
        self._upper = upper
        self._bounds = bounds

    def __contains__(self, x):
        if self._bounds is None:
            return False
        if self._lower is not None:
            if self._bounds[0] == "[":
                if x < self._lower:
                    return False
            elif x <= self._lower:
                return False
        if self._upper is not None:
            if self._bounds[1] == "]":
                if x > self._upper:
                    return False
            elif x >= self._upper:
                return False
        return True


def xstr(value, nullStr="", falseAsNull=False):
    """GenomicsDBData ``xstr`` as used by bin_index.py:64 (str of a non-null value)."""
    if value is None:
        return nullStr
    if falseAsNull and value is False:
        return nullStr
    return str(value)


class BinTable:
    """Per-(chrom, level) sorted (lo, hi, path) lists; deepest-containing search."""

    def __init__(self, lengths: Dict[str, int]):
        self.by: Dict[Tuple[str, int], Tuple[List[int], List[Tuple[int, int, str]]]] = {}
        for name, L in lengths.items():
            per: Dict[int, List[Tuple[int, int, str]]] = {}
            for level, path, lo, hi in generate_binindexref(name, L):
                per.setdefault(level, []).append((lo, hi, path))
            for level, lst in per.items():
                lst.sort()
                self.by[("chr" + name, level)] = ([r[0] for r in lst], lst)

    def find(self, chrm: str, start: int, end: int):
        for level in range(13, -1, -1):
            ent = self.by.get((chrm, level))
            if ent is None:
                continue
            los, lst = ent
            k = bisect.bisect_left(los, start) - 1
            if k < 0:
                continue
            lo, hi, path = lst[k]
            if lo < start <= hi and lo < end <= hi:
                return {"chromosome": chrm, "global_bin_path": path,
                        "location": LeftOpenRange(lo, hi), "bin_level": 1 + 2 * level}
        return None


class PortBinIndex:
    """Reference-structured port of ``BinIndex`` (bin_index.py:16-75) used as the
    CPU baseline: one-bin cache served only for L13 bins (:66-71, nlevel>=27,
    range containment through a ``__contains__`` call like NumericRange), table
    search on a miss in place of the SQL round trip (:43-56)."""

    def __init__(self, table: BinTable):
        self._table = table
        self._currentBin = {}

    def _update_current_bin_index(self, chrm, start, end):
        self._currentBin = self._table.find(chrm, start, end)

    def find_bin_index(self, chrm, start, end=None):
        if end is None:
            end = start
        if "chr" not in chrm:
            chrm = "chr" + xstr(chrm)
        if bool(self._currentBin):
            if self._currentBin["bin_level"] >= 27:
                brange = self._currentBin["location"]
                if self._currentBin["chromosome"] == chrm \
                        and start in brange and end in brange:
                    return self._currentBin["global_bin_path"]
        self._update_current_bin_index(chrm, start, end)
        return self._currentBin["global_bin_path"]  # None -> TypeError, as :75


# ---------------------------------------------------------------------------
# a4/a5: allele normalisation (lcp) and end inference
#   variant_annotator.py:82-121 (__normalize_alleles: strip the longest common
#   prefix; SNVs untouched :97-98) and :36-79 (infer_variant_end_location).
# ---------------------------------------------------------------------------
def common_prefix(ref: bytes, alt: bytes) -> int:
    if len(ref) == 1 and len(alt) == 1:
        return 0  # SNV: no normalisation (:97-98), even when ref == alt
    n = 0
    m = min(len(ref), len(alt))
    while n < m and ref[n] == alt[n]:
        n += 1
    return n


def infer_end(pos: int, ref, alt) -> Tuple[int, int]:
    """Return ``(end, lcp)``; ``start`` stays at the VCF POS
    (vcf_variant_loader.py:310)."""
    if isinstance(ref, str):
        ref = ref.encode()
    if isinstance(alt, str):
        alt = alt.encode()
    r, a = len(ref), len(alt)
    lcp = common_prefix(ref, alt)
    nr, na = r - lcp, a - lcp
    if r == 1 and a == 1:
        return pos, lcp
    if r == a:
        if ref == alt[::-1]:  # inversion (:61-62)
            return pos + r - 1, lcp
        return pos + nr - 1, lcp  # substitution (:65)
    if na >= 1:  # insertion / indel (:67-74)
        if nr >= 1:
            return pos + nr, lcp
        if r > 1:
            return pos + r - 1, lcp
        return pos + 1, lcp
    if nr == 0:  # deletion (:77-79)
        return pos + r - 1, lcp
    return pos + nr, lcp


# ---------------------------------------------------------------------------
# a6/a8: metaseq id and short primary key
#   variant_annotator.py:124-126; primary_key_generator.py:99-122
# ---------------------------------------------------------------------------
MAX_SEQUENCE_LENGTH = 50  # primary_key_generator.py:53


def metaseq_id(chrom: str, pos: int, ref: str, alt: str) -> str:
    return ":".join((str(chrom), str(pos), ref, alt))


def is_long(ref: str, alt: str, max_len: int = MAX_SEQUENCE_LENGTH) -> bool:
    return len(ref) + len(alt) > max_len


def primary_key(chrom: str, pos: int, ref: str, alt: str, external_id: Optional[str] = None,
                digest: Optional[str] = None, max_len: int = MAX_SEQUENCE_LENGTH) -> str:
    pk = [str(chrom), str(pos)]
    if len(ref) + len(alt) <= max_len:
        pk += [ref, alt]
    else:
        if digest is None:
            raise ValueError("long allele needs a VRS digest (parity unpinned)")
        pk.append(digest)
    if external_id is not None:
        pk.append(external_id)
    return ":".join(pk)


class PortPKGenerator(object):
    """The reference ``VariantPKGenerator.generate_primary_key``'s per-call
    structure (primary_key_generator.py:99-122): the metaseq id split on ':' and the
    key joined from the pieces; short alleles only (long ones: parity unpinned)."""

    def __init__(self, maxSequenceLength=MAX_SEQUENCE_LENGTH):
        self._maxSequenceLength = maxSequenceLength

    def generate_primary_key(self, metaseqId, externalId=None):
        chrm, position, ref, alt = metaseqId.split(":")
        pk = [chrm, position]
        if len(ref) + len(alt) <= self._maxSequenceLength:
            pk.extend([ref, alt])
        else:
            raise ValueError("long allele needs a VRS digest (parity unpinned)")
        if externalId is not None:
            pk.append(externalId)
        return ":".join(pk)


def c1_port_loop(names, pos, refs, alts, exts, bin_index) -> int:
    """Reference-structured per-record path SURVEY.md §6 measured the reference
    on (the C1 CPU baseline), with the reference's per-record objects, in the
    loader's order (vcf_variant_loader.py:243-311): an annotator per alt allele
    (variant_annotator.py:21-27, metaseq id :124-126), the primary key from its
    metaseq id (primary_key_generator.py:99-122), its normalized alleles (:309), end
    inference on a second annotator (vcf_parser.py:225-231 builds one per call;
    variant_annotator.py:36-79 normalizes again) and the one-bin-cached
    find_bin_index (bin_index.py:59-75), one record at a time."""
    pkg = PortPKGenerator()
    for c, p, r, a, e in zip(names, pos, refs, alts, exts):
        va = PortVariantAnnotator(r, a, c, p)
        pkg.generate_primary_key(va.metaseq, e)
        va.get_normalized_alleles()
        end = PortVariantAnnotator(r, a, c, p).infer_variant_end_location()
        bin_index.find_bin_index(c, p, end)
    return len(pos)


# ---------------------------------------------------------------------------
# a9: sha512t24u (GA4GH computed-identifier digest) — the pinnable primitive.
#   primary_key_generator.py:147-165 drops the 'ga4gh:VA.' prefix of the
#   ga4gh_identify() result.  The Allele/SequenceLocation serialisation below is
#   the published VRS 1.x compact form; PARITY UNPINNED (no vrs-python here).
# ---------------------------------------------------------------------------
def sha512t24u(blob: bytes) -> str:
    return base64.urlsafe_b64encode(hashlib.sha512(blob).digest()[:24]).decode()


# The digest serialisation (VRS "Computed Identifiers"): keys sorted, compact
# separators, a nested identifiable object or a ga4gh CURIE ("ga4gh:SQ.<digest>")
# written as its bare digest.  schema "1.2" (VRS 1.2 / 1.3, vrs-python 0.7-0.8 — the
# python-jsonschema-objects era whose ``Translator._from_gnomad(..., require_validation=)``
# and ``.for_json()`` primary_key_generator.py:137,142 call): SequenceInterval of
# Number, LiteralSequenceExpression — what K4 implements.  schema "1.1": the same rules
# over SimpleInterval / SequenceState, the form of vrs-python's published VRS 1.1
# example, which tests/test_oracle_golden.py reproduces digit for digit to pin the rules.
def vrs_location_blob(sequence_digest: str, start: int, end: int, schema: str = "1.2") -> bytes:
    if schema == "1.1":
        return ('{"interval":{"end":%d,"start":%d,"type":"SimpleInterval"},"sequence_id":"%s",'
                '"type":"SequenceLocation"}' % (end, start, sequence_digest)).encode()
    return ('{"interval":{"end":{"type":"Number","value":%d},"start":{"type":"Number","value":%d},'
            '"type":"SequenceInterval"},"sequence_id":"%s","type":"SequenceLocation"}'
            % (end, start, sequence_digest)).encode()


def vrs_allele_blob(location_digest: str, state: bytes, schema: str = "1.2") -> bytes:
    kind = b"SequenceState" if schema == "1.1" else b"LiteralSequenceExpression"
    return (b'{"location":"' + location_digest.encode() + b'","state":{"sequence":"' + state
            + b'","type":"' + kind + b'"},"type":"Allele"}')


def vrs_allele_digest(sequence_digest: str, pos: int, ref, alt, schema: str = "1.2") -> str:
    """gnomAD-style ``chr-pos-ref-alt`` → Allele with interval (pos-1, pos-1+len(ref)]
    and literal state ``alt`` (no normalisation: primary_key_generator.py:53,83)."""
    if isinstance(ref, str):
        ref = ref.encode()
    if isinstance(alt, str):
        alt = alt.encode()
    start = pos - 1
    loc = sha512t24u(vrs_location_blob(sequence_digest, start, start + len(ref), schema))
    return sha512t24u(vrs_allele_blob(loc, alt, schema))


# ---------------------------------------------------------------------------
# a12: in-batch dedup — keep the first occurrence of each primary key
#   (stable input order).  Reference: removeDuplicates.sql:2-24 groups by
#   record_primary_key per chromosome and keeps one row.
# ---------------------------------------------------------------------------
def dedup_keep(keys: Sequence) -> List[int]:
    seen = set()
    keep = []
    for k in keys:
        if k in seen:
            keep.append(0)
        else:
            seen.add(k)
            keep.append(1)
    return keep


# ---------------------------------------------------------------------------
# §8f rank 3: display attributes
#   variant_annotator.py:134-241 (get_display_attributes), with the external
#   GenomicsDBData helpers it calls restated as published:
#   truncate(s, n) = s if len(s) <= n else s[:n] + '...', reverse(s) = s[::-1].
#   Returns the dict in the reference's insertion order (dict.update() of an
#   existing key keeps its position).
# ---------------------------------------------------------------------------
def _truncate(s: str, n: int) -> str:
    return s if len(s) <= n else s[:n] + "..."


def _trunc_allele(s: str, long: bool = False) -> str:  # variant_annotator.py:8-10
    return _truncate(s, 100) if long else _truncate(s, 8)


def normalized_alleles(ref: str, alt: str, snv_div_minus: bool = False) -> Tuple[str, str]:
    """variant_annotator.py:82-121."""
    if len(ref) == 1 and len(alt) == 1:
        return ref, alt
    lcp = 0
    while lcp < len(ref) and lcp < len(alt) and ref[lcp] == alt[lcp]:
        lcp += 1
    if lcp == 0:
        return ref, alt
    nref, nalt = ref[lcp:], alt[lcp:]
    if snv_div_minus:
        nref = nref or "-"
        nalt = nalt or "-"
    return nref, nalt


def display_attributes(chrom: str, pos: int, ref: str, alt: str) -> dict:
    """variant_annotator.py:134-241 (position is the int VCF POS)."""
    r, a = len(ref), len(alt)
    nref_acc, nalt_acc = normalized_alleles(ref, alt)
    nr, na = len(nref_acc), len(nalt_acc)
    nref, nalt = normalized_alleles(ref, alt, True)
    end, _ = infer_end(pos, ref, alt)
    at = {"location_start": pos, "location_end": pos}
    nmid = ":".join((str(chrom), str(pos), nref, nalt))
    if nmid != metaseq_id(chrom, pos, ref, alt):
        at["normalized_metaseq_id"] = nmid
    if r == 1 and a == 1:
        at.update(variant_class="single nucleotide variant", variant_class_abbrev="SNV",
                  display_allele=ref + ">" + alt, sequence_allele=ref + "/" + alt)
    elif r == a:
        if ref == alt[::-1]:
            at.update(variant_class="inversion", variant_class_abbrev="MNV", display_allele="inv" + ref,
                      sequence_allele=_trunc_allele(ref) + "/" + _trunc_allele(alt), location_end=end)
        else:
            at.update(variant_class="substitution", variant_class_abbrev="MNV",
                      display_allele=nref + ">" + nalt,
                      sequence_allele=_trunc_allele(nref) + "/" + _trunc_allele(nalt),
                      location_start=pos, location_end=end)
    elif na >= 1:
        at["location_start"] = pos + 1
        orig = ref[1:]
        ndup = orig.count(nalt)
        dup = orig == nalt or (ndup > 0 and len(orig) / ndup == len(nalt))
        pre = "dup" if dup else "ins"
        if nr >= 1:
            at.update(location_end=end, display_allele="del" + _trunc_allele(nref, True) + pre +
                      _trunc_allele(nalt, True), sequence_allele=_trunc_allele(nref) + "/" +
                      _trunc_allele(nalt), variant_class="indel", variant_class_abbrev="INDEL")
        elif end != pos + 1:
            at.update(location_end=end, display_allele="del" + _trunc_allele(orig, True) + pre +
                      _trunc_allele(nalt, True), sequence_allele=_trunc_allele(nref) + "/" +
                      _trunc_allele(nalt), variant_class="indel", variant_class_abbrev="INDEL")
        else:
            at.update(location_end=pos + 1, display_allele=pre + _trunc_allele(nalt, True),
                      sequence_allele=pre + _trunc_allele(nalt),
                      variant_class="duplication" if dup else "insertion",
                      variant_class_abbrev=pre.upper())
    else:
        at.update(variant_class="deletion", variant_class_abbrev="DEL", location_end=end,
                  location_start=pos + 1, display_allele="del" + _trunc_allele(nref, True),
                  sequence_allele=_trunc_allele(nref) + "/-")
    return at


class PortVariantAnnotator(object):
    """The reference ``VariantAnnotator``'s per-call structure
    (variant_annotator.py:21-241): the metaseq id joined in the constructor, each
    method normalising the alleles again as the reference does (:46, :147-152).
    The CPU baseline of the drop-in per-call figures (bench.py --workload dropin)."""

    def __init__(self, refAllele, altAllele, chrom, position):
        self.ref, self.alt, self.chrom, self.position = refAllele, altAllele, chrom, position
        self.metaseq = ":".join((xstr(chrom), xstr(position), refAllele, altAllele))

    def get_normalized_alleles(self, snvDivMinus=False):
        ref, alt = self.ref, self.alt
        if len(ref) == 1 and len(alt) == 1:
            return ref, alt
        last = -1
        for i in range(len(ref)):  # :100-107, slice compares as the reference does
            if ref[i:i + 1] == alt[i:i + 1]:
                last = i
            else:
                break
        if last >= 0:
            nalt = alt[last + 1:]
            if not nalt and snvDivMinus:
                nalt = "-"
            nref = ref[last + 1:]
            if not nref and snvDivMinus:
                nref = "-"
            return nref, nalt
        return ref, alt

    def infer_variant_end_location(self, rsPosition=None):
        ref, alt = self.ref, self.alt
        nref, nalt = self.get_normalized_alleles()
        r, a, nr, na = len(ref), len(alt), len(nref), len(nalt)
        position = int(self.position)
        if r == 1 and a == 1:
            return position
        if r == a:
            if ref == alt[::-1]:
                return position + r - 1
            return position + nr - 1
        if na >= 1:
            if nr >= 1:
                return position + nr
            if nr == 0 and r > 1:
                return position + r - 1
            return position + 1
        if nr == 0:
            return position + r - 1
        return position + nr

    def get_display_attributes(self, rsPosition=None):
        return display_attributes(xstr(self.chrom), self.position, self.ref, self.alt)


# ---------------------------------------------------------------------------
# §8f rank 2: INFO FREQ -> allele_frequencies, COPY row, .mapping line
#   vcf_parser.py:76-114 (INFO parse: '\x2c'->',', '\x59'->'/', '#'->':',
#   split ';', first '=', numeric coercion), :200-222 (get_frequencies),
#   vcf_variant_loader.py:320-346 (COPY values, '#'-joined), load_vcf_file.py:116-117
#   (mapping line = variant id TAB str(list of dicts)).
# ---------------------------------------------------------------------------
def to_numeric(value):
    """GenomicsDBData ``to_numeric``: int, else float, else unchanged."""
    try:
        return int(value)
    except (ValueError, TypeError):
        try:
            return float(value)
        except (ValueError, TypeError):
            return value


def parse_info(info: str) -> dict:
    s = info.replace("\\x2c", ",").replace("\\x59", "/").replace("#", ":")
    d = dict(item.split("=", 1) if "=" in item else [item, True] for item in s.split(";"))
    return {k: (to_numeric(v) if isinstance(v, str) else v) for k, v in d.items()}


def frequencies(info: dict, alt_field: str, allele: str):
    """vcf_parser.py:200-222; raises like the reference on malformed FREQ."""
    g = info.get("FREQ")
    if g is None:
        return None
    alts = alt_field.split(",")
    k = alts.index(allele) + 1
    popf = {p.split(":")[0]: p.split(":")[1] for p in g.split("|")}
    out = {pop: {"gmaf": to_numeric(f.split(",")[k])} for pop, f in popf.items()
           if f.split(",")[k] not in (".", "0")}
    return None if not out else out


def xstr_json(value, nullStr="", falseAsNull=False) -> str:
    """``xstr`` as applied to the COPY values: None -> nullStr, False -> nullStr
    with falseAsNull, dicts -> ``json.dumps`` (the JSONB columns'
    serialisation), else ``str``."""
    import json
    if value is None:
        return nullStr
    if falseAsNull and value is False:
        return nullStr
    if isinstance(value, (dict, list)):
        return json.dumps(value)
    return str(value)


def copy_row(chrom: str, pos: int, ref: str, alt: str, pk: str, bin_path: str, alg_id,
             ref_snp_id: Optional[str], is_multi: bool, freq) -> str:
    """One COPY line (vcf_variant_loader.py:320-343), without the newline."""
    return "#".join(["chr" + chrom, pk, str(pos), metaseq_id(chrom, pos, ref, alt), bin_path,
                     xstr_json(alg_id), xstr_json(ref_snp_id, nullStr="NULL"),
                     xstr_json(is_multi, falseAsNull=True, nullStr="NULL"),
                     xstr_json(display_attributes(chrom, pos, ref, alt), nullStr="NULL"),
                     xstr_json(freq, nullStr="NULL")])


def mapping_line(variant_id: str, mapping: List[dict]) -> str:
    """load_vcf_file.py:116-117: ``print(id, pk, sep='\\t')``."""
    return "%s\t%s" % (variant_id, mapping)


VCF_FIELDS = ["chrom", "pos", "id", "ref", "alt", "qual", "filter", "info"]


def parse_vcf_line(line: str) -> dict:
    """VcfEntryParser.parse_entry (vcf_parser.py:76-114) + get_variant /
    get_refsnp (:127-169).  Raises what the reference raises."""
    values = line.split("\t")
    try:
        entry = dict(zip(VCF_FIELDS, values)) if len(values) == len(VCF_FIELDS) \
            else {f: values[i] for i, f in enumerate(VCF_FIELDS)}
        ent = {k: to_numeric(v) for k, v in entry.items()}
        if "info" in ent:
            ent["info"] = parse_info(ent["info"])
    except IndexError:
        raise IndexError("The number of fields in the VCF entry do not match")
    except Exception as err:  # noqa: BLE001 — the reference wraps everything else
        raise ImportError(str(err))
    chrom = xstr(ent["chrom"])
    if chrom == "MT":
        chrom = "M"
    alts = ent["alt"].split(",")
    vid = ent["id"]
    if vid == "." or vid.startswith("rs"):
        vid = ":".join((chrom.replace("chr", ""), xstr(ent["pos"]), ent["ref"], ent["alt"]))
    if "rs" in ent["id"]:
        rs = ent["id"]
    elif "RS" in ent["info"]:
        rs = "rs" + str(ent["info"]["RS"])
    else:
        rs = None
    return {"id": vid, "ref_snp_id": rs, "ref": ent["ref"], "alt_field": ent["alt"], "alts": alts,
            "is_multi": len(alts) > 1, "chromosome": xstr(chrom).replace("chr", ""),
            "position": int(ent["pos"]), "info": ent["info"]}


def existing_match(existing: Dict[str, int], metaseq: str, check_alt: bool = True) -> int:
    """--skipExisting lookup (VariantRecord.exists, database/variant.py:287-309 ->
    map_variants(id, firstHitOnly=True, checkAltVariants=True), external SQL):
    index of the first existing row with this metaseq id, else of the switched
    alleles, else -1.  ``existing`` maps id -> first index."""
    k = existing.get(metaseq, -1)
    if k < 0 and check_alt:
        c, p, r, a = metaseq.split(":")
        k = existing.get(":".join((c, p, a, r)), -1)
    return k


def load_line(line: str, lengths: Sequence[int], alg_id="1", max_len: int = MAX_SEQUENCE_LENGTH,
              bin_index: Optional["PortBinIndex"] = None, existing: Optional[Dict[str, int]] = None,
              payloads: Optional[List[List[dict]]] = None):
    """One line of the load driver (load_vcf_file.py:101-119 ->
    VCFVariantLoader.parse_variant, vcf_variant_loader.py:259-391, short keys
    only).  Returns ``(error_type_name | None, mapping_lines, copy_rows)``;
    on an error the rows written before it are returned too.  With
    ``bin_index`` (a :class:`PortBinIndex`) the bin comes from the reference's
    cached lookup structure (the CPU baseline), else from the closed form."""
    rows: List[str] = []
    try:
        v = parse_vcf_line(line.rstrip())
        mapping = []
        for alt in v["alts"]:
            if alt == ".":
                continue
            ms = metaseq_id(v["chromosome"], v["position"], v["ref"], alt)
            if len(ms.split(":")) != 4:
                raise ValueError("too many values to unpack")
            if is_long(v["ref"], alt, max_len):
                raise ValueError("long allele: VRS digest (parity unpinned)")
            pk = primary_key(v["chromosome"], v["position"], v["ref"], alt, v["ref_snp_id"], max_len=max_len)
            if existing is not None:  # vcf_variant_loader.py:285-291
                k = existing_match(existing, ms)
                if k >= 0:
                    mapping += payloads[k]
                    continue
            end, _ = infer_end(v["position"], v["ref"], alt)
            chrm = v["chromosome"] if "chr" in v["chromosome"] else "chr" + v["chromosome"]
            name = chrm[3:] if chrm.startswith("chr") else None
            L = lengths[CHROM_NAMES.index(name)] if name in CHROM_NAMES else None
            if bin_index is not None:
                path = bin_index.find_bin_index(v["chromosome"], v["position"], end)
            else:
                code, _ = bin_code(L, v["position"], end)
                if code == BIN_NONE:
                    raise TypeError("'NoneType' object is not subscriptable")
                path = format_bin_path(name, code)
            freq = frequencies(v["info"], v["alt_field"], alt)
            rows.append(copy_row(v["chromosome"], v["position"], v["ref"], alt, pk, path, alg_id,
                                 v["ref_snp_id"], v["is_multi"], freq))
            mapping.append({"primary_key": pk, "bin_index": path})
        return None, [mapping_line(v["id"], mapping)], rows
    except Exception as err:  # noqa: BLE001
        return type(err).__name__, [], rows


# ---------------------------------------------------------------------------
# L8 histogram (per-shard counters all-gathered across GPUs)
# ---------------------------------------------------------------------------
L8_WIDTH = INC[8]


def l8_offsets(lengths: Sequence[int]) -> List[int]:
    off = [0]
    for L in lengths:
        off.append(off[-1] + (L + L8_WIDTH - 1) // L8_WIDTH)
    return off


def l8_histogram_np(chrom, start, status, lengths) -> np.ndarray:
    off = np.asarray(l8_offsets(lengths), dtype=np.int64)
    chrom = np.asarray(chrom, dtype=np.int64)
    start = np.asarray(start, dtype=np.int64)
    ok = (np.asarray(status) == STATUS_OK) | (np.asarray(status) == STATUS_END_BEFORE_START)
    idx = off[np.clip(chrom[ok], 0, len(lengths) - 1)] + (start[ok] - 1) // L8_WIDTH
    return np.bincount(idx, minlength=int(off[-1])).astype(np.uint32)
