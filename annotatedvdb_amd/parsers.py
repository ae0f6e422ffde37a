"""Host-side VCF entry parsing — drop-in for the parts of
``Util/lib/python/parsers/vcf_parser.py`` (``VcfEntryParser``, :34-240) that feed
the bin/key path: field split, numeric coercion, INFO parsing, chromosome
normalisation (``MT``→``M`` :136-137, ``chr`` strip :150), multi-allelic split
(:138), variant id (:140-142) and refSNP id (:158-169).

This is text handling on the host (SURVEY.md §8f rank 1 is a GPU tokenizer);
the numeric work on the parsed records runs in the kernels.  End inference is
delegated to the GPU-backed ``VariantAnnotator``.
"""

from __future__ import annotations

import csv
import re
from types import SimpleNamespace

from .variant_annotator import VariantAnnotator

# Every ASCII string int() or float() accepts matches this (a superset: the
# characters of a number, or nan / inf / infinity, between str.isspace()
# whitespace); a string that does not match is returned without trying either.
_NUMISH = re.compile(r"[\s\x1c-\x1f+\-]*(?:[0-9_.eE+\-]+|nan|inf|infinity)[\s\x1c-\x1f]*", re.I)
_NOT_INT = re.compile(r"[.eEnNiIaAfFtTyY]")  # int() accepts none of these


def to_numeric(value):
    """int, else float, else the value (GenomicsDBData ``to_numeric`` behaviour).
    ASCII strings take a fast path with the same result: plain digits go to
    int(), text that cannot be a number is returned as is, and text int()
    cannot accept goes straight to float() (the conversions that would raise
    and be caught are skipped)."""
    if value.__class__ is str and value.isascii():
        if value.isdigit() and len(value) < 4000:
            return int(value)
        if _NUMISH.fullmatch(value) is None:
            return value
        if _NOT_INT.search(value) is not None:
            try:
                return float(value)
            except (ValueError, TypeError):
                return value
    try:
        return int(value)
    except (ValueError, TypeError):
        try:
            return float(value)
        except (ValueError, TypeError):
            return value


def convert_str2numeric_values(d: dict) -> dict:
    return {k: (to_numeric(v) if isinstance(v, str) else v) for k, v in d.items()}


def _xstr(v, nullStr="", falseAsNull=False):
    if v is None:
        return nullStr
    if falseAsNull and v is False:
        return nullStr
    return str(v)


_MISSING = object()

DEFAULT_FIELDS = ["chrom", "pos", "id", "ref", "alt", "qual", "filter", "info"]


class _LazyInfo(object):
    """An INFO string not yet split into its dict (vcf_parser.py:101-110)."""

    __slots__ = ("s",)

    def __init__(self, s: str):
        self.s = s

    def raw(self) -> dict:
        """The INFO dict before numeric coercion (vcf_parser.py:101-108)."""
        infoStr = self.s.replace("\\x59", "/").replace("#", ":")
        return dict(item.split("=", 1) if "=" in item else [item, True] for item in infoStr.split(";"))

    def resolve(self) -> dict:
        return convert_str2numeric_values(self.raw())


class VcfEntryParser(object):
    """Drop-in for the reference ``VcfEntryParser`` (hot-path subset)."""

    def __init__(self, entry, headerFields=None, identityOnly=False, verbose=False, debug=False,
                 loader=None):
        self.__debug = debug
        self.__verbose = verbose
        self._header_fields = ["chrom", "pos", "id", "ref", "alt"] if identityOnly \
            else DEFAULT_FIELDS if headerFields is None \
            else [x.lower().replace("#", "") for x in headerFields]
        self.__raw_info = None
        self.__entry = None if entry is None else self.parse_entry(entry)

    def parse_entry(self, inputStr):
        """vcf_parser.py:76-114.  The INFO dict is built and coerced on first
        use (get_info / get_refsnp / get_entry): the per-line loader reads at
        most RS, RSPOS and FREQ of it, and an INFO value the reference could not
        parse still raises here, at parse time."""
        fields = self._header_fields
        values = inputStr.split("\t")
        try:
            entry = dict(zip(fields, values)) if len(fields) == len(values) \
                else {field: values[index] for index, field in enumerate(fields)}
            result = convert_str2numeric_values(entry)
            if "info" in result:
                # (a numeric INFO has no .replace: the reference's ImportError, raised now)
                infoStr = result["info"].replace("\\x2c", ",")
                result["info"] = _LazyInfo(infoStr)
        except IndexError:
            raise IndexError("The number of fields in the VCF entry do not match number expected "
                             "from provided VCF Header")
        except Exception as err:
            raise ImportError(f"Unable to parse VCF entry: {inputStr}; ERROR: {str(err)}")
        return result

    def update_chromosome(self, chrmMap):
        self.__verify_entry()
        if chrmMap is not None:
            self.__entry["chrom"] = chrmMap.get(self.__entry["chrom"])

    def get_variant(self, dbSNP=False, namespace=False):
        """vcf_parser.py:127-155"""
        chrom = _xstr(self.get("chrom"))
        if chrom == "MT":
            chrom = "M"
        altAlleles = self.get("alt").split(",")
        vid = self.get("id")
        if vid == "." or vid.startswith("rs"):
            vid = ":".join((chrom.replace("chr", ""), _xstr(self.get("pos")), self.get("ref"), self.get("alt")))
        variant = {
            "id": vid,
            "ref_snp_id": self.get_refsnp(),
            "ref_allele": self.get("ref"),
            "alt_alleles": altAlleles,
            "is_multi_allelic": len(altAlleles) > 1,
            "chromosome": _xstr(chrom).replace("chr", ""),
            "position": int(self.get("pos")),
            "rs_position": self.get_info("RSPOS"),
        }
        return SimpleNamespace(**variant) if namespace else variant

    def get_refsnp(self):
        """vcf_parser.py:158-169"""
        self.__verify_entry()
        if "rs" in self.__entry["id"]:
            return self.__entry["id"]
        if "info" in self.__entry:
            rs = self._info_value("RS")
            if rs is not _MISSING:
                return "rs" + str(rs)
        return None

    def _info_value(self, key):
        """One coerced INFO value (or _MISSING) without coercing the whole dict."""
        info = self.__entry["info"]
        if isinstance(info, _LazyInfo):
            raw = self.__raw_info
            if raw is None:
                raw = self.__raw_info = info.raw()
            v = raw.get(key, _MISSING)
            return to_numeric(v) if v.__class__ is str else v
        return info.get(key, _MISSING)

    def _info(self) -> dict:
        info = self.__entry["info"]
        if isinstance(info, _LazyInfo):
            info = self.__entry["info"] = info.resolve()
        return info

    def get_entry(self):
        if self.__entry is not None and "info" in self.__entry:
            self._info()
        return self.__entry

    def get(self, key, raiseError=True):
        self.__verify_entry()
        try:
            if key == "info" and "info" in self.__entry:
                return self._info()
            return self.__entry[key]
        except KeyError as err:
            if raiseError:
                raise err
            return None

    def get_info(self, key, default=None):
        self.__verify_entry()
        if "info" not in self.__entry:
            return None
        v = self._info_value(key)
        return default if v is _MISSING else v

    def get_frequencies(self, allele):
        """vcf_parser.py:195-222 (INFO FREQ)."""
        vcfGMAFs = self.get_info("FREQ")
        if vcfGMAFs is None:
            return None
        zeroValues = [".", "0"]
        altAlleles = self.get("alt").split(",")
        altIndex = altAlleles.index(allele) + 1
        populationFrequencies = {pop.split(":")[0]: pop.split(":")[1] for pop in vcfGMAFs.split("|")}
        vcfFreqs = {pop: {"gmaf": to_numeric(freq.split(",")[altIndex])}
                    for pop, freq in populationFrequencies.items()
                    if freq.split(",")[altIndex] not in zeroValues}
        return None if len(vcfFreqs) == 0 else vcfFreqs

    def infer_variant_end_location(self, alt):
        """vcf_parser.py:225-231 (GPU-backed VariantAnnotator)."""
        annotator = VariantAnnotator(self.get("ref"), alt, self.get("chrom"), int(self.get("pos")))
        return annotator.infer_variant_end_location()

    def __verify_entry(self):
        assert self.__entry is not None, \
            "DEBUG - must set value of _entry in the VCF parser before attempting to access"


class ChromosomeMap(object):
    """Drop-in for ``ChromosomeMap`` (Util/lib/python/parsers/chromosome_map_parser.py:
    27-91): a tab-delimited file with ``source_id`` and ``chromosome`` columns
    (e.g. RefSeq accession -> chromosome); values lose their ``chr``.  ``get``
    raises ``KeyError`` for an unknown id, as the reference's dict lookup does.
    The loaders hand ``chromosome_map()`` to the K0 tokenizer / K5h (an
    ``avdb_chrom_map`` table) instead of calling ``get`` per line."""

    def __init__(self, fileName, verbose=False, debug=False):
        self._verbose = verbose
        self._debug = debug
        self._fileName = fileName
        with open(fileName, "r") as fh:
            self._map = {row["source_id"]: row["chromosome"].replace("chr", "")
                         for row in csv.DictReader(fh, delimiter="\t")}

    def chromosome_map(self):
        return self._map

    def get_sequence_id(self, chrmNum):
        """The first source id mapped to ``chrmNum`` (or 'chr' + it), else None."""
        for sequenceId, cn in self._map.items():
            if cn == chrmNum or cn == "chr" + _xstr(chrmNum):
                return sequenceId
        return None

    def get(self, sequenceId):
        return self._map[sequenceId]
