"""Chromosome universe and assembly length tables.

The reference recognises 25 contigs ``chr1..chr22, chrX, chrY, chrM``
(``Util/lib/python/enums/chromosomes.py:9-38``; partition list in
``Load/lib/sql/annotatedvdb_schema/tables/createVariant.sql:29-50``).  Inside
this package a contig is a ``u8`` index into that list, in exactly that order.

Chromosome lengths only reach the reference through the ``BinIndexRef`` table
that ``BinIndex/bin/generate_bin_index_references.py:17-25,86-106`` builds from a
``chrom<TAB>length`` map.  Only an hg19 map ships
(``Load/data/hg19_chr_map.txt``); GRCh38 lengths (UCSC hg38 primary assembly)
are an input assumption, recorded in SURVEY.md Appendix B.  Lengths only matter
for end-of-chromosome clipping (``generate_bin_index_references.py:62-65``).
"""

from __future__ import annotations

from typing import Dict, List, Sequence

# order == u8 chromosome code (0..24)
CHROM_NAMES: List[str] = [str(i) for i in range(1, 23)] + ["X", "Y", "M"]
N_CHROM = len(CHROM_NAMES)

GRCH38_LENGTHS: Dict[str, int] = {
    "1": 248956422, "2": 242193529, "3": 198295559, "4": 190214555,
    "5": 181538259, "6": 170805979, "7": 159345973, "8": 145138636,
    "9": 138394717, "10": 133797422, "11": 135086622, "12": 133275309,
    "13": 114364328, "14": 107043718, "15": 101991189, "16": 90338345,
    "17": 83257441, "18": 80373285, "19": 58617616, "20": 64444167,
    "21": 46709983, "22": 50818468, "X": 156040895, "Y": 57227415,
    "M": 16569,
}

# hg19 as shipped in the reference (Load/data/hg19_chr_map.txt:1-25)
GRCH37_LENGTHS: Dict[str, int] = {
    "1": 249250621, "2": 243199373, "3": 198022430, "4": 191154276,
    "5": 180915260, "6": 171115067, "7": 159138663, "8": 146364022,
    "9": 141213431, "10": 135534747, "11": 135006516, "12": 133851895,
    "13": 115169878, "14": 107349540, "15": 102531392, "16": 90354753,
    "17": 81195210, "18": 78077248, "19": 59128983, "20": 63025520,
    "21": 48129895, "22": 51304566, "X": 155270560, "Y": 59373566,
    "M": 16569,
}

ASSEMBLIES = {"GRCh38": GRCH38_LENGTHS, "GRCh37": GRCH37_LENGTHS,
              "hg38": GRCH38_LENGTHS, "hg19": GRCH37_LENGTHS}

_CODE = {name: i for i, name in enumerate(CHROM_NAMES)}
UNKNOWN_CHROM = 255


def chrom_code(name) -> int:
    """Map a chromosome label to its u8 code, or ``UNKNOWN_CHROM``.

    Accepts ``'1'``, ``1``, ``'chr1'``, ``'MT'``/``'chrMT'`` (the VCF parser maps
    ``MT``→``M`` at ``Util/lib/python/parsers/vcf_parser.py:136-137`` and strips
    ``chr`` at :150; ``find_bin_index`` prepends ``chr`` when absent,
    ``BinIndex/lib/python/bin_index.py:64``).
    """
    s = str(name)
    if s.startswith("chr"):
        s = s[3:]
    if s == "MT":
        s = "M"
    return _CODE.get(s, UNKNOWN_CHROM)


def bin_index_chrom_code(chrm) -> int:
    """Chromosome code exactly as ``BinIndex.find_bin_index`` resolves it.

    ``bin_index.py:64`` prepends ``'chr'`` when the substring ``'chr'`` is absent,
    and the SQL then matches ``BinIndexRef.chromosome`` literally — so ``'MT'``
    (→ ``'chrMT'``) is *not* ``chrM`` there and maps to nothing.
    """
    s = str(chrm)
    if "chr" not in s:
        s = "chr" + s
    if not s.startswith("chr"):
        return UNKNOWN_CHROM
    return _CODE.get(s[3:], UNKNOWN_CHROM)


def length_table(assembly="GRCh38", lengths: Dict[str, int] | None = None) -> List[int]:
    """Per-code chromosome lengths (``u32`` list of ``N_CHROM``)."""
    table = lengths if lengths is not None else ASSEMBLIES[assembly]
    return [int(table[n]) for n in CHROM_NAMES]


def read_chr_map(path: str) -> Dict[str, int]:
    """Read a ``chrom<TAB>length`` map (the generator's input format,
    ``generate_bin_index_references.py:17-25``)."""
    out: Dict[str, int] = {}
    with open(path) as fh:
        for line in fh:
            line = line.rstrip()
            if not line:
                continue
            chrom, length = line.split("\t")
            c = chrom[3:] if chrom.startswith("chr") else chrom
            out["M" if c == "MT" else c] = int(length)
    return out


def chrom_label(code: int) -> str:
    return "chr" + CHROM_NAMES[code]


def names_to_codes(names: Sequence) -> List[int]:
    return [chrom_code(n) for n in names]
