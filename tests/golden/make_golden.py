#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE's own Python code.

Runs only in the build container (``/root/reference`` does not exist on the
GPU box); its outputs are the committed fixtures under ``tests/golden/``.
Nothing from the reference is copied: its modules are imported in place from
``/root/reference`` and executed verbatim.  Absent third-party dependencies
(GenomicsDBData, niagads, psycopg2, ga4gh vrs-python, pysam) are replaced by
minimal stand-ins.  Only ``xstr(str|int)`` and
``convert_str2numeric_values`` influence pinned outputs; both are mapped to
their published behaviour (``str()``; int/float coercion of numeric strings).

The SQL function ``find_bin_index(chr,start,end)`` lives in the external
GenomicsDBData project.  The fake cursor answers ``BIN_INDEX_SQL``
(``BinIndex/lib/python/bin_index.py:9-14``) by a *table search* over the
``BinIndexRef`` rows produced by running the reference generator
(``BinIndex/bin/generate_bin_index_references.py:28-83``) verbatim: the deepest
row whose ``(lo,hi]`` contains both ``start`` and ``end`` — the convention the
reference's own cache test pins (``bin_index.py:70``).  No closed form is used
here, so the fixtures are independent of the restatement under ``oracle/``.

Outputs (all small, gzip):
  binindexref_summary.json    per-chrom/per-level row counts + sha256 of rows
  binindexref_chrM_chr21.tsv.gz  full rows for two chromosomes
  bin_queries.tsv.gz          (chrom, start, end) -> path | TypeError
  end_infer.tsv.gz            (pos, ref, alt) -> lcp, end  (VariantAnnotator)
  vcf_lines.tsv.gz            VCF line -> parse_variant mapping + COPY prefix
  long_alleles.tsv.gz         long-allele records -> end + bin (PK unpinned)
  kat.json                    known-answer tests
  c1_prefix.tsv.gz            BASELINE config C1 (annotatedvdb_amd.synth.np_c1, seed 1):
                              the first 100,000 records -> end, bin path, primary key
  bin_queries_wide.tsv.gz     (round 6, --only scale) 200,000 queries in random order over
                              all 25 contigs (half uniform over contigs), spans to 1 Mb
  bin_sequence.tsv.gz         (round 6, --only scale) ~100,000 queries in loader order
                              through ONE BinIndex: walks along every contig, so its
                              one-bin L13 cache (bin_index.py:66-71) serves most of them,
                              with end < start records (AT/AT -> pos - 1) after
                              cache hits, broad spans that leave a non-leaf bin cached,
                              unmappable queries that leave no bin cached
  vcf_lines_100k.tsv.gz       (round 6, --only scale) 100,000 more VCF lines, as vcf_lines
  adsp_load.tsv.gz            the load driver with VCFVariantLoader('ADSP') and
  adsp_existing.json          --skipExisting over a stub validator answering from
                              adsp_existing.json: per line COPY rows (is_adsp_variant
                              column), .mapping, is_adsp_variant updates, counters

Usage:  python tests/golden/make_golden.py [--quick] [--only all|load|c1|adsp|chrmap|scale]
"""

from __future__ import annotations

import argparse
import bisect
import gzip
import hashlib
import importlib.util
import io
import json
import os
import random
import sys
import types

sys.dont_write_bytecode = True  # /root/reference is writable: leave no __pycache__

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from annotatedvdb_amd.chromosomes import CHROM_NAMES, GRCH38_LENGTHS  # noqa: E402

# --------------------------------------------------------------------------
# stand-ins for absent dependencies
# --------------------------------------------------------------------------


def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def _xstr(value, nullStr="", falseAsNull=False):
    if value is None:
        return nullStr
    if falseAsNull and value is False:
        return nullStr
    if isinstance(value, (dict, list)):
        return json.dumps(value)
    return str(value)


def _to_numeric(value):
    try:
        return int(value)
    except (ValueError, TypeError):
        try:
            return float(value)
        except (ValueError, TypeError):
            return value


def _convert_str2numeric_values(d):
    return {k: (_to_numeric(v) if isinstance(v, str) else v) for k, v in d.items()}


def _warning(*args, **kw):
    pass


def _die(*args):
    raise SystemExit(" ".join(str(a) for a in args))


class NumericRange:
    """psycopg2.extras.NumericRange containment semantics."""

    def __init__(self, lower=None, upper=None, bounds="[)", empty=False):
        self.lower, self.upper, self._bounds = lower, upper, bounds

    def __contains__(self, x):
        if self.lower is not None:
            if self._bounds[0] == "[":
                if x < self.lower:
                    return False
            elif x <= self.lower:
                return False
        if self.upper is not None:
            if self._bounds[1] == "]":
                if x > self.upper:
                    return False
            elif x >= self.upper:
                return False
        return True

    def __repr__(self):
        return f"NumericRange({self.lower}, {self.upper}, '{self._bounds}')"


class ProgrammingError(Exception):
    pass


class DatabaseError(Exception):
    pass


class BinTable:
    """BinIndexRef rows, searched the way an index scan would: per level, the
    row whose (lo,hi] holds ``start``; answer = deepest one that also holds
    ``end``."""

    def __init__(self):
        self.rows = []  # (chrom, level, global_bin, path, lo, hi)
        self.by = {}

    def add(self, chrom, level, gbin, path, rng):
        self.rows.append((chrom, level, gbin, path, rng.lower, rng.upper))

    def finalize(self):
        by = {}
        for r in self.rows:
            by.setdefault((r[0], r[1]), []).append(r)
        self.by = {}
        for k, lst in by.items():
            lst.sort(key=lambda r: r[4])
            self.by[k] = ([r[4] for r in lst], lst)

    def find(self, chrom, start, end):
        for level in range(13, -1, -1):
            ent = self.by.get((chrom, level))
            if ent is None:
                continue
            los, lst = ent
            k = bisect.bisect_left(los, start) - 1  # last lo < start
            if k < 0:
                continue
            r = lst[k]
            if r[4] < start <= r[5] and r[4] < end <= r[5]:
                return r
        return None


TABLE = BinTable()


class FakeCursor:
    def __init__(self):
        self._res = None

    def execute(self, sql, params=None):
        if "find_bin_index" not in sql:
            self._res = None
            return
        chrm, start, end = params
        r = TABLE.find(chrm, start, end)
        if r is None:
            self._res = None
        else:
            self._res = {"chromosome": r[0], "global_bin_path": r[3],
                         "location": NumericRange(r[4], r[5], "(]"),
                         "bin_level": 1 + 2 * r[1]}

    def fetchone(self):
        return self._res

    def close(self):
        pass


class FakeDatabase:
    def __init__(self, *a, **kw):
        pass

    def connect(self):
        pass

    def cursor(self, *a, **kw):
        return FakeCursor()

    def close(self):
        pass

    def commit(self):
        pass

    def rollback(self):
        pass


def install_stubs():
    utils = dict(xstr=_xstr, warning=_warning, die=_die,
                 truncate=lambda s, n: s if len(s) <= n else s[:n] + "...",
                 reverse=lambda s: s[::-1],
                 print_dict=lambda d, pretty=False: json.dumps(d, default=str),
                 print_args=lambda a, pretty=True: str(a),
                 to_numeric=_to_numeric, deep_update=lambda a, b: a.update(b) or a,
                 convert_str2numeric_values=_convert_str2numeric_values,
                 int_to_alpha=lambda i: str(i), verify_path=os.path.exists)
    _mod("GenomicsDBData")
    _mod("GenomicsDBData.Util")
    _mod("GenomicsDBData.Util.utils", **utils)
    _mod("GenomicsDBData.Util.list_utils",
         qw=lambda s, returnTuple=False: tuple(s.split()) if returnTuple else s.split(),
         is_subset=lambda a, b: set(a) <= set(b),
         is_equivalent_list=lambda a, b: sorted(a) == sorted(b))
    _mod("GenomicsDBData.Util.auto_viv_dict", AutoVivificationDict=dict)
    _mod("GenomicsDBData.Util.postgres_dbi", Database=FakeDatabase,
         raise_pg_exception=lambda e, returnError=False: (_ for _ in ()).throw(e))
    _mod("niagads")
    _mod("niagads.db")
    _mod("niagads.db.postgres", Database=FakeDatabase,
         raise_pg_exception=lambda e, returnError=False: None)
    _mod("niagads.utils")
    _mod("niagads.utils.string", xstr=_xstr)
    _mod("psycopg2", DatabaseError=DatabaseError, ProgrammingError=ProgrammingError)
    _mod("psycopg2.extras", NumericRange=NumericRange, execute_values=lambda *a, **k: None)

    class _NoVRS:
        def __init__(self, *a, **k):
            self.normalize = False

        def _from_gnomad(self, *a, **k):
            raise ValueError("vrs-python / SeqRepo not available (parity unpinned)")

    _mod("ga4gh")
    _mod("ga4gh.core", ga4gh_identify=lambda x: None, ga4gh_serialize=lambda x: b"")
    _mod("ga4gh.vrs")
    _mod("ga4gh.vrs.extras")
    _mod("ga4gh.vrs.extras.translator", Translator=_NoVRS)
    _mod("ga4gh.vrs.dataproxy", create_dataproxy=lambda uri: None)
    _mod("pysam")

    # package layout: AnnotatedVDB.{Util,BinIndex} -> reference lib dirs
    pkg = _mod("AnnotatedVDB")
    pkg.__path__ = []
    u = _mod("AnnotatedVDB.Util")
    u.__path__ = [os.path.join(REF, "Util/lib/python")]
    b = _mod("AnnotatedVDB.BinIndex")
    b.__path__ = [os.path.join(REF, "BinIndex/lib/python")]
    # database/__init__.py ships empty but loaders import names from it
    _mod("AnnotatedVDB.Util.database", VariantRecord=object,
         VARIANT_ID_TYPES=["REFSNP", "METASEQ", "PRIMARY_KEY"]).__path__ = [
        os.path.join(REF, "Util/lib/python/database")]


# --------------------------------------------------------------------------
# BinIndexRef via the reference generator
# --------------------------------------------------------------------------


def build_binindexref():
    path = os.path.join(REF, "BinIndex/bin/generate_bin_index_references.py")
    spec = importlib.util.spec_from_file_location("avdb_ref_generate_bins", path)
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)  # __name__ != "__main__": main block not run

    class _ChrMap(dict):
        def iteritems(self):  # py2 call at generate_bin_index_references.py:30
            return iter(self.items())

    class _Cur:
        def execute(self, sql, params):
            chrom, level, gbin, bpath, rng = params
            TABLE.add(chrom, level, gbin, bpath, rng)

    gen.increments = [-1, 64000000, 32000000, 16000000, 8000000, 4000000, 2000000,
                      1000000, 500000, 250000, 125000, 62500, 31250, 15625]
    gen.numLevels = len(gen.increments)
    gen.binCount = 0
    gen.insertSql = "INSERT"
    gen.cursor = _Cur()
    gen.database = FakeDatabase()
    gen.args = types.SimpleNamespace(commit=False)
    gen.chrMap = _ChrMap(("chr" + c, GRCH38_LENGTHS[c]) for c in CHROM_NAMES)
    gen.load_bins()
    TABLE.finalize()


# --------------------------------------------------------------------------
# fixture writers
# --------------------------------------------------------------------------


def wtsv(name, header, rows):
    p = os.path.join(HERE, name)
    with gzip.open(p, "wt", compresslevel=9) as fh:
        fh.write("\t".join(header) + "\n")
        for r in rows:
            fh.write("\t".join(str(x) for x in r) + "\n")
    print(f"wrote {p} ({len(rows)} rows, {os.path.getsize(p)} B)")


def summary():
    counts = {}
    h = hashlib.sha256()
    for r in TABLE.rows:
        counts.setdefault(r[0], [0] * 14)[r[1]] += 1
        h.update(("\t".join(str(x) for x in r) + "\n").encode())
    out = {"assembly": "GRCh38", "n_rows": len(TABLE.rows),
           "n_leaves": sum(v[13] for v in counts.values()),
           "rows_sha256": h.hexdigest(),
           "row_format": "chromosome\\tlevel\\tglobal_bin\\tglobal_bin_path\\tlo\\thi  (location=(lo,hi]) in generation order",
           "per_chrom_level_counts": counts,
           "lengths": {("chr" + c): GRCH38_LENGTHS[c] for c in CHROM_NAMES}}
    p = os.path.join(HERE, "binindexref_summary.json")
    with open(p, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"wrote {p}: {out['n_rows']} rows, {out['n_leaves']} leaves")
    wtsv("binindexref_chrM_chr21.tsv.gz",
         ["chromosome", "level", "global_bin", "global_bin_path", "lo", "hi"],
         [r for r in TABLE.rows if r[0] in ("chrM", "chr21")])


def boundary_positions(L, rng):
    ps = {1, 2, L, L - 1}
    for lvl in range(1, 14):
        inc = 64000000 >> (lvl - 1)
        k = rng.randrange(0, max(1, L // inc) + 1)
        b = k * inc
        for d in (-1, 0, 1, 2):
            if 1 <= b + d <= L:
                ps.add(b + d)
    return sorted(ps)


def gen_bin_queries(bi, n, rng):
    """(chrom,start,end) -> verbatim BinIndex.find_bin_index answer."""
    qs = []
    tot = sum(GRCH38_LENGTHS.values())
    weights = [GRCH38_LENGTHS[c] / tot for c in CHROM_NAMES]
    for _ in range(n):
        c = rng.choices(CHROM_NAMES, weights)[0]
        L = GRCH38_LENGTHS[c]
        u = rng.random()
        s = rng.randint(1, L)
        if u < 0.4:
            e = None  # SNV, end defaults to start (bin_index.py:63)
        elif u < 0.7:
            e = min(L, s + int(rng.expovariate(1 / 8)))
        else:
            e = min(L, s + int(10 ** rng.uniform(1.7, 6)))
        qs.append((c, s, e))
    # boundaries on every chromosome
    for c in CHROM_NAMES:
        L = GRCH38_LENGTHS[c]
        ps = boundary_positions(L, rng)
        for p in ps:
            qs.append((c, p, None))
            for q in ps:
                if q >= p and rng.random() < 0.15:
                    qs.append((c, p, q))
        # whole-chromosome and just-inside spans
        qs += [(c, 1, L), (c, 1, 1), (c, L, L), (c, 64000000 if L > 64000000 else 1, L)]
    # unmappable: past end, start 0, unknown contigs, 'MT' (→ 'chrMT')
    for c in CHROM_NAMES:
        L = GRCH38_LENGTHS[c]
        qs += [(c, L + 1, None), (c, L, L + 1), (c, 0, 5)]
    qs += [("Un", 100, None), ("MT", 100, None), ("chr23", 5, 5), ("chrX", 1000, 1000)]
    # ordering: half sorted (exercises the one-bin cache), half as generated
    half = len(qs) // 2
    srt = sorted(qs[:half], key=lambda q: (CHROM_NAMES.index(q[0]) if q[0] in CHROM_NAMES else 99, q[1]))
    qs = srt + qs[half:]
    rows = []
    for c, s, e in qs:
        try:
            ans = bi.find_bin_index(c, s, e)
        except TypeError:
            ans = "TypeError"
        rows.append((c, s, "" if e is None else e, ans))
    return rows


def gen_bin_queries_wide(bi, n, rng):
    """n queries in random order (so the one-bin cache rarely serves one: the
    table-search answers) over all 25 contigs — half drawn uniformly over the
    contigs, so chrM / chrY / chr21 get as many as chr1, half by length — with
    35 % points, 25 % geometric(1/8) spans, 40 % log-uniform spans up to 1 Mb
    (some running past the contig end: TypeError rows)."""
    tot = sum(GRCH38_LENGTHS.values())
    weights = [GRCH38_LENGTHS[c] / tot for c in CHROM_NAMES]
    rows = []
    for _ in range(n):
        c = rng.choice(CHROM_NAMES) if rng.random() < 0.5 else rng.choices(CHROM_NAMES, weights)[0]
        L = GRCH38_LENGTHS[c]
        s = rng.randint(1, L)
        u = rng.random()
        if u < 0.35:
            e = None
        elif u < 0.6:
            e = min(L, s + int(rng.expovariate(1 / 8)))
        else:
            e = s + int(10 ** rng.uniform(0, 6))
        name = c if rng.random() < 0.7 else "chr" + c
        try:
            ans = bi.find_bin_index(name, s, e)
        except TypeError:
            ans = "TypeError"
        rows.append((name, s, "" if e is None else e, ans))
    return rows


def gen_bin_sequence(bi, n, rng):
    """About n queries in the order a position-sorted load makes them, all through
    the one BinIndex ``bi`` (its cache state carries from query to query, as in
    vcf_variant_loader.py:310-311).  Every contig is walked from a random start in
    steps of mean ~2 kb, so most queries fall in the L13 leaf (15,625 bp) the
    previous one cached.  Per query: 58 % points, 14 % short spans, 5 % broad
    spans (log-uniform to 1 Mb: a non-leaf bin is then cached and the next query
    misses), 12 % end = start - 1 (identical ref/alt, SURVEY A.3 — served from the
    cached leaf when both ends are inside it, otherwise the SQL lookup of the
    swapped pair), 4 % end = start - k (k up to 40,000), 3 % positions on a leaf
    boundary, 2 % unmappable (past the end, start 0, 'MT', unknown contigs: the
    cache is then empty), 2 % a jump back to an earlier position."""
    tot = sum(GRCH38_LENGTHS.values())
    per = {c: max(200, int(n * 0.5 / 25 + n * 0.5 * GRCH38_LENGTHS[c] / tot)) for c in CHROM_NAMES}
    rows = []
    for c in CHROM_NAMES:
        L = GRCH38_LENGTHS[c]
        p = rng.randint(1, max(1, L // 3))
        name = c if rng.random() < 0.5 else "chr" + c
        for _ in range(per[c]):
            p += int(rng.expovariate(1 / 2000))
            if p > L:
                p = rng.randint(1, L)
            u = rng.random()
            s, e, nm = p, None, name
            if u < 0.58:
                pass
            elif u < 0.72:
                e = min(L, p + int(rng.expovariate(1 / 8)))
            elif u < 0.77:
                e = min(L, p + int(10 ** rng.uniform(4.2, 6)))
            elif u < 0.89:
                e = p - 1
            elif u < 0.93:
                e = max(0, p - rng.randint(2, 40000))
            elif u < 0.96:
                b = (p // 15625) * 15625
                s = max(1, b + rng.choice((0, 1, 2)))
                e = rng.choice((None, s - 1, s + 1, b + 15625))
                if e is not None:
                    e = min(L, max(0, e))
            elif u < 0.98:
                k = rng.randrange(5)
                s, e, nm = [(L + 1, None, name), (0, 5, name), (p, p, "MT"), (p, None, "Un"),
                            (p, L + 1, name)][k]
            else:
                s = max(1, p - rng.randint(1, 200000))
                e = None if rng.random() < 0.5 else s + rng.randint(0, 20)
            try:
                ans = bi.find_bin_index(nm, s, e)
            except TypeError:
                ans = "TypeError"
            rows.append((nm, s, "" if e is None else e, ans))
    return rows


ALPH = "ACGT"


def rand_allele(rng, n, alph=ALPH):
    return "".join(rng.choice(alph) for _ in range(n))


def gen_allele_pair(rng):
    """Adversarial ref/alt pairs: shared prefixes, palindromes, equal alleles,
    symbolic alleles."""
    u = rng.random()
    if u < 0.25:
        return rand_allele(rng, 1), rand_allele(rng, 1)
    if u < 0.45:  # insertion/deletion sharing an anchor/prefix
        p = rand_allele(rng, rng.randint(1, 6))
        return p + rand_allele(rng, rng.randint(0, 6)), p + rand_allele(rng, rng.randint(0, 6))
    if u < 0.6:  # MNV / same length
        n = rng.randint(2, 8)
        a = rand_allele(rng, n, "AC" if rng.random() < 0.5 else ALPH)
        b = rand_allele(rng, n, "AC" if rng.random() < 0.5 else ALPH)
        return a, b
    if u < 0.7:  # inversion
        a = rand_allele(rng, rng.randint(2, 9), "AT")
        return a, a[::-1]
    if u < 0.75:  # identical alleles (AT/AT quirk)
        a = rand_allele(rng, rng.randint(1, 5))
        return a, a
    if u < 0.8:
        return rand_allele(rng, 1), rng.choice(["<DEL>", "<INS>", "*", "<DUP:TANDEM>", "N"])
    n1, n2 = rng.randint(1, 25), rng.randint(1, 25)
    return rand_allele(rng, n1, "AC"), rand_allele(rng, n2, "AC")


def gen_end_infer(VariantAnnotator, n, rng):
    rows = []
    for _ in range(n):
        ref, alt = gen_allele_pair(rng)
        pos = rng.randint(1, 248956422)
        va = VariantAnnotator(ref, alt, "1", pos)
        nref, nalt = va.get_normalized_alleles()
        end = va.infer_variant_end_location()
        lcp = len(ref) - len(nref)
        assert len(alt) - len(nalt) == lcp
        rows.append((pos, ref, alt, lcp, end, va.get_metaseq_id()))
    return rows


def gen_vcf_lines(n, rng, long_frac=0.0):
    lines = []
    tot = sum(GRCH38_LENGTHS.values())
    weights = [GRCH38_LENGTHS[c] / tot for c in CHROM_NAMES]
    recs = []
    for _ in range(n):
        c = rng.choices(CHROM_NAMES, weights)[0]
        L = GRCH38_LENGTHS[c]
        pos = rng.randint(1, max(1, L - 3000))
        recs.append((c, pos))
    recs.sort(key=lambda r: (CHROM_NAMES.index(r[0]), r[1]))
    for c, pos in recs:
        nalt = 1 if rng.random() < 0.85 else rng.randint(2, 4)
        ref, alt0 = gen_allele_pair(rng)
        alts = [alt0] + [gen_allele_pair(rng)[1] for _ in range(nalt - 1)]
        if rng.random() < 0.01:
            alts = ["."]
        if rng.random() < long_frac:
            ref = rand_allele(rng, rng.randint(40, 400))
            alts = [ref[0]] if rng.random() < 0.5 else [ref[0] + rand_allele(rng, rng.randint(50, 300))]
        u = rng.random()
        vid = ("rs%d" % rng.randint(1, 10**9)) if u < 0.5 else ("." if u < 0.8 else "id%d" % rng.randint(1, 999))
        info = []
        if rng.random() < 0.4:
            info.append("RS=%d" % rng.randint(1, 10**9))
        if rng.random() < 0.3:
            info.append("RSPOS=%d" % pos)
        info.append("VC=SNV" if rng.random() < 0.5 else "dbSNPBuildID=151")
        cs = rng.choice([c, "chr" + c]) if c != "M" else rng.choice(["M", "MT", "chrM"])
        lines.append("\t".join([cs, str(pos), vid, ref, ",".join(alts), ".", ".", ";".join(info)]))
    # duplicate lines (in-batch dedup fixtures)
    for i in range(0, len(lines), 50):
        lines.insert(i + 1, lines[i])
    return lines


def run_loader(lines):
    from AnnotatedVDB.Util.loaders import VCFVariantLoader
    loader = VCFVariantLoader("dbSNP")
    loader.initialize_pk_generator("GRCh38", "/nonexistent")
    loader.initialize_bin_indexer(None)
    loader._alg_invocation_id = "1"
    loader.initialize_copy_sql()
    from AnnotatedVDB.Util.parsers import VcfEntryParser
    rows = []
    for line in lines:
        loader.reset_copy_buffer()
        try:
            mapping = loader.parse_variant(line)
        except Exception as err:  # reference raises (e.g. ':' inside an allele)
            mapping = {"__error__": type(err).__name__}
        copy = loader.copy_buffer().getvalue().splitlines()
        # pinned COPY columns: chromosome, record_primary_key, position, metaseq_id, bin_index
        copy5 = ["#".join(r.split("#")[:5]) for r in copy]
        entry = VcfEntryParser(line)
        alts = entry.get("alt").split(",")
        ends = [entry.infer_variant_end_location(a) if a != "." else "" for a in alts]
        rows.append((line.replace("\t", "\\t"), json.dumps(mapping, separators=(",", ":")),
                     json.dumps(copy5, separators=(",", ":")), json.dumps(ends)))
    return rows


FREQ_VALUES = ["0.9990", "0.0010", "0", ".", "1", "0.0", "0.00001", "0.0001", "12.50", "5.", ".5",
               "007", "00", "0.5", "0.123456789012345", "0.1234567890123456", "1e-05", "-0.5", "nan",
               "0.9986", "0.001353", "0.01861", "0.0005901", "100.0", "1234567890123456789.5"]
POPS = ["GnomAD", "Korea1K", "dbGaP_PopFreq", "1000Genomes", "TOPMED", "ALSPAC", "TWINSUK"]


def gen_freq(rng, nalt):
    """An INFO FREQ value; mostly well-formed (one ref + one value per ALT),
    sometimes short (IndexError in the reference), duplicate populations, or
    pathological entries."""
    u = rng.random()
    pops = rng.sample(POPS, rng.randint(1, 4))
    if u < 0.03:
        pops.append(pops[0])  # duplicate population: dict keeps the last value
    items = []
    for p in pops:
        nv = nalt + 1 if rng.random() > 0.03 else nalt  # short list -> IndexError
        vals = [rng.choice(FREQ_VALUES) if rng.random() < 0.3 else "0.%04d" % rng.randint(0, 9999)
                for _ in range(nv)]
        items.append(p + ":" + ",".join(vals))
    v = "|".join(items)
    if rng.random() < 0.01:
        v = v.replace(":", "", 1)  # population without ':' -> IndexError
    return v


def gen_load_lines(n, rng):
    """VCF lines for the full load-driver output (COPY rows + .mapping line):
    dbSNP-like INFO with FREQ, every allele class, multi-allelic and repeated
    ALTs, symbolic alleles, refSNP from ID or INFO, short alleles (ref+alt <= 50,
    so every primary key is pinnable)."""
    tot = sum(GRCH38_LENGTHS.values())
    weights = [GRCH38_LENGTHS[c] / tot for c in CHROM_NAMES]
    recs = []
    for _ in range(n):
        c = rng.choices(CHROM_NAMES, weights)[0]
        L = GRCH38_LENGTHS[c]
        u = rng.random()
        pos = rng.randint(1, L) if u > 0.01 else rng.choice([1, 2, L, L - 1, 15625, 15626])
        recs.append((c, pos))
    recs.sort(key=lambda r: (CHROM_NAMES.index(r[0]), r[1]))
    lines = []
    for c, pos in recs:
        nalt = 1 if rng.random() < 0.85 else rng.randint(2, 4)
        ref, alt0 = gen_allele_pair(rng)
        alts = [alt0] + [gen_allele_pair(rng)[1] for _ in range(nalt - 1)]
        u = rng.random()
        if u < 0.02:
            alts = ["."]
        elif u < 0.04 and nalt > 1:
            alts[1] = alts[0]  # repeated ALT: altAlleles.index() finds the first
        elif u < 0.06:
            alts.append(".")
        elif u < 0.09:  # tandem duplications / repeats (dup vs ins display class)
            unit = rand_allele(rng, rng.randint(1, 4))
            ref = rand_allele(rng, 1) + unit * rng.randint(1, 4)
            alts = [ref + unit * rng.randint(1, 2)]
        elif u < 0.11:  # long-ish deletions / insertions (display truncation at 8)
            ref = rand_allele(rng, rng.randint(9, 30))
            alts = [ref[0]] if rng.random() < 0.5 else [ref + rand_allele(rng, rng.randint(1, 15))]
        alts = [a for a in alts if len(ref) + len(a) <= 50] or [ref[0] if ref else "A"]
        u = rng.random()
        vid = ("rs%d" % rng.randint(1, 10**9)) if u < 0.55 else ("." if u < 0.85 else "id%d" % rng.randint(1, 999))
        info = []
        if rng.random() < 0.4:
            info.append("RS=%d" % rng.randint(1, 10**9))
        info.append("dbSNPBuildID=151")
        if rng.random() < 0.7:
            info.append("FREQ=" + gen_freq(rng, len(alts)))
        elif rng.random() < 0.02:
            info.append("FREQ")
        if rng.random() < 0.3:
            info.append("VC=SNV")
        cs = rng.choice([c, "chr" + c]) if c != "M" else rng.choice(["M", "MT", "chrM"])
        lines.append("\t".join([cs, str(pos), vid, ref, ",".join(alts), ".", ".", ";".join(info)]))
    for i in range(0, len(lines), 40):  # adjacent duplicate lines
        lines.insert(i + 1, lines[i])
    return lines


def run_load_driver(lines):
    """Per line, what Load/bin/load_vcf_file.py:101-119 produces: the COPY
    buffer rows (all columns) and the .mapping line(s), or the exception type."""
    from AnnotatedVDB.Util.loaders import VCFVariantLoader
    loader = VCFVariantLoader("dbSNP")
    loader.initialize_pk_generator("GRCh38", "/nonexistent")
    loader.initialize_bin_indexer(None)
    loader._alg_invocation_id = "1"
    loader.initialize_copy_sql()
    rows = []
    for line in lines:
        loader.reset_copy_buffer()
        try:
            pkm = loader.parse_variant(line.rstrip())
            mapping = ["%s\t%s" % (k, v) for k, v in pkm.items()]  # print(k, v, sep='\t')
            err = ""
        except Exception as e:  # noqa: BLE001
            mapping, err = [], type(e).__name__
        copy = loader.copy_buffer().getvalue().splitlines()
        rows.append((line.replace("\t", "\\t"), err, json.dumps(mapping, separators=(",", ":")),
                     json.dumps(copy, separators=(",", ":"))))
    return rows


# RefSeq accessions of the GRCh38 primary assembly (NC_0000xx.yy; MT = NC_012920.1), the
# CHROM values of NCBI's own dbSNP VCFs: what chromosome maps translate
REFSEQ = {"1": "NC_000001.11", "2": "NC_000002.12", "3": "NC_000003.12", "4": "NC_000004.12",
          "5": "NC_000005.10", "6": "NC_000006.12", "7": "NC_000007.14", "8": "NC_000008.11",
          "9": "NC_000009.12", "10": "NC_000010.11", "11": "NC_000011.10", "12": "NC_000012.12",
          "13": "NC_000013.11", "14": "NC_000014.9", "15": "NC_000015.10", "16": "NC_000016.10",
          "17": "NC_000017.11", "18": "NC_000018.10", "19": "NC_000019.10", "20": "NC_000020.11",
          "21": "NC_000021.9", "22": "NC_000022.11", "X": "NC_000023.11", "Y": "NC_000024.10",
          "M": "NC_012920.1"}
PVCF_HEADER = ["#CHROM", "POS", "ID", "REF", "ALT", "QUAL", "FILTER", "INFO", "FORMAT", "S1"]


def write_chrmap(path):
    """A ChromosomeMap file (source_id, chromosome, chromosome_order_num, length):
    the 25 accessions -> chrN, plus entries the loader must get exactly right: a
    numeric source id (Python coerces that CHROM to int before the lookup:
    KeyError), an unplaced scaffold (-> chrUn..., no bin: TypeError), a value
    without 'chr' and an 'MT' value."""
    rows = [("source_id", "chromosome", "chromosome_order_num", "length")]
    for i, c in enumerate(CHROM_NAMES):
        rows.append((REFSEQ[c], "chr" + c, str(i + 1), str(GRCH38_LENGTHS[c])))
    rows += [("7", "chr7", "7", str(GRCH38_LENGTHS["7"])),
             ("NT_187361.1", "chrUn_KI270302v1", "26", "2274"),
             ("CM000685.2", "X", "23", str(GRCH38_LENGTHS["X"])),
             ("J01415.2", "MT", "25", "16569")]
    with open(path, "w") as fh:
        for r in rows:
            fh.write("\t".join(r) + "\n")


def gen_chrmap_lines(n, rng):
    """gen_load_lines' records with CHROM as an accession (most lines), a
    chromosome name (not in the map: KeyError), a numeric id that is in the map
    (KeyError), the scaffold, the 'X'/'MT' aliases; and pVCF columns (FORMAT +
    one sample; some lines short of the header: IndexError, some with extra)."""
    out = []
    alias = {"X": "CM000685.2", "M": "J01415.2"}
    for ln in gen_load_lines(n, rng):
        f = ln.split("\t")
        c = f[0].replace("chr", "")
        c = "M" if c == "MT" else c
        u = rng.random()
        if u < 0.85 or c not in REFSEQ:
            f[0] = REFSEQ.get(c, f[0])
        elif u < 0.89:
            f[0] = c  # a plain name: not a source id
        elif u < 0.92 and c in alias:
            f[0] = alias[c]
        elif u < 0.94:
            f[0] = "7"
        elif u < 0.96:
            f[0] = "NT_187361.1"
        else:
            f[0] = REFSEQ[c]
        u = rng.random()
        if u < 0.9:
            f += ["GT", rng.choice(["0/1", "1/1", "./."])]
        elif u < 0.95:
            f += ["GT", "0/1", "extra"]
        out.append("\t".join(f))
    return out


def run_chrmap_driver(lines, map_path):
    """run_load_driver with the loader's chromosome map and pVCF header set
    (VCFVariantLoader.set_chromosome_map / set_vcf_header_fields)."""
    from AnnotatedVDB.Util.loaders import VCFVariantLoader
    from AnnotatedVDB.Util.parsers.chromosome_map_parser import ChromosomeMap
    loader = VCFVariantLoader("dbSNP")
    loader.initialize_pk_generator("GRCh38", "/nonexistent")
    loader.initialize_bin_indexer(None)
    loader._alg_invocation_id = "1"
    loader.initialize_copy_sql()
    loader.set_chromosome_map(ChromosomeMap(map_path))
    loader.set_vcf_header_fields(PVCF_HEADER)
    rows = []
    for line in lines:
        loader.reset_copy_buffer()
        try:
            pkm = loader.parse_variant(line.rstrip())
            mapping = ["%s\t%s" % (k, v) for k, v in pkm.items()]
            err = ""
        except Exception as e:  # noqa: BLE001
            mapping, err = [], type(e).__name__
        copy = loader.copy_buffer().getvalue().splitlines()
        rows.append((line.replace("\t", "\\t"), err, json.dumps(mapping, separators=(",", ":")),
                     json.dumps(copy, separators=(",", ":"))))
    return rows


def gen_display_attrs(VariantAnnotator, n, rng):
    """(chrom, pos, ref, alt) -> json.dumps(get_display_attributes()) incl. long
    alleles (truncation at 8 and 100 characters)."""
    rows = []
    for i in range(n):
        u = rng.random()
        if u < 0.7:
            ref, alt = gen_allele_pair(rng)
        elif u < 0.8:
            unit = rand_allele(rng, rng.randint(1, 5))
            ref = rand_allele(rng, 1) + unit * rng.randint(1, 40)
            alt = ref + unit * rng.randint(1, 3) if rng.random() < 0.7 else ref[0] + unit
        elif u < 0.9:
            ref = rand_allele(rng, rng.randint(1, 250))
            alt = ref[:rng.randint(0, len(ref))] + rand_allele(rng, rng.randint(0, 250))
            if not alt:
                alt = "A"
        else:
            ref = rand_allele(rng, rng.randint(2, 150), "AT")
            alt = ref[::-1] if rng.random() < 0.5 else rand_allele(rng, len(ref), "AT")
        c = rng.choice(CHROM_NAMES)
        pos = rng.randint(1, GRCH38_LENGTHS[c])
        va = VariantAnnotator(ref, alt, c, pos)
        rows.append((c, pos, ref, alt, json.dumps(va.get_display_attributes())))
    return rows


def gen_long_alleles(VariantAnnotator, bi, n, rng):
    rows = []
    tot = sum(GRCH38_LENGTHS.values())
    weights = [GRCH38_LENGTHS[c] / tot for c in CHROM_NAMES]
    for _ in range(n):
        c = rng.choices(CHROM_NAMES, weights)[0]
        L = GRCH38_LENGTHS[c]
        pos = rng.randint(1, max(1, L - 5000))
        u = rng.random()
        if u < 0.4:
            ref = rand_allele(rng, rng.randint(51, 2000))
            alt = ref[0]
        elif u < 0.8:
            ref = rand_allele(rng, 1)
            alt = ref + rand_allele(rng, rng.randint(50, 2000))
        else:
            ref = rand_allele(rng, rng.randint(20, 600))
            alt = rand_allele(rng, rng.randint(31, 600))
        va = VariantAnnotator(ref, alt, c, pos)
        end = va.infer_variant_end_location()
        lcp = len(ref) - len(va.get_normalized_alleles()[0])
        try:
            b = bi.find_bin_index(c, pos, end)
        except TypeError:
            b = "TypeError"
        rows.append((c, pos, ref, alt, lcp, end, b))
    return rows


def gen_c1_prefix(VariantAnnotator, bi, n):
    """The C1 records (chr22; the generator the bench and the GPU
    tests use) through the reference's per-alt path (vcf_variant_loader.py:
    243-311): VariantAnnotator -> metaseq id, VariantPKGenerator.generate_primary_key
    (short path; every C1 allele pair has len(ref)+len(alt) <= 50), then
    infer_variant_end_location and BinIndex.find_bin_index(chrom, POS, end)."""
    from AnnotatedVDB.Util.primary_key_generator import VariantPKGenerator
    from annotatedvdb_amd import synth
    pkg = VariantPKGenerator("GRCh38", "/nonexistent")
    d = synth.np_c1(synth.C1_N, seed=1)
    heap = d["heap"].tobytes()
    rows = []
    for i in range(n):
        o, r, a = int(d["allele_off"][i]), int(d["ref_len"][i]), int(d["alt_len"][i])
        ref, alt = heap[o:o + r].decode(), heap[o + r:o + r + a].decode()
        pos = int(d["pos"][i])
        ext = int(d["ext_id"][i])
        va = VariantAnnotator(ref, alt, "22", pos)
        pk = pkg.generate_primary_key(va.get_metaseq_id(), "rs%d" % ext if ext else None)
        end = VariantAnnotator(ref, alt, "22", pos).infer_variant_end_location()
        try:
            b = bi.find_bin_index("22", pos, end)
        except TypeError:
            b = "TypeError"
        rows.append((pk, end, b))
    return rows


class StubVariantRecord:
    """Stands in for database.variant.VariantRecord (variant.py:287-309) over an
    in-memory export: ``exists(id)`` answers map_variants(id, firstHitOnly=True,
    checkAltVariants=True) (external SQL, unpinned) as: the metaseq-id table M
    (exact, then with the alleles switched), else the primary-key table P."""
    M = {}
    P = {}

    def __init__(self, *a, **k):
        pass

    def use_legacy_pk(self, flag):
        pass

    def close(self):
        pass

    def exists(self, variantId, returnMatch=False):
        m = self.M.get(variantId)
        if m is None:
            f = variantId.split(":")
            if len(f) == 4:
                m = self.M.get(":".join((f[0], f[1], f[3], f[2])))
        if m is None and variantId in self.P:
            m = [{"primary_key": variantId, "bin_index": self.P[variantId]}]
        if m is None:
            return None if returnMatch else False
        return m if returnMatch else True


def adsp_existing(lines, rng):
    """Existing rows for the ADSP fixture, derived from the input's own records:
    ~10 % of the alts by metaseq id (3 % of them with the alleles switched), and
    ~12 % of the alts that carry a refSNP id by primary key only (keys with an
    external id: 5 fields, never a metaseq id)."""
    from AnnotatedVDB.Util.parsers import VcfEntryParser
    from AnnotatedVDB.Util.primary_key_generator import VariantPKGenerator
    pkg = VariantPKGenerator("GRCh38", "/nonexistent")
    M, P = {}, {}
    for line in lines:
        try:
            v = VcfEntryParser(line).get_variant(namespace=True)
        except Exception:  # noqa: BLE001
            continue
        for alt in v.alt_alleles:
            if alt == ".":
                continue
            ms = ":".join((str(v.chromosome), str(v.position), v.ref_allele, alt))
            try:
                pk = pkg.generate_primary_key(ms, v.ref_snp_id)
            except Exception:  # noqa: BLE001
                continue
            u = rng.random()
            payload = [{"primary_key": pk, "bin_index": "chr%s.L1.B%d" % (v.chromosome, rng.randint(1, 4))}]
            if u < 0.07:
                M[ms] = payload
            elif u < 0.10:
                M[":".join((str(v.chromosome), str(v.position), alt, v.ref_allele))] = payload
            elif u < 0.22 and v.ref_snp_id is not None and len(pk.split(":")) == 5:
                P[pk] = "chr%s" % v.chromosome
    return M, P


def run_adsp_driver(lines, M, P):
    """Load/bin/load_vcf_file.py:101-119 with --datasource ADSP --skipExisting:
    per line the COPY rows, .mapping line(s) or exception type, the
    is_adsp_variant update values and the counter deltas."""
    import AnnotatedVDB.Util.loaders.variant_loader as VL
    from AnnotatedVDB.Util.loaders import VCFVariantLoader
    StubVariantRecord.M, StubVariantRecord.P = M, P
    VL.VariantRecord = StubVariantRecord
    loader = VCFVariantLoader("ADSP")
    loader.initialize_pk_generator("GRCh38", "/nonexistent")
    loader.initialize_bin_indexer(None)
    loader._alg_invocation_id = "1"
    loader.initialize_copy_sql()
    loader.set_skip_existing(True, None)
    keys = ("line", "variant", "skipped", "duplicates", "update")
    rows = []
    for line in lines:
        loader.reset_copy_buffer()
        loader.reset_update_buffer()
        before = [loader.get_count(k) for k in keys]
        try:
            pkm = loader.parse_variant(line.rstrip())
            mapping = ["%s\t%s" % (k, v) for k, v in pkm.items()]
            err = ""
        except Exception as e:  # noqa: BLE001
            mapping, err = [], type(e).__name__
        copy = loader.copy_buffer().getvalue().splitlines()
        upd = [list(x) for x in loader.update_buffer()]
        delta = [loader.get_count(k) - b for k, b in zip(keys, before)]
        rows.append((line.replace("\t", "\\t"), err, json.dumps(mapping, separators=(",", ":")),
                     json.dumps(copy, separators=(",", ":")), json.dumps(upd, separators=(",", ":")),
                     json.dumps(delta)))
    return rows


def kats(VariantAnnotator, bi):
    cases = [
        ("1", 1510801, "C", "T", None),
        ("13", 32936731, "G", "C", None),
        ("1", 148893911, "TGGCCAACA", "TAGCCAACG", "rs71261250"),
        ("22", 11212877, "TAAAATATCAAAGTACACCAAATACATATTATATACTGTACAC", "T", None),
        ("M", 11257, "C", "T", "rs377469212"),
        ("22", 16050115, "G", "A", None),
        ("22", 16050115, "G", "GT", None),
        ("1", 100, "AT", "AT", None),
        ("1", 100, "ATA", "ATA", None),
        ("1", 100, "A", "<DEL>", None),
        ("1", 100, "A", "*", None),
    ]
    out = []
    for c, pos, ref, alt, rs in cases:
        va = VariantAnnotator(ref, alt, c, pos)
        end = va.infer_variant_end_location()
        try:
            b = bi.find_bin_index(c, pos, end)
        except TypeError:
            b = None
        pk = None
        if len(ref) + len(alt) <= 50:
            pk = va.get_metaseq_id() + (":" + rs if rs else "")
        out.append({"chrom": c, "pos": pos, "ref": ref, "alt": alt, "rsid": rs,
                    "end": end, "bin_index": b, "metaseq_id": va.get_metaseq_id(),
                    "primary_key": pk})
    # in-repo KAT (GRCh37 DB): Util/lib/python/database/variant.py:162-163
    out.append({"source": "Util/lib/python/database/variant.py:162-163",
                "chrom": "1", "pos": 1510801, "ref": "C", "alt": "T",
                "bin_index_expected": "chr1.L1.B1.L2.B1.L3.B1.L4.B1.L5.B1.L6.B1.L7.B2.L8.B2.L9.B1.L10.B1.L11.B1.L12.B1.L13.B1"})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--only", choices=["all", "load", "c1", "adsp", "chrmap", "scale"], default="all",
                    help="'load': only the load-driver fixtures (vcf_load, display_attrs); "
                         "'c1': only the C1 prefix fixture")
    a = ap.parse_args()
    rng = random.Random(a.seed)
    install_stubs()
    build_binindexref()

    from AnnotatedVDB.BinIndex.bin_index import BinIndex
    from AnnotatedVDB.Util.variant_annotator import VariantAnnotator
    bi = BinIndex(None, verbose=False)

    k = 0.1 if a.quick else 1.0
    if a.only == "adsp":
        arng = random.Random(a.seed + 2)
        lines = gen_load_lines(int(3000 * k), arng)
        M, P = adsp_existing(lines, arng)
        with open(os.path.join(HERE, "adsp_existing.json"), "w") as fh:
            json.dump({"metaseq": M, "primary_key": P}, fh, separators=(",", ":"))
        wtsv("adsp_load.tsv.gz", ["line", "error", "mapping", "copy_rows", "updates", "counter_deltas"],
             run_adsp_driver(lines, M, P))
        print("existing: %d metaseq ids, %d primary keys" % (len(M), len(P)))
        print("done")
        return
    if a.only == "chrmap":
        mp = os.path.join(HERE, "chrmap_grch38.tsv")
        write_chrmap(mp)
        crng = random.Random(a.seed + 3)
        wtsv("chrmap_load.tsv.gz", ["line", "error", "mapping", "copy_rows"],
             run_chrmap_driver(gen_chrmap_lines(int(3000 * k), crng), mp))
        print("done")
        return
    if a.only == "scale":  # round 6: the section 7 volumes, their own seed stream
        srng = random.Random(a.seed + 6)
        wtsv("bin_queries_wide.tsv.gz", ["chrom", "start", "end", "bin_index"],
             gen_bin_queries_wide(BinIndex(None, verbose=False), int(200000 * k), srng))
        seq = gen_bin_sequence(BinIndex(None, verbose=False), int(100000 * k), srng)
        wtsv("bin_sequence.tsv.gz", ["chrom", "start", "end", "bin_index"], seq)
        lines = gen_vcf_lines(int(100000 * k), srng)
        lines = [ln for ln in lines if all(len(ln.split("\t")[3]) + len(x) <= 50
                                           for x in ln.split("\t")[4].split(","))]
        wtsv("vcf_lines_100k.tsv.gz", ["line", "mapping", "copy_prefix", "ends"], run_loader(lines))
        print("sequence: %d queries, %d end < start" % (
            len(seq), sum(1 for r in seq if r[2] != "" and int(r[2]) < int(r[1]))))
        print("done")
        return
    if a.only == "c1":
        wtsv("c1_prefix.tsv.gz", ["primary_key", "end", "bin_index"],
             gen_c1_prefix(VariantAnnotator, BinIndex(None, verbose=False), int(100000 * k)))
        print("done")
        return
    # load-driver fixtures: their own seed stream, so the older fixtures stay byte-identical
    lrng = random.Random(a.seed + 1)
    wtsv("vcf_load.tsv.gz", ["line", "error", "mapping", "copy_rows"],
         run_load_driver(gen_load_lines(int(4000 * k), lrng)))
    wtsv("display_attrs.tsv.gz", ["chrom", "pos", "ref", "alt", "attributes"],
         gen_display_attrs(VariantAnnotator, int(6000 * k), lrng))
    if a.only == "load":
        print("done")
        return
    summary()
    rows = gen_bin_queries(bi, int(30000 * k), rng)
    for r in rows[:3]:
        print(r)
    wtsv("bin_queries.tsv.gz", ["chrom", "start", "end", "bin_index"], rows)
    wtsv("end_infer.tsv.gz", ["pos", "ref", "alt", "lcp", "end", "metaseq_id"],
         gen_end_infer(VariantAnnotator, int(40000 * k), rng))
    wtsv("long_alleles.tsv.gz", ["chrom", "pos", "ref", "alt", "lcp", "end", "bin_index"],
         gen_long_alleles(VariantAnnotator, BinIndex(None, verbose=False), int(600 * k), rng))
    lines = gen_vcf_lines(int(8000 * k), rng)
    lines = [ln for ln in lines if all(len(ln.split("\t")[3]) + len(x) <= 50
                                       for x in ln.split("\t")[4].split(","))]
    wtsv("vcf_lines.tsv.gz", ["line", "mapping", "copy_prefix", "ends"], run_loader(lines))
    with open(os.path.join(HERE, "kat.json"), "w") as fh:
        json.dump(kats(VariantAnnotator, BinIndex(None, verbose=False)), fh, indent=1)
    print("done")


if __name__ == "__main__":
    main()
