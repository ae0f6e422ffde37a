"""Drop-in ``VCFVariantLoader`` record-prep stage
(``Util/lib/python/loaders/vcf_variant_loader.py:56-391`` and the parts of
``variant_loader.py:82-486`` it relies on).

``parse_variant(line)`` keeps the reference's contract — it returns
``{variant.id: [{'primary_key': pk, 'bin_index': path}, ...]}`` and appends one
``#``-delimited COPY row per alt allele (:320-343) — and ``parse_variants(lines)``
does the same for a whole batch with one pass of the GPU kernels:

    host   VCF text -> per-alt SoA (chrom u8, pos, REF/ALT heap, refSNP key)
    K2     end inference + smallest enclosing bin      (avdb_record_prep)
    K4     long-allele key digests (if any)            (avdb_vrs_digest)
    K3     in-batch primary-key dedup (optional)       (avdb_pk_dedup)
    host   ltree path / key text, COPY rows, mapping

``load_vcf_text(text)`` is the whole-batch GPU path of the load driver
(Load/bin/load_vcf_file.py:101-119): K0 tokenize, K2, K4, (K3), then K5 writes
the COPY rows and the .mapping lines as text on the device; lines the GPU does
not render byte-exact are rendered here, in place.

``parse_variant`` is ``parse_variants([line])``: one code path, one set of
semantics.  Exceptions match the reference at the same record: ``ValueError``
when a key cannot be built (e.g. ``':'`` inside an allele breaks
``metaseqId.split(':')``, primary_key_generator.py:106, through the retry
ladder :234-256), ``TypeError`` when the location has no bin
(bin_index.py:75).  ``--skipExisting`` checks a key set of the rows already
loaded (``existing.ExistingVariants``, K6) instead of the database.  The
loader's database hand-offs keep the reference's surface: ``set_cursor`` /
``load_variants`` give the COPY buffer to the caller's cursor exactly as
variant_loader.py:395-405,479-486 do (``copy_expert(copy_sql, buffer, 2**10)``,
then a fresh buffer), ``update_variants`` hands the update buffer over as
:457-476 do, and ``set_algorithm_invocation`` takes the AlgorithmInvocation id
from a provider the caller installs (``set_algorithm_invocation_provider``) in
place of the row insert (:431-437).  ``update_existing`` (rewriting loaded rows)
stays out of scope and raises ``NotImplementedError``.  The ADSP datasource checks
every alt's primary key against the rows already loaded (``is_duplicate(recordPK)``,
vcf_variant_loader.py:303-307) through the same exported key set (K7 keys, K6
text probe): a loaded key becomes an ``is_adsp_variant`` update in
``update_buffer()`` instead of a COPY row, and COPY rows carry the extra
``is_adsp_variant`` column (:336-337).  Display attributes come from
K5a (``avdb_display_attributes``); alleles must be ASCII (VCF 4.x REF/ALT).
"""

from __future__ import annotations

import logging
import re
from io import StringIO
from typing import Dict, List, Optional, Sequence

import numpy as np

from .chromosomes import UNKNOWN_CHROM, bin_index_chrom_code
from .parsers import VcfEntryParser, _xstr

REQUIRED_COPY_FIELDS = ["chromosome", "record_primary_key", "position", "metaseq_id", "bin_index",
                        "row_algorithm_id"]
ALLOWABLE_COPY_FIELDS = ["chromosome", "record_primary_key", "position", "is_multi_allelic",
                         "is_adsp_variant", "ref_snp_id", "metaseq_id", "bin_index", "display_attributes",
                         "allele_frequencies", "cadd_scores", "adsp_most_severe_consequence",
                         "adsp_ranked_consequences", "loss_of_function", "vep_output", "adsp_qc",
                         "gwas_flags", "other_annotation", "row_algorithm_id"]


class _AltError(Exception):
    pass


_ALG_INVOCATION_PROVIDER = None


def set_algorithm_invocation_provider(provider):
    """Install ``provider(callingScript, comment, commit) -> id``, the stand-in for
    the AlgorithmInvocation row insert ``VCFVariantLoader.set_algorithm_invocation``
    makes in the reference (variant_loader.py:431-437, algorithm_invocation.py:28-47).
    ``None`` removes it."""
    global _ALG_INVOCATION_PROVIDER
    _ALG_INVOCATION_PROVIDER = provider


def _split_sql(sql):
    """psycopg2.extras._split_sql's rule: the text before and after the one ``%s``
    placeholder, with ``%%`` turned back into ``%``; any other ``%`` escape, a
    second ``%s`` or none at all raise ``ValueError``.  ``sql`` is str or bytes
    and the parts keep its type."""
    b = isinstance(sql, bytes)
    pct, ess = (b"%", b"s") if b else ("%", "s")
    pre, post = [], []
    cur = pre
    for tok in re.split(rb"(%.)" if b else r"(%.)", sql):
        if len(tok) != 2 or tok[:1] != pct:
            cur.append(tok)
        elif tok[1:] == ess:
            if cur is not pre:
                raise ValueError("the query contains more than one '%s' placeholder")
            cur = post
        elif tok[1:] == pct:
            cur.append(pct)
        else:
            raise ValueError("unsupported format character: %r" % (tok[1:],))
    if cur is pre:
        raise ValueError("the query doesn't contain any '%s' placeholder")
    j = b"" if b else ""
    return j.join(pre), j.join(post)


def _execute_values(cur, sql, argslist, template=None, page_size=100):
    """psycopg2.extras.execute_values (what variant_loader.py:471 calls): the
    ``VALUES %s`` placeholder expanded to one page of mogrified rows per
    ``execute``.  Uses psycopg2's own when it is importable; otherwise the same
    rule (``_split_sql``), every part in the type of ``sql`` (psycopg2 encodes a
    str query with the connection's encoding first; a cursor without a
    connection gets the text as it came)."""
    try:
        from psycopg2.extras import execute_values
    except ImportError:
        execute_values = None
    if execute_values is not None:
        return execute_values(cur, sql, argslist, template=template, page_size=page_size)
    b = isinstance(sql, bytes)
    pre, post = _split_sql(sql)
    rows = list(argslist)
    for lo in range(0, len(rows), page_size):
        page = rows[lo:lo + page_size]
        parts = []
        for row in page:
            t = template or "(" + ",".join(["%s"] * len(row)) + ")"
            v = cur.mogrify(t, row)
            if b and not isinstance(v, bytes):
                v = v.encode()
            elif not b and isinstance(v, bytes):
                v = v.decode()
            parts.append(v)
        cur.execute(pre + (b"," if b else ",").join(parts) + post)


_SLOW = object()  # parse_variant: the line needs the general path
_RS_NUM = re.compile(r"rs([1-9][0-9]{0,17})\Z")  # refSNP ids K8h renders (engine.ExtIdInterner)
_KEY_OK = 0       # AVDB_KEY_OK
_CHROM_CODES: Dict[str, int] = {}


class VCFVariantLoader(object):
    """GPU-backed drop-in for the reference ``VCFVariantLoader``'s record prep."""

    def __init__(self, datasource, verbose=False, debug=False, device=None):
        self.logger = logging.getLogger(__name__)
        self._verbose = verbose
        self._debug = debug
        self._datasource = datasource.lower() if datasource is not None else None
        self._device = device
        self._alg_invocation_id = None
        self._pk_generator = None
        self._bin_indexer = None
        self._engine = None
        self._counters = {}
        self._chromosome_map = None
        self._resume_after_variant = None
        self._resume = True
        self._current_variant = {}
        self._copy_buffer = None
        self._copy_fields = None
        self._copy_sql = None
        self._skip_existing = False
        self._existing = None
        self._update_existing = False
        self._vcf_header_fields = None
        self.last_load_stats = None
        self._match = None
        self._adsp_dup = None
        self._cursor = None
        self._batch_update = False
        self._update_sql = None
        self._update_buffer = []
        self._fail_at_variant = None
        self._log_skips = False
        self._initialize_counters()
        self.initialize_copy_buffer()
        self.logger.info(type(self).__name__ + " initialized")

    # ---- configuration (variant_loader.py / vcf_variant_loader.py) ---------
    def initialize_bin_indexer(self, gusConfigFile, genomeBuild=None, chromosome_lengths=None):
        """variant_loader.py:357-362.  The reference's bins come from whatever
        assembly its BinIndexRef table was built for; here the chromosome lengths
        follow ``genomeBuild`` (default: the PK generator's build, which
        load_vcf_file.py:62-63 initializes first; else GRCh38) or an explicit
        ``chromosome_lengths`` table."""
        from .bin_index import BinIndex
        from .chromosomes import ASSEMBLIES
        build = genomeBuild
        if build is None and self._pk_generator is not None:
            build = self._pk_generator.genome_build()
        build = build or "GRCh38"
        if chromosome_lengths is None and build not in ASSEMBLIES:
            raise ValueError("unknown genome build %r: pass chromosome_lengths (one per chr1..22,X,Y,M)" % build)
        self._bin_indexer = BinIndex(gusConfigFile, verbose=False, assembly=build if build in ASSEMBLIES
                                     else "GRCh38", chromosome_lengths=chromosome_lengths, device=self._device)
        self._engine = self._bin_indexer._engine

    def initialize_pk_generator(self, genomeBuild, seqrepoProxyPath, **kw):
        from .primary_key_generator import VariantPKGenerator
        self._pk_generator = VariantPKGenerator(genomeBuild, seqrepoProxyPath, device=self._device, **kw)

    def set_algorithm_invocation_id(self, alg_id):
        """Stands in for ``set_algorithm_invocation`` (variant_loader.py:431-437),
        which inserts an AlgorithmInvocation row (database, out of scope)."""
        self._alg_invocation_id = _xstr(alg_id)

    def set_algorithm_invocation(self, callingScript, comment, commit=True):
        """variant_loader.py:431-437.  The reference inserts an
        AnnotatedVDB.AlgorithmInvocation row through its own database connection
        (algorithm_invocation.py:28-47) and keeps the returned id; here the id
        comes from the provider installed with
        :func:`set_algorithm_invocation_provider` (called with the same three
        arguments), e.g. one that runs that INSERT ... RETURNING on the caller's
        connection.  Without a provider: NotImplementedError (no database here)."""
        provider = _ALG_INVOCATION_PROVIDER
        if provider is None:
            raise NotImplementedError("AlgorithmInvocation rows live in the database: install a provider with "
                                      "annotatedvdb_amd.loaders.set_algorithm_invocation_provider(fn), or call "
                                      "set_algorithm_invocation_id()")
        self._alg_invocation_id = _xstr(provider(callingScript, comment, commit))

    def alg_invocation_id(self):
        return self._alg_invocation_id

    get_algorithm_invocation_id = alg_invocation_id

    def initialize_copy_sql(self, copyFields=None):
        fields = list(REQUIRED_COPY_FIELDS) + ["ref_snp_id", "is_multi_allelic", "display_attributes",
                                                "allele_frequencies"]
        if copyFields:
            fields.extend(copyFields)
        if not set(fields) <= set(ALLOWABLE_COPY_FIELDS):
            raise ValueError("Copy fields include invalid columns from AnnotatedVDB.Variant")
        if self.is_adsp() and "is_adsp_variant" not in fields:
            fields.append("is_adsp_variant")
        self._copy_fields = fields
        self._copy_sql = "COPY AnnotatedVDB.Variant(" + ",".join(fields) + \
            ") FROM STDIN WITH (NULL 'NULL', DELIMITER '#')"

    def set_chromosome_map(self, chrmMap):
        self._chromosome_map = chrmMap

    def set_vcf_header_fields(self, fields):
        self._vcf_header_fields = fields

    def _gpu_vcf_opts(self):
        """K0 / K5h options for this loader's header fields and chromosome map, or
        ``_SLOW`` when the text must be parsed line by line on the host: a header
        whose first eight fields are not the standard ones (their positions would
        move), or a chromosome map object without its ``chromosome_map()`` dict."""
        from .parsers import DEFAULT_FIELDS
        min_fields = 0
        if self._vcf_header_fields:
            hf = [x.lower().replace("#", "") for x in self._vcf_header_fields]
            if hf[:8] != DEFAULT_FIELDS:
                return _SLOW
            min_fields = len(hf)
        cm = None
        if self._chromosome_map is not None:
            get_map = getattr(self._chromosome_map, "chromosome_map", None)
            if get_map is None:
                return _SLOW
            cm = self._engine.chrom_map(get_map(), key=id(self._chromosome_map))
        if not min_fields and cm is None:
            return None
        return self._engine.vcf_opts(min_fields, cm)

    def vcf_header_fields(self):
        return self._vcf_header_fields

    def set_skip_existing(self, skipDuplicates, gusConfigFile=None, existing=None):
        """``--skipExisting`` (variant_loader.py:159-162): the rows already loaded
        come as an :class:`~annotatedvdb_amd.existing.ExistingVariants` key set
        (an export of AnnotatedVDB.Variant) instead of a database connection."""
        if skipDuplicates and existing is None:
            raise NotImplementedError("--skipExisting needs the existing rows: pass existing=ExistingVariants(...) "
                                      "(exported from AnnotatedVDB.Variant); there is no database here")
        self._skip_existing = bool(skipDuplicates)
        self._existing = existing if skipDuplicates else None

    def is_duplicate(self, variantId, returnMatch=False):
        """variant_loader.py:173-174 for a metaseq id, against the key set (K6)."""
        from .chromosomes import CHROM_NAMES
        from .engine import pack_records
        if self._existing is None:
            raise ValueError("set_skip_existing(True, existing=...) first")
        c, p, r, a = variantId.split(":")
        code = CHROM_NAMES.index(c) if c in CHROM_NAMES else 255
        b = pack_records([code], [int(p)], [r.encode()], [a.encode()]).to(self._engine.device)
        m, k = self._existing.probe(b)
        k0 = int(m.cpu()[0]) if int(k.cpu()[0]) != 255 else self._existing.resolve_host(variantId)
        if k0 < 0:
            return None if returnMatch else False
        return self._existing.payload(k0) if returnMatch else True

    def skip_existing(self):
        return self._skip_existing

    def set_update_existing(self, updateExisting):
        if updateExisting:
            raise NotImplementedError("updating existing rows needs the database; out of scope")

    def update_existing(self):
        return self._update_existing

    def get_datasource(self):
        return self._datasource

    def is_dbsnp(self):
        return self._datasource == "dbsnp"

    def is_adsp(self):
        return self._datasource == "adsp"

    def is_eva(self):
        return self._datasource == "eva"

    def bin_indexer(self):
        return self._bin_indexer

    def pk_generators(self):
        return self._pk_generator

    # ---- resume (variant_loader.py:342-354,440-454) -------------------------
    def resume_load(self):
        return self._resume

    def set_resume_after_variant(self, variantId):
        self._resume_after_variant = variantId
        self._resume = False

    def _update_resume_status(self, variantId):
        if not self.resume_load():
            self.increment_counter("skipped")
            self._resume = variantId == self._resume_after_variant
            if self.resume_load() is True:
                self.logger.warning(("Resuming after", self._resume_after_variant))

    # ---- counters and COPY buffer ---------------------------------------------
    def _initialize_counters(self, additionalCounters=None):
        self._counters = {"line": 0, "variant": 0, "skipped": 0, "duplicates": 0, "update": 0}
        for ac in additionalCounters or []:
            self._counters[ac] = 0

    def get_count(self, counter):
        return self._counters[counter]

    def increment_counter(self, counter, by=1):
        self._counters[counter] = self._counters[counter] + by

    def initialize_copy_buffer(self):
        self._copy_buffer = StringIO()

    def close_copy_buffer(self):
        self._copy_buffer.close()

    def reset_copy_buffer(self):
        self.close_copy_buffer()
        self.initialize_copy_buffer()

    def copy_buffer(self, sizeOnly=False):
        return self._copy_buffer.tell() if sizeOnly else self._copy_buffer

    def add_copy_str(self, copyStr):
        self._copy_buffer.write(copyStr + "\n")

    # ---- database hand-offs (variant_loader.py:395-405,457-486) --------------
    def cursor(self):
        return self._cursor

    def set_cursor(self, cursor):
        """The caller's database cursor (psycopg2 or anything with its
        ``copy_expert`` / ``execute`` / ``mogrify``)."""
        self._cursor = cursor

    def load_variants(self):
        """COPY the buffered rows (variant_loader.py:479-486): the buffer goes to
        the caller's cursor as ``copy_expert(copy_sql, buffer, 2**10)``, then a
        fresh buffer starts.  Errors propagate (the reference passes them through
        raise_pg_exception, which re-raises)."""
        self._copy_buffer.seek(0)
        self._cursor.copy_expert(self._copy_sql, self._copy_buffer, 2 ** 10)
        self.reset_copy_buffer()

    def get_copy_fileds(self):
        return self._copy_fields

    def set_update_sql(self, sql):
        self._update_sql = sql

    def set_batch_update(self):
        """Updates as one SQL string buffer executed at once (variant_loader.py:146-150)."""
        self._batch_update = True
        self.initialize_update_buffer()

    def initialize_update_buffer(self):
        self._update_buffer = StringIO() if self._batch_update else []

    def close_update_buffer(self):
        if self._batch_update:
            self._update_buffer.close()

    def log_skips(self):
        self._log_skips = True

    def set_fail_at_variant(self, variant):
        self._fail_at_variant = variant

    def fail_at_variant(self):
        return self._fail_at_variant

    def is_fail_at_variant(self):
        return self._fail_at_variant == self.get_current_variant_id()

    def debug(self):
        return self._debug

    # ---- ADSP update buffer (variant_loader.py:290-300; vcf_variant_loader.py:222-226)
    def update_buffer(self, sizeOnly=False):
        """``(record_primary_key, 'chr' + chromosome)`` per ADSP alt whose key was
        already loaded (the values of the is_adsp_variant UPDATE,
        vcf_variant_loader.py:222-226); a SQL string buffer after
        ``set_batch_update()`` (variant_loader.py:298-304)."""
        if self._batch_update:
            return self._update_buffer.tell() if sizeOnly else self._update_buffer
        return len(self._update_buffer) if sizeOnly else self._update_buffer

    def reset_update_buffer(self):
        self.close_update_buffer()
        self.initialize_update_buffer()

    def update_variants(self):
        """Execute the update buffer on the caller's cursor (variant_loader.py:457-476):
        ``execute_values(cursor, update_sql, buffer, page_size=2**10)`` (psycopg2's,
        or the same paging over ``cursor.mogrify`` when psycopg2 is absent), or the
        batch string with ``cursor.execute``; then a fresh buffer."""
        if self._update_sql is None:
            raise ValueError("must set update sql (VariantLoader.set_update_sql(sql) before attempting update")
        if self.update_buffer(sizeOnly=True) > 0:
            if self._batch_update:
                self._update_buffer.seek(0)
                self._cursor.execute(self._update_buffer.getvalue())
            else:
                _execute_values(self._cursor, self._update_sql, self._update_buffer, page_size=2 ** 10)
            self.reset_update_buffer()
        else:
            self.logger.warning("update called on empty buffer")

    def close(self):
        self.close_copy_buffer()
        self.close_update_buffer()

    @property
    def _current_variant(self):
        v = self._cur_variant
        if v.__class__ is _LineVariant:  # a K5h line: parsed on first use
            v = self._cur_variant = v.resolve()
        return v

    @_current_variant.setter
    def _current_variant(self, v):
        self._cur_variant = v

    def get_current_variant(self, toStr=False):
        return str(self._current_variant) if toStr else self._current_variant

    def get_current_variant_id(self):
        v = self._cur_variant
        if v.__class__ is _LineVariant:
            return v.id
        return v.id if v else None

    # ---- record prep ----------------------------------------------------------
    def parse_variant(self, line, flags=None):
        """One VCF line -> ``{variant.id: [{primary_key, bin_index}, ...]}``
        (vcf_variant_loader.py:351-391).

        The loader's per-line call (load_vcf_file.py:112) takes a lean path: the
        host parse, ONE library call for all of the line's alts (K8h: end, bin,
        key, ltree path, display JSON), the COPY rows.  A line that path does not
        settle with certainty — a parse error, a key the PK generator must build
        (long alleles, ':' in an allele, non-rs ids), an unmappable bin, a FREQ
        the reference would fail on, resume/skip-existing/ADSP modes — goes
        through ``parse_variants([line])``, which raises where the reference
        raises (nothing is emitted before that decision)."""
        if flags is None and isinstance(line, str):
            out = self._parse_line_fast(line)
            if out is not _SLOW:
                return out
        return self.parse_variants([line], flags)[0]

    def _parse_line_fast(self, line):
        if (self._bin_indexer is None or self._pk_generator is None or self._existing is not None
                or self.is_adsp() or self._resume is not True):
            return _SLOW
        out = _SLOW
        vo = self._gpu_vcf_opts()
        if vo is not _SLOW:
            out = self._parse_line_k5h(line, vo)
        if out is _SLOW:
            out = self._parse_line_k8h(line)
        return out

    def _parse_line_k5h(self, line, vcf_opts=None):
        """The whole line in one library call (K5h, ``avdb_vcf_line_host``): COPY
        rows and the .mapping line as the K5 kernels render them."""
        try:
            raw = line.encode("ascii")
        except UnicodeEncodeError:
            return _SLOW
        st, copy, mp, r = self._engine.line_host().run(raw, _xstr(self._alg_invocation_id).encode(),
                                                       self._pk_generator.max_sequence_length(), vcf_opts=vcf_opts)
        if copy is None:
            return _SLOW
        # .mapping line: id TAB [{'primary_key': '<pk>', 'bin_index': '<path>'}, ...] (keys and
        # paths K5 renders hold no quote), i.e. str() of the list parse_variant returns
        vid, rest = mp[:-1].split("\t", 1)
        parts = rest.split("'")
        self.increment_counter("line")
        for _ in range(r.n_skip):
            self.logger.warning("Skipping variant " + vid + "; no alt allele (alt = .)")
        if r.n_skip:
            self.increment_counter("skipped", r.n_skip)
        self._copy_buffer.write(copy)
        self.increment_counter("variant", r.n_rows)
        self._current_variant = _LineVariant(line, vid, self)
        return {vid: [{"primary_key": pk, "bin_index": p} for pk, p in zip(parts[3::8], parts[7::8])]}

    def _parse_line_k8h(self, line):
        """Host parse (chromosome map / custom header honoured) + one K8h call for
        the line's alts (end, bin, key, path, display JSON)."""
        try:
            entry = VcfEntryParser(line, self._vcf_header_fields)
            entry.update_chromosome(self._chromosome_map)
            v = entry.get_variant(dbSNP=self.is_dbsnp(), namespace=True)
        except Exception:  # noqa: BLE001 — parse_variants raises it with the reference's counters
            return _SLOW
        pos = v.position
        ref = v.ref_allele
        alts = [a for a in v.alt_alleles if a != "."]
        rs = v.ref_snp_id
        if rs is None:
            ext = 0
        else:
            m = _RS_NUM.match(rs)
            if m is None:
                return _SLOW
            ext = int(m.group(1))
        chrom = _xstr(v.chromosome)
        ps = _xstr(pos)
        n = len(alts)
        if n:
            if not (0 < pos < 4294967296):
                return _SLOW
            code = _CHROM_CODES.get(chrom)
            if code is None:
                code = _CHROM_CODES[chrom] = min(bin_index_chrom_code(chrom), 255)
            rb = ref.encode()
            res = self._engine.small().run([code] * n, [pos] * n, refs=[rb] * n, alts=[a.encode() for a in alts],
                                           ext=[ext] * n, want=7, max_seq_len=self._pk_generator.max_sequence_length())
            if res is None:
                return _SLOW
            ks, paths, keys, disp, dst = res["key_state"], res["path"], res["key"], res["display"], res["disp_state"]
            freqs = []
            for i in range(n):
                if ks[i] != _KEY_OK or paths[i] is None or dst[i] != 0:
                    return _SLOW
                try:
                    freqs.append(_freq_str(entry, alts[i]))
                except Exception:  # noqa: BLE001
                    return _SLOW
        # -- the line is settled: emit exactly as vcf_variant_loader.py:273-348 --
        self.increment_counter("line")
        self._current_variant = v
        head = "chr" + chrom
        tail = "#".join((_xstr(self._alg_invocation_id), _xstr(rs, nullStr="NULL"),
                         "True" if v.is_multi_allelic else "NULL"))
        mapping = []
        i = 0
        for alt in v.alt_alleles:
            if alt == ".":
                self.logger.warning("Skipping variant " + v.id + "; no alt allele (alt = .)")
                self.increment_counter("skipped")
                continue
            pk, path = keys[i], paths[i]
            self._copy_buffer.write("#".join((head, pk, ps, ":".join((chrom, ps, ref, alt)), path, tail, disp[i],
                                              freqs[i])) + "\n")
            self.increment_counter("variant")
            mapping.append({"primary_key": pk, "bin_index": path})
            i += 1
        return {v.id: mapping}

    def parse_variants(self, lines: Sequence, flags=None, errors: str = "raise", dedup: bool = False,
                       keep_override=None):
        """Batched ``parse_variant``.  ``errors='raise'`` stops at the first
        failing line exactly like a loop of ``parse_variant`` would (earlier
        lines fully applied, the failing line's earlier alts applied);
        ``errors='record'`` returns the exception object for failing lines.
        ``dedup=True`` also skips the COPY row of any alt whose primary key
        already appeared in this batch (keep-first; the reference leaves that
        to removeDuplicates.sql) and counts it under ``'duplicates'``."""
        if self._bin_indexer is None or self._pk_generator is None:
            raise ValueError("initialize_bin_indexer() and initialize_pk_generator() first")
        if flags is not None:
            raise NotImplementedError("update flags are a database-update feature; out of scope")
        if not dedup and keep_override is None and len(lines) <= self.PER_LINE_MAX:
            # a batch too small to pay for the GPU launches: the per-line path line by
            # line (the same results; lines it does not settle take this function's
            # general path one at a time, which raises / records where the reference raises)
            out = []
            for line in lines:
                r = self._parse_line_fast(line) if isinstance(line, str) else _SLOW
                if r is _SLOW:
                    r = self._parse_batch([line], errors, dedup, keep_override)[0]
                out.append(r)
            return out
        return self._parse_batch(lines, errors, dedup, keep_override)

    def prepare_batch(self, records: Sequence, dedup: bool = True, errors: str = "raise") -> List[tuple]:
        """The additive batch entry SURVEY.md §8b proposes: per alt record
        ``(chromosome, position, ref, alt[, ref_snp_id])`` — the fields
        ``__parse_alt_alleles`` works from (vcf_variant_loader.py:259-348) — the
        tuple ``(end, bin_index, primary_key, keep)``, computed for the whole
        batch on the GPU (K2 end + bin, K3 keep-first, K4 digests for long
        alleles) instead of one call chain per alt:

        * ``end``: ``infer_variant_end_location`` (variant_annotator.py:36-79);
        * ``bin_index``: the ltree path ``find_bin_index(chromosome, position,
          end)`` returns (bin_index.py:59-75), ``None`` where the reference
          raises ``TypeError`` (an unknown contig or a position past its end);
        * ``primary_key``: ``generate_primary_key(metaseq id, ref_snp_id)``
          (primary_key_generator.py:99-122);
        * ``keep``: False for a record whose primary key an earlier record of
          the batch already has (removeDuplicates.sql:2-24 keeps the first);
          all True with ``dedup=False``.

        A record whose key the reference would not build (``ValueError``:
        primary_key_generator.py:117) raises it (``errors='raise'``) or gets the
        exception object in place of its tuple (``errors='record'``)."""
        if self._bin_indexer is None or self._pk_generator is None:
            raise ValueError("initialize_bin_indexer() and initialize_pk_generator() first")
        if errors not in ("raise", "record"):
            raise ValueError("errors must be 'raise' or 'record'")
        recs = [tuple(r) + (None,) * (5 - len(r)) for r in records]
        n = len(recs)
        if n == 0:
            return []
        from .engine import ExtIdInterner, pack_records
        eng = self._engine
        interner = ExtIdInterner()
        codes = np.asarray([min(bin_index_chrom_code(r[0]), 255) for r in recs], dtype=np.uint8)
        pos = [int(r[1]) for r in recs]
        db = pack_records(codes, pos, [str(r[2]).encode() for r in recs], [str(r[3]).encode() for r in recs],
                          [interner.key(r[4]) for r in recs]).to(eng.device)
        d_end, d_code, _, _ = eng.record_prep(db, want_lcp=False)
        keep = np.ones(n, dtype=np.uint8)
        if dedup:
            # K3 compares chromosome codes; the key text holds the label as given,
            # so labels that share a code ('1' / 'chr1', unknown contigs) are told
            # apart by comparing one code per distinct label instead
            labels: Dict[str, int] = {}
            lab = [labels.setdefault(str(r[0]), len(labels)) for r in recs]
            label_codes = {int(codes[i]) for i in {v: i for i, v in enumerate(lab)}.values()}
            ddb = db
            if len(label_codes) < len(labels):
                if len(labels) > 255:
                    raise ValueError("prepare_batch: more than 255 distinct chromosome labels in one batch")
                ddb = pack_records(lab, pos, [str(r[2]).encode() for r in recs], [str(r[3]).encode() for r in recs],
                                   [interner.key(r[4]) for r in recs]).to(eng.device)
            keep = eng.pk_dedup(ddb, grouped=False).cpu().numpy()[:n]
        ends = d_end.cpu().numpy().view(np.uint32)
        paths = eng.format_paths(codes, d_code.cpu().numpy())
        items = [("%s:%s:%s:%s" % (r[0], r[1], r[2], r[3]), r[4]) for r in recs]
        try:
            pks: List = list(self._pk_generator.generate_primary_keys(items))
        except ValueError:
            pks = []
            for it in items:  # isolate the failing records
                try:
                    pks.append(self._pk_generator.generate_primary_keys([it])[0])
                except ValueError as err:
                    if errors == "raise":
                        raise
                    pks.append(err)
        return [pk if isinstance(pk, Exception) else (int(ends[i]), paths[i], pk, bool(keep[i]))
                for i, pk in enumerate(pks)]

    #: parse_variants batches up to this many lines run line by line on the host
    #: path (K5h / K8h, ~5 us per line on the MI355X box's host); larger ones as
    #: device batches (load_vcf_text is the bulk path: K0 + K2 + K5 on the GPU)
    PER_LINE_MAX = 1 << 20

    def _parse_batch(self, lines, errors, dedup, keep_override):
        # ---- phase 1: host parse (stops at the first parse error) --------------
        parsed = []  # (entry, variant) | ("skip",) | ("error", exc)
        for line in lines:
            if self.resume_load() is False and self._resume_after_variant is None:
                parsed.append(("error", ValueError("Must set VariantLoader resume_afer_variant if resuming load")))
                break
            try:
                entry = VcfEntryParser(line, self._vcf_header_fields) if isinstance(line, str) else line
                if not self.resume_load():
                    self._update_resume_status(entry.get("id"))
                    parsed.append(("skip",))
                    continue
                entry.update_chromosome(self._chromosome_map)
                variant = entry.get_variant(dbSNP=self.is_dbsnp(), namespace=True)
                parsed.append((entry, variant))
            except Exception as err:  # noqa: BLE001 — re-raised in phase 3
                parsed.append(("error", err))
                if errors == "raise":
                    break

        # ---- phase 2: per-alt records -> GPU --------------------------------
        recs = self._records_of(parsed)
        db = codes = None
        small = None
        if recs:
            from .engine import ExtIdInterner, pack_records
            from . import _native as N
            interner = ExtIdInterner()
            codes = np.asarray([min(bin_index_chrom_code(r[5].chromosome), 255) for r in recs],
                               dtype=np.uint8)
            pos = [r[5].position for r in recs]
            refs = [r[5].ref_allele.encode() for r in recs]
            alts = [r[1].encode() for r in recs]
            ext = [interner.key(r[5].ref_snp_id) for r in recs]
            if not dedup and keep_override is None and self._existing is None and all(0 < p < 2 ** 32 for p in pos):
                # the per-line drop-in path: K2 + K7 + K5a in one launch (K8), no copies
                small = self._engine.small().run(
                    codes, pos, refs=refs, alts=alts, ext=ext,
                    want=N.SMALL_PATH | N.SMALL_KEY | N.SMALL_DISPLAY,
                    max_seq_len=self._pk_generator.max_sequence_length())
            if small is None:
                db = pack_records(codes, pos, refs, alts, ext).to(self._engine.device)
        if small is not None:
            paths, pks, keep, disp = self._small_prep(recs, small)
        else:
            paths, pks, keep, disp = self._gpu_prep(recs, db, codes, dedup, keep_override)
        # ---- phase 3: emit in order --------------------------------------------
        return self._emit(parsed, recs, paths, pks, keep, disp, errors)

    def parse_vcf_text(self, text, errors: str = "raise", dedup: bool = False):
        """``parse_variants`` for raw VCF text, tokenized on the GPU (K0).

        Line semantics follow the load driver (Load/bin/load_vcf_file.py:101-119):
        lines are rstripped and ``#`` lines are skipped; one result per data
        line.  Text the GPU does not canonicalise (flagged lines) is parsed by
        ``VcfEntryParser`` for those lines only."""
        from .engine import (VCF_COMMENT, VCF_HOST_FLAGS, VCF_ID_METASEQ, VCF_ID_RS, VCF_INFO_RS,
                             ExtIdInterner)
        from .chromosomes import CHROM_NAMES
        from types import SimpleNamespace
        if self._bin_indexer is None or self._pk_generator is None:
            raise ValueError("initialize_bin_indexer() and initialize_pk_generator() first")
        vo = self._gpu_vcf_opts()
        if not self.resume_load() or vo is _SLOW:
            # resume / a header with moved fields: exact per-line semantics
            return self.parse_variants(_data_lines(bytes(text)), errors=errors, dedup=dedup)
        raw = bytes(text)
        eng = self._engine
        vb = eng.vcf_tokenize(raw, vo)
        L = vb.lines_host()
        db = vb.records
        rec_line = vb.rec_line.cpu().numpy()
        codes = db.chrom.cpu().numpy().copy()
        # ---- phase 1: per-line variant views from the line table ---------------
        parsed = []
        line_idx = []          # data-line index -> parsed index
        host_patch = {}        # line -> (chrom code, pos, ext key)
        interner = ExtIdInterner()
        stop = False
        for li in range(vb.n_lines):
            rec = L[li]
            fl = int(rec["flags"])
            if fl & VCF_COMMENT:
                line_idx.append(-1)
                continue
            line_idx.append(len(parsed))
            if stop:
                continue
            st = int(rec["start"])
            line = raw[st:st + int(rec["len"])].decode("utf-8")
            code = int(rec["chrom"])
            try:
                if fl & (VCF_HOST_FLAGS | 0x102) or code == 255 or int(rec["n_rec"]) == 0:
                    entry = VcfEntryParser(line, self._vcf_header_fields)
                    entry.update_chromosome(self._chromosome_map)
                    v = entry.get_variant(dbSNP=self.is_dbsnp(), namespace=True)
                    if fl & VCF_HOST_FLAGS:
                        host_patch[li] = (min(bin_index_chrom_code(v.chromosome), 255), v.position,
                                          interner.key(v.ref_snp_id))
                else:
                    f = rec["field"]
                    ref = line[f[3]:f[4] - 1]
                    altf = line[f[4]:f[5] - 1]
                    chrom = CHROM_NAMES[code]
                    pos = int(rec["pos"])
                    if fl & VCF_ID_RS:
                        rs = line[f[2]:f[3] - 1]
                    elif fl & VCF_INFO_RS:
                        rs = "rs%d" % int(rec["ext_id"])
                    else:
                        rs = None
                    vid = "%s:%d:%s:%s" % (chrom, pos, ref, altf) if fl & VCF_ID_METASEQ else line[f[2]:f[3] - 1]
                    alts = altf.split(",")
                    v = SimpleNamespace(id=vid, ref_snp_id=rs, ref_allele=ref, alt_alleles=alts,
                                        is_multi_allelic=len(alts) > 1, chromosome=chrom, position=pos,
                                        rs_position=None)
                    entry = _LazyEntry(line)
                parsed.append((entry, v))
            except Exception as err:  # noqa: BLE001 — re-raised in phase 3
                parsed.append(("error", err))
                if errors == "raise":
                    stop = True
        # ---- phase 2: records are already on the device; patch host-resolved lines
        if host_patch:
            import torch
            idx = [i for i, l in enumerate(rec_line.tolist()) if l in host_patch]
            if idx:
                vals = [host_patch[int(rec_line[i])] for i in idx]
                it = torch.tensor(idx, dtype=torch.int64, device=eng.device)
                db.chrom[it] = torch.tensor([v[0] for v in vals], dtype=torch.uint8, device=eng.device)
                db.pos[it] = torch.tensor([v[1] for v in vals], dtype=torch.int64).to(torch.int32).to(eng.device)
                db.ext_id[it] = torch.tensor([v[2] if v[2] < (1 << 63) else v[2] - (1 << 64) for v in vals],
                                             dtype=torch.int64, device=eng.device)
                codes[idx] = [v[0] for v in vals]
        recs = self._records_of(parsed)
        # GPU records map 1:1 onto recs (same line order, ALT != '.'), except for
        # lines that stopped early on a parse error
        keep_rows = [i for i, l in enumerate(rec_line.tolist())
                     if line_idx[l] >= 0 and line_idx[l] < len(parsed) and parsed[line_idx[l]][0] != "error"]
        if len(keep_rows) != rec_line.size:
            import torch
            sel = torch.tensor(keep_rows, dtype=torch.int64, device=eng.device)
            db = _select(db, sel)
            codes = codes[keep_rows]
        assert db.n == len(recs), (db.n, len(recs))
        paths, pks, keep, disp = self._gpu_prep(recs, db if recs else None, codes, dedup)
        return self._emit(parsed, recs, paths, pks, keep, disp, errors)

    def load_vcf_text(self, text, dedup: bool = False, errors: str = "raise",
                      batch_bytes: int = 256 << 20, mapping_out=None) -> str:
        """The load driver (Load/bin/load_vcf_file.py:101-119) on the GPU for a
        block of VCF text: appends every COPY row to ``copy_buffer()`` and
        returns the .mapping text (one ``id<TAB>[{...}]`` line per data line).
        Text larger than ``batch_bytes`` runs as consecutive device batches cut at
        line boundaries (bounded HBM and host memory); ``dedup`` (keep-first per
        primary key, our addition) applies within each batch.

        ``mapping_out`` (a file-like ``write``) receives the .mapping text as each
        batch completes, as the driver prints each line's mapping before reading
        the next (load_vcf_file.py:116-117).  When a line raises
        (``errors='raise'``), everything before it — COPY rows, .mapping text,
        counters — has been emitted exactly as a loop of ``parse_variant`` would
        have; the .mapping text of the lines before it is also attached to the
        exception as ``avdb_partial_mapping``."""
        raw = bytes(text)
        done = []

        def emit(t):
            if mapping_out is not None:
                mapping_out.write(t)
            done.append(t)

        i = 0
        try:
            while i < len(raw) or (i == 0 and not raw):
                j = min(len(raw), i + batch_bytes)
                if j < len(raw):
                    k = raw.rfind(b"\n", i, j)
                    if k >= i:
                        j = k + 1
                    else:  # one line longer than a batch
                        k = raw.find(b"\n", j)
                        j = len(raw) if k < 0 else k + 1
                emit(self._load_vcf_batch(raw[i:j], dedup, errors))
                i = j
                if not raw:
                    break
        except Exception as err:  # noqa: BLE001 — re-raised with the partial mapping text
            part = getattr(err, "avdb_partial_mapping", "")
            if mapping_out is not None and part:
                mapping_out.write(part)
            try:
                err.avdb_partial_mapping = "".join(done) + part
            except AttributeError:
                pass
            raise
        return "".join(done)

    def _load_vcf_batch(self, raw: bytes, dedup: bool, errors: str) -> str:
        """One device batch of :meth:`load_vcf_text`.

        K0 tokenizes, K2 infers ends and bins, K4 digests long keys, K3 marks
        in-batch duplicates when ``dedup``, K6 checks the rows already loaded
        (``--skipExisting``: metaseq ids; ADSP: the K7 primary keys), and K5
        writes both texts on the device.  Lines K5 leaves to the host
        (``AVDB_LINE_HOST``) are rendered through ``parse_variants`` and spliced
        in at their position; with ``errors='raise'`` the first failing line
        raises after everything before it (and its own earlier alts) was
        emitted, as a loop of ``parse_variant`` would."""
        import torch
        from .engine import VCF_HOST_FLAGS
        from . import _native as N
        if self._bin_indexer is None or self._pk_generator is None:
            raise ValueError("initialize_bin_indexer() and initialize_pk_generator() first")
        vo = self._gpu_vcf_opts()
        if not self.resume_load() or vo is _SLOW or (self.is_adsp() and self._existing is None):
            # resume / a header with moved fields / ADSP without a validator (the
            # reference's is_duplicate raises on it): exact per-line semantics
            out = self.parse_variants(_data_lines(raw), errors=errors, dedup=dedup)
            return "".join("".join("%s\t%s\n" % kv for kv in o.items()) for o in out
                           if isinstance(o, dict))
        eng = self._engine
        vb = eng.vcf_tokenize(raw, vo)
        n = vb.n_lines
        if n == 0:
            return ""
        db = vb.records
        # K0 lines with host-resolved fields: resolve chrom/pos/refSNP key on the host
        # before K2/K3 see the records (same as parse_vcf_text)
        flags = vb.lines[: n * 80].view(torch.int32).view(n, 20)[:, 18]
        hl = torch.nonzero((flags & VCF_HOST_FLAGS) != 0).squeeze(1).cpu().tolist()
        if hl:
            self._patch_host_records(raw, vb, hl)
        end, code, status, _ = eng.record_prep(db, want_lcp=False)
        digest = None
        mx = self._pk_generator.max_sequence_length()
        if db.n and bool(((db.ref_len + db.alt_len) > mx).any()) and self._pk_generator.has_sequence_digests():
            digest, _ = self._pk_generator._eng().vrs_digest(db, mx)
        keep = eng.pk_dedup(db, grouped=False) if dedup and db.n else None
        ex = m_dev = None
        if self._existing is not None and db.n:  # --skipExisting: K6 hash join, consumed by K5
            m_dev, k = self._existing.probe(db)
            ex = self._existing.format_args(m_dev, k)
        adsp_dup = kt = None
        if self.is_adsp() and db.n:
            # is_duplicate(recordPK): the primary keys as text (K7), probed against the
            # exported keys (K6); keys K7 cannot render belong to host lines
            kt = eng.primary_keys(db, digest=digest, max_seq_len=mx)
            pm = self._existing.probe_primary_keys(kt.keys, kt.key_off, db.n, skip=kt.state[: db.n])
            adsp_dup = (pm >= 0).to(torch.uint8)
        fr = eng.vcf_format(vb, end, code, status, digest, keep, alg_id=_xstr(self._alg_invocation_id),
                            max_seq_len=mx, existing=ex, adsp=self.is_adsp(), adsp_dup=adsp_dup)
        state = fr.line_state.cpu().numpy()
        copy_off = fr.copy_off.cpu().numpy()
        map_off = fr.map_off.cpu().numpy()
        copy_raw = fr.copy.cpu().numpy().tobytes().decode("ascii")
        map_raw = fr.mapping.cpu().numpy().tobytes().decode("ascii")
        ctr = fr.counters.cpu().numpy()
        host = np.nonzero(state == N.LINE_HOST)[0]
        n_data = int(np.count_nonzero(state != N.LINE_SKIP))
        rec_off = vb.rec_off.cpu().numpy()
        # ADSP updates of GPU-rendered lines, in record order: (line, pk, 'chr' + chrom)
        gpu_updates = []
        if adsp_dup is not None:
            dup = adsp_dup.cpu().numpy().astype(bool)
            if m_dev is not None:
                dup &= m_dev.cpu().numpy() < 0  # skipped as existing first (vcf_variant_loader.py:285-291)
            rec_line = vb.rec_line.cpu().numpy()
            idx = np.nonzero(dup & (state[rec_line] == N.LINE_GPU))[0]
            if len(idx):
                ko = kt.key_off.cpu().numpy()
                kb = kt.keys.cpu().numpy().tobytes()
                ch = db.chrom.cpu().numpy()
                from .chromosomes import CHROM_NAMES
                gpu_updates = [(int(rec_line[i]), kb[ko[i]:ko[i + 1]].decode("ascii"), "chr" + CHROM_NAMES[ch[i]])
                               for i in idx.tolist()]
        self.last_load_stats = {"lines": n_data, "gpu_lines": n_data - len(host), "host_lines": len(host),
                                "copy_bytes": len(copy_raw), "mapping_bytes": len(map_raw)}

        def add_gpu_counters(upto=None):
            """counters of the GPU-rendered lines (vcf_variant_loader.py:279,288,306,344;
            variant_loader.py:94), or of those before line ``upto``"""
            if upto is None:
                self.increment_counter("line", n_data - len(host))
                self.increment_counter("variant", int(ctr[N.CTR_COPY_ROWS]))
                self.increment_counter("skipped", int(ctr[N.CTR_SKIPPED_ALTS]))
                self.increment_counter("duplicates", int(ctr[N.CTR_DUP_ROWS]))
                self.increment_counter("update", int(ctr[N.CTR_ADSP_UPDATES]))
                return
            self._add_partial_counters(vb, state, rec_off, copy_raw[: int(copy_off[upto])], keep, m_dev,
                                       adsp_dup, upto)

        u = 0  # next GPU update to flush
        if len(host) == 0:
            self._copy_buffer.write(copy_raw)
            self._update_buffer.extend(x[1:] for x in gpu_updates)
            add_gpu_counters()
            return map_raw
        keep_h = keep.cpu().numpy() if keep is not None else None
        # the host lines' table rows in one transfer
        Lh = vb.lines[: n * 80].view(n, 80)[torch.from_numpy(host).to(eng.device)].cpu().numpy()
        Lh = Lh.view(np.uint64).reshape(len(host), 10)
        maps = []
        c0 = m0 = 0
        for hi, li in enumerate(host.tolist()):
            # GPU text (and ADSP updates) of the lines before this one
            self._copy_buffer.write(copy_raw[c0:copy_off[li]])
            maps.append(map_raw[m0:map_off[li]])
            c0, m0 = int(copy_off[li]), int(map_off[li])
            while u < len(gpu_updates) and gpu_updates[u][0] < li:
                self._update_buffer.append(gpu_updates[u][1:])
                u += 1
            st, ln = int(Lh[hi, 0]), int(Lh[hi, 1] & 0xFFFFFFFF)
            line = raw[st:st + ln].decode("utf-8")
            kov = None if keep_h is None else keep_h[rec_off[li]:rec_off[li + 1]]
            try:
                res = self.parse_variants([line], errors="raise", keep_override=kov)[0]
            except Exception as err:  # noqa: BLE001
                if errors == "raise":
                    add_gpu_counters(upto=li)
                    try:
                        err.avdb_partial_mapping = "".join(maps)
                    except AttributeError:
                        pass
                    raise
                maps.append("")
                continue
            maps.append("".join("%s\t%s\n" % kv for kv in res.items()))
        self._copy_buffer.write(copy_raw[c0:])
        maps.append(map_raw[m0:])
        self._update_buffer.extend(x[1:] for x in gpu_updates[u:])
        add_gpu_counters()
        return "".join(maps)

    def _add_partial_counters(self, vb, state, rec_off, copy_text, keep, match, adsp_dup, upto):
        """Counters of the GPU-rendered lines before line ``upto`` (the failing
        line), from the per-line / per-record arrays."""
        from . import _native as N
        n = vb.n_lines
        L = vb.lines_host()
        gl = np.nonzero(state[:upto] == N.LINE_GPU)[0]
        self.increment_counter("line", len(gl))
        self.increment_counter("variant", copy_text.count("\n"))
        r_end = int(rec_off[upto])
        on_gpu = np.zeros(r_end, dtype=bool)
        for li in gl.tolist():
            on_gpu[int(rec_off[li]):int(rec_off[li + 1])] = True
        skipped = int((L["n_alt"][gl].astype(np.int64) - L["n_rec"][gl]).sum())
        matched = np.zeros(r_end, dtype=bool)
        if match is not None:
            matched = match[:r_end].cpu().numpy() >= 0
        skipped += int((matched & on_gpu).sum())
        upd = np.zeros(r_end, dtype=bool)
        if adsp_dup is not None:
            upd = (adsp_dup[:r_end].cpu().numpy() != 0) & ~matched
        self.increment_counter("update", int((upd & on_gpu).sum()))
        self.increment_counter("skipped", skipped)
        if keep is not None:
            dup = (keep[:r_end].cpu().numpy() == 0) & ~matched & ~upd
            self.increment_counter("duplicates", int((dup & on_gpu).sum()))

    def _patch_host_records(self, raw, vb, line_ids):
        """Host resolution of K0-flagged lines' chrom / pos / refSNP key in the
        device records (the GPU only canonicalises plain text)."""
        import torch
        from .engine import ExtIdInterner
        eng = self._engine
        db = vb.records
        n = vb.n_lines
        Lh = vb.lines[: n * 80].view(torch.uint8).view(n, 80)[torch.tensor(line_ids, device=eng.device)]
        Lh = Lh.cpu().numpy()
        rec_off = vb.rec_off[torch.tensor(line_ids, device=eng.device)].cpu().numpy()
        nrec = vb.rec_off[torch.tensor(line_ids, device=eng.device) + 1].cpu().numpy() - rec_off
        interner = ExtIdInterner()
        idx, vals = [], []
        for k in range(len(line_ids)):
            w = np.frombuffer(Lh[k].tobytes(), dtype=np.uint64)
            st, ln = int(w[0]), int(w[1] & 0xFFFFFFFF)
            try:
                e = VcfEntryParser(raw[st:st + ln].decode("utf-8"), self._vcf_header_fields)
                e.update_chromosome(self._chromosome_map)
                v = e.get_variant(dbSNP=self.is_dbsnp(), namespace=True)
            except Exception:  # noqa: BLE001 — the host renderer raises it at this line
                continue
            key = interner.key(v.ref_snp_id)
            for j in range(int(nrec[k])):
                idx.append(int(rec_off[k]) + j)
                vals.append((min(bin_index_chrom_code(v.chromosome), 255), v.position, key))
        if idx:
            it = torch.tensor(idx, dtype=torch.int64, device=eng.device)
            db.chrom[it] = torch.tensor([x[0] for x in vals], dtype=torch.uint8, device=eng.device)
            db.pos[it] = torch.tensor([x[1] for x in vals], dtype=torch.int64).to(torch.int32).to(eng.device)
            db.ext_id[it] = torch.tensor([x[2] if x[2] < (1 << 63) else x[2] - (1 << 64) for x in vals],
                                         dtype=torch.int64, device=eng.device)

    # ---- shared pieces --------------------------------------------------------
    def _records_of(self, parsed):
        """Per-alt record descriptors [line, alt, metaseq, pk_error, long, variant]."""
        recs = []
        max_len = self._pk_generator.max_sequence_length()
        for li, p in enumerate(parsed):
            if len(p) != 2 or p[0] in ("skip", "error"):
                continue
            entry, v = p
            for alt in v.alt_alleles:
                if alt == ".":
                    continue
                ref = v.ref_allele
                metaseq = ":".join((_xstr(v.chromosome), _xstr(v.position), ref, alt))
                pk_err = None
                if len(metaseq.split(":")) != 4:
                    # metaseqId.split(':') fails on every rung of the retry ladder
                    pk_err = ValueError("too many values to unpack (expected 4)")
                recs.append([li, alt, metaseq, pk_err, len(ref) + len(alt) > max_len, v])
        return recs

    def _small_prep(self, recs, res):
        """K8's outputs as ``_gpu_prep`` returns them.  Keys K8 rendered are used
        as is; the others (long alleles: the VRS digest; ':' in an allele; ids
        without a canonical form) go through the PK generator, which raises where
        the reference raises."""
        from . import _native as N
        n = len(recs)
        pks: List[Optional[str]] = [None] * n
        ks = res["key_state"]
        items, idx = [], []
        for i, r in enumerate(recs):
            if r[3] is not None:
                continue
            if ks[i] == N.KEY_OK:
                pks[i] = res["key"][i]
            else:
                items.append((r[2], r[5].ref_snp_id))
                idx.append(i)
        if items:
            try:
                for i, k in zip(idx, self._pk_generator.generate_primary_keys(items)):
                    pks[i] = k
            except ValueError:
                for i, it in zip(idx, items):  # isolate the failing records
                    try:
                        pks[i] = self._pk_generator.generate_primary_keys([it])[0]
                    except ValueError as err:
                        recs[i][3] = err
        self._match = None
        self._adsp_dup = None
        if self.is_adsp() and self._existing is not None:
            self._adsp_dup = [pk is not None and self._existing.has_primary_key(pk) for pk in pks]
        disp = [d if st == 0 else None for d, st in zip(res["display"], res["disp_state"])]
        return res["path"], pks, None, disp

    def _gpu_prep(self, recs, db, codes, dedup, keep_override=None):
        """K2 (+K3) and K5a on the device batch, then ltree text, primary keys
        and display-attribute JSON per record."""
        n = len(recs)
        pks: List[Optional[str]] = [None] * n
        if not n:
            return [], pks, None, []
        eng = self._engine
        d_end, d_code, d_status, _ = eng.record_prep(db, want_lcp=False)
        if keep_override is not None:
            keep = np.asarray(keep_override, dtype=np.uint8)
        else:
            d_keep = eng.pk_dedup(db, grouped=False) if dedup else None
            keep = d_keep.cpu().numpy() if d_keep is not None else None
        code = d_code.cpu().numpy().view(np.uint32)
        paths = eng.format_paths(np.asarray(codes, dtype=np.uint8), code)
        disp = _display_texts(eng, db, d_end)
        self._match = None
        if self._existing is not None:  # --skipExisting (K6)
            m, k = self._existing.probe(db)
            m, k = m.cpu().numpy(), k.cpu().numpy()
            for i in np.nonzero(k == 255)[0]:
                # (a record whose key cannot be built raises before this check)
                m[i] = self._existing.resolve_host(recs[i][2]) if recs[i][3] is None else -1
            self._match = m
        # primary keys (short: text; long: K4 digests in one launch)
        items, idx = [], []
        for i, r in enumerate(recs):
            if r[3] is None:
                items.append((r[2], r[5].ref_snp_id))
                idx.append(i)
        try:
            keys = self._pk_generator.generate_primary_keys(items)
            for i, k in zip(idx, keys):
                pks[i] = k
        except ValueError:
            for i, it in zip(idx, items):  # isolate the failing records
                try:
                    pks[i] = self._pk_generator.generate_primary_keys([it])[0]
                except ValueError as err:
                    recs[i][3] = err
        # ADSP: is_duplicate(recordPK) against the exported keys (vcf_variant_loader.py:303-307)
        self._adsp_dup = None
        if self.is_adsp() and self._existing is not None:
            self._adsp_dup = [pk is not None and self._existing.has_primary_key(pk) for pk in pks]
        return paths, pks, keep, disp

    def _emit(self, parsed, recs, paths, pks, keep, disp, errors):
        out = []
        ri = 0
        for li, p in enumerate(parsed):
            self.increment_counter("line")
            if p[0] == "skip":
                out.append(None)
                continue
            if p[0] == "error":
                if errors == "raise":
                    raise p[1]
                out.append(p[1])
                continue
            entry, v = p
            self._current_variant = v
            mapping = []
            failed = None
            for alt in v.alt_alleles:
                if alt == ".":
                    self.logger.warning("Skipping variant " + v.id + "; no alt allele (alt = .)")
                    self.increment_counter("skipped")
                    continue
                r = recs[ri]
                i = ri
                ri += 1
                # same order of failure as vcf_variant_loader.py:282-328: key, bin, FREQ
                if r[3] is not None:
                    failed = r[3] if isinstance(r[3], Exception) else ValueError(str(r[3]))
                    break
                if self._match is not None and self._match[i] >= 0:  # vcf_variant_loader.py:285-291
                    mapping += self._existing.payload(int(self._match[i]))
                    self.increment_counter("skipped")
                    continue
                if self.is_adsp():  # vcf_variant_loader.py:303-307
                    if self._adsp_dup is None:  # no validator: the reference's None.exists(...)
                        failed = AttributeError("'NoneType' object has no attribute 'exists'")
                        break
                    if self._adsp_dup[i]:
                        self._update_buffer.append((pks[i], "chr" + _xstr(v.chromosome)))
                        self.increment_counter("update")
                        continue
                path = paths[i]
                if path is None:
                    failed = TypeError("'NoneType' object is not subscriptable")
                    break
                try:
                    freq = _freq_str(entry, alt)
                except Exception as err:  # noqa: BLE001 — raised by get_frequencies, as the reference
                    failed = err
                    break
                if disp[i] is None:
                    failed = ValueError("non-ASCII allele: outside the GPU path's contract")
                    break
                pk = pks[i]
                if keep is not None and not keep[i]:
                    self.increment_counter("duplicates")
                else:
                    self.add_copy_str("#".join([
                        "chr" + _xstr(v.chromosome), pk, _xstr(v.position), r[2], path,
                        _xstr(self._alg_invocation_id), _xstr(v.ref_snp_id, nullStr="NULL"),
                        _xstr(v.is_multi_allelic, falseAsNull=True, nullStr="NULL"), disp[i], freq]
                        + (["True"] if self.is_adsp() else [])))  # is_adsp_variant (:336-337)
                    self.increment_counter("variant")
                mapping.append({"primary_key": pk, "bin_index": path})
            if failed is not None:
                if errors == "raise":
                    raise failed
                out.append(failed)
                ri = _next_line_start(recs, ri, li)  # past this line's remaining alts
                continue
            out.append({v.id: mapping})
        return out

class _LineVariant:
    """The current variant of a line K5h rendered: its id is known, the
    namespace (VcfEntryParser.get_variant) is built only if someone asks."""

    __slots__ = ("line", "id", "loader")

    def __init__(self, line, vid, loader):
        self.line, self.id, self.loader = line, vid, loader

    def resolve(self):
        ld = self.loader
        e = VcfEntryParser(self.line, ld._vcf_header_fields)
        e.update_chromosome(ld._chromosome_map)
        return e.get_variant(dbSNP=ld.is_dbsnp(), namespace=True)


class _LazyEntry:
    """Stands in for a parsed VcfEntryParser when only INFO FREQ may be needed."""

    __slots__ = ("_line", "_e")

    def __init__(self, line):
        self._line = line
        self._e = None

    def get_frequencies(self, alt):
        if "FREQ" not in self._line:
            return None
        if self._e is None:
            self._e = VcfEntryParser(self._line)
        return self._e.get_frequencies(alt)


def _display_texts(eng, db, d_end) -> List[Optional[str]]:
    """K5a display-attribute JSON per record (None: non-ASCII alleles)."""
    text, off, state = eng.display_attributes(db, d_end)
    raw = text.cpu().numpy().tobytes().decode("ascii")
    o = off.cpu().numpy()
    st = state.cpu().numpy()
    return [raw[o[i]:o[i + 1]] if st[i] == 0 else None for i in range(len(st))]


def _data_lines(raw: bytes) -> List[str]:
    """The load driver's lines (load_vcf_file.py:101-105): split at '\\n', each
    rstripped, '#' lines skipped.  An interior empty line stays (the reference
    parses it and raises); only the segment after a final newline is dropped."""
    parts = raw.decode("utf-8").split("\n")
    if parts and parts[-1] == "":
        parts.pop()
    return [ln.rstrip() for ln in parts if not ln.startswith("#")]


def _select(b, idx):
    from .engine import RecordBatch
    return RecordBatch(chrom=b.chrom[idx], pos=b.pos[idx], allele_off=b.allele_off[idx],
                       ref_len=b.ref_len[idx], alt_len=b.alt_len[idx], heap=b.heap,
                       ext_id=b.ext_id[idx])


def _next_line_start(recs, ri, li):
    while ri < len(recs) and recs[ri][0] == li:
        ri += 1
    return ri


def _freq_str(entry, alt):
    """xstr(get_frequencies(alt), nullStr='NULL') (vcf_variant_loader.py:313,329);
    exceptions propagate as in the reference."""
    import json
    f = entry.get_frequencies(alt)
    return "NULL" if f is None else json.dumps(f)
