"""INTEGRATION.md §1 run verbatim: the reference load driver's loop
(Load/bin/load_vcf_file.py:50-221) with the drop-in loader, against a fake
database cursor, over the reference's own load-driver output
(tests/golden/vcf_load.tsv.gz, produced by the verbatim VCFVariantLoader).

The code blocks are read out of INTEGRATION.md and exec'd as written; the
test supplies only what the reference driver has around them (args, the
database handle, the mmap'd file, print_args, the invocation-id provider).
The per-line recipe runs on the CPU with the host-only engine (AVDB_DEVICE=host:
parse_variant is the library's per-call host path, K5h / K8h); the batched
recipe runs the GPU kernels (K0 / K2 / K5) and is a GPU test."""

import gzip
import io
import json
import os
import re
from types import SimpleNamespace

import pytest

from conftest import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COPY_SQL_FIELDS = ("chromosome,record_primary_key,position,metaseq_id,bin_index,row_algorithm_id,ref_snp_id,"
                   "is_multi_allelic,display_attributes,allele_frequencies")


def recipe(name):
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"<!-- recipe: %s -->\s*```python\n(.*?)```" % re.escape(name), text, re.S)
    assert m, name
    return m.group(1)


class FakeCursor:
    """What the loader needs of a psycopg2 cursor: copy_expert / execute / mogrify."""

    def __init__(self):
        self.copies = []
        self.executed = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def copy_expert(self, sql, fh, size):
        self.copies.append((sql, fh.read(), size))

    def execute(self, sql, args=None):
        self.executed.append((sql, args))

    def mogrify(self, template, row):
        return template % tuple("'%s'" % v if isinstance(v, str) else str(v) for v in row)


class FakeDatabase:
    def __init__(self):
        self.cur = FakeCursor()

    def cursor(self):
        return self.cur


def golden_rows():
    out = []
    with gzip.open(os.path.join(GOLDEN, "vcf_load.tsv.gz"), "rt") as fh:
        fh.readline()
        for line in fh:
            raw, err, mapping, copy = line.rstrip("\n").split("\t")
            out.append((raw.replace("\\t", "\t"), err or None, json.loads(mapping), json.loads(copy)))
    return out


def run_recipe(tmp_path, blocks, lines, commit_after=500):
    """Write the lines as a VCF, exec the recipe blocks with the driver's
    surroundings; returns (namespace, database, mapping text)."""
    vcf = tmp_path / "chrT.vcf"
    vcf.write_text("##fileformat=VCFv4.1\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n"
                   + "".join(ln + "\n" for ln in lines))
    invocations = []
    db = FakeDatabase()
    args = SimpleNamespace(datasource="dbSNP", verbose=False, debug=False, commit=False, genomeBuild="GRCh38",
                           seqrepoProxyPath=None, gusConfigFile=None, skipExisting=False, commitAfter=commit_after)
    ns = {"args": args, "database": db, "fileName": str(vcf),
          "print_args": lambda a, pretty: json.dumps(vars(a), sort_keys=True),
          "new_algorithm_invocation": lambda script, params, commit: invocations.append(
              (script, params, commit)) or 1}
    from annotatedvdb_amd import loaders
    try:
        with open(vcf, "rb") as fh:
            ns["mappedFile"] = fh
            for b in blocks:
                exec(compile(recipe(b), "INTEGRATION.md:" + b, "exec"), ns)
    finally:
        loaders.set_algorithm_invocation_provider(None)
    assert invocations == [("load_vcf_result", json.dumps(vars(args), sort_keys=True), False)]
    mapping = open(str(vcf) + ".mapping").read()
    return ns, db, mapping


def check_against_golden(ns, db, mapping, rows, commit_after):
    copy_sql = "COPY AnnotatedVDB.Variant(%s) FROM STDIN WITH (NULL 'NULL', DELIMITER '#')" % COPY_SQL_FIELDS
    assert all(sql == copy_sql and size == 2 ** 10 for sql, _, size in db.cur.copies)
    got = "".join(text for _, text, _ in db.cur.copies)
    want = "".join(r + "\n" for _, _, _, copy in rows for r in copy)
    assert got == want
    assert mapping == "".join(m + "\n" for _, _, maps, _ in rows for m in maps)
    # one COPY per commitAfter lines, and one for the rest (load_vcf_file.py:135-142,177-178)
    assert len(db.cur.copies) == len(rows) // commit_after + 1
    loader = ns["loader"]
    assert loader.copy_buffer(sizeOnly=True) == 0
    assert loader.get_count("variant") == sum(len(c) for _, _, _, c in rows)
    assert loader.alg_invocation_id() == "1"


@pytest.fixture
def host_engine(monkeypatch):
    from annotatedvdb_amd import _native as N
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("libavdb_hip.so not built")
    monkeypatch.setenv("AVDB_DEVICE", "host")
    from annotatedvdb_amd import engine
    yield
    engine._ENGINES.pop("host", None)


def test_per_line_recipe_verbatim_vs_reference_load_driver(tmp_path, host_engine):
    """Every line the reference loaded without error (3,802 of 4,100): the COPY
    text the cursor receives and the .mapping file equal the reference's."""
    rows = [r for r in golden_rows() if r[1] is None]
    ns, db, mapping = run_recipe(tmp_path, ["setup", "per-line"], [r[0] for r in rows], commit_after=500)
    check_against_golden(ns, db, mapping, rows, 500)


def test_per_line_recipe_raises_where_the_reference_raised(tmp_path, host_engine):
    """A line the reference raised on ends the recipe with the same exception
    type; everything committed before it reached the cursor."""
    rows = golden_rows()
    k = next(i for i, r in enumerate(rows) if r[1] is not None and i > 40)
    err = rows[k][1]
    lines = [r[0] for r in rows[:k + 1] if r[1] is None or r is rows[k]]
    with pytest.raises(Exception) as ei:
        run_recipe(tmp_path, ["setup", "per-line"], lines, commit_after=10)
    assert type(ei.value).__name__ == err.split(":")[0]


def test_loader_cursor_surface(host_engine):
    """update_variants / set_batch_update / set_algorithm_invocation without a
    provider, against variant_loader.py:431-437,457-486."""
    from annotatedvdb_amd.loaders import VCFVariantLoader, set_algorithm_invocation_provider
    ld = VCFVariantLoader("ADSP")
    with pytest.raises(NotImplementedError):
        ld.set_algorithm_invocation("x", "y")
    set_algorithm_invocation_provider(lambda s, p, c: 42)
    try:
        ld.set_algorithm_invocation("x", "y", commit=False)
    finally:
        set_algorithm_invocation_provider(None)
    assert ld.alg_invocation_id() == "42"
    cur = FakeCursor()
    ld.set_cursor(cur)
    assert ld.cursor() is cur
    with pytest.raises(ValueError, match="must set update sql"):
        ld.update_variants()  # the reference driver's ADSP commit without build_update_sql raises the same
    ld.set_update_sql("UPDATE AnnotatedVDB.Variant v SET is_adsp_variant = true FROM (VALUES %s) AS d("
                      "record_primary_key, chromosome) WHERE v.chromosome = d.chromosome")
    ld.update_variants()  # empty buffer: a warning, nothing executed
    assert cur.executed == []
    ld.update_buffer().extend([("1:100:A:G", "chr1"), ("2:5:C:T:rs9", "chr2")])
    ld.update_variants()
    assert cur.executed == [("UPDATE AnnotatedVDB.Variant v SET is_adsp_variant = true FROM (VALUES "
                             "('1:100:A:G','chr1'),('2:5:C:T:rs9','chr2')) AS d(record_primary_key, chromosome) "
                             "WHERE v.chromosome = d.chromosome", None)]
    assert ld.update_buffer(sizeOnly=True) == 0
    # psycopg2's _split_sql rule: '%%' is a literal '%', every part keeps
    # the query's type (bytes here), and a second placeholder is refused
    ld.set_update_sql(b"UPDATE v SET note = 'x%%' FROM (VALUES %s) AS d(k, c)")
    ld.update_buffer().extend([("1:100:A:G", "chr1")])
    ld.update_variants()
    assert cur.executed[-1] == (b"UPDATE v SET note = 'x%' FROM (VALUES ('1:100:A:G','chr1')) AS d(k, c)", None)
    ld.set_update_sql("UPDATE v SET a = %s FROM (VALUES %s) AS d")
    ld.update_buffer().extend([("1:100:A:G", "chr1")])
    with pytest.raises(ValueError, match="more than one"):
        ld.update_variants()
    ld.update_buffer().clear()
    ld.set_batch_update()
    ld.update_buffer().write("UPDATE x;")
    ld.update_variants()
    assert cur.executed[-1] == ("UPDATE x;", None)
    ld.add_copy_str("a#b")
    ld.load_variants()
    assert cur.copies == [(ld._copy_sql, "a#b\n", 1024)] and ld.copy_buffer(sizeOnly=True) == 0


def test_host_engine_refuses_kernels(host_engine):
    """The host-only engine serves the per-call host entries only: a batch kernel
    entry raises NativeUnavailable (never a CPU substitute)."""
    import torch
    from annotatedvdb_amd import _native as N
    from annotatedvdb_amd.engine import default_engine
    eng = default_engine()
    assert eng.host_only
    with pytest.raises(N.NativeUnavailable):
        eng.bin_assign(torch.zeros(4, dtype=torch.uint8), torch.ones(4, dtype=torch.int32))


@pytest.mark.gpu
def test_batched_recipe_verbatim_vs_reference_load_driver(tmp_path):
    """The batched recipe (load_vcf_text per block of commitAfter lines, K0/K2/K5
    on the GPU) gives the cursor the reference's COPY text and the reference's
    .mapping file."""
    rows = [r for r in golden_rows() if r[1] is None]
    ns, db, mapping = run_recipe(tmp_path, ["setup", "batched"], [r[0] for r in rows], commit_after=500)
    check_against_golden(ns, db, mapping, rows, 500)
