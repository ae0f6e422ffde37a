"""K8h (``avdb_small_prep_host``): the library's per-call host entry — the
kernels' own record arithmetic (infer_end / classify / bin_path / display_json,
compiled for both sides) serving one ``find_bin_index`` miss or one
``parse_variant`` line — against the reference's own outputs (golden files).

It needs no GPU: a context made with device -1 and host arrays.  The GPU
tests (test_gpu_dropin.py) check the same entry and K8 through the drop-in
classes and against each other."""

import ctypes
import gzip
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

N = pytest.importorskip("annotatedvdb_amd._native")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("libavdb_hip.so not built")
    return N.load_library()


@pytest.fixture(scope="module")
def ctx(lib):
    from annotatedvdb_amd.chromosomes import length_table
    lens = length_table("GRCh38")
    h = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(lens))(*lens)
    N.check("avdb_ctx_create", lib.avdb_ctx_create(-1, arr, len(lens), ctypes.byref(h)))
    yield h
    lib.avdb_ctx_destroy(h)


def k8h(lib, ctx, chrom, pos, refs=None, alts=None, ends=None, ext=None, want=7, max_seq_len=50,
        caps=(1 << 22, 1 << 22, 1 << 23)):
    """One avdb_small_prep_host call over numpy arrays; returns a dict."""
    n = len(pos)
    keep = []

    def arr(x, dt):
        a = np.ascontiguousarray(np.asarray(x, dtype=dt))
        keep.append(a)
        return a.ctypes.data

    b = N.SmallBatch()
    b.chrom, b.pos = arr(chrom, np.uint8), arr(pos, np.uint32)
    if refs is not None:
        rl = np.array([len(r) for r in refs], dtype=np.uint32)
        al = np.array([len(a) for a in alts], dtype=np.uint32)
        off = np.zeros(n, dtype=np.uint64)
        if n:
            off[1:] = np.cumsum(rl.astype(np.uint64) + al)[:-1]
        heap = b"".join(r + a for r, a in zip(refs, alts)) or b"\0"
        b.allele_off, b.ref_len, b.alt_len = arr(off, np.uint64), arr(rl, np.uint32), arr(al, np.uint32)
        b.heap = arr(np.frombuffer(heap, dtype=np.uint8), np.uint8)
        b.heap_bytes = len(heap)
        ks, ds = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
        keep += [ks, ds]
        b.key_state, b.disp_state = ks.ctypes.data, ds.ctypes.data
        if ext is not None:
            b.ext_id = arr(ext, np.uint64)
    else:
        b.end_in = arr(ends, np.uint32)
        want &= 1
    eo, co, so = np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(n, np.uint8)
    offs = np.zeros(3 * (n + 1), np.uint32)
    texts = [np.zeros(c, np.uint8) for c in caps]
    ov = np.zeros(2, np.uint32)
    keep += [eo, co, so, offs, ov] + texts
    b.end_out, b.code, b.status, b.off_out, b.overflow = (eo.ctypes.data, co.ctypes.data, so.ctypes.data,
                                                          offs.ctypes.data, ov.ctypes.data)
    for k in range(3):
        b.text_out[k] = texts[k].ctypes.data
        b.text_cap[k] = caps[k]
    b.n, b.max_seq_len, b.want = n, max_seq_len, want
    N.check("avdb_small_prep_host", lib.avdb_small_prep_host(ctx, ctypes.byref(b)))
    out = {"end": eo, "code": co, "status": so, "overflow": int(ov[0])}
    if refs is not None:
        out["key_state"], out["disp_state"] = ks, ds
    for k, name in enumerate(("path", "key", "display")):
        if not (want >> k) & 1:
            continue
        o = offs[k * (n + 1): (k + 1) * (n + 1)]
        raw = texts[k][: int(o[n])].tobytes().decode("ascii")
        out[name] = [raw[o[i]:o[i + 1]] if o[i + 1] > o[i] else None for i in range(n)]
    return out


def read_tsv(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as fh:
        header = fh.readline().rstrip("\n").split("\t")
        return [dict(zip(header, line.rstrip("\n").split("\t"))) for line in fh]


def codes(names):
    from annotatedvdb_amd.chromosomes import bin_index_chrom_code
    return [min(bin_index_chrom_code(c), 255) for c in names]


def test_k8h_bin_queries_vs_reference(lib, ctx):
    """36,147 (chrom, start, end) -> path answers of the reference BinIndex over
    the verbatim-generated BinIndexRef (TypeError rows: no path)."""
    rows = read_tsv("bin_queries.tsv.gz")
    for lo in range(0, len(rows), 20000):
        part = rows[lo:lo + 20000]
        res = k8h(lib, ctx, codes([r["chrom"] for r in part]), [int(r["start"]) for r in part],
                  ends=[int(r["end"] or r["start"]) for r in part])
        for r, p in zip(part, res["path"]):
            assert (p or "TypeError") == r["bin_index"], r


def test_k8h_end_inference_vs_reference(lib, ctx):
    """40,000 adversarial allele pairs: end = VariantAnnotator.infer_variant_end_location."""
    rows = read_tsv("end_infer.tsv.gz")
    ch = [r["metaseq_id"].split(":")[0] for r in rows]
    res = k8h(lib, ctx, codes(ch), [int(r["pos"]) for r in rows], refs=[r["ref"].encode() for r in rows],
              alts=[r["alt"].encode() for r in rows], want=0)
    assert res["end"].astype(np.int64).tolist() == [int(r["end"]) for r in rows]


def test_k8h_display_attributes_vs_reference(lib, ctx):
    """6,000 reference get_display_attributes dicts as json.dumps text, key order included."""
    rows = read_tsv("display_attrs.tsv.gz")
    res = k8h(lib, ctx, codes([r["chrom"] for r in rows]), [int(r["pos"]) for r in rows],
              refs=[r["ref"].encode() for r in rows], alts=[r["alt"].encode() for r in rows], want=4)
    for r, d in zip(rows, res["display"]):
        assert d == json.dumps(json.loads(r["attributes"])), r


def test_k8h_c1_prefix_vs_reference(lib, ctx):
    """The first 100,000 C1 records: end, ltree path and primary key equal the
    reference's VariantAnnotator / BinIndex / VariantPKGenerator output."""
    from annotatedvdb_amd import synth
    with gzip.open(os.path.join(GOLDEN, "c1_prefix.tsv.gz"), "rt") as fh:
        fh.readline()
        rows = [ln.rstrip("\n").split("\t") for ln in fh]
    d = synth.np_c1(synth.C1_N, seed=1)
    n = len(rows)
    heap = d["heap"].tobytes()
    o, rl, al = d["allele_off"][:n].tolist(), d["ref_len"][:n].tolist(), d["alt_len"][:n].tolist()
    refs = [heap[x:x + y] for x, y in zip(o, rl)]
    alts = [heap[x + y:x + y + z] for x, y, z in zip(o, rl, al)]
    for lo in range(0, n, 25000):
        sl = slice(lo, lo + 25000)
        res = k8h(lib, ctx, d["chrom"][sl], d["pos"][sl], refs=refs[sl], alts=alts[sl],
                  ext=d["ext_id"][sl].astype(np.uint64), want=3)
        for i, (pk, e, path) in enumerate(rows[sl]):
            assert res["key"][i] == pk and str(res["end"][i]) == e and res["path"][i] == path, lo + i


def test_k8h_kats(lib, ctx):
    """SURVEY A.5 / database/variant.py:162-163 known answers."""
    kats = json.load(open(os.path.join(GOLDEN, "kat.json")))
    kats = [k for k in kats if "primary_key" in k and len(k["ref"]) + len(k["alt"]) <= 50]
    res = k8h(lib, ctx, codes([k["chrom"] for k in kats]), [k["pos"] for k in kats],
              refs=[k["ref"].encode() for k in kats], alts=[k["alt"].encode() for k in kats],
              ext=[int(k["rsid"][2:]) if k.get("rsid") else 0 for k in kats], want=3)
    for k, e, p, key in zip(kats, res["end"], res["path"], res["key"]):
        assert (int(e), p, key) == (k["end"], k["bin_index"], k["primary_key"]), k


def test_k8h_states_and_overflow(lib, ctx):
    """Key states (':' in an allele, non-ASCII, long, interned ids), unmappable
    records and a text stream over its capacity."""
    refs = [b"A", b"A:C", b"A\xc3\xa9", b"A" * 40, b"G"]
    alts = [b"T", b"T", b"T", b"C" * 11, b"C"]
    res = k8h(lib, ctx, [0, 0, 0, 0, 200], [100, 100, 100, 100, 100], refs=refs, alts=alts,
              ext=[5, 0, 0, 0, 0], want=7)
    assert res["key_state"].tolist() == [N.KEY_OK, N.KEY_HOST, N.KEY_HOST, N.KEY_NEED_DIGEST, N.KEY_HOST]
    assert res["disp_state"].tolist() == [0, 0, 1, 0, 0]
    assert res["key"][0] == "1:100:A:T:rs5" and res["key"][1] is None
    assert res["status"][4] == N.STATUS_UNKNOWN_CHROM and res["path"][4] is None
    small = k8h(lib, ctx, [0, 0], [100, 200], refs=[b"A", b"A"], alts=[b"T", b"G"], want=7, caps=(100, 8, 4096))
    assert small["overflow"] == N.SMALL_PATH | N.SMALL_KEY


def test_k8h_argument_checks(lib, ctx):
    b = N.SmallBatch()
    assert lib.avdb_small_prep_host(ctx, ctypes.byref(b)) == N.AVDB_EINVAL
    assert lib.avdb_small_prep_host(None, ctypes.byref(b)) == N.AVDB_EINVAL


def load_rows():
    with gzip.open(os.path.join(GOLDEN, "vcf_load.tsv.gz"), "rt") as fh:
        fh.readline()
        out = []
        for line in fh:
            raw, err, mapping, copy = line.rstrip("\n").split("\t")
            out.append((raw.replace("\\t", "\t"), err or None, json.loads(mapping), json.loads(copy)))
        return out


def test_k5h_lines_vs_reference_load_driver(lib, ctx):
    """Every line of the reference load-driver fixture (4,100 lines, dbSNP datasource):
    a line K5h renders gives exactly the reference's COPY rows and .mapping line; a
    line the reference raised on, or that needs the host, is never rendered."""
    from annotatedvdb_amd.chromosomes import length_table  # noqa: F401
    rows = load_rows()
    rendered = 0
    for raw, err, mapping, copy in rows:
        b = raw.encode("utf-8")
        opts = N.FormatOpts(b"1", 50, 0)
        res = N.LineResult()
        cb, mb = ctypes.create_string_buffer(1 << 16), ctypes.create_string_buffer(1 << 16)
        N.check("k5h", lib.avdb_vcf_line_host(ctx, b, len(b), ctypes.byref(opts), None, cb, 1 << 16, mb, 1 << 16,
                                              ctypes.byref(res)))
        if res.state != N.LINE_GPU:
            continue
        assert err is None, (raw, err)
        rendered += 1
        got_copy = cb.raw[:res.copy_bytes].decode().splitlines()
        got_map = mb.raw[:res.map_bytes].decode()
        assert got_copy == copy, raw
        assert got_map == "".join(m + "\n" for m in mapping), raw
        assert res.n_rows == len(copy)
    assert rendered > 2000, rendered


def test_k5h_edges(lib, ctx):
    """Comment lines are SKIP; short, non-ASCII, unknown-contig and long-allele
    lines go to the caller (HOST); buffers too small give ERANGE with the sizes."""
    def run(b, cap=1 << 12):
        opts = N.FormatOpts(b"7", 50, 0)
        res = N.LineResult()
        cb, mb = ctypes.create_string_buffer(cap), ctypes.create_string_buffer(cap)
        rc = lib.avdb_vcf_line_host(ctx, b, len(b), ctypes.byref(opts), None, cb, cap, mb, cap, ctypes.byref(res))
        return rc, res, cb.raw[:res.copy_bytes].decode(errors="replace"), mb.raw[:res.map_bytes].decode(errors="replace")
    assert run(b"#CHROM\tPOS")[1].state == N.LINE_SKIP
    assert run(b"1\t100\t.\tA")[1].state == N.LINE_HOST
    assert run(b"chrUn\t100\t.\tA\tG\t.\t.\t.")[1].state == N.LINE_HOST
    assert run(b"1\t100\t.\tA\t" + b"G" * 60 + b"\t.\t.\t.")[1].state == N.LINE_HOST
    rc, res, c, m = run(b"1\t100\trs5\tA\tG,.\t.\t.\tRS=5")
    assert rc == 0 and res.state == N.LINE_GPU and res.n_skip == 1 and res.n_rows == 1
    assert c.startswith("chr1#1:100:A:G:rs5#100#1:100:A:G#chr1.L1.B1") and c.endswith("#7#rs5#True#" + c.split("#")[8]
                                                                                       + "#NULL\n")
    assert m.startswith("1:100:A:G,.\t[{'primary_key': '1:100:A:G:rs5', 'bin_index': 'chr1.L1.B1")
    rc, res, _, _ = run(b"1\t100\trs5\tA\tG\t.\t.\tRS=5", cap=16)
    assert rc == N.AVDB_ERANGE and res.copy_bytes > 16
    opts = N.FormatOpts(b"1", 50, 0)
    assert lib.avdb_vcf_line_host(None, b"x", 1, ctypes.byref(opts), None, None, 0, None, 0,
                                  ctypes.byref(N.LineResult())) == N.AVDB_EINVAL


def test_format_opts_struct_size_checked(lib, ctx):
    """avdb_format_opts carries its size (ABI 2): a caller built against another
    layout is refused instead of read past its struct."""
    opts = N.FormatOpts(b"1", 50, 0)
    opts.struct_size = ctypes.sizeof(N.FormatOpts) - 8
    res = N.LineResult()
    b = b"1\t100\trs5\tA\tG\t.\t.\tRS=5"
    cb = ctypes.create_string_buffer(4096)
    assert lib.avdb_vcf_line_host(ctx, b, len(b), ctypes.byref(opts), None, cb, 4096, cb, 4096,
                                  ctypes.byref(res)) == N.AVDB_EINVAL
    assert b"struct_size" in lib.avdb_last_error()


def test_k5h_chromosome_map_and_pvcf_header_vs_reference(lib, ctx):
    """K5h with a ChromosomeMap (RefSeq accessions as CHROM) and a pVCF header
    (FORMAT + a sample column) against the reference loader run with the same map
    and header (chrmap_load.tsv.gz, make_golden.py --only chrmap): every line K5h
    renders is byte-exact; lines the reference raised on (KeyError for unmapped /
    numeric CHROM, IndexError for lines short of the header, ...) are never rendered."""
    from annotatedvdb_amd.engine import ChromMap
    from annotatedvdb_amd.parsers import ChromosomeMap

    class _Eng:  # what ChromMap needs of an engine
        pass
    e = _Eng()
    e.lib, e.ctx = lib, ctx
    cmap = ChromMap(e, ChromosomeMap(os.path.join(GOLDEN, "chrmap_grch38.tsv")).chromosome_map())
    vo = N.VcfOpts(10, cmap.handle)
    with gzip.open(os.path.join(GOLDEN, "chrmap_load.tsv.gz"), "rt") as fh:
        fh.readline()
        rows = [ln.rstrip("\n").split("\t") for ln in fh]
    rendered = 0
    for raw, err, mapping, copy in rows:
        b = raw.replace("\\t", "\t").encode()
        opts, res = N.FormatOpts(b"1", 50, 0), N.LineResult()
        cb, mb = ctypes.create_string_buffer(1 << 16), ctypes.create_string_buffer(1 << 16)
        N.check("k5h", lib.avdb_vcf_line_host(ctx, b, len(b), ctypes.byref(opts), ctypes.byref(vo), cb, 1 << 16,
                                              mb, 1 << 16, ctypes.byref(res)))
        if res.state != N.LINE_GPU:
            continue
        assert not err, (raw, err)
        rendered += 1
        assert cb.raw[:res.copy_bytes].decode().splitlines() == json.loads(copy), raw
        assert mb.raw[:res.map_bytes].decode() == "".join(m + "\n" for m in json.loads(mapping)), raw
    assert rendered > 0.8 * sum(1 for r in rows if not r[1]), rendered
    cmap.close()


def test_k8a_variant_annotator_vs_reference(lib):
    """The drop-in VariantAnnotator (one K8a call per instance through the
    avdb_percall binding) on every golden pair: end, normalized alleles (both
    snvDivMinus forms), metaseq id; and every reference display-attribute dict,
    key order included."""
    from annotatedvdb_amd.variant_annotator import VariantAnnotator
    for r in read_tsv("end_infer.tsv.gz"):
        va = VariantAnnotator(r["ref"], r["alt"], "1", int(r["pos"]))
        assert va.infer_variant_end_location() == int(r["end"]), r
        lcp = int(r["lcp"])
        snv = len(r["ref"]) == 1 and len(r["alt"]) == 1
        want = (r["ref"], r["alt"]) if snv or lcp == 0 else (r["ref"][lcp:], r["alt"][lcp:])
        assert va.get_normalized_alleles() == want, r
        if not snv and lcp:
            assert va.get_normalized_alleles(True) == (want[0] or "-", want[1] or "-"), r
        assert va.get_metaseq_id() == r["metaseq_id"]
    for r in read_tsv("display_attrs.tsv.gz"):
        d = VariantAnnotator(r["ref"], r["alt"], r["chrom"], int(r["pos"])).get_display_attributes()
        assert json.dumps(d) == r["attributes"], r


def test_k8a_variant_annotator_edges(lib):
    """Quirks the reference has and the binding's edges."""
    from annotatedvdb_amd.variant_annotator import VariantAnnotator
    from oracle import avdb_oracle as O
    assert VariantAnnotator("AT", "AT", "1", 100).infer_variant_end_location() == 99  # end < start
    assert VariantAnnotator("ATA", "ATA", "1", 100).infer_variant_end_location() == 102  # palindrome
    assert VariantAnnotator("A", "<DEL>", "1", 100).infer_variant_end_location() == 101
    assert VariantAnnotator("A", "*", "1", 100).infer_variant_end_location() == 100
    big = 10 ** 12  # a Python int beyond u32: the end is position + the library's relative end
    assert VariantAnnotator("CAGT", "CG", "1", big).infer_variant_end_location() == big + 3
    assert VariantAnnotator("CAGT", "CG", "1", "100").infer_variant_end_location() == 103
    with pytest.raises(ValueError):
        VariantAnnotator("CAGT", "CG", "1", "x").infer_variant_end_location()
    with pytest.raises(ValueError):
        VariantAnnotator("CÅ", "C", "1", 100).infer_variant_end_location()
    # a display text beyond the binding's stack buffer (inversions keep the whole allele)
    inv = "ACGT" * 700
    ref, alt = inv, inv[::-1]
    want = O.display_attributes("7", 5000, ref, alt)
    got = VariantAnnotator(ref, alt, "7", 5000).get_display_attributes()
    assert got == want and list(got) == list(want)
    sub = "A" * 1500
    want = O.display_attributes("7", 5000, "G" + sub, "GC" + sub[1:] + "T")
    assert VariantAnnotator("G" + sub, "GC" + sub[1:] + "T", "7", 5000).get_display_attributes() == want
    d = VariantAnnotator("CAG", "C", "chrUn_KI270302v1", 100).get_display_attributes()
    assert d["normalized_metaseq_id"] == "chrUn_KI270302v1:100:AG:-"
    assert list(d) == ["location_start", "location_end", "normalized_metaseq_id", "variant_class",
                       "variant_class_abbrev", "display_allele", "sequence_allele"]


# INFO refSNP cases (vcf_parser.py:155-169 via parse_info, :38-52): the last entry
# whose key is exactly "RS" decides; an int value gives rs<value>, anything the
# reference coerces otherwise (bare key, float, text, 0, > 18 digits) is the host's.
# value: the refSNP number, 0 = no refSNP (NULL), None = the line goes to the host
INFO_RS_CASES = [
    ("RS=5", 5), ("RS=123;RSPOS=7", 123), ("RSPOS=7;RS=123", 123), ("RS=1;RS=2", 2),
    ("RS=12;RS", None), ("RS", None), ("RS=", None), ("RS=0", None), ("RS=007", 7),
    ("RS=12a", None), ("RS=5.0", None), ("X=1;RS=99;Y", 99), ("RSX=4", 0), ("xRS=4", 0),
    ("VC=SNV;FREQ=a:0.1,0.2", 0), ("RS=12345678901234567", 12345678901234567),
    ("RS=123456789012345678", 123456789012345678), ("RS=1234567890123456789", None),
    ("RS=1234567890123456;VC=SNV", 1234567890123456), ("RS=123456789012345", 123456789012345),
    ("RS=55;dbSNPBuildID=151;SSR=0;VC=SNV;FREQ=1000Genomes:0.9876,0.0124", 55), ("RS=5 ", 5),
    ("RS=5=6", None), ("R=1;S=2", 0), ("RS=8;R", 8), (".", 0),
]


def info_rs_lines():
    """(line, expected) with every case at eight alignments of the INFO field, and
    once with sample columns after INFO."""
    out = []
    for info, want in INFO_RS_CASES:
        for s in range(8):
            pre = ("Z" * s + "=1;") if s else ""
            out.append(("1\t100\t.\tA\tG\t.\t.\t%s%s" % (pre, info), want))
        out.append(("1\t100\t.\tA\tG\t.\t.\t%s\tGT\t0/1" % info.rstrip(), want))
    return out


def test_k5h_info_refsnp_edges(lib, ctx):
    """The INFO refSNP scan (one SWAR pass over the INFO words) on the per-line
    host entry: rs<value> in the COPY row's ref_snp_id column, NULL without one,
    and the host for every value the reference would coerce to something else."""
    for line, want in info_rs_lines():
        b = line.encode()
        opts = N.FormatOpts(b"1", 50, 0)
        res = N.LineResult()
        cb, mb = ctypes.create_string_buffer(1 << 14), ctypes.create_string_buffer(1 << 14)
        N.check("k5h", lib.avdb_vcf_line_host(ctx, b, len(b), ctypes.byref(opts), None, cb, 1 << 14, mb, 1 << 14,
                                              ctypes.byref(res)))
        if want is None:
            assert res.state == N.LINE_HOST, line
            continue
        assert res.state == N.LINE_GPU, line
        col = cb.raw[:res.copy_bytes].decode().split("#")[6]
        assert col == ("rs%d" % want if want else "NULL"), (line, col)


def test_dropin_bin_index_replays_reference_sequence():
    """The drop-in BinIndex (its one-bin L13 cache over K1h, the library's host
    entry; a host-only engine, no GPU) replays the reference's whole loader-order
    sequence (tests/golden/bin_sequence.tsv.gz, ~100,000 queries through one
    verbatim BinIndex): every answer in order, end < start records after cache
    hits and TypeErrors (empty cache afterwards) included."""
    from annotatedvdb_amd.bin_index import BinIndex
    rows = read_tsv("bin_sequence.tsv.gz")
    bi = BinIndex(None, verbose=False, device="host")
    for r in rows:
        end = int(r["end"]) if r["end"] else None
        try:
            got = bi.find_bin_index(r["chrom"], int(r["start"]), end)
        except TypeError:
            got = "TypeError"
        assert got == r["bin_index"], r


def test_k8h_bin_queries_wide_vs_reference(lib, ctx):
    """200,000 reference answers over all 25 contigs, spans to 1 Mb (K8h per record)."""
    rows = read_tsv("bin_queries_wide.tsv.gz")
    for lo in range(0, len(rows), 50000):
        part = rows[lo:lo + 50000]
        res = k8h(lib, ctx, codes([r["chrom"] for r in part]), [int(r["start"]) for r in part],
                  ends=[int(r["end"] or r["start"]) for r in part])
        for r, p in zip(part, res["path"]):
            assert (p or "TypeError") == r["bin_index"], r
