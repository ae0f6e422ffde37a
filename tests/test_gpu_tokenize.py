"""K0 (avdb_vcf_count_lines / parse_lines / emit) on edge-case texts against the
reference-structured per-line parse (oracle.parse_vcf_line: VcfEntryParser
parse_entry + get_variant, vcf_parser.py:76-169) and the per-ALT explode with
the '.' skip (vcf_variant_loader.py:273-280): for every line K0 resolved on the
GPU (no host flag), its records — contig code, POS, REF and ALT bytes, refSNP
key, line and ALT index — must be the oracle's; every line's record count must
match its records.  Empty and one-byte texts, CRLF, lines longer than a parse
tile, a misaligned device view, a heap larger than the text, and the
chromosome map + pVCF header."""

import gzip
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _golden_text(name="vcf_lines.tsv.gz"):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as fh:
        fh.readline()
        lines = [line.rstrip("\n").split("\t")[0].replace("\\t", "\t") for line in fh]
    return ("\n".join(lines) + "\n").encode()


def _check(engine, text, opts=None, chrom_of=None, dev_text=None):
    """K0 vs the oracle; returns (lines, records, lines checked)."""
    from annotatedvdb_amd.chromosomes import CHROM_NAMES
    from annotatedvdb_amd.engine import VCF_COMMENT, VCF_HOST_FLAGS
    from oracle import avdb_oracle as O
    vb = engine.vcf_tokenize(dev_text if dev_text is not None else text, opts)
    n = vb.n_lines
    raw_lines = text.split(b"\n")
    if text.endswith(b"\n") or not text:
        raw_lines = raw_lines[:-1]
    assert n == len(raw_lines)
    L = vb.lines_host()
    b = vb.records
    nr = int(b.n)
    ro = vb.rec_off[: n + 1].cpu().numpy()
    assert nr == (int(ro[n]) if n else 0)
    chrom, pos = b.chrom[:nr].cpu().numpy(), b.pos[:nr].cpu().numpy().view(np.uint32)
    off, rl, al = b.allele_off[:nr].cpu().numpy(), b.ref_len[:nr].cpu().numpy(), b.alt_len[:nr].cpu().numpy()
    ext = b.ext_id[:nr].cpu().numpy().view(np.uint64)
    heap = b.heap.cpu().numpy().tobytes()
    rline, ralt = vb.rec_line[:nr].cpu().numpy(), vb.rec_alt[:nr].cpu().numpy()
    checked = 0
    for li, raw in enumerate(raw_lines):
        k0, k1 = int(ro[li]), int(ro[li + 1])
        assert k1 - k0 == int(L[li]["n_rec"]), li
        assert (rline[k0:k1] == li).all()
        fl = int(L[li]["flags"])
        if fl & (VCF_COMMENT | VCF_HOST_FLAGS) or k1 == k0 or int(L[li]["chrom"]) == 255:
            continue
        line = raw.decode().rstrip()
        if chrom_of is not None:
            f = line.split("\t")
            line = "\t".join([chrom_of(f[0])] + f[1:])
        v = O.parse_vcf_line(line)
        alts = [(i, a) for i, a in enumerate(v["alts"]) if a != "."]
        assert k1 - k0 == len(alts), line
        rs = v["ref_snp_id"]
        want_ext = int(rs[2:]) if rs else 0
        for r, (ai, a) in zip(range(k0, k1), alts):
            assert CHROM_NAMES[chrom[r]] == v["chromosome"] and pos[r] == v["position"], line
            assert heap[off[r]:off[r] + rl[r]] == v["ref"].encode(), line
            assert heap[off[r] + rl[r]:off[r] + rl[r] + al[r]] == a.encode(), line
            assert ext[r] == want_ext and ralt[r] == ai, line
        checked += 1
    return n, nr, checked


def _synth(n, seed):
    from annotatedvdb_amd import synth
    return synth.vcf_text(n, seed=seed)


def test_k0_golden_and_dbsnp_text(engine):
    _check(engine, _golden_text())
    n, _, checked = _check(engine, _golden_text("vcf_lines_100k.tsv.gz"))
    assert n == 102000 and checked > 95000
    t = _synth(60000, 31)
    n, nr, checked = _check(engine, t)
    assert n == t.count(b"\n") and nr > n and checked > 0.95 * n
    _check(engine, t[:-1])  # no trailing newline
    _check(engine, t[: len(t) // 2 + 7])  # ends inside a line


@pytest.mark.parametrize("text", [b"", b"\n", b"\n\n\n", b"a", b"#x\n", b"1\t5\t.\tA\tG\t.\t.\t.",
                                  b"1\t5\t.\tA\tG\t.\t.\t.\r\n\r\n2\t7\trs3\tC\tT,.\t.\t.\t.\n"])
def test_k0_tiny_texts(engine, text):
    _check(engine, text)


def test_k0_short_lines_and_empty_lines(engine):
    lines = [b"%d\t%d\t.\tA\tG\t.\t.\t." % (1 + i % 22, 1000 + i) for i in range(40000)]
    n, nr, checked = _check(engine, b"\n".join(lines) + b"\n")
    assert checked == n == nr == 40000
    _check(engine, b"\n" * 70000)


def test_k0_long_lines(engine):
    """Lines longer than a parse tile's staged text, a line of 70 kB, and
    REF/ALT fields of kilobytes."""
    base = _synth(3000, 37).split(b"\n")[:-1]
    long_info = b"1\t777\trs5\tACGT\tA,AC\t.\t.\tX=" + b"Y" * 9000
    huge = b"2\t888\t.\tC\tG,T\t.\t.\tZ=" + b"Q" * 70000
    wide = b"3\t999\trs1\t" + b"A" * 6000 + b"\t" + b"C" * 5000 + b",G\t.\t.\t."
    lines = base[:500] + [long_info] + base[500:1000] + [huge] + base[1000:2000] + [wide] + base[2000:]
    _check(engine, b"\n".join(lines) + b"\n")


def test_k0_misaligned_view(engine):
    t = _synth(5000, 41)
    d = torch.frombuffer(bytearray(b"xyz" + t), dtype=torch.uint8).to(engine.device)[3:]
    _check(engine, t, dev_text=d)


def test_k0_heap_larger_than_text(engine):
    ref = b"ACGT" * 500
    alts = b",".join([b"A"] * 400)
    line = b"4\t1234\trs9\t" + ref + b"\t" + alts + b"\t.\t.\t."
    t = b"\n".join([line] * 3) + b"\n"
    n, nr, checked = _check(engine, t)
    assert nr == 1200 and checked == 3


def test_k0_chrom_map_and_header(engine):
    from annotatedvdb_amd import synth
    lines = synth.vcf_text(4000, seed=43).decode().splitlines()
    acc = {str(i + 1): "NC_%06d.11" % (i + 1) for i in range(22)}
    back = {v: k for k, v in acc.items()}
    text = "\n".join("\t".join([acc.get(l.split("\t")[0], "NC_X")] + l.split("\t")[1:]) for l in lines) + "\n"
    cm = engine.chrom_map(back)
    opts = engine.vcf_opts(chrom_map=cm, min_fields=8)
    n, nr, checked = _check(engine, text.encode(), opts, chrom_of=lambda c: back.get(c, c))
    assert checked > 0.8 * n


def _starts_path(engine, text: bytes):
    """K0 through the line-starts pass: a count workspace of the minimum size and
    the original avdb_vcf_parse_lines entry (no window counts)."""
    import ctypes
    from annotatedvdb_amd import _native as N
    from annotatedvdb_amd.engine import VCF_LINE_DTYPE
    lib = engine.lib
    t = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(engine.device)
    nb = t.numel()
    s = N.stream_handle(engine.device)
    ws0 = torch.empty(N.VCF_COUNT_WORKSPACE_BYTES, dtype=torch.uint8, device=engine.device)
    nl = torch.zeros(1, dtype=torch.int64, device=engine.device)
    N.check("count", lib.avdb_vcf_count_lines(engine.ctx, N.ptr(t), nb, N.ptr(ws0), ws0.numel(), N.ptr(nl), s))
    n_lines = int(nl.item()) + (0 if text.endswith(b"\n") else 1)
    sz = ctypes.c_size_t()
    lib.avdb_vcf_workspace_size(nb, n_lines, ctypes.byref(sz))
    ws = torch.empty(int(sz.value), dtype=torch.uint8, device=engine.device)
    lines = torch.empty(max(1, n_lines) * VCF_LINE_DTYPE.itemsize, dtype=torch.uint8, device=engine.device)
    ro = torch.empty(n_lines + 1, dtype=torch.int64, device=engine.device)
    ho = torch.empty(n_lines + 1, dtype=torch.int64, device=engine.device)
    N.check("parse", lib.avdb_vcf_parse_lines(engine.ctx, N.ptr(t), nb, n_lines, N.ptr(ws0), N.ptr(ws), ws.numel(),
                                              N.ptr(lines), N.ptr(ro), N.ptr(ho), None, s))
    torch.cuda.synchronize()
    return n_lines, lines[: n_lines * 80].cpu().numpy(), ro.cpu().numpy(), ho.cpu().numpy()


@pytest.mark.parametrize("which", ["golden", "dbsnp", "short", "empty_lines", "long", "crlf_tail", "big"])
def test_k0_window_parse_equals_starts_pass(engine, which):
    """The window parse (line starts found in 24 KB windows, AVDB_VCF_PARSE_WIN_KB,
    from the count pass's per-window newline counts) gives the same line table and
    offsets as the line-starts pass, byte for byte, including lines across window
    edges and lines longer than a window.  "big" (~200 MB) makes each count
    sub-chunk (text / 4,096) hold several parse windows, so a window's first line
    index sums the windows before it in its sub-chunk, with 70 kB lines laid
    across window edges throughout."""
    if which == "golden":
        text = _golden_text()
    elif which == "dbsnp":
        text = _synth(60000, 53)
    elif which == "short":
        text = b"\n".join(b"%d\t%d\t.\tA\tG\t.\t.\t." % (1 + i % 22, 1000 + i) for i in range(50000)) + b"\n"
    elif which == "empty_lines":
        text = b"\n" * 90001 + b"1\t5\t.\tA\tG\t.\t.\t."
    elif which == "long":
        base = _synth(4000, 59).split(b"\n")[:-1]
        huge = b"2\t888\t.\tC\tG,T\t.\t.\tZ=" + b"Q" * 70000
        text = b"\n".join(base[:2000] + [huge] + base[2000:] + [huge]) + b"\n"
    elif which == "big":
        tile = _synth(60000, 67).split(b"\n")[:-1]
        huge = b"3\t4242\trs7\tG\tA,C\t.\t.\tZ=" + b"Q" * 70000
        parts = []
        for k in range(30):
            parts += tile[: 7000 + 997 * k] + [huge] + tile[7000 + 997 * k:]
        text = b"\n".join(parts) + b"\n"
        assert len(text) > 4096 * 25 * 1024  # sub-chunk (text / 4,096) > one 24 KB window
    else:
        text = _synth(20000, 61).replace(b"\n", b"\r\n")[:-3]
    n0, lines0, ro0, ho0 = _starts_path(engine, text)
    vb = engine.vcf_tokenize(text)
    assert vb.n_lines == n0
    assert (vb.lines[: n0 * 80].cpu().numpy() == lines0).all()
    assert (vb.rec_off[: n0 + 1].cpu().numpy() == ro0).all()
    assert (vb.heap_off[: n0 + 1].cpu().numpy() == ho0).all()


@pytest.mark.parametrize("which", ["golden", "dbsnp", "long", "big", "short", "edges", "empty", "no_final_nl",
                                   "blank", "huge_heap"])
@pytest.mark.parametrize("count_free", [True, False])
def test_k0_records_without_line_table(engine, which, count_free):
    """vcf_tokenize(want_lines=False) — no public line table: the count-free path
    (avdb_vcf_parse_local + avdb_vcf_emit_local: windows write their lines to slots
    of their own, one scan of the window totals) or, count_free=False, count ->
    parse -> avdb_vcf_emit_ws from 32-byte records — gives the same record SoA,
    allele heap, offsets and back-references as the tokenizer with the table.
    "short": 17-byte lines; "edges": blank lines, CRLF, lines of one field, a final
    line without '\n'; "blank": 8 M empty lines around dbSNP lines — more lines in a
    parse window than its 1,024 slots, so the count-free call falls back to the
    counted path; "huge_heap": a line whose records hold 9 MB of heap (> 2^23 bytes,
    past the slot's in-window offsets), so the count-free call falls back too."""
    if which == "short":
        text = b"".join(b"%d\t%d\t.\tA\tG\t.\t.\t.\n" % (1 + i % 9, 10 + i % 90) for i in range(300000))
    elif which == "golden":
        text = _golden_text()
    elif which == "dbsnp":
        text = _synth(60000, 71)
    elif which == "long":
        base = _synth(4000, 73).split(b"\n")[:-1]
        huge = b"2\t888\t.\tC\tG,T\t.\t.\tZ=" + b"Q" * 70000
        text = b"\n".join(base[:2000] + [huge] + base[2000:] + [huge]) + b"\n"
    elif which == "edges":
        base = _synth(3000, 83).split(b"\n")[:-1]
        odd = [b"", b"\r", b"1\t77\t.\tA\tG\t.\t.\t.\r", b"X", b"\t\t", b"2\t9\t.\tA\tC,.,T\t.\t.\tRS=5"]
        text = b"\n".join(x for k, line in enumerate(base) for x in ((line, odd[k % len(odd)]) if k % 7 == 0
                                                                      else (line,)))
    elif which == "empty":
        text = b""
    elif which == "blank":
        text = _synth(2000, 91) + b"\n" * 8_000_000 + _synth(2000, 93)
    elif which == "huge_heap":
        big = b"1\t5\t.\t" + b"A" * 90000 + b"\t" + b",".join([b"C"] * 100) + b"\t.\t.\t."
        text = _synth(2000, 95) + big + b"\n" + _synth(2000, 97)
    elif which == "no_final_nl":
        text = _synth(5000, 89).rstrip(b"\n")
    else:
        tile = _synth(60000, 79).split(b"\n")[:-1]
        text = b"\n".join(tile * 25) + b"\n"
    a = engine.vcf_tokenize(text)
    b = engine.vcf_tokenize(text, want_lines=False, count_free=count_free)
    assert engine.last_vcf_path == ("counted" if which in ("blank", "huge_heap") or not count_free else "local")
    assert b.lines is None and a.n_lines == b.n_lines and a.records.n == b.records.n
    assert torch.equal(a.rec_off, b.rec_off) and torch.equal(a.heap_off, b.heap_off)
    for f in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "ext_id"):
        assert torch.equal(getattr(a.records, f), getattr(b.records, f)), f
    nh = int(a.heap_off[a.n_lines])  # (the heap buffer holds at least one byte)
    assert torch.equal(a.records.heap[:nh], b.records.heap[:nh])
    assert torch.equal(a.rec_line, b.rec_line) and torch.equal(a.rec_alt, b.rec_alt)


def _same_records(engine, text, opts=None, path="local"):
    """The count-free records path (vcf_tokenize(want_lines=False)) against the
    tokenizer with its line table, on the same text (bytes or a device tensor)."""
    a = engine.vcf_tokenize(text, opts)
    b = engine.vcf_tokenize(text, opts, want_lines=False)
    assert engine.last_vcf_path == path
    assert a.n_lines == b.n_lines and a.records.n == b.records.n
    assert torch.equal(a.rec_off, b.rec_off) and torch.equal(a.heap_off, b.heap_off)
    for f in ("chrom", "pos", "allele_off", "ref_len", "alt_len", "ext_id"):
        assert torch.equal(getattr(a.records, f), getattr(b.records, f)), f
    nh = int(a.heap_off[a.n_lines])
    assert torch.equal(a.records.heap[:nh], b.records.heap[:nh])
    assert torch.equal(a.rec_line, b.rec_line) and torch.equal(a.rec_alt, b.rec_alt)


def test_k0_count_free_opts_views_and_wide_alleles(engine):
    """The count-free path with a chromosome map and header width (avdb_vcf_opts), on
    a misaligned device view, with REF / ALT of kilobytes (lines parsed from global
    memory, 17 KB of allele bytes in one window's heap slots), and the tiny texts.  A
    window whose records hold more allele bytes than its 24 KB of heap slots (three
    lines of a 2 KB REF x 400 ALTs: 2.4 MB of heap from 6 KB of text) takes the
    counted path, with the same records."""
    from annotatedvdb_amd import synth
    lines = synth.vcf_text(4000, seed=43).decode().splitlines()
    acc = {str(i + 1): "NC_%06d.11" % (i + 1) for i in range(22)}
    back = {v: k for k, v in acc.items()}
    text = "\n".join("\t".join([acc.get(l.split("\t")[0], "NC_X")] + l.split("\t")[1:]) for l in lines) + "\n"
    _same_records(engine, text.encode(), engine.vcf_opts(chrom_map=engine.chrom_map(back), min_fields=8))
    t = _synth(5000, 41)
    _same_records(engine, torch.frombuffer(bytearray(b"xyz" + t), dtype=torch.uint8).to(engine.device)[3:])
    base = _synth(3000, 37).split(b"\n")[:-1]
    wide = b"3\t999\trs1\t" + b"A" * 6000 + b"\t" + b"C" * 5000 + b",G\t.\t.\t."
    many = b"4\t1234\trs9\t" + b"ACGT" * 500 + b"\t" + b",".join([b"A"] * 400) + b"\t.\t.\t."
    _same_records(engine, b"\n".join(base[:1000] + [wide] + base[1000:]) + b"\n")
    _same_records(engine, b"\n".join(base[:1000] + [wide] + base[1000:2000] + [many] * 3 + base[2000:]) + b"\n",
                  path="counted")
    for tiny in (b"\n", b"\n\n\n", b"a", b"#x\n", b"1\t5\t.\tA\tG\t.\t.\t.",
                 b"1\t5\t.\tA\tG\t.\t.\t.\r\n\r\n2\t7\trs3\tC\tT,.\t.\t.\t.\n"):
        _same_records(engine, tiny)


@pytest.mark.parametrize("pad", [0, 120])
def test_k0_info_refsnp_edges(engine, pad):
    """The INFO refSNP scan in K0's staged window parse (the cases of
    test_percall_host.INFO_RS_CASES at eight INFO alignments, plus sample columns
    after INFO, repeated so lines sit at every window position): EXT_HOST exactly
    where the reference would not give rs<int>, else the record's refSNP key.
    pad 0: short lines, several parse rounds per window (the gathered INFO scan);
    pad 120: a FILTER of 120 bytes, one round per window (each line's last "RS"
    candidate from the workgroup's bitmap pass, the scan only where it cannot
    decide)."""
    from annotatedvdb_amd.engine import VCF_EXT_HOST, VCF_INFO_RS
    from test_percall_host import info_rs_lines
    cases = [(line.replace("\t.\t.\t", "\t.\t%s\t" % ("F" * pad), 1) if pad else line, w)
             for line, w in info_rs_lines()]
    # a dbSNP-shaped line between cases shifts the following case by one byte per repeat
    filler = [b"1\t%d\trs1\tA\tG\t.\t.\t%s" % (200 + k, b"Q" * (1 + k % 64)) for k in range(len(cases) * 3)]
    lines, want = [], []
    for k in range(len(cases) * 3):
        line, w = cases[k % len(cases)]
        lines += [line.encode(), filler[k]]
        want += [w, 1]
    text = b"\n".join(lines) + b"\n"
    vb = engine.vcf_tokenize(text)
    L = vb.lines_host()
    ro = vb.rec_off[: vb.n_lines + 1].cpu().numpy()
    ext = vb.records.ext_id[: int(vb.records.n)].cpu().numpy().view(np.uint64)
    assert vb.n_lines == len(lines)
    for li, w in enumerate(want):
        fl = int(L[li]["flags"])
        if w is None:
            assert fl & VCF_EXT_HOST and fl & VCF_INFO_RS, lines[li]
            continue
        assert not fl & VCF_EXT_HOST, lines[li]
        assert int(ro[li + 1]) - int(ro[li]) == 1 and int(ext[ro[li]]) == w, (lines[li], int(ext[ro[li]]))
        assert bool(fl & VCF_INFO_RS) == (w != 0 and li % 2 == 0), lines[li]
