"""Host-side logic on CPU: VCF text -> records (vs the reference's own loader
output in tests/golden/vcf_lines.tsv.gz), record packing, shard planning."""

import gzip
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from annotatedvdb_amd import shard
from annotatedvdb_amd.chromosomes import CHROM_NAMES, GRCH38_LENGTHS, bin_index_chrom_code, length_table
from annotatedvdb_amd.parsers import VcfEntryParser
from oracle import avdb_oracle as O


def golden_lines(name="vcf_lines.tsv.gz"):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as fh:
        fh.readline()
        for line in fh:
            raw, mapping, copy5, ends = line.rstrip("\n").split("\t")
            yield raw.replace("\\t", "\t"), json.loads(mapping), json.loads(copy5), json.loads(ends)


def oracle_path(chrom, start, end):
    code = bin_index_chrom_code(chrom)
    if code >= 25:
        return None
    c, _ = O.bin_code(length_table()[code], start, end)
    return None if c == O.BIN_NONE else O.format_bin_path(CHROM_NAMES[code], c)


@pytest.mark.parametrize("name,least", [("vcf_lines.tsv.gz", 7000), ("vcf_lines_100k.tsv.gz", 95000)])
def test_vcf_lines_host_parse_plus_oracle_reproduce_reference_loader(name, least):
    """VcfEntryParser (host) + oracle arithmetic reproduce the reference
    loader's mapping, COPY prefix and end coordinates on every golden line."""
    n = 0
    for raw, mapping, copy5, ends in golden_lines(name):
        entry = VcfEntryParser(raw)
        try:
            v = entry.get_variant(namespace=True)
        except Exception as err:  # noqa: BLE001
            assert "__error__" in mapping, (raw, err)
            continue
        exp_rows = []
        got_map = []
        error = None
        for k, alt in enumerate(v.alt_alleles):
            if alt == ".":
                continue
            metaseq = O.metaseq_id(v.chromosome, v.position, v.ref_allele, alt)
            if len(metaseq.split(":")) != 4:
                error = "ValueError"
                break
            end, _ = O.infer_end(v.position, v.ref_allele, alt)
            assert end == ends[k]
            path = oracle_path(v.chromosome, v.position, end)
            if path is None:
                error = "TypeError"
                break
            pk = O.primary_key(v.chromosome, v.position, v.ref_allele, alt, v.ref_snp_id)
            got_map.append({"primary_key": pk, "bin_index": path})
            exp_rows.append("#".join(["chr" + v.chromosome, pk, str(v.position), metaseq, path]))
        if error:
            assert mapping == {"__error__": error}, raw
        else:
            assert mapping == {v.id: got_map}, raw
            assert copy5 == exp_rows
        n += 1
    assert n > least


def test_pack_records_layout():
    from annotatedvdb_amd.engine import ExtIdInterner, pack_records
    it = ExtIdInterner()
    keys = [it.key(x) for x in [None, "rs5", "rs0", "rs5", "foo", "rs007", "foo"]]
    assert keys[0] == 0 and keys[1] == keys[3] == 5
    assert keys[4] == keys[6] and keys[4] >> 63 == 1 and keys[2] != keys[5] and keys[2] >> 63 == 1
    assert it.to_str(keys[4]) == "foo" and it.to_str(5) == "rs5"
    b = pack_records([0, 1, 2], [10, 20, 30], [b"A", b"CAT", b""], [b"G", b"C", b"TT"], keys[:3])
    heap = b.heap.numpy().tobytes()
    off = b.allele_off.numpy()
    rl = b.ref_len.numpy()
    al = b.alt_len.numpy()
    assert heap == b"AGCATCTT"
    assert list(off) == [0, 2, 6] and list(rl) == [1, 3, 0] and list(al) == [1, 1, 2]
    assert b.ext_id.numpy()[2] < 0  # 2^63|k stored as int64 bit pattern


def test_shard_plan_covers_genome_once():
    lens = length_table()
    for w in (1, 2, 4, 8):
        plan = shard.plan(w)
        cover = {}
        for ps in plan:
            for p in ps:
                cover.setdefault(p.chrom, []).append((p.lo, p.hi))
        for c, L in enumerate(lens):
            iv = sorted(cover[c])
            assert iv[0][0] == 0 and iv[-1][1] == L
            assert all(a[1] == b[0] for a, b in zip(iv, iv[1:]))
        assert shard.imbalance(plan) < 1.02
    plan = shard.plan(8)
    assert shard.shard_of(plan, 0, 1) >= 0
    assert shard.shard_of(plan, 24, GRCH38_LENGTHS["M"]) >= 0


def test_synthetic_numpy_generators_shape():
    from annotatedvdb_amd import synth
    c, s = synth.np_point_snvs(10000, seed=1)
    assert np.all(np.diff(c.astype(np.int64) * 2**32 + s) >= 0)
    lens = np.asarray(length_table())
    assert np.all(s >= 1) and np.all(s <= lens[c])
    c, s, e = synth.np_spans(10000, seed=1)
    assert np.all(e >= s) and np.all(e <= lens[c])
    assert np.mean(e == s) > 0.4


def test_dbsnp_allele_mix():
    """The keyed C4 generator (bench --workload c4k): SURVEY 8d's 90 / 8 / 2 %
    mix, short indels keep ref+alt <= 50, anchored indels, rsids everywhere,
    sorted positions inside the requested pieces."""
    from annotatedvdb_amd import shard, synth
    plan = shard.plan(8)
    b = synth.dbsnp_alleles(100000, seed=4, device="cpu", pieces=plan[3])
    rl, al = b.ref_len.long(), b.alt_len.long()
    tot = rl + al
    assert abs((tot == 2).float().mean().item() - 0.90) < 0.01
    assert abs(((tot > 2) & (tot <= 50)).float().mean().item() - 0.08) < 0.01
    assert abs((tot > 50).float().mean().item() - 0.02) < 0.005
    assert bool((b.ext_id > 0).all())
    c, p = b.chrom.numpy().astype(np.int64), b.pos.numpy().astype(np.int64)
    assert np.all(np.diff(c * 2**32 + p) >= 0)
    assert all(shard.shard_of(plan, int(x), int(y)) == 3 for x, y in zip(c[::997], p[::997]))
    heap, off = b.heap.numpy(), b.allele_off.numpy()
    indel = ((tot > 2) & (tot <= 50) & ((rl == 1) | (al == 1))).numpy()
    i = np.nonzero(indel)[0][:500]
    assert np.array_equal(heap[off[i]], heap[off[i] + rl.numpy()[i]])  # alt[0] == ref[0]


def test_bench_step_does_not_shadow_main_buffers():
    """bench.py's step() closes over run_workload()'s resident buffers; a local of the
    same name anywhere in step() breaks every workload (UnboundLocalError)."""
    import ast
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")).read()
    tree = ast.parse(src)
    main = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "run_workload")
    step = next(n for n in ast.walk(main) if isinstance(n, ast.FunctionDef) and n.name == "step")
    stored = {n.id for n in ast.walk(step) if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Store)}
    assert not stored & {"chrom", "start", "end", "code", "hist", "ctr", "batch", "text", "eng"}, stored


def test_piece_table_and_line_owner_oracle():
    """The flat piece tables K9 stages and the host restatement of its line
    placement agree with shard_of on every piece boundary."""
    from annotatedvdb_amd import shard
    from annotatedvdb_amd.chromosomes import length_table
    lens = length_table()
    for world in (1, 2, 3, 8):
        plan = shard.plan(world, lens)
        base, count, rank = shard.piece_table(plan, lens)
        assert count.sum() == len(rank) == len(shard.pieces(lens))
        chrom, pos = [], []
        for p in shard.pieces(lens):
            for x in (p.lo + 1, p.hi, (p.lo + p.hi) // 2):
                chrom.append(p.chrom)
                pos.append(x)
        own = shard.owner_of_lines(plan, chrom, pos, [0] * len(pos))
        assert [shard.shard_of(plan, c, x) for c, x in zip(chrom, pos)] == own.tolist()
        # comments: nobody; unplaced (unknown contig / host-resolved POS): rank 0; past the end: last piece
        o = shard.owner_of_lines(plan, [0, 255, 3, 24], [5, 5, 5, 10 ** 9], [0x001, 0, 0x004, 0])
        assert o[0] == -1 and o[1] == 0 and o[2] == 0 and o[3] == shard.shard_of(plan, 24, lens[24])


def test_driver_file_assignment_lpt(tmp_path):
    from annotatedvdb_amd import load_vcf_file
    fs = []
    for i, sz in enumerate([50, 10, 40, 30, 20]):
        f = tmp_path / ("f%d" % i)
        f.write_bytes(b"x" * sz)
        fs.append(str(f))
    a = load_vcf_file.assign_files(fs, 2)
    assert sorted(sum(a, [])) == sorted(fs)
    assert a[0] == [fs[0], fs[1], fs[4]] and a[1] == [fs[2], fs[3]]


@pytest.mark.parametrize("gz", [False, True])
def test_load_driver_streams_blocks_at_line_boundaries(tmp_path, gz):
    """load_vcf_file.iter_batches: blocks of about --batchBytes ending after a
    newline (a longer line stays whole), concatenating to the file."""
    import gzip as gzm
    from annotatedvdb_amd.load_vcf_file import iter_batches
    lines = [("%d\t" % i) + "A" * (i * 37 % 300) for i in range(500)]
    data = ("\n".join(lines)).encode()  # no final newline
    p = tmp_path / ("x.vcf.gz" if gz else "x.vcf")
    if gz:
        with gzm.open(p, "wb") as fh:
            fh.write(data)
    else:
        p.write_bytes(data)
    for bb in (1, 64, 1000, 1 << 20):
        blocks = list(iter_batches(str(p), bb))
        assert b"".join(blocks) == data
        assert all(b.endswith(b"\n") for b in blocks[:-1])
        assert all(len(b) <= bb + 400 for b in blocks)


def test_keyed_handoff_stamps():
    """engine._stamp / _stamp_ok: a hand-off matches only the same
    tensor objects at the same versions — not a new tensor at a recycled
    address, not an in-place edit, not a missing / extra tensor."""
    import torch
    from annotatedvdb_amd.engine import _stamp, _stamp_ok
    a, b = torch.zeros(8), torch.ones(8)
    st = _stamp(a, b, None)
    assert _stamp_ok(st, a, b, None)
    assert not _stamp_ok(st, a, b, a)
    assert not _stamp_ok(st, b, a, None)
    a.add_(0)
    assert not _stamp_ok(st, a, b, None)
    st = _stamp(a)
    del a
    c = torch.zeros(8)
    assert not _stamp_ok(st, c)
    assert not _stamp_ok(None, c)
