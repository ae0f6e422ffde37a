"""K9 (genome-piece sharding of VCF text) and the multi-rank load driver
(annotatedvdb_amd/load_vcf_file.py, the counterpart of Load/bin/load_vcf_file.py):
every data line lands on exactly one rank, and the union of the ranks' COPY
rows and .mapping lines equals the single-process output (world 2, gloo, both
ranks on the one GPU of the box)."""

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _text(n, seed):
    from annotatedvdb_amd import synth
    lines = synth.vcf_text(n, seed=seed).decode().splitlines()
    # comments, an unknown contig, a chr-prefixed contig and MT: every kind of placement
    lines.insert(0, "##fileformat=VCFv4.2")
    lines.insert(1, "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO")
    lines.insert(500, "chrUn_KI270302v1\t100\trs9\tA\tG\t.\t.\tRS=9")
    lines.insert(900, "chr7\t1000\trs8\tA\tG\t.\t.\tRS=8")
    lines.insert(1200, "MT\t300\t.\tC\tT\t.\t.\t.")
    return ("\n".join(lines) + "\n").encode()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_k9_select_partitions_every_line_once(engine, world):
    from annotatedvdb_amd import shard
    from annotatedvdb_amd.engine import VCF_LINE_DTYPE
    raw = _text(20000, seed=31)
    vb = engine.vcf_tokenize(raw)
    L = vb.lines_host()
    plan = shard.plan(world, engine.lengths)
    owner = shard.owner_of_lines(plan, L["chrom"], L["pos"], L["flags"])
    lines = raw.decode().split("\n")[:-1]
    got = []
    for r in range(world):
        t = engine.vcf_select(vb, plan, r).cpu().numpy().tobytes().decode()
        exp = [ln for ln, o in zip(lines, owner) if o == r]
        assert t.split("\n")[:-1] == exp, r
        got += exp
    data = [ln for ln in lines if not ln.startswith("#")]
    assert sorted(got) == sorted(data)


def _driver(rank, world, port, argv, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from annotatedvdb_amd import load_vcf_file
    q.put((rank, load_vcf_file.main(argv)))


def _outputs(out_dir, suffix):
    rows = []
    for f in sorted(os.listdir(out_dir)):
        if f.endswith(suffix):
            rows += open(os.path.join(out_dir, f)).read().splitlines()
    return rows


def test_driver_two_ranks_equal_single_process(engine, tmp_path):
    import torch.multiprocessing as mp
    from annotatedvdb_amd import load_vcf_file
    vcf = tmp_path / "in.vcf"
    vcf.write_bytes(_text(30000, seed=32).replace(b"chrUn_KI270302v1\t100\trs9\tA\tG\t.\t.\tRS=9\n", b""))
    single = tmp_path / "single"
    tot1 = load_vcf_file.main(["--fileName", str(vcf), "--outDir", str(single), "--algInvocationId", "7",
                               "--batchBytes", str(1 << 20)])
    multi = tmp_path / "multi"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    argv = ["--fileName", str(vcf), "--outDir", str(multi), "--algInvocationId", "7", "--backend", "gloo",
            "--batchBytes", str(1 << 20)]
    procs = [ctx.Process(target=_driver, args=(r, 2, port, argv, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    one_copy, one_map = _outputs(single, ".copy"), _outputs(single, ".mapping")
    two_copy, two_map = _outputs(multi, ".copy"), _outputs(multi, ".mapping")
    assert len(one_copy) > 30000 and sorted(two_copy) == sorted(one_copy)
    assert sorted(two_map) == sorted(one_map)
    # both ranks did work, and the node totals (all-gathered) equal the single run
    assert all(os.path.getsize(multi / ("in.vcf.r%d.copy" % r)) > 0 for r in range(2))
    assert res[0] == res[1] == tot1


def test_driver_files_per_rank(engine, tmp_path):
    """--dir/--extension/--chr: whole files dealt to ranks, as the reference's
    one-worker-per-file pool (load_vcf_file.py:307-313)."""
    from annotatedvdb_amd import load_vcf_file
    from annotatedvdb_amd import synth
    lines = synth.vcf_text(6000, seed=33).decode().splitlines()
    d = tmp_path / "vcfs"
    d.mkdir()
    for c in ("1", "2", "22"):
        sel = [ln for ln in lines if ln.split("\t")[0] == c]
        (d / ("chr%s.vcf" % c)).write_text("\n".join(sel) + "\n")
    assert load_vcf_file.assign_files([str(d / "chr1.vcf"), str(d / "chr2.vcf"), str(d / "chr22.vcf")], 2)[0] \
        == [str(d / "chr1.vcf")]
    out = tmp_path / "out"
    tot = load_vcf_file.main(["--dir", str(d), "--extension", "vcf", "--chr", "1,2,22", "--outDir", str(out)])
    n = sum(1 for ln in lines if ln.split("\t")[0] in ("1", "2", "22"))
    assert tot["line"] == n and len(_outputs(out, ".mapping")) == n


def _driver_rc(rank, world, port, argv, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from annotatedvdb_amd import load_vcf_file
    try:
        q.put((rank, "ok", load_vcf_file.main(argv)))
    except load_vcf_file.LoadFailed as err:
        q.put((rank, "failed", str(err)))
        raise SystemExit(1)


def test_driver_rank_failure_reaches_every_rank(engine, tmp_path):
    """A line that raises on one rank (an unknown contig: K9 gives it to rank 0,
    the loader raises TypeError as the reference does) fails that rank's file
    only; the other rank loads its share, the failure travels in the all-gathered
    counters, and every rank exits non-zero instead of waiting on a dead peer."""
    import torch.multiprocessing as mp
    vcf = tmp_path / "in.vcf"
    vcf.write_bytes(_text(6000, seed=34))
    assert b"chrUn_KI270302v1" in vcf.read_bytes()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    argv = ["--fileName", str(vcf), "--outDir", str(tmp_path / "multi"), "--backend", "gloo",
            "--batchBytes", str(1 << 16)]
    procs = [ctx.Process(target=_driver_rc, args=(r, 2, port, argv, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (st, v) for r, st, v in (q.get(timeout=300) for _ in range(2))}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 1
    assert res[0][0] == res[1][0] == "failed"
    assert "this rank: 1" in res[0][1] and "this rank: 0" in res[1][1]
    assert os.path.getsize(tmp_path / "multi" / "in.vcf.r1.copy") > 0
