"""Multi-rank path on CPU (gloo, world_size 2): shard-local binning needs no
exchange, and the all-gathered per-rank L8 histograms / counters equal the
single-process answer over the union of the shards."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from annotatedvdb_amd import shard
from annotatedvdb_amd.chromosomes import length_table


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_records(pieces, n, seed):
    """Synthetic records inside this rank's pieces (numpy; oracle-sized)."""
    rng = np.random.default_rng(seed)
    lens = np.array([p.length for p in pieces], dtype=np.float64)
    counts = np.floor(n * lens / lens.sum()).astype(np.int64)
    counts[0] += n - counts.sum()
    chrom, start = [], []
    for p, k in zip(pieces, counts):
        chrom.append(np.full(k, p.chrom, dtype=np.uint8))
        start.append(p.lo + 1 + (rng.random(k) * p.length).astype(np.int64))
    chrom = np.concatenate(chrom)
    start = np.concatenate(start)
    L = np.asarray(length_table(), dtype=np.int64)[chrom]
    span = np.where(rng.random(n) < 0.7, 0, (10 ** rng.uniform(0, 6, n)).astype(np.int64))
    end = np.minimum(start + span, L)
    return chrom, start, end


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from annotatedvdb_amd import distributed as D
    from oracle import avdb_oracle as O
    ri = D.init("gloo")
    pieces = D.my_pieces(ri)
    chrom, start, end = _rank_records(pieces, n, seed=100 + rank)
    lens = length_table()
    # every record lies in one of this rank's pieces
    assert all(shard.shard_of(shard.plan(world), int(c), int(s)) == rank
               for c, s in zip(chrom[::97], start[::97]))
    codes, status = O.bin_codes_np(chrom, start, end, lens)   # the per-rank kernel's job
    hist = torch.from_numpy(O.l8_histogram_np(chrom, start, status, lens).astype(np.int32))
    ctr = torch.zeros(32, dtype=torch.int64)
    ctr[20] = len(chrom)
    ctr[16:20] = torch.from_numpy(np.bincount(status, minlength=4).astype(np.int64))
    # the bench's exchange object: over gloo the torch.distributed one (RCCL process
    # groups take the C ABI's avdb_hist_allgather, tests/test_gpu_rccl.py)
    ex = D.node_exchange(None, ri)
    assert isinstance(ex, D.TorchExchange)
    node_hist, node_ctr = ex.allgather(hist, ctr)
    t = D.max_over_ranks(float(rank + 1), ri)
    q.put((rank, chrom, start, end, codes, node_hist.numpy(), node_ctr.numpy(), t))
    D.finalize(ri)


@pytest.mark.parametrize("world", [2])
def test_gloo_allgather_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n = 20000
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from oracle import avdb_oracle as O
    lens = length_table()
    chrom = np.concatenate([r[1] for r in res])
    start = np.concatenate([r[2] for r in res])
    end = np.concatenate([r[3] for r in res])
    codes, status = O.bin_codes_np(chrom, start, end, lens)
    # shard-local results == whole-batch results (no exchange needed)
    assert np.array_equal(np.concatenate([r[4] for r in res]), codes)
    exp_hist = O.l8_histogram_np(chrom, start, status, lens)
    for r in res:
        assert np.array_equal(r[5].astype(np.uint32), exp_hist)
        assert r[6][20] == len(chrom)
        assert r[7] == float(world)  # max over ranks


def _rccl_fail_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from annotatedvdb_amd import distributed as D

    def no_id():
        raise OSError("no RCCL here")
    D.RcclExchange.new_id = staticmethod(no_id)
    ri = D.init("gloo")
    try:
        D.node_exchange(None, ri, kind="rccl")
        got = "no error"
    except RuntimeError as e:
        got = str(e)
    # the bench's fallback, then one more collective: every rank must still be in step
    t = D.max_over_ranks(float(rank + 1), ri)
    q.put((rank, got, t))
    D.finalize(ri)


def test_rccl_exchange_setup_failure_reaches_every_rank():
    """When rank 0 cannot make the RCCL id, every rank raises from node_exchange
    (rank 0's error travels with the broadcast), so the bench's fallback to the
    torch.distributed exchange is taken on all ranks together and the next
    collective does not hang (gloo, world 2)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rccl_fail_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, got, t in res:
        assert "RCCL unique id on rank 0 failed" in got and "no RCCL here" in got, (rank, got)
        assert t == float(world)
