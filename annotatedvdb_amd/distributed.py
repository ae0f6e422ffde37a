"""Multi-GPU orchestration: one process per GPU, genome pieces sharded by
length-balanced LPT (``shard.plan``), no record exchange.  The single
collective is an all-gather of every rank's L8 histogram and counters
 — RCCL (``nccl`` backend) over xGMI on MI355X nodes, ``gloo``
for the CPU tests.

The reference's only parallelism is one OS process per chromosome file
(``Load/bin/load_vcf_file.py:307-313``) with no communication at all; the
all-gather replaces the per-file log summaries with node-level statistics.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from . import shard


@dataclass
class RankInfo:
    rank: int
    world: int
    local: int

    @property
    def distributed(self) -> bool:
        return self.world > 1


def rank_info() -> RankInfo:
    return RankInfo(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def device_index(ri: RankInfo) -> int:
    """GPU of this rank: LOCAL_RANK (one process per GPU).  Only a rehearsal
    with more ranks than GPUs (``AVDB_DIST_BACKEND=gloo`` on a 1-GPU box) wraps."""
    n = torch.cuda.device_count()
    return ri.local % n if n else ri.local


def init(backend: Optional[str] = None) -> RankInfo:
    """Initialise the process group from torchrun's environment (no-op at N=1).
    ``AVDB_DIST_BACKEND`` overrides the backend (``gloo`` rehearses the N>1 path
    with several ranks sharing one GPU; RCCL refuses two ranks on one device)."""
    ri = rank_info()
    backend = os.environ.get("AVDB_DIST_BACKEND", backend)
    if ri.distributed and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(ri.local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", ri.local))
        else:
            dist.init_process_group(backend)
    return ri


def my_pieces(ri: RankInfo, lengths=None) -> List[shard.Piece]:
    return shard.plan(ri.world, lengths)[ri.rank]


def allgather_stats(hist: torch.Tensor, counters: torch.Tensor, ri: RankInfo
                    ) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-gather every rank's L8 histogram and counters; returns the node
    totals (sum over ranks).  One collective per tensor, issued back to back."""
    if not ri.distributed:
        return hist.clone(), counters.clone()
    dev = hist.device
    if dist.get_backend() == "gloo" and dev.type != "cpu":
        # gloo rehearsal of the N>1 path with several ranks on one GPU: the
        # exchange goes through host memory (RCCL never takes this branch)
        hist, counters = hist.cpu(), counters.cpu()
    hs = [torch.empty_like(hist) for _ in range(ri.world)]
    cs = [torch.empty_like(counters) for _ in range(ri.world)]
    dist.all_gather(hs, hist)
    dist.all_gather(cs, counters)
    return torch.stack(hs).sum(0).to(dev), torch.stack(cs).sum(0).to(dev)


class RcclExchange:
    kind = "rccl (avdb_hist_allgather, C ABI)"
    """The node exchange through the C ABI (``avdb_hist_allgather``, SURVEY.md
    §8b) instead of ``torch.distributed``: for a caller that binds only
    ``libavdb_hip.so``.  Rank 0 makes the id (``new_id``) and hands its bytes to
    the other ranks out of band; every rank builds its communicator with its
    rank.  ``allgather`` returns the node totals (sum over ranks), as
    ``allgather_stats`` does."""

    def __init__(self, engine, world: int, rank: int, unique_id: bytes):
        import ctypes
        from . import _native as N
        self._N = N
        self.engine = engine
        self.world = world
        comm = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(unique_id), N.RCCL_ID_BYTES)
        N.check("avdb_rccl_comm_init", engine.lib.avdb_rccl_comm_init(engine.ctx, world, rank, buf,
                                                                     ctypes.byref(comm)))
        self.comm = comm

    @staticmethod
    def new_id() -> bytes:
        import ctypes
        from . import _native as N
        buf = ctypes.create_string_buffer(N.RCCL_ID_BYTES)
        N.check("avdb_rccl_unique_id", N.load_library().avdb_rccl_unique_id(buf))
        return buf.raw

    def allgather(self, hist: torch.Tensor, counters: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        import ctypes
        N, e = self._N, self.engine
        # avdb_hist_allgather reads u32 bins and u64 counters from raw device pointers
        if hist.dtype not in (torch.int32, torch.uint32) or counters.dtype not in (torch.int64, torch.uint64):
            raise ValueError("hist must be int32/uint32 and counters int64/uint64 (got %s, %s)"
                             % (hist.dtype, counters.dtype))
        if not (hist.is_contiguous() and counters.is_contiguous()):
            raise ValueError("hist and counters must be contiguous")
        if hist.device != e.device or counters.device != e.device:
            raise ValueError("hist and counters must be on the engine's device %s" % e.device)
        nb, nc = hist.numel(), counters.numel()
        sz = ctypes.c_size_t()
        N.check("avdb_hist_allgather_workspace_size",
                e.lib.avdb_hist_allgather_workspace_size(self.world, nb, nc, ctypes.byref(sz)))
        ws = torch.empty(int(sz.value), dtype=torch.uint8, device=hist.device)
        node_h, node_c = torch.empty_like(hist), torch.empty_like(counters)
        N.check("avdb_hist_allgather", e.lib.avdb_hist_allgather(
            e.ctx, self.comm, N.ptr(hist), nb, N.ptr(counters), nc, N.ptr(node_h), N.ptr(node_c), N.ptr(ws),
            ws.numel(), e._stream()))
        return node_h, node_c

    def close(self):
        if self.comm:
            self._N.check("avdb_rccl_comm_destroy", self.engine.lib.avdb_rccl_comm_destroy(self.comm))
            self.comm = None


class TorchExchange:
    """The node exchange through ``torch.distributed`` (``allgather_stats``): the
    gloo CPU tests and the gloo rehearsal of the N>1 bench path."""
    kind = "torch.distributed"

    def __init__(self, ri: RankInfo):
        self.ri = ri

    def allgather(self, hist: torch.Tensor, counters: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        return allgather_stats(hist, counters, self.ri)

    def close(self):
        pass


def node_exchange(engine, ri: RankInfo, kind: Optional[str] = None):
    """The job's one exchange: ``RcclExchange`` — the C ABI's
    ``avdb_hist_allgather``, what a caller binding only ``libavdb_hip.so`` runs —
    when the process group is RCCL (``nccl``), ``TorchExchange`` otherwise.
    ``kind`` / ``AVDB_EXCHANGE`` (``rccl`` | ``torch``) override the choice; ``rccl``
    at a world of one builds a one-rank communicator (the GPU test of this path on
    a one-GPU box).  Rank 0 makes the RCCL id and the process group carries its
    bytes to the other ranks (the out-of-band step ``RcclExchange`` leaves to its
    caller)."""
    kind = kind or os.environ.get("AVDB_EXCHANGE")
    if kind is None:
        kind = "rccl" if ri.distributed and dist.get_backend() == "nccl" else "torch"
    if kind == "torch":
        return TorchExchange(ri)
    if kind != "rccl":
        raise ValueError("exchange kind must be 'rccl' or 'torch', not %r" % (kind,))
    # rank 0's outcome (the id, or why it could not make one) goes to every rank, so
    # all ranks raise together and a caller's fallback is the same on every rank
    # (a rank left waiting in the broadcast while rank 0 falls back would hang the job)
    uid, err = None, None
    if ri.rank == 0:
        try:
            uid = RcclExchange.new_id()
        except Exception as e:  # noqa: BLE001 (re-raised on every rank below)
            err = "%s: %s" % (type(e).__name__, e)
    if ri.distributed:
        box = [uid, err]
        dist.broadcast_object_list(box, src=0)
        uid, err = box
    if err is not None:
        raise RuntimeError("RCCL unique id on rank 0 failed: " + err)
    return RcclExchange(engine, ri.world, ri.rank, uid)


def max_over_ranks(value: float, ri: RankInfo, device=None) -> float:
    if not ri.distributed:
        return value
    if dist.get_backend() == "gloo":
        device = None
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(ri: RankInfo):
    if ri.distributed:
        dist.barrier()


def finalize(ri: RankInfo):
    if ri.distributed and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
