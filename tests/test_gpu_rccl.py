"""The node exchange in the C ABI (SURVEY.md §8b ``avdb_hist_allgather``):
RCCL all-gather of the per-rank L8 histogram + counters, summed on the device.
A one-GPU box can only form a world of one (RCCL refuses two ranks on one
device); the multi-rank orchestration is covered by the gloo tests."""

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def test_hist_allgather_c_abi_world_of_one(engine):
    from annotatedvdb_amd import distributed as D
    from annotatedvdb_amd import _native as N
    ex = D.RcclExchange(engine, world=1, rank=0, unique_id=D.RcclExchange.new_id())
    try:
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        hist = torch.randint(0, 1 << 20, (engine.n_l8,), dtype=torch.int32, device="cuda", generator=g)
        ctr = torch.randint(0, 1 << 40, (N.N_COUNTERS,), dtype=torch.int64, device="cuda", generator=g)
        nh, nc = ex.allgather(hist, ctr)
        torch.cuda.synchronize()
        assert torch.equal(nh, hist) and torch.equal(nc, ctr)
        # odd sizes (the histogram slot is padded to 8 bytes before the counters)
        nh, nc = ex.allgather(hist[:7].contiguous(), ctr[:3].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(nh, hist[:7]) and torch.equal(nc, ctr[:3])
    finally:
        ex.close()


def test_node_exchange_picks_c_abi_rccl(engine):
    """bench.py's exchange object (distributed.node_exchange): with AVDB_EXCHANGE=rccl
    at a world of one it is the C ABI's avdb_hist_allgather, as on an RCCL node."""
    from annotatedvdb_amd import distributed as D
    from annotatedvdb_amd import _native as N
    ri = D.RankInfo(0, 1, 0)
    ex = D.node_exchange(engine, ri, kind="rccl")
    try:
        assert isinstance(ex, D.RcclExchange)
        hist = torch.arange(engine.n_l8, dtype=torch.int32, device="cuda")
        ctr = torch.arange(N.N_COUNTERS, dtype=torch.int64, device="cuda") * 3
        nh, nc = ex.allgather(hist, ctr)
        torch.cuda.synchronize()
        assert torch.equal(nh, hist) and torch.equal(nc, ctr)
    finally:
        ex.close()
    assert isinstance(D.node_exchange(engine, ri), D.TorchExchange)  # world 1, no process group
