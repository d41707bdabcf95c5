"""Multi-process (world_size 2, gloo, CPU) tests of the multi-GPU plumbing:
bench.combine_ranks (max-over-ranks timing + the one all-reduce of scaler
totals) and the node sharding used by the multi-node workloads."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench

        wall, devt, ok = bench.combine_ranks(10.0 + rank, 5.0 * (rank + 1), torch.tensor(7 + rank), 7 + rank,
                                             torch.device("cpu"), world)
        bad = bench.combine_ranks(1.0, 1.0, torch.tensor(3), 4 if rank == 1 else 3,
                                  torch.device("cpu"), world)[2]
        q.put((rank, wall, devt, ok, bad))
    finally:
        dist.destroy_process_group()


def test_combine_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, wall, devt, ok, bad in res:
        assert wall == 11.0 and devt == 10.0   # max over ranks
        assert ok is True                      # sum of got == sum of expected
        assert bad is False                    # one rank's mismatch is seen by every rank


def test_combine_ranks_single():
    import bench

    assert bench.combine_ranks(3.0, 2.0, torch.tensor(5), 5, torch.device("cpu"), 1) == (3.0, 2.0, True)


def _tree_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import types

        import bench

        wl = types.SimpleNamespace(lnl=torch.tensor([-(rank + 1) * 100.5], dtype=torch.float64),
                                   sums=torch.tensor([rank, 2], dtype=torch.int64), n=1000)
        q.put((rank, bench.Tree64Workload.post(wl, world, torch.device("cpu"))))
    finally:
        dist.destroy_process_group()


def test_tree64_site_shards_lnl_allreduce_gloo_world2():
    """tree64 at N GPUs: every rank sweeps the tree over its own block of sites;
    the tree lnL and scaler totals are summed over ranks by one all-reduce."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in res:
        assert out["root_lnl_rank0"] == -(rank + 1) * 100.5
        assert out["tree_lnl_all_ranks"] == -301.5
        assert out["scaler_events_all_ranks"] == 5
        assert out["alignment_sites"] == 2000
