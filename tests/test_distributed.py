"""Multi-process (world_size 2, gloo, CPU) tests of the multi-GPU path:
bench.combine_ranks (max-over-ranks timing + the one all-reduce of scaler
totals), the partition of BASELINE configs[3]'s independent nodes over ranks
(plfx.shard, the reference's ceil rule include.h:181-189) and the one lnL
all-reduce (bench.reduce_node_lnls): each rank evaluates its share of real
nodes with the oracle, and the reduced per-node lnL, job lnL and scaler totals
equal the single-process values bit for bit."""
import os
import socket

import numpy as np
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


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q, *args)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench

        wall, devt, ok = bench.combine_ranks(10.0 + rank, 5.0 * (rank + 1), torch.tensor(7 + rank), 7 + rank,
                                             torch.device("cpu"), world)
        bad = bench.combine_ranks(1.0, 1.0, torch.tensor(3), 4 if rank == 1 else 3,
                                  torch.device("cpu"), world)[2]
        skew = bench.rank_clock_spread(100.0 + 25e-6 * rank, 200.0 - 40e-6 * rank, torch.device("cpu"),
                                       world)
        mx = bench.max_over_ranks(3.5 * (rank + 1), torch.device("cpu"), world)
        q.put((rank, wall, devt, ok, bad, skew, mx))
    finally:
        dist.destroy_process_group()


def test_combine_ranks_gloo_world2():
    for rank, wall, devt, ok, bad, skew, mx in _spawn(_worker, 2):
        assert mx == 7.0
        assert wall == 11.0 and devt == 10.0   # max over ranks
        assert ok is True                      # sum of got == sum of expected
        assert bad is False                    # one rank's mismatch is seen by every rank
        # the ranks' region-start / -end clocks: max - min, in us, on every rank
        assert abs(skew[0] - 25.0) < 1e-3 and abs(skew[1] - 40.0) < 1e-3


def test_combine_ranks_single():
    import bench

    assert bench.combine_ranks(3.0, 2.0, torch.tensor(5), 5, torch.device("cpu"), 1) == (3.0, 2.0, True)
    assert bench.rank_clock_spread(5.0, 6.0, torch.device("cpu"), 1) == (0.0, 0.0)


# --- BASELINE configs[3] on the CPU: real nodes, the product's partition, the
# one all-reduce, the oracle's plf() + root lnL as each rank's "GPU" ---------
TOTAL_NODES, SITES = 64, 301  # 64: the ceil split is defined for 2, 3 and 8 ranks


def _node_inputs(oracle, j):
    """Node j's inputs (global index j: identical for any rank count)."""
    d = oracle.gen_hostmem(SITES, np.float64, 1000 + j)
    w = ((np.arange(SITES) + j) % 3 + 1).astype(np.int32)
    return d, w


def _node_lnl(oracle, j):
    d, w = _node_inputs(oracle, j)
    x3, _, inc = oracle.plf(d["x1"], d["x2"], d["EV"], d["left"], d["right"], w)
    return oracle.root_lnl(4, 4, x3, SITES, wgt=w, scaler_sums=np.array([inc])), inc


def _nodes_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle
        import plfx

        off, cnt = plfx.shard(TOTAL_NODES, world, rank)
        vals = [_node_lnl(oracle, j) for j in range(off, off + cnt)]
        per, tot, ev = bench.reduce_node_lnls([v[0] for v in vals], [v[1] for v in vals], off,
                                              TOTAL_NODES, torch.device("cpu"), world)
        q.put((rank, off, cnt, per, tot, ev))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_nodes_partition_lnl_allreduce_equals_single_process(oracle, world):
    """configs[3] at world 2, 3 and 8 (gloo): ranks take the reference's ceil
    split of the nodes, evaluate their nodes (oracle plf + root lnL), and one
    all-reduce gives every rank the per-node lnL vector, the job lnL and the
    scaler totals of the single-process run -- bit for bit (so well inside the
    1e-12 relative bound)."""
    import bench

    single = [_node_lnl(oracle, j) for j in range(TOTAL_NODES)]
    exp_per, exp_tot, exp_ev = bench.reduce_node_lnls([v[0] for v in single], [v[1] for v in single],
                                                      0, TOTAL_NODES, torch.device("cpu"), 1)
    assert exp_ev == sum(v[1] for v in single) > 0
    res = _spawn(_nodes_worker, world)
    covered = sorted((off, cnt) for _, off, cnt, *_ in res)
    assert sum(c for _, c in covered) == TOTAL_NODES and covered[0][0] == 0
    for rank, off, cnt, per, tot, ev in res:
        assert np.array_equal(per, exp_per)
        assert tot == exp_tot and ev == exp_ev
        assert abs(tot - exp_tot) <= 1e-12 * abs(exp_tot)


def _tree_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import types

        import bench

        wl = types.SimpleNamespace(lnl=torch.tensor([-(rank + 1) * 100.5], dtype=torch.float64),
                                   sums=torch.tensor([rank, 2], dtype=torch.int64), n=1000)
        q.put((rank, bench.Tree64Workload.post(wl, world, rank, torch.device("cpu"))))
    finally:
        dist.destroy_process_group()


def test_tree64_site_shards_lnl_allreduce_gloo_world2():
    """tree64 at N GPUs: every rank sweeps the tree over its own block of sites;
    the tree lnL and scaler totals are summed over ranks by one all-reduce."""
    for rank, out in _spawn(_tree_worker, 2):
        assert out["root_lnl_rank0"] == -(rank + 1) * 100.5
        assert out["tree_lnl_all_ranks"] == -301.5
        assert out["scaler_events_all_ranks"] == 5
        assert out["alignment_sites"] == 2000


# --- tree64's site sharding with real per-rank sweeps: a 16-taxon tree over
# TREE_SITES sites, split by the reference's ceil rule (plfx.shard); each rank
# sweeps the whole tree over its block with the oracle and takes its block's
# root lnL; bench's one all-reduce must give the single-process tree lnL -----
TREE_TAXA, TREE_SITES = 16, 1001


def _tree_block(oracle, off, cnt):
    """The tree lnL and per-op scaler sums of sites [off, off + cnt)."""
    rng = np.random.default_rng(77)
    tips = [rng.random(16 * TREE_SITES) for _ in range(TREE_TAXA)]
    ops = oracle.balanced_tree_ops(TREE_TAXA)
    pm = rng.random(ops.shape[0] * 128) * 0.25
    EV = rng.random(16) * 0.25
    wgt = (np.arange(TREE_SITES) % 3 + 1).astype(np.int32)[off:off + cnt]
    clv = [t[16 * off:16 * (off + cnt)].copy() for t in tips]
    clv += [np.zeros(16 * cnt) for _ in range(ops.shape[0])]
    sums, _ = oracle.traverse(4, 4, ops, clv, pm, EV, cnt, wgt)
    return oracle.root_lnl(4, 4, clv[-1], cnt, wgt=wgt, scaler_sums=sums), sums


def _tree_shard_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import types

        import bench
        import oracle
        import plfx

        off, cnt = plfx.shard(TREE_SITES, world, rank)
        lnl, sums = _tree_block(oracle, off, cnt)
        wl = types.SimpleNamespace(lnl=torch.tensor([lnl], dtype=torch.float64),
                                   sums=torch.from_numpy(sums), n=cnt)
        q.put((rank, off, cnt, bench.Tree64Workload.post(wl, world, rank, torch.device("cpu"))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tree_site_shards_equal_single_process(oracle, world):
    """Each rank's block sweep + the one lnL all-reduce = the whole-alignment
    tree lnL (1e-12 relative: only the summation order differs) and exactly
    its scaler events; the blocks tile the alignment (ragged last block)."""
    exp_lnl, exp_sums = _tree_block(oracle, 0, TREE_SITES)
    assert int(exp_sums.sum()) > 0  # deep levels underflow: the correction is exercised
    res = _spawn(_tree_shard_worker, world)
    blocks = sorted((off, cnt) for _, off, cnt, _ in res)
    assert blocks[0][0] == 0 and sum(c for _, c in blocks) == TREE_SITES
    assert all(a[0] + a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
    for _, _, _, out in res:
        assert abs(out["tree_lnl_all_ranks"] - exp_lnl) <= 1e-12 * abs(exp_lnl)
        assert out["scaler_events_all_ranks"] == int(exp_sums.sum())
