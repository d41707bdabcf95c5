"""GPU tests of BASELINE configs[3] end to end through bench.py: 512-node
style workloads split over ranks with the reference's ceil rule, the real HIP
kernels, the per-node root lnL and the ONE all-reduce.  On the one-GPU box the
ranks share the device: 2 ranks over gloo, and 1 rank under
torch.distributed.run over RCCL (the nccl backend), so the RCCL collective is
exercised on hardware.  The all-reduced lnL of N ranks must equal the
1-rank value bit for bit (the reduction is exact by construction,
bench.reduce_node_lnls) and the oracle's lnL of the same nodes within 1e-12."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
NODES, SITES = 12, 4099


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(nproc, args, env, timeout=300):
    """bench.py under torch.distributed.run on a fresh 127.0.0.1 port.  The
    port is picked free and released before the launcher binds it, so another
    process can take it in between: the launcher then fails in its rendezvous
    (EADDRINUSE) before any rank starts -- nothing ran on the GPU -- and only
    that case is launched again on a new port (at most twice)."""
    for _ in range(3):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"), *args]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=str(ROOT))
        if not (r.returncode != 0 and "EADDRINUSE" in r.stderr and "{" not in r.stdout):
            return r
    return r


def _bench(nproc, backend, *extra):
    args = ["--gpus", str(nproc), "--workload", "nodes512", "--nodes", str(NODES), "--sites",
            str(SITES), "--steps", "3", "--warmup", "1", "--no-cpu-baseline", *extra]
    env = {**os.environ, "PLFX_DIST_BACKEND": backend, "OMP_NUM_THREADS": "4"}
    r = _torchrun(nproc, args, env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def _oracle_lnls(oracle):
    """The same nodes (bench.NodesWorkload: node j from a generator seeded
    SEED + 1 + j) evaluated by the oracle: plf() then root lnL."""
    import torch

    import bench
    import plfx

    a = bench.parse(["--workload", "nodes512", "--nodes", str(NODES), "--sites", str(SITES)])
    dev = torch.device("cuda", 0)
    with plfx.Context(0) as ctx:
        wl = bench.NodesWorkload(ctx, a, dev, None, torch.float64, 8, 1, 0)
        EV = wl.EV.cpu().numpy()
        out = []
        for nd in wl.nodes:
            h = {k: nd[k].cpu().numpy() for k in ("x1", "x2", "left", "right")}
            x3, _, inc = oracle.plf(h["x1"], h["x2"], EV, h["left"], h["right"])
            out.append((oracle.root_lnl(4, 4, x3, SITES, scaler_sums=np.array([inc])), inc))
        del wl
    return out


def test_nodes_two_ranks_gloo_equal_one_rank_rccl(oracle):
    """2 ranks (gloo) and 1 rank (RCCL under torch.distributed.run) on the
    same 12 nodes: identical job lnL and scaler totals, equal to the oracle."""
    one = _bench(1, "nccl")
    two = _bench(2, "gloo")
    assert one["config"]["distributed"] == "nccl" and two["config"]["distributed"] == "gloo"
    assert one["check"] == two["check"] == "ok"
    assert one["scaling"] == "strong" and one["config"]["nodes_in_job"] == NODES
    c1, c2 = one["config"], two["config"]
    k = "lnl_all_nodes_all_ranks"
    assert c1[k] == c2[k]                                     # bit for bit
    assert c1["scaler_events_all_ranks"] == c2["scaler_events_all_ranks"] == NODES * ((SITES + 3) // 4)
    assert c1["lnl_rank_nodes"] == [0, NODES] and c2["lnl_rank_nodes"] == [0, NODES // 2]
    exp = _oracle_lnls(oracle)
    tot = sum(v[0] for v in exp)
    assert abs(c1[k] - tot) <= 1e-12 * abs(tot)
    assert sum(v[1] for v in exp) == c1["scaler_events_all_ranks"]
    assert np.allclose(c1["lnl_first_nodes"], [v[0] for v in exp[:4]], rtol=1e-12, atol=0)


def test_nodes_three_ranks_ragged_split():
    """12 nodes over 3 ranks (4 each) and the default node workload at 2
    ranks: the one all-reduce carries every rank's values (gloo on one GPU)."""
    three = _bench(3, "gloo")
    one = _bench(1, "gloo")
    assert three["config"]["lnl_all_nodes_all_ranks"] == one["config"]["lnl_all_nodes_all_ranks"]
    assert three["config"]["scaler_events_all_ranks"] == one["config"]["scaler_events_all_ranks"]
    r = _torchrun(2, ["--gpus", "2", "--sites", "65536", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                      "--buffer-sets", "2", "--no-nodes512"],
                  {**os.environ, "PLFX_DIST_BACKEND": "gloo", "OMP_NUM_THREADS": "4"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert d["n_gpus"] == 2 and len(d["config"]["lnl_per_rank"]) == 2
    assert d["config"]["lnl_all_ranks"] == sum(d["config"]["lnl_per_rank"])
    assert d["config"]["scaler_events_all_ranks"] == 2 * (65536 // 4)
    assert "nodes512" not in d["config"]  # --no-nodes512


def test_bench_gpus_two_without_outer_launcher():
    """`python bench.py --gpus 2` as the driver may invoke it, with NO outer
    torch.distributed.run: bench.py starts the launcher as a child, and the
    relayed stdout is exactly one JSON line from two ranks (gloo on the
    one-GPU box: both ranks fold onto GPU 0)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PLFX_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--sites", "65536", "--steps", "3",
           "--warmup", "1", "--no-cpu-baseline", "--buffer-sets", "2", "--nodes", "12"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(ROOT), env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["check"] == "ok" and len(d["config"]["lnl_per_rank"]) == 2
    assert d["config"]["launcher"] == "torch.distributed.run started by bench.py"
    assert d["config"]["distributed"] == "gloo"
    assert d["config"]["scaler_events_all_ranks"] == 2 * (65536 // 4)
    assert d["value_device"] >= d["value"] > 0 and d["barrier_skew_us"] >= 0
    # the ranks start at one agreed instant; the per-rank barrier-bracketed
    # wall is reported beside the job time
    assert d["wall_barrier_ms_per_step"] > 0 and d["ms_per_step"] > 0
    # the default invocation also times BASELINE configs[3]: 12 nodes, 6 per rank
    sub = d["config"]["nodes512"]
    assert sub["check"] == "ok" and sub["scaling"] == "strong" and sub["nodes_per_rank"] == 6
    assert sub["nodes_in_job"] == 12 and sub["scaler_events_all_ranks"] == 12 * (65536 // 4)
    assert sub["value_device"] >= sub["value"] > 0 and sub["barrier_skew_us"] >= 0
    _assert_checked(d, 2, nodes=12)


def _assert_checked(d, world, nodes):
    """Every record of a default-invocation line carries its oracle windows,
    summed over the ranks, with no mismatch: the node line (one window per
    rank), nodes512 (one per node), tree64 (63 inner CLVs per rank), protein
    FMA and exact (one per rank)."""
    c = d["config"]
    assert d["check"] == "ok"
    assert c["check_windows"] == world and c["windows_mismatched"] == 0
    expect = {"nodes512": nodes, "tree64": 63 * world}
    for k, n in expect.items():
        assert c[k]["check"] == "ok" and c[k]["check_windows"] == n and c[k]["windows_mismatched"] == 0, k
    assert c["tree64"]["scaler_events_all_ranks"] > 0 and c["tree64"]["value"] > 0
    for p in (c["protein"], c["protein"]["valu_fma"], c["protein"]["exact"]):
        assert p["check"] == "ok" and p["check_windows"] == world and p["windows_mismatched"] == 0
        assert p["steps"] >= 200 and p["value_device"] >= p["value"] > 0
    # the exact record carries its VALU floor (roofline-style `valu` dict)
    assert isinstance(c["protein"]["exact"].get("valu"), dict) and "bound" in c["protein"]["exact"]["valu"]
    assert "not MFMA" in c["protein"]["valu_fma"]["workload"]


@pytest.mark.parametrize("per_launch", [1, 32])
def test_nodes512_full_size_windows(oracle, per_launch):
    """BASELINE configs[3] at full size on one GPU, as bench.py times it: the
    512 nodes x 2^20 f64 sites of bench.NodesWorkload (201 GB of CLVs) in one
    launch per node over two lanes (the default), and in 16 interleaved
    32-node launches.  A 1024-site window of every node is
    checked bit for bit against the oracle on that window (x3 and scaler
    bytes; every 64th node also against the reference's own plf() in
    double), and every node's scaler sum is its N/4 rescaled sites."""
    import torch

    import bench
    import plfx

    n = 1 << 20
    a = bench.parse(["--workload", "nodes512", "--per-launch", str(per_launch)])
    assert a.nodes == 512 and a.sites == n
    dev = torch.device("cuda", 0)
    with plfx.Context(0) as ctx:
        wl = bench.NodesWorkload(ctx, a, dev, None, torch.float64, 8, 1, 0)
        assert wl.cnt == 512 and len(wl.launchers) == (512 if per_launch == 1 else 16)
        assert wl.lanes == 2
        lanes = [torch.cuda.Stream(), torch.cuda.Stream()]
        ctx.set_streams(2)
        torch.cuda.synchronize()
        for lane, st_ in enumerate(lanes):  # as the bench's lanes issue one step
            wl.issue(0, lane, 2, st_.cuda_stream)
        torch.cuda.synchronize()
        ctx.set_streams(1)
        EV = wl.EV.cpu().numpy()
        ones = np.ones(1024, dtype=np.int32)
        for j, nd in enumerate(wl.nodes):
            lo = (j * 40961) % (n - 1024)
            sl = slice(16 * lo, 16 * (lo + 1024))
            h = {k: nd[k][sl].cpu().numpy() for k in ("x1", "x2", "x3")}
            e3, esc, _ = oracle.plf(h["x1"], h["x2"], EV, nd["left"].cpu().numpy(),
                                    nd["right"].cpu().numpy(), ones)
            assert np.array_equal(h["x3"].view(np.uint64), e3.view(np.uint64)), j
            assert np.array_equal(nd["scaler"][lo:lo + 1024].cpu().numpy(), esc), j
            if j % 64 == 0 and oracle.ref_available(np.float64):
                # and through the reference's own plf() (its double build)
                r3, rinc = oracle.ref_plf_f64(h["x1"], h["x2"], EV, nd["left"].cpu().numpy(),
                                              nd["right"].cpu().numpy(), ones)
                assert np.array_equal(h["x3"].view(np.uint64), r3.view(np.uint64)), j
                assert rinc == int(esc.sum()), j
        assert wl.sums.cpu().tolist() == [n // 4] * 512
        del wl
    torch.cuda.empty_cache()


def test_eight_ranks_gloo_rehearsal():
    """The driver's N = 8 layout rehearsed on the box's one GPU: 8 ranks under
    torch.distributed.run (gloo, every rank's device folded onto GPU 0) for the
    default node workload -- with its config.nodes512 sub-record (16 nodes, 2
    per rank) -- and for --workload nodes512: one JSON line, every rank's lnL
    in the one all-reduce, the scaler totals exact, value_device >= value,
    and the nodes512 job lnL equal to one rank's bit for bit."""
    def run(nproc, *args):
        r = _torchrun(nproc, ["--gpus", str(nproc), "--steps", "3", "--warmup", "1", "--no-cpu-baseline", *args],
                      {**os.environ, "PLFX_DIST_BACKEND": "gloo", "OMP_NUM_THREADS": "2"})
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        assert len(lines) == 1, r.stdout
        return json.loads(lines[0])

    d = run(8, "--sites", "65536", "--buffer-sets", "2", "--nodes", "16")
    assert d["n_gpus"] == 8 and d["check"] == "ok" and len(d["config"]["lnl_per_rank"]) == 8
    assert d["config"]["scaler_events_all_ranks"] == 8 * (65536 // 4)
    # N > 1 honesty fields: device-time rate and the ranks' barrier-exit spread
    assert d["value_device"] >= d["value"] > 0 and d["barrier_skew_us"] >= 0
    _assert_checked(d, 8, nodes=16)
    # BASELINE configs[3] rides along in the default invocation: 16 nodes over
    # 8 ranks, its one lnL all-reduce equal to one rank's bit for bit
    s8 = d["config"]["nodes512"]
    d1 = run(1, "--sites", "65536", "--buffer-sets", "2", "--nodes", "16")
    s1 = d1["config"]["nodes512"]
    assert s8["check"] == s1["check"] == "ok" and s8["scaling"] == "strong"
    assert s8["nodes_per_rank"] == 2 and s1["nodes_per_rank"] == 16 and s8["nodes_in_job"] == 16
    assert s8["lnl_all_nodes_all_ranks"] == s1["lnl_all_nodes_all_ranks"]
    assert s8["scaler_events_all_ranks"] == s1["scaler_events_all_ranks"] == 16 * (65536 // 4)
    assert s8["value_device"] >= s8["value"] > 0 and s8["extra_wall_s"] > 0
    assert d1["barrier_skew_us"] == 0.0 and d1["value_device"] >= d1["value"]
    e8 = run(8, "--workload", "nodes512", "--nodes", "16", "--sites", "4099")
    e1 = run(1, "--workload", "nodes512", "--nodes", "16", "--sites", "4099")
    assert e8["check"] == e1["check"] == "ok" and e8["scaling"] == "strong"
    k = "lnl_all_nodes_all_ranks"
    assert e8["config"][k] == e1["config"][k]
    assert e8["config"]["scaler_events_all_ranks"] == e1["config"]["scaler_events_all_ranks"] == 16 * ((4099 + 3) // 4)


def test_corrupted_rank_fails_every_check():
    """A single flipped bit inside one rank's check window (--corrupt-rank 1,
    after each timed region) turns the line red at world 2: exit 3,
    `check` CHECK_FAILED, and exactly one mismatched window in the node line
    and in each sub-record."""
    r = _torchrun(2, ["--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--sites", "65536",
                      "--buffer-sets", "2", "--nodes", "4", "--corrupt-rank", "1"],
                  {**os.environ, "PLFX_DIST_BACKEND": "gloo", "OMP_NUM_THREADS": "4"})
    assert r.returncode != 0, r.stdout[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    c = d["config"]
    assert d["check"] == "CHECK_FAILED"
    assert c["check_windows"] == 2 and c["windows_mismatched"] == 1
    for k in ("nodes512", "tree64"):
        assert c[k]["check"] == "CHECK_FAILED" and c[k]["windows_mismatched"] == 1, k
    for p in (c["protein"], c["protein"]["valu_fma"], c["protein"]["exact"]):
        assert p["check"] == "CHECK_FAILED" and p["windows_mismatched"] == 1
