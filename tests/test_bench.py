"""CPU tests of bench.py's host logic: the self-contained `--gpus N` entry
(torch.distributed.run started as a child when no launcher set WORLD_SIZE,
fail-fast when too few GPUs are visible for RCCL)."""
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PLFX_DIST_BACKEND")}
    env.update(kw)
    return env


def test_gpus_n_fails_fast_without_enough_gpus():
    """--gpus 2 under the default nccl backend on a host with fewer than 2
    visible GPUs (this container has none): a clear message and a non-zero
    exit before any rank is started, no traceback."""
    t0 = time.time()
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300, env=_env(),
                       cwd=str(ROOT))
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr and "PLFX_DIST_BACKEND=gloo" in r.stderr
    assert "Traceback" not in r.stderr and r.stdout == ""
    assert time.time() - t0 < 120


def test_self_launch_command_is_the_drivers():
    """The child command is the driver's own N > 1 invocation: one node,
    N ranks, 127.0.0.1 rendezvous, bench.py with the same arguments."""
    argv = ["--gpus", "8", "--workload", "nodes512", "--steps", "5"]
    cmd = bench.self_launch_cmd(8, argv, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-len(argv) - 1].endswith("bench.py") and cmd[-len(argv):] == argv


def test_launched_rank_does_not_relaunch(monkeypatch):
    """Under a launcher (WORLD_SIZE set) bench.py must not start another one:
    main() goes straight to the rank path (checked here up to the
    --gpus/WORLD_SIZE consistency exit, before any GPU work)."""
    monkeypatch.setenv("WORLD_SIZE", "3")
    called = []
    monkeypatch.setattr(bench, "self_launch", lambda *a: called.append(a))
    try:
        bench.main(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    except SystemExit as e:
        assert "WORLD_SIZE=3" in str(e.code)
    assert called == []


def test_sites_defaults_per_workload_and_explicit_values_kept():
    """--sites unset: each workload's BASELINE size (node / nodes512 2^20,
    protein / prottree64 2^18, swemu1024 1024); an explicit --sites, 2^20
    included, is used as given (the round-4 sentinel turned an explicit 2^20
    protein request into 2^18), and the PMC key names the sites that run."""
    for wl, n in (("node", 1 << 20), ("nodes512", 1 << 20), ("tree64", 1 << 20),
                  ("protein", 1 << 18), ("prottree64", 1 << 18), ("swemu1024", 1024)):
        a = bench.parse(["--workload", wl])
        assert a.sites == n, wl
    for wl in ("protein", "prottree64", "swemu1024", "node"):
        a = bench.parse(["--workload", wl, "--sites", str(1 << 20)])
        assert a.sites == 1 << 20, wl
    assert bench.traffic_key(bench.parse(["--workload", "protein", "--exact"])).endswith("sites262144")
    assert bench.traffic_key(bench.parse(["--workload", "protein", "--sites", "1048576"])).endswith(
        "sites1048576")
    a = bench.parse([])
    assert a.workload == "node" and not a.no_nodes512 and a.nodes == 512
    assert bench.parse(["--no-nodes512"]).no_nodes512


def test_speedup_fields_labelled():
    """The node line's speed-ups: like for like against the stated baseline
    (dtype, cores) and the sw_emu path; the reference's f32 -O0 one-thread
    row kept with its basis spelled out."""
    cb = {"value": 4.0e8, "cores": 16, "swemu_path": {"value": 1.0e8, "cores": 16},
          "reference_plf_O0_f32_1thread": 4.0e6}
    out = bench.speedup_fields(1.6e10, 1.2e8, cb, "f64")
    s = out["speedup_vs_cpu_baseline"]
    assert s["excluding_pcie"] == 40.0 and s["including_pcie"] == 0.3
    assert s["vs_swemu_path_excluding_pcie"] == 160.0
    assert "f64" in s["basis"] and "16 cores" in s["basis"]
    r = out["speedup_vs_reference_plf"]
    assert r["excluding_pcie"] == 4000.0
    assert "f32" in r["basis"] and "-O0" in r["basis"] and "1 thread" in r["basis"]
    assert "not like for like" in r["basis"]
    out = bench.speedup_fields(1.0, 1.0, {"value": 1.0, "cores": 1}, "f32")
    assert "speedup_vs_reference_plf" not in out
    assert "vs_swemu_path_excluding_pcie" not in out["speedup_vs_cpu_baseline"]


class _WL:
    bytes_per_step = 12345


def _record(tmp_path, tag, code, val=4.0e8, sites=1 << 20):
    import json

    rec = {"kernel": "plf_dna_f64_pair_kernel", "sites": sites, "dtype": "f64",
           "hbm_bytes_per_launch": val}
    if code is not None:
        rec["code"] = code
    p = tmp_path / f"{tag}_node_pmc_traffic.json"
    p.write_text(json.dumps(rec))
    return p


def test_traffic_record_tied_to_code(tmp_path):
    """roofline.traffic comes only from a PMC record whose code stamp (sha256
    of the counted kernel's gfx950 machine code) matches the library being
    timed: a mismatched or unstamped record is refused (traffic null,
    traffic_stale true, traffic_source naming it); an older record that still
    matches the code is used instead of a newer stale one."""
    from plfx import codeobj

    lib = codeobj.default_lib()
    good = codeobj.stamp(["plf_dna_f64_pair_kernel"], lib)
    assert len(good["plf_dna_f64_pair_kernel"]) == 64
    a = bench.parse(["--traffic-json", str(tmp_path / "x.json")])

    t = bench.traffic_record(a, _WL(), lib)
    assert t["traffic"] is None and not t["traffic_stale"] and t["traffic_source"] is None

    _record(tmp_path, "r05", {"plf_dna_f64_pair_kernel": "0" * 64}, val=1.0)
    t = bench.traffic_record(a, _WL(), lib)
    assert t["traffic"] is None and t["traffic_stale"]
    assert t["traffic_source"].endswith("r05_node_pmc_traffic.json")
    assert "plf_dna_f64_pair_kernel" in t["traffic_note"]

    _record(tmp_path, "r04", None, val=2.0)  # unstamped: refused too
    assert bench.traffic_record(a, _WL(), lib)["traffic"] is None

    _record(tmp_path, "r03", good, val=3.0)
    t = bench.traffic_record(a, _WL(), lib)
    assert t["traffic"] == 3.0 and not t["traffic_stale"]
    assert t["traffic_source"].endswith("r03_node_pmc_traffic.json")

    _record(tmp_path, "r06", good, val=6.0, sites=4096)  # another configuration: ignored
    assert bench.traffic_record(a, _WL(), lib)["traffic"] == 3.0


def test_code_hash_names_kernels_exactly():
    """The stamp hashes every instantiation of exactly the named kernel."""
    from plfx import codeobj

    lib = codeobj.default_lib()
    inst = codeobj.kernel_instantiations(lib, "plf_dna_kernel")
    assert inst and all("14plf_dna_kernel" in s for s in inst)
    assert codeobj.kernel_code_sha256(lib, "plf_dna_kernel") != codeobj.kernel_code_sha256(
        lib, "plf_dna_f64_pair_kernel")
    ok, why = codeobj.check_stamp({"no_such_kernel": "0" * 64}, lib)
    assert not ok and "no_such_kernel" in why


def test_codeobj_walks_every_bundle(tmp_path):
    """the .hip_fatbin section holds one offload bundle per HIP
    translation unit; a kernel in a later bundle must resolve.  A synthetic
    library whose .hip_fatbin puts a padded host-only bundle in front of the
    real one still resolves every kernel to the same hash."""
    import struct

    from plfx import codeobj

    lib = codeobj.default_lib()
    data = bytearray(lib.read_bytes())
    name, addr, off, size, _, _ = next(s for s in codeobj._sections(bytes(data)) if s[0] == ".hip_fatbin")
    fat = bytes(data[off:off + size])
    # a first bundle with only a host entry, padded to 4096, then the real one
    host = b"host-x86_64-unknown-linux-gnu-"
    hdr = codeobj._BUNDLE_MAGIC + struct.pack("<Q", 1) + struct.pack("<QQQ", 4096, 0, len(host)) + host
    first = hdr + bytes(4096 - len(hdr))
    # splice: the new section content replaces the old at the same offset,
    # appended at the end of the file with the section header pointed there
    new = first + fat
    shoff = struct.unpack_from("<Q", data, 0x28)[0]
    shentsize, shnum, _ = struct.unpack_from("<HHH", data, 0x3A)
    for i in range(shnum):
        h = shoff + i * shentsize
        if struct.unpack_from("<Q", data, h + 24)[0] == off and struct.unpack_from("<Q", data, h + 32)[0] == size:
            struct.pack_into("<QQ", data, h + 24, len(data), len(new))
    data += new
    p = tmp_path / "libtwo.so"
    p.write_bytes(bytes(data))
    # one code object per HIP translation unit of libplfx (plf_kernels.hip,
    # plf_prot_valu.hip, plf_prot_valu_exact.hip), the host-only bundle
    # contributing none
    assert len(codeobj.gfx950_code_objects(p)) == len(codeobj.gfx950_code_objects(lib)) == 3
    for k in ("plf_dna_f64_pair_kernel", "plf_dna_kernel", "root_lnl_kernel", "plf_prot_valu_fma_kernel"):
        assert codeobj.kernel_code_sha256(p, k) == codeobj.kernel_code_sha256(lib, k)


def test_every_stamped_kernel_resolves():
    """Every kernel named in a committed PMC record's code stamp
    (profiles/*_pmc_traffic.json) names code that exists in the library's
    gfx950 code objects (its hash may differ when the kernel changed)."""
    import json

    from plfx import codeobj

    lib = codeobj.default_lib()
    seen = 0
    for path in sorted((ROOT / "profiles").glob("*_pmc_traffic.json")):
        code = json.loads(path.read_text()).get("code") or {}
        for k in code:
            assert codeobj.kernel_instantiations(lib, k), (path.name, k)
            seen += 1
    assert seen > 0


def test_launch_check_against_record_shapes():
    """a PMC record counts only for the dispatch it measured --
    the timed graph's kernel nodes (mangled names, grid and workgroup sizes)
    must dispatch the record's kernels with the recorded shapes."""
    mangled = "_ZN4plfx3dev23plf_dna_f64_pair_kernelILi2ELb1ELi1ELb1EEEvPKdS3_Pd"
    rec = {"plf_dna_f64_pair_kernel": [[262144, 256]]}
    ok, why = bench.launch_check(rec, [(mangled, 262144, 256)] * 20)
    assert ok and "counted grid" in why
    ok, why = bench.launch_check(rec, [(mangled, 131072, 256)])
    assert not ok and "dispatched as" in why
    ok, why = bench.launch_check(rec, [("_ZN4plfx3dev14plf_dna_kernelIfEEvv", 262144, 256)])
    assert not ok and "not dispatched" in why
    assert not bench.launch_check(None, [(mangled, 1, 1)])[0]      # old record: does not count
    assert bench.launch_check(rec, None)[0]                        # no graph: not checked
    assert bench.launch_check(None, None)[0]


def test_traffic_not_reported_under_dispatch_knobs(monkeypatch):
    """A library env knob that changes the dispatched instantiation (the
    segmented node kernel keeps the base name and the grid, so neither the
    code stamp nor the launch shapes can tell) withholds `traffic`."""
    a = bench.parse(["--steps", "1"])

    class W:
        bytes_per_step = 0

    monkeypatch.setenv("PLFX_NODE_SEGMENTS", "1")
    r = bench.traffic_record(a, W())
    assert r["traffic"] is None and "PLFX_NODE_SEGMENTS" in r["traffic_note"]
    # values that keep the default dispatch do not withhold it
    for v in ("auto", "-1", ""):
        monkeypatch.setenv("PLFX_NODE_SEGMENTS", v)
        assert "knob" not in bench.traffic_record(a, W())["traffic_note"]
    monkeypatch.delenv("PLFX_NODE_SEGMENTS")
    monkeypatch.setenv("PLFX_MAX_BLOCKS", "0")
    assert "knob" not in bench.traffic_record(a, W())["traffic_note"]
    monkeypatch.setenv("PLFX_MAX_BLOCKS", "64")
    assert "PLFX_MAX_BLOCKS" in bench.traffic_record(a, W())["traffic_note"]
    monkeypatch.delenv("PLFX_MAX_BLOCKS")
    for v in ("", "1"):
        monkeypatch.setenv("PLFX_STREAMS", v)
        assert "knob" not in bench.traffic_record(a, W())["traffic_note"]
    monkeypatch.setenv("PLFX_STREAMS", "2")
    assert "PLFX_STREAMS" in bench.traffic_record(a, W())["traffic_note"]


def test_pmc_tools_record_launch_shapes():
    """The PMC record tools read the dispatch shapes from rocprofv3's counter
    CSV (demangled or truncated kernel names), as bench.py compares them."""
    import importlib.util

    def load(name):
        spec = importlib.util.spec_from_file_location(name, ROOT / "tools" / f"{name}.py")
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        return m

    pt, ps = load("pmc_traffic"), load("pmc_step")
    assert pt.shapes(ROOT / "profiles" / "r04_node_pmc_fetch.csv", "plf_dna_f64_pair_kernel") == [[262144, 256]]
    tree = ps.launch_shapes(ROOT / "profiles" / "r04_tree64_pmc_fetch.csv")
    assert tree["plf_dna_f64_deep_kernel"] == [[131072, 512]]


def test_sub_records_arguments():
    """The default invocation's sub-records: configs[3] / [2] at --sites,
    configs[4] at --sites / 4 (2^18 by default) with at least 200 timed steps
    after 300 warm-up ones, exact only for protein_exact; opt-outs parse."""
    a = bench.parse(["--steps", "20", "--warmup", "5"])
    assert bench.SUB_RECORDS == ("nodes512", "tree64", "protein", "protein_valu", "protein_exact")
    t = bench.sub_args(a, "tree64")
    assert (t.workload, t.sites, t.steps, t.warmup, t.exact, t.tips) == ("tree64", 1 << 20, 20, 5, False, False)
    p = bench.sub_args(a, "protein")
    assert (p.workload, p.sites, p.steps, p.warmup, p.exact) == ("protein", 1 << 18, 200, 300, False)
    e = bench.sub_args(a, "protein_exact")
    assert e.exact and e.sites == 1 << 18 and bench.traffic_name(e) == "protein_exact"
    v = bench.sub_args(a, "protein_valu")
    assert v.valu and not v.exact and v.steps == 200 and bench.traffic_name(v) == "protein_valu"
    assert bench.traffic_key(v) == "protein:f64:valu:dense:fuse3:sites262144"
    assert not p.valu
    assert bench.traffic_key(t) == "tree64:f64:fma:dense:fuse3:sites1048576"
    assert bench.traffic_key(p) == "protein:f64:fma:dense:fuse3:sites262144"
    assert a.workload == "node" and a.steps == 20  # the line's own arguments are untouched
    b = bench.parse(["--no-tree64", "--no-protein", "--corrupt-rank", "1"])
    assert b.no_tree64 and b.no_protein and b.corrupt_rank == 1
    assert bench.parse([]).corrupt_rank == -1


def test_common_start_only_on_one_node():
    """the agreed start instant only when every rank shares this
    node's CLOCK_MONOTONIC and the clocks agree within 1 s; ranks on several
    machines (LOCAL_WORLD_SIZE < WORLD_SIZE) or far-apart clocks start on
    their own after the barrier, never spinning on another machine's clock."""
    assert bench.use_common_start(10.0005, 10.0, 8, {"LOCAL_WORLD_SIZE": "8"})
    assert bench.use_common_start(10.0005, 10.0, 2, {})
    assert not bench.use_common_start(10.0005, 10.0, 16, {"LOCAL_WORLD_SIZE": "8"})
    assert not bench.use_common_start(86400.0, 10.0, 8, {"LOCAL_WORLD_SIZE": "8"})
    assert not bench.use_common_start(1.0, 1.0, 8, {"LOCAL_WORLD_SIZE": "x"})


def test_flip_bit_and_window_offsets():
    """The --corrupt-rank hook flips exactly the lowest bit of one element."""
    import torch

    t = torch.arange(8, dtype=torch.float64)
    before = t.clone()
    bench.flip_bit(t, 5)
    diff = (t.view(torch.int64) ^ before.view(torch.int64)).tolist()
    assert diff == [0, 0, 0, 0, 0, 1, 0, 0]
    f = torch.ones(4, dtype=torch.float32)
    bench.flip_bit(f, 0)
    assert f[0].item() != 1.0 and f[1:].eq(1).all()


def test_region_lanes():
    """Lanes: the node and protein workloads (independent nodes on rotating
    buffer sets) alternate their steps over 2 streams by default; a workload
    without lanes, an odd set count or a count not dividing the sets is
    refused when asked for more; --lanes 1 is the single launch stream; the
    sub-records pass --lanes on to all but tree64."""
    from types import SimpleNamespace as NS

    a = bench.parse([])
    assert a.lanes is None
    assert bench.region_lanes(NS(lanes=2, R=4), a) == 2
    assert bench.region_lanes(NS(R=1), a) == 1  # tree64 / nodes512 declare none
    assert bench.region_lanes(NS(lanes=2, R=4), bench.parse(["--lanes", "1"])) == 1
    for wl, n in ((NS(lanes=2, R=4), "3"), (NS(R=4), "2"), (NS(lanes=2, R=4), "0")):
        with pytest.raises(SystemExit):
            bench.region_lanes(wl, bench.parse(["--lanes", n]))
    b = bench.parse(["--lanes", "1"])
    assert bench.sub_args(b, "protein").lanes == 1 and bench.sub_args(b, "protein_exact").lanes == 1
    assert bench.sub_args(b, "tree64").lanes is None and bench.sub_args(b, "nodes512").lanes == 1
    assert a.per_launch == 1 and bench.parse(["--per-launch", "32"]).per_launch == 32
