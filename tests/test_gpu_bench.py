"""GPU tests of bench.py's single-rank lines other than the driver's default:
every workload the bench can time carries its own oracle windows (VERDICT r05
item 3 applies to every record, not only the N > 1 ones), and the default
invocation also runs in f32 with all its sub-records.  Small sizes; one bench
process per case (the test runner itself runs once)."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def _bench(*args, expect_rc=0):
    cmd = [sys.executable, str(ROOT / "bench.py"), "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--buffer-sets", "2", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(ROOT))
    assert r.returncode == expect_rc, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("args,windows", [
    (("--workload", "tree64", "--sites", "4099"), 63),
    (("--workload", "tree64", "--tips", "--sites", "4099"), 63),
    (("--workload", "tree64", "--fuse", "2", "--sites", "4099"), 63),
    (("--workload", "protein", "--sites", "4099"), 1),
    (("--workload", "protein", "--exact", "--sites", "4099"), 1),
    (("--workload", "protein", "--valu", "--sites", "4099"), 1),
    (("--workload", "protein", "--tips", "--sites", "4099"), 1),
    (("--workload", "protein", "--dtype", "f32", "--sites", "4099"), 1),
    (("--workload", "nodes512", "--nodes", "6", "--sites", "4099"), 6),
    (("--workload", "nodes512", "--nodes", "70", "--per-launch", "32", "--sites", "4099"), 70),
    (("--workload", "node", "--lanes", "1", "--sites", "4099"), 1),
    (("--workload", "node", "--launch", "bound", "--sites", "4099"), 1),
    (("--workload", "protein", "--lanes", "1", "--sites", "4099"), 1),
    (("--workload", "protein", "--launch", "bound", "--valu", "--sites", "4099"), 1),
])
def test_workload_lines_carry_oracle_windows(args, windows):
    d = _bench(*args)
    c = d["config"]
    assert d["check"] == "ok"
    assert c["check_windows"] == windows and c["windows_mismatched"] == 0
    assert c["region_start"] == "single rank"
    assert d["value"] > 0 and d["roofline"]["frac"] > 0
    # node / protein steps alternate over 2 streams unless --lanes 1
    want = 1 if "--lanes" in args or args[1] == "tree64" else 2
    assert c["lanes"] == want == d["roofline"]["lanes"]


def test_default_invocation_f32_with_every_sub_record():
    """The default command in f32: the node line and its four sub-records,
    each oracle-checked (tree64 against the reference's plf() composed per
    node in its float build, or the oracle's traversal)."""
    d = _bench("--dtype", "f32", "--sites", "65536", "--nodes", "4")
    c = d["config"]
    assert d["check"] == "ok" and d["dtype"] == "f32"
    assert c["check_windows"] == 1 and c["windows_mismatched"] == 0
    for k, n in (("nodes512", 4), ("tree64", 63)):
        assert c[k]["check"] == "ok" and c[k]["check_windows"] == n and c[k]["windows_mismatched"] == 0
        assert c[k]["dtype"] == "f32"
    for p in (c["protein"], c["protein"]["exact"]):
        assert p["check"] == "ok" and p["check_windows"] == 1 and p["dtype"] == "f32"
        assert p["lanes"] == 2
    assert c["lanes"] == 2 and c["nodes512"]["lanes"] == 2 and c["tree64"]["lanes"] == 1
    assert "valu_fma" not in c["protein"]  # the VALU FMA form is f64 only


def test_corrupted_single_rank_line_fails():
    """--corrupt-rank 0 at one rank: the node line and every sub-record fail
    their windows, the command exits 3."""
    d = _bench("--sites", "65536", "--nodes", "2", "--corrupt-rank", "0", expect_rc=3)
    c = d["config"]
    assert d["check"].startswith("CHECK_FAILED")
    assert c["windows_mismatched"] == 1
    for k in ("nodes512", "tree64"):
        assert c[k]["check"] == "CHECK_FAILED" and c[k]["windows_mismatched"] == 1
    for p in (c["protein"], c["protein"]["valu_fma"], c["protein"]["exact"]):
        assert p["windows_mismatched"] == 1 and p["check"] == "CHECK_FAILED"


def test_sweep_small_sites_one_and_two_lanes():
    """bench.py --sweep: per-call cost at small site counts on one stream and
    over two lanes (independent outputs), every path's outputs checked."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--sweep", "--sweep-sites", "1,1000,65537"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(ROOT))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert d["check"] == "ok" and [row["sites"] for row in d["rows"]] == [1, 1000, 65537]
    for row in d["rows"]:
        assert row["check"] == "ok" and 0 < row["graph_two_lanes_us_per_call"] and 0 < row["graph_us_per_call"]
