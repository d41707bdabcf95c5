"""CPU tests of the C-ABI library: it loads, exports exactly what
include/plfx.h declares, and its host-side sizing/packing (testbench_info,
app/src/include.h:150-266; packing, app/src/host_mem.cpp:221-243) equals the
oracle's restatement.  No GPU compute is issued here."""
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import PKG, ROOT

HEADER = ROOT / "include" / "plfx.h"
LIB = PKG / "plfx" / "libplfx.so"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(plfx_[a-z0-9_]+)\s*\(", text)))


def exported_functions():
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], check=True,
                         capture_output=True, text=True).stdout
    return sorted({l.split()[-1] for l in out.splitlines() if " T " in l})


def test_library_built():
    assert LIB.exists(), "run __graft_entry__.build() first"


def test_exports_match_header():
    decl = declared_functions()
    assert len(decl) >= 20
    assert exported_functions() == decl


def test_python_binding_lists_all_exports():
    import plfx

    assert sorted(plfx.EXPORTS) == declared_functions()
    L = plfx.load()
    for name in plfx.EXPORTS:
        assert getattr(L, name) is not None


def test_version():
    import plfx

    assert plfx.load().plfx_get_version() == 10300


def _cases():
    rng = np.random.default_rng(5)
    cases = [(1024, 1, 8192, 1, 1), (1000, 3, 1024, 0, 1), (10**6, 9, 8192, 1, 1),
             (1, 1, 1024, 0, 1), (17, 2, 16288, 1, 1), (999, 4, 1024, 0, 0), (2**27, 8, 16384, 1, 1)]
    for _ in range(40):
        N = int(rng.integers(1, 5_000_000))
        P = int(rng.integers(1, 10))
        if (P - 1) * -(-N // P) >= N:
            continue
        W = int(rng.choice([1024, 8192, 16288, 16384]))
        cases.append((N, P, W, int(rng.integers(0, 2)), int(rng.integers(0, 2))))
    return cases


@pytest.mark.parametrize("N,P,W,layout,aie", _cases())
def test_testbench_sizing_matches_oracle(oracle, N, P, W, layout, aie):
    import plfx

    t = plfx.Testbench(N, P, W, layout, aie)
    o = oracle.Testbench(N, P, W, layout, aie)
    assert t.alignments_per_instance() == o.alignments_per_instance()
    assert t.alignments_padding() == o.alignments_padding()
    assert t.elements_per_instance() == o.elements_per_instance()
    assert t.instance_elements_left() == o.instance_elements_left()
    assert t.instance_elements_right() == o.instance_elements_right()
    assert t.num_windows_per_instance() == o.num_windows_per_instance()
    for k in range(P):
        assert t.alignments_per_instance(k) == o.alignments_per_instance(k)
        assert t.instance_site_offset(k) == o.instance_site_offset(k)
        assert t.instance_active_elements_left(k) == o.instance_active_elements_left(k)
        assert t.instance_active_elements_right(k) == o.instance_active_elements_right(k)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("layout,P,W", [(0, 3, 1024), (1, 3, 1024), (1, 1, 8192), (0, 2, 16288)])
def test_pack_instance_matches_oracle(oracle, dtype, layout, P, W):
    import plfx

    n = 1000
    d = oracle.gen_hostmem(n, dtype, 3)
    t = plfx.Testbench(n, P, W, layout, plfx.AIE_WINDOW)
    o = oracle.Testbench(n, P, W, layout)
    for k in range(P):
        L, R = t.pack_instance(k, d["EV"], d["left"], d["right"], d["x1"], d["x2"])
        oL, oR = oracle.pack_instance(o, k, d["EV"], d["left"], d["right"], d["x1"], d["x2"])
        assert np.array_equal(L, oL) and np.array_equal(R, oR)


def build_dropin(tmp_dir):
    exe = Path(tmp_dir) / "dropin_main"
    src = ROOT / "tests" / "dropin_main.cpp"
    r = subprocess.run(["g++", "-O1", "-std=c++17", f"-I{ROOT / 'include'}", str(src), "-o", str(exe),
                        f"-L{PKG / 'plfx'}", "-lplfx", f"-Wl,-rpath,{PKG / 'plfx'}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_dropin_header_compiles(tmp_path):
    """include/plfx_plf.hpp provides plf() with the reference's signature."""
    assert build_dropin(tmp_path).exists()
