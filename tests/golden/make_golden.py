#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run once in the container that has /root/reference (the GPU box does not):

    make -C oracle && python tests/golden/make_golden.py

Every expected OUTPUT here comes from the reference's own plf()
(/root/reference/app/src/plf.cpp, built unmodified into
oracle/_ref/libplfref_O0.so with the reference's host flags) or from the
reference's own AIE test data (/root/reference/aie/data).  The INPUTS follow
the reference's host_mem protocol (app/src/host_mem.cpp:179-209) with a fixed
seed, drawn by oracle/plf_oracle.c's restatement of std::mt19937 +
std::uniform_real_distribution<double>; that engine is itself pinned by
mt19937.npz, whose draws come from the C++ standard library (a 20-line probe
program this script writes and compiles in a temp dir).

Files:
  aie_kat.npz          AIE golden vectors + stimuli (aie/data), parsed to floats
  mt19937.npz          std::mt19937(20250117) raw draws + canonical doubles
  hostmem_f32_n*.npz   reference plf() x3 bit patterns, per-site scaler bytes,
                       scalerIncrement; inputs included for the small sizes
  hostmem_f32_n65536.json  sha256 of the reference x3 / scaler bytes + sums
  edge_f32.npz         hand-built edge sites (exact 2^-32 boundary, NaN, inf,
                       negative zero, denormals, all-zero, ragged weights)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "oracle"))
import oracle as O  # noqa: E402

OUT = Path(__file__).resolve().parent


def ref_per_site(x1, x2, EV, left, right, wgt):
    """Reference plf() run site by site to recover the per-site scaler byte
    (the reference CPU path only returns the weighted sum)."""
    n = x1.size // 16
    x3, inc = O.ref_plf(x1, x2, EV, left, right, wgt)
    ones = np.ones(1, np.int32)
    sc = np.empty(n, np.uint8)
    for i in range(n):
        _, s = O.ref_plf(x1[16 * i:16 * i + 16], x2[16 * i:16 * i + 16], EV, left, right, ones)
        sc[i] = s
    return x3, sc, inc


def make_mt():
    src = r"""
#include <random>
#include <cstdio>
int main(){ std::mt19937 g(20250117u);
  for(int i=0;i<2000;i++) printf("%u\n", (unsigned)g());
  std::mt19937 h(20250117u); std::uniform_real_distribution<> dis(0.0f,1.0f);
  for(int i=0;i<1000;i++) printf("%a\n", dis(h));
  return 0; }
"""
    with tempfile.TemporaryDirectory() as td:
        p = Path(td)
        (p / "mt.cpp").write_text(src)
        subprocess.run(["g++", "-O1", "-o", str(p / "mt"), str(p / "mt.cpp")], check=True)
        out = subprocess.run([str(p / "mt")], check=True, capture_output=True, text=True).stdout.split()
    raw = np.array([int(t) for t in out[:2000]], np.uint32)
    dbl = np.array([float.fromhex(t) for t in out[2000:]], np.float64)
    np.savez_compressed(OUT / "mt19937.npz", seed=np.uint32(20250117), raw=raw, canonical=dbl)


def make_kat():
    k = O.parse_aie_kat()
    np.savez_compressed(OUT / "aie_kat.npz", **{kk: np.asarray(v) for kk, v in k.items()})
    # the reference plf() on the KAT site is exactly the golden (checked in tests)


def make_hostmem(n, with_inputs):
    g = O.gen_hostmem(n, np.float32)
    x3, sc, inc = ref_per_site(g["x1"], g["x2"], g["EV"], g["left"], g["right"], g["wgt"])
    assert int(sc.sum()) == inc
    d = dict(seed=np.uint32(O.SEED), n=np.int64(n), x3=x3, scaler=sc, scalerIncrement=np.int64(inc))
    if with_inputs:
        d.update({k: g[k] for k in ("EV", "left", "right", "x1", "x2", "wgt")})
    np.savez_compressed(OUT / f"hostmem_f32_n{n}.npz", **d)


def make_hash(n):
    g = O.gen_hostmem(n, np.float32)
    x3, inc = O.ref_plf(g["x1"], g["x2"], g["EV"], g["left"], g["right"], g["wgt"])
    # per-site bytes via weights = 2^site-bit trick is not possible; use
    # the documented generator invariant instead: every 4th site scales.
    rec = dict(seed=O.SEED, n=n, scalerIncrement=int(inc),
               x3_sha256=hashlib.sha256(x3.tobytes()).hexdigest(),
               source="reference plf() (oracle/_ref/libplfref_O0.so), host_mem protocol")
    (OUT / f"hostmem_f32_n{n}.json").write_text(json.dumps(rec, indent=1) + "\n")


def make_edge():
    """Edge sites: inputs hand-picked so that x3 hits the scaling boundary.

    With left = right = identity-ish P and EV = identity, x3[c*4+l] =
    x1[c*4+l]*x2[c*4+l]; this lets us place x3 values exactly."""
    eye = np.eye(4, dtype=np.float32).reshape(16)
    left = np.tile(eye, 4)
    right = np.tile(eye, 4)
    EV = eye.copy()
    m = np.float32(2.0 ** -32)
    below = np.nextafter(m, np.float32(0))
    vals = [
        np.full(16, below),                      # all just below -> scale
        np.full(16, m),                          # exactly 2^-32 -> no scale (strict <)
        np.r_[np.full(15, below), m],            # one at boundary -> no scale
        np.r_[np.full(15, below), -below],       # negative tiny -> scale (|x|)
        np.zeros(16),                            # all zero -> scale
        -np.zeros(16),                           # negative zeros -> scale
        np.r_[np.full(15, below), np.nan],       # NaN -> no scale
        np.r_[np.full(15, below), np.inf],       # inf -> no scale
        np.full(16, np.float32(1e-40)),          # denormals -> scale
        np.full(16, np.float32(0.5)),            # normal -> no scale
        np.r_[np.full(8, below), np.full(8, np.float32(3.0))],
        np.full(16, np.float32(-1e-11)),         # negative -> scale
    ]
    x1 = np.concatenate([np.asarray(v, np.float32) for v in vals])
    x2 = np.ones_like(x1)
    n = x1.size // 16
    wgt = (np.arange(n, dtype=np.int32) * 7 + 3).astype(np.int32)
    x3, sc, inc = ref_per_site(x1, x2, EV, left, right, np.ones(n, np.int32))
    x3w, incw = O.ref_plf(x1, x2, EV, left, right, wgt)
    assert np.array_equal(x3.view(np.uint32), x3w.view(np.uint32))
    np.savez_compressed(OUT / "edge_f32.npz", EV=EV, left=left, right=right, x1=x1, x2=x2,
                        wgt=wgt, x3=x3, scaler=sc, scalerIncrement=np.int64(incw))


def make_tree64():
    """BASELINE configs[2]'s 64-taxon post-order sweep, as the composition of
    the reference's own plf() (oracle.ref_traverse: the unmodified plf.cpp,
    float build and double instantiation, one call per inner node), dense, state-coded and
    mixed tips: per op the sha256 of the parent CLV's bytes, the
    per-site scaler bytes and the weighted scaler sum, plus the root CLV."""
    d = {}
    for dt in (np.float32, np.float64):
        for mode in O.TREE_GOLDEN_TIPS:
            k = f"{'f32' if dt == np.float32 else 'f64'}_{mode}"
            c = O.tree_golden_case(dt, mode)
            nops = c["ops"].shape[0]
            clv = [t.copy() for t in c["tips"]] + [np.zeros(16 * c["n"], dt) for _ in range(nops)]
            sums, scal = O.ref_traverse(c["ops"], clv, c["pm"], c["EV"], c["n"], c["wgt"], want_scalers=True)
            assert sums.sum() > 0
            d[f"{k}_inputs_sha256"] = np.array(O.tree_case_digest(c))
            d[f"{k}_x3_sha256"] = np.array([O.clv_digest(clv[int(p)]) for p in c["ops"][:, 0]])
            d[f"{k}_scaler"] = np.stack(scal)
            d[f"{k}_sums"] = sums
            d[f"{k}_root"] = clv[int(c["ops"][-1, 0])]
    d["n"] = np.int64(O.TREE_GOLDEN_N)
    d["seed"] = np.int64(O.TREE_GOLDEN_SEED)
    d["source"] = np.array("reference plf() per inner node (oracle/_ref/libplfref_O0.so, "
                           "libplfref_f64_O0.so), oracle.ref_traverse")
    np.savez_compressed(OUT / "tree64.npz", **d)


def main():
    if O.ref_lib("O0") is None:
        sys.exit("oracle/_ref/libplfref_O0.so missing: run `make -C oracle` where /root/reference exists")
    make_mt()
    make_kat()
    make_hostmem(1024, True)
    make_hostmem(1000, True)
    make_hostmem(4096, False)
    make_hash(65536)
    make_edge()
    make_tree64()
    for f in sorted(OUT.iterdir()):
        print(f"{f.name:32s} {f.stat().st_size:9d} B")


if __name__ == "__main__":
    main()
