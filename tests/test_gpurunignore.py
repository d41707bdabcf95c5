"""CPU test: nothing a GPU run loads is listed in .gpurunignore (the snapshot
that travels to the GPU box omits those paths): the built libraries, the
oracle and its reference build, the golden fixtures, the code-stamped traffic
records bench.py reads, and the sources."""
import fnmatch
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

NEEDED = [
    "amd-versal-phylogenetic-likelihood-function_amd/plfx/libplfx.so",
    "amd-versal-phylogenetic-likelihood-function_amd/plfx/__init__.py",
    "amd-versal-phylogenetic-likelihood-function_amd/csrc/plf_dna.hpp",
    "oracle/liboracle.so",
    "oracle/_ref/libplfref_O0.so",
    "oracle/_ref/libplfref_f64_O0.so",
    "oracle/_ref/libplfref_fma.so",
    "oracle/_ref/libplfref_f64_fma.so",
    "tests/golden/tree64.npz",
    "tests/golden/hostmem_f32_n1024.npz",
    "profiles/r04_node_pmc_traffic.json",
    "bench.py",
    "__graft_entry__.py",
]


def patterns():
    out = []
    for ln in (ROOT / ".gpurunignore").read_text().splitlines():
        ln = ln.strip()
        if ln and not ln.startswith("#"):
            out.append(ln)
    return out


def ignored(rel, pats):
    for p in pats:
        if p.startswith("./"):  # anchored at the top
            if fnmatch.fnmatch(rel, p[2:]) or rel.startswith(p[2:].rstrip("*") + "/") and p.endswith("/*"):
                return True
        elif fnmatch.fnmatch(rel, p) or fnmatch.fnmatch(Path(rel).name, p):
            return True
    return False


def test_nothing_a_gpu_run_loads_is_ignored():
    pats = patterns()
    bad = [r for r in NEEDED if ignored(r, pats)]
    assert not bad, bad
