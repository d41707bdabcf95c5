"""Identify the gfx950 machine code of a kernel inside libplfx.so.

Used to tie a committed rocprofv3 PMC record (HBM bytes per launch) to the
code it was counted on: the record carries `kernel_code_sha256` of the kernel
it measured, and bench.py only reports the record's traffic while the
library it times hashes to the same value (otherwise `traffic` is null and
`traffic_stale` true).

Layout walked here (no external tools, so it runs on the GPU box as is):
libplfx.so (ELF64) -> section `.hip_fatbin` -> its clang offload bundles
(`__CLANG_OFFLOAD_BUNDLE__`, uncompressed; one per HIP translation unit) ->
the entries whose triple names gfx950 -> those code objects (ELF64) ->
`.symtab`, merged.  A kernel's hash covers,
for every symbol that names the kernel (its mangled identifier) (all its
template instantiations, sorted by symbol name), the function's instruction
bytes and its 64-byte kernel descriptor (`<sym>.kd`) with the
position-dependent `kernel_code_entry_byte_offset` field (bytes 16..23)
zeroed -- so relinking the library with other kernels around it keeps the
hash, while any change to this kernel's instructions, register counts or
LDS size changes it.
"""
from __future__ import annotations

import hashlib
import struct
from pathlib import Path

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf: bytes):
    """[(name, addr, offset, size, link, entsize)] of an ELF64 little-endian image's sections."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not an ELF64 little-endian image")
    shoff = struct.unpack_from("<Q", elf, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stro = hdrs[shstrndx][4]

    def name(off):
        end = elf.index(b"\0", stro + off)
        return elf[stro + off:end].decode()

    return [(name(h[0]), h[3], h[4], h[5], h[6], h[9]) for h in hdrs]


def gfx950_code_objects(lib: str | Path) -> list[bytes]:
    """Every gfx950 code object embedded in `lib`: the .hip_fatbin section
    holds one clang offload bundle per HIP translation unit linked in
    (concatenated, each aligned), walked here bundle by bundle -- a kernel
    may live in any of them, whatever the link order.  Compressed bundles
    (CCOB) are refused with a ValueError."""
    data = Path(lib).read_bytes()
    secs = {s[0]: s for s in _sections(data)}
    if ".hip_fatbin" not in secs:
        raise ValueError(f"{lib}: no .hip_fatbin section")
    _, _, off, size, _, _ = secs[".hip_fatbin"]
    fat = data[off:off + size]
    if fat.lstrip(b"\0").startswith(b"CCOB"):
        raise ValueError(f"{lib}: compressed offload bundle (CCOB) not supported")
    out, pos = [], fat.find(_BUNDLE_MAGIC)
    if pos < 0:
        raise ValueError(f"{lib}: .hip_fatbin holds no uncompressed offload bundle")
    while pos >= 0:
        n = struct.unpack_from("<Q", fat, pos + len(_BUNDLE_MAGIC))[0]
        p = pos + len(_BUNDLE_MAGIC) + 8
        end = p
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            end = max(end, pos + eoff + esize)
            if "gfx950" in triple and esize:
                out.append(fat[pos + eoff:pos + eoff + esize])
        pos = fat.find(_BUNDLE_MAGIC, max(end, p))
    if not out:
        raise ValueError(f"{lib}: no gfx950 entry in the offload bundles")
    return out


def gfx950_code_object(lib: str | Path) -> bytes:
    """The first gfx950 code object of `lib` (see gfx950_code_objects)."""
    return gfx950_code_objects(lib)[0]


def _symbols(co: bytes):
    secs = _sections(co)
    symtab = next(s for s in secs if s[0] == ".symtab")
    strtab = secs[symtab[4]]
    out = []
    for i in range(symtab[3] // 24):
        st_name, st_info, _, st_shndx, st_value, st_size = struct.unpack_from(
            "<IBBHQQ", co, symtab[2] + 24 * i)
        if st_shndx == 0 or st_shndx >= len(secs):
            continue
        end = co.index(b"\0", strtab[2] + st_name)
        nm = co[strtab[2] + st_name:end].decode()
        sec = secs[st_shndx]
        out.append((nm, st_info & 0xF, sec[2] + (st_value - sec[1]), st_size))
    return out


def _named(sym: str, kernel: str) -> bool:
    """`sym` (Itanium-mangled) names the function `kernel`: its identifier
    appears length-prefixed, so plf_dna_kernel does not match
    plf_dna_kernel_x or my_plf_dna_kernel."""
    return f"{len(kernel)}{kernel}" in sym


def _all_symbols(lib: str | Path):
    """{name: (code object, type, offset, size)} over every gfx950 code object."""
    out = {}
    for co in gfx950_code_objects(lib):
        for nm, typ, off, size in _symbols(co):
            if nm not in out or (size and not out[nm][3]):
                out[nm] = (co, typ, off, size)
    return out


def kernel_code_sha256(lib: str | Path, kernel: str) -> str:
    """sha256 over every instantiation of `kernel` (base name, e.g.
    "plf_dna_f64_pair_kernel") in `lib`'s gfx950 code objects: instruction
    bytes + kernel descriptor (entry offset zeroed), by symbol name."""
    syms = _all_symbols(lib)
    funcs = sorted(nm for nm, (_, typ, _, size) in syms.items()
                   if _named(nm, kernel) and typ == 2 and size > 0)  # STT_FUNC
    if not funcs:
        raise KeyError(f"no kernel named *{kernel}* in {lib}")
    h = hashlib.sha256()
    for nm in funcs:
        co, _, off, size = syms[nm]
        h.update(nm.encode() + b"\0")
        h.update(co[off:off + size])
        kd = syms.get(nm + ".kd")
        if kd is not None:
            b = bytearray(kd[0][kd[2]:kd[2] + kd[3]])
            b[16:24] = bytes(8)  # kernel_code_entry_byte_offset: where the linker put it
            h.update(bytes(b))
    return h.hexdigest()


def kernel_instantiations(lib: str | Path, kernel: str) -> list[str]:
    return sorted(nm for nm, (_, typ, _, size) in _all_symbols(lib).items()
                  if _named(nm, kernel) and typ == 2 and size > 0)


def default_lib() -> Path:
    return Path(__file__).resolve().parent / "libplfx.so"


def stamp(kernels, lib: str | Path | None = None) -> dict:
    """The `code` stamp a PMC record carries: {kernel: kernel_code_sha256}
    for every kernel whose counters it holds."""
    lib = default_lib() if lib is None else lib
    return {k: kernel_code_sha256(lib, k) for k in sorted(set(kernels))}


def check_stamp(code: dict | None, lib: str | Path | None = None):
    """(ok, reason): whether `lib` still holds the machine code the stamp was
    taken on.  An unstamped record cannot be tied to any code: not ok."""
    if not code:
        return False, "record carries no code stamp"
    lib = default_lib() if lib is None else lib
    bad = []
    for k, h in sorted(code.items()):
        try:
            if kernel_code_sha256(lib, k) != h:
                bad.append(k)
        except (KeyError, ValueError, OSError):
            bad.append(k)
    if bad:
        return False, "code changed since the record: " + ", ".join(bad)
    return True, "code unchanged"
