"""Per-kernel machine-code identity of the gfx950 code object inside a built
library (measurement infrastructure: bench.py and tools/make_traffic.py).

A PMC record (profiles/rNN/traffic_*.json) belongs to the machine code it was
counted on.  Round 5 matched records by the sha256 of the whole kernel source
file, so an edit to one kernel (the large-K sampler) orphaned the unchanged
dense kernel's record.  This hashes what actually ran
instead: the .text bytes of each instantiation of one kernel family plus its
kernel descriptor (VGPR / LDS / scratch configuration), with the descriptor's
code-entry offset zeroed because it moves whenever another kernel grows.  The
code object has no relocations and the sampler kernels hold no PC-relative
references (checked by `pc_relative_free`), so the bytes do not depend on
where the linker placed the function.

Layout walked here:
  host ELF (.so) -> section .hip_fatbin -> clang offload bundle
  ("__CLANG_OFFLOAD_BUNDLE__", entry count, {offset, size, triple}) ->
  the hipv4-amdgcn-amd-amdhsa--gfx950 device ELF -> .symtab FUNC symbols
  (kernel entry points) and OBJECT symbols "<name>.kd" (descriptors).
"""
from __future__ import annotations

import hashlib
import struct

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _sections(elf: bytes):
    """{name: (offset, size, addr)} of a little-endian ELF64 image."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError("not an ELF64 image")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for i in range(shnum):
        name, typ, _flags, addr, off, size = struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
        hdrs.append((name, typ, addr, off, size))
    stroff = hdrs[shstrndx][3]
    out = {}
    for name, typ, addr, off, size in hdrs:
        end = elf.index(b"\0", stroff + name)
        out[elf[stroff + name:end].decode()] = (off, size, addr)
    return out


def device_code_object(lib_path: str, target: str = _TARGET) -> bytes:
    """The device ELF for `target` embedded in a hipcc-built shared library."""
    with open(lib_path, "rb") as f:
        host = f.read()
    secs = _sections(host)
    if ".hip_fatbin" not in secs:
        raise ValueError(f"{lib_path}: no .hip_fatbin section")
    off, size, _ = secs[".hip_fatbin"]
    fb = host[off:off + size]
    if not fb.startswith(_BUNDLE_MAGIC):
        raise ValueError(f"{lib_path}: unsupported offload bundle (compressed?)")
    n, = struct.unpack_from("<Q", fb, len(_BUNDLE_MAGIC))
    p = len(_BUNDLE_MAGIC) + 8
    for _ in range(n):
        eoff, esize, tlen = struct.unpack_from("<QQQ", fb, p)
        p += 24
        triple = fb[p:p + tlen].decode()
        p += tlen
        if triple == target:
            return fb[eoff:eoff + esize]
    raise ValueError(f"{lib_path}: no {target} code object")


def kernels(co: bytes):
    """{mangled kernel name: (text bytes, descriptor bytes with the entry
    offset zeroed)} for every kernel of a device code object."""
    secs = _sections(co)
    symoff, symsize, _ = secs[".symtab"]
    stroff = secs[".strtab"][0]
    funcs, kds = {}, {}
    for i in range(symsize // 24):
        name, info, _other, _shndx, value, size = struct.unpack_from("<IBBHQQ", co, symoff + 24 * i)
        typ = info & 0xF
        if typ not in (1, 2) or size == 0:       # STT_OBJECT, STT_FUNC
            continue
        s = co[stroff + name:co.index(b"\0", stroff + name)].decode()
        # a shared code object maps file offset == virtual address for its
        # loadable sections; locate through the owning section to be safe
        for off, sz, addr in secs.values():
            if addr and addr <= value < addr + sz:
                raw = co[off + value - addr:off + value - addr + size]
                break
        else:
            continue
        if typ == 2:
            funcs[s] = raw
        elif s.endswith(".kd"):
            kd = bytearray(raw)
            kd[16:24] = b"\0" * 8        # kernel_code_entry_byte_offset: layout-dependent
            kds[s[:-3]] = bytes(kd)
    return {k: (t, kds.get(k, b"")) for k, t in funcs.items()}


def mangled_prefix(family: str, first_template_arg: int | None = None) -> str:
    """Itanium-mangled prefix of lda::<family><first_template_arg, ...>
    (e.g. k_sample_big<64, ...> -> _ZN3lda12k_sample_bigILi64E)."""
    p = f"_ZN3lda{len(family)}{family}"
    if first_template_arg is not None:
        p += f"ILi{int(first_template_arg)}E"
    return p


def pc_relative_free(text: bytes) -> bool:
    """True when the kernel holds no s_getpc_b64 (gfx9 SOP1 opcode 28), i.e.
    no PC-relative data reference whose immediate would move with layout."""
    for i in range(0, len(text) - 3, 4):
        w, = struct.unpack_from("<I", text, i)
        if (w >> 23) == 0b101111101 and ((w >> 8) & 0xFF) == 28:
            return False
    return True


def family_sha256(lib_path: str, family: str, first_template_arg: int | None = None) -> str | None:
    """sha256 over every instantiation of one kernel family (sorted by name:
    each name, its text and its descriptor); None when none is present."""
    ks = kernels(device_code_object(lib_path))
    pre = mangled_prefix(family, first_template_arg)
    names = sorted(k for k in ks if k.startswith(pre))
    if not names:
        return None
    h = hashlib.sha256()
    for k in names:
        t, kd = ks[k]
        h.update(k.encode() + b"\0")
        h.update(t)
        h.update(kd)
    return h.hexdigest()


def family_of(kernel: str):
    """'k_sample_big<64, 2, 12, false>' / 'k_sample<C=8>' -> ('k_sample_big', 64)."""
    name, _, rest = kernel.partition("<")
    arg = rest.split(",")[0].split(">")[0].strip()
    if arg.startswith("C="):
        arg = arg[2:]
    return name.strip(), (int(arg) if arg.isdigit() else None)
