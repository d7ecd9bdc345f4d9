"""Per-kernel resources of the shipped library, read from its embedded gfx950 code objects.

Every HIP translation unit of liblpgnn_hip.so carries a clang offload bundle whose gfx950 entry is
an AMDHSA ELF; each kernel has a 64-byte kernel descriptor (symbol ``<name>.kd``) whose second
dword is ``private_segment_fixed_size`` -- the per-lane scratch the kernel needs.  The library's
rule is that NO shipped kernel uses scratch: the one bitwise mismatch we
ever saw between two bf16 FC tiles came from a register-spilling kernel whose spill code dropped
the last dword of a partially reused AGPR tuple (hipcc "Reload Reuse"; fc_bf16.hip header).

``python tools/kernel_resources.py [lib.so]`` prints one line per kernel; exits 1 if any uses
scratch.  ``make`` runs it after linking; tests/test_abi.py runs it too.
"""
from __future__ import annotations

import os
import struct
import subprocess
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(blob: bytes):
    """Yield the gfx950 AMDHSA ELF images of every offload bundle in ``blob``."""
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, idl = struct.unpack_from("<QQQ", blob, p)
            p += 24
            ident = blob[p:p + idl]
            p += idl
            if b"amdgcn" in ident and size:
                img = blob[pos + off:pos + off + size]
                if img[:4] != b"\x7fELF":
                    raise RuntimeError(f"compressed or unknown code object for {ident!r}")
                yield img
        pos = blob.find(MAGIC, pos + 24)


def _kernel_descriptors(elf: bytes):
    """{symbol name without '.kd': 64-byte kernel descriptor} of one ELF64 code object."""
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    secs = []
    for i in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, shoff + i * shentsize)
        secs.append((name, typ, addr, off, size, link, entsize))
    out = {}
    for (name, typ, addr, off, size, link, entsize) in secs:
        if typ != 2:  # SHT_SYMTAB
            continue
        stroff = secs[link][3]
        for k in range(size // entsize):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from(
                "<IBBHQQ", elf, off + k * entsize)
            end = elf.index(b"\0", stroff + st_name)
            sym = elf[stroff + st_name:end].decode()
            if not sym.endswith(".kd") or st_shndx == 0 or st_shndx >= len(secs):
                continue
            s = secs[st_shndx]
            fo = s[3] + (st_value - s[2])
            out[sym[:-3]] = elf[fo:fo + 64]
    return out


def kernels(lib_path: str):
    """[(mangled name, lds bytes, scratch bytes per lane)] for every kernel of the library."""
    blob = open(lib_path, "rb").read()
    rows = []
    for img in _code_objects(blob):
        for name, kd in _kernel_descriptors(img).items():
            group, private = struct.unpack_from("<II", kd, 0)
            rows.append((name, group, private))
    if not rows:
        raise RuntimeError(f"no gfx950 kernel descriptors found in {lib_path}")
    return rows


def is_ours(mangled: str) -> bool:
    """A kernel of this repository (namespace lpg), not a rocPRIM template instantiation."""
    return mangled.startswith("_ZN3lpg")


def _demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return r.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return list(names)


def main(argv):
    here = os.path.dirname(os.path.abspath(__file__))
    lib = argv[1] if len(argv) > 1 else os.path.join(here, "..", "lp-gnn_amd", "lpgnn", "liblpgnn_hip.so")
    rows = kernels(lib)
    bad = vendor = 0
    for (name, group, private), dm in zip(rows, _demangle([r[0] for r in rows])):
        ours = is_ours(name)
        flag = "ok" if not private else ("SCRATCH" if ours else "vendor")
        bad += bool(private and ours)
        vendor += bool(private and not ours)
        if (private and ours) or "-v" in argv:
            print(f"{flag:7s} scratch={private:4d} B/lane lds={group:6d} B  {dm[:160]}")
    print(f"{len(rows)} kernels: {bad} of ours use scratch; {vendor} rocPRIM library kernels do (radix sort of the "
          f"device pack, checked bitwise against the host pack by the tests)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
