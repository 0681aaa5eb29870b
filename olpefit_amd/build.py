"""Build libolpe.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with
the repo snapshot to the GPU box)."""
from __future__ import annotations

import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libolpe.so")
SOURCES = [os.path.join(CSRC, f) for f in ("olpe.hip", "olpe_comm.hip", "olpe_moments.hip",
                                            "olpe_csv.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("olpe_device.h", "olpe_internal.h",
                                                 "exp_table.h", "olpe_comm_proto.h")] + [
    os.path.join(REPO, "include", h) for h in ("olpe.h", "olpe_test.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-shared", "-std=c++17",
         # numpy evaluates a*b + c as two rounded ops; keep that order in the
         # control path and the per-pixel expression (fma only where written)
         "-ffp-contract=off",
         # MachineLICM hoists the loop's FP64 constants (ocml polynomial coefficients,
         # LDS slice addresses) out of the sampler loop into registers and then spills
         # them: without it the sampler kernel has no spills (+5 % fast, +6 % 3-source)
         "-mllvm", "-disable-machine-licm",
         "-Wall", "-Wno-unused-function"]


def _elf_sections(data: bytes) -> dict:
    """{name: bytes} of the sections of an ELF64 little-endian image ({} if it is none)."""
    import struct
    if len(data) < 64 or data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        return {}
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    if shoff == 0 or shoff + shnum * shentsize > len(data) or shstrndx >= shnum:
        return {}
    def sec(i):
        return struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
    _, _, _, _, stroff, _ = sec(shstrndx)
    out = {}
    for i in range(shnum):
        nm, _, _, _, off, size = sec(i)
        end = data.index(b"\0", stroff + nm)
        out[data[stroff + nm:end].decode()] = data[off:off + size]
    return out


def _elf_section(path: str, name: str) -> bytes:
    """The bytes of one section of an ELF64 little-endian file (None if absent)."""
    with open(path, "rb") as f:
        return _elf_sections(f.read()).get(name)


# the sections of a device code object that carry its code: instructions, kernel
# descriptors, metadata (register counts, LDS / scratch sizes)
CODE_SECTIONS = (".text", ".rodata", ".note")


def fatbin_digest(fat: bytes, kernel: bytes = b"olpe_gibbs_kernel") -> str:
    """kernel_digest of a .hip_fatbin section: the hash of the code sections of the
    device code objects in the clang offload bundles that name `kernel` (all bundles if
    none does; a bundle's raw bytes where it holds no parsable code object).  Symbol
    tables and hash sections are left out: their order follows the per-build unit ids
    (__hip_cuid_*), which change with the compile command, not with the code."""
    import hashlib
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), fat)]
    bundles = [fat[a:b] for a, b in zip(starts, starts[1:] + [len(fat)])] or [fat]
    mine = [b for b in bundles if kernel in b] or bundles
    h = hashlib.sha256(b"code:")
    for b in mine:
        secs = {}
        i = b.find(b"\x7fELF")
        while i >= 0 and not secs:
            secs = _elf_sections(b[i:])
            i = b.find(b"\x7fELF", i + 4)
        if any(n in secs for n in CODE_SECTIONS):
            for n in CODE_SECTIONS:
                h.update(n.encode() + secs.get(n, b""))
        else:
            h.update(b"raw:" + b)
    return h.hexdigest()[:16]


def kernel_digest(lib: str = LIB) -> str:
    """16 hex digits identifying the sampler's device code: tags measured per-kernel
    counts (profiles/valu_counts.json) with the code they were measured on.  It is the
    hash of the code sections of the built library's code object that holds the sampler
    kernel (its .hip_fatbin section has one clang offload bundle per HIP source: an edit
    to host code, a comment, a diagnostic build's hook, another source's kernels
    (olpe_moments.hip) or a change of the compile command's source list leaves it
    unchanged); without a library, the hash of the flags and the device
    sources' text."""
    import hashlib
    try:
        fat = _elf_section(lib, ".hip_fatbin")
    except OSError:
        fat = None
    if fat:
        return fatbin_digest(fat)
    h = hashlib.sha256(" ".join(FLAGS).encode())
    for f in ("olpe.hip", "olpe_device.h", "exp_table.h"):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def needs_build(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return LIB
    tmp = LIB + ".tmp"
    cmd = [HIPCC, *FLAGS, "-o", tmp, *SOURCES, "-lrccl"]
    if verbose:
        print("[olpefit_amd] " + " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    if "--print-flags" in sys.argv:      # for tools/diag_build.sh and tools/build_rev.sh
        print(" ".join(f for f in FLAGS if f not in ("-Wall", "-Wno-unused-function")))
    else:
        build(force="--force" in sys.argv)
