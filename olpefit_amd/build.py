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
SOURCES = [os.path.join(CSRC, f) for f in ("olpe.hip", "olpe_comm.hip", "olpe_moments.hip", "olpe_csv.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("olpe_device.h", "olpe_internal.h",
                                                 "exp_table.h")] + [
    os.path.join(REPO, "include", "olpe.h")]
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


def _elf_section(path: str, name: str) -> bytes:
    """The bytes of one section of an ELF64 little-endian file (None if absent)."""
    import struct
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        return None
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sec(i):
        return struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
    _, _, _, _, stroff, _ = sec(shstrndx)
    for i in range(shnum):
        nm, _, _, _, off, size = sec(i)
        end = data.index(b"\0", stroff + nm)
        if data[stroff + nm:end].decode() == name:
            return data[off:off + size]
    return None


def fatbin_digest(fat: bytes, kernel: bytes = b"olpe_gibbs_kernel") -> str:
    """kernel_digest of a .hip_fatbin section: the hash of the clang offload bundles
    that name `kernel` (all of them if none does)."""
    import hashlib
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), fat)]
    bundles = [fat[a:b] for a, b in zip(starts, starts[1:] + [len(fat)])] or [fat]
    mine = [b for b in bundles if kernel in b] or bundles
    return hashlib.sha256(b"fatbin:" + b"".join(mine)).hexdigest()[:16]


def kernel_digest(lib: str = LIB) -> str:
    """16 hex digits identifying the sampler's device code: tags measured per-kernel
    counts (profiles/valu_counts.json) with the code they were measured on.  It is the
    hash of the built library's code-object bundles that hold the sampler kernel (its
    .hip_fatbin section has one clang offload bundle per HIP source: the same bytes
    whenever that source's device code is the same -- an edit to host code, a comment,
    a diagnostic build's hook or another source's kernels (olpe_moments.hip) leaves it
    unchanged); without a library, the hash of the flags and the device sources'
    text."""
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
