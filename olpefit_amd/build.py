"""Build libolpe.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with
the repo snapshot to the GPU box)."""
from __future__ import annotations

import os
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


def kernel_digest() -> str:
    """16 hex digits over the device sources and flags: tags measured per-kernel
    counts (profiles/valu_counts.json) with the code they were measured on."""
    import hashlib
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
