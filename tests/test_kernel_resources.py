"""Register / scratch budget of the bench sampler kernels (CPU: a device-only hipcc
compile with the resource-usage remarks, no GPU).

The 64x64 two-source sampler runs 12 waves per workgroup (3 per SIMD) for most
launches, which caps a wave at 168 VGPRs; DESIGN.md §3 relies on it having no scratch
at all (spilled column terms once cost a 16-wave variant 0.25 GB of extra HBM writes
per launch).  The 16-wave samplers (configs[2], configs[1]) must fit 128 VGPRs with at
most the one small spill DESIGN.md §3 accounts for.  A change that breaks either fails
here before it reaches a GPU.

"No scratch" means no scratch memory instruction in the kernel and no spilled VGPR:
since the work-unit loop the compiler reserves a 36-B private segment
frame for these kernels that no instruction touches (its SGPR spills live in VGPR
lanes), so the reserved size alone is not the criterion.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def usage():
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("hipcc not available")
    from olpefit_amd import build
    flags = [f for f in build.FLAGS if f not in ("-shared", "-fPIC", "-Wall",
                                                  "-Wno-unused-function")]
    cmd = [HIPCC, *flags, "--cuda-device-only", "-c", "-o", os.devnull,
           os.path.join(REPO, "olpefit_amd", "csrc", "olpe.hip"),
           "-Rpass-analysis=kernel-resource-usage"]
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "olpe.s")
        cmd[cmd.index("-c")] = "-S"
        cmd[cmd.index(os.devnull)] = asm
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=900).stderr
        text = open(asm).read()
    # scratch memory instructions per kernel body
    bodies = {}
    for m in re.finditer(r"^(_Z\S*olpe_gibbs_kernel\S*):[^\n]*\n(.*?)^\.Lfunc_end", text, re.M | re.S):
        bodies[m.group(1)] = len(re.findall(r"^\s+(scratch_|buffer_(load|store)\S*.*off(en|set)?.*s\[0:3\])",
                                            m.group(2), re.M))
    res = {}
    name = None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            res[name] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill): (\d+)", line)
        if m and name:
            res[name][m.group(1)] = int(m.group(2))
    for name, v in res.items():
        v["scratch_insts"] = bodies.get(name, -1)
    return res


def _kernel(usage, nsrc, nt, lds, wpb, fast):
    key = (f"olpe_gibbs_kernelILi{nsrc}ELi{nt}ELb{int(lds)}ELi{wpb}ELb{int(fast)}E")
    hits = [v for k, v in usage.items() if key in k]
    assert hits, f"kernel {key} not found in the resource remarks"
    return hits[0]


@pytest.mark.parametrize("fast", [True, False])
def test_bench_sampler_has_no_scratch(usage, fast):
    k = _kernel(usage, 2, 64, True, 12, fast)
    assert k["scratch_insts"] == 0 and k["VGPRs Spill"] == 0, k
    assert k["VGPRs"] <= 168, k


def test_sixteen_wave_samplers_fit_four_waves_per_simd(usage):
    # the configs[2] / configs[1] FAST sampler and the 2-source EXACT one at 16 waves
    # (DESIGN.md §3): 128 VGPRs at most; FAST keeps the shape-table prefetch at the cost
    # of one 8-byte spill (one store per walker, three reloads), EXACT spills nothing
    k = _kernel(usage, 2, 64, True, 16, True)
    assert k["VGPRs"] <= 128 and k["VGPRs Spill"] <= 2 and 0 <= k["scratch_insts"] <= 4, k
    k = _kernel(usage, 2, 64, True, 16, False)
    assert k["VGPRs"] <= 128 and k["VGPRs Spill"] == 0 and k["scratch_insts"] == 0, k


def test_other_bench_configs_have_no_scratch(usage):
    # configs[4] (3-source 128x128: the lockstep LDS-ring sampler of 12 waves and the
    # global-memory sampler, 3 workgroups of 4 waves) and the 3-source 64x64 LDS sampler
    for args in [(3, 128, False, 12, True), (3, 128, False, 4, True), (3, 64, True, 12, True)]:
        k = _kernel(usage, *args)
        assert k["scratch_insts"] == 0 and k["VGPRs Spill"] == 0, (args, k)


def test_moment_fold_kernels_have_no_scratch():
    """The HBM-bound fold kernels (olpe_moments.hip): the one-wave-per-
    walker fold keeps 16 loads in flight per lane in registers -- no spill, and few
    enough VGPRs that the 4-wave blocks fill the CUs."""
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("hipcc not available")
    from olpefit_amd import build
    flags = [f for f in build.FLAGS if f not in ("-shared", "-fPIC", "-Wall",
                                                  "-Wno-unused-function")]
    cmd = [HIPCC, *flags, "--cuda-device-only", "-c", "-o", os.devnull,
           os.path.join(REPO, "olpefit_amd", "csrc", "olpe_moments.hip"),
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600).stderr
    res, name = {}, None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            res[name] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill): (\d+)", line)
        if m and name:
            res[name][m.group(1)] = int(m.group(2))
    for kern in ("fold_rows_kernel", "fold_cols_kernel"):
        hits = [v for k, v in res.items() if kern in k]
        assert hits, kern
        v = hits[0]
        assert v["ScratchSize [bytes/lane]"] == 0 and v["VGPRs Spill"] == 0, (kern, v)
        assert v["VGPRs"] <= 128, (kern, v)
