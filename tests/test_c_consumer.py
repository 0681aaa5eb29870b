"""The C-ABI from plain C (tests/c/abi_consumer.c, gcc -std=c99 -Wall -Werror against
include/olpe.h and the in-tree libolpe.so): the header compiles without a C++ compiler,
the library links and runs from a C program with no Python in it, and -- on the GPU --
the one-shot entry point olpe_run_gibbs reproduces the reference's own
trajectories (tests/golden/c32.npz, written by apf_step2.py's lines) from C."""
import csv
import io
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "olpefit_amd")


@pytest.fixture(scope="module")
def consumer(tmp_path_factory):
    if not os.path.exists(os.path.join(LIBDIR, "libolpe.so")):
        pytest.fail("libolpe.so not built (python -m olpefit_amd.build)")
    exe = str(tmp_path_factory.mktemp("c") / "abi_consumer")
    cmd = ["gcc", "-std=c99", "-O1", "-Wall", "-Wextra", "-Werror",
           "-I", os.path.join(REPO, "include"), os.path.join(REPO, "tests", "c", "abi_consumer.c"),
           "-L", LIBDIR, "-lolpe", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath-link,/opt/rocm/lib",
           "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_consumer_host_calls(consumer):
    """Host-only entry points from C: the version, the device count, the chain-row
    formatter (the bytes Python's csv.writer writes for the reference's float rows, the
    NaN seed row first), and olpe_create -- an error on a host without a GPU, never a CPU
    fallback."""
    from olpefit_amd import _lib
    lib = _lib.load()
    r = subprocess.run([consumer, "csv"], capture_output=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = r.stdout.decode()                  # (bytes: keep csv.writer's \r\n)
    assert out.startswith(f"version {lib.olpe_version()}\n")
    import ctypes as C
    n = C.c_int(0)
    lib.olpe_device_count(C.byref(n))
    assert f"\ndevices {n.value}\n" in out
    buf = io.StringIO(newline="")
    w = csv.writer(buf)
    w.writerow([float("nan")] * 3)
    w.writerows([[1.0, 0.1, -2.5e-7], [12345678901234567.0, 1e16, 0.0]])
    assert buf.getvalue() in out
    if n.value == 0:
        assert out.rstrip().endswith("create rc -2")      # OLPE_EHIP, no context
    else:
        assert out.rstrip().endswith("create rc 0 ctx")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fast", "exact"])
def test_c_consumer_runs_the_reference_trajectories(consumer, golden, tmp_path, mode):
    """olpe_run_gibbs from C on the 32x32 fixture's cutout, start and seeds: every
    walker's state after each iteration equals the reference's own trajectory (the
    tolerances of test_gpu_parity.py) and the tries / accepts counters are the ones the
    reference's accept decisions give."""
    from olpefit_amd import core
    g = golden("c32")
    img = np.asarray(g["image"], np.float32)
    n = img.shape[0]
    mask, pois2, rn2, _, _ = core.noise_model(img, 1.0, 1, 1, 2)
    seeds = np.asarray(g["seeds"], np.uint32)
    W = len(seeds)
    L = int(g["traj_len"].min())
    p0 = np.array(g["p_init"], np.float64)
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(np.array([n, 2, W, L, 1 if mode == "fast" else 0], "<i4").tobytes())
        f.write(np.array([rn2], "<f8").tobytes())
        f.write(np.ascontiguousarray(img, "<f4").tobytes())
        f.write(np.ascontiguousarray(pois2, "<f4").tobytes())
        f.write(np.ascontiguousarray(mask, np.uint8).tobytes())
        f.write(seeds.astype("<u4").tobytes())
        f.write(p0.astype("<f8").tobytes())
    outp = tmp_path / "out.bin"
    r = subprocess.run([consumer, "run", str(inp), str(outp)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    print(r.stdout.strip())
    # the initial chi^2 the C program computed through olpe_chi2_batch, against the
    # reference's (apf_step2.py:289), within the chi^2 tolerance
    chi0 = float(r.stdout.split("initial chi2")[1])
    assert chi0 == pytest.approx(float(p0[-1]), rel=1e-11 if mode == "fast" else 1e-12)
    PS, P = 17, 16
    raw = np.fromfile(outp, "<f8")
    o = 0
    state = raw[o:o + W * PS].reshape(W, PS); o += W * PS
    tries = raw[o:o + W * P].reshape(W, P); o += W * P
    accepts = raw[o:o + W * P].reshape(W, P); o += W * P
    chain = raw[o:o + W * L * PS].reshape(W, L, PS)
    rtol = 1e-9 if mode == "fast" else 1e-10
    np.testing.assert_allclose(chain, g["traj_params"][:, :L], rtol=rtol)
    np.testing.assert_allclose(state, g["traj_params"][:, L - 1], rtol=rtol)
    for w in range(W):
        r_w = g["traj_r"][w, :L]
        a_w = g["traj_acc"][w, :L]
        assert np.array_equal(tries[w], np.bincount(r_w, minlength=P)), w
        assert np.array_equal(accepts[w], np.bincount(r_w[a_w], minlength=P)), w
