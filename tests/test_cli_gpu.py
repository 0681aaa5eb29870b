"""End-to-end apf_step2 CLI on the GPU: synthetic FITS + step-1 guess -> chain files,
compared with the chain files the reference's own loop wrote (tests/golden/*_csv) for
the same image, guess, seed and accept_min; then read back through the step-3 contract.

Values: rel 1e-10 (exact eval) / 1e-9 (fast eval); acceptance-rate text: identical
(it depends only on the accept decisions)."""
import os

import numpy as np
import pytest

from olpefit_amd import pipeline, step2, step3, synth

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name,nsrc,mode", [("c64", 2, "exact"), ("c64", 2, "fast"),
                                            ("c64_3", 3, "exact")])
def test_cli_matches_reference_chain_files(tmp_path, golden, name, nsrc, mode):
    g = golden(name)
    n = g["image"].shape[0]
    path = synth.write_case(str(tmp_path), n, nsrc)
    argv = [path, "--walkers", "1", "--seed", "1000", "--accept-min", str(int(g["accept_min"])),
            "--burn-in", str(int(g["burn_in"])), "--chunk", "130", "-q"]
    if mode == "exact":
        argv.append("--exact")
    out = step2.main(argv, nsrc=nsrc)
    got = np.genfromtxt(out + "0_finalarray_mpi.csv", delimiter=",")
    ref = np.genfromtxt(os.path.join(GOLDEN, f"{name}_csv", "0_finalarray_mpi.csv"), delimiter=",")
    assert got.shape == ref.shape
    assert np.all(np.isnan(got[0]))
    np.testing.assert_allclose(got[1:], ref[1:], rtol=1e-10 if mode == "exact" else 1e-9)
    with open(out + "0_acceptance_rate.csv") as f, \
            open(os.path.join(GOLDEN, f"{name}_csv", "0_acceptance_rate.csv")) as h:
        assert f.read() == h.read()


def test_cli_multi_walker_files_feed_step3(tmp_path):
    path = synth.write_case(str(tmp_path), 32, 2)
    out = step2.main([path, "--walkers", "6", "--seed", "7", "--iters", "400", "--burn-in", "100",
                      "--gpus", "1", "-q"])
    c = step3.load_chains(out, 6, additional_burnin=1)
    assert c.shape == (301, 6, 17)                     # counts 100..400
    assert np.all(np.isfinite(c))
    s = step3.summary(c)
    assert abs(s["xcs"]["mean"] - synth.truth_params(32)[0]) < 0.5


def test_cli_seeds_are_gpu_count_independent(tmp_path):
    """Seeds come from the global walker index, so a sharded run (two contexts on the
    same GPU here) writes the same chains as a single-context run."""
    path = synth.write_case(str(tmp_path / "a"), 32, 2)
    out = step2.main([path, "--walkers", "5", "--seed", "11", "--iters", "200", "--burn-in", "0",
                      "-q", "--no-csv", "--npy"])
    one = [np.load(out + f"{w}_chain.npy") for w in range(5)]
    path2 = synth.write_case(str(tmp_path / "b"), 32, 2)
    from olpefit_amd.core import Sampler  # noqa: F401
    import olpefit_amd.step2 as s2
    args = [path2, "--walkers", "5", "--seed", "11", "--iters", "200", "--burn-in", "0", "-q",
            "--no-csv", "--npy", "--gpus", "2"]
    orig = s2.Shard.__init__

    def same_device(self, img, hdr, nsrc, device, *a, **k):     # 2 shards, 1 physical GPU
        orig(self, img, hdr, nsrc, 0, *a, **k)
    s2.Shard.__init__ = same_device
    try:
        out2 = s2.main(args)
    finally:
        s2.Shard.__init__ = orig
    for w in range(5):
        np.testing.assert_array_equal(np.load(out2 + f"{w}_chain.npy"), one[w])


def test_step2a_then_step2_from_2a(tmp_path):
    """apf_step2a writes step2a.csv (one walker, 5000 steps by default; 300 here);
    apf_step2 -i 2a starts every walker from its last row (apf_step2.py:248-256)."""
    path = synth.write_case(str(tmp_path), 32, 2)
    out = step2.main([path, "--iters", "300", "--seed", "5", "-q"], nsrc=2, variant="2a")
    a = np.genfromtxt(out + "step2a.csv", delimiter=",")
    assert a.shape == (301, 17) and np.all(np.isnan(a[0]))
    assert os.path.exists(out + "step2a_acceptance_rate")
    out2 = step2.main([path, "-i", "2a", "--walkers", "3", "--iters", "20", "--burn-in", "0",
                       "--seed", "9", "-q", "--no-csv", "--npy"])
    c0 = np.load(out2 + "0_chain.npy")
    # the first row differs from step2a's last row in at most one parameter + chi^2
    diff = np.nonzero(c0[0, :16] != a[-1, :16])[0]
    assert diff.size <= 1
