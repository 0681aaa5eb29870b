"""Pin the oracle: NumPy restatement vs fixtures produced by the reference's own code
(tests/golden/make_golden.py executed apf_step2.py / apf_step2_3body.py line ranges
with astropy 4.3.1).  CPU only.

Tolerances (fp64): model pixels rel 1e-13 of the image peak (transcendental ulps of
NumPy's SIMD exp/sin/cos between NumPy builds), chi^2 rel 1e-12, trajectories: the
proposed index and the accept decision must be identical at every iteration, proposal
values / chi^2 / parameters rel 1e-12.
"""
import numpy as np
import pytest

from oracle import olpe_oracle as ora
from oracle.legacy_rng import LegacyMT

# *_nan: the c32 / c64 cutouts with NaN, -inf and +inf data pixels (make_golden.py
# ``nonfinite``): the reference's np.ma chi_squared drops them (apf_step2.py:134-137)
CASES = ["c32", "c64", "c64_3", "c128_3", "c32_nan", "c64_nan", "c64_3_nan", "c128_3_nan"]


def test_rng_numpy_stream_frozen(golden):
    g = golden("rng")
    for i, s in enumerate(g["seeds"]):
        rs = np.random.RandomState(int(s))
        assert np.array_equal(rs.randint(0, 2 ** 32, size=1500, dtype=np.uint64), g["raw"][i])
        assert np.array_equal(np.random.RandomState(int(s)).standard_normal(400), g["gauss"][i])
        assert np.array_equal(np.random.RandomState(int(s)).rand(400), g["unif"][i])


def test_rng_restatement_matches_golden(golden):
    """Appendix-B restatement (what the HIP kernel implements) is bit-exact."""
    g = golden("rng")
    for i, s in enumerate(g["seeds"]):
        mt = LegacyMT(int(s))
        assert [mt.next_u32() for _ in range(1500)] == [int(v) for v in g["raw"][i]]
        mt = LegacyMT(int(s))
        assert np.array_equal([mt.gauss() for _ in range(400)], g["gauss"][i])
        mt = LegacyMT(int(s))
        assert np.array_equal([mt.rand() for _ in range(400)], g["unif"][i])
        mt = LegacyMT(int(s))
        assert [mt.randint(16) for _ in range(400)] == list(g["randint16"][i])
        mt = LegacyMT(int(s))
        assert [mt.randint(19) for _ in range(400)] == list(g["randint19"][i])


def test_first_outputs_known_answers():
    # first outputs for seeds 0, 1, 5489, 12345, 2**32-1
    want = {0: 2357136044, 1: 1791095845, 5489: 3499211612, 12345: 3992670690,
            2 ** 32 - 1: 419326371}
    for s, v in want.items():
        assert LegacyMT(s).next_u32() == v


@pytest.mark.parametrize("name", CASES)
def test_noise_model_and_init(golden, name):
    g = golden(name)
    img = g["image"]
    nsrc = int(g["nsrc"])
    dm, err, sat, rn = ora.noise_model(img, 1.0, 1, 1, 2)
    assert np.array_equal(np.ma.getmaskarray(dm), g["mask"])
    assert np.array_equal(err, g["err"], equal_nan=True)
    assert sat == g["satlevel"] and rn == g["readnoise"]
    p0 = ora.initial_parameters(img, g["guess"], nsrc)
    assert np.array_equal(p0[:-1], g["p_init"][:-1])
    with np.errstate(all="ignore"):
        chi = ora.chi_squared(dm, ora.build_analytical_model(p0, img.shape[0], nsrc), err)
    np.testing.assert_allclose(float(chi), g["p_init"][-1], rtol=1e-12)


@pytest.mark.parametrize("name", CASES)
def test_model_and_chi2(golden, name):
    g = golden(name)
    img = g["image"]
    n = img.shape[0]
    nsrc = int(g["nsrc"])
    dm, err, _, _ = ora.noise_model(img, 1.0, 1, 1, 2)
    for k, p in enumerate(g["params"]):
        with np.errstate(all="ignore"):
            m = ora.build_analytical_model(p, n, nsrc)
            c = ora.chi_squared(dm, m, err)
        ref = g["models"][k]
        scale = np.max(np.abs(ref))
        assert np.max(np.abs(m - ref)) <= 1e-13 * scale, (name, k)
        np.testing.assert_allclose(float(c), g["chi2"][k], rtol=1e-12)


@pytest.mark.parametrize("name", CASES)
def test_trajectories(golden, name):
    g = golden(name)
    img = g["image"]
    nsrc = int(g["nsrc"])
    dm, err, _, _ = ora.noise_model(img, 1.0, 1, 1, 2)
    for w, seed in enumerate(g["seeds"]):
        L = int(g["traj_len"][w])
        walker = ora.Walker(dm, err, g["p_init"], int(seed), nsrc)
        for i in range(L):
            r, new, chi, dice, acc = walker.step()
            assert r == g["traj_r"][w, i], (name, w, i)
            assert acc == g["traj_acc"][w, i], (name, w, i)
            assert dice == g["traj_dice"][w, i]
            np.testing.assert_allclose(new, g["traj_new"][w, i], rtol=1e-12)
            np.testing.assert_allclose(chi, g["traj_chi"][w, i], rtol=1e-12)
            np.testing.assert_allclose(walker.parameters, g["traj_params"][w, i], rtol=1e-12)


@pytest.mark.parametrize("name", ["c32_nan", "c64_nan"])
def test_nonfinite_pixels_drop_out(golden, name):
    """The fixture's chi^2 values are finite and equal the sum over the pixels that are
    neither saturation-masked nor non-finite in D or err -- the mask the product stages
    (core.noise_model + olpe_create)."""
    from olpefit_amd.core import noise_model
    g = golden(name)
    img = g["image"]
    n = img.shape[0]
    assert not np.all(np.isfinite(img))
    mask, pois2, rn2, _, _ = noise_model(img, 1.0, 1, 1, 2)
    err = np.sqrt(rn2 + pois2.astype(np.float64))
    assert np.array_equal(mask, g["mask"] | ~np.isfinite(img) | ~np.isfinite(err))
    keep = ~mask
    for k, p in enumerate(g["params"][:6]):
        m = ora.build_analytical_model(p, n, 2)
        chi = np.sum(((img.astype(np.float64)[keep] - m[keep]) / err[keep]) ** 2)
        assert np.isfinite(g["chi2"][k])
        np.testing.assert_allclose(chi, g["chi2"][k], rtol=1e-12)


@pytest.mark.parametrize("name,walker", [("c64_long", 3), ("c128_3_long", 1),
                                         ("c32_long", 1), ("c64_3_long", 0)])
def test_oracle_long_chain_matches_reference(golden, name, walker):
    """The round-4 long fixtures (make_golden.py ``long``: the reference's own loop to
    accept_min 340 / 90): one walker's whole chain (5,775 / 1,945 iterations) from the
    oracle equals the reference's row for row."""
    g = golden(name)
    nsrc = int(g["nsrc"])
    dm, err, _, _ = ora.noise_model(g["image"], 1.0, 1, 1, 2)
    L = int(g["traj_len"][walker])
    w = ora.Walker(dm, err, g["p_init"], int(g["seeds"][walker]), nsrc)
    chain, _ = w.run(L)
    np.testing.assert_allclose(chain, g["traj_params"][walker, :L], rtol=1e-12, atol=0)


@pytest.mark.parametrize("name,walker,iters", [("c64_long", 2, 800), ("c128_3_long", 0, 250),
                                               ("c32_long", 1, 600)])
def test_astropy_oracle_is_the_reference(name, walker, iters):
    """oracle/astropy_timing.py (bench.py's reference-cost CPU baseline): the oracle's
    walker with astropy Gaussian2D objects per proposal, under the image's python3.9 /
    numpy 1.26 / astropy 4.3.1, gives the reference's own chains BIT FOR BIT (the long
    fixtures were written by the reference's lines under the same interpreter)."""
    import json
    import os
    import subprocess
    py = "/opt/conda/bin/python3.9"
    if not os.path.exists(py):
        pytest.skip("no /opt/conda python3.9")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([py, os.path.join(repo, "oracle", "astropy_timing.py"), "--check",
                        os.path.join(repo, "tests", "golden", f"{name}.npz"), str(walker),
                        str(iters)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["rows"] == iters and d["bit_equal"] is True


def test_oracle_posterior_run_matches_reference(golden):
    """Round 5's posterior fixture (make_golden.py ``posterior``: the reference's own
    loop, ~20,000 iterations per walker, stored as every 50th row, every draw and accept
    decision, and each walker's whole-chain mean / M2): walker 0 of the 64x64 case from
    the oracle -- every draw and decision, the stored rows and the walker's moments."""
    g = golden("c64_post")
    nsrc = int(g["nsrc"])
    L, every = int(g["L"]), int(g["every"])
    dm, err, _, _ = ora.noise_model(g["image"], 1.0, 1, 1, 2)
    w = ora.Walker(dm, err, g["p_init"], int(g["seeds"][0]), nsrc)
    chain, tr = w.run(L, trace=True)
    assert np.array_equal(np.array([t[0] for t in tr], np.uint8), g["draws"][0])
    assert np.array_equal(np.packbits(np.array([t[4] for t in tr], bool)), g["acc_bits"][0])
    np.testing.assert_allclose(chain[every - 1::every], g["rows_sub"][0], rtol=1e-12, atol=0)
    np.testing.assert_allclose(chain.mean(axis=0), g["mean"][0], rtol=1e-13)
    np.testing.assert_allclose(((chain - chain.mean(axis=0)) ** 2).sum(axis=0), g["m2"][0],
                               rtol=1e-8)
