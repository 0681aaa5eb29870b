"""Host-side file surface (CPU): CSV / acceptance bytes vs the reference's own writer
output (golden *_csv written by apf_step2.py:355-365 under make_golden.py), FITS I/O vs
astropy-written files, path/guess/initial-vector logic, and the step-3 read contract."""
import os

import numpy as np
import pytest

from olpefit_amd import fitsio, pipeline, step3, synth
from oracle import olpe_oracle as ora

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["c32", "c64", "c64_3", "c128_3", "c32_nan", "c64_nan", "c64_3_nan", "c128_3_nan"]


def _rows_and_counters(g, w):
    """Reference file content after the last write (count = last multiple of 10)."""
    L = int(g["traj_len"][w])
    last = (L // 10) * 10
    burn = int(g["burn_in"])
    first = max(burn, 1)
    rows = g["traj_params"][w, first - 1:last]
    npar = rows.shape[1] - 1
    tries = np.zeros(npar)
    acc = np.zeros(npar)
    for i in range(last):
        r = g["traj_r"][w, i]
        tries[r] += 1
        acc[r] += g["traj_acc"][w, i]
    return rows, tries, acc


@pytest.mark.parametrize("name", CASES)
def test_chain_csv_bytes_match_reference_writer(golden, name):
    g = golden(name)
    rows, _, _ = _rows_and_counters(g, 0)
    text = pipeline.format_rows(pipeline.with_seed_row(rows))
    with open(os.path.join(GOLDEN, f"{name}_csv", "0_finalarray_mpi.csv"), newline="") as f:
        ref = f.read()
    assert text == ref


@pytest.mark.parametrize("name", CASES)
def test_acceptance_text_matches_reference(golden, name):
    g = golden(name)
    for w in range(len(g["seeds"])):
        _, tries, acc = _rows_and_counters(g, w)
        with open(os.path.join(GOLDEN, f"{name}_csv", f"{w}_acceptance_rate.csv")) as f:
            assert pipeline.acceptance_text(acc, tries) == f.read()


def test_written_rows_rule():
    assert pipeline.written_rows(847, 5) == 836          # rows for counts 5..840
    assert pipeline.written_rows(237, 0) == 230          # counts 1..230
    assert pipeline.written_rows(9, 0) == 0
    assert pipeline.written_rows(6000, 6000) == 1


def test_fits_reader_matches_astropy_files():
    exp = np.load(os.path.join(GOLDEN, "fits_expected.npz"))
    d, h = fitsio.getdata_header(os.path.join(GOLDEN, "astropy_f32.fits"))
    assert d.dtype == np.dtype(">f4") and np.array_equal(d, exp["f32"])
    assert h["itime"] == 1.0 and h["COADDS"] == 1 and h["sampmode"] == 2
    assert h["OBJECT"] == "synthetic"
    d, h = fitsio.getdata_header(os.path.join(GOLDEN, "astropy_u16.fits"))
    assert np.array_equal(d, exp["u16"]) and h["SAMPMODE"] == 3
    d, _ = fitsio.getdata_header(os.path.join(GOLDEN, "astropy_f64.fits"))
    assert np.array_equal(d, exp["f64"])


def test_fits_roundtrip(tmp_path):
    img, _ = synth.make_image(32, 2, 0)
    p = str(tmp_path / "x.fits")
    fitsio.write(p, img, synth.HEADER)
    d, h = fitsio.getdata_header(p)
    assert np.array_equal(d, img) and h["multisam"] == 1
    assert os.path.getsize(p) % 2880 == 0


def test_paths_and_guess(tmp_path):
    path = synth.write_case(str(tmp_path), 32, 2)
    directory, frame, out = pipeline.image_paths(path)
    assert frame == "00001" and out == directory + "00001_apf_results/"
    g = pipeline.read_guess(directory + "00001_initialguess")
    assert np.allclose(g, synth.guess_values(32, 2))


@pytest.mark.parametrize("name", CASES)
def test_initial_parameters_match_reference(golden, name):
    g = golden(name)
    p = pipeline.initial_parameters(g["image"], g["guess"], int(g["nsrc"]))
    assert np.array_equal(p[:-1], g["p_init"][:-1])
    assert np.array_equal(p, ora.initial_parameters(g["image"], g["guess"], int(g["nsrc"])))


def test_noise_model_matches_oracle(golden):
    from olpefit_amd.core import noise_model
    g = golden("c64")
    mask, pois2, rn2, sat, rn = noise_model(g["image"], 1.0, 1, 1, 2)
    assert np.array_equal(mask, g["mask"])
    err = np.sqrt(rn2 + pois2.astype(np.float64))
    assert np.array_equal(err, g["err"])


def test_gelman_rubin_equals_the_per_walker_loop():
    """step3.gelman_rubin reduces the transposed chains row by row; apf_step3.py:260-276
    loops over the walkers (np.mean / np.std of each column).  Same pairwise sums over
    the same values: the same bits, C- or Fortran-ordered input, odd shapes."""
    from olpefit_amd import step3

    def loop(p, d=16):
        N, M = float(p.shape[0]), float(p.shape[1])
        w, b = np.zeros(p.shape[1]), np.zeros(p.shape[1])
        om = np.mean(p)
        for i in range(p.shape[1]):
            w[i] = np.std(p[:, i]) ** 2
            b[i] = (np.mean(p[:, i]) - om) ** 2
        w = (1. / M) * np.sum(w)
        b = (N / (M - 1)) * np.sum(b)
        psrf = (((N - 1) / N) * w + ((M + 1) / (M * N)) * b) / w
        return psrf, np.sqrt(((d + 3) // (d + 1)) * psrf)
    rng = np.random.default_rng(11)
    for t in range(60):
        p = rng.normal(size=(int(rng.integers(2, 300)), int(rng.integers(2, 200))))
        p = p * rng.uniform(1e-3, 1e3) + rng.uniform(-1e4, 1e4)
        if t % 2:
            p = np.asfortranarray(p)
        assert step3.gelman_rubin(p) == loop(p)


def test_step3_reader_and_gelman_rubin(tmp_path, golden):
    """Write chains with the build's writer, read them back with the step-3 contract
    (equal lengths, NaN row dropped by additional_burnin=1) and compare GR with the
    hand-pinned fixture (tests/golden/make_gr_golden.py: exact rational arithmetic,
    Python-2 integer (d+3)/(d+1) == 1) for 17- and 20-column chains.  Tolerance rel
    1e-9: float64 cancellation in the variances against the exact values; the
    Python-3 factor sqrt(19/17) would be off by 5.7e-2."""
    g = golden("gr")
    for tag, nsrc, names in (("2", 2, step3.NAMES_2), ("3", 3, step3.NAMES_3)):
        chains = g[f"chains{tag}"]                    # [N, M, PS]
        N, M, ps = chains.shape
        d = tmp_path / tag
        d.mkdir()
        for w in range(M):
            pipeline.write_chain_csv(str(d / f"{w}_finalarray_mpi.csv"),
                                     pipeline.with_seed_row(chains[:, w, :]))
        c = step3.load_chains(str(d), M, additional_burnin=1)
        assert c.shape == (N, M, ps)
        assert np.array_equal(c, chains)              # repr round trip is exact
        for k in range(ps - 1):
            ps1, rc1 = step3.gelman_rubin(c[:, :, k])
            np.testing.assert_allclose(ps1, g[f"psrf{tag}"][k], rtol=1e-9)
            np.testing.assert_allclose(rc1, g[f"rc{tag}"][k], rtol=1e-9)
            assert rc1 == np.sqrt(ps1)                # factor (16+3)//(16+1) == 1
            ps2, rc2 = ora.gelman_rubin(c[:, :, k])
            assert ps1 == ps2 and rc1 == rc2
        s = step3.summary(c, nsrc=nsrc)
        assert list(s) == names[:-1]
        np.testing.assert_allclose([s[n]["gr_rc"] for n in names[:-1]], g[f"rc{tag}"],
                                   rtol=1e-9)
    # a float d divides as floats, as it would in the reference with d = 16.
    x = g["chains2"][:, :, 0]
    assert step3.gelman_rubin(x, d=16.0)[1] == np.sqrt((19 / 17) * step3.gelman_rubin(x)[0])
    # unequal lengths are an error, as in the reference's [length, ncor] assignment
    chains = g["chains2"]
    pipeline.write_chain_csv(str(tmp_path / "2" / "3_finalarray_mpi.csv"),
                             pipeline.with_seed_row(chains[:10, 3, :]))
    with pytest.raises(ValueError):
        step3.load_chains(str(tmp_path / "2"), 5)


def test_headless_step1_guess(tmp_path):
    from olpefit_amd import step1
    path = synth.write_case(str(tmp_path), 64, 2)
    img, _ = fitsio.getdata_header(path)
    p = synth.truth_params(64, 2)
    out = step1.main([str(tmp_path), "--star", str(p[0] + 2.3), str(p[1] - 1.7),
                      "--companion", str(p[2] + 1.1), str(p[3] + 0.4), "--sky", "3.7", "2.2"])
    assert out == [str(tmp_path) + "/00001_initialguess"]
    g = pipeline.read_guess(out[0])
    # apf_step1.py:145-152: 21x21 argmax around the truncated click, + 0.5 px
    ys, xs = np.unravel_index(np.argmax(img), img.shape)
    assert (g[0], g[1]) == (xs + 0.5, ys + 0.5)
    assert g[4] == 3 and g[5] == 2
    box = img[int(p[3] + 0.4) - 11:int(p[3] + 0.4) + 10, int(p[2] + 1.1) - 11:int(p[2] + 1.1) + 10]
    yc, xc = np.unravel_index(np.argmax(box), box.shape)
    assert g[2] == int(p[2] + 1.1) - 11 + xc + 0.5 and g[3] == int(p[3] + 0.4) - 11 + yc + 0.5
    text = open(out[0]).read()
    assert text.endswith("\n") and len(text.split()) == 6


def test_headless_step1_three_body(tmp_path):
    """3body/apf_step1_3body.py:165-197: 8x8 box image[y-4:y+4, x-4:x+4] around each
    truncated click, integer argmax position, file "xca yca xcb ycb xcc ycc bkgdx bkgdy"."""
    from olpefit_amd import step1
    path = synth.write_case(str(tmp_path), 64, 3)
    img, _ = fitsio.getdata_header(path)
    p = synth.truth_params(64, 3)
    clicks = [(p[0] + 1.6, p[1] - 0.8), (p[2] - 1.2, p[3] + 2.1), (p[4] + 0.3, p[5] + 0.9)]
    argv = [str(tmp_path), "--star", str(clicks[0][0]), str(clicks[0][1])]
    for c in clicks[1:]:
        argv += ["--companion", str(c[0]), str(c[1])]
    out = step1.main(argv + ["--sky", "5.9", "3.1"], three_body=True)
    text = open(out[0]).read()
    assert text.endswith("\n")
    vals = text.split()
    assert len(vals) == 8 and all(v.lstrip("-").isdigit() for v in vals)
    for k, (x, y) in enumerate(clicks):
        xm, ym = int(x), int(y)
        box = img[ym - 4:ym + 4, xm - 4:xm + 4]
        yc, xc = np.unravel_index(np.argmax(box), box.shape)
        assert (int(vals[2 * k]), int(vals[2 * k + 1])) == (xm - 4 + xc, ym - 4 + yc)
    assert vals[6:] == ["5", "3"]
    g = pipeline.read_guess(out[0])
    assert len(g) == 8
    with pytest.raises(SystemExit):      # two companions (B, C) required
        step1.main(argv[:7] + ["--sky", "5.9", "3.1"], three_body=True)


@pytest.mark.parametrize("sampmode", [2, 3, 1])
def test_noise_model_header_cases_equal_oracle(sampmode):
    """apf_step2.py:176-210 for the header values the reference branches on: sampmode 3
    (MCDS: saturation scaled by multisam / itime, readnoise 38 / sqrt(multisam)), 2
    (CDS) and any other; coadds and multisam > 1; float32 and float64 frames.  The
    product's mask and err equal the oracle's (masked_greater's mask; err bit for bit)."""
    from olpefit_amd import core, synth
    from oracle import olpe_oracle as ora
    img32, _ = synth.make_image(48, 2, 4)
    for img in (img32, img32.astype(np.float64) * 1.7):
        for coadds, multisam, itime in ((1, 1, 1.0), (5, 8, 0.25), (10, 16, 30.0), (2, 2, 0.05)):
            mask, pois2, rn2, sat, rn = core.noise_model(img, itime, coadds, multisam, sampmode)
            dm, err, sat_o, rn_o = ora.noise_model(img, itime, coadds, multisam, sampmode)
            assert sat == sat_o and rn == rn_o
            np.testing.assert_array_equal(mask, np.ma.getmaskarray(dm))
            got = np.sqrt(rn2 + pois2.astype(np.float64))
            assert np.array_equal(got, err)


def test_native_acceptance_files_equal_numpy_str(tmp_path):
    """olpe_acceptance_write / _format (host-only) print accepts / tries as str() of the
    float64 array does (apf_step2.py:362-365): fixed notation with NumPy's 8-digit
    'maxprec' cut (dyadic ties included), padding and 75-column wrapping; rows NumPy
    prints in scientific notation or with NaN fall back to str().  Bytes compared over
    random rows of 1-40 values and a walker set mixing both kinds."""
    import ctypes as C
    from olpefit_amd import _lib
    lib = _lib.load()

    def native(x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        n = C.c_size_t(0)
        _lib.check(lib.olpe_acceptance_format(x.ctypes.data_as(_lib._pd), x.size, None, 0,
                                              C.byref(n)))
        if n.value == 0:
            return None
        buf = C.create_string_buffer(n.value)
        _lib.check(lib.olpe_acceptance_format(x.ctypes.data_as(_lib._pd), x.size, buf, n.value,
                                              C.byref(n)))
        return buf.raw[:n.value].decode()
    rng = np.random.default_rng(7)
    native_rows = 0
    for t in range(3000):
        p = int(rng.choice([1, 3, 16, 19, 40]))
        k = t % 6
        if k == 0:
            tries = rng.integers(1, 200000, p).astype(float)
            x = np.floor(tries * rng.random(p)) / tries
        elif k == 1:
            tries = rng.integers(1, 50, p).astype(float)
            x = np.floor(tries * rng.random(p)) / tries
        elif k == 2:
            x = rng.integers(0, 513, p) / 512.0                # ties at the 9th digit
        elif k == 3:
            x = rng.random(p) * rng.choice([1, 10, 100, 1000])
        elif k == 4:
            x = np.round(rng.random(p), int(rng.integers(1, 10)))
        else:
            x = rng.random(p)
            x[rng.random(p) < 0.3] = 0.0
            x[rng.random(p) < 0.1] = 1.0
        got = native(x)
        if got is not None:
            native_rows += 1
            assert got == str(x), (x, got)
    assert native_rows > 2500
    assert native(np.array([0.5, 5e-5])) is None and native(np.array([0.5, np.nan])) is None
    # the writer: native rows and fallbacks give the files write_acceptance gives
    W, P = 64, 16
    tries = rng.integers(1, 100000, (W, P)).astype(float)
    acc = np.floor(tries * rng.random((W, P)))
    tries[3, 5] = acc[3, 5] = 0.0                             # NaN: fallback
    acc[7] = tries[7] * 0.5
    acc[7, 2] = tries[7, 2] * 1e-5                            # scientific: fallback
    a = [str(tmp_path / f"a{w}") for w in range(W)]
    b = [str(tmp_path / f"b{w}") for w in range(W)]
    pipeline.write_acceptance_files(a, acc, tries, threads=4)
    for w in range(W):
        pipeline.write_acceptance(b[w], acc[w], tries[w])
        assert open(a[w], "rb").read() == open(b[w], "rb").read(), w
    # written to a temporary name and renamed over the file (a kill mid-write
    # leaves the previous file): rewriting replaces every file whole, no .tmp is left
    old = {w: open(a[w], "rb").read() for w in range(W)}
    pipeline.write_acceptance_files(a, acc + 1, tries + 2, threads=4)
    assert not list(tmp_path.glob("*.tmp"))
    assert all(open(a[w], "rb").read() != old[w] for w in range(W) if w != 3)
    # a failed rename (the target is a directory) leaves no '<path>.tmp' either, native
    # or Python
    from olpefit_amd._lib import OlpeError
    d = tmp_path / "dir_target"
    d.mkdir()
    with pytest.raises(OlpeError):
        pipeline.write_acceptance_files([str(d)], acc[:1], tries[:1], threads=1)
    with pytest.raises(OSError):
        pipeline.write_acceptance(str(d), acc[0], tries[0])
    assert not list(tmp_path.glob("*.tmp")) and d.is_dir()


def test_native_csv_formatter_equals_repr():
    """olpe_csv_format (host-only, no GPU) writes what csv.writer writes for float rows
    (repr of each value): edge values, random magnitudes over 10^+-30, integers, and
    random bit patterns (subnormals, huge exponents, NaN payloads)."""
    rs = np.random.RandomState(0)
    edge = [0.0, -0.0, 1e-5, 1e-4, 1.5e-7, 1e16, 1e15, 1234567890123456.0,
            12345678901234567.0, np.nan, -np.nan, np.inf, -np.inf, 5e-324,
            1.7976931348623157e308, 0.1, 1 / 3, 100.0, -2.5, 1e22, 1e-300,
            9.999999999999999e-5, 0.00010000000000000002]
    x = np.concatenate([edge, rs.normal(size=30000) * 10.0 ** rs.randint(-30, 30, size=30000),
                        rs.randint(-10 ** 6, 10 ** 6, size=3000).astype(float),
                        rs.randint(0, 2 ** 63, size=30000, dtype=np.int64).view(np.float64)])
    x = x[:len(x) // 7 * 7].reshape(-1, 7)
    ref = "".join(",".join(repr(v) for v in row) + "\r\n" for row in x.tolist())
    assert pipeline.format_rows(x) == ref
    assert pipeline.format_rows(x[:3], nan_row=True) == "nan,nan,nan,nan,nan,nan,nan\r\n" + \
        "".join(",".join(repr(v) for v in row) + "\r\n" for row in x[:3].tolist())


def test_native_chain_writer_threads(tmp_path):
    """olpe_csv_write_chains: one file per walker from writer threads, bytes equal to
    the single-file formatter with the NaN seed row; an unwritable path is OLPE_EIO."""
    from olpefit_amd._lib import OlpeError
    rs = np.random.RandomState(5)
    chains = rs.normal(size=(37, 21, 17)) * 1e3
    paths = [str(tmp_path / f"{w}_finalarray_mpi.csv") for w in range(37)]
    pipeline.write_chain_csvs(paths, chains, threads=8)
    for w in (0, 17, 36):
        with open(paths[w], newline="") as f:
            assert f.read() == pipeline.format_rows(pipeline.with_seed_row(chains[w]))
    with pytest.raises(OlpeError):
        pipeline.write_chain_csvs([str(tmp_path / "no_dir" / "x.csv")], chains[:1])


def test_mpiexec_launch_like_the_reference(tmp_path, monkeypatch):
    """``mpiexec -n W python apf_step2.py <image>`` (the reference's launch, one walker per
    rank): --walkers defaults to W, and every rank but 0 leaves before touching the image
    or the GPU (rank 0 runs all W walkers; its run is the GPU CLI tests' path)."""
    from olpefit_amd import step2
    for k in [k for pair in step2.MPI_ENV for k in pair]:
        monkeypatch.delenv(k, raising=False)
    assert step2.mpi_world() == (0, 1)
    assert step2.parse(["a/N2.x.fits"], 2).walkers == 24
    for rk, sz in step2.MPI_ENV:
        assert step2.mpi_world({rk: "3", sz: "48"}) == (3, 48)
    assert step2.mpi_world({"PMI_RANK": "5", "PMI_SIZE": "4"}) == (0, 1)      # inconsistent
    monkeypatch.setenv("OMPI_COMM_WORLD_RANK", "2")
    monkeypatch.setenv("OMPI_COMM_WORLD_SIZE", "48")
    args = step2.parse(["a/N2.x.fits"], 3)
    assert (args.walkers, args.mpi_rank, args.mpi_size) == (48, 2, 48)
    assert step2.parse(["a/N2.x.fits", "--walkers", "7"], 2).walkers == 7
    assert step2.parse(["a/N2.x.fits"], 2, variant="2a").walkers == 1     # 2a: one walker
    image = str(tmp_path / "N2.20090531.29966.LDIF.fits")                  # never opened
    out = step2.main([image, "-q"], nsrc=2)
    assert out == str(tmp_path) + "/29966_apf_results/" and not os.path.exists(out)


def test_native_chain_reader_equals_genfromtxt(tmp_path):
    """step3.load_chains parses the chain files natively (olpe_csv_read_chains); the
    values are np.genfromtxt's (the reference's reader, apf_step3.py:169-186) bit for
    bit, including repr edge values, NaN / inf, subnormals and -0.0."""
    rs = np.random.RandomState(3)
    M, N, ps = 7, 45, 17
    chains = rs.normal(size=(M, N, ps)) * 10.0 ** rs.randint(-320, 300, size=(M, N, ps))
    chains[0, 3, :6] = [np.nan, np.inf, -np.inf, -0.0, 5e-324, 1e16]
    chains[2, 7, :4] = [0.1 + 0.2, 1e-5, 123456789012345678.0, -2.2250738585072014e-308]
    paths = [str(tmp_path / f"{w}_finalarray_mpi.csv") for w in range(M)]
    pipeline.write_chain_csvs(paths, chains, nan_row=True)
    for burn in (0, 1, 5):
        got = step3.load_chains(str(tmp_path), M, additional_burnin=burn)
        ref = np.stack([np.genfromtxt(p, delimiter=",") for p in paths], axis=1)[burn:]
        assert got.shape == ref.shape == (N + 1 - burn, M, ps)
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))   # bit for bit
    for threads in (1, 3):
        assert np.array_equal(step3.load_chains(str(tmp_path), M, threads=threads)[:, :, 1:],
                              chains.transpose(1, 0, 2)[:, :, 1:])
    # blank fields are missing values (NaN) and blank lines are skipped, as genfromtxt
    with open(paths[1], "ab") as f:
        f.write(b"\r\n")
    with open(paths[4], "r+b") as f:
        text = f.read().replace(b",", b", ", 3)
        f.seek(0)
        f.write(text)
    got = step3.load_chains(str(tmp_path), M, additional_burnin=0)
    ref = np.stack([np.genfromtxt(p, delimiter=",") for p in paths], axis=1)
    assert np.array_equal(got, ref, equal_nan=True)
    # shape errors name the file; garbage is an error, not a silent NaN
    pipeline.write_chain_csv(paths[5], pipeline.with_seed_row(chains[5, :10]))
    with pytest.raises(ValueError, match="5_finalarray_mpi.csv"):
        step3.load_chains(str(tmp_path), M)
    pipeline.write_chain_csvs(paths[5:6], chains[5:6], nan_row=True)
    with open(paths[6], "r+b") as f:
        f.seek(40)
        f.write(b"x")
    with pytest.raises(ValueError, match="not a number"):
        step3.load_chains(str(tmp_path), M)


def test_npy_sidecar_loader(tmp_path):
    """load_chains(source="npy") reads the --npy sidecars (no NaN seed row: it counts as
    the first additional_burnin row) to the same array as the CSV path."""
    rs = np.random.RandomState(4)
    M, N = 3, 20
    chains = rs.normal(size=(M, N, 17))
    paths = [str(tmp_path / f"{w}_finalarray_mpi.csv") for w in range(M)]
    pipeline.write_chain_csvs(paths, chains, nan_row=True)
    pipeline.append_npy_chains([str(tmp_path / f"{w}_chain.npy") for w in range(M)], chains, N, 0)
    for burn in (0, 1, 4, N + 1):
        assert np.array_equal(step3.load_chains(str(tmp_path), M, burn, source="npy"),
                              step3.load_chains(str(tmp_path), M, burn), equal_nan=True)


def _moments_vector(chains, centre=None):
    """The olpe_moments_summary layout from chains [N, M, PS] on the host (two-pass)."""
    N, M, ps = chains.shape
    mean = chains.mean(axis=0)                                  # [M, PS]
    m2 = ((chains - mean) ** 2).sum(axis=0)
    c = mean.mean(axis=0) if centre is None else centre
    out = np.zeros(5 * ps)
    out[0], out[1] = N, M
    out[2:2 + ps] = mean.sum(axis=0)
    out[2 + ps:2 + 2 * ps] = m2.sum(axis=0)
    out[2 + 2 * ps:2 + 3 * ps] = ((mean - c) ** 2).sum(axis=0)
    out[2 + 3 * ps:2 + 4 * ps - 1] = 10.0
    out[2 + 4 * ps - 1:] = 4.0
    return out


@pytest.mark.parametrize("nsrc", [2, 3])
def test_summary_from_moments_equals_summary(golden, nsrc):
    """The moment form of step 3's statistics (mean, std, GR PSRF / RC) equals
    step3.summary over the chains (the reference's arithmetic, apf_step3.py:258-278) on
    the hand-pinned GR fixture's chains.  Those are built to stress cancellation (a
    column of mean -148.9 whose walkers' means differ by 1e-2): there both forms sit
    within 1.2e-12 / 3.8e-12 of the fixture's exact rational PSRF, so the test asks
    5e-12 of each against the exact values and of the two forms against each other
    (1e-12 on real chains: tests/test_cli_gpu.py)."""
    g = golden("gr")
    tag = "2" if nsrc == 2 else "3"
    chains = g["chains" + tag]
    ref = step3.summary(chains, nsrc=nsrc)
    got = step3.summary_from_moments(_moments_vector(chains), nsrc=nsrc)
    for k, (name, r) in enumerate(ref.items()):
        for key in ("mean", "std", "gr_psrf", "gr_rc"):
            np.testing.assert_allclose(got[name][key], r[key], rtol=5e-12, err_msg=(name, key))
        np.testing.assert_allclose(got[name]["gr_psrf"], g["psrf" + tag][k], rtol=5e-12)
        np.testing.assert_allclose(got[name]["gr_rc"], g["rc" + tag][k], rtol=5e-12)
        assert got[name]["acceptance"] == 0.4
    # several contexts (step 2's --gpus shards) combine to the same vector
    parts = [_moments_vector(chains[:, :2]), _moments_vector(chains[:, 2:])]
    for p in parts:
        p[2 + 2 * chains.shape[2]:2 + 3 * chains.shape[2]] = 0
    centre = step3.pooled_mean(parts)
    dev = [_moments_vector(chains[:, :2], centre), _moments_vector(chains[:, 2:], centre)]
    comb = step3.combine_moments(parts, dev)
    np.testing.assert_allclose(comb[2:], _moments_vector(chains)[2:] * np.r_[
        np.ones(3 * chains.shape[2]), 2 * np.ones(2 * chains.shape[2] - 2)], rtol=1e-12)


def test_step3_cli_reads_step2_output(tmp_path, golden, capsys):
    """apf_step3.py's front end (arguments image, system, -s, -a; apf_step3.py:64-84): it
    reads the step-2 files of <frame>_apf_results/ (native loader), slices the burn-in
    and prints the reference's Gelman-Rubin lines (:258-278); the statistics equal
    step3.summary of the same chains, from the CSV files, the .npy sidecars or step 2's
    posterior_summary.json."""
    import json
    g = golden("gr")
    chains = g["chains2"]                                   # [N, M, 17]
    N, M, ps = chains.shape
    image = str(tmp_path / "N2.20250127.00042.LDIF.fits")
    outdir = pipeline.image_paths(image)[2]
    os.makedirs(outdir)
    paths = [outdir + f"{w}_finalarray_mpi.csv" for w in range(M)]
    pipeline.write_chain_csvs(paths, chains.transpose(1, 0, 2), nan_row=True)
    pipeline.append_npy_chains([outdir + f"{w}_chain.npy" for w in range(M)],
                               chains.transpose(1, 0, 2), N, 0)
    ref = step3.summary(chains[2:], nsrc=2)                 # -a 3: the NaN row + 2 rows
    out = step3.main([image, "HIP 1234", "-s", str(M), "-a", "3"])
    text = capsys.readouterr().out
    assert "Mean and stdev Gelman-Rubin stat for parameter chains:" in text
    assert "Number of jumps after additional burn in: %d" % (N + 1 - 3) in text
    for k, r in ref.items():
        for key in ("mean", "median", "std", "gr_rc"):
            assert out["parameters"][k][key] == r[key], (k, key)
    assert json.load(open(outdir + "step3_summary.json"))["rows_per_walker"] == N - 2
    npy = step3.main([image, "x", "-s", str(M), "-a", "3", "--npy", "-q"])
    assert npy["parameters"] == out["parameters"]
    # --from-moments: step 2's device-moment summary (here from host moments)
    m = _moments_vector(chains)
    with open(outdir + "posterior_summary.json", "w") as f:
        json.dump(step3.summary_from_moments(m, 2), f)
    mom = step3.main([image, "x", "-s", str(M), "--from-moments", "-q"])
    full = step3.summary(chains, nsrc=2)
    for k, r in full.items():
        np.testing.assert_allclose(mom["parameters"][k]["gr_rc"], r["gr_rc"], rtol=5e-12)
    with pytest.raises(ValueError):
        step3.main([image, "x", "-s", str(M + 1), "--from-moments", "-q"])
    # the moments cover every recorded row (additional_burnin 1): a larger -a cannot be
    # applied to them and is refused instead of being reported as applied
    with pytest.raises(SystemExit) as ei:
        step3.main([image, "x", "-s", str(M), "--from-moments", "-a", "3", "-q"])
    assert ei.value.code == 2
    assert step3.main([image, "x", "-s", str(M), "--from-moments", "-a", "1", "-q"])[
        "additional_burnin"] == 1
    # a step-2 run shorter than its burn-in leaves only the NaN seed row: a clear error
    pipeline.write_chain_csvs(paths, np.zeros((M, 0, ps)), nan_row=True)
    with pytest.raises(ValueError, match="none left"):
        step3.main([image, "x", "-s", str(M), "-q"])
