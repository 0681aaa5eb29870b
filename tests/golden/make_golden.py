"""Generate the golden fixtures that pin the oracle (run ONCE, in the survey container).

    /opt/conda/bin/python3.9 tests/golden/make_golden.py

Needs astropy 4.3.1 (conda py3.9) and read access to the reference checkout at
/root/reference.  The reference scripts are Python 2 and cannot be imported whole
(SURVEY.md §8(c)), but the line ranges executed here are valid Python 3: the
reference's OWN function definitions (apf_step2.py:63-148 / 3body:63-141), its setup
statements (noise model, initial guess, initial chi^2) and its sampler loop
(apf_step2.py:298-338 / 3body:324-373) run unmodified in a namespace that provides
``np``, ``models`` (astropy 4.3.1), the image/header, the step-1 guess and a stand-in
MPI communicator whose ``barrier()`` (called once per iteration at apf_step2.py:338)
snapshots the loop state.  The chain/CSV writer lines (apf_step2.py:346-351, :355-365)
run the same way, so the CSV fixtures are the bytes the reference writes.

Only data leaves this script: inputs and outputs in ``*.npz`` / ``*.csv`` / ``*.fits``
(no reference source text is stored).
"""
import io
import os
import sys
import tempfile
import textwrap

import numpy as np

# astropy 4.3.1 needs NumPy names removed in NumPy >= 1.25
for _name, _val in (("asscalar", lambda a: a.item()), ("alen", len),
                    ("product", np.prod), ("cumproduct", np.cumprod),
                    ("sometrue", np.any), ("alltrue", np.all)):
    if not hasattr(np, _name):
        setattr(np, _name, _val)

from astropy.modeling import models  # noqa: E402
from astropy.io import fits  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from olpefit_amd import synth, fitsio  # noqa: E402

REF = "/root/reference"


def lines(path, a, b):
    """Source text of lines a..b (1-based, inclusive), dedented."""
    with open(os.path.join(REF, path)) as f:
        src = f.read().split("\n")
    return textwrap.dedent("\n".join(src[a - 1:b]))


def compile_ranges(path, ranges):
    return [compile(lines(path, a, b), f"{path}:{a}-{b}", "exec") for a, b in ranges]


TWO = dict(
    path="apf_step2.py",
    funcs=(63, 148),
    setup=[(176, 188), (197, 210), (215, 217), (234, 237), (242, 245), (265, 273),
           (276, 276), (283, 285), (289, 289)],
    loop=(298, 338),
    stack=(346, 351),
    write=(355, 365),
)
THREE = dict(
    path="3body/apf_step2_3body.py",
    funcs=(63, 141),
    setup=[(167, 179), (188, 201), (220, 241), (246, 249), (255, 265), (292, 295),
           (298, 298), (307, 309), (313, 313)],
    loop=(324, 373),
    stack=(381, 386),
    write=(390, 400),
)


class _Comm:
    def __init__(self, cb):
        self.cb = cb

    def barrier(self):
        self.cb()


def reference_namespace(spec, image, header, guess):
    ns = {"np": np, "models": models, "image": image, "imhdr": header,
          "guess": np.array(guess), "rank": 0, "csv": __import__("csv")}
    for code in compile_ranges(spec["path"], [spec["funcs"]]):
        exec(code, ns)
    with np.errstate(all="ignore"):
        for code in compile_ranges(spec["path"], spec["setup"]):
            exec(code, ns)
    return ns


def run_reference_loop(spec, image, header, guess, seed, accept_min, burn_in, outdir,
                       rank):
    """Execute the reference loop for one walker (np.random.seed(seed)).  Returns the
    per-iteration trace and the initial parameter vector."""
    ns = reference_namespace(spec, image, header, guess)
    p_init = ns["parameters"].copy()
    n = len(p_init)
    ns.update(accept_min=accept_min, burn_in=burn_in, rank=rank,
              output_directory=outdir + "/",
              total_parameters=[[np.nan] for _ in range(n)])
    stack, write = compile_ranges(spec["path"], [spec["stack"], spec["write"]])
    trace = []

    def on_barrier():
        acc = ns["accept"] == "yes"
        chi = ns["chi_proposal"]
        chi = np.nan if chi is np.ma.masked else float(chi)
        trace.append((int(ns["rand"]), float(ns["new"]), chi, float(ns["dice"]), acc,
                      ns["parameters"].copy()))
        if ns["count"] >= ns["burn_in"]:
            exec(stack, ns)
            exec(write, ns)

    ns["comm"] = _Comm(on_barrier)
    np.random.seed(seed)
    loop, = compile_ranges(spec["path"], [spec["loop"]])
    with np.errstate(all="ignore"):
        exec(loop, ns)
    return trace, p_init, ns


def param_cases(n, nsrc, p_init, rs):
    """Parameter vectors for model/chi^2 fixtures: initial guess, truth, random
    perturbations and edge cases."""
    truth = np.append(synth.truth_params(n, nsrc), 0.0)
    cases = [p_init.copy(), truth]
    k = 16 if nsrc == 2 else 19
    pos = list(range(4 if nsrc == 2 else 6))
    for _ in range(8):
        p = truth.copy()
        p[pos] += rs.uniform(-1.5, 1.5, size=len(pos))
        off = 4 if nsrc == 2 else 6
        p[off:off + 2] = rs.uniform(-0.5, 0.5, size=2)
        sig = slice(10, 14) if nsrc == 2 else slice(13, 17)
        p[sig] = p[sig] * rs.uniform(0.6, 1.6, size=4)
        th = [14, 15] if nsrc == 2 else [17, 18]
        p[th] = rs.uniform(-np.pi, np.pi, size=2)
        cases.append(p)
    # edge cases
    e = truth.copy(); e[0] = -20.0; e[1] = n + 15.0; cases.append(e)     # source off-image
    e = truth.copy(); s = 10 if nsrc == 2 else 13; e[s] = 0.3; e[s + 1] = 0.35
    cases.append(e)                                                        # tiny core
    e = truth.copy(); r = 8 if nsrc == 2 else 11; e[r] = 1.3; cases.append(e)  # ratio > 1
    e = truth.copy(); s = 12 if nsrc == 2 else 15; e[s] = 0.9; e[s + 1] = 7.0
    th = 15 if nsrc == 2 else 18; e[th] = 0.785; cases.append(e)           # elongated
    assert all(len(c) == k + 1 for c in cases)
    return np.array(cases)


def bad_pixels(n, nsrc):
    """Non-finite data pixels (row, col, value) for the ``*_nan`` cases: NaN and -inf
    in the star's wing (below the saturation mask), by the companion and in the sky,
    and one +inf (already masked by masked_greater, apf_step2.py:188).  The pixels the
    initial guess reads (amplitudes, apf_step2.py:267-268; sky box, :269-271) stay
    finite."""
    g = synth.guess_values(n, nsrc)
    rs, cs = int(g[1] - 1), int(g[0] - 1)
    rc, cc = int(g[3] - 1), int(g[2] - 1)
    # (the 3-source script reads its amplitudes at int(y + 0.5), int(x + 0.5), i.e. one
    # pixel further, 3body/apf_step2_3body.py:258-260: keep that pixel finite too)
    dc = 2 if nsrc == 3 else 1
    return [(rs - 2, cs - 1, np.nan), (rs - 2, cs + 2, -np.inf), (rc + dc, cc + 1, np.nan),
            (rc - 1, cc, -np.inf), (n - 3, n - 5, -np.inf), (n // 2 + 6, 4, np.nan),
            (n - 2, 3, np.inf)]


def make_case(name, n, nsrc, n_walkers, accept_min, burn_in, n_model=None, nonfinite=False):
    spec = TWO if nsrc == 2 else THREE
    image, _ = synth.make_image(n, nsrc, seed=0)
    if nonfinite:
        for r, c, v in bad_pixels(n, nsrc):
            image[r, c] = v
    image = image.astype(">f4")                  # what fits.open returns for BITPIX -32
    header = dict((k.lower(), v) for k, v in synth.HEADER.items())
    guess = synth.guess_values(n, nsrc)
    ns = reference_namespace(spec, image, header, guess)
    p_init = ns["parameters"].copy()
    rs = np.random.RandomState(42)
    cases = param_cases(n, nsrc, p_init, rs)
    if n_model is not None:
        cases = cases[:n_model]
    models_ = []
    chis = []
    with np.errstate(all="ignore"):
        for p in cases:
            m = ns["build_analytical_model"](p)
            c = ns["chi_squared"](ns["image_nanmask"], m, ns["err"])
            models_.append(np.asarray(m, dtype=np.float64))
            chis.append(np.nan if c is np.ma.masked else float(c))
    out = dict(image=np.asarray(image, dtype=np.float32), guess=np.array(guess),
               mask=np.ma.getmaskarray(ns["image_nanmask"]),
               err=np.asarray(ns["err"], dtype=np.float64),
               readnoise=np.float64(ns["readnoise"]), satlevel=np.float64(ns["satlevel"]),
               p_init=p_init, params=cases, models=np.array(models_), chi2=np.array(chis),
               nsrc=np.int64(nsrc))
    seeds = np.arange(1000, 1000 + n_walkers)
    traj = {}
    csv_files = {}
    with tempfile.TemporaryDirectory() as td:
        for w, s in enumerate(seeds):
            tr, p0, _ = run_reference_loop(spec, image, header, guess, int(s), accept_min,
                                           burn_in, td, w)
            traj[w] = tr
            if w == 0:                           # keep one chain file per case (size)
                with open(os.path.join(td, f"{w}_finalarray_mpi.csv"), "rb") as f:
                    csv_files[f"{w}_finalarray_mpi.csv"] = f.read()
            with open(os.path.join(td, f"{w}_acceptance_rate.csv"), "rb") as f:
                csv_files[f"{w}_acceptance_rate.csv"] = f.read()
    lens = [len(traj[w]) for w in range(n_walkers)]
    L = max(lens)
    P = len(p_init)
    t_r = np.full((n_walkers, L), -1, np.int64)
    t_new = np.full((n_walkers, L), np.nan)
    t_chi = np.full((n_walkers, L), np.nan)
    t_dice = np.full((n_walkers, L), np.nan)
    t_acc = np.zeros((n_walkers, L), bool)
    t_par = np.full((n_walkers, L, P), np.nan)
    for w in range(n_walkers):
        for i, (r, nv, c, d, a, par) in enumerate(traj[w]):
            t_r[w, i], t_new[w, i], t_chi[w, i], t_dice[w, i], t_acc[w, i] = r, nv, c, d, a
            t_par[w, i] = par
    out.update(seeds=seeds, traj_len=np.array(lens), traj_r=t_r, traj_new=t_new,
               traj_chi=t_chi, traj_dice=t_dice, traj_acc=t_acc, traj_params=t_par,
               accept_min=np.int64(accept_min), burn_in=np.int64(burn_in))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    cdir = os.path.join(HERE, f"{name}_csv")
    os.makedirs(cdir, exist_ok=True)
    for fn, data in csv_files.items():
        with open(os.path.join(cdir, fn), "wb") as f:
            f.write(data)
    print(name, "iterations per walker:", lens, "chi2[0]:", chis[0])


def make_long_case(name, n, nsrc, n_walkers, accept_min, burn_in):
    """Round 4: long reference-executed chains, for posterior-level parity against the
    reference's own lines (not only the oracle).  The same harness as make_case, run
    to a larger accept_min; only the parameter rows (the state after every iteration,
    what the chain files hold past burn-in) and the accept flags are stored."""
    spec = TWO if nsrc == 2 else THREE
    image, _ = synth.make_image(n, nsrc, seed=0)
    image = image.astype(">f4")
    header = dict((k.lower(), v) for k, v in synth.HEADER.items())
    guess = synth.guess_values(n, nsrc)
    seeds = np.arange(1000, 1000 + n_walkers)
    rows, accs, p0 = [], [], None
    with tempfile.TemporaryDirectory() as td:
        for w, s in enumerate(seeds):
            # burn_in past the run: the reference's O(n^2) stacking and rewrite of the
            # chain file is skipped (the rows come from the trace), not its sampling
            tr, p0, _ = run_reference_loop(spec, image, header, guess, int(s), accept_min,
                                           10 ** 9, td, w)
            rows.append(np.array([t[5] for t in tr]))
            accs.append(np.array([t[4] for t in tr]))
            print(name, "walker", w, "iterations", len(tr), flush=True)
    lens = np.array([len(r) for r in rows])
    L = lens.max()
    P = len(p0)
    t_par = np.full((n_walkers, L, P), np.nan)
    t_acc = np.zeros((n_walkers, L), bool)
    for w in range(n_walkers):
        t_par[w, :lens[w]] = rows[w]
        t_acc[w, :lens[w]] = accs[w]
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), image=np.asarray(image, np.float32),
                        guess=np.array(guess), p_init=p0, seeds=seeds, traj_len=lens,
                        traj_params=t_par, traj_acc=t_acc, accept_min=np.int64(accept_min),
                        nsrc=np.int64(nsrc))
    print(name, "iterations per walker:", list(lens))


def _posterior_walker(args):
    spec_name, n, nsrc, seed, accept_min = args
    spec = TWO if spec_name == "two" else THREE
    np.seterr(all="ignore")
    image, _ = synth.make_image(n, nsrc, seed=0)
    image = image.astype(">f4")
    header = dict((k.lower(), v) for k, v in synth.HEADER.items())
    guess = synth.guess_values(n, nsrc)
    with tempfile.TemporaryDirectory() as td:
        tr, p0, ns = run_reference_loop(spec, image, header, guess, int(seed), accept_min,
                                        10 ** 9, td, 0)
    rows = np.array([t[5] for t in tr])
    accs = np.array([t[4] for t in tr])
    draws = np.array([t[0] for t in tr], np.uint8)
    return (rows, accs, p0, np.asarray(ns["total_tries"], np.float64),
            np.asarray(ns["total_accept"], np.float64), draws)


def make_posterior_case(name, n, nsrc, n_walkers, accept_min, every=50):
    """Round 5: ~20,000-iteration chains of the reference's own loop (the verdict's
    'posterior runs are oracle-only'), stored compactly: every ``every``-th row, every
    accept decision (bit-packed), each walker's whole-chain mean and sum of squared
    deviations per column (what step 3's statistics need, apf_step3.py:258-278), the
    tries / accepts counters and the final state.  Walkers run in parallel processes."""
    import multiprocessing as mp
    seeds = np.arange(1000, 1000 + n_walkers)
    with mp.get_context("fork").Pool(min(n_walkers, os.cpu_count() or 1)) as pool:
        res = pool.map(_posterior_walker, [("two" if nsrc == 2 else "three", n, nsrc, int(s),
                                            accept_min) for s in seeds])
    lens = np.array([len(r[0]) for r in res])
    L = int(lens.min())                   # every walker's first L iterations
    P = res[0][2].size
    sub = np.arange(every - 1, L, every)  # rows after iterations every, 2 every, ...
    rows_sub = np.array([r[0][sub] for r in res])
    acc_bits = np.array([np.packbits(r[1][:L]) for r in res])
    mean = np.array([r[0][:L].mean(axis=0) for r in res])
    m2 = np.array([((r[0][:L] - r[0][:L].mean(axis=0)) ** 2).sum(axis=0) for r in res])
    # (the draws -- the parameter index of every iteration -- and the accept bits give
    # the tries / accepts after L iterations; the reference's total_tries / total_accept
    # at its own stop are kept as well)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), image=np.asarray(
        synth.make_image(n, nsrc, seed=0)[0].astype(">f4"), np.float32),
        guess=np.array(synth.guess_values(n, nsrc)), p_init=res[0][2], seeds=seeds,
        traj_len=lens, L=np.int64(L), every=np.int64(every), rows_sub=rows_sub,
        acc_bits=acc_bits, draws=np.array([r[5][:L] for r in res]), mean=mean, m2=m2,
        final=np.array([r[0][L - 1] for r in res]),
        stop_tries=np.array([r[3] for r in res]), stop_accepts=np.array([r[4] for r in res]),
        accept_min=np.int64(accept_min), nsrc=np.int64(nsrc))
    print(name, "iterations per walker:", list(lens), "kept", L, "P", P, flush=True)


def make_rng():
    seeds = [0, 1, 5489, 12345, 2 ** 32 - 1] + list(range(1000, 1008))
    raw, gauss, unif, ri16, ri19 = [], [], [], [], []
    for s in seeds:
        raw.append(np.random.RandomState(s).randint(0, 2 ** 32, size=1500, dtype=np.uint64))
        gauss.append(np.random.RandomState(s).standard_normal(400))
        unif.append(np.random.RandomState(s).rand(400))
        ri16.append(np.random.RandomState(s).randint(0, 16, size=400))
        ri19.append(np.random.RandomState(s).randint(0, 19, size=400))
    np.savez_compressed(os.path.join(HERE, "rng.npz"), seeds=np.array(seeds, np.uint64),
                        raw=np.array(raw, np.uint64), gauss=np.array(gauss),
                        unif=np.array(unif), randint16=np.array(ri16),
                        randint19=np.array(ri19))


def make_fits():
    """FITS files written by astropy (the reference's reader) + expected arrays."""
    rs = np.random.RandomState(7)
    f32 = (rs.normal(0, 100, size=(32, 32))).astype(np.float32)
    hdu = fits.PrimaryHDU(f32)
    for k, v in synth.HEADER.items():
        hdu.header[k] = v
    hdu.header["OBJECT"] = "synthetic"
    hdu.writeto(os.path.join(HERE, "astropy_f32.fits"), overwrite=True)
    i16 = rs.randint(0, 60000, size=(16, 24)).astype(np.uint16)
    hdu2 = fits.PrimaryHDU(i16)                  # astropy stores uint16 as int16 + BZERO
    hdu2.header["SAMPMODE"] = 3
    hdu2.writeto(os.path.join(HERE, "astropy_u16.fits"), overwrite=True)
    f64 = rs.normal(0, 1, size=(8, 8))
    fits.PrimaryHDU(f64).writeto(os.path.join(HERE, "astropy_f64.fits"), overwrite=True)
    # our writer, read back by astropy
    td = tempfile.mkdtemp()
    p = os.path.join(td, "ours.fits")
    fitsio.write(p, f32, synth.HEADER)
    back = fits.open(p)[0]
    assert np.array_equal(back.data, f32) and back.header["itime"] == 1.0
    np.savez_compressed(os.path.join(HERE, "fits_expected.npz"), f32=f32,
                        u16=fits.open(os.path.join(HERE, "astropy_u16.fits"))[0].data,
                        f64=f64)


if __name__ == "__main__":
    np.seterr(all="ignore")
    if sys.argv[1:] == ["long"]:
        # round 4: >= 5,000 iterations x 4 walkers (64x64, 2 sources) and >= 1,500 x 2
        # (128x128, 3 sources) from the reference's own loop
        make_long_case("c64_long", 64, 2, n_walkers=4, accept_min=340, burn_in=0)
        make_long_case("c128_3_long", 128, 3, n_walkers=2, accept_min=90, burn_in=0)
        sys.exit(0)
    if sys.argv[1:] == ["long2"]:
        # configs[0]'s shape (32x32, 2 sources) past its 1,000 iterations, and the 3-source
        # 64x64 cutout past 2,000
        make_long_case("c32_long", 32, 2, n_walkers=2, accept_min=75, burn_in=0)
        make_long_case("c64_3_long", 64, 3, n_walkers=2, accept_min=115, burn_in=0)
        sys.exit(0)
    if sys.argv[1:] == ["posterior"]:
        # round 5: ~20,000 iterations per walker from the reference's own loop, 8 walkers
        # at 64x64 (2 sources) and 4 at 128x128 (3 sources)
        make_posterior_case("c64_post", 64, 2, n_walkers=8, accept_min=1200)
        make_posterior_case("c128_3_post", 128, 3, n_walkers=4, accept_min=1000)
        sys.exit(0)
    if sys.argv[1:] == ["nonfinite3"]:
        # round 4: the 3-source twins with non-finite data pixels (3body
        # apf_step2_3body.py's chi_squared is the same np.ma arithmetic)
        make_case("c64_3_nan", 64, 3, n_walkers=2, accept_min=20, burn_in=0, nonfinite=True)
        make_case("c128_3_nan", 128, 3, n_walkers=2, accept_min=6, burn_in=0, n_model=4,
                  nonfinite=True)
        sys.exit(0)
    if sys.argv[1:] == ["nonfinite"]:
        # round 3: cutouts with NaN / -inf / +inf data pixels (the reference's np.ma
        # chi_squared drops them, apf_step2.py:134-137 on the array from :188)
        make_case("c32_nan", 32, 2, n_walkers=3, accept_min=40, burn_in=5, nonfinite=True)
        make_case("c64_nan", 64, 2, n_walkers=2, accept_min=30, burn_in=5, nonfinite=True)
        sys.exit(0)
    make_rng()
    make_fits()
    make_case("c32", 32, 2, n_walkers=4, accept_min=40, burn_in=5)
    make_case("c64", 64, 2, n_walkers=4, accept_min=30, burn_in=5)
    make_case("c64_3", 64, 3, n_walkers=2, accept_min=20, burn_in=0)
    make_case("c128_3", 128, 3, n_walkers=2, accept_min=6, burn_in=0, n_model=4)
