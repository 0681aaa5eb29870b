"""CPU ORACLE for the apf_step2 Gibbs/Metropolis-Hastings hot path.

TEST INFRASTRUCTURE ONLY.  This module is imported by ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` -- as the
checker and as the timed CPU baseline.  The product (``olpefit_amd``) never imports
it: the sampler runs only through the HIP library and fails loudly without it.

It is a plain-NumPy restatement of the reference's arithmetic.  Every function cites
the reference line it follows (paths relative to the reference checkout):

* ``apf_step2.py``                -- 2-source sampler (16 params + chi^2)
* ``3body/apf_step2_3body.py``    -- 3-source twin (19 params + chi^2)
* astropy 4.3.1 ``Gaussian2D.evaluate``
  (``astropy/modeling/functional_models.py:366-381``), the third-party function the
  reference calls through ``models.Gaussian2D(...)(x, y)``.  The reference pins no
  astropy version; 4.3.1 is the copy in the survey container.
* NumPy legacy ``RandomState`` (MT19937 + polar Box-Muller): used directly -- the
  reference calls the global ``np.random`` whose stream is frozen by NumPy policy.

Pinning: ``tests/golden/make_golden.py`` executes the reference's own function
definitions and loop body (line ranges of apf_step2.py / apf_step2_3body.py) with
astropy 4.3.1 in the survey container, and ``tests/test_oracle_golden.py`` checks this
restatement against those fixtures.
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------------------------
# Parameter layouts
# ----------------------------------------------------------------------------------

#: apf_step2.py:234 jump widths (index = parameter index)
WIDTHS_2 = np.array([0.01, 0.01, 0.3, 0.3, 0.08, 0.09, 0.0025, 0.02, 0.001, 0.0008,
                     0.002, 0.002, 0.001, 0.001, 0.008, 0.01])
#: apf_step2.py:215 / :217
NORM_2 = [0, 1, 2, 3, 4, 5, 8, 14, 15]
LOGNORM_2 = [6, 7, 9, 10, 11, 12, 13]

#: 3body/apf_step2_3body.py:220-238
WIDTHS_3 = np.array([0.01, 0.01, 0.3, 0.3, 0.3, 0.3, 0.08, 0.09, 0.0025, 0.02, 0.02,
                     0.001, 0.0008, 0.002, 0.002, 0.001, 0.001, 0.008, 0.01])
#: 3body/apf_step2_3body.py:292 / :295
NORM_3 = [0, 1, 2, 3, 4, 5, 6, 7, 11, 17, 18]
LOGNORM_3 = [8, 9, 10, 12, 13, 14, 15, 16]


def layout(nsrc: int):
    """(n_params, widths, norm, lognorm) for the 2- or 3-source sampler."""
    if nsrc == 2:
        return 16, WIDTHS_2, NORM_2, LOGNORM_2
    if nsrc == 3:
        return 19, WIDTHS_3, NORM_3, LOGNORM_3
    raise ValueError("nsrc must be 2 or 3")


#: NIRC2 PSF width used for the initial guess, apf_step2.py:242-245
FWHM_MAS = 50
PIXSCALE_MAS = 9.95
SIGMA0 = (FWHM_MAS / PIXSCALE_MAS) / 2.35


# ----------------------------------------------------------------------------------
# Model (apf_step2.py:78-132, astropy Gaussian2D.evaluate)
# ----------------------------------------------------------------------------------

def gaussian2d(x, y, amplitude, x_mean, y_mean, x_stddev, y_stddev, theta):
    """astropy 4.3.1 ``Gaussian2D.evaluate`` (functional_models.py:366-381), same
    operation order: ``A*exp(-((a*dx**2) + (b*dx*dy) + (c*dy**2)))``."""
    cost2 = np.cos(theta) ** 2
    sint2 = np.sin(theta) ** 2
    sin2t = np.sin(2. * theta)
    xstd2 = x_stddev ** 2
    ystd2 = y_stddev ** 2
    xdiff = x - x_mean
    ydiff = y - y_mean
    a = 0.5 * ((cost2 / xstd2) + (sint2 / ystd2))
    b = 0.5 * ((sin2t / xstd2) - (sin2t / ystd2))
    c = 0.5 * ((sint2 / xstd2) + (cost2 / ystd2))
    return amplitude * np.exp(-((a * xdiff ** 2) + (b * xdiff * ydiff) +
                                (c * ydiff ** 2)))


#: the Gaussian evaluator build_2d_gaussian calls (use_astropy_models swaps it)
_GAUSS2D = gaussian2d


def use_astropy_models(models):
    """Evaluate every Gaussian the way the reference does, through astropy objects:
    ``models.Gaussian2D(amplitude=..., x_mean=..., y_mean=..., x_stddev=...,
    y_stddev=..., theta=...)(x, y)`` (apf_step2.py:98-102) -- the object construction
    and parameter validation the reference pays for twice per source per proposal
    (about 85 % of its build_2d_gaussian).  The values are those of
    ``gaussian2d`` (astropy's call is its ``evaluate``); only the cost differs.  Used by
    oracle/astropy_timing.py (/opt/conda python3.9 + astropy 4.3.1) for the CPU
    baseline of the reference's own loop cost on the GPU box's cores."""
    global _GAUSS2D

    def g(x, y, amplitude, x_mean, y_mean, x_stddev, y_stddev, theta):
        return models.Gaussian2D(amplitude=amplitude, x_mean=x_mean, y_mean=y_mean,
                                 x_stddev=x_stddev, y_stddev=y_stddev, theta=theta)(x, y)
    _GAUSS2D = g


def grid(n: int):
    """``y, x = np.mgrid[:ysize, :xsize]`` (apf_step2.py:94) for a square n x n image
    (the reference is square-only: apf_step2.py:237 swaps the axes)."""
    y, x = np.mgrid[:n, :n]
    return y, x


def build_2d_gaussian(yx, xc, yc, dx, dy, total_amplitude, amplituderatio, background,
                      narrow_sigma_x, narrow_sigma_y, wide_sigma_x, wide_sigma_y,
                      narrow_theta, wide_theta):
    """apf_step2.py:78-103: narrow + wide Gaussian, wide centred at (xc+dx, yc+dy).
    Returns ``wide + narrow`` in that order (:102)."""
    y, x = yx
    total_amplitude = total_amplitude - background                      # :95
    wide_amplitude = total_amplitude * amplituderatio                   # :96
    narrow_amplitude = total_amplitude - wide_amplitude                 # :97
    narrow = _GAUSS2D(x, y, narrow_amplitude, xc, yc, narrow_sigma_x,
                      narrow_sigma_y, narrow_theta)                     # :98-99
    wide = _GAUSS2D(x, y, wide_amplitude, xc + dx, yc + dy, wide_sigma_x,
                    wide_sigma_y, wide_theta)                           # :100-101
    return wide + narrow                                                # :102


def build_analytical_model(p, n: int, nsrc: int = 2, bkgd_mode: int = 0, yx=None):
    """apf_step2.py:106-124 (2 sources) / 3body/apf_step2_3body.py:106-125 (3 sources).

    bkgd_mode 0 reproduces the reference quirk: the constant background is p[12]
    (the wide sigma_x in the 2-source layout, apf_step2.py:119-120); bkgd_mode 1 uses
    p[9] (the dead code at :126-132).  In the 3-source layout p[12] *is* the
    background and bkgd_mode is ignored.
    """
    if yx is None:
        yx = grid(n)
    p = np.asarray(p, dtype=np.float64)
    if nsrc == 2:
        psfa = build_2d_gaussian(yx, p[0], p[1], p[4], p[5], p[6], p[8], p[9], p[10],
                                 p[11], p[12], p[13], p[14], p[15])   # :115
        psfb = build_2d_gaussian(yx, p[2], p[3], p[4], p[5], p[7], p[8], p[9], p[10],
                                 p[11], p[12], p[13], p[14], p[15])   # :116
        bkgd = np.ndarray(shape=(n, n), dtype=float)                   # :119
        bkgd.fill(p[12] if bkgd_mode == 0 else p[9])                   # :120 / :128
        return psfa + psfb + bkgd                                      # :123
    if nsrc == 3:
        args = (p[6], p[7])
        shared = (p[11], p[12], p[13], p[14], p[15], p[16], p[17], p[18])
        psfa = build_2d_gaussian(yx, p[0], p[1], *args, p[8], *shared)  # 3body :115
        psfb = build_2d_gaussian(yx, p[2], p[3], *args, p[9], *shared)  # :116
        psfc = build_2d_gaussian(yx, p[4], p[5], *args, p[10], *shared)  # :117
        bkgd = np.ndarray(shape=(n, n), dtype=float)                     # :120
        bkgd.fill(p[12])                                                 # :121
        return psfa + psfb + psfc + bkgd                                 # :124
    raise ValueError("nsrc must be 2 or 3")


def chi_squared(data, model, error):
    """apf_step2.py:134-137 on the np.ma masked image.  NumPy masked semantics are
    kept: masked pixels drop out, ``**2`` also masks non-finite entries
    (``np.ma.power``), and an all-masked sum returns ``np.ma.masked`` (treated as a
    rejected proposal by :144 because ``bool(masked) is False``)."""
    chisquared_per_pixel = ((data - model) / error) ** 2
    return np.sum(chisquared_per_pixel)


def accept_reject(chisquare_current, chisquare_proposal, rng):
    """apf_step2.py:139-148: p = exp(-(chi_p - chi_c)/2); dice = rand(); accept iff
    dice < p."""
    p_accept = np.exp(-(chisquare_proposal - chisquare_current) / 2.)
    dice = rng.rand()
    accept = bool(dice < p_accept)
    return accept, p_accept, dice


def proposal(rng, value, width):
    """apf_step2.py:63-65 (``normal(value, width, 1)``, element 0 taken at :307)."""
    return rng.normal(value, width, 1)[0]


def logproposal(rng, value, width):
    """apf_step2.py:66-70: ``10**normal(log10(value), width, 1)``."""
    with np.errstate(all="ignore"):
        logvalue = np.log10(value)
        lognew = rng.normal(logvalue, width, 1)
        return (10 ** lognew)[0]


def draw_index(rng, n_params: int):
    """apf_step2.py:302 ``randint(0,16)`` / 3body :328 ``randint(0,19)``."""
    return int(rng.randint(0, n_params))


# ----------------------------------------------------------------------------------
# Setup (apf_step2.py:176-210, :258-289)
# ----------------------------------------------------------------------------------

def noise_model(image, itime, coadds, multisam, sampmode):
    """apf_step2.py:176-210.  Returns (image_nanmask, err, satlevel, readnoise).

    ``itime`` is the raw header value (seconds); :176 multiplies it by 1000.
    For a float32 image the Poisson term ``sqrt(|D|)**2`` stays float32 (:207-210)."""
    itime = float(itime) * 1000.
    coadds = float(coadds)
    multisam = float(multisam)
    if sampmode == 3:
        satlevel = coadds * 24000.0 * (1.0 - 0.1 * (multisam - 1.0) / (itime / 1000.))
    else:
        satlevel = coadds * 22000.0
    image_nanmask = np.ma.masked_greater(image, 0.8 * satlevel)      # :188
    rnoise = np.ndarray(shape=image.shape, dtype=float)               # :197
    if sampmode == 3.0:
        readnoise = (38.0 / np.sqrt(multisam)) * (np.sqrt(coadds))
    elif sampmode == 2.0:
        readnoise = 38 * (np.sqrt(coadds))
    else:
        readnoise = 38 * (np.sqrt(coadds))
    rnoise.fill(readnoise)
    pois = np.sqrt(np.abs(image))                                      # :207
    err = np.sqrt(rnoise ** 2 + pois ** 2)                             # :210
    return image_nanmask, err, satlevel, readnoise


def initial_parameters(image, guess, nsrc: int = 2):
    """apf_step2.py:264-273 (2 sources) / 3body/apf_step2_3body.py:255-265 (3 sources).
    The chi^2 slot is left 0 here; :283-289 fills it."""
    sigma = SIGMA0
    if nsrc == 2:
        xcs, ycs, xcc, ycc = guess[0], guess[1], guess[2], guess[3]
        amps = image[int(ycs - 1), int(xcs - 1)]
        ampc = image[int(ycc - 1), int(xcc - 1)]
        box = image[int(guess[5]):int(guess[5]) + 10, int(guess[4]):int(guess[4]) + 10]
        bkgd = np.median(box)
        return np.array([xcs, ycs, xcc, ycc, 0., 0., amps, ampc, 0.2, bkgd, sigma, sigma,
                         sigma * 3, sigma * 3, 0., 0., 0.])
    xca, yca, xcb, ycb, xcc, ycc = guess[:6]
    ampa = image[int(yca - 0.5 + 1), int(xca - 0.5 + 1)]
    ampb = image[int(ycb - 0.5 + 1), int(xcb - 0.5 + 1)]
    ampc = image[int(ycc - 0.5 + 1), int(xcc - 0.5 + 1)]
    box = image[int(guess[7]):int(guess[7]) + 10, int(guess[6]):int(guess[6]) + 10]
    bkgd = np.median(box)
    return np.array([xca, yca, xcb, ycb, xcc, ycc, 0., 0., ampa, ampb, ampc, 0.2, bkgd,
                     sigma, sigma, sigma * 3, sigma * 3, 0., 0., 0.])


# ----------------------------------------------------------------------------------
# Sampler loop (apf_step2.py:298-365; 3body :324-400)
# ----------------------------------------------------------------------------------

class Walker:
    """One independent walker = one MPI rank of the reference.

    ``rng`` is a ``np.random.RandomState(seed)``: identical to the reference's global
    ``np.random`` after ``np.random.seed(seed)``.
    """

    def __init__(self, image_nanmask, err, p0, seed, nsrc=2, bkgd_mode=0):
        self.data = image_nanmask
        self.err = err
        self.n = image_nanmask.shape[0]
        self.nsrc = nsrc
        self.bkgd_mode = bkgd_mode
        self.np_, self.widths, self.norm, self.lognorm = layout(nsrc)
        self.rng = np.random.RandomState(seed)
        self.yx = grid(self.n)
        self.parameters = np.array(p0, dtype=np.float64).copy()
        self.total_tries = np.zeros(self.np_)
        self.total_accept = np.zeros(self.np_)
        self.count = 0

    def model(self, p):
        return build_analytical_model(p, self.n, self.nsrc, self.bkgd_mode, self.yx)

    def chi2(self, p):
        return chi_squared(self.data, self.model(p), self.err)

    def init_chi2(self):
        """apf_step2.py:283-289."""
        with np.errstate(all="ignore"):
            self.parameters[-1] = self.chi2(self.parameters)

    def step(self):
        """One iteration of apf_step2.py:300-333.  Returns the trace record
        (r, new, chi_proposal, dice, accepted)."""
        rand = draw_index(self.rng, self.np_)                       # :302
        self.total_tries[rand] += 1                                  # :304
        if rand in self.norm:                                        # :306
            new = proposal(self.rng, self.parameters[rand], self.widths[rand])
        else:
            new = logproposal(self.rng, self.parameters[rand], self.widths[rand])
        parameters_proposal = self.parameters.copy()                 # :312
        parameters_proposal[rand] = new
        with np.errstate(all="ignore"):
            chi_proposal = self.chi2(parameters_proposal)           # :314-316
            accept, p_accept, dice = accept_reject(self.parameters[-1], chi_proposal,
                                                   self.rng)         # :318
        if accept:                                                   # :321-327
            self.total_accept[rand] += 1
            self.parameters[rand] = new
            self.parameters[-1] = chi_proposal
        self.count += 1                                              # :333
        chi_f = np.nan if chi_proposal is np.ma.masked else float(chi_proposal)
        return rand, float(new), chi_f, float(dice), accept

    def run(self, n_iters, burn_in=0, record_stride=1, trace=False):
        """Run ``n_iters`` iterations.  Returns (chain, trace) where ``chain`` holds
        the state after every iteration whose count c satisfies c >= burn_in and
        (c - burn_in) % record_stride == 0 (apf_step2.py:342-351 with stride 1)."""
        rows, tr = [], []
        for _ in range(n_iters):
            rec = self.step()
            if trace:
                tr.append(rec)
            c = self.count
            if c >= burn_in and (c - burn_in) % record_stride == 0:
                rows.append(self.parameters.copy())
        chain = np.array(rows).reshape(-1, self.np_ + 1)
        return chain, tr


def run_walkers(image_nanmask, err, p0, seeds, n_iters, nsrc=2, bkgd_mode=0, burn_in=0,
                record_stride=1, trace=False):
    """Run independent walkers serially; returns lists of (chain, trace, walker)."""
    out = []
    for s in seeds:
        w = Walker(image_nanmask, err, p0, int(s), nsrc, bkgd_mode)
        if p0[-1] == 0.0 or not np.isfinite(p0[-1]):
            w.init_chi2()
        chain, tr = w.run(n_iters, burn_in, record_stride, trace)
        out.append((chain, tr, w))
    return out


# ----------------------------------------------------------------------------------
# Step 3 read contract + Gelman-Rubin (apf_step3.py:169-205, :258-278)
# ----------------------------------------------------------------------------------

def gelman_rubin(chains, d=16):
    """apf_step3.py:260-278 (3body/apf_step3_3body.py:294-310).  ``chains``: array
    [length, ncor] for one parameter.  Returns (PSRF, RC).

    Python-2 semantics: the reference's ``(d+3)/(d+1)`` with int d = 16 is integer
    division (== 1), so RC = sqrt(PSRF)."""
    p = np.asarray(chains, dtype=np.float64)
    N, M = float(p.shape[0]), float(p.shape[1])
    ncor = p.shape[1]
    w, b = np.zeros(ncor), np.zeros(ncor)
    overall_mean = np.mean(p)
    for i in range(ncor):
        chain_mean = np.mean(p[:, i])
        w[i] = np.std(p[:, i]) ** 2
        b[i] = (chain_mean - overall_mean) ** 2
    w = (1. / M) * np.sum(w)
    b = (N / (M - 1)) * np.sum(b)
    pooled_variance = ((N - 1) / N) * w + ((M + 1) / (M * N)) * b
    psrf = pooled_variance / w
    rc = np.sqrt(((d + 3) // (d + 1)) * psrf)       # Python 2 int division: 19 / 17 == 1
    return psrf, rc
