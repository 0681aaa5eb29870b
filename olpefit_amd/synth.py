"""Synthetic NIRC2-shaped cutouts -- deterministic test/bench data.

There are no sample images in the reference, so every run uses data
made here: a float32 N x N primary-HDU FITS with the NIRC2 header cards the reference
reads (apf_step2.py:176-179), named ``N2.<date>.<frame>.LDIF.fits`` so that
apf_step2.py:170's ``split('.')[-3]`` gives ``<frame>``, plus the step-1 guess file
``<frame>_initialguess`` (apf_step1.py:166-175 writes the same 6 numbers; the 3-body
step 1 writes 8).

The truth image is rendered with the reference's own model formula (including the
2-source p[12] background quirk, apf_step2.py:119-120).  This is data generation,
not the hot path: it is plain NumPy.
"""
from __future__ import annotations

import os

import numpy as np

from . import fitsio

SIGMA0 = (50 / 9.95) / 2.35          # apf_step2.py:242-245
HEADER = {"ITIME": 1.0, "COADDS": 1, "MULTISAM": 1, "SAMPMODE": 2}


def _gauss(x, y, amp, x0, y0, sx, sy, th):
    cost2 = np.cos(th) ** 2
    sint2 = np.sin(th) ** 2
    sin2t = np.sin(2. * th)
    a = 0.5 * ((cost2 / sx ** 2) + (sint2 / sy ** 2))
    b = 0.5 * ((sin2t / sx ** 2) - (sin2t / sy ** 2))
    c = 0.5 * ((sint2 / sx ** 2) + (cost2 / sy ** 2))
    dx = x - x0
    dy = y - y0
    return amp * np.exp(-((a * dx ** 2) + (b * dx * dy) + (c * dy ** 2)))


def truth_params(n: int, nsrc: int = 2) -> np.ndarray:
    """Truth parameter vector in the reference layout (without the chi^2 slot)."""
    xs, ys = n / 2 - 0.3, n / 2 + 0.2
    xc, yc = xs + n / 5, ys - n / 6
    s = SIGMA0
    if nsrc == 2:
        # xcs ycs xcc ycc dx dy amps ampc ratio bkgd sx sy sx2 sy2 th th2
        return np.array([xs, ys, xc, yc, 0.1, -0.1, 3.0e4, 2.0e3, 0.2, 30.0,
                         s, s * 1.05, 3 * s, 3 * s * 1.05, 0.05, 0.10])
    xb, yb = xs - n / 4, ys + n / 5
    # xca yca xcb ycb xcc ycc dx dy ampa ampb ampc ratio bkgd sx sy sx2 sy2 th th2
    return np.array([xs, ys, xc, yc, xb, yb, 0.1, -0.1, 3.0e4, 2.0e3, 1.5e3, 0.2, 30.0,
                     s, s * 1.05, 3 * s, 3 * s * 1.05, 0.05, 0.10])


def render(p, n: int, nsrc: int = 2) -> np.ndarray:
    """Noise-free model image (float64) with the reference's layout and quirks."""
    y, x = np.mgrid[:n, :n]
    if nsrc == 2:
        srcs = [(p[0], p[1], p[6]), (p[2], p[3], p[7])]
        dx, dy, ratio, off = p[4], p[5], p[8], p[9]
        s1x, s1y, s2x, s2y, t1, t2 = p[10:16]
        bkgd = p[12]                         # apf_step2.py:120 quirk
    else:
        srcs = [(p[0], p[1], p[8]), (p[2], p[3], p[9]), (p[4], p[5], p[10])]
        dx, dy, ratio, off = p[6], p[7], p[11], p[12]
        s1x, s1y, s2x, s2y, t1, t2 = p[13:19]
        bkgd = p[12]
    img = np.zeros((n, n))
    for xc, yc, amp in srcs:
        tot = amp - off
        wide = tot * ratio
        narrow = tot - wide
        img = img + (_gauss(x, y, wide, xc + dx, yc + dy, s2x, s2y, t2) +
                     _gauss(x, y, narrow, xc, yc, s1x, s1y, t1))
    return img + bkgd


def make_image(n: int, nsrc: int = 2, seed: int = 0, readnoise: float = 38.0):
    """float32 image = model + N(0, sqrt(readnoise^2 + |model|)), RandomState(seed)."""
    p = truth_params(n, nsrc)
    m = render(p, n, nsrc)
    rng = np.random.RandomState(seed)
    noise = rng.normal(0.0, 1.0, size=(n, n)) * np.sqrt(readnoise ** 2 + np.abs(m))
    return (m + noise).astype(np.float32), p


def guess_values(n: int, nsrc: int = 2):
    """Step-1-style guess: truth positions + 0.5 px and a sky box at (2, 2)."""
    p = truth_params(n, nsrc)
    k = 4 if nsrc == 2 else 6
    return [float(v) + 0.5 for v in p[:k]] + [2.0, 2.0]


def write_case(directory: str, n: int, nsrc: int = 2, seed: int = 0,
               date: str = "20250127", frame: str = "00001") -> str:
    """Write ``N2.<date>.<frame>.LDIF.fits`` and ``<frame>_initialguess`` into
    ``directory``.  Returns the FITS path."""
    os.makedirs(directory, exist_ok=True)
    img, _ = make_image(n, nsrc, seed)
    path = os.path.join(directory, f"N2.{date}.{frame}.LDIF.fits")
    fitsio.write(path, img, HEADER)
    g = guess_values(n, nsrc)
    # apf_step1.py:172-175: str() of each value, space separated, sky box as ints
    words = [str(v) for v in g[:-2]] + [str(int(g[-2])), str(int(g[-1]))]
    with open(os.path.join(directory, f"{frame}_initialguess"), "w") as f:
        f.write(" ".join(words) + "\n")
    return path
