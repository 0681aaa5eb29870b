"""Headless step 1: the initial-guess file without the GUI.

apf_step1.py asks for three mouse clicks per image (companion, star, sky; :71-142),
truncates them to ints, takes the maximum of a 21x21 aperture around each source click
(:145-163) and writes ``<dir>/<frame>_initialguess`` = "xcs ycs xcc ycc bkgdx bkgdy"
(:166-175).  Here the click positions are arguments; everything after the clicks is
the reference's arithmetic.  3-source guesses (8 values: A, B, C, sky) take
3body/apf_step1_3body.py's 8x8 box and integer positions (``main(three_body=True)``,
the ``3body/apf_step1_3body.py`` front end).
"""
from __future__ import annotations

import argparse
import glob
import os
import sys

import numpy as np

from . import fitsio


def aperture_max(image, xm: int, ym: int):
    """apf_step1.py:145-152 / :155-162: 21x21 box from (xm-11, ym-11), argmax,
    + 0.5 px.  Returns (x, y)."""
    ymin = ym - 11
    xmin = xm - 11
    apr = image[ymin:ymin + 21, xmin:xmin + 21]
    c = np.unravel_index(np.argmax(apr), apr.shape)        # findmax, :56-60
    return xmin + c[1] + 0.5, ymin + c[0] + 0.5


def aperture_max_3body(image, xm: int, ym: int):
    """3body/apf_step1_3body.py:165-186: the 8x8 box image[ym-4:ym+4, xm-4:xm+4],
    argmax, integer position (no half-pixel shift).  Returns (x, y).  (The reference
    script names the truncated clicks xma/xmb/xmc at :88-140 but reads xca/xcb/xcc here,
    so it stops with a NameError; the click is what it means.)"""
    apr = image[ym - 4:ym + 4, xm - 4:xm + 4]
    c = np.unravel_index(np.argmax(apr), apr.shape)
    return xm - 4 + int(c[1]), ym - 4 + int(c[0])


def guess(image, sources, sky, three_body: bool = False):
    """sources: [(x, y), ...] clicks (star first, then companions); sky: (x, y).
    Returns the guess values in the file order (apf_step1.py:172 / 3body :193:
    star, companions, sky)."""
    box = aperture_max_3body if three_body else aperture_max
    vals = []
    for (x, y) in sources:
        vals.extend(box(image, int(x), int(y)))
    vals.extend([int(sky[0]), int(sky[1])])
    return vals


def guess_path(image_path: str) -> str:
    """apf_step1.py:167-169: ``directory + '/' + basename.split('.')[2] + '_initialguess'``."""
    directory = os.path.dirname(image_path)
    base = os.path.basename(image_path)
    return directory + '/' + base.split('.')[2] + '_initialguess'


def write_guess(path: str, vals) -> None:
    """apf_step1.py:172-175: str() of each value, space separated, newline."""
    with open(path, "w") as f:
        f.write(" ".join(str(v) for v in vals) + "\n")


def main(argv=None, three_body: bool = False):
    """three_body: 3body/apf_step1_3body.py's aperture (8x8 box, integer positions) and
    exactly two companions (B, C)."""
    ap = argparse.ArgumentParser(prog="apf_step1_3body" if three_body else "apf_step1")
    ap.add_argument("directory", help="directory holding *.LDIF.fits (no trailing '/')")
    ap.add_argument("--star", nargs=2, type=float, required=True, metavar=("X", "Y"))
    ap.add_argument("--companion", nargs=2, type=float, action="append", required=True,
                    metavar=("X", "Y"), help="repeat for a second companion (3-source)")
    ap.add_argument("--sky", nargs=2, type=float, required=True, metavar=("X", "Y"))
    ap.add_argument("--pattern", default="*.LDIF.fits")
    args = ap.parse_args(sys.argv[1:] if argv is None else argv)
    if three_body and len(args.companion) != 2:
        ap.error("the 3-source step 1 takes two --companion positions (B and C)")
    out = []
    for path in sorted(glob.glob(os.path.join(args.directory, args.pattern))):
        image, _ = fitsio.getdata_header(path)
        vals = guess(image, [tuple(args.star)] + [tuple(c) for c in args.companion], args.sky,
                     three_body)
        gp = guess_path(path)
        write_guess(gp, vals)
        print("Initial guess:", vals, "->", gp)
        out.append(gp)
    return out
