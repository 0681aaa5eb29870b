"""Step-3 read contract and convergence summary.

apf_step3.py reads the step-2 chain files (:169-186), drops ``additional_burnin`` rows
(:81-84, :190-205; default 1 = the NaN seed row) and computes Gelman-Rubin statistics
with d = 16 (:258-278) before its (out-of-scope) distortion / refraction / plotting
stages.  This module is that read + statistics front end, usable on the build's output.
"""
from __future__ import annotations

import os

import numpy as np

NAMES_2 = ["xcs", "ycs", "xcc", "ycc", "dx", "dy", "amps", "ampc", "ampratio", "bkgd",
           "sigmax", "sigmay", "sigmax2", "sigmay2", "theta", "theta2", "chisquare"]
NAMES_3 = ["xca", "yca", "xcb", "ycb", "xcc", "ycc", "dx", "dy", "ampa", "ampb", "ampc",
           "ampratio", "bkgd", "sigmax", "sigmay", "sigmax2", "sigmay2", "theta", "theta2",
           "chisquare"]


def load_chains(input_directory: str, ncor: int, additional_burnin: int = 1):
    """apf_step3.py:169-205: returns an array [length - additional_burnin, ncor, PS].

    The chain length is taken from walker 0 and every walker file must have it (the
    reference assigns columns into [length, ncor] arrays, :174-186)."""
    first = np.genfromtxt(os.path.join(input_directory, "0_finalarray_mpi.csv"), delimiter=",")
    first = np.atleast_2d(first)
    length, ps = first.shape
    out = np.zeros((length, ncor, ps))
    for i in range(ncor):
        a = np.atleast_2d(np.genfromtxt(os.path.join(input_directory, f"{i}_finalarray_mpi.csv"),
                                        delimiter=","))
        if a.shape != (length, ps):
            raise ValueError(f"walker {i}: chain shape {a.shape} != walker 0's {(length, ps)}")
        out[:, i, :] = a
    return out[additional_burnin:length]


def gelman_rubin(p, d: int = 16):
    """apf_step3.py:260-276 (3body/apf_step3_3body.py:294-310) for one parameter:
    p [N, M] (rows, walkers) -> (PSRF, RC).

    The reference is Python 2 without ``from __future__ import division``, so its
    ``RC = np.sqrt(((d+3)/(d+1))*PSRF)`` with the int ``d = 16`` (:264, :276) divides
    19 by 17 as integers: the factor is 1 and RC = sqrt(PSRF).  Integer ``d`` keeps
    that floor division here; a float ``d`` divides as floats, as it would there."""
    p = np.asarray(p, dtype=np.float64)
    N, M = float(p.shape[0]), float(p.shape[1])
    ncor = p.shape[1]
    w, b = np.zeros(ncor), np.zeros(ncor)
    overall_mean = np.mean(p)
    for i in range(ncor):                        # per column, as the reference does
        chain_mean = np.mean(p[:, i])
        w[i] = np.std(p[:, i]) ** 2
        b[i] = (chain_mean - overall_mean) ** 2
    w = (1. / M) * np.sum(w)
    b = (N / (M - 1)) * np.sum(b)
    pooled = ((N - 1) / N) * w + ((M + 1) / (M * N)) * b
    psrf = pooled / w
    factor = (d + 3) // (d + 1) if isinstance(d, (int, np.integer)) else (d + 3) / (d + 1)
    return psrf, np.sqrt(factor * psrf)


def summary(chains, nsrc: int = 2):
    """Per-parameter mean, median, std and Gelman-Rubin PSRF / RC over [N, M, PS]
    chains (the chi^2 column is not a GR parameter: apf_step3.py:260,
    3body/apf_step3_3body.py:294)."""
    names = NAMES_2 if nsrc == 2 else NAMES_3
    out = {}
    for k, name in enumerate(names[:-1]):
        x = chains[:, :, k]
        psrf, rc = gelman_rubin(x)
        out[name] = {"mean": float(np.mean(x)), "median": float(np.median(x)),
                     "std": float(np.std(x)), "gr_psrf": float(psrf), "gr_rc": float(rc)}
    return out
