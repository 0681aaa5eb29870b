"""Gelman-Rubin fixture for the step-3 contract (apf_step3.py:258-278,
3body/apf_step3_3body.py:292-310), pinned by hand rather than by executing the
reference: the reference is Python 2, and running its lines under Python 3 would turn
``(d+3)/(d+1)`` (int d = 16, apf_step3.py:264,276) into 19/17 instead of Python 2's
integer 1.  So this script restates the formula in exact rational arithmetic
(``fractions.Fraction``) with the Python-2 integer quotient written out, and stores
only data: the chain sets and the expected PSRF / RC per parameter.

    python tests/golden/make_gr_golden.py      # writes tests/golden/gr.npz

Chains: 2-source (17 columns: 16 parameters + chi^2) and 3-source (20 columns) sets of
walkers x rows drawn from seeded normals with per-walker offsets, so that RC is
visibly above 1.
"""
import os
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

D = 16
PY2_FACTOR = (D + 3) // (D + 1)        # Python 2: 19 / 17 == 1 for ints
assert PY2_FACTOR == 1


def exact_psrf(p):
    """p [N, M] float64 -> PSRF as a Fraction, following apf_step3.py:266-275 term by
    term (np.std is the ddof=0 standard deviation, so std**2 is the mean squared
    deviation from the column mean)."""
    N, M = p.shape
    cols = [[Fraction(float(v)) for v in p[:, i]] for i in range(M)]
    overall = sum(sum(c) for c in cols) / (N * M)
    w = []
    b = []
    for c in cols:
        mean = sum(c) / N
        w.append(sum((v - mean) ** 2 for v in c) / N)
        b.append((mean - overall) ** 2)
    W = Fraction(1, M) * sum(w)
    B = Fraction(N, M - 1) * sum(b)
    pooled = Fraction(N - 1, N) * W + Fraction(M + 1, M * N) * B
    return pooled / W


def make_set(rs, n_rows, n_walkers, ps):
    offs = rs.normal(scale=0.3, size=(1, n_walkers, ps))
    scale = 10.0 ** rs.uniform(-3, 3, size=(1, 1, ps))
    return (rs.normal(size=(n_rows, n_walkers, ps)) + offs) * scale + 100.0 * rs.normal(size=ps)


def main():
    rs = np.random.RandomState(20251016)
    out = {}
    for tag, ps, n_rows, n_walkers in (("2", 17, 40, 5), ("3", 20, 33, 4)):
        chains = make_set(rs, n_rows, n_walkers, ps)          # [N, M, PS]
        npar = ps - 1
        psrf = np.array([float(exact_psrf(chains[:, :, k])) for k in range(npar)])
        out[f"chains{tag}"] = chains
        out[f"psrf{tag}"] = psrf
        # RC = sqrt(PY2_FACTOR * PSRF) with the factor 1
        out[f"rc{tag}"] = np.sqrt(PY2_FACTOR * psrf)
    out["d"] = np.array(D)
    np.savez(os.path.join(HERE, "gr.npz"), **out)


if __name__ == "__main__":
    main()
