"""Check olpe::sincos_small (olpe_device.h, FAST kernels' sin/cos for |theta| <= pi/4)
against the exact values and numpy's sin/cos, with an exact (Decimal) emulation of the
device's fma (one rounding) and multiplications.

    python tools/check_sincos.py [N]

Prints the largest error in ulp of sin and cos over N random arguments in
[-pi/4, pi/4] plus the end points, and how far FAST's trig terms (cos^2, sin^2,
2 sin cos) lie from astropy's (np.cos(t)**2, np.sin(t)**2, np.sin(2t)).
"""
import math
import random
import sys
from decimal import Decimal, getcontext

import numpy as np

getcontext().prec = 60

S = [2.8114572543455207632e-15, -7.6471637318198164759e-13, 1.6059043836821614599e-10,
     -2.5052108385441718775e-8, 2.7557319223985890653e-6, -1.9841269841269841270e-4,
     8.3333333333333333333e-3, -1.6666666666666666667e-1]
C = [4.7794773323873852974e-14, -1.1470745597729724714e-11, 2.0876756987868098979e-9,
     -2.7557319223985890653e-7, 2.4801587301587301587e-5, -1.3888888888888888889e-3,
     4.1666666666666666667e-2, -0.5]


def fma(a, b, c):
    return float(Decimal(a) * Decimal(b) + Decimal(c))


def mul(a, b):
    return float(Decimal(a) * Decimal(b))


def sincos_small(th):
    """Operation-for-operation restatement of olpe::sincos_small."""
    t = mul(th, th)
    p = fma(t, S[0], S[1])
    for k in S[2:]:
        p = fma(t, p, k)
    s = fma(mul(th, t), p, th)
    q = fma(t, C[0], C[1])
    for k in C[2:]:
        q = fma(t, q, k)
    c = fma(t, q, 1.0)
    return s, c


def exact(th):
    x = Decimal(th)
    s, c, term, k = Decimal(0), Decimal(0), Decimal(1), 0
    while k < 60:
        if k % 4 == 0:
            c += term
        elif k % 4 == 1:
            s += term
        elif k % 4 == 2:
            c -= term
        else:
            s -= term
        k += 1
        term = term * x / k
    return s, c


def ulps(got, ref):
    return abs(float((Decimal(got) - ref) / Decimal(math.ulp(float(ref)))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    rnd = random.Random(7)
    lim = 0.78539816339744830962
    xs = [rnd.uniform(-lim, lim) for _ in range(n)] + [lim, -lim, 1e-8, 0.05, 0.1]
    ws = wc = 0.0
    wt = [0.0, 0.0, 0.0]
    for th in xs:
        s, c = sincos_small(th)
        rs, rc = exact(th)
        ws = max(ws, ulps(s, rs))
        wc = max(wc, ulps(c, rc))
        fast = (mul(c, c), mul(s, s), 2.0 * mul(s, c))
        ref = (np.cos(th) ** 2, np.sin(th) ** 2, np.sin(2.0 * th))
        for i in range(3):
            if ref[i] != 0:
                wt[i] = max(wt[i], abs(fast[i] - ref[i]) / math.ulp(ref[i]))
    print(f"sincos_small over {len(xs)} arguments in [-pi/4, pi/4]: sin {ws:.3f} ulp, "
          f"cos {wc:.3f} ulp (exact reference)")
    print(f"trig terms vs astropy's numpy forms: cos^2 {wt[0]:.1f}, sin^2 {wt[1]:.1f}, "
          f"sin 2t {wt[2]:.1f} ulp")


if __name__ == "__main__":
    main()
