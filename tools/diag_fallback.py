"""Which sweep the sampler's steps take (diagnostic build only):

    tools/diag_build.sh fb -DOLPE_DIAG_FALLBACK
    OLPE_LIB=diag/fb/libolpe.so python tools/diag_fallback.py [config | n nsrc walkers]

Runs bench.py's workload for one config (a few 100-iteration launches) and prints the
share of walker-steps that took the FAST3 sweep, and of the fallbacks (FAST2, V table,
exact) the guard sent the others to."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    from olpefit_amd import _lib, synth
    from olpefit_amd.core import Sampler
    from olpefit_amd.pipeline import initial_parameters
    if len(sys.argv) > 3:                 # any shape: n nsrc walkers
        n, nsrc, W = (int(v) for v in sys.argv[1:4])
        cfg = f"{n}x{n}/{nsrc}"
    else:
        cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
        W, n, nsrc = bench.CONFIGS[cfg]
    img, _ = synth.make_image(n, nsrc, 0)
    s = Sampler(img, 1.0, 1, 1, 2, nsrc=nsrc)
    p0 = initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    p0[-1] = s.chi_squared(p0)
    s.seed(1000 + np.arange(W))
    s.set_state(np.tile(p0, (W, 1)))
    for _ in range(4):
        s.run(100, burn_in=0, record_stride=10, read_chain=False)
    out = (C.c_ulonglong * 4)()
    _lib.check(_lib.load().olpe_diag_fallback(out))
    v = np.array(list(out), dtype=float)
    tot = v.sum()
    print(f"config {cfg}: {int(tot)} sweeps: FAST3 {v[0] / tot:.4%}, FAST2 {v[1] / tot:.4%}, "
          f"V table {v[2] / tot:.4%}, exact {v[3] / tot:.4%}")


if __name__ == "__main__":
    main()
