"""Work-unit diagnostics: kernel time and chunk hand-off waits of the
bench workload at a given walker count, for several chunk counts (OLPE_UNITS).

    python tools/unit_diag.py [walkers=4096] [units=1,2,3,6,12] [n=64] [nsrc=2] [iters=100]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    ulist = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,3,6,12").split(",")]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    nsrc = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 100
    from olpefit_amd import synth
    from olpefit_amd.core import Sampler
    from olpefit_amd.pipeline import initial_parameters
    img, _ = synth.make_image(n, nsrc, 0)
    p0 = initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    for u in ulist:
        os.environ["OLPE_UNITS"] = str(u)
        s = Sampler(img, 1.0, 1, 1, 2, nsrc=nsrc)
        p0[-1] = s.chi_squared(p0)
        s.seed(1000 + np.arange(W))
        s.set_state(np.tile(p0, (W, 1)))
        for _ in range(2):
            s.run_async(iters, burn_in=0, record_stride=10)
        s.sync()
        w0, t0 = s.unit_stats()
        steps = 10
        for _ in range(steps):
            s.run_async(iters, burn_in=0, record_stride=10)
        s.sync()
        w1, t1 = s.unit_stats()
        km = s.kernel_times(steps)
        ms = float(np.mean(km))
        waits = (w1 - w0) / steps
        wait_ms = (t1 - t0) / steps / 1e6
        print(f"W={W} iters={iters} units={s.last_units()} kernel_ms={ms:.3f} "
              f"rate={W * iters / ms / 1e3:.4g} M/s "
              f"waits/launch={waits:.0f} wave-ms waiting/launch={wait_ms:.2f} "
              f"(= {wait_ms / ms:.1f} of {W * u} units' slots)", flush=True)
        s.close()


if __name__ == "__main__":
    main()
