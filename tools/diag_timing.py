"""Per-section cycle split of the sampler step (diagnostic build only).

    tools/diag_build.sh timing -DOLPE_DIAG_TIMING
    OLPE_LIB=diag/timing/libolpe.so python tools/diag_timing.py [walkers] [iters] [n] [nsrc]

For the 128x128 ring sampler run one walker per wave (walkers = 12 x CUs, OLPE_UNITS=1):
lanes 7 / 8 then hold the ring's barrier waits (first phase of a step / the others).

The diagnostic kernel accumulates s_memtime deltas per wave over the sections of a
step and writes them over the trace buffer; this prints the mean per walker-step.
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from olpefit_amd import synth  # noqa: E402
from olpefit_amd.core import Sampler  # noqa: E402
from olpefit_amd.pipeline import initial_parameters  # noqa: E402

NAMES = ["randint+tries", "proposal (gauss, log/exp10)", "coef+model -> LDS",
         "sweep (guard, setup, rows)", "wave_sum", "accept", "chain record"]


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    nsrc = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    img, _ = synth.make_image(n, nsrc, 0)
    s = Sampler(img, 1.0, 1, 1, 2, nsrc=nsrc, device=0)
    p0 = initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    p0[-1] = s.chi_squared(p0)
    s.seed(1000 + np.arange(W))
    s.set_state(np.tile(p0, (W, 1)))
    s.enable_trace(True)
    s.run(iters, burn_in=0, record_stride=10)        # warm-up
    t0 = time.perf_counter()
    s.run(iters, burn_in=0, record_stride=10)
    wall = time.perf_counter() - t0
    kms = s.last_kernel_ms()
    full = s.trace(iters).reshape(W, -1)
    tr = full[:, :7] / iters                           # ticks per step, per walker
    if n == 128:
        print(f"ring barrier wait per step: first phase {full[:, 7].mean() / iters:.0f}, "
              f"other phases {full[:, 8].mean() / iters:.0f} ticks")
    else:
        print(f"column terms per step: setup {full[:, 7].mean() / iters:.3f}, "
              f"refresh after accept {full[:, 8].mean() / iters:.3f}")
    tot = tr.sum(axis=1)
    print(f"walkers {W} iters {iters} kernel {kms:.2f} ms (wall {wall * 1e3:.1f} ms)")
    print(f"per-wave step total: mean {tot.mean():.0f} ticks (min {tot.min():.0f}, "
          f"max {tot.max():.0f}); ticks/s if busy the whole kernel: "
          f"{tot.mean() * iters / (kms * 1e-3):.3g}")
    for k, name in enumerate(NAMES):
        print(f"  {name:30s} {tr[:, k].mean():9.0f}  {100 * tr[:, k].mean() / tot.mean():5.1f} %")
    s.close()


if __name__ == "__main__":
    main()
