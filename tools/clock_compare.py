"""Round 5: is the SMU's reported GFX clock (amdsmi current_gfxclks, bench.SmiClock) the
clock the sampler runs at?  With the -DOLPE_DIAG_SPAN library each unit records its
s_memtime cycles and 100 MHz s_memrealtime span in the trace; this runs bench.py's
configs[2] launches back to back (warm-up, then N timed ones with the SMU sampled every
10 ms) and prints, per traced launch, the in-kernel clock against the SMU's samples.

    OLPE_LIB=diag/span/libolpe.so python tools/clock_compare.py [launches] [warmup]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from olpefit_amd import synth  # noqa: E402
from olpefit_amd.core import Sampler  # noqa: E402
from olpefit_amd.pipeline import initial_parameters  # noqa: E402


def main():
    n_l = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    W, iters = 65536, 100
    img, _ = synth.make_image(64, 2, 0)
    p0 = initial_parameters(img, synth.guess_values(64, 2), 2)
    s = Sampler(img, 1.0, 1, 1, 2, nsrc=2)
    p0[-1] = s.chi_squared(p0)
    s.seed(1000 + np.arange(W))
    s.set_state(np.tile(p0, (W, 1)))
    s.enable_trace(True)
    clock = bench.SmiClock(Sampler.device_pci_id(0))
    for _ in range(warm):
        s.run_async(iters, burn_in=0, record_stride=10)
    s.sync()
    for rnd in range(3):
        clock.start()
        t0 = time.perf_counter()
        for _ in range(n_l):
            s.run_async(iters, burn_in=0, record_stride=10)
        s.sync()
        t1 = time.perf_counter()
        smi, ns = clock.stop()
        km = float(np.mean(s.kernel_times(min(n_l, 64))))
        tr = s.trace(iters).reshape(W, -1)[:, :5]        # the last launch's units
        dur = (tr[:, 1] - tr[:, 0]) * 1e-8                # s
        inker = tr[:, 4] / dur / 1e9                      # GHz
        q = " ".join(f"{np.percentile(inker, p):.3f}" for p in (0, 10, 50, 90, 100))
        print(f"round {rnd}: {n_l} launches in {t1 - t0:.3f} s ({km:.3f} ms each); SMU mean "
              f"{smi:.3f} GHz over {ns} samples; last launch in-kernel s_memtime GHz "
              f"(units 0/10/50/90/100 %): {q}; cycle-weighted {tr[:, 4].sum() / dur.sum() / 1e9:.3f}")
    s.close()


if __name__ == "__main__":
    main()
