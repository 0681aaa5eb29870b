"""Walker-steps/s of the sampler on cutout shapes beside the bench's configs (one GPU,
FAST, bench.py's step: 100 iterations, a chain row every 10, device-resident inputs).

    python tools/other_shapes.py [--steps K]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from olpefit_amd import synth  # noqa: E402
from olpefit_amd.core import Sampler  # noqa: E402
from olpefit_amd.pipeline import initial_parameters  # noqa: E402

SHAPES = [  # (n, nsrc, walkers)
    (32, 2, 65536), (32, 3, 65536), (64, 3, 32768), (128, 2, 16384), (48, 2, 32768)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    for n, nsrc, W in SHAPES:
        img, _ = synth.make_image(n, nsrc, 0)
        s = Sampler(img, 1.0, 1, 1, 2, nsrc=nsrc)
        s.set_eval_mode("fast")
        p0 = initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
        p0[-1] = s.chi_squared(p0)
        s.seed(np.arange(W))
        s.set_state(np.tile(p0, (W, 1)))
        for _ in range(args.warmup):
            s.run_async(100, burn_in=0, record_stride=10)
        s.sync()
        for _ in range(args.steps):
            s.run_async(100, burn_in=0, record_stride=10)
        s.sync()
        ms = np.asarray(s.kernel_times(args.steps))
        rate = W * 100 / (ms.mean() * 1e-3)
        print(f"{n}x{n}, {nsrc} sources, {W} walkers: {rate:.3e} walker-steps/s "
              f"(kernel {ms.mean():.3f} ms per 100 iterations, chunks per walker "
              f"{s.last_units()})", flush=True)
        s.close()


if __name__ == "__main__":
    main()
