"""Dump sampler states of one shape (diagnostics): n nsrc walkers iters stride -> npy."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from olpefit_amd import synth  # noqa: E402
from olpefit_amd.core import Sampler  # noqa: E402
from olpefit_amd.pipeline import initial_parameters  # noqa: E402

n, nsrc, W, it, stride = (int(v) for v in sys.argv[1:6])
img, _ = synth.make_image(n, nsrc, 0)
s = Sampler(img, 1.0, 1, 1, 2, nsrc=nsrc)
p0 = initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
p0[-1] = s.chi_squared(p0)
s.seed(1000 + np.arange(W))
s.set_state(np.tile(p0, (W, 1)))
chain = s.run(it, burn_in=0, record_stride=stride)
np.save(sys.argv[6], chain.astype(np.float64))
print("saved", chain.shape)
