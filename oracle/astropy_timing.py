"""CPU baseline of the reference's own loop cost, runnable on the GPU box (TEST /
BENCH INFRASTRUCTURE, like the rest of oracle/: only bench.py's cpu_baseline leg and
tests/ run it; the product never does).

    /opt/conda/bin/python3.9 oracle/astropy_timing.py <n> <nsrc> <seed> <iters> [--sync] [--port]
    /opt/conda/bin/python3.9 oracle/astropy_timing.py --check <fixture.npz> <walker> <iters>

The reference cannot travel to the GPU box (its sources stay in the build container),
but its arithmetic's third-party piece does: the image ships /opt/conda's python3.9
with astropy 4.3.1.  This runs oracle/olpe_oracle.py's Walker -- the line-cited
restatement of apf_step2.py:298-338 -- with ``use_astropy_models``, i.e. with every
Gaussian built as an astropy ``Gaussian2D`` object per proposal as apf_step2.py:98-102
does, and prints one JSON line {"iters", "seconds", "iters_per_s"} for the walker's
loop (the setup and the import excluded; with ``--sync`` it prints "ready" after the
warm-up and starts the loop when a line arrives on stdin, so that the processes of one
measurement run together).  ``--check`` runs the walker of a
reference-executed fixture (tests/golden/*_long.npz, produced by the reference's own
lines under the same python3.9 / numpy 1.26 / astropy 4.3.1) and compares every row.
``--port`` times the plain NumPy port instead (no astropy objects) under the same
interpreter, so that the reference-cost / port ratio bench.py reports is like for like
(the port had been timed under the bench's own python only).
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

# astropy 4.3.1 needs NumPy names removed in NumPy >= 1.25
for _name, _val in (("asscalar", lambda a: a.item()), ("alen", len),
                    ("product", np.prod), ("cumproduct", np.cumprod),
                    ("sometrue", np.any), ("alltrue", np.all)):
    if not hasattr(np, _name):
        setattr(np, _name, _val)

import warnings  # noqa: E402
warnings.filterwarnings("ignore")
from astropy.modeling import models  # noqa: E402

from oracle import olpe_oracle as ora  # noqa: E402

if "--port" not in sys.argv[1:]:
    ora.use_astropy_models(models)


def walker(image, nsrc, p0, seed):
    dm, err, _, _ = ora.noise_model(np.asarray(image, dtype=np.float32), 1.0, 1, 1, 2)
    w = ora.Walker(dm, err, p0, seed, nsrc)
    if p0[-1] == 0.0:
        w.init_chi2()
    return w


def main(argv):
    if argv[0] == "--check":
        with np.load(argv[1], allow_pickle=False) as z:
            g = {k: z[k] for k in z.files}
        wk, iters = int(argv[2]), int(argv[3])
        w = walker(g["image"], int(g["nsrc"]), g["p_init"], int(g["seeds"][wk]))
        chain, _ = w.run(iters)
        ref = g["traj_params"][wk, :iters]
        print(json.dumps({"rows": iters, "bit_equal": bool(np.array_equal(chain, ref)),
                          "max_rel": float(np.nanmax(np.abs(chain - ref) /
                                                     np.maximum(np.abs(ref), 1e-300)))}))
        return 0
    from olpefit_amd import synth
    n, nsrc, seed, iters = (int(a) for a in argv[:4])
    img, _ = synth.make_image(n, nsrc, 0)
    p0 = ora.initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    w = walker(img, nsrc, p0, seed)
    w.run(3)                                   # warm-up (astropy's first-call caches)
    if "--sync" in argv[4:]:                   # start with the other processes
        print("ready", flush=True)
        sys.stdin.readline()
    t = time.perf_counter()
    w.run(iters)
    dt = time.perf_counter() - t
    print(json.dumps({"iters": iters, "seconds": dt, "iters_per_s": iters / dt}))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
