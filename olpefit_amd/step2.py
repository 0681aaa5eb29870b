"""apf_step2 command line: the reference's CLI and file surface over the GPU sampler.

Reference: apf_step2.py (2 sources) and 3body/apf_step2_3body.py (3 sources).  Kept:
positional ``image``, ``-i {1,2a}`` (2-source only), the output directory
``<dir>/<frame>_apf_results/``, ``{w}_finalarray_mpi.csv`` (NaN first row, PS columns,
rows from count == burn_in, written up to the last multiple of 10) and
``{w}_acceptance_rate.csv`` per walker w (the reference's MPI rank), and the run-length
semantics: the run ends at the first iteration where some walker has tried every
parameter ``accept_min`` times (apf_step2.py:300 + the lockstep barrier at :338).

Added flags: ``--walkers`` (the reference's MPI size), ``--seed``, ``--iters`` (fixed
length instead of accept_min), ``--record-stride``, ``--gpus``, ``--exact``,
``--fixed-bkgd``, ``--chunk``, ``--no-csv``, ``--npy``.
"""
from __future__ import annotations

import argparse
import os
import sys
import threading
import time

import numpy as np

from . import fitsio, pipeline
from .core import Sampler


def parse(argv, nsrc, variant="2"):
    prog = {"2": "apf_step2", "2a": "apf_step2a"}[variant] + ("" if nsrc == 2 else "_3body")
    ap = argparse.ArgumentParser(prog=prog)
    ap.add_argument("image", type=str)
    if variant == "2a":
        # apf_step2a.py: one walker, n_steps = 5000 (:39), no MPI, writes step2a.csv
        ap.set_defaults(walkers=1, iters=5000, burn_in=0, accept_min=0, initial_guess_option="1")
    if nsrc == 2 and variant == "2":
        ap.add_argument("-i", "--initial_guess_option", type=str,
                        help="-i 1 for the step 1 guess, -i 2a for the step 2a output")
    ap.add_argument("--walkers", type=int, default=24 if variant == "2" else 1,
                    help="independent walkers (the reference's MPI processes)")
    ap.add_argument("--accept-min", type=int, default=100000,
                    help="stop when a walker has tried every parameter this often")
    ap.add_argument("--burn-in", type=int,
                    default=6000 if (nsrc == 2 and variant == "2") else 0)
    ap.add_argument("--iters", type=int, default=0 if variant == "2" else 5000,
                    help="run exactly this many iterations (overrides --accept-min; use a "
                         "multiple of 10 to mirror the reference's write cadence)")
    ap.add_argument("--seed", type=int, default=None,
                    help="walker w uses np.random.seed(seed + w) (default: OS entropy)")
    ap.add_argument("--record-stride", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--device", type=int, default=0, help="first HIP device")
    ap.add_argument("--exact", action="store_true", help="exact per-pixel exp evaluation")
    ap.add_argument("--fixed-bkgd", action="store_true",
                    help="background = p[9] instead of the reference's p[12] (2-source)")
    ap.add_argument("--chunk", type=int, default=20000, help="iterations per kernel launch")
    ap.add_argument("--no-csv", action="store_true")
    ap.add_argument("--npy", action="store_true", help="also write {w}_chain.npy")
    ap.add_argument("-q", "--quiet", action="store_true")
    return ap.parse_args(argv)


class Shard:
    """The walkers [w0, w0 + W) on one GPU."""

    def __init__(self, img, hdr, nsrc, device, w0, W, p0, seeds, exact, bkgd_mode):
        self.s = Sampler(img, hdr["ITIME"], hdr["COADDS"], hdr["MULTISAM"], hdr["SAMPMODE"],
                         nsrc=nsrc, bkgd_mode=bkgd_mode, device=device)
        self.s.set_eval_mode("exact" if exact else "fast")
        self.w0, self.W = w0, W
        p = p0.copy()
        with np.errstate(all="ignore"):
            p[-1] = self.s.chi_squared(p)                       # apf_step2.py:283-289
        self.p_init = p
        self.s.seed(seeds[w0:w0 + W])
        self.s.set_state(np.tile(p, (W, 1)))
        self.chunks = []

    def snapshot(self):
        return self.s.get_state(), self.s.rng_state(), self.s.count

    def restore(self, snap):
        (st, t, a), (mt, g), count = snap
        self.s.set_state(st, t, a)
        self.s.set_rng_state(mt, g)
        self.s.reset_count(count)

    def run(self, n, burn_in, stride, accept_min):
        chain = self.s.run(n, burn_in=burn_in, record_stride=stride, accept_min=accept_min)
        self.chunks.append(chain if chain is not None else np.zeros((self.W, 0, self.s.ps)))

    def chain(self):
        if not self.chunks:
            return np.zeros((self.W, 0, self.s.ps))
        return np.concatenate(self.chunks, axis=1)


def _parallel(shards, fn):
    errs = []

    def body(sh):
        try:
            fn(sh)
        except BaseException as e:      # re-raised in the caller
            errs.append(e)
    ts = [threading.Thread(target=body, args=(sh,)) for sh in shards]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def main(argv=None, nsrc=2, variant="2"):
    """variant "2": apf_step2 (many walkers, {w}_finalarray_mpi.csv); "2a": the single
    walker warm-up of apf_step2a.py writing step2a.csv / step2a_acceptance_rate
    (:324-331), which ``apf_step2.py -i 2a`` then starts from (apf_step2.py:248-256)."""
    args = parse(sys.argv[1:] if argv is None else argv, nsrc, variant)
    say = (lambda *a: None) if args.quiet else print
    image, hdr = fitsio.getdata_header(args.image)              # apf_step2.py:160-161
    directory, frame, outdir = pipeline.image_paths(args.image)  # :164-170
    say(outdir)
    os.makedirs(outdir, exist_ok=True)                           # :172-173
    if getattr(args, "initial_guess_option", None) == "2a":      # :248-256
        say("I am taking the initial guess from Step 2a output")
        p0 = pipeline.read_step2a(outdir + "step2a.csv")
    else:
        say("I am taking the initial guess from Step 1 output")
        guess = pipeline.read_guess(directory + frame + "_initialguess")
        p0 = pipeline.initial_parameters(image, guess, nsrc)
    W = args.walkers
    base = args.seed if args.seed is not None else int.from_bytes(os.urandom(4), "little")
    seeds = (base + np.arange(W, dtype=np.int64)) & 0xFFFFFFFF
    say(f"walkers {W}, seeds {base}..{base + W - 1} (np.random.seed semantics)")
    ng = max(1, min(args.gpus, W))
    bounds = [(g * W) // ng for g in range(ng + 1)]
    shards = [Shard(image, hdr, nsrc, args.device + g, bounds[g], bounds[g + 1] - bounds[g], p0,
                    seeds, args.exact, 1 if args.fixed_bkgd else 0) for g in range(ng)]
    say("Found initial chi-squared:", shards[0].p_init[-1])
    say("Initial guess:", shards[0].p_init)

    burn, stride = args.burn_in, args.record_stride
    t0 = time.perf_counter()
    if args.iters:
        total = args.iters
        done = 0
        while done < total:
            n = min(args.chunk, total - done)
            _parallel(shards, lambda sh: sh.run(n, burn, stride, 0))
            done += n
            say("Loop count:", done)
        stop = total
    else:
        # accept_min semantics: the run ends at the first count C where some walker has
        # min(total_tries) >= accept_min (apf_step2.py:300); with the lockstep barrier
        # every file then holds rows up to L = the last multiple of 10 <= C (:355).
        # Chunks start at multiples of 10, so L lies inside the chunk that found C: that
        # chunk is re-run from its snapshot (RNG included, hence identical) up to L.
        chunk = ((args.chunk + 9) // 10) * 10
        done = 0
        stop = None
        while stop is None:
            snaps = [sh.snapshot() for sh in shards]
            _parallel(shards, lambda sh: sh.run(chunk, burn, stride, args.accept_min))
            done += chunk
            hits = np.concatenate([sh.s.done_at() for sh in shards])
            hits = hits[hits >= 0]
            say("Loop count:", done)
            if hits.size:
                stop = (int(hits.min()) // 10) * 10
                for sh, sn in zip(shards, snaps):
                    sh.chunks.pop()
                    sh.restore(sn)
                rest = stop - (done - chunk)
                if rest > 0:
                    _parallel(shards, lambda sh: sh.run(rest, burn, stride, 0))
    # files (apf_step2.py:355-365): NaN first row + the recorded rows, acceptance =
    # str(total_accept / total_tries) at the final count
    for sh in shards:
        chain = sh.chain()
        _, tries, acc = sh.s.get_state()
        if not args.no_csv:
            names = [(f"{sh.w0 + k}_finalarray_mpi.csv", f"{sh.w0 + k}_acceptance_rate.csv")
                     if variant == "2" else ("step2a.csv", "step2a_acceptance_rate")
                     for k in range(sh.W)]
            # chain files: native formatter + writer threads (libolpe olpe_csv_*)
            # (step 2a names one file for every walker: written in order, the last wins)
            pipeline.write_chain_csvs([outdir + c for c, _ in names],
                                      chain.reshape(sh.W, -1, chain.shape[-1]),
                                      threads=0 if variant == "2" else 1)
            for k, (_, acc_name) in enumerate(names):
                pipeline.write_acceptance(outdir + acc_name, acc[k], tries[k])
        if args.npy:
            for k in range(sh.W):
                np.save(outdir + f"{sh.w0 + k}_chain.npy", chain[k])
    say("done with loop")
    return outdir
