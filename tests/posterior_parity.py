"""Posterior-level parity on the bench workload (BASELINE.json north star: posterior
means / sigmas of the GPU chains against the NumPy reference on identical seeds).

    python tools/posterior_parity.py [--walkers 16] [--iters 2000] [--burn 500] [--mode fast]
                                     [--config 2|4]

Runs W walkers (seeds 1000 + w, the bench's step-1 style start) on the synthetic 64x64
two-source cutout (--config 4: the 128x128 three-source one, on the lockstep ring
sampler) through libolpe, and the same walkers through the oracle
(oracle/olpe_oracle.py, one process per walker), then prints per-parameter posterior
mean and sigma of the pooled chains, their differences, and the truth the frame was
rendered from.  The oracle is the checker here, never the thing measured.
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

NAMES = ["xcs", "ycs", "xcc", "ycc", "dx", "dy", "amps", "ampc", "ratio", "bkgd",
         "sx", "sy", "sx2", "sy2", "th", "th2"]
# 3-source layout (3body/apf_step2_3body.py:266-288)
NAMES3 = ["x1", "y1", "x2", "y2", "x3", "y3", "dx", "dy", "amp1", "amp2", "amp3", "ratio",
          "bkgd", "sx", "sy", "sx2", "sy2", "th", "th2"]


def _setup(n, nsrc):
    from olpefit_amd import synth
    from olpefit_amd.pipeline import initial_parameters
    from oracle import olpe_oracle as ora
    img, _ = synth.make_image(n, nsrc, 0)
    dm, err, _, _ = ora.noise_model(img, 1.0, 1, 1, 2)
    p0 = initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    with np.errstate(all="ignore"):
        p0[-1] = float(ora.chi_squared(dm, ora.build_analytical_model(p0, n, nsrc), err))
    return img, dm, err, p0


def _oracle_walker(args):
    n, nsrc, seed, iters, burn = args
    from oracle import olpe_oracle as ora
    _, dm, err, p0 = _setup(n, nsrc)
    chain, _ = ora.Walker(dm, err, p0, seed, nsrc=nsrc).run(iters, burn_in=burn)
    return chain


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--walkers", type=int, default=16)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--burn", type=int, default=500)
    ap.add_argument("--mode", default="fast", choices=["fast", "exact"])
    ap.add_argument("--config", type=int, default=2, choices=[2, 4])
    args = ap.parse_args()
    n, nsrc = (64, 2) if args.config == 2 else (128, 3)
    names = NAMES if nsrc == 2 else NAMES3
    npar = len(names)
    from olpefit_amd import synth
    from olpefit_amd.core import Sampler
    img, dm, err, p0 = _setup(n, nsrc)
    seeds = 1000 + np.arange(args.walkers)
    s = Sampler(img, 1.0, 1, 1, 2, nsrc=nsrc)
    s.set_eval_mode(args.mode)
    s.seed(seeds)
    s.set_state(np.tile(p0, (args.walkers, 1)))
    gpu = s.run(args.iters, burn_in=args.burn, record_stride=1)
    s.moments_accumulate()
    from olpefit_amd import step3
    summ = step3.summary_from_moments(s.allreduce_moments(), nsrc)
    with mp.get_context("spawn").Pool(min(16, args.walkers)) as pool:
        ref = np.stack(pool.map(_oracle_walker, [(n, nsrc, int(sd), args.iters, args.burn)
                                                 for sd in seeds]))
    assert gpu.shape == ref.shape, (gpu.shape, ref.shape)
    g = gpu.reshape(-1, gpu.shape[-1])[:, :npar]
    r = ref.reshape(-1, ref.shape[-1])[:, :npar]
    truth = synth.truth_params(n, nsrc)
    print(f"{args.walkers} walkers x {args.iters} iterations (burn-in {args.burn}), "
          f"{args.mode} evaluation, {n}x{n} {nsrc}-source synthetic cutout; "
          f"{g.shape[0]} pooled samples")
    print(f"{'param':>6} {'truth':>12} {'mean gpu':>16} {'mean ref':>16} {'|dmean|':>9} "
          f"{'sigma gpu':>12} {'|dsigma|/sigma':>14}")
    worst = 0.0
    for k, name in enumerate(names):
        mg, mr = g[:, k].mean(), r[:, k].mean()
        sg, sr = g[:, k].std(), r[:, k].std()
        ds = abs(sg - sr) / sr if sr > 0 else abs(sg - sr)
        worst = max(worst, abs(mg - mr) / max(abs(mr), 1e-300))
        print(f"{name:>6} {truth[k]:12.6g} {mg:16.10g} {mr:16.10g} {abs(mg - mr):9.2e} "
              f"{sg:12.6g} {ds:14.2e}")
    # step 3's statistics from the device moments (posterior_summary.json's numbers)
    # against step 3's arithmetic over the oracle's chains
    rs = step3.summary(ref.transpose(1, 0, 2), nsrc)
    keys = list(rs)
    dm = max(abs(summ[k]["mean"] - rs[k]["mean"]) / max(abs(rs[k]["mean"]), 1e-300) for k in keys)
    dsd = max(abs(summ[k]["std"] - rs[k]["std"]) / max(rs[k]["std"], 1e-300) for k in keys)
    dgr = max(abs(summ[k]["gr_rc"] - rs[k]["gr_rc"]) / rs[k]["gr_rc"] for k in keys)
    dc = max(abs(summ[k]["mean"] - rs[k]["mean"]) for k in keys[:2 * nsrc])
    print(f"device-moment summary vs step3.summary of the oracle chains: max relative "
          f"|dmean| {dm:.2e}, |dsigma| {dsd:.2e}, |dGR RC| {dgr:.2e}; centroid |dmean| "
          f"{dc:.2e} px")
    same = np.mean(np.isclose(gpu, ref, rtol=1e-8, atol=1e-9))
    print(f"max relative |dmean| {worst:.2e}; centroid |dmean| (px) "
          f"{max(abs(g[:, k].mean() - r[:, k].mean()) for k in range(2 * nsrc)):.2e}; "
          f"chain entries equal to rtol 1e-8: {same * 100:.4f} %")


if __name__ == "__main__":
    main()
