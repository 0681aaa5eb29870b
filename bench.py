"""Benchmark: walker-steps/s of the apf_step2 Gibbs/MH hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3] [--mode exact|fast]

A bench *step* is one launch of the fused sampler kernel: every walker on the GPU
runs ``--iters`` Gibbs iterations (apf_step2.py:300-351: parameter draw, proposal,
full-image model + chi^2, accept/reject), recording its state every ``--stride``
iterations into an HBM chain buffer.  Inputs (cutout, sigma map, walker state, RNG
state) are resident in HBM before the timed region.

Workload (BASELINE.json configs[2]): 65,536 walkers per
GPU on a synthetic 64x64 two-source NIRC2 cutout, fp64, chain stride 10.  For N > 1
GPUs the driver launches one process per GPU (torch.distributed.run); walkers are
sharded with seeds 1000 + global walker index, there is no communication while
sampling, and the end-of-run RCCL all-gather of final states (outside the timed
region, reported as ``allgather_ms``) is the only exchange.  ``scaling`` is "weak".

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# BASELINE.json configs -> (walkers per GPU, image side, nsrc)
# (keys are BASELINE.json config indices; [0] is the 1-walker CPU plumbing case and
# [3] is configs[2] sharded over 8 GPUs, i.e. this bench at --gpus 8)
CONFIGS = {
    1: (4096, 64, 2),
    2: (65536, 64, 2),
    4: (16384, 128, 3),
}
CONFIG_NAMES = {
    1: "configs[1]: 4,096 walkers, 64x64 2-source cutout, fp64",
    2: "configs[2]: 65,536 walkers/GPU, 64x64 2-source cutout, fp64, LDS-resident image",
    4: "configs[4]: 3-source 128x128 cutout, 16,384 walkers/GPU, fp64",
}
FP64_LANE_PEAK = 78.6e12 / 2      # MI355X FP64 vector: 78.6 TFLOP/s with FMA = 2
EXP_OPS = 20                      # FP64 VALU ops of one ocml exp(f64)
EXP_TAB_OPS = 12                  # FP64 VALU ops of olpe::exp_tab (FAST3 setup)


def work_per_step(n: int, nsrc: int, mode: str) -> float:
    """FP64 VALU lane-ops of one walker-step's model + chi^2 evaluation.

    exact: per pixel-Gaussian 7 ops + one exp (E = 20), per pixel G-1 combines +
           background + 3 residual ops, per column-Gaussian 4 hoisted ops.
    fast:  the FAST3 sweep every guarded step of this workload takes: per pixel, with
           the four-row update, 2 sets x (5m-1)/4 (m = nsrc Gaussians per set; G
           multiplies + G-2 adds per pixel without it) + 2 fma (the two shape tables,
           background folded in) + 2 fma (residual, accumulate); column terms (2 table exps, E_TAB = 12, + 10
           ops per column) only for the Gaussians the drawn parameter changes -- 12 of
           the 16 (19) parameters change 2 (NSRC) Gaussians, the rest none -- the other
           terms are cached (the refresh after an accept is not counted); shape tables
           rebuilt for one set (one exp + 3 ops per row) on the 6 draws that change one."""
    g = 2 * nsrc
    if mode == "exact":
        return n * n * (g * (7 + EXP_OPS) + g + 3) + 4 * n * g
    np_ = 16 if nsrc == 2 else 19
    changed = (12 * 2 if nsrc == 2 else (6 * 2 + 2 * 3 + 6 * 3)) / np_
    if n > 64:                       # two column passes: no column-term cache
        changed = g
    # four-row update (n >= 64): 2 sets x (5m - 1)/4 per pixel + 4; m = nsrc Gaussians
    # per set (a 16-wave 2-source sampler, OLPE_WPB=16, uses the two-row one: (3m-1) + 4)
    if n >= 64:
        per_px = (5 * nsrc - 1) / 2 + 4
    else:
        per_px = 2 * g + 2
    return (n * n * per_px + n * changed * (2 * EXP_TAB_OPS + 10)
            + n * (EXP_TAB_OPS + 3) * 6 / np_)


def sec8d_work(n: int, nsrc: int) -> float:
    """SURVEY.md §8(d)'s exp-form count Np*(12G+8) + E*Np*G (reference formula)."""
    g = 2 * nsrc
    return n * n * (12 * g + 8) + EXP_OPS * n * n * g


# ----------------------------------------------------------------------------------
# CPU baseline (oracle, one walker per process like one MPI rank per walker)
# ----------------------------------------------------------------------------------
def _cpu_worker(args):
    n, nsrc, seed, iters = args
    from olpefit_amd import synth
    from oracle import olpe_oracle as ora
    img, _ = synth.make_image(n, nsrc, 0)
    dm, err, _, _ = ora.noise_model(img, 1.0, 1, 1, 2)
    p0 = ora.initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    w = ora.Walker(dm, err, p0, seed, nsrc)
    w.init_chi2()
    t = time.perf_counter()
    w.run(iters)
    return time.perf_counter() - t


def cpu_baseline(n: int, nsrc: int, iters: int, procs: int):
    with mp.get_context("spawn").Pool(procs) as pool:
        pool.map(_cpu_worker, [(n, nsrc, 1, 5)] * procs)          # import warm-up
        t0 = time.perf_counter()
        times = pool.map(_cpu_worker, [(n, nsrc, 1000 + i, iters) for i in range(procs)])
        wall = time.perf_counter() - t0
    steps = procs * iters
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": steps / wall, "unit": "walker-steps/s", "cores": procs, "kind": "port",
            "sample": f"oracle/olpe_oracle.py NumPy restatement, {procs} processes x 1 walker "
                      f"x {iters} iterations, {n}x{n} {nsrc}-source cutout "
                      f"({sum(times):.1f} s CPU); cpu: {cpu_model or platform.processor()}"}


def load_traffic(path: str):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


# ----------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--walkers", type=int, default=0, help="override walkers per GPU")
    ap.add_argument("--iters", type=int, default=100, help="Gibbs iterations per step")
    ap.add_argument("--stride", type=int, default=10, help="chain record stride")
    ap.add_argument("--mode", default="fast", choices=["exact", "fast"])
    ap.add_argument("--no-alt", action="store_true",
                    help="skip the single-GPU measurement of the other eval mode")
    ap.add_argument("--cpu-iters", type=int, default=None,
                    help="oracle iterations per CPU process (default: about 12-20 s of CPU "
                         "work in total: 6000 at 64x64, 6000*64^2/n^2 otherwise, at least 500)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on device 0, no RCCL "
                         "all-gather (RCCL refuses two ranks on one device)")
    args = ap.parse_args()

    from olpefit_amd import dist as odist
    rank, world, local = odist.env()
    group = odist.HostGroup(rank, world)
    barrier, allmax = group.barrier, group.allmax

    from olpefit_amd import synth
    from olpefit_amd.core import Sampler

    wpg, n, nsrc = CONFIGS[args.config]
    if args.walkers:
        wpg = args.walkers
    img, _ = synth.make_image(n, nsrc, 0)
    s = Sampler(img, 1.0, 1, 1, 2, nsrc=nsrc, device=0 if args.share_gpu else local)
    # step-1 style start (apf_step2.py:264-289) for every walker
    from olpefit_amd.pipeline import initial_parameters
    p0 = initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    p0[-1] = s.chi_squared(p0)
    s.seed(odist.walker_seeds(1000, rank * wpg, wpg))      # weak scaling: wpg per GPU
    s.set_state(np.tile(p0, (wpg, 1)))

    def measure(mode, steps, warmup):
        s.set_eval_mode(mode)
        for _ in range(warmup):
            s.run_async(args.iters, burn_in=0, record_stride=args.stride)
        s.sync()
        barrier()
        s.sync()
        t0 = time.perf_counter()
        kms = []
        for _ in range(steps):
            s.run_async(args.iters, burn_in=0, record_stride=args.stride)
            kms.append(s.last_kernel_ms())      # HIP events on the launch stream
        s.sync()
        barrier()
        t1 = time.perf_counter()
        return allmax(t1 - t0), float(np.mean(kms))

    elapsed, kernel_ms = measure(args.mode, args.steps, args.warmup)
    alt = None
    if world == 1 and not args.no_alt:
        other = "exact" if args.mode == "fast" else "fast"
        alt_steps = max(2, args.steps // 2)
        e2, k2 = measure(other, alt_steps, 1)
        alt = (other, alt_steps, e2, k2)

    # end-of-run exchange: RCCL all-gather of final walker states
    gather_ms = None
    gather_err = None
    if world > 1 and not args.share_gpu:
        # outside the timed region; an error here (reported by libolpe) is recorded in
        # the JSON line instead of losing the measurement
        try:
            uid = group.broadcast(Sampler.comm_unique_id() if rank == 0 else None)
            s.comm_init(uid, world, rank)
            barrier()
            tg = time.perf_counter()
            allst = s.allgather_state()
            gather_ms = allmax(time.perf_counter() - tg) * 1e3
            if allst.shape != (world * wpg, s.ps):
                raise RuntimeError(f"all-gather returned {allst.shape}")
        except Exception as e:          # noqa: BLE001 -- reported, not hidden
            gather_err = f"{type(e).__name__}: {e}"
            print(f"[bench rank {rank}] all-gather failed: {gather_err}", file=sys.stderr)

    if rank != 0:
        s.close()
        group.close()
        return

    total = world * wpg * args.iters * args.steps
    value = total / elapsed
    steps_per_launch = wpg * args.iters
    traffic = load_traffic(args.traffic)

    def traffic_of(mode):
        # PMC bytes per launch, measured for this config at the default launch shape
        # (walkers, iterations, stride); null for any other workload
        if args.walkers or args.iters != 100 or args.stride != 10:
            return None
        key = mode if args.config == 2 else f"c{args.config}_{mode}"
        return (traffic or {}).get(key, {}).get("bytes_per_launch")

    def roofline(mode, kernel_ms):
        # achieved = SURVEY.md §8(d)'s algorithmic work per walker-step (the exp-form
        # count, E = 20) x walker-steps per launch / HIP-event kernel time.  The FAST
        # algorithm does fewer operations than that count (no per-pixel exp), so its
        # frac can exceed 1; executed_* is the operation count the kernel really issues
        # (work_per_step) and measures how well the FP64 VALU is used.
        algo = sec8d_work(n, nsrc)
        secs = kernel_ms * 1e-3
        achieved = steps_per_launch * algo / secs / 1e12
        ops = work_per_step(n, nsrc, mode)
        executed = steps_per_launch * ops / secs / 1e12
        peak = FP64_LANE_PEAK / 1e12
        return {
            "bound": "fp64-valu",
            "achieved": achieved,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": achieved / peak,
            "traffic": traffic_of(mode),
            "kernel": "olpe_gibbs_kernel",
            "kernel_ms": kernel_ms,
            "algorithmic_work_per_walker_step": algo,
            "walker_steps_per_launch": steps_per_launch,
            "executed_work_per_walker_step": ops,
            "executed_achieved": executed,
            "executed_frac": executed / peak,
            "note": "FP64 VALU lane-ops (FMA counted once; SURVEY.md 8(d)) per second, peak "
                    "= 78.6 TFLOP/s / 2; achieved uses the 8(d) exp-form work Np(12G+8) + "
                    "E Np G, executed_* the kernel's own operation count (DESIGN.md §4); "
                    "traffic = PMC FETCH_SIZE*2 + WRITE_SIZE bytes per launch "
                    "(profiles/pmc_traffic.json)",
        }

    out = {
        "metric": "walker-steps/sec (= model evals/sec) on 64x64 2-source cutout, 1/2/4/8 GPU",
        "value": value,
        "unit": "walker-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic NIRC2-shaped cutout (olpefit_amd/synth.py), step-1 style start",
        "config": {"workload": CONFIG_NAMES[args.config], "walkers_per_gpu": wpg,
                   "image": f"{n}x{n}", "sources": nsrc, "iters_per_step": args.iters,
                   "chain_stride": args.stride, "eval": args.mode,
                   "parallelism": f"walker-sharded x{world}"},
        "roofline": roofline(args.mode, kernel_ms),
        "allgather_ms": gather_ms,
    }
    if gather_err:
        out["allgather_error"] = gather_err
    if alt:
        other, alt_steps, e2, k2 = alt
        out["alt_eval"] = {"eval": other,
                           "value": world * wpg * args.iters * alt_steps / e2,
                           "ms_per_step": e2 / alt_steps * 1e3,
                           "roofline": roofline(other, k2)}
    if not args.no_cpu_baseline and world == 1:
        procs = min(16, os.cpu_count() or 1)
        cpu_iters = args.cpu_iters or max(500, 6000 * 64 * 64 // (n * n))
        out["cpu_baseline"] = cpu_baseline(n, nsrc, cpu_iters, procs)
    print(json.dumps(out))
    s.close()
    group.close()


if __name__ == "__main__":
    main()
