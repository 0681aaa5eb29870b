"""Benchmark: walker-steps/s of the apf_step2 Gibbs/MH hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 0-4] [--mode exact|fast]

A bench *step* is one launch of the fused sampler kernel: every walker on the GPU
runs ``--iters`` Gibbs iterations (apf_step2.py:300-351: parameter draw, proposal,
full-image model + chi^2, accept/reject), recording its state every ``--stride``
iterations into an HBM chain buffer.  Inputs (cutout, sigma map, walker state, RNG
state) are resident in HBM before the timed region.

Workload (BASELINE.json configs[2]): 65,536 walkers per
GPU on a synthetic 64x64 two-source NIRC2 cutout, fp64, 20 launches of 100 iterations
at chain stride 10 (``--config 0 / 1 / 3 / 4``: the other configs at their §8(d) runs,
``DEFAULTS``).  N > 1 GPUs run one process per GPU: ``--gpus N`` starts the N ranks
itself when no launcher did (``launch_ranks``), or takes them from torchrun / mpirun
(``WORLD_SIZE`` must equal N).  Walkers are sharded with seeds 1000 + global walker
index, there is no communication while sampling, and the end-of-run RCCL exchange
(outside the timed region) is the only one: all-gather of the final states
(``allgather_ms``) and the chain concatenation (all-gather of the last launch's chain
rows over xGMI, in walker ranges that bound the receive buffer: ``chain_gather_ms`` /
``_bytes`` / ``_gbs``).  ``scaling`` is "weak".  The host group (barrier,
max-over-ranks time, RCCL id) is stdlib TCP, no PyTorch.

Roofline: the kernel is FP64-VALU bound.  ``roofline.frac`` = executed
FP64 VALU lane-ops per second / 39.3e12 (78.6 TFLOP/s with FMA = 2), the executed
count per walker-step read from the rocprofv3 SQ counters of this config
(profiles/valu_counts.json, tools/pmc_valu.sh) times the live HIP-event rate;
``valu_issue_frac`` does the same with all VALU instructions.  The HBM figures use the
PMC FETCH/WRITE bytes per launch (profiles/pmc_traffic.json).

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import platform
import signal
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# BASELINE.json configs -> (walkers per GPU, image side, nsrc)
# (keys are BASELINE.json config indices; [3] is configs[2] sharded over 8 GPUs, i.e.
# this bench at --gpus 8)
CONFIGS = {
    0: (1, 32, 2),
    1: (4096, 64, 2),
    2: (65536, 64, 2),
    4: (16384, 128, 3),
}
CONFIGS[3] = CONFIGS[2]               # configs[3] = configs[2]'s 65,536 walkers on each of 8 GPUs
CONFIG_NAMES = {
    0: "configs[0]: 1 walker, 32x32 2-source cutout, 1,000 iterations (plumbing reference)",
    1: "configs[1]: 4,096 walkers, 64x64 2-source cutout, fp64",
    2: "configs[2]: 65,536 walkers/GPU, 64x64 2-source cutout, fp64, LDS-resident image",
    # (BASELINE configs[4] is 131,072 walkers on 8 GPUs: one GPU runs one shard of it)
    4: ("configs[4]'s per-GPU shard on 1 GPU (16,384 of 131,072 walkers, 3-source 128x128 "
        "cutout, fp64; the whole of configs[4] is --gpus 8)"),
}
CONFIG3 = ("configs[3]: 524,288 walkers sharded 8 x MI355X (65,536 per GPU, 64x64 2-source "
           "cutout, fp64), RCCL chain all-gather at the end")
CONFIG4 = ("configs[4]: 131,072 walkers sharded 8 x MI355X (16,384 per GPU, 3-source 128x128 "
           "cutout, fp64), RCCL chain all-gather at the end")


def workload_name(config: int, world: int, wpg: int, n: int | None = None,
                  nsrc: int | None = None, iters: int | None = None,
                  stride: int | None = None, steps: int | None = None) -> str:
    """The line's ``config.workload``, derived from what actually ran: a BASELINE config
    is named only when (walkers per GPU, side, sources) are that config's SURVEY 8(d)
    shape -- configs[2]'s per-GPU shape at 8 ranks is configs[3], on 2 / 4 ranks its weak
    scaling -- and anything else is ``custom: ...`` with its sizes.  A run whose
    iterations per launch, stride or timed launches differ from the config's 8(d) run
    (DEFAULTS) says so after the name."""
    n = CONFIGS[config][1] if n is None else n
    nsrc = CONFIGS[config][2] if nsrc is None else nsrc
    gpus = f"{world} GPU{'s' if world > 1 else ''}"
    shape = (wpg, n, nsrc)
    if shape != CONFIGS[config]:
        name = (f"custom: {world} x {wpg:,} walkers ({wpg:,} per GPU on {gpus}), {n}x{n} "
                f"{nsrc}-source cutout, fp64 (not a BASELINE config's shape; --config "
                f"{config} sizes {CONFIGS[config][0]:,} walkers, {CONFIGS[config][1]}x"
                f"{CONFIGS[config][1]}, {CONFIGS[config][2]} sources)")
    elif config in (2, 3) and world == 8:
        name = CONFIG3
    elif config == 4 and world == 8:
        name = CONFIG4
    elif config == 3:
        name = (f"configs[3]'s per-GPU shards on {gpus} ({world} x {wpg:,} of 524,288 "
                f"walkers; the whole of configs[3] is --gpus 8)")
    elif world > 1:
        name = (f"configs[{config}]'s shape per GPU, weak-scaled over "
                f"{gpus} ({world} x {wpg:,} walkers, {n}x{n} {nsrc}-source cutout, fp64"
                + ("; configs[3] is 8 x 65,536)" if config == 2 else
                   "; configs[4] is 8 x 16,384)" if config == 4 else ")"))
    else:
        name = CONFIG_NAMES[config]
    d = DEFAULTS[config]
    run = dict(iters=iters, stride=stride, steps=steps)
    if any(v is not None and v != d[k] for k, v in run.items()):
        name += (f" [run: {steps if steps is not None else d['steps']} launches x "
                 f"{iters if iters is not None else d['iters']} iterations at stride "
                 f"{stride if stride is not None else d['stride']}; 8(d)'s run: {d['steps']} x "
                 f"{d['iters']} at stride {d['stride']}]")
    return name


# SURVEY.md 8(d)'s run of each config: iterations per launch (a bench step), chain record
# stride ("every step for configs 1-2 and with stride 10 otherwise"), timed steps and
# warm-up steps, so that the timed steps cover the config's iteration count: configs[0]
# 1,000 iterations, configs[1] 10,000, configs[2] 2,000, configs[4] 500
DEFAULTS = {
    0: dict(iters=1000, stride=1, steps=1, warmup=1),
    1: dict(iters=1000, stride=1, steps=10, warmup=60),
    2: dict(iters=100, stride=10, steps=20, warmup=40),
    4: dict(iters=100, stride=10, steps=5, warmup=35),
}
# (warm-up: ~0.5 s of launches before the timed ones.  Same-box A/B, round 5
# (profiles/r05/warmup/): the timed launches run at the same speed after 2-5 warm-up
# launches as after 0.5 s, but the power controller's telemetry (SmiClock, the line's
# clock) still reads low within ~0.3 s of a run's first launch -- configs[1] 1.64-1.70
# GHz after 2 where 0.5 s of warm-up reads 2.07 -- so the clock is read after it settles)
DEFAULTS[3] = DEFAULTS[2]
# seconds after a rank's first launch before its SMU clock reading counts as settled
CLOCK_SETTLE_S = 0.3
# BASELINE.json's metric, character for character (its "64\u00d764")
METRIC = "walker-steps/sec (= model evals/sec) on 64\u00d764 2-source cutout, 1/2/4/8 GPU"
FP64_LANE_PEAK = 78.6e12 / 2      # MI355X FP64 vector: 78.6 TFLOP/s with FMA = 2
HBM_PEAK = 8.0e12                 # MI355X HBM3E spec (MI355X_MICROARCH.md)
# one exp of the EXACT sweep (olpe::exp_neg, ocml's sequence without its range selects):
EXP_OPS = 16                      # FP64 VALU instructions, ISA count (mul, rint, 2 + 11 fma,
                                  # ldexp): SURVEY.md 8(d)'s E
EXP_LANE_OPS = 14                 # of them in the SQ FP64 classes (FMA/MUL/ADD; rint and
                                  # ldexp are not): the operation count stays a lower bound
EXP_TAB_OPS = 12                  # FP64 VALU ops of olpe::exp_tab (FAST3 setup)


def work_per_step(n: int, nsrc: int, mode: str) -> float:
    """FP64 VALU lane-ops of one walker-step's model + chi^2 evaluation.

    exact: per pixel-Gaussian 7 ops + one exp (14 counted ops), per pixel G-1 combines +
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
        return n * n * (g * (7 + EXP_LANE_OPS) + g + 3) + 4 * n * g
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


def mt_words_per_step(nsrc: int) -> float:
    """MT19937 words one Gibbs iteration draws: randint(0, P) (one
    word for P = 16; masked rejection, 32/19 words on average, for P = 19), the
    proposal's gauss() (polar method: 4 words per attempt, accepted with probability
    pi/4, two deviates per acceptance: 8/pi words per deviate) and accept_reject's
    rand() (2 words)."""
    return (1.0 if nsrc == 2 else 32.0 / 19.0) + 8.0 / np.pi + 2.0


def algorithmic_bytes(W: int, nrec: int, iters: int, nsrc: int) -> dict:
    """HBM bytes one sampler launch must move: the recorded chain rows,
    every walker's state, counters and RNG scalars in and out, and the MT19937 state
    advance -- each drawn word retires one key word, read and rewritten once per 624
    draws (8 B per word)."""
    ps = 17 if nsrc == 2 else 20
    np_ = ps - 1
    parts = {"chain_rows": W * nrec * ps * 8,
             "state_counters_in_out": W * 2 * (ps * 8 + 2 * np_ * 4 + 24),
             "mt_state_advance": W * iters * mt_words_per_step(nsrc) * 8}
    parts["total"] = sum(parts.values())
    return parts


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


def host_cpus():
    """(cores usable by this process, CPUs in its affinity mask, cgroup CPU quota or
    None, model name).  On the GPU box the affinity mask shows the whole machine
    while the job's cgroup quota grants a share of it; more processes than the
    quota only time-slice."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return cores, aff, quota, model or platform.processor()


def cpu_baseline(n: int, nsrc: int, total_iters: int, procs: int | None = None):
    """The oracle (one walker per process, like one MPI rank per walker) on every core
    this job may use (or ``procs`` processes), ``total_iters`` walker-steps in all (about
    12 s of CPU work)."""
    cores, aff, quota, model = host_cpus()
    procs = procs or cores
    iters = max(200, total_iters // procs)
    with mp.get_context("spawn").Pool(procs) as pool:
        pool.map(_cpu_worker, [(n, nsrc, 1, 5)] * procs)          # import warm-up
        t0 = time.perf_counter()
        times = pool.map(_cpu_worker, [(n, nsrc, 1000 + i, iters) for i in range(procs)])
        wall = time.perf_counter() - t0
    steps = procs * iters
    return {"value": steps / wall, "unit": "walker-steps/s", "cores": procs, "kind": "port",
            "affinity_cpus": aff, "cgroup_cpu_quota": quota, "cpu_model": model,
            "sample": f"oracle/olpe_oracle.py NumPy restatement, {procs} processes ("
                      f"{'one per usable core' if procs == cores else 'of the usable cores'}: "
                      f"affinity {aff} CPUs, cgroup quota "
                      f"{'none' if quota is None else f'{quota:g}'}) x 1 walker x {iters} "
                      f"iterations, {n}x{n} {nsrc}-source cutout ({sum(times):.1f} s CPU); "
                      f"cpu: {model}"}


CONDA_PY = "/opt/conda/bin/python3.9"       # the image's python with astropy 4.3.1


def reference_like_baseline(n: int, nsrc: int, total_iters: int, procs: int | None = None,
                            port: bool = False):
    """The reference's own loop cost on this box's cores: ``procs`` processes of
    oracle/astropy_timing.py (the oracle's walker with every Gaussian built as an
    astropy ``Gaussian2D`` object per proposal, as apf_step2.py:98-102 does; its chains
    are bit-equal to the reference's own, tests/test_oracle_golden.py), started
    together after their imports, ``total_iters`` walker-steps in all.  ``port``: the
    plain NumPy port under the same python3.9 instead (the like-for-like denominator of
    the reference-cost ratio).  None when the image's python3.9 / astropy is missing."""
    import subprocess
    if not os.path.exists(CONDA_PY):
        return None
    cores, aff, quota, model = host_cpus()
    procs = procs or cores
    iters = max(100, total_iters // procs)
    script = os.path.join(REPO, "oracle", "astropy_timing.py")
    ps = [subprocess.Popen([CONDA_PY, script, str(n), str(nsrc), str(1000 + i), str(iters),
                            "--sync"] + (["--port"] if port else []), stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                           stderr=subprocess.DEVNULL, text=True) for i in range(procs)]
    res = []
    try:
        # every process imported astropy and warmed up: start their loops together
        # (a process that does not get there within 180 s voids the measurement)
        import select
        deadline = time.monotonic() + 180.0
        for p in ps:
            if not select.select([p.stdout], [], [], max(0.0, deadline - time.monotonic()))[0]:
                return None
            if p.stdout.readline().strip() != "ready":
                return None
        for p in ps:
            p.stdin.write("go\n")
            p.stdin.flush()
        for p in ps:
            out, _ = p.communicate(timeout=600)
            if p.returncode != 0:
                return None
            res.append(json.loads(out.strip().splitlines()[-1]))
    except (subprocess.TimeoutExpired, OSError, ValueError, IndexError):
        return None              # no reference-cost figure rather than no bench line
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
                p.wait()
    secs = max(r["seconds"] for r in res)
    if port:
        return {"value": procs * iters / secs, "unit": "walker-steps/s", "cores": procs,
                "kind": "port (NumPy, under the astropy baseline's interpreter)",
                "sample": f"oracle/astropy_timing.py --port under {CONDA_PY}: {procs} processes "
                          f"x 1 walker x {iters} iterations, {n}x{n} {nsrc}-source cutout"}
    return {"value": procs * iters / secs, "unit": "walker-steps/s", "cores": procs,
            "kind": "port (astropy Gaussian2D objects per proposal, as the reference)",
            "sample": f"oracle/astropy_timing.py under {CONDA_PY} (astropy 4.3.1): {procs} "
                      f"processes started together x 1 walker x {iters} iterations, {n}x{n} "
                      f"{nsrc}-source cutout ({sum(r['seconds'] for r in res):.1f} s CPU); "
                      f"cpu: {model}",
            "pinned": "chains bit-equal to the reference's own loop "
                      "(tests/test_oracle_golden.py::test_astropy_oracle_is_the_reference)"}


def csv_emission(s, nw: int, threads: int) -> dict:
    """Write the last launch's chain rows of walkers [0, nw) as ``{w}_finalarray_mpi.csv``
    (the all-NaN seed row, then the rows; csv.writer's bytes, apf_step2.py:342-360)
    into a temporary directory with the native threaded writer; returns the time."""
    import shutil
    import tempfile
    from olpefit_amd import pipeline
    rows = s.chain()[:nw]
    d = tempfile.mkdtemp(prefix="olpe_csv_")
    try:
        paths = [os.path.join(d, f"{w}_finalarray_mpi.csv") for w in range(nw)]
        t = time.perf_counter()
        pipeline.write_chain_csvs(paths, rows, nan_row=True, threads=threads)
        dt = time.perf_counter() - t
        nbytes = sum(os.path.getsize(p) for p in paths)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"files": nw, "rows_per_file": int(rows.shape[1]) + 1, "bytes": nbytes,
            "ms": dt * 1e3, "mb_per_s": nbytes / dt / 1e6, "threads": threads,
            "note": "outside the timed region (SURVEY.md 8(d)); the native csv.writer-exact "
                    "writer (olpe_csv_write_chains), files created in a temporary directory"}


def reference_ratio(n: int, nsrc: int, path: str):
    """The reference's own apf_step2 loop against the port on one core of the build
    container (tests/golden/time_reference.py --json; the reference cannot travel to the
    GPU box): ``reference_over_port`` = the reference's iterations/s / the port's (< 1:
    the reference is slower).  None without a timing for this shape."""
    data = load_json(path) or {}
    ent = data.get(f"{n}x{n}_{nsrc}")
    if not ent:
        return None
    return {"reference_over_port": ent["reference_over_port"],
            "reference_iters_per_s_one_core": ent["reference_iters_per_s"],
            "port_iters_per_s_one_core": ent["port_iters_per_s"],
            "timing_cpu": ent["cpu_model"], "timing_iterations": ent["iterations"],
            "timing_file": os.path.relpath(path, REPO)}


# stdout carries exactly one line, the JSON: RCCL prints its banner ("RCCL version ...")
# to stdout when a communicator is created, so the exchange runs with fd 1 pointed at
# stderr (``_quiet_stdout``) and fd 1 is restored before anything is printed
_SAVED_STDOUT = None


def _quiet_stdout():
    global _SAVED_STDOUT
    sys.stdout.flush()
    _libc_fflush()
    _SAVED_STDOUT = os.dup(1)
    os.dup2(2, 1)


def _libc_fflush():
    # C stdio buffers what the library printed (RCCL's banner goes through printf): flush
    # it while fd 1 still points at stderr
    try:
        import ctypes
        ctypes.CDLL(None).fflush(None)
    except (OSError, AttributeError):
        pass


def _restore_stdout():
    global _SAVED_STDOUT
    fd, _SAVED_STDOUT = _SAVED_STDOUT, None
    if fd is not None:
        _libc_fflush()
        os.dup2(fd, 1)
        os.close(fd)


def _comm_timeout(rank: int, make_report, timeout: float):
    """Watchdog of the end-of-run RCCL exchange: rank 0 prints the measurement with the
    error, then every rank leaves with status 3 (os._exit: the hung collective never
    returns; the launcher and CI see the failure, the JSON line keeps the numbers)."""
    print(f"[bench rank {rank}] RCCL exchange still running after {timeout:g} s: giving up",
          file=sys.stderr)
    _restore_stdout()
    if rank == 0:
        out = make_report()
        out["comm_error"] = f"TimeoutError: RCCL exchange did not finish within {timeout:g} s"
        print(json.dumps(out), flush=True)
    sys.stderr.flush()
    os._exit(3)


def fault_drill(s, rank: int, world: int, barrier, group) -> dict:
    """After the exchange, on the real communicator: one rank's step of the moments
    all-reduce is made to fail (olpe_moments_fault, include/olpe_test.h) and every rank
    calls it -- every rank must return an error and none may wait (olpe_comm_proto.h); once
    cleared, the next call must give every rank the summary it had before.  Two cases:
    the last rank's uniformity words never reach its device (3: it sends the poisoned
    default), and rank 0's round-1 sums never come back (4: it enters round 2 as failed).
    The multi-rank counterpart of tests/test_comm_protocol.py (verdict r05 item 1, ADVICE
    r05); it runs outside the timed region."""
    ref = s.allreduce_moments()
    barrier()
    cases = []
    t0 = time.perf_counter()
    for where, who in ((3, world - 1), (4, 0)):
        if rank == who:
            s.moments_fault(where)
        barrier()
        try:
            s.allreduce_moments()
            code = 0
        except Exception as e:          # noqa: BLE001 -- the error is the expected outcome
            code = int(getattr(e, "code", -99))
        barrier()
        if rank == who:
            s.moments_fault(0)
        barrier()
        after = s.allreduce_moments()
        same = bool(np.allclose(after, ref, rtol=1e-12, atol=0.0))
        views = group.allgather([code, same])
        cases.append({"fault": where, "rank": who, "codes": [v[0] for v in views],
                      "recovered": all(v[1] for v in views)})
    return {"cases": cases, "ms": (time.perf_counter() - t0) * 1e3,
            "ok": all(all(c != 0 for c in k["codes"]) and k["recovered"] for k in cases),
            "note": "codes per rank: -2 = this rank's forced step (OLPE_EHIP), -5 = failed "
                    "on another rank (OLPE_ECOMM); every rank must report one and then "
                    "recover the same summary"}


def load_json(path: str):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


class SmiClock:
    """The GFX clock the power controller reports for one GPU -- ROCm's amdsmi package
    (``current_gfxclks``: MHz per XCD, the SMU's metrics table) -- sampled every
    ``period`` s from a host thread between start() and stop().  It reads the driver's
    metrics only (no GPU queue, no kernel).  The chip holds its FP64 load below the 2.4 GHz
    spec clock by an amount that differs from box to box; a probe kernel
    queued after the launches reads the boost clock the idle chip jumps back to within
    tens of microseconds, so the clock is sampled while they run."""
    AMDSMI = "/opt/rocm/share/amd_smi"

    def __init__(self, pci: str, period: float = 0.01):
        import threading
        if self.AMDSMI not in sys.path and os.path.isdir(self.AMDSMI):
            sys.path.append(self.AMDSMI)
        import amdsmi
        amdsmi.amdsmi_init()
        self._smi = amdsmi
        self._h = next(h for h in amdsmi.amdsmi_get_processor_handles()
                       if amdsmi.amdsmi_get_gpu_device_bdf(h).lower() == pci.lower())
        self._read()                                 # fails here if the table is unreadable
        self.period = period
        self._samples, self._stop, self._th = [], threading.Event(), None

    def _read(self) -> float:
        m = self._smi.amdsmi_get_gpu_metrics_info(self._h)
        v = [x for x in (m.get("current_gfxclks") or [])
             if isinstance(x, (int, float)) and 0 < x < 10000]
        if not v and isinstance(m.get("current_gfxclk"), (int, float)):
            v = [m["current_gfxclk"]]
        if not v:
            raise RuntimeError("no GFX clock in the metrics table")
        return sum(v) / len(v) / 1e3                 # GHz, mean over the XCDs

    def start(self):
        import threading
        self._samples, self._stop = [], threading.Event()

        def run():
            while not self._stop.is_set():
                try:
                    self._samples.append(self._read())
                except Exception:                    # noqa: BLE001 -- a sample lost
                    pass
                self._stop.wait(self.period)
        self._th = threading.Thread(target=run, daemon=True)
        self._th.start()

    def stop(self):
        """(mean GHz over the samples, number of samples); (None, 0) if there were none."""
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=5)
        n = len(self._samples)
        return (sum(self._samples) / n if n else None), n


def clock_meter(sampler_cls, pci: str):
    """The clock sampler of this rank's GPU, or None where the metrics are not readable
    (no amdsmi, no GPU: the line then carries no live clock).  A stand-in sampler class
    may bring its own (``clock_meter``, tests/bench_stub.py)."""
    own = getattr(sampler_cls, "clock_meter", None)
    if own is not None:
        return own(pci)
    # (built in a daemon thread with a time limit: a metrics library that blocks must not
    # hold up the measurement -- the line then simply has no clock)
    import threading
    box = []

    def build():
        try:
            box.append(SmiClock(pci))
        except Exception:                            # noqa: BLE001
            pass
    th = threading.Thread(target=build, daemon=True)
    th.start()
    th.join(timeout=15)
    return box[0] if box else None


def sampler_class():
    """The per-GPU sampler, ``olpefit_amd.core.Sampler`` (libolpe.so).  The CPU tests of
    the launcher and of the N > 1 reporting set OLPE_BENCH_SAMPLER=module:Class to a
    stand-in that runs no kernel (tests/bench_stub.py); the product has no other."""
    spec = os.environ.get("OLPE_BENCH_SAMPLER")
    if spec:
        import importlib
        mod, _, cls = spec.partition(":")
        return getattr(importlib.import_module(mod), cls)
    from olpefit_amd.core import Sampler
    return Sampler


# ----------------------------------------------------------------------------------
# rank launcher: `bench.py --gpus N` without a launcher's environment
# ----------------------------------------------------------------------------------
def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, grace_s: float = 30.0) -> int:
    """Start ``n`` ranks of this script (one process per GPU, LOCAL_RANK = device) and
    relay rank 0's output -- the reference's launch-sized world (``mpiexec -n W python
    apf_step2.py``, apf_step2.py:27-29, :50-57) without an external launcher.

    The parent makes no HIP call (it imports neither libolpe nor the sampler), so the
    children own the GPUs.  Rank 0's stdout (the JSON line) is copied to this stdout; the
    other ranks' stdout and every rank's stderr go to this stderr.  Returns 0 if every
    rank exits 0, else the first non-zero status; when a rank fails, the others get
    ``grace_s`` to finish (a rank blocked in the host group on a dead peer would wait for
    its timeout) and are then terminated -- only the processes started here."""
    import subprocess
    env0 = dict(os.environ)
    port = _free_port()
    # one node: the ranks meet on the loopback address whatever MASTER_ADDR says
    env0.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                OLPE_BENCH_LAUNCHED="1")
    env0.setdefault("TORCHELASTIC_RUN_ID", f"bench-{os.getpid()}-{port}")
    procs = []

    try:
        import ctypes
        prctl = ctypes.CDLL(None, use_errno=True).prctl
    except (OSError, AttributeError):
        prctl = None

    def die_with_parent():
        # (in the child between fork and exec) a rank must not outlive the launcher, or
        # a killed launcher would leave ranks holding the GPUs: PR_SET_PDEATHSIG (1)
        if prctl is not None:
            prctl(1, signal.SIGTERM, 0, 0, 0)

    def stop_all(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        sys.exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, stop_all)
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env, stdout=subprocess.PIPE if r == 0 else 2,
                                      stderr=None, text=True, preexec_fn=die_with_parent))

    def pump():
        for line in procs[0].stdout:
            sys.stdout.write(line)
            sys.stdout.flush()

    t = threading.Thread(target=pump, daemon=True)
    t.start()
    status = 0
    deadline = None
    live = set(range(n))
    while live:
        for r in sorted(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.discard(r)
            if rc != 0:
                print(f"[bench launcher] rank {r} exited with status {rc}", file=sys.stderr)
                if status == 0:
                    status = rc if rc > 0 else 128 - rc
                    deadline = time.monotonic() + grace_s
        if live and deadline is not None and time.monotonic() > deadline:
            for r in sorted(live):
                print(f"[bench launcher] terminating rank {r} after a peer failed",
                      file=sys.stderr)
                procs[r].terminate()
            for r in sorted(live):
                try:
                    procs[r].wait(timeout=10)
                except subprocess.TimeoutExpired:
                    procs[r].kill()
                    procs[r].wait()
            live.clear()
        time.sleep(0.05)
    t.join(timeout=10)
    return status


# ----------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU, default 1).  Without a launcher's "
                         "WORLD_SIZE, N > 1 starts the N ranks itself; under torchrun / "
                         "mpirun it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: the config's, DEFAULTS)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps first (default: the config's, DEFAULTS)")
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS),
                    help="BASELINE.json config index: 0 one walker 32x32, 1 4,096 walkers, "
                         "2 65,536 walkers per GPU (default), 3 = 2 over 8 GPUs, 4 3-source "
                         "128x128 (16,384 per GPU)")
    ap.add_argument("--walkers", type=int, default=0, help="override walkers per GPU")
    ap.add_argument("--iters", type=int, default=None,
                    help="Gibbs iterations per step (default: the config's, DEFAULTS)")
    ap.add_argument("--stride", type=int, default=None,
                    help="chain record stride (default: the config's, DEFAULTS)")
    ap.add_argument("--mode", default="fast", choices=["exact", "fast"])
    ap.add_argument("--no-alt", action="store_true",
                    help="skip the single-GPU measurement of the other eval mode")
    ap.add_argument("--cpu-steps", type=int, default=None,
                    help="oracle walker-steps in all, spread over one process per usable "
                         "core (default: about 12 s of CPU work: 96,000 at 64x64, scaled by "
                         "64^2/n^2 otherwise)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-csv", action="store_true",
                    help="skip the (untimed) CSV-emission figure of the last launch's rows")
    ap.add_argument("--no-reference-like", action="store_true",
                    help="skip the astropy-object (reference-cost) CPU baseline")
    ap.add_argument("--cpu-steps-ref", type=int, default=None,
                    help="walker-steps of the astropy-object baseline in all (default 24,000 "
                         "at 64x64, scaled by 64^2/n^2)")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--reference-timing",
                    default=os.path.join(REPO, "profiles", "r04", "reference_cpu_timing.json"))
    ap.add_argument("--valu", default=os.path.join(REPO, "profiles", "valu_counts.json"))
    ap.add_argument("--gather-mib", type=float, default=1024.0,
                    help="N > 1: MiB of chain rows per rank per all-gather range")
    ap.add_argument("--comm-timeout", type=float, default=240.0,
                    help="N > 1: seconds the end-of-run RCCL exchange may take before rank 0 "
                         "reports the measurement without it")
    ap.add_argument("--exchange", action="store_true",
                    help="run the end-of-run RCCL exchange (state and chain all-gather, "
                         "moments all-reduce) even with one rank (a one-rank communicator)")
    ap.add_argument("--verify-exchange", action="store_true",
                    help="also gather every range into host memory and check that this "
                         "rank's block equals its own chain rows (exchange_verified)")
    ap.add_argument("--fault-drill", action="store_true",
                    help="with --exchange on one rank: run the collectives' fault drill "
                         "(on by default whenever N > 1; bench.fault_drill)")
    ap.add_argument("--no-fault-drill", action="store_true",
                    help="N > 1: skip the fault drill after the exchange")
    ap.add_argument("--no-moments", action="store_true",
                    help="do not fold each launch's rows into the device moments")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on device 0, no RCCL "
                         "all-gather (RCCL refuses two ranks on one device)")
    ap.add_argument("--share-gpu-rccl", action="store_true",
                    help="rehearsal of the exchange's error path: every rank on device 0 "
                         "and the RCCL exchange attempted (RCCL refuses it; the line "
                         "carries comm_error)")
    args = ap.parse_args()
    if args.gpus is not None and args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus > 1:
            # no launcher: this process starts the ranks and makes no HIP call itself
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif args.gpus is not None and int(env_world) != args.gpus:
        ap.error(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
    dflt = DEFAULTS[args.config]
    for k in ("iters", "stride", "steps", "warmup"):
        if getattr(args, k) is None:
            setattr(args, k, dflt[k])
    # the per-config default shape (the profiled one: profiles/valu_counts.json)
    default_shape = not args.walkers and args.iters == dflt["iters"] \
        and args.stride == dflt["stride"]

    from olpefit_amd import dist as odist
    rank, world, local = odist.env()
    group = odist.HostGroup(rank, world)
    barrier, allmax = group.barrier, group.allmax

    from olpefit_amd import synth
    Sampler = sampler_class()

    wpg, n, nsrc = CONFIGS[args.config]
    if args.walkers:
        wpg = args.walkers
    img, _ = synth.make_image(n, nsrc, 0)
    shared = args.share_gpu or args.share_gpu_rccl
    device = 0 if shared else odist.rank_device(local, Sampler.device_count())
    s = Sampler(img, 1.0, 1, 1, 2, nsrc=nsrc, device=device)
    # which process / device each rank is (the line names them: one process per GPU);
    # the PCI bus ids tell whether the ranks really hold distinct GPUs, whatever each
    # process sees as its device 0..n-1
    placement = group.allgather([rank, local, device, os.getpid(),
                                 Sampler.device_pci_id(device), odist.node_id()])
    pci = [p[4] for p in placement]
    dup = odist.shared_gpus([(p[5], p[4]) for p in placement])
    if world > 1 and not shared and dup:
        # the same verdict on every rank (the gathered list is the same everywhere); a
        # GPU is (node, PCI bus id): identical nodes repeat bus ids
        print(f"[bench rank {rank}] ranks share a GPU (PCI {pci}, shared {dup}): one "
              "process per GPU needs as many GPUs as ranks (--share-gpu for a rehearsal "
              "on fewer)", file=sys.stderr)
        s.close()
        group.close()
        sys.exit(4)
    # step-1 style start (apf_step2.py:264-289) for every walker
    from olpefit_amd.pipeline import initial_parameters
    p0 = initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    p0[-1] = s.chi_squared(p0)
    s.seed(odist.walker_seeds(1000, rank * wpg, wpg))      # weak scaling: wpg per GPU
    s.set_state(np.tile(p0, (wpg, 1)))
    clock = clock_meter(Sampler, placement[rank][4])   # this rank's GPU (its PCI bus id)

    first_launch = []          # when this rank queued its first sampler launch

    def measure(mode, steps, warmup):
        # launches are queued back to back (no host sync between them) and their
        # HIP-event durations read afterwards (olpe_kernel_times)
        s.set_eval_mode(mode)
        if not first_launch:
            first_launch.append(time.perf_counter())
        for _ in range(warmup):
            s.run_async(args.iters, burn_in=0, record_stride=args.stride)
            if not args.no_moments:
                s.moments_accumulate()
        s.sync()
        barrier()
        s.sync()
        t0 = time.perf_counter()
        if clock is not None:
            clock.start()
        kms = []
        for i in range(steps):
            s.run_async(args.iters, burn_in=0, record_stride=args.stride)
            if not args.no_moments:
                # the launch's rows into the whole-run posterior moments (a separate,
                # HBM-bound kernel on the same stream: inside the timed step, outside
                # the sampler's kernel_ms)
                s.moments_accumulate()
            if (i + 1) % 64 == 0:                # the event ring holds 64 launches
                kms.extend(s.kernel_times(64))
        s.sync()
        barrier()
        t1 = time.perf_counter()
        clk, nclk = clock.stop() if clock is not None else (None, 0)
        if steps % 64:
            kms.extend(s.kernel_times(steps % 64))
        km = float(np.mean(kms))
        # every rank's mean sampler time and its own timed-region seconds (one gather, on
        # every rank alike): a scaling shortfall is then attributable from the line --
        # a slow GPU (per_rank_kernel_ms spread) or time outside the sampler kernels
        # (and the GFX clock the SMU reported over the timed launches, SmiClock, with the
        # seconds between this rank's first launch and the timed ones: the telemetry
        # reads low for ~0.3 s after a run starts)
        per_rank = group.allgather([km, t1 - t0, clk, nclk, t0 - first_launch[0]])
        return allmax(t1 - t0), km, per_rank

    elapsed, kernel_ms, per_rank = measure(args.mode, args.steps, args.warmup)
    units = s.last_units()          # chunks per walker of the timed launches
    st, tries, accs = s.get_state()
    acceptance = float(accs.sum() / max(1.0, tries.sum()))
    alt = None
    if world == 1 and not args.no_alt:
        other = "exact" if args.mode == "fast" else "fast"
        alt_steps = max(2, args.steps // 2)
        e2, k2, pr2 = measure(other, alt_steps, 1)
        alt = (other, alt_steps, e2, k2,
               pr2[0][2] if min(p[4] for p in pr2) >= CLOCK_SETTLE_S else None)

    def report(elapsed, kernel_ms, units, acceptance, comm, alt=None):
        """rank 0's JSON line (without the CPU baseline)."""
        total = world * wpg * args.iters * args.steps
        value = total / elapsed
        steps_per_launch = wpg * args.iters
        traffic = load_json(args.traffic) or {}
        valu = load_json(args.valu) or {}
        from olpefit_amd.build import kernel_digest
        digest = kernel_digest()

        def key(mode):
            return mode if args.config in (2, 3) else f"c{args.config}_{mode}"

        def roofline(mode, kernel_ms, clock_ghz=None):
            """FP64-VALU roofline of the sampler kernel.  frac: executed
            FP64 lane-ops (rocprofv3 SQ counts per walker-step, profiles/valu_counts.json)
            x the live HIP-event walker-step rate / the FP64 vector peak."""
            secs = kernel_ms * 1e-3
            rate = steps_per_launch / secs                   # walker-steps/s of the kernel
            peak = FP64_LANE_PEAK / 1e12
            vc = valu.get(key(mode))       # per walker-step, measured at the default shape
            out = {"bound": "fp64-valu", "peak": peak, "unit": "TFLOP/s",
                   "kernel": "olpe_gibbs_kernel", "kernel_ms": kernel_ms,
                   "walker_steps_per_launch": steps_per_launch}
            if vc:
                out.update(
                    achieved=rate * vc["fp64_lane_ops_per_step"] / 1e12,
                    frac=rate * vc["fp64_lane_ops_per_step"] / FP64_LANE_PEAK,
                    frac_source="counters",
                    fp64_lane_ops_per_walker_step=vc["fp64_lane_ops_per_step"],
                    valu_per_walker_step=vc["valu_per_step"],
                    valu_issue_frac=rate * vc["valu_per_step"] * 64 / FP64_LANE_PEAK,
                    counts_stale=vc.get("kernel_digest") != digest)
                prof = vc.get("profile")
                if prof:
                    # the profiling session the counts come from (tools/roofline_session.sh):
                    # its rocprofv3 kernel time, HIP-event time and clock, and the frac
                    # they give -- reproducible from the committed profiles/ files; this
                    # line's frac differs from it by this box's speed (kernel_ms ratio)
                    out["profile"] = dict(prof, frac_ratio_live_over_profile=(
                        prof["rocprof_kernel_ms"] / kernel_ms))
                    if prof.get("clock_ghz"):
                        # the chip holds ~2.0-2.26 GHz under this FP64 load, not the 2.4 GHz
                        # of the peak (MI355X_MICROARCH.md 'DVFS give-back'): the session's
                        # fraction of the FP64 issue rate at the clock it held
                        out["profile"]["frac_of_held_clock_peak"] = (
                            prof["frac"] * 2.4 / prof["clock_ghz"])
            else:                       # no counters for this shape: the model's own count
                ops = work_per_step(n, nsrc, mode)
                out.update(achieved=rate * ops / 1e12, frac=rate * ops / FP64_LANE_PEAK,
                           frac_source="operation count (model + chi^2 only; lower bound)",
                           fp64_lane_ops_per_walker_step=ops)
            if clock_ghz:
                # this box's clock right after the timed launches, and the fraction of the
                # FP64 peak at that clock (the peak scales with the clock: 2.4 GHz spec)
                out["clock_ghz_live"] = clock_ghz
                out["frac_of_held_clock_live"] = out["frac"] * 2.4 / clock_ghz
            ops = work_per_step(n, nsrc, mode)
            out["model_chi2_frac"] = rate * ops / FP64_LANE_PEAK
            algo = sec8d_work(n, nsrc)
            out["equivalent_exp_form_rate"] = rate * algo / 1e12
            out["exp_form_work_per_walker_step"] = algo
            tb = traffic.get(key(mode), {}).get("bytes_per_launch") if default_shape else None
            nrec = args.iters // args.stride if args.stride else 0
            alg = algorithmic_bytes(wpg, nrec, args.iters, nsrc)
            out["algorithmic_bytes"] = alg
            out["traffic_over_algorithmic"] = tb / alg["total"] if tb else None
            out["traffic"] = tb
            out["hbm_gbs"] = tb / secs / 1e9 if tb else None
            out["hbm_frac"] = tb / secs / HBM_PEAK if tb else None
            out["note"] = (
                "frac = executed FP64 VALU lane-ops (64 x SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64 "
                "per walker-step, FMA counted once) x HIP-event rate / 78.6e12/2; "
                "valu_issue_frac = all VALU instructions x 64 / the same peak; model_chi2_frac = "
                "the model + chi^2 operations alone (DESIGN.md §4); equivalent_exp_form_rate = "
                "SURVEY.md 8(d)'s exp-form count Np(12G+8) + E Np G (E = 16) at this rate, in T "
                "lane-ops/s: FAST does far fewer operations, so it is no utilisation figure; "
                "traffic = PMC FETCH_SIZE*2 + WRITE_SIZE bytes per launch "
                "(profiles/pmc_traffic.json), algorithmic_bytes = chain rows + walker state "
                "in/out + the MT19937 state advance (8 B per drawn word); the north star's >= 40 % HBM-read roofline does "
                "not apply to an LDS-resident FP64-VALU-bound kernel (SURVEY.md 8(d)): hbm_frac "
                "is reported, not targeted")
            return out

        out = {
            "metric": METRIC,
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
            "config": {"workload": workload_name(args.config, world, wpg, n, nsrc,
                                                 args.iters, args.stride, args.steps),
                       "walkers_per_gpu": wpg,
                       "image": f"{n}x{n}", "sources": nsrc, "iters_per_step": args.iters,
                       "chain_stride": args.stride, "eval": args.mode,
                       "chunks_per_walker": units,
                       "parallelism": f"walker-sharded x{world}",
                       "devices": [p[2] for p in placement],
                       "pci_bus_ids": sorted(set(pci)),
                       "nodes": len({p[5] for p in placement}),
                       "local_ranks": [p[1] for p in placement],
                       "launcher": ("bench.py --gpus" if os.environ.get("OLPE_BENCH_LAUNCHED")
                                    else "environment" if "WORLD_SIZE" in os.environ
                                    else "none (1 rank)")},
            # (the clock fields only when every rank's telemetry had settled: the same
            # test as clock_settled below)
            "roofline": roofline(args.mode, kernel_ms,
                                 per_rank[0][2] if min(p[4] for p in per_rank) >= CLOCK_SETTLE_S
                                 else None),
            "acceptance": acceptance,
            "allgather_ms": None,
        }
        # where the timed region went, per rank: each rank's mean HIP-event sampler time
        # per launch, and the share of the (max-over-ranks) timed region outside the
        # slowest rank's sampler kernels -- the moments fold, launch gaps, the barriers
        kmax = max(p[0] for p in per_rank)
        out["per_rank_kernel_ms"] = {"min": min(p[0] for p in per_rank), "max": kmax,
                                     "ranks": [p[0] for p in per_rank]}
        out["per_rank_elapsed_s"] = {"min": min(p[1] for p in per_rank),
                                     "max": max(p[1] for p in per_rank)}
        out["per_rank_clock_ghz"] = [p[2] for p in per_rank]
        lead = min(p[4] for p in per_rank)
        out["clock_settled"] = lead >= CLOCK_SETTLE_S
        out["clock_note"] = (
            "per_rank_clock_ghz / roofline.clock_ghz_live: the GFX clock the SMU reported "
            "(amdsmi current_gfxclks, mean over the XCDs) sampled every 10 ms over the "
            f"timed launches ({per_rank[0][3]} samples on rank 0), which began {lead:.2f} s "
            "after the first launch; frac_of_held_clock_live = frac x 2.4 GHz / that clock. "
            "It agrees with the sampler's own s_memtime rate to ~4 % once settled; within "
            "~0.3 s of a run's first launch the telemetry reads low while the kernels already "
            "run at full speed (clock_settled false: the roofline's clock fields are then omitted)")
        out["host_overhead_frac"] = 1.0 - kmax * 1e-3 * args.steps / elapsed
        out["host_overhead_note"] = (
            "1 - max over ranks of (mean sampler kernel ms x steps) / the max-over-ranks "
            "timed region: the moments fold kernel (inside the step, outside kernel_ms), "
            "launch gaps and the host-group barriers")
        out.update(comm)
        if alt:
            other, alt_steps, e2, k2, c2 = alt
            out["alt_eval"] = {"eval": other,
                               "value": world * wpg * args.iters * alt_steps / e2,
                               "ms_per_step": e2 / alt_steps * 1e3,
                               "roofline": roofline(other, k2, c2)}
        return out

    # end-of-run exchange over RCCL/xGMI, outside the timed region:
    # all-gather of the final walker states, then the chain concatenation -- the last
    # launch's chain rows of every rank, gathered range by range so that the receive
    # buffer stays under --gather-mib per rank.  An error (reported by libolpe) is
    # recorded in the JSON line instead of losing the measurement.
    comm = {}
    watchdog = None
    moments = None

    def watchdog_cancel():
        if watchdog is not None:
            watchdog.cancel()

    if (world > 1 or args.exchange) and not args.share_gpu:
        # watchdog: a hung exchange (never observed; RCCL init or a collective waiting on
        # a lost peer) must not cost the measurement -- rank 0 prints its line with the
        # error after --comm-timeout s and every rank exits
        watchdog = threading.Timer(args.comm_timeout, _comm_timeout,
                                   (rank, lambda: report(elapsed, kernel_ms, units, acceptance,
                                                         dict(comm)), args.comm_timeout))
        watchdog.daemon = True
        watchdog.start()
        _quiet_stdout()
        try:
            uid = group.broadcast(Sampler.comm_unique_id() if rank == 0 else None)
            # the library's own bound on every wait for the other ranks (olpe_comm_timeout:
            # past it the communicator is aborted and the call raises), inside the
            # watchdog's, so that a lost peer ends in comm_error rather than the watchdog
            s.comm_timeout(0.8 * args.comm_timeout)
            # every rank alive and here before RCCL's set-up, which itself waits for all
            # ranks without a bound (olpe_comm_init): a dead peer fails this barrier
            barrier()
            s.comm_init(uid, world, rank)
            # RCCL's own view of the communicator on every rank (ncclCommCount /
            # ncclCommUserRank), not the arguments it was created with
            views = group.allgather(list(s.comm_info()))
            comm["comm"] = {"rccl_nranks": views[0][0],
                            "rccl_ranks": [v[1] for v in views],
                            "rccl_nranks_agree": all(v[0] == views[0][0] for v in views)}
            if views[0][0] != world or [v[1] for v in views] != list(range(world)):
                raise RuntimeError(f"RCCL sees {views} for a world of {world}")
            barrier()
            tg = time.perf_counter()
            allst = s.allgather_state()
            comm["allgather_ms"] = allmax(time.perf_counter() - tg) * 1e3
            if allst.shape != (world * wpg, s.ps):
                raise RuntimeError(f"all-gather returned {allst.shape}")
            if not np.array_equal(allst[rank * wpg:(rank + 1) * wpg], s.get_state()[0]):
                raise RuntimeError("all-gathered states differ from this rank's")
            if not args.no_moments:
                tm = time.perf_counter()
                moments = s.allreduce_moments()               # over every rank's walkers
                comm["moments_allreduce_ms"] = allmax(time.perf_counter() - tm) * 1e3
                # the walker total the all-reduce summed (slot 1): every rank's walkers
                comm["comm"]["walkers_allreduced"] = int(moments[1])
            per_walker = s._nrec * s.ps * 8
            wn = max(1, min(wpg, int(args.gather_mib * 2 ** 20 // max(1, per_walker))))
            s.allgather_chain(0, min(wn, wpg), out=False)         # warm-up (buffer, rings)
            barrier()
            tc = time.perf_counter()
            for w0 in range(0, wpg, wn):
                s.allgather_chain(w0, min(wn, wpg - w0), out=False)
            t = allmax(time.perf_counter() - tc)
            nbytes = world * wpg * per_walker
            comm.update(chain_gather_ms=t * 1e3, chain_gather_bytes=nbytes,
                        chain_gather_ranges=(wpg + wn - 1) // wn,
                        chain_gather_range_walkers=min(wn, wpg),
                        chain_gather_gbs=nbytes * (world - 1) / world / t / 1e9
                        if world > 1 else None)
            if args.verify_exchange:
                # every range into host memory: this rank's block must be its own rows
                local = s.chain()
                for w0 in range(0, wpg, wn):
                    got = s.allgather_chain(w0, min(wn, wpg - w0))
                    if got.shape[0] != world or not np.array_equal(got[rank],
                                                                   local[w0:w0 + wn]):
                        raise RuntimeError(f"gathered range [{w0}, {w0 + wn}) differs from "
                                           f"rank {rank}'s chain")
                comm["exchange_verified"] = True
            if (world > 1 or args.fault_drill) and not args.no_fault_drill \
                    and not args.no_moments:
                comm["comm"]["fault_drill"] = fault_drill(s, rank, world, barrier, group)
        except Exception as e:          # noqa: BLE001 -- reported, not hidden
            comm["comm_error"] = f"{type(e).__name__}: {e}"
            print(f"[bench rank {rank}] RCCL exchange failed: {comm['comm_error']}",
                  file=sys.stderr)
        finally:
            _restore_stdout()

    if world > 1 and args.share_gpu and not args.no_moments:
        # ranks sharing one GPU have no RCCL: their moments are summed over the host
        # group instead (the two rounds of olpe_comm_allreduce_moments: the pooled mean,
        # then the squared deviations about it; step3.combine_moments)
        from olpefit_amd import step3
        parts = group.allgather(s.moments_summary().tolist())
        cparts = group.allgather(s.moments_summary(step3.pooled_mean(parts)).tolist())
        moments = step3.combine_moments(parts, cparts)

    if rank != 0:
        watchdog_cancel()
        s.close()
        group.close()
        return

    watchdog_cancel()
    out = report(elapsed, kernel_ms, units, acceptance, comm, alt)
    if moments is None and world == 1 and not args.exchange and not args.no_moments:
        moments = s.allreduce_moments()          # no communicator: this context alone
    if moments is not None:
        # step 3's posterior statistics from the whole-run device moments (every timed and
        # warm-up launch of every rank), without a chain read
        from olpefit_amd import step3
        summ = step3.summary_from_moments(moments, nsrc)
        names = step3.NAMES_2 if nsrc == 2 else step3.NAMES_3
        rc = [summ[k]["gr_rc"] for k in names[:-1]]
        out["posterior"] = {
            "rows_per_walker": summ["_rows_per_walker"], "walkers": summ["_walkers"],
            "means": {k: summ[k]["mean"] for k in names[:4]},
            "stds": {k: summ[k]["std"] for k in names[:4]},
            # Gelman-Rubin needs two walkers or more (configs[0] has one: null)
            "gr_rc_max": max(rc) if all(np.isfinite(rc)) else None,
            "acceptance": sum(summ[k]["accepts"] for k in names[:-1])
            / sum(summ[k]["tries"] for k in names[:-1])}
    if world == 1 and not args.no_csv and getattr(s, "_nrec", 0):
        # "timing excludes CSV emission, which is reported separately" --
        # the last launch's rows of (up to) 4,096 walkers written as the reference's
        # per-walker chain files by the native writer, outside the timed region
        out["csv_emission"] = csv_emission(s, min(s.W, 4096), host_cpus()[0])
    value = out["value"]
    if not args.no_cpu_baseline and world == 1:
        cpu_steps = args.cpu_steps or max(4000, 96000 * 64 * 64 // (n * n))
        # configs[0] is the one-walker plumbing case: the GPU's one walker beside the
        # oracle's one walker on one core, the reference's 1,000 iterations
        cb = (cpu_baseline(n, nsrc, args.cpu_steps or 1000, procs=1) if args.config == 0
              else cpu_baseline(n, nsrc, cpu_steps))
        out["cpu_baseline"] = cb
        out["gpu_over_cpu"] = value / cb["value"]
        if not args.no_reference_like:
            # configs[0]: one walker on one core, the reference's 1,000 iterations
            ref_steps, ref_procs = ((1000, 1) if args.config == 0 else
                                    (args.cpu_steps_ref or max(1600, 24000 * 64 * 64 // (n * n)),
                                     None))
            rl = reference_like_baseline(n, nsrc, ref_steps, procs=ref_procs)
            if rl:
                # the reference's loop cost measured on these cores (the astropy-object
                # oracle), beside the NumPy port above; and the port under the same
                # python3.9, so that their ratio is like for like
                cb["reference_like"] = rl
                out["gpu_over_reference_like"] = value / rl["value"]
                p39 = reference_like_baseline(n, nsrc, ref_steps, procs=ref_procs, port=True)
                if p39:
                    rl["port_same_interpreter"] = p39
                    rl["reference_over_port_same_interpreter"] = rl["value"] / p39["value"]
        ref = reference_ratio(n, nsrc, args.reference_timing)
        if ref and "reference_like" in cb:
            # one reference figure: the one measured on this box.  The build container's
            # reference/port ratio is kept for the record, not turned into a second rate
            # (its port and this box's ran under different interpreters and CPUs)
            cb["build_container_reference_timing"] = ref
        elif ref:
            # the reference itself is slower than the port on the same core: its rate on
            # these cores, derived from the ratio measured in the build container
            cb.update(ref)
            cb["reference_value_derived"] = cb["value"] * ref["reference_over_port"]
            out["gpu_over_reference"] = value / cb["reference_value_derived"]
            out["gpu_over_reference_note"] = (
                "derived: cpu_baseline.value x reference_over_port, the reference/port "
                "speed ratio measured on one core of the build container "
                "(profiles/r04/reference_cpu_timing.json), not on this box; reported only "
                "when the box cannot run the astropy-object baseline (reference_like)")
    print(json.dumps(out))
    s.close()
    group.close()


if __name__ == "__main__":
    main()
