"""apf_step2 command line: the reference's CLI and file surface over the GPU sampler.

Reference: apf_step2.py (2 sources), 3body/apf_step2_3body.py (3 sources) and
apf_step2a.py (the single-walker warm-up).  Kept: positional ``image``, ``-i {1,2a}``
(2-source only), the output directory ``<dir>/<frame>_apf_results/``,
``{w}_finalarray_mpi.csv`` (NaN first row, PS columns, rows from count == burn_in,
written up to the last multiple of 10) and ``{w}_acceptance_rate.csv`` per walker w
(the reference's MPI rank), and the run-length semantics: the run ends at the first
iteration where some walker has tried every parameter ``accept_min`` times
(apf_step2.py:300 + the lockstep barrier at :338).

Output is streamed.  The reference rewrites every file each 10 iterations
(apf_step2.py:355-365), so a killed run leaves its chains on disk; here each kernel
launch (a *chunk*, a multiple of 10 iterations) appends its rows to the per-walker
files and rewrites the acceptance files, so the files always hold what the
reference's files hold at that count, host memory is bounded by one chunk, and a
checkpoint (walker state, counters, RNG streams, moments, file sizes) at most once a
minute (``--checkpoint-secs``) makes a killed run resumable (``--resume``) with the same
chains as an uninterrupted one.  Every launch's rows are also folded into per-walker
moments on the device, and the run ends by writing ``posterior_summary.json``: step 3's
means, sigmas, Gelman-Rubin PSRF / RC and acceptance (apf_step3.py:258-278,
apf_step2.py:362-365) without reading a chain back.

Launched like the reference (``mpiexec -n W python apf_step2.py <image>``), rank 0 runs
all W walkers and the other ranks exit (``MPI_ENV``).  Added flags: ``--walkers`` (the
reference's MPI size), ``--seed``, ``--iters`` (fixed
length instead of accept_min), ``--record-stride``, ``--gpus``, ``--exact``,
``--fixed-bkgd``, ``--chunk``, ``--mem-budget``, ``--checkpoint-secs``,
``--checkpoint-every``, ``--resume``, ``--no-csv``, ``--npy``.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

from . import _lib, dist, fitsio, pipeline, step3
from .core import Sampler

MAX_CHUNK = 20000          # iterations per launch when memory allows

# The reference is launched as ``mpiexec -n W python apf_step2.py <image>``: one walker
# per MPI rank.  Launched that way, this build runs all W walkers in
# rank 0's process on the GPU(s) and the other ranks leave at once, so the same command
# line gives the same files.  (rank, size) variables of the common launchers:
MPI_ENV = (("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE"),     # Open MPI
           ("PMI_RANK", "PMI_SIZE"),                             # MPICH / Intel MPI (Hydra)
           ("MV2_COMM_WORLD_RANK", "MV2_COMM_WORLD_SIZE"))       # MVAPICH2


def mpi_world(environ=None):
    """(rank, size) of an MPI launch, (0, 1) outside one."""
    env = os.environ if environ is None else environ
    for rk, sz in MPI_ENV:
        if rk in env and sz in env:
            try:
                rank, size = int(env[rk]), int(env[sz])
            except ValueError:
                continue
            if size >= 1 and 0 <= rank < size:
                return rank, size
    return 0, 1


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
    ap.add_argument("--walkers", type=int, default=None if variant == "2" else 1,
                    help="independent walkers (the reference's MPI processes; default: the "
                         "size of an mpiexec launch, else 24)")
    ap.add_argument("--accept-min", type=int, default=100000,
                    help="stop when a walker has tried every parameter this often")
    ap.add_argument("--burn-in", type=int,
                    default=6000 if (nsrc == 2 and variant == "2") else 0)
    ap.add_argument("--iters", type=int, default=0 if variant == "2" else 5000,
                    help="run exactly this many iterations (overrides --accept-min); the "
                         "files hold rows up to the last multiple of 10, as the "
                         "reference's (apf_step2.py:355)")
    ap.add_argument("--seed", type=int, default=None,
                    help="walker w uses np.random.seed(seed + w) (default: OS entropy)")
    ap.add_argument("--record-stride", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--device", type=int, default=0, help="first HIP device")
    ap.add_argument("--exact", action="store_true", help="exact per-pixel exp evaluation")
    ap.add_argument("--fixed-bkgd", action="store_true",
                    help="background = p[9] instead of the reference's p[12] (2-source)")
    ap.add_argument("--chunk", type=int, default=0,
                    help="iterations per kernel launch (rounded up to a multiple of 10; "
                         f"default: as many as --mem-budget allows, at most {MAX_CHUNK})")
    ap.add_argument("--mem-budget", type=float, default=1.0,
                    help="GiB of chain rows per launch (host copy; the device buffer is "
                         "also kept under a quarter of free device memory)")
    ap.add_argument("--checkpoint-secs", type=float, default=60.0,
                    help="write a resumable checkpoint after a launch when this many seconds "
                         "have passed since the last one (0 = no time-based checkpoints); a "
                         "checkpoint holds the MT keys, 2.5 KB per walker")
    ap.add_argument("--checkpoint-every", type=int, default=0,
                    help="also write one every N launches (0 = only by time)")
    ap.add_argument("--resume", action="store_true",
                    help="continue the run recorded in the output directory's checkpoint")
    ap.add_argument("--share-gpu", action="store_true",
                    help="one process per rank (torchrun): every rank on --device instead "
                         "of LOCAL_RANK's GPUs (a rehearsal on a one-GPU host)")
    ap.add_argument("--no-csv", action="store_true")
    ap.add_argument("--npy", action="store_true", help="also write {w}_chain.npy")
    ap.add_argument("--timing", action="store_true",
                    help="print where the wall time went (launches, files, checkpoints)")
    ap.add_argument("-q", "--quiet", action="store_true")
    args = ap.parse_args(argv)
    args.mpi_rank, args.mpi_size = mpi_world() if variant == "2" else (0, 1)
    if args.walkers is None:
        args.walkers = args.mpi_size if args.mpi_size > 1 else 24
    if variant == "2a" and args.walkers != 1:
        ap.error("apf_step2a runs one walker (it writes a single step2a.csv)")
    if args.walkers < 1 or args.record_stride < 1 or args.chunk < 0:
        ap.error("--walkers and --record-stride must be >= 1, --chunk >= 0")
    return args


class Shard:
    """The walkers [w0, w0 + W) on one GPU."""

    def __init__(self, img, hdr, nsrc, device, w0, W, p0, seeds, exact, bkgd_mode):
        self.s = Sampler(img, hdr["ITIME"], hdr["COADDS"], hdr["MULTISAM"], hdr["SAMPMODE"],
                         nsrc=nsrc, bkgd_mode=bkgd_mode, device=device)
        self.s.set_eval_mode("exact" if exact else "fast")
        self.device = device
        self.w0, self.W = w0, W
        p = p0.copy()
        with np.errstate(all="ignore"):
            p[-1] = self.s.chi_squared(p)                       # apf_step2.py:283-289
        self.p_init = p
        self.s.seed(seeds[w0:w0 + W])
        self.s.set_state(np.tile(p, (W, 1)))
        self.last = None                 # the last launch's chain [W, nrec, PS]

    def snapshot(self):
        # (the moments need no snapshot: a launch is folded in only when it is kept)
        return self.s.get_state(), self.s.rng_state(), self.s.count

    def restore(self, snap):
        (st, t, a), (mt, g), count = snap
        self.s.set_state(st, t, a)
        self.s.set_rng_state(mt, g)
        self.s.reset_count(count)

    def run(self, n, burn_in, stride, accept_min):
        chain = self.s.run(n, burn_in=burn_in, record_stride=stride, accept_min=accept_min)
        self.last = chain if chain is not None else np.zeros((self.W, 0, self.s.ps))


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


class _Background:
    """One host job at a time beside the GPU work: the previous launch's chain-file
    appends (and a checkpoint's acceptance files) while the next launch runs.  wait()
    joins it and re-raises its error."""

    def __init__(self):
        self.t, self.err = None, None

    def start(self, fn):
        self.wait()

        def body():
            try:
                fn()
            except BaseException as e:      # re-raised by wait()
                self.err = e
        self.t = threading.Thread(target=body, daemon=True)
        self.t.start()

    def wait(self):
        if self.t is not None:
            self.t.join()
            self.t = None
        if self.err is not None:
            e, self.err = self.err, None
            raise e


def device_free_bytes(device: int) -> int:
    f, t = C.c_longlong(0), C.c_longlong(0)
    _lib.check(_lib.load().olpe_device_mem(int(device), C.byref(f), C.byref(t)))
    return int(f.value)


def chunk_size(shards, stride: int, requested: int, budget_gib: float) -> int:
    """Iterations per launch: ``requested`` (rounded up to a multiple of 10), or the
    largest multiple of 10 (<= MAX_CHUNK) whose chain rows -- W x (n/stride + 1) x PS x
    8 bytes -- fit the host budget over all shards and a quarter of each device's free
    memory.  At 65,536 walkers and stride 1 that is a few hundred iterations."""
    if requested:
        return max(10, ((requested + 9) // 10) * 10)
    ps = shards[0].s.ps
    host_rows = budget_gib * 2 ** 30 / (sum(sh.W for sh in shards) * ps * 8)
    dev_rows = min(device_free_bytes(sh.device) / 4 / (sh.W * ps * 8) for sh in shards)
    rows = max(1.0, min(host_rows, dev_rows) - 1)
    n = int(rows * stride) // 10 * 10
    return int(min(MAX_CHUNK, max(10, n)))


class Output:
    """The per-walker files of one run: chain CSVs (+ optional .npy sidecars) grown by
    each launch, acceptance files rewritten at each launch, and the checkpoint."""

    def __init__(self, outdir, shards, variant, csv, npy, base=0):
        # base: the process's first global walker (checkpoint arrays are indexed from it)
        self.outdir, self.shards, self.csv, self.npy = outdir, shards, csv, npy
        self.base = base
        if variant == "2":
            self.names = [[(f"{sh.w0 + k}_finalarray_mpi.csv", f"{sh.w0 + k}_acceptance_rate.csv")
                           for k in range(sh.W)] for sh in shards]
        else:                                   # apf_step2a.py:320-331 (one walker)
            self.names = [[("step2a.csv", "step2a_acceptance_rate")] for _ in shards]
        self.npy_names = [[f"{sh.w0 + k}_chain.npy" for k in range(sh.W)] for sh in shards]
        self.sizes = [np.zeros(sh.W, dtype=np.int64) for sh in shards]
        self.npy_rows = 0

    def _paths(self, g, which):
        return [self.outdir + n[which] for n in self.names[g]]

    def start(self):
        """The NaN seed row (apf_step2.py:278-279) of every chain file."""
        for g, sh in enumerate(self.shards):
            if self.csv:
                empty = np.zeros((sh.W, 0, sh.s.ps))
                pipeline.write_chain_csvs(self._paths(g, 0), empty, nan_row=True)
                self.sizes[g] = np.array([os.path.getsize(p) for p in self._paths(g, 0)])
            if self.npy:
                pipeline.append_npy_chains([self.outdir + n for n in self.npy_names[g]],
                                           np.zeros((sh.W, 0, sh.s.ps)), 0, 0)

    def truncate(self, sizes, npy_rows):
        """Back to a checkpoint: rows appended after it are dropped (they are re-run).
        A file shorter than the checkpoint recorded is not this run's: refused (a
        truncate would pad it with NUL bytes)."""
        for g, sh in enumerate(self.shards):
            mine = sizes[sh.w0 - self.base:sh.w0 - self.base + sh.W]
            if self.csv:
                for p, n in zip(self._paths(g, 0), mine):
                    have = os.path.getsize(p) if os.path.exists(p) else -1
                    if have < int(n):
                        raise ValueError(f"--resume: {p} holds {have} bytes, fewer than the "
                                         f"{int(n)} the checkpoint recorded: not this run's file")
                for p, n in zip(self._paths(g, 0), mine):
                    with open(p, "r+b") as f:
                        f.truncate(int(n))
                self.sizes[g] = np.array(mine, dtype=np.int64)
        if self.npy:
            for g, sh in enumerate(self.shards):
                pipeline.append_npy_chains([self.outdir + n for n in self.npy_names[g]],
                                           np.zeros((sh.W, 0, sh.s.ps)), 0, npy_rows)
        self.npy_rows = npy_rows

    def fold(self):
        """Fold every shard's last launch into its device moments (queued on the device
        before the next launch, which overwrites the rows)."""
        for sh in self.shards:
            if sh.last.shape[1]:
                sh.s.moments_accumulate()

    def append(self, lasts):
        """Append a launch's rows (lasts[g]: shard g's [W][rows][PS]) to the chain files;
        host-only, so it may run beside the next launch."""
        def body(g):
            last = lasts[g]
            rows = last.shape[1]
            if self.csv and rows:
                # one writer thread per shard for step 2a, where the files are shared
                self.sizes[g] = pipeline.append_chain_csvs(self._paths(g, 0), last)
            if self.npy and rows:
                pipeline.append_npy_chains([self.outdir + n for n in self.npy_names[g]],
                                           last, rows, self.npy_rows)
            return rows
        rows = [0] * len(self.shards)

        def run(sh):
            g = self.shards.index(sh)
            rows[g] = body(g)
        _parallel(self.shards, run)
        self.npy_rows += rows[0]

    def commit(self):
        """Append every shard's last launch and fold it into the device moments."""
        self.fold()
        self.append([sh.last for sh in self.shards])

    def acceptance_counts(self):
        """Every shard's (tries, accepts) now, for write_acceptance."""
        return [sh.s.get_state()[1:] for sh in self.shards]

    def write_acceptance(self, counts=None):
        """Rewrite the acceptance files, str(total_accept / total_tries) per walker
        (apf_step2.py:362-365, written once count >= burn_in, :342).  The reference
        rewrites them with the chain every 10 iterations; here at each checkpoint and at
        the end of the run (the count the chain files end at), so a resumed run and an
        uninterrupted one leave the same files.  (Per launch, 65,536 walkers' NumPy prints
        took longer than the launch ran; the native writer formats them as NumPy does.)
        counts: acceptance_counts() taken earlier (host-only then, so it may run beside
        the next launch)."""
        if not self.csv:
            return
        counts = counts if counts is not None else self.acceptance_counts()

        def run(sh):
            g = self.shards.index(sh)
            tries, acc = counts[g]
            pipeline.write_acceptance_files(self._paths(g, 1), acc, tries)
        _parallel(self.shards, run)

    def all_sizes(self):
        return np.concatenate(self.sizes)


def checkpoint_path(outdir, variant, rank=0, world=1):
    if world > 1:        # one per rank of a multi-process run (its walkers only)
        return outdir + f"step2_checkpoint.rank{rank}of{world}.npz"
    return outdir + ("step2_checkpoint.npz" if variant == "2" else "step2a_checkpoint.npz")


def save_checkpoint(path, shards, out, count, config):
    st, tr, ac, mt, ga, mm, mq = [], [], [], [], [], [], []
    nmom = 0
    for sh in shards:
        s, t, a = sh.s.get_state()
        m, g = sh.s.rng_state()
        nmom, mmean, mm2 = sh.s.moments()
        st.append(s), tr.append(t), ac.append(a), mt.append(m), ga.append(g)
        mm.append(mmean), mq.append(mm2)
    tmp = path + ".tmp.npz"
    np.savez(tmp, state=np.concatenate(st), tries=np.concatenate(tr),
             accepts=np.concatenate(ac), mt=np.concatenate(mt), gauss=np.concatenate(ga),
             mom_n=np.int64(nmom), mom_mean=np.concatenate(mm), mom_m2=np.concatenate(mq),
             count=np.int64(count), csv_sizes=out.all_sizes(), npy_rows=np.int64(out.npy_rows),
             config=np.array(json.dumps(config, sort_keys=True)))
    os.replace(tmp, path)


def load_checkpoint(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def run_id_path(outdir, variant):
    return outdir + ("step2_run_id" if variant == "2" else "step2a_run_id")


def posterior_summary(shards, nsrc, group=None):
    """step3.summary_from_moments over every shard's walkers (two passes: the pooled
    mean, then the walkers' deviations about it); with a host group, over every rank's
    shards (the vectors are 2 + 3 PS + 2 P doubles: gathered over TCP, exact in JSON)."""
    def everywhere(vecs):
        vecs = [np.asarray(v, dtype=np.float64) for v in vecs]
        if group is None or group.world <= 1:
            return vecs
        return [np.asarray(v) for part in group.allgather([v.tolist() for v in vecs])
                for v in part]
    parts = everywhere([sh.s.moments_summary() for sh in shards])
    centre = step3.pooled_mean(parts)
    dev = everywhere([sh.s.moments_summary(centre) for sh in shards])
    return step3.summary_from_moments(step3.combine_moments(parts, dev), nsrc)


def main(argv=None, nsrc=2, variant="2"):
    """variant "2": apf_step2 (many walkers, {w}_finalarray_mpi.csv); "2a": the single
    walker warm-up of apf_step2a.py writing step2a.csv / step2a_acceptance_rate
    (:320-331), which ``apf_step2.py -i 2a`` then starts from (apf_step2.py:248-256)."""
    args = parse(sys.argv[1:] if argv is None else argv, nsrc, variant)
    # one process per GPU under torchrun (RANK / WORLD_SIZE / LOCAL_RANK): rank r runs
    # walkers [r W / N, (r+1) W / N) and writes their files; ranks agree through the
    # stdlib-TCP host group on the seed base, the run id, the launch length, the
    # accept_min stop and the checkpoints, and sum their moments for the summary
    rank, world, local = dist.env()
    if variant != "2" or args.mpi_size > 1 or "LOCAL_RANK" not in os.environ:
        rank, world, local = 0, 1, 0
    group = dist.HostGroup(rank, world) if world > 1 else None
    say = (lambda *a: None) if (args.quiet or rank > 0) else print
    if args.mpi_rank > 0:
        # an mpiexec launch: rank 0 runs every walker (see MPI_ENV)
        say(f"MPI rank {args.mpi_rank} of {args.mpi_size}: rank 0 runs all "
            f"{args.walkers} walkers on the GPU; nothing to do here")
        return pipeline.image_paths(args.image)[2]
    image, hdr = fitsio.getdata_header(args.image)              # apf_step2.py:160-161
    directory, frame, outdir = pipeline.image_paths(args.image)  # :164-170
    say(outdir)
    os.makedirs(outdir, exist_ok=True)                           # :172-173
    ckpt = checkpoint_path(outdir, variant, rank, world)
    resume = load_checkpoint(ckpt) if args.resume else None
    if args.resume and resume is None:
        raise FileNotFoundError(ckpt)
    config = {"image": os.path.abspath(args.image), "nsrc": nsrc, "variant": variant,
              "walkers": args.walkers, "accept_min": args.accept_min, "burn_in": args.burn_in,
              "iters": args.iters, "stride": args.record_stride, "exact": args.exact,
              "fixed_bkgd": args.fixed_bkgd, "csv": not args.no_csv, "npy": args.npy,
              "ranks": world}
    if resume is not None:
        old = json.loads(str(resume["config"]))
        old.setdefault("ranks", 1)
        base, p0, run_id = old.pop("seed"), np.array(old.pop("p0")), old.pop("run_id", None)
        try:
            with open(run_id_path(outdir, variant)) as f:
                on_disk = f.read().strip()
        except OSError:
            on_disk = None
        if run_id is None or on_disk != run_id:
            raise ValueError(f"--resume: {ckpt} belongs to run {run_id}, the files in {outdir} "
                             f"to run {on_disk}")
        if old != config:
            diff = {k: (old.get(k), config.get(k)) for k in set(old) | set(config)
                    if old.get(k) != config.get(k)}
            raise ValueError(f"--resume: the checkpoint was written with other settings {diff}")
        say(f"Resuming from {ckpt} at count {int(resume['count'])}")
    else:
        if getattr(args, "initial_guess_option", None) == "2a":  # :248-256
            say("I am taking the initial guess from Step 2a output")
            p0 = pipeline.read_step2a(outdir + "step2a.csv")
        else:
            say("I am taking the initial guess from Step 1 output")
            guess = pipeline.read_guess(directory + frame + "_initialguess")
            p0 = pipeline.initial_parameters(image, guess, nsrc)
        base = args.seed if args.seed is not None else int.from_bytes(os.urandom(4), "little")
        run_id = os.urandom(8).hex()
        if group is not None:
            base, run_id = group.broadcast([base, run_id])        # rank 0's
    config.update(seed=base, p0=[float(v) for v in p0], run_id=run_id)
    W = args.walkers
    seeds = (base + np.arange(W, dtype=np.int64)) & 0xFFFFFFFF
    say(f"walkers {W}, seeds {base}..{base + W - 1} (np.random.seed semantics)"
        + (f", {world} ranks" if world > 1 else ""))
    pw0, pW = dist.shard(W, world, rank)              # this process's walkers
    if pW < 1:
        raise ValueError(f"{W} walkers over {world} ranks: rank {rank} has none")
    ng = max(1, min(args.gpus, pW))
    if args.share_gpu:
        dev0 = args.device
    elif args.gpus == 1 and world > 1:
        # (the branch depends on --gpus alone, the same on every rank, so every rank
        # takes part in the allgather below: pW, and with it ng, can differ by one)
        # one GPU per rank: LOCAL_RANK's device, or device 0 when the launcher gave each
        # process its own GPU (as bench.py; dist.rank_device), and no two ranks on one
        # GPU unless --share-gpu says so: (node, PCI bus id) pairs, gathered so that
        # every rank reaches the same verdict; identical nodes repeat bus ids
        from .core import Sampler
        dev0 = args.device + dist.rank_device(local, Sampler.device_count() - args.device)
        placement = group.allgather([dist.node_id(), Sampler.device_pci_id(dev0)])
        dup = dist.shared_gpus(placement)
        if dup:
            raise RuntimeError(f"ranks share a GPU ({dup}): one process per GPU needs as "
                               "many GPUs as ranks (--share-gpu for a rehearsal on fewer)")
    else:
        # --gpus G contexts per rank: LOCAL_RANK's block of G devices (the same stride on
        # every rank, whatever its shard size)
        dev0 = args.device + local * args.gpus
    bounds = [pw0 + (g * pW) // ng for g in range(ng + 1)]
    shards = [Shard(image, hdr, nsrc, dev0 + g, bounds[g], bounds[g + 1] - bounds[g], p0,
                    seeds, args.exact, 1 if args.fixed_bkgd else 0) for g in range(ng)]
    say("Found initial chi-squared:", shards[0].p_init[-1])
    say("Initial guess:", shards[0].p_init)

    out = Output(outdir, shards, variant, csv=not args.no_csv, npy=args.npy, base=pw0)
    count = 0
    if resume is not None:
        count = int(resume["count"])
        if group is not None and len(set(group.allgather(count))) != 1:
            raise ValueError("--resume: the ranks' checkpoints are at different counts")
        for sh in shards:
            sl = slice(sh.w0 - pw0, sh.w0 - pw0 + sh.W)
            sh.restore(((resume["state"][sl], resume["tries"][sl], resume["accepts"][sl]),
                        (resume["mt"][sl], resume["gauss"][sl]), count))
        if "mom_n" in resume:
            for sh in shards:
                sl = slice(sh.w0 - pw0, sh.w0 - pw0 + sh.W)
                sh.s.set_moments(int(resume["mom_n"]), resume["mom_mean"][sl],
                                 resume["mom_m2"][sl])
        out.truncate(resume["csv_sizes"], int(resume["npy_rows"]))
    else:
        # a fresh run: a checkpoint left by an earlier run in this directory must not be
        # resumable against the files rewritten now
        if os.path.exists(ckpt):
            os.remove(ckpt)
        if rank == 0:
            with open(run_id_path(outdir, variant), "w") as f:
                f.write(run_id + "\n")
        out.start()

    burn, stride = args.burn_in, args.record_stride
    chunk = chunk_size(shards, stride, args.chunk, args.mem_budget)
    if group is not None:                 # every rank launches the same iterations
        chunk = int(-group.allmax(-chunk))
    launches = 0
    last_ckpt = time.monotonic()
    tm = {}                                 # --timing: seconds per kind of work

    class timed:
        def __init__(self, key):
            self.key = key

        def __enter__(self):
            self.t0 = time.perf_counter()

        def __exit__(self, *exc):
            tm[self.key] = tm.get(self.key, 0.0) + time.perf_counter() - self.t0

    t_loop = time.perf_counter()

    bg = _Background()

    def settle():
        with timed("waiting for the file writer"):
            bg.wait()

    def commit():
        # the launch's rows are folded into the device moments now (queued before the
        # next launch) and appended to the files beside the next launch (bg).
        # Checkpoints are spaced by time (and optionally by launches), not written per
        # launch: one holds every walker's MT key (190 MB at 65,536 walkers).  Rank 0's
        # clock decides for every rank, so that all checkpoints hold the same count.
        nonlocal launches, last_ckpt
        with timed("moment fold"):
            out.fold()
        lasts = [sh.last for sh in shards]
        settle()                          # the files take the launches in order
        bg.start(lambda: out.append(lasts))
        launches += 1
        now = time.monotonic()
        due = bool((args.checkpoint_every and launches % args.checkpoint_every == 0) or
                   (args.checkpoint_secs > 0 and now - last_ckpt >= args.checkpoint_secs))
        if group is not None:
            due = bool(group.broadcast(due))
        if due:
            settle()                      # the recorded file sizes
            counts = out.acceptance_counts() if count >= max(burn, 1) else None
            with timed("checkpoints"):
                save_checkpoint(ckpt, shards, out, count, config)
            if counts is not None:        # the checkpoint's count, beside the next launch
                bg.start(lambda: out.write_acceptance(counts))
            last_ckpt = time.monotonic()

    def final_acceptance():
        settle()
        if count >= max(burn, 1):
            with timed("acceptance files"):
                out.write_acceptance()

    def run(n, accept_min=0, record=True):
        with timed("launches (sampler + chain copy)"):
            _parallel(shards, lambda sh: sh.run(n, burn, stride if record else 0, accept_min))

    if args.iters:
        # the files hold rows up to L = the last multiple of 10 <= iters (:355); the
        # iterations after L change no file
        last = (args.iters // 10) * 10
        while count < last:
            n = min(chunk, last - count)
            run(n)
            count += n
            commit()
            say("Loop count:", count)
        final_acceptance()                # the files' count: the last multiple of 10
        if args.iters > max(count, last):
            run(args.iters - max(count, last), record=False)
    else:
        # accept_min semantics: the run ends at the first count C where some walker has
        # min(total_tries) >= accept_min (apf_step2.py:300); with the lockstep barrier
        # every file then holds rows up to L = the last multiple of 10 <= C (:355).
        # Launches start at multiples of 10, so L lies inside the launch that found C:
        # that launch is re-run from its snapshot (RNG included, hence identical) up to L.
        # Every walker's tries sum to the count, so min(tries) <= count / NP: no walker can
        # reach accept_min before count = NP * accept_min, and only the launches from
        # there on need the snapshot for the re-run (the MT keys, 2.5 KB per walker: 164 MB
        # per launch at 65,536 walkers)
        n_par = shards[0].s.ps - 1
        while True:
            need = args.accept_min <= 0 or count + chunk >= n_par * args.accept_min
            with timed("snapshots"):
                snaps = [sh.snapshot() for sh in shards] if need else None
            run(chunk, args.accept_min)
            with timed("launches (sampler + chain copy)"):
                hits = np.concatenate([sh.s.done_at() for sh in shards])
            hits = hits[hits >= 0]
            if group is not None:         # the earliest hit over every rank's walkers
                first = group.allmax(-float(hits.min()) if hits.size else -np.inf)
                hits = np.array([int(-first)]) if np.isfinite(first) else hits[:0]
            # after the reduction, so that every rank raises (`need` is the same on every
            # rank) instead of one rank leaving its peers in the collective
            if hits.size and snaps is None:
                raise RuntimeError(f"accept_min reached at count {int(hits.min())} before "
                                   f"{n_par} x {args.accept_min} iterations")
            if not hits.size:
                count += chunk
                commit()
                say("Loop count:", count)
                continue
            stop = (int(hits.min()) // 10) * 10
            for sh, sn in zip(shards, snaps):
                sh.restore(sn)
            if stop > count:
                run(stop - count)
                count = stop
                commit()
            final_acceptance()
            say("Loop count:", count)
            break
    t_summ = time.perf_counter()
    if variant == "2":
        summ = posterior_summary(shards, nsrc, group)
        if rank == 0:
            with open(outdir + "posterior_summary.json", "w") as f:
                json.dump(summ, f, indent=1)
        if summ["_rows_per_walker"] > 1:
            say("Posterior (device moments):", {k: round(summ[k]["mean"], 6)
                                                for k in list(summ)[:4]})
    tm["posterior summary"] = time.perf_counter() - t_summ
    if args.timing and rank == 0:
        total = time.perf_counter() - t_loop
        print(f"timing ({launches} launches of {chunk} iterations, {total:.2f} s):")
        for k, v in sorted(tm.items(), key=lambda kv: -kv[1]):
            print(f"  {k:32s} {v:8.2f} s")
        print(f"  {'other':32s} {total - sum(tm.values()):8.2f} s")
    if os.path.exists(ckpt):
        os.remove(ckpt)                  # the run is complete: nothing to resume
    for sh in shards:
        sh.s.close()
    if group is not None:
        group.barrier()                   # every rank's files are complete
        group.close()
    say("done with loop")
    return outdir
