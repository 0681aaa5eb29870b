"""Step-3 read contract and convergence summary.

apf_step3.py reads the step-2 chain files (:169-186), drops ``additional_burnin`` rows
(:81-84, :190-205; default 1 = the NaN seed row) and computes Gelman-Rubin statistics
with d = 16 (:258-278) before its (out-of-scope) distortion / refraction / plotting
stages.  This module is that read + statistics front end, usable on the build's output.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

NAMES_2 = ["xcs", "ycs", "xcc", "ycc", "dx", "dy", "amps", "ampc", "ampratio", "bkgd",
           "sigmax", "sigmay", "sigmax2", "sigmay2", "theta", "theta2", "chisquare"]
NAMES_3 = ["xca", "yca", "xcb", "ycb", "xcc", "ycc", "dx", "dy", "ampa", "ampb", "ampc",
           "ampratio", "bkgd", "sigmax", "sigmay", "sigmax2", "sigmay2", "theta", "theta2",
           "chisquare"]


def load_chains(input_directory: str, ncor: int, additional_burnin: int = 1,
                source: str = "csv", threads: int = 0):
    """apf_step3.py:169-205: returns an array [length - additional_burnin, ncor, PS].

    The chain length is taken from walker 0 and every walker file must have it (the
    reference assigns columns into [length, ncor] arrays, :174-186).  ``source="csv"``
    parses the ``{i}_finalarray_mpi.csv`` files natively from a pool of threads
    (olpe_csv_read_chains: the values np.genfromtxt returns, bit for bit);
    ``source="npy"`` reads the ``{i}_chain.npy`` sidecars step 2 writes with ``--npy``
    (the same rows without the NaN seed row, which counts as one burn-in row)."""
    from . import _lib
    if source == "npy":
        paths = [os.path.join(input_directory, f"{i}_chain.npy") for i in range(ncor)]
        first = np.load(paths[0], mmap_mode="r")
        length, ps = first.shape[0] + 1, first.shape[1]
        burn = min(max(0, int(additional_burnin)), length)
        out = np.empty((length - burn, ncor, ps))
        if burn == 0:
            out[0] = np.nan                     # the seed row the CSV files start with
        lo, o = max(0, burn - 1), 1 if burn == 0 else 0
        for i, p in enumerate(paths):
            a = np.load(p, mmap_mode="r")
            if a.shape != first.shape:
                raise ValueError(f"walker {i}: chain shape {a.shape} != walker 0's {first.shape}")
            out[o:, i, :] = a[lo:]
        return out
    if source != "csv":
        raise ValueError("source must be 'csv' or 'npy'")
    lib = _lib.load()
    paths = [os.fsencode(os.path.join(input_directory, f"{i}_finalarray_mpi.csv"))
             for i in range(ncor)]
    rows, cols = C.c_longlong(0), C.c_int(0)
    _lib.check(lib.olpe_csv_shape(paths[0], C.byref(rows), C.byref(cols)))
    length, ps = rows.value, cols.value
    skip = min(max(0, int(additional_burnin)), length)
    out = np.empty((length - skip, ncor, ps))
    arr = (C.c_char_p * ncor)(*paths)
    rc = lib.olpe_csv_read_chains(arr, ncor, length, ps, skip,
                                  out.ctypes.data_as(C.POINTER(C.c_double)), int(threads))
    if rc == _lib.EINVAL:
        raise ValueError(lib.olpe_last_error().decode(errors="replace"))
    _lib.check(rc)
    return out


def gelman_rubin(p, d: int = 16):
    """apf_step3.py:260-276 (3body/apf_step3_3body.py:294-310) for one parameter:
    p [N, M] (rows, walkers) -> (PSRF, RC).

    The reference is Python 2 without ``from __future__ import division``, so its
    ``RC = np.sqrt(((d+3)/(d+1))*PSRF)`` with the int ``d = 16`` (:264, :276) divides
    19 by 17 as integers: the factor is 1 and RC = sqrt(PSRF).  Integer ``d`` keeps
    that floor division here; a float ``d`` divides as floats, as it would there."""
    p = np.asarray(p, dtype=np.float64)
    # (NumPy floats: one walker gives NaN, as summary_from_moments does, not a raise)
    N, M = np.float64(p.shape[0]), np.float64(p.shape[1])
    overall_mean = np.mean(p)
    # the reference's per-column loop (np.mean / np.std of p[:, i]) as row reductions of
    # the transpose: the same pairwise sums over the same values, so the same bits
    # (a Python loop over 65,536 walkers took 45 s of step 3)
    pt = np.ascontiguousarray(p.T)
    chain_mean = np.mean(pt, axis=1)
    w = np.std(pt, axis=1) ** 2
    b = (chain_mean - overall_mean) ** 2
    w = (1. / M) * np.sum(w)
    b = (N / (M - 1)) * np.sum(b)
    pooled = ((N - 1) / N) * w + ((M + 1) / (M * N)) * b
    psrf = pooled / w
    factor = (d + 3) // (d + 1) if isinstance(d, (int, np.integer)) else (d + 3) / (d + 1)
    return psrf, np.sqrt(factor * psrf)


def summary(chains, nsrc: int = 2):
    """Per-parameter mean, median, std and Gelman-Rubin PSRF / RC over [N, M, PS]
    chains (the chi^2 column is not a GR parameter: apf_step3.py:260,
    3body/apf_step3_3body.py:294)."""
    names = NAMES_2 if nsrc == 2 else NAMES_3
    out = {}
    for k, name in enumerate(names[:-1]):
        x = chains[:, :, k]
        psrf, rc = gelman_rubin(x)
        out[name] = {"mean": float(np.mean(x)), "median": float(np.median(x)),
                     "std": float(np.std(x)), "gr_psrf": float(psrf), "gr_rc": float(rc)}
    return out


def summary_from_moments(m, nsrc: int = 2, d: int = 16):
    """The statistics of ``summary`` (minus the median, which no moment gives) from the
    device-accumulated whole-run moments -- ``Sampler.allreduce_moments()``, the
    olpe_moments_summary layout with the centre at the pooled mean -- without reading a
    chain.  Over N rows per walker (all recorded rows: step 3's default
    additional_burnin = 1) and M walkers, as apf_step3.py:258-278 computes them:

    * mean = sum_w mean_w / M (= np.mean over all rows: every walker has N rows);
    * std = sqrt((sum_w M2_w + N sum_w (mean_w - mean)^2) / (N M)) (np.std over all rows);
    * w = (1/M) sum_w M2_w / N, b = N/(M-1) sum_w (mean_w - mean)^2, PSRF =
      ((N-1)/N w + (M+1)/(M N) b) / w, RC = sqrt(((d+3)//(d+1)) PSRF) (Python 2's
      integer division, see gelman_rubin);
    * acceptance = whole-run accepts / tries per parameter (apf_step2.py:362-365)."""
    names = NAMES_2 if nsrc == 2 else NAMES_3
    m = np.asarray(m, dtype=np.float64)
    ps = len(names)
    np_ = ps - 1
    if m.shape != (2 + 3 * ps + 2 * np_,):
        raise ValueError(f"moments vector of length {m.size}, expected {2 + 3 * ps + 2 * np_}")
    N, M = np.float64(m[0]), np.float64(m[1])      # NumPy floats: M = 1 gives NaN, not a raise
    sums, m2, dev = m[2:2 + ps], m[2 + ps:2 + 2 * ps], m[2 + 2 * ps:2 + 3 * ps]
    tries, acc = m[2 + 3 * ps:2 + 3 * ps + np_], m[2 + 3 * ps + np_:]
    factor = (d + 3) // (d + 1) if isinstance(d, (int, np.integer)) else (d + 3) / (d + 1)
    out = {}
    with np.errstate(all="ignore"):
        for k, name in enumerate(names):
            mean = sums[k] / M
            std = np.sqrt((m2[k] + N * dev[k]) / (N * M))
            ent = {"mean": float(mean), "std": float(std)}
            if k < np_:
                w = (1. / M) * (m2[k] / N)
                b = (N / (M - 1)) * dev[k]
                psrf = (((N - 1) / N) * w + ((M + 1) / (M * N)) * b) / w
                ent.update(gr_psrf=float(psrf), gr_rc=float(np.sqrt(factor * psrf)),
                           acceptance=float(acc[k] / tries[k]), tries=float(tries[k]),
                           accepts=float(acc[k]))
            out[name] = ent
    out["_rows_per_walker"] = int(N)
    out["_walkers"] = int(M)
    return out


def combine_moments(parts, centre_parts):
    """One summary vector from several contexts of one process (step 2's ``--gpus``
    shards): ``parts`` = each context's ``moments_summary()`` (no centre),
    ``centre_parts`` = each context's ``moments_summary(centre)`` about the pooled mean
    of ``parts`` (``pooled_mean(parts)``)."""
    parts = np.asarray(parts)
    out = parts.sum(axis=0)
    out[0] = parts[0][0]
    if not np.all(parts[:, 0] == parts[0][0]):
        raise ValueError("contexts folded different numbers of rows")
    ps = out.size // 5                 # OLPE_MOMENTS_LEN = 2 + 3 PS + 2 (PS - 1)
    out[2 + 2 * ps:2 + 3 * ps] = np.asarray(centre_parts)[:, 2 + 2 * ps:2 + 3 * ps].sum(axis=0)
    return out


def pooled_mean(parts):
    parts = np.asarray(parts)
    ps = parts.shape[1] // 5
    return parts[:, 2:2 + ps].sum(axis=0) / parts[:, 1].sum()


def main(argv=None, nsrc: int = 2):
    """The step-3 command line up to the statistics this build covers: apf_step3.py's
    arguments (positional ``image`` and ``system``, ``-s/--size`` walkers,
    ``-a/--additional_burnin``, :64-84), its read of the chain files (:160-186, native
    loader), its burn-in slice (:190-205) and its Gelman-Rubin statistics (:258-278),
    printed as the reference prints them, then per-parameter mean / median / sigma and
    the acceptance (``posterior_summary.json`` when step 2 wrote one), written to
    ``<frame>_apf_results/step3_summary.json``.  The distortion, refraction and
    separation / PA stages after :278 need the NIRC2 distortion tables the reference
    does not ship and a network name resolver: out of scope.
    ``--from-moments`` skips the chain files and uses step 2's device moments."""
    import argparse
    import json
    import sys
    from . import pipeline
    ap = argparse.ArgumentParser(prog="apf_step3" + ("" if nsrc == 2 else "_3body"))
    ap.add_argument("image", help="the path to the image under study", type=str)
    ap.add_argument("system", help="name of the system (Simbad look-up: not used here)",
                    type=str)
    ap.add_argument("-s", "--size", help="Number of processes", type=str, required=True)
    ap.add_argument("-a", "--additional_burnin", type=int,
                    help="Additional burn in to apply to chains")
    ap.add_argument("--from-moments", action="store_true",
                    help="statistics from step 2's posterior_summary.json (device moments; "
                         "additional_burnin 1) instead of the chain files")
    ap.add_argument("--npy", action="store_true", help="read the {i}_chain.npy sidecars")
    ap.add_argument("-q", "--quiet", action="store_true")
    args = ap.parse_args(sys.argv[1:] if argv is None else argv)
    say = (lambda *a: None) if args.quiet else print
    ncor = int(np.int_(args.size))                                  # :76-77
    additional_burnin = args.additional_burnin or 1                 # :81-84
    _, _, input_directory = pipeline.image_paths(args.image)       # :138-143
    names = NAMES_2 if nsrc == 2 else NAMES_3
    if args.from_moments and additional_burnin != 1:
        # the device moments fold every recorded row (additional_burnin = 1): a larger
        # burn-in cannot be taken out of them afterwards
        ap.error(f"--from-moments covers every recorded row (additional_burnin 1); "
                 f"-a {additional_burnin} needs the chain files")
    if args.from_moments:
        with open(input_directory + "posterior_summary.json") as f:
            summ = json.load(f)
        if summ.get("_walkers") != ncor:
            raise ValueError(f"posterior_summary.json holds {summ.get('_walkers')} walkers, "
                             f"-s gives {ncor}")
        stats = {k: summ[k] for k in names[:-1]}
        length = summ["_rows_per_walker"] + 1
    else:
        say('Importing parameter arrays...')                        # :167
        chains = load_chains(input_directory, ncor, 0, source="npy" if args.npy else "csv")
        length = chains.shape[0]
        if length - additional_burnin < 1:
            raise ValueError(f"{input_directory}: {length} rows per walker file, none left "
                             f"after additional_burnin = {additional_burnin} (step 2's "
                             f"burn-in may exceed its run)")
        say('Parameter array shape:', length)                       # :172
        chains = chains[additional_burnin:length]                   # :190-205
        stats = summary(chains, nsrc)
    N = length - additional_burnin
    say("Number of total jumps per walker:", length)                # :202-204
    say("Number of jumps after additional burn in:", N)
    say("Number of total samples after burn-in: ", N * ncor)
    rc = np.array([stats[k]["gr_rc"] for k in names[:-1]])
    say('Mean and stdev Gelman-Rubin stat for parameter chains:', np.mean(rc), np.std(rc))
    say('GR for positions:', *rc[:4])                               # :277-278
    if not args.from_moments:
        try:
            with open(input_directory + "posterior_summary.json") as f:
                moments = json.load(f)
            for k in names[:-1]:
                for key in ("acceptance", "tries", "accepts"):
                    if key in moments.get(k, {}):
                        stats[k][key] = moments[k][key]
        except (OSError, ValueError):
            pass
    for k in names[:-1]:
        s = stats[k]
        say(f"{k:>9} mean {s['mean']:.10g} median {s.get('median', float('nan')):.10g} "
            f"std {s['std']:.6g} GR {s['gr_rc']:.6f}")
    out = {"walkers": ncor, "rows_per_walker": N, "additional_burnin": additional_burnin,
           "source": "moments" if args.from_moments else ("npy" if args.npy else "csv"),
           "gr_rc_mean": float(np.mean(rc)), "gr_rc_std": float(np.std(rc)),
           "parameters": stats}
    with open(input_directory + "step3_summary.json", "w") as f:
        json.dump(out, f, indent=1)
    return out
