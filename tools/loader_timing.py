"""Step-3 loader timing at configs[1]'s walker count: a 4,096-walker
step-2 CLI run of 2,000 iterations (burn-in 0: 2,001 rows per file with the NaN seed row,
--npy sidecars too) on the GPU, then the chain files read back through the step-3
contract three ways, timed:

  * step3.load_chains(source="csv"): the native threaded parser (olpe_csv_read_chains)
  * step3.load_chains(source="npy"): the --npy sidecars
  * np.genfromtxt, the reference's reader (apf_step3.py:169-186), on a sample of files,
    scaled to all of them
and the posterior summary from the device moments (posterior_summary.json) checked
against step3.summary of the loaded chains at rtol 1e-12.  Prints one JSON line.

    python tools/loader_timing.py [--walkers 4096] [--iters 2000] [--dir /tmp/olpe_lt]
"""
import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--walkers", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "olpe_lt"))
    ap.add_argument("--sample", type=int, default=32, help="files read by genfromtxt")
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    from olpefit_amd import step2, step3, synth
    shutil.rmtree(args.dir, ignore_errors=True)
    path = synth.write_case(args.dir, 64, 2)
    t0 = time.perf_counter()
    out = step2.main([path, "--walkers", str(args.walkers), "--seed", "1000", "--iters",
                      str(args.iters), "--burn-in", "0", "--npy", "-q"])
    t_cli = time.perf_counter() - t0
    csv_bytes = sum(os.path.getsize(out + f"{w}_finalarray_mpi.csv") for w in range(args.walkers))
    res = {"walkers": args.walkers, "iters": args.iters, "cli_s": t_cli, "csv_bytes": csv_bytes,
           "threads": args.threads, "cpu_count": os.cpu_count()}
    t0 = time.perf_counter()
    c = step3.load_chains(out, args.walkers, threads=args.threads)
    res["load_csv_s"] = time.perf_counter() - t0
    res["shape"] = list(c.shape)
    res["load_csv_gbs"] = csv_bytes / res["load_csv_s"] / 1e9
    t0 = time.perf_counter()
    c_npy = step3.load_chains(out, args.walkers, source="npy")
    res["load_npy_s"] = time.perf_counter() - t0
    res["npy_equal_csv"] = bool(np.array_equal(c_npy, c))
    del c_npy
    t0 = time.perf_counter()
    k = min(args.sample, args.walkers)
    ref = np.stack([np.genfromtxt(out + f"{w}_finalarray_mpi.csv", delimiter=",")
                    for w in range(k)], axis=1)[1:]
    t_g = time.perf_counter() - t0
    res["genfromtxt_sample_files"] = k
    res["genfromtxt_sample_s"] = t_g
    res["genfromtxt_all_s_est"] = t_g * args.walkers / k
    res["csv_bit_equal_genfromtxt_sample"] = bool(np.array_equal(
        c[:, :k].view(np.uint64), ref.view(np.uint64)))
    res["speedup_vs_genfromtxt"] = res["genfromtxt_all_s_est"] / res["load_csv_s"]
    with open(out + "posterior_summary.json") as f:
        summ = json.load(f)
    t0 = time.perf_counter()
    s = step3.summary(c)
    res["step3_summary_s"] = time.perf_counter() - t0
    worst = 0.0
    for name, r in s.items():
        for key in ("mean", "std", "gr_psrf", "gr_rc"):
            worst = max(worst, abs(summ[name][key] - r[key]) / abs(r[key]))
    res["moments_vs_summary_max_rel"] = worst
    res["moments_match_rtol_1e-12"] = worst <= 1e-12
    print(json.dumps(res), flush=True)
    shutil.rmtree(args.dir, ignore_errors=True)
    return 0 if res["moments_match_rtol_1e-12"] and res["csv_bit_equal_genfromtxt_sample"] else 1


if __name__ == "__main__":
    sys.exit(main())
