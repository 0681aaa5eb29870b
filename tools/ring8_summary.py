"""Summarise tools/gpu_r05_ring8.sh: the configs[4] ring sampler at 2 and 3 waves per
SIMD (8 / 12 waves per workgroup, the same sweep and register budget), and the bound it
puts on a 4-waves-per-SIMD (16-wave) ring (verdict r04 item 4).

    python tools/ring8_summary.py gpurun_out/r05_ring8 profiles/r05/ring8

Per wave count and repetition: walker-steps/s of the kernel (rocprofv3 mean of the
timed dispatches, and the bench line's HIP events), VALU instructions per walker-step
(SQ_INSTS_VALU), the clock (GRBM_GUI_ACTIVE / 8 XCDs / dispatch time) and the VALU issue
fraction at that clock: issue(k) = 64 x VALU per walker-step x rate / 39.3e12 x 2.4 GHz /
the held clock (a wave64 VALU instruction occupies its SIMD 4 cycles at the FP64 rate).

Bound.  Model each wave of a SIMD as ready to issue with probability p, independently:
the SIMD issues with probability u(k) = 1 - (1 - p)^k at k waves.  The measured
u(3) / u(2) fixes p, and u(4) / u(3) is then the most a fourth wave can add at the same
instructions per walker-step -- before the extra instructions a 128-VGPR layout costs
(the two-row update: 12 instead of 11 FP64 per pixel with three sources).  Since waves
do not stall independently (they share the lockstep barriers), the model overstates
what a fourth wave adds, so it is an upper bound.  (Measured, round 5: the issue
fraction rose 1.68x from 2 to 3 waves -- more than the 1.5x of the waves themselves --
so the model's fit degenerates to p -> 0, u(k) proportional to k, and the bound is the
linear one, 4/3: not below 3 %.  The 16-wave ring was then built and measured,
profiles/r05/ring16/summary.json: issue 0.72 -> 0.82 at the held clock, eaten by 12.8 %
more VALU per walker-step; level, -0.6 %.)
"""
import csv
import json
import os
import shutil
import statistics
import sys

PEAK = 78.6e12 / 2            # FP64 lane-ops/s at the 2.4 GHz spec clock
SPEC_GHZ = 2.4
GIBBS = "olpe_gibbs_kernel"


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def line(path):
    with open(path) as f:
        return json.loads([x for x in f.read().splitlines() if x.startswith("{")][-1])


def one(d, log_dir, rg, rep):
    b = line(os.path.join(log_dir, f"bench_w{rg}_{rep}.log"))
    pline = line(os.path.join(log_dir, f"prof_w{rg}_{rep}.log"))
    wsteps = pline["roofline"]["walker_steps_per_launch"]
    steps = pline["steps"]
    trace = sorted((r for r in rows(os.path.join(d, "prof", "run_kernel_trace.csv"))
                    if GIBBS in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    timed = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace[-steps:]]
    kms = statistics.fmean(timed)
    disp = {}
    for r in rows(os.path.join(d, "valu", "run_counter_collection.csv")):
        if GIBBS not in r["Kernel_Name"]:
            continue
        e = disp.setdefault(r["Dispatch_Id"], {})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
        e["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    vals = list(disp.values())
    valu = statistics.fmean(v["SQ_INSTS_VALU"] for v in vals) / wsteps
    fp64 = statistics.fmean(sum(v[c] for c in v if c.endswith("_F64")) for v in vals) / wsteps
    ghz = statistics.median(v["GRBM_GUI_ACTIVE"] / 8 / v["_ns"] for v in vals)
    rate = wsteps / (kms * 1e-3)
    issue_spec = 64 * valu * rate / PEAK
    return {"waves_per_workgroup": rg, "waves_per_simd": rg // 4, "rep": rep,
            "rocprof_kernel_ms": kms, "hip_event_kernel_ms": pline["roofline"]["kernel_ms"],
            "bench_value": b["value"], "bench_kernel_ms": b["roofline"]["kernel_ms"],
            "kernel_walker_steps_per_s": rate, "valu_per_walker_step": valu,
            "fp64_lane_ops_per_walker_step": 64 * fp64, "clock_ghz": ghz,
            "valu_issue_frac_spec": issue_spec,
            "valu_issue_frac_held_clock": issue_spec * SPEC_GHZ / ghz,
            "frac": 64 * fp64 * rate / PEAK}


def main():
    src, dst = sys.argv[1:3]
    waves = [int(x) for x in sys.argv[3:]] or [12, 8]
    os.makedirs(dst, exist_ok=True)
    res = []
    for rep in (1, 2):
        for rg in waves:
            d = os.path.join(src, f"w{rg}_{rep}")
            if not os.path.isdir(d):
                continue
            res.append(one(d, src, rg, rep))
            for sub, name in (("prof/run_kernel_stats.csv", f"kernel_stats_w{rg}_{rep}.csv"),
                              ("valu/run_counter_collection.csv", f"pmc_valu_w{rg}_{rep}.csv")):
                p = os.path.join(d, sub)
                if sub.startswith("valu"):
                    rs = rows(p)
                    with open(p) as f:
                        hdr = next(csv.reader(f))
                    with open(os.path.join(dst, name), "w", newline="") as f:
                        w = csv.DictWriter(f, fieldnames=hdr, quoting=csv.QUOTE_NONNUMERIC)
                        w.writeheader()
                        w.writerows(r for r in rs if GIBBS in r["Kernel_Name"])
                else:
                    shutil.copyfile(p, os.path.join(dst, name))
            for lg in (f"bench_w{rg}_{rep}.log", f"prof_w{rg}_{rep}.log"):
                shutil.copyfile(os.path.join(src, lg), os.path.join(dst, lg))

    def mean(rg, k):
        return statistics.fmean(r[k] for r in res if r["waves_per_workgroup"] == rg)

    if 8 not in waves:
        # another pair (the 16-wave ring against the 12-wave one): the runs side by side
        out = {"runs": res}
        for rg in waves:
            out[f"w{rg}"] = {k: mean(rg, k) for k in ("kernel_walker_steps_per_s",
                             "valu_per_walker_step", "fp64_lane_ops_per_walker_step",
                             "clock_ghz", "valu_issue_frac_spec", "valu_issue_frac_held_clock")}
        with open(os.path.join(dst, "summary.json"), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps({k: v for k, v in out.items() if k != "runs"}, indent=1))
        return

    u2 = mean(8, "valu_issue_frac_held_clock")
    u3 = mean(12, "valu_issue_frac_held_clock")
    r32 = u3 / u2
    # 1 - (1-p)^3 = r (1 - (1-p)^2): with q = 1 - p, q^2 (r - q) = r - 1 ... solve by bisection
    def f(q):
        return (1 - q ** 3) - r32 * (1 - q ** 2)
    lo, hi = 1e-9, 1 - 1e-9
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        if f(lo) * f(mid) <= 0:
            hi = mid
        else:
            lo = mid
    q = 0.5 * (lo + hi)
    u4_over_u3 = (1 - q ** 4) / (1 - q ** 3) if 0 < q < 1 else 1.0
    # the 16-wave layout's extra FP64 work per pixel (three sources: two-row update 3m-1
    # per two rows per set = 2 x 8/2 + 4 = 12 against the four-row update's 11)
    extra = 12.0 / 11.0
    summary = {
        "runs": res,
        "throughput_12_over_8": mean(12, "kernel_walker_steps_per_s") /
                                mean(8, "kernel_walker_steps_per_s"),
        "issue_held_clock_2_waves": u2, "issue_held_clock_3_waves": u3,
        "issue_ratio_3_over_2": r32,
        "model_p_ready": 1 - q,
        "model_issue_ratio_4_over_3": u4_over_u3,
        "bound_4_waves_gain_same_code": u4_over_u3 - 1,
        "sweep_fp64_cost_of_128_vgpr_layout": extra - 1,
        "note": __doc__.split("Bound.")[1].strip(),
    }
    with open(os.path.join(dst, "ring8_bound.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k not in ("runs", "note")}, indent=1))
    for r in res:
        print(r["waves_per_workgroup"], r["rep"], round(r["kernel_walker_steps_per_s"] / 1e6, 2),
              "M/s  valu", round(r["valu_per_walker_step"], 1), " clock", round(r["clock_ghz"], 3),
              " issue(held)", round(r["valu_issue_frac_held_clock"], 3))


if __name__ == "__main__":
    main()
