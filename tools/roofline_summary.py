"""Summarise one tools/roofline_session.sh shape into the committed profile files.

    python tools/roofline_summary.py <tag> <key> <session_dir>

<session_dir> (gpurun_out/<tag>_<key>/) holds, from ONE session on one box:
  prof/   rocprofv3 --kernel-trace --stats of a bench run (run_kernel_trace.csv,
          run_kernel_stats.csv) and bench_line.log, that run's JSON line;
  valu/   rocprofv3 --pmc SQ_INSTS_VALU{,_FMA,_MUL,_ADD,_TRANS}_F64 + GRBM_GUI_ACTIVE;
  fetch/, write/   rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE.
Writes profiles/<tag>/: kernel_stats_<key>.csv (as rocprofv3 wrote it),
kernel_trace_<key>.csv, pmc_valu_<key>.csv, pmc_fetch_<key>.csv, pmc_write_<key>.csv
(the sampler's and the moment fold's rows), bench_line_<key>.log and roofline.json[key]:

  rocprof_kernel_ms   mean rocprofv3 duration of the bench's TIMED sampler dispatches
                      (the last `steps` olpe_gibbs_kernel rows of the trace)
  hip_event_kernel_ms the same dispatches by the bench's HIP events (its JSON line)
  fp64_lane_ops_per_walker_step = 64 x (FMA + MUL + ADD + TRANS)_F64 per dispatch /
                      walker-steps per launch; valu_per_walker_step likewise
  clock_ghz           GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration (MI355X_MICROARCH.md)
  frac                = lane-ops x walker-steps per launch / rocprof_kernel_ms / 39.3e12
  traffic             FETCH_SIZE x 2 + WRITE_SIZE bytes per launch (gfx950 correction)

and copies the counts, with the session's kernel time as ``profile``, into
profiles/valu_counts.json[key] (bench.py reports it beside its live frac) and the bytes
into profiles/pmc_traffic.json[key].
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PEAK = 78.6e12 / 2
GIBBS = "olpe_gibbs_kernel"
KEEP = (GIBBS, "fold_rows_kernel", "fold_cols_kernel", "summary_stage")
FP64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
        "SQ_INSTS_VALU_TRANS_F64")


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def filtered_copy(src, dst):
    rs = rows(src)
    with open(src) as f:
        header = next(csv.reader(f))
    with open(dst, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=header, quoting=csv.QUOTE_NONNUMERIC)
        w.writeheader()
        for r in rs:
            if any(k in r["Kernel_Name"] for k in KEEP):
                w.writerow(r)


def counters(path):
    """{dispatch id: {counter: value, '_ns': duration}} of the sampler's dispatches."""
    out = {}
    for r in rows(path):
        if GIBBS not in r["Kernel_Name"]:
            continue
        d = out.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return list(out.values())


def main():
    tag, key, d = sys.argv[1:4]
    from olpefit_amd.build import kernel_digest
    pdir = os.path.join(REPO, "profiles", tag)
    os.makedirs(pdir, exist_ok=True)
    with open(os.path.join(d, "bench_line.log")) as f:
        line = json.loads([x for x in f.read().splitlines() if x.startswith("{")][-1])
    roof = line["roofline"]
    steps, wsteps = line["steps"], roof["walker_steps_per_launch"]
    trace = [r for r in rows(os.path.join(d, "prof", "run_kernel_trace.csv"))
             if GIBBS in r["Kernel_Name"]]
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    timed = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace[-steps:]]
    rocprof_ms = statistics.fmean(timed)
    stats = [r for r in rows(os.path.join(d, "prof", "run_kernel_stats.csv"))
             if GIBBS in r["Name"]][0]
    valu = counters(os.path.join(d, "valu", "run_counter_collection.csv"))
    per = {c: statistics.fmean(v[c] for v in valu) / wsteps for c in ("SQ_INSTS_VALU", *FP64)}
    fp64 = sum(per[c] for c in FP64)
    clocks = [v["GRBM_GUI_ACTIVE"] / 8 / v["_ns"] for v in valu]
    fetch = statistics.fmean(v["FETCH_SIZE"] for v in counters(
        os.path.join(d, "fetch", "run_counter_collection.csv")))
    write = statistics.fmean(v["WRITE_SIZE"] for v in counters(
        os.path.join(d, "write", "run_counter_collection.csv")))
    traffic = 2 * fetch * 1024 + write * 1024
    files = {}
    for name, src in (("kernel_stats", "prof/run_kernel_stats.csv"),
                      ("kernel_trace", "prof/run_kernel_trace.csv"),
                      ("pmc_valu", "valu/run_counter_collection.csv"),
                      ("pmc_fetch", "fetch/run_counter_collection.csv"),
                      ("pmc_write", "write/run_counter_collection.csv")):
        dst = os.path.join(pdir, f"{name}_{key}.csv")
        if name == "kernel_stats":
            shutil.copyfile(os.path.join(d, src), dst)
        else:
            filtered_copy(os.path.join(d, src), dst)
        files[name] = os.path.relpath(dst, REPO)
    shutil.copyfile(os.path.join(d, "bench_line.log"), os.path.join(pdir, f"bench_line_{key}.log"))
    files["bench_line"] = f"profiles/{tag}/bench_line_{key}.log"
    lane_ops = 64 * fp64
    entry = {
        "walker_steps_per_launch": wsteps,
        "timed_dispatches": steps,
        "rocprof_kernel_ms": rocprof_ms,
        "rocprof_kernel_ms_min": min(timed),
        "rocprof_avg_all_dispatches_ms": float(stats["AverageNs"]) / 1e6,
        "hip_event_kernel_ms": roof["kernel_ms"],
        "fp64_lane_ops_per_walker_step": lane_ops,
        "valu_per_walker_step": per["SQ_INSTS_VALU"],
        "clock_ghz": statistics.median(clocks),
        "frac": lane_ops * wsteps / (rocprof_ms * 1e-3) / PEAK,
        "frac_hip_events": lane_ops * wsteps / (roof["kernel_ms"] * 1e-3) / PEAK,
        "valu_issue_frac": 64 * per["SQ_INSTS_VALU"] * wsteps / (rocprof_ms * 1e-3) / PEAK,
        "traffic_bytes_per_launch": traffic,
        "hbm_gbs": traffic / (rocprof_ms * 1e-3) / 1e9,
        "bench_value": line["value"],
        "files": files,
        "kernel_digest": kernel_digest(),
    }
    entry["arithmetic"] = (
        f"frac = {lane_ops:.1f} lane-ops x {wsteps:.0f} walker-steps / {rocprof_ms:.4f} ms / "
        f"{PEAK:.4g} = {entry['frac']:.4f}")
    out = os.path.join(pdir, "roofline.json")
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[key] = entry
    json.dump(data, open(out, "w"), indent=1)
    # the counts bench.py uses, with this session as their profile
    vpath = os.path.join(REPO, "profiles", "valu_counts.json")
    vdata = json.load(open(vpath)) if os.path.exists(vpath) else {}
    vdata[key] = {
        "valu_per_step": per["SQ_INSTS_VALU"], "fp64_per_step": fp64,
        "fp64_lane_ops_per_step": lane_ops,
        "mix_per_step": {c.replace("SQ_INSTS_VALU_", ""): per[c] for c in FP64},
        "dispatches": len(valu), "walker_steps_per_launch": wsteps,
        "kernel_digest": kernel_digest(), "source": files["pmc_valu"],
        "profile": {"tag": tag, "rocprof_kernel_ms": rocprof_ms,
                    "hip_event_kernel_ms": roof["kernel_ms"], "clock_ghz": entry["clock_ghz"],
                    "frac": entry["frac"], "valu_issue_frac": entry["valu_issue_frac"],
                    "files": f"profiles/{tag}/roofline.json[{key}]"},
    }
    json.dump(vdata, open(vpath, "w"), indent=1)
    tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    tdata = json.load(open(tpath)) if os.path.exists(tpath) else {}
    tdata[key] = {"fetch_kb_raw": fetch, "write_kb": write, "fetch_bytes": 2 * fetch * 1024,
                  "write_bytes": write * 1024, "bytes_per_launch": traffic,
                  "source": f"{files['pmc_fetch']} / {files['pmc_write']} (separate passes; "
                            "FETCH_SIZE x2, gfx950 wide-read correction)"}
    json.dump(tdata, open(tpath, "w"), indent=1)
    print(key, json.dumps({k: v for k, v in entry.items() if k != "files"}))


if __name__ == "__main__":
    main()
