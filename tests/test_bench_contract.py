"""bench.py's JSON contract, checked on CPU: the metric string is BASELINE.json's and the
committed round-3 bench lines (profiles/r03/bench*.log, measured on an MI355X) carry
the fields the driver and the judge read (roofline with a fraction <= 1, cpu_baseline,
a value consistent with the step time)."""
import json
import os

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_metric_is_baselines():
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert bench.METRIC == json.load(f)["metric"]


@pytest.mark.parametrize("name,cfg", [("bench", 2), ("bench_c1", 1), ("bench_c4", 4)])
def test_committed_bench_lines(name, cfg):
    d = _last_json(os.path.join(REPO, "profiles", "r03", f"{name}.log"))
    assert d["metric"] == bench.METRIC and d["unit"] == "walker-steps/s"
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["dtype"] == "f64" and d["vs_baseline"] is None
    wpg, n, nsrc = bench.CONFIGS[cfg]
    c = d["config"]
    assert c["walkers_per_gpu"] == wpg and c["image"] == f"{n}x{n}" and c["sources"] == nsrc
    assert c["workload"] == bench.CONFIG_NAMES[cfg]
    # value = walker-steps of the timed launches / their wall time
    steps = wpg * c["iters_per_step"] * d["steps"]
    assert d["value"] == pytest.approx(steps / (d["ms_per_step"] * d["steps"] * 1e-3), rel=1e-9)
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms"):
        assert k in r
    assert r["frac_source"] == "counters" and r["counts_stale"] is False
    assert 0 < r["frac"] <= 1 and 0 < r["valu_issue_frac"] <= 1
    assert r["achieved"] == pytest.approx(r["frac"] * r["peak"], rel=1e-9)
    # the kernel's HIP-event time is the step time up to launch gaps (back-to-back queue)
    assert r["kernel_ms"] <= d["ms_per_step"] * 1.02
    # the profiling session the counts come from (profiles/r03/roofline.json): the line's
    # frac is the session's scaled by the box's speed, within a few per cent of it
    p = r["profile"]
    assert p["frac"] * p["frac_ratio_live_over_profile"] == pytest.approx(r["frac"], rel=1e-9)
    assert abs(r["frac"] / p["frac"] - 1) < 0.03
    assert r["algorithmic_bytes"]["total"] > 0 and 1 < r["traffic_over_algorithmic"] < 2
    assert d["posterior"]["walkers"] == wpg and d["posterior"]["rows_per_walker"] > 0
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["unit"] == "walker-steps/s" and cb["cores"] >= 1
    assert cb["value"] > 0 and cb["sample"]
