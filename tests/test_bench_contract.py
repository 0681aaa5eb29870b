"""bench.py's JSON contract, checked on CPU: the metric string is BASELINE.json's and the
committed round-3 bench lines (profiles/r03/bench*.log, measured on an MI355X) carry
the fields the driver and the judge read (roofline with a fraction <= 1, cpu_baseline,
a value consistent with the step time)."""
import json
import os

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


LEGACY_C4 = "configs[4]: 3-source 128x128 cutout, 16,384 walkers/GPU, fp64"


def _last_json(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_metric_is_baselines():
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert bench.METRIC == json.load(f)["metric"]


@pytest.mark.parametrize("where,name,cfg", [
    ("r03", "bench", 2), ("r03", "bench_c1", 1), ("r03", "bench_c4", 4),
    ("r04/final", "bench", 2), ("r04/final", "bench_c1", 1), ("r04/final", "bench_c4", 4),
    ("r05/final", "bench", 2), ("r05/final", "bench_c1", 1), ("r05/final", "bench_c4", 4),
    ("r06/final", "bench", 2), ("r06/final", "bench_c1", 1), ("r06/final", "bench_c4", 4)])
def test_committed_bench_lines(where, name, cfg):
    d = _last_json(os.path.join(REPO, "profiles", where, f"{name}.log"))
    assert d["metric"] == bench.METRIC and d["unit"] == "walker-steps/s"
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["dtype"] == "f64" and d["vs_baseline"] is None
    wpg, n, nsrc = bench.CONFIGS[cfg]
    c = d["config"]
    assert c["walkers_per_gpu"] == wpg and c["image"] == f"{n}x{n}" and c["sources"] == nsrc
    # (rounds 3-5 printed configs[4]'s shard as "configs[4]: ..."; verdict r05 item 3
    # renamed it to what it is, one GPU's shard of BASELINE's 8-GPU configs[4])
    assert c["workload"] == (LEGACY_C4 if cfg == 4 and not where.startswith("r06")
                             else bench.CONFIG_NAMES[cfg])
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
    assert abs(r["frac"] / p["frac"] - 1) < 0.06      # box to box: +-4 % seen
    assert r["algorithmic_bytes"]["total"] > 0 and 1 < r["traffic_over_algorithmic"] < 2
    assert d["posterior"]["walkers"] == wpg and d["posterior"]["rows_per_walker"] > 0
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["unit"] == "walker-steps/s" and cb["cores"] >= 1
    assert cb["value"] > 0 and cb["sample"]
    if where.startswith(("r04", "r05", "r06")):
        # round 4: SURVEY 8(d)'s shape per config, the held clock
        dflt = bench.DEFAULTS[cfg]
        assert c["iters_per_step"] == dflt["iters"] and c["chain_stride"] == dflt["stride"]
        assert d["steps"] * c["iters_per_step"] == {1: 10000, 2: 2000, 4: 500}[cfg]
        assert p["tag"] == ("r06" if where.startswith("r06") else "r04")
        assert 0 < p["frac_of_held_clock_peak"] < 1
        assert c["devices"] == [0] and c["launcher"] == "none (1 rank)"
    if where.startswith("r04"):
        # the reference/port ratio of the build container turned into a derived rate
        assert 0 < cb["reference_over_port"] < 1
        assert d["gpu_over_reference"] == pytest.approx(
            d["value"] / (cb["value"] * cb["reference_over_port"]), rel=1e-9)
    if where.startswith(("r05", "r06")):
        # round 5: one reference figure (measured on the box), the port also timed under
        # that figure's interpreter, and the line's own attribution of the step
        assert "gpu_over_reference" not in d and "reference_value_derived" not in cb
        rl = cb["reference_like"]
        assert 0 < rl["reference_over_port_same_interpreter"] < 1
        assert rl["reference_over_port_same_interpreter"] == pytest.approx(
            rl["value"] / rl["port_same_interpreter"]["value"], rel=1e-9)
        assert d["per_rank_kernel_ms"]["ranks"] == [r["kernel_ms"]]
        assert d["host_overhead_frac"] == pytest.approx(
            1 - r["kernel_ms"] * 1e-3 * d["steps"] / (d["ms_per_step"] * d["steps"] * 1e-3),
            rel=1e-6)
        assert 0 <= d["host_overhead_frac"] < 0.03
        # the profiling session of this round reproduces the line's frac (verdict r04
        # item 6): profiles/r05/roofline.json
        with open(os.path.join(REPO, "profiles", where.split("/")[0], "roofline.json")) as f:
            sess = json.load(f)[{1: "c1_fast", 2: "fast", 4: "c4_fast"}[cfg]]
        assert abs(r["frac"] / sess["frac"] - 1) < 0.03


def test_committed_config0_line():
    """configs[0] (1 walker, 32x32, 1,000 iterations): the GPU's one walker beside the
    oracle's one walker on one core (profiles/r04/final/bench_c0.log)."""
    d = _last_json(os.path.join(REPO, "profiles", "r04", "final", "bench_c0.log"))
    c = d["config"]
    assert c["walkers_per_gpu"] == 1 and c["image"] == "32x32" and c["iters_per_step"] == 1000
    assert d["steps"] == 1 and d["cpu_baseline"]["cores"] == 1
    assert d["value"] > d["cpu_baseline"]["value"] > d["cpu_baseline"]["reference_value_derived"]
    assert d["cpu_baseline"]["reference_like"]["cores"] == 1


@pytest.mark.parametrize("name", ["bench", "bench_c1", "bench_c4"])
def test_committed_lines_carry_the_reference_cost_measured_on_the_box(name):
    """The reference's loop cost measured on the GPU box's cores (the astropy-object
    oracle, bit-equal to the reference's chains) beside the NumPy port: slower than the
    port, and the GPU's lead over it is value / its rate."""
    d = _last_json(os.path.join(REPO, "profiles", "r04", "final", f"{name}.log"))
    cb = d["cpu_baseline"]
    rl = cb["reference_like"]
    assert rl["cores"] == cb["cores"] and 0 < rl["value"] < cb["value"]
    assert d["gpu_over_reference_like"] == pytest.approx(d["value"] / rl["value"], rel=1e-9)


@pytest.mark.parametrize("path", ["r04/c/bench_gpus8_share.log", "r04/a/bench_gpus2.log",
                                  "r04/d/bench_c3_one_gpu.log"])
def test_rehearsal_shapes_are_not_named_configs2(path):
    """Verdict r04 item 2: round 4's rehearsal lines printed configs[2]'s name beside
    8,192 / 2,048 / 524,288 walkers per GPU; the workload is now derived from the shape
    that ran, so those shapes are named ``custom``."""
    d = _last_json(os.path.join(REPO, "profiles", path))
    c = d["config"]
    n = int(c["image"].split("x")[0])
    name = bench.workload_name(2, d["n_gpus"], c["walkers_per_gpu"], n, c["sources"],
                               c["iters_per_step"], c["chain_stride"], d["steps"])
    assert name.startswith("custom: ") and not name.startswith("configs[2]")
    assert f"{c['walkers_per_gpu']:,} walkers" in name


def test_default_workload_names_are_unchanged():
    for cfg in (0, 1, 2, 4):
        wpg, n, nsrc = bench.CONFIGS[cfg]
        d = bench.DEFAULTS[cfg]
        assert bench.workload_name(cfg, 1, wpg, n, nsrc, d["iters"], d["stride"],
                                   d["steps"]) == bench.CONFIG_NAMES[cfg]
    d = bench.DEFAULTS[2]
    assert bench.workload_name(2, 8, 65536, 64, 2, d["iters"], d["stride"],
                               d["steps"]) == bench.CONFIG3
    # another run length keeps the name and says what ran
    w = bench.workload_name(2, 1, 65536, 64, 2, 1000, 10, 20)
    assert w.startswith(bench.CONFIG_NAMES[2]) and "20 launches x 1000 iterations" in w
    # configs[4]'s shape under --config 2 is custom (the config names the 2-source shape)
    assert bench.workload_name(2, 1, 16384, 128, 3).startswith("custom: ")
    # configs[4]: a shard of the 8-GPU config on one GPU, the whole config at 8
    assert "16,384 of 131,072 walkers" in bench.CONFIG_NAMES[4]
    assert bench.workload_name(4, 8, 16384) == bench.CONFIG4
    assert bench.workload_name(4, 4, 16384).startswith("configs[4]'s shape per GPU, weak-scaled")


def test_smi_clock_parses_and_samples_the_metrics_table():
    """bench.SmiClock: the mean of the valid per-XCD GFX clocks of the SMU's metrics
    table (MHz -> GHz; 'N/A' and the 65535 filler dropped), sampled from a thread between
    start() and stop(); clock_meter gives None where no GPU's metrics can be read."""
    import time
    import bench

    class FakeSmi:
        def __init__(self):
            self.calls = 0

        def amdsmi_get_gpu_metrics_info(self, h):
            self.calls += 1
            return {"current_gfxclks": [2000, 2100, 65535, "N/A"], "current_gfxclk": 1}

    c = object.__new__(bench.SmiClock)
    c._smi, c._h, c.period, c._th = FakeSmi(), None, 0.005, None
    assert c._read() == pytest.approx(2.05)
    c.start()
    time.sleep(0.05)
    ghz, n = c.stop()
    assert n >= 2 and ghz == pytest.approx(2.05)
    c._smi.amdsmi_get_gpu_metrics_info = lambda h: {"current_gfxclks": ["N/A"],
                                                     "current_gfxclk": 1950}
    assert c._read() == pytest.approx(1.95)
    assert bench.clock_meter(object, "0000:ff:00.0") is None      # no such GPU here


def test_committed_exchange_lines_round6():
    """The one-rank RCCL exchange on the final tree for configs[2] and configs[4] (verdict
    r05 item 2): every gathered range verified, RCCL's own view of the communicator and
    the walker total the moments all-reduce summed in the line."""
    for name, w, ps in (("bench_exchange", 65536, 17), ("bench_c4_exchange", 16384, 20)):
        d = _last_json(os.path.join(REPO, "profiles", "r06", "final", f"{name}.log"))
        assert d["exchange_verified"] is True and "comm_error" not in d
        assert d["comm"] == {"rccl_nranks": 1, "rccl_ranks": [0], "rccl_nranks_agree": True,
                             "walkers_allreduced": w}
        assert d["chain_gather_bytes"] == w * 10 * ps * 8
        assert d["moments_allreduce_ms"] > 0 and d["posterior"]["walkers"] == w
