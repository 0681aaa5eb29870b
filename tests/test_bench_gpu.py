"""bench.py on the GPU: the N > 1 end-of-run exchange code run with a one-rank RCCL
communicator (--exchange), which is what can be checked before a multi-GPU lease: the
state all-gather, the moments all-reduce and the range-wise chain all-gather, with every
gathered range compared against the rank's own chain rows (--verify-exchange)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    r = subprocess.run([sys.executable, "bench.py", *args], cwd=REPO, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    # stdout is the one JSON line (RCCL's banner goes to stderr during the exchange)
    assert len([ln for ln in r.stdout.splitlines() if ln.strip()]) == 1, r.stdout[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_exchange_one_rank():
    W = 2048
    d = _bench("--exchange", "--verify-exchange", "--fault-drill", "--walkers", str(W),
               "--steps", "2", "--warmup", "1", "--gather-mib", "1", "--no-cpu-baseline",
               "--no-alt")
    assert "comm_error" not in d, d.get("comm_error")
    assert d["n_gpus"] == 1 and d["exchange_verified"] is True
    per_walker = 10 * 17 * 8                         # 100 iterations at stride 10, PS = 17
    assert d["chain_gather_bytes"] == W * per_walker
    assert d["chain_gather_range_walkers"] == 2 ** 20 // per_walker
    assert d["chain_gather_ranges"] == -(-W // (2 ** 20 // per_walker))
    assert d["chain_gather_ms"] > 0 and d["chain_gather_gbs"] is None     # one rank
    assert d["allgather_ms"] > 0 and d["moments_allreduce_ms"] > 0
    p = d["posterior"]
    assert p["walkers"] == W and p["rows_per_walker"] == 3 * 10        # warm-up + 2 steps
    assert 0 < p["acceptance"] < 1 and abs(p["means"]["xcs"] - 31.7) < 0.6
    # the fault drill through RCCL (one rank: both forced steps fail it, the summary
    # recovers); on N > 1 it runs by default after the exchange
    drill = d["comm"].pop("fault_drill")
    assert drill["ok"] is True
    assert [(c["fault"], c["codes"], c["recovered"]) for c in drill["cases"]] == [
        (3, [-2], True), (4, [-2], True)]
    # RCCL's own view (ncclCommCount / ncclCommUserRank) and the all-reduced walker total
    assert d["comm"] == {"rccl_nranks": 1, "rccl_ranks": [0], "rccl_nranks_agree": True,
                         "walkers_allreduced": W}


def test_bench_exchange_one_rank_configs4():
    """configs[4]'s exchange (3 sources, 128x128: PS = 20-column chain rows and the
    OLPE_MOMENTS_LEN(20, 19) moments) through RCCL with a one-rank communicator: the
    uniformity check, the moments all-reduce and the range-wise chain all-gather, every
    range verified against the rank's own rows (3body/apf_step2_3body.py:381-400)."""
    W = 1536
    d = _bench("--config", "4", "--exchange", "--verify-exchange", "--walkers", str(W),
               "--steps", "2", "--warmup", "1", "--gather-mib", "1", "--no-cpu-baseline",
               "--no-alt")
    assert "comm_error" not in d, d.get("comm_error")
    assert d["config"]["sources"] == 3 and d["config"]["image"] == "128x128"
    assert d["exchange_verified"] is True
    per_walker = 10 * 20 * 8                         # 100 iterations at stride 10, PS = 20
    assert d["chain_gather_bytes"] == W * per_walker
    assert d["chain_gather_range_walkers"] == 2 ** 20 // per_walker
    assert d["chain_gather_ranges"] == -(-W // (2 ** 20 // per_walker))
    assert d["moments_allreduce_ms"] > 0 and d["allgather_ms"] > 0
    assert d["comm"]["rccl_nranks"] == 1 and d["comm"]["walkers_allreduced"] == W
    p = d["posterior"]
    assert p["walkers"] == W and p["rows_per_walker"] == 3 * 10
    assert 0 < p["acceptance"] < 1


def test_bench_default_line_has_posterior_and_profile():
    d = _bench("--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-alt")
    assert d["posterior"]["walkers"] == 65536 and d["posterior"]["rows_per_walker"] == 30
    r = d["roofline"]
    assert r["frac_source"] == "counters" and 0 < r["frac"] <= 1


def test_bench_gpus_flag_two_ranks_share_gpu():
    """`bench.py --gpus 2` from a plain process (no launcher environment): the parent
    starts two ranks, makes no HIP call itself, and relays rank 0's line for the two
    ranks' walkers (on the one-GPU box both share device 0: --share-gpu, no RCCL)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--share-gpu",
                        "--walkers", "2048", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-alt"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "walker-sharded x2"
    assert d["config"]["local_ranks"] == [0, 1] and d["config"]["devices"] == [0, 0]
    assert d["config"]["launcher"] == "bench.py --gpus"
    assert d["value"] == pytest.approx(2 * 2048 * 100 * 2 / (d["ms_per_step"] * 2e-3),
                                       rel=1e-9)
    assert d["posterior"]["walkers"] == 2 * 2048


def test_bench_gpus_two_ranks_need_two_gpus():
    """Without --share-gpu, two ranks on a one-GPU box would time-share the card (and
    RCCL refuses them): the ranks compare their devices' PCI bus ids and all exit 4.
    With two or more GPUs visible the same command runs one rank per GPU."""
    from olpefit_amd.core import Sampler
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--walkers", "512",
                        "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-alt"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    if Sampler.device_count() == 1:
        assert r.returncode == 4, r.stderr[-2000:]
        assert "ranks share a GPU" in r.stderr
    else:
        assert r.returncode == 0, r.stderr[-2000:]
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["n_gpus"] == 2 and len(d["config"]["pci_bus_ids"]) == 2


def test_bench_ranks_sharing_the_gpu_attempt_rccl():
    """The only multi-rank RCCL path a one-GPU box can run: two ranks on device 0 try to
    join one communicator (RCCL's bootstrap over both ranks completes, then it refuses two
    ranks on one GPU); every rank leaves the exchange with the error, rank 0's line
    carries it beside the measurement, and the launch exits 0 -- nobody waits."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--share-gpu-rccl",
                        "--walkers", "2048", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--comm-timeout", "120"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert "ncclCommInitRankConfig" in d["comm_error"] and "invalid usage" in d["comm_error"]
    assert r.stderr.count("RCCL exchange failed") == 2       # both ranks, not one
