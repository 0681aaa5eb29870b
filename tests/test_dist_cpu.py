"""The N>1 path on CPU: two (and three) ranks run the host orchestration of bench.py
/ olpefit_amd.dist -- the torch-free TCP host group (rendezvous next to a port that is
already taken, as torchrun's agent store takes MASTER_PORT), shard ranges,
global-index seeds, barrier, max/sum over ranks, id broadcast -- with the oracle
standing in for the per-GPU sampler, and the gathered per-rank chains equal a
single-process run of all walkers (chains do not depend on the number of GPUs)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from olpefit_amd import dist as odist


def _oracle_chains(seeds, n_iters):
    from olpefit_amd import synth
    from oracle import olpe_oracle as ora
    img, _ = synth.make_image(32, 2, 0)
    dm, err, _, _ = ora.noise_model(img, 1.0, 1, 1, 2)
    p0 = ora.initial_parameters(img, synth.guess_values(32, 2), 2)
    out = []
    for sd in seeds:
        w = ora.Walker(dm, err, p0, int(sd))
        w.init_chi2()
        out.append(w.run(n_iters)[0])
    return np.array(out)


def _rank_main(rank, world, port, total, n_iters, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    r, w, _ = odist.env()
    g = odist.HostGroup(r, w, timeout_s=120)
    w0, n = odist.shard(total, w, r)
    seeds = odist.walker_seeds(1000, w0, n)
    uid = g.broadcast(b"x" * 128 if r == 0 else None)
    g.barrier()
    chains = _oracle_chains(seeds, n_iters)
    t = g.allmax(float(r + 1))
    tot = g.allsum(float(n))
    gathered = g.allgather([w0, chains.tolist()])
    if r == 0:
        q.put((uid, t, tot, gathered, "torch" in sys.modules))
    g.close()


@pytest.mark.parametrize("world,total", [(2, 5), (3, 5), (8, 11)])
def test_multi_rank_sharding_matches_single_process(world, total):
    # (8 ranks: the configs[3] / SCALE rank count, shards of 1 and 2 walkers)
    n_iters = 60
    # MASTER_PORT held by another listener, as torchrun's agent store holds it
    taken = socket.socket()
    taken.bind(("127.0.0.1", 0))
    taken.listen(1)
    port = taken.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, total, n_iters, q))
             for r in range(world)]
    for p in procs:
        p.start()
    uid, tmax, tot, gathered, torch_loaded = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    taken.close()
    assert uid == b"x" * 128 and tmax == float(world) and tot == float(total)
    assert not torch_loaded                       # the host group needs no PyTorch
    got = np.concatenate([np.array(c).reshape(-1, n_iters, 17)
                          for _, c in sorted(gathered, key=lambda x: x[0])], axis=0)
    ref = _oracle_chains(odist.walker_seeds(1000, 0, total), n_iters)
    np.testing.assert_array_equal(got, ref)


def test_shard_and_seed_helpers():
    assert [odist.shard(10, 3, r) for r in range(3)] == [(0, 3), (3, 3), (6, 4)]
    assert sum(odist.shard(524288, 8, r)[1] for r in range(8)) == 524288
    s = odist.walker_seeds(2 ** 32 - 2, 0, 4)
    assert list(s) == [2 ** 32 - 2, 2 ** 32 - 1, 0, 1]
    g = odist.HostGroup(0, 1)
    assert g.allmax(3.5) == 3.5 and g.broadcast("a") == "a"


def test_shared_gpu_verdict_is_per_node():
    """identical nodes report the same PCI bus ids, so a GPU is a (node, bus
    id) pair -- two nodes' GPU 0 are two GPUs; two ranks on one node's GPU 0 are not."""
    a, b = "0000:05:00.0", "0000:06:00.0"
    assert odist.shared_gpus([("n0", a), ("n1", a)]) == []
    assert odist.shared_gpus([("n0", a), ("n0", b), ("n1", a), ("n1", b)]) == []
    assert odist.shared_gpus([("n0", a), ("n1", a), ("n0", a)]) == [("n0", a)]
    assert odist.node_id()                       # boot id or host name, never empty
    os.environ["OLPE_NODE_ID"] = "fake"
    try:
        assert odist.node_id() == "fake"
    finally:
        del os.environ["OLPE_NODE_ID"]


def test_bench_comm_watchdog_reports_and_exits():
    """bench.py's watchdog of the end-of-run RCCL exchange: rank 0 prints its JSON line
    with the timeout as comm_error (the measurement survives a hung collective) and the
    process leaves with status 3, so the launcher sees the failure."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import bench, threading, time\n"
            "t = threading.Timer(0.2, bench._comm_timeout, (0, lambda: {'value': 1.0}, 0.2))\n"
            "t.start()\n"
            "time.sleep(30)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=repo, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 3, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["value"] == 1.0 and out["comm_error"].startswith("TimeoutError")
