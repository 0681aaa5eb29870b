"""End-to-end apf_step2 CLI on the GPU: synthetic FITS + step-1 guess -> chain files,
compared with the chain files the reference's own loop wrote (tests/golden/*_csv) for
the same image, guess, seed and accept_min; then read back through the step-3 contract.

Values: rel 1e-10 (exact eval) / 1e-9 (fast eval); acceptance-rate text: identical
(it depends only on the accept decisions)."""
import os

import numpy as np
import pytest

from olpefit_amd import pipeline, step2, step3, synth

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name,nsrc,mode", [("c64", 2, "exact"), ("c64", 2, "fast"),
                                            ("c64_3", 3, "exact")])
def test_cli_matches_reference_chain_files(tmp_path, golden, name, nsrc, mode):
    g = golden(name)
    n = g["image"].shape[0]
    path = synth.write_case(str(tmp_path), n, nsrc)
    argv = [path, "--walkers", "1", "--seed", "1000", "--accept-min", str(int(g["accept_min"])),
            "--burn-in", str(int(g["burn_in"])), "--chunk", "130", "-q"]
    if mode == "exact":
        argv.append("--exact")
    out = step2.main(argv, nsrc=nsrc)
    got = np.genfromtxt(out + "0_finalarray_mpi.csv", delimiter=",")
    ref = np.genfromtxt(os.path.join(GOLDEN, f"{name}_csv", "0_finalarray_mpi.csv"), delimiter=",")
    assert got.shape == ref.shape
    assert np.all(np.isnan(got[0]))
    np.testing.assert_allclose(got[1:], ref[1:], rtol=1e-10 if mode == "exact" else 1e-9)
    with open(out + "0_acceptance_rate.csv") as f, \
            open(os.path.join(GOLDEN, f"{name}_csv", "0_acceptance_rate.csv")) as h:
        assert f.read() == h.read()


def test_cli_multi_walker_files_feed_step3(tmp_path):
    path = synth.write_case(str(tmp_path), 32, 2)
    out = step2.main([path, "--walkers", "6", "--seed", "7", "--iters", "400", "--burn-in", "100",
                      "--gpus", "1", "-q"])
    c = step3.load_chains(out, 6, additional_burnin=1)
    assert c.shape == (301, 6, 17)                     # counts 100..400
    assert np.all(np.isfinite(c))
    s = step3.summary(c)
    assert abs(s["xcs"]["mean"] - synth.truth_params(32)[0]) < 0.5


def test_cli_seeds_are_gpu_count_independent(tmp_path, monkeypatch):
    """Seeds come from the global walker index, so a sharded run (two contexts on the
    same GPU here) writes the same chains as a single-context run."""
    path = synth.write_case(str(tmp_path / "a"), 32, 2)
    out = step2.main([path, "--walkers", "5", "--seed", "11", "--iters", "200", "--burn-in", "0",
                      "-q", "--no-csv", "--npy"])
    one = [np.load(out + f"{w}_chain.npy") for w in range(5)]
    path2 = synth.write_case(str(tmp_path / "b"), 32, 2)
    _same_device_shards(monkeypatch)                         # 2 shards, 1 physical GPU
    out2 = step2.main([path2, "--walkers", "5", "--seed", "11", "--iters", "200", "--burn-in",
                       "0", "-q", "--no-csv", "--npy", "--gpus", "2"])
    for w in range(5):
        np.testing.assert_array_equal(np.load(out2 + f"{w}_chain.npy"), one[w])


def test_cli_under_mpiexec_equals_walkers_flag(tmp_path, monkeypatch):
    """``mpiexec -n 3 python apf_step2.py <image>`` (the reference's launch): rank 0 runs
    the three walkers and writes the same files as ``--walkers 3`` in one process."""
    for k in [k for pair in step2.MPI_ENV for k in pair]:
        monkeypatch.delenv(k, raising=False)
    args = ["--seed", "21", "--iters", "120", "--burn-in", "20", "-q"]
    path = synth.write_case(str(tmp_path / "a"), 32, 2)
    out = step2.main([path, "--walkers", "3", *args])
    path2 = synth.write_case(str(tmp_path / "b"), 32, 2)
    monkeypatch.setenv("PMI_RANK", "0")
    monkeypatch.setenv("PMI_SIZE", "3")
    out2 = step2.main([path2, *args])
    for w in range(3):
        for name in (f"{w}_finalarray_mpi.csv", f"{w}_acceptance_rate.csv"):
            with open(out + name, "rb") as f, open(out2 + name, "rb") as g:
                assert f.read() == g.read()
    assert not os.path.exists(out2 + "3_finalarray_mpi.csv")


def _oracle_walkers(n, nsrc, seeds, iters):
    from oracle import olpe_oracle as ora
    img, _ = synth.make_image(n, nsrc, 0)
    dm, err, _, _ = ora.noise_model(img, 1.0, 1, 1, 2)
    p0 = ora.initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    out = []
    for sd in seeds:
        w = ora.Walker(dm, err, p0, int(sd), nsrc)
        w.init_chi2()
        chain, _ = w.run(iters)
        out.append((chain, w))
    return out


def test_step2a_matches_oracle_then_step2_from_2a(tmp_path):
    """apf_step2a (reference apf_step2a.py:271-331): one walker, n_steps iterations, rows
    from count 1 written up to the last multiple of 10 (305 -> 300 rows), acceptance
    text str(total_accept / total_tries) at count 300 -- against the oracle walker with
    the same seed (values rel 1e-9, FAST eval; acceptance text identical).  Then
    apf_step2 -i 2a starts every walker from step2a.csv's last row
    (apf_step2.py:248-256)."""
    path = synth.write_case(str(tmp_path), 32, 2)
    out = step2.main([path, "--iters", "305", "--seed", "5", "-q"], nsrc=2, variant="2a")
    a = np.genfromtxt(out + "step2a.csv", delimiter=",")
    assert a.shape == (301, 17) and np.all(np.isnan(a[0]))
    (ref, w), = _oracle_walkers(32, 2, [5], 300)
    np.testing.assert_allclose(a[1:], ref, rtol=1e-9, atol=0)
    with open(out + "step2a_acceptance_rate") as f:
        assert f.read() == pipeline.acceptance_text(w.total_accept, w.total_tries)
    assert not os.path.exists(out + "step2a_checkpoint.npz")      # removed when complete
    out2 = step2.main([path, "-i", "2a", "--walkers", "3", "--iters", "20", "--burn-in", "0",
                       "--seed", "9", "-q", "--no-csv", "--npy"])
    c0 = np.load(out2 + "0_chain.npy")
    assert c0.shape == (20, 17)
    # the first row differs from step2a's last row in at most one parameter + chi^2
    diff = np.nonzero(c0[0, :16] != a[-1, :16])[0]
    assert diff.size <= 1


def _same_device_shards(monkeypatch):
    """--gpus N on the one-GPU box: every shard's context on device 0."""
    orig = step2.Shard.__init__

    def same_device(self, img, hdr, nsrc, device, *a, **k):
        orig(self, img, hdr, nsrc, 0, *a, **k)
    monkeypatch.setattr(step2.Shard, "__init__", same_device)


@pytest.mark.parametrize("gpus,extra", [(1, ["--chunk", "30"]), (2, ["--chunk", "30"]),
                                        (1, ["--mem-budget", "0.0001"])])
def test_cli_accept_min_multi_walker_stop(tmp_path, golden, monkeypatch, gpus, extra):
    """accept_min with several walkers (apf_step2.py:300 + the lockstep barrier at :338):
    the run ends at the global earliest count C at which some walker has tried every
    parameter accept_min times, and every file holds rows burn_in..L, L = the last
    multiple of 10 <= C (:355).  The reference's own per-walker trajectories
    (tests/golden/c32.npz: 4 seeds, each run to its own accept_min) give the expected
    rows and acceptance counters; two shards (two contexts on the one GPU) must write
    the same files, and so must a launch size set by the memory budget."""
    g = golden("c32")
    C = int(g["traj_len"].min())
    L = (C // 10) * 10
    burn = int(g["burn_in"])
    if gpus > 1:
        _same_device_shards(monkeypatch)
    path = synth.write_case(str(tmp_path), 32, 2)
    out = step2.main([path, "--walkers", "4", "--seed", "1000", "--accept-min",
                      str(int(g["accept_min"])), "--burn-in", str(burn), "--gpus", str(gpus),
                      "-q", *extra])
    for w in range(4):
        got = np.genfromtxt(out + f"{w}_finalarray_mpi.csv", delimiter=",")
        assert got.shape == (L - burn + 2, 17)
        np.testing.assert_allclose(got[1:], g["traj_params"][w][burn - 1:L], rtol=1e-9)
        r = g["traj_r"][w][:L]
        tries = np.bincount(r, minlength=16).astype(float)
        acc = np.bincount(r[g["traj_acc"][w][:L].astype(bool)], minlength=16).astype(float)
        with open(out + f"{w}_acceptance_rate.csv") as f:
            assert f.read() == pipeline.acceptance_text(acc, tries)


def test_cli_three_source_feeds_step3(tmp_path):
    """3body/apf_step2_3body.py -> step 3 (3body/apf_step3_3body.py:169-189 read, 20
    columns; GR :292-310 with Python-2 RC = sqrt(PSRF)); chains against the oracle."""
    path = synth.write_case(str(tmp_path), 32, 3)
    out = step2.main([path, "--walkers", "3", "--seed", "40", "--iters", "120", "-q"], nsrc=3)
    c = step3.load_chains(out, 3, additional_burnin=1)
    assert c.shape == (120, 3, 20)
    for w, (ref, _) in enumerate(_oracle_walkers(32, 3, [40, 41, 42], 120)):
        np.testing.assert_allclose(c[:, w, :], ref, rtol=1e-9)
    s = step3.summary(c, nsrc=3)
    assert list(s) == step3.NAMES_3[:-1]
    # the step-3 front end (3body/apf_step3_3body.py's arguments) on the same files
    cli = step3.main([path, "system", "-s", "3", "-q"], nsrc=3)["parameters"]
    for name in s:
        for key in ("mean", "median", "std"):
            assert cli[name][key] == s[name][key]
    for name in s:
        assert s[name]["gr_rc"] == np.sqrt(s[name]["gr_psrf"]) or np.isnan(s[name]["gr_rc"])
    # the device-moment summary of the 20-column chains (posterior_summary.json)
    import json
    with open(out + "posterior_summary.json") as f:
        summ = json.load(f)
    for name, r in s.items():
        # (a parameter some walker never moved has a within-chain variance of exactly 0
        # here and of NumPy's rounding of the mean otherwise: GR compared where every
        # walker's chain varies)
        moved = np.all(np.ptp(c[:, :, step3.NAMES_3.index(name)], axis=0) > 0)
        for key in ("mean", "std") + (("gr_psrf", "gr_rc") if moved else ()):
            np.testing.assert_allclose(summ[name][key], r[key], rtol=1e-12, err_msg=(name, key))


def test_headless_three_source_pipeline(tmp_path):
    """3body step 1 (headless: 8x8 aperture, integer positions) -> 3body step 2 (its
    initial guess read from step 1's file, 3body/apf_step2_3body.py:255-265) -> 3body
    step 3: the chains start at step 1's positions and step 3 reads them."""
    from olpefit_amd import step1
    path = synth.write_case(str(tmp_path), 64, 3)
    t = synth.truth_params(64, 3)
    gp = step1.main([str(tmp_path), "--star", str(t[0] + 1.2), str(t[1] - 0.7),
                     "--companion", str(t[2] - 0.4), str(t[3] + 1.1),
                     "--companion", str(t[4] + 0.6), str(t[5] + 0.3),
                     "--sky", "4", "5"], three_body=True)
    guess = pipeline.read_guess(gp[0])
    assert len(guess) == 8 and np.all(guess == np.round(guess))
    out = step2.main([path, "--walkers", "4", "--seed", "5", "--iters", "100", "-q"], nsrc=3)
    c = step3.load_chains(out, 4, additional_burnin=1)
    assert c.shape == (100, 4, 20) and np.all(np.isfinite(c))
    # the first recorded state is one Gibbs step from the initial vector: at most one
    # parameter moved, so at most one of the six positions differs from step 1's
    moved = np.sum(c[0, :, :6] != guess[None, :6], axis=1)
    assert np.all(moved <= 1), c[0, :, :6]
    cli = step3.main([path, "system", "-s", "4", "-q"], nsrc=3)
    assert cli["walkers"] == 4 and len(cli["parameters"]) == 19


@pytest.mark.parametrize("mode", ["iters", "accept_min"])
def test_cli_resume_after_interrupt(tmp_path, monkeypatch, mode):
    """A run killed after a launch's rows reached the files but before its checkpoint
    was written resumes (--resume) from the previous checkpoint: the files are cut back
    to the checkpoint's sizes, the launch is re-run from the saved walker state and RNG
    streams, and every file ends byte-equal to an uninterrupted run's."""
    path = synth.write_case(str(tmp_path / "ref"), 32, 2)
    path2 = synth.write_case(str(tmp_path / "cut"), 32, 2)
    run = ["--walkers", "3", "--seed", "21", "--burn-in", "15", "--chunk", "40", "--npy", "-q",
           "--checkpoint-every", "1"]
    run += ["--iters", "205"] if mode == "iters" else ["--accept-min", "25"]
    ref = step2.main([path, *run])
    calls = {"n": 0}
    orig = step2.save_checkpoint

    def dying(*a, **k):
        calls["n"] += 1
        if calls["n"] == 3:
            raise KeyboardInterrupt("killed")
        orig(*a, **k)
    monkeypatch.setattr(step2, "save_checkpoint", dying)
    with pytest.raises(KeyboardInterrupt):
        step2.main([path2, *run])
    monkeypatch.setattr(step2, "save_checkpoint", orig)
    cut = step2.main([path2, *run, "--resume"])
    for w in range(3):
        for name in (f"{w}_finalarray_mpi.csv", f"{w}_acceptance_rate.csv"):
            with open(ref + name, "rb") as f, open(cut + name, "rb") as h:
                assert f.read() == h.read(), name
        np.testing.assert_array_equal(np.load(cut + f"{w}_chain.npy"),
                                      np.load(ref + f"{w}_chain.npy"))
    assert not os.path.exists(cut + "step2_checkpoint.npz")


_RSS_RUN = r"""
import resource, sys
sys.path.insert(0, {repo!r})
from olpefit_amd import step2
out = step2.main([{path!r}, "--walkers", "1024", "--seed", "5", "--iters", "{iters}",
                  "--burn-in", "0", "--record-stride", "10", "--chunk", "500", "--no-csv",
                  "--npy", "-q"])
print(out)
print(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss)
"""


def test_cli_host_memory_bounded_by_launch(tmp_path):
    """Streamed output (apf_step2.py:342-365 without the O(n^2) rewrite): 1,024 walkers
    for 1,000 and for 8,000 iterations (stride 10, launches of 500) -- the chain on disk
    grows by 95 MB, the process's peak RSS by far less than that (one launch's rows are
    7 MB), and every walker's .npy holds all its rows."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rss = {}
    for iters in (1000, 8000):
        d = tmp_path / f"r{iters}"
        d.mkdir()
        path = synth.write_case(str(d), 32, 2)
        r = subprocess.run([sys.executable, "-c", _RSS_RUN.format(repo=repo, path=path,
                                                                   iters=iters)],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = r.stdout.strip().splitlines()
        rss[iters] = int(lines[-1]) * 1024                             # ru_maxrss: KiB
        out = lines[-2]
        for w in (0, 1023):
            c = np.load(out + f"{w}_chain.npy")
            assert c.shape[1] == 17 and c.shape[0] in (iters // 10, iters // 10 + 1)
            assert np.all(np.isfinite(c[-iters // 10:]))
    grow = rss[8000] - rss[1000]
    assert grow < 40e6, (rss, grow)


def test_cli_posterior_summary_from_device_moments(tmp_path):
    """SURVEY.md §8(f) row 1 at configs[1]'s size: a 4,096-walker CLI run folds every
    launch's rows into device moments and writes posterior_summary.json; its means,
    sigmas and Gelman-Rubin PSRF / RC equal step3.summary over the chain files read back
    through the step-3 contract (apf_step3.py:169-186, :258-278) at rtol 1e-12, and its
    tries / accepts totals equal the walkers' acceptance counters."""
    import json
    W, iters, burn = 4096, 300, 100
    path = synth.write_case(str(tmp_path), 64, 2)
    out = step2.main([path, "--walkers", str(W), "--seed", "3", "--iters", str(iters),
                      "--burn-in", str(burn), "--chunk", "70", "-q"])
    with open(out + "posterior_summary.json") as f:
        summ = json.load(f)
    c = step3.load_chains(out, W)
    assert c.shape == (iters - burn + 1, W, 17)
    assert summ["_rows_per_walker"] == c.shape[0] and summ["_walkers"] == W
    ref = step3.summary(c)
    for name, r in ref.items():
        for key in ("mean", "std", "gr_psrf", "gr_rc"):
            np.testing.assert_allclose(summ[name][key], r[key], rtol=1e-12, err_msg=(name, key))
    assert sum(summ[n]["tries"] for n in ref) == W * iters
    rates = [np.array(open(out + f"{w}_acceptance_rate.csv").read().strip("[]").split(),
                      dtype=float) for w in (0, 1)]
    assert all(np.all((r >= 0) & (r <= 1)) for r in rates)


def test_cli_checkpoints_spaced_by_time(tmp_path, monkeypatch):
    """Checkpoints (each holds every walker's MT key) are written by time, not per
    launch: 40 launches of a short run write none by default, one every 8 launches with
    --checkpoint-every 8; the run still completes and removes its checkpoint."""
    calls = []
    orig = step2.save_checkpoint

    def counting(*a, **k):
        calls.append(1)
        orig(*a, **k)
    monkeypatch.setattr(step2, "save_checkpoint", counting)
    for extra, want in (([], 0), (["--checkpoint-every", "8"], 5)):
        calls.clear()
        path = synth.write_case(str(tmp_path / f"r{want}"), 32, 2)
        out = step2.main([path, "--walkers", "64", "--seed", "2", "--iters", "400", "--burn-in",
                          "0", "--chunk", "10", "-q", *extra])
        assert len(calls) == want
        assert not os.path.exists(out + "step2_checkpoint.npz")


def test_cli_resume_refuses_another_runs_files(tmp_path, monkeypatch):
    """A fresh run removes a checkpoint an earlier run left in its directory, so a later
    --resume cannot mix two runs; a checkpoint whose run id differs from
    the files', or whose recorded file sizes exceed the files', is refused."""
    path = synth.write_case(str(tmp_path), 32, 2)
    run = ["--walkers", "2", "--seed", "5", "--iters", "200", "--burn-in", "0", "--chunk", "20",
           "-q", "--checkpoint-every", "1"]
    orig = step2.save_checkpoint
    calls = {"n": 0}

    def dying(*a, **k):
        calls["n"] += 1
        if calls["n"] == 3:
            raise KeyboardInterrupt("killed")
        orig(*a, **k)
    monkeypatch.setattr(step2, "save_checkpoint", dying)
    with pytest.raises(KeyboardInterrupt):
        step2.main([path, *run])                           # leaves a checkpoint
    outdir = pipeline.image_paths(path)[2]
    ck = outdir + "step2_checkpoint.npz"
    assert os.path.exists(ck)
    saved = open(ck, "rb").read()
    calls["n"] = 2
    with pytest.raises(KeyboardInterrupt):
        step2.main([path, *run])                           # fresh run, killed early
    assert not os.path.exists(ck)                          # the stale checkpoint is gone
    with pytest.raises(FileNotFoundError):
        step2.main([path, *run, "--resume"])
    with open(ck, "wb") as f:                              # an old run's checkpoint back
        f.write(saved)
    with pytest.raises(ValueError, match="belongs to run"):
        step2.main([path, *run, "--resume"])
    monkeypatch.setattr(step2, "save_checkpoint", orig)
    # same run id, but files shorter than the checkpoint recorded
    with open(ck, "wb") as f:
        f.write(saved)
    z = dict(np.load(ck))
    with open(outdir + "step2_run_id", "w") as f:
        import json
        f.write(json.loads(str(z["config"]))["run_id"] + "\n")
    with open(outdir + "0_finalarray_mpi.csv", "r+b") as f:
        f.truncate(10)
    with pytest.raises(ValueError, match="fewer than"):
        step2.main([path, *run, "--resume"])


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", ["iters", "accept_min"])
def test_cli_torchrun_ranks_equal_one_process(tmp_path, mode):
    """apf_step2 launched one process per GPU (torchrun; here 2 ranks sharing the one
    GPU, --share-gpu): each rank runs its contiguous walker range and writes its walkers'
    files; the ranks agree on the launch length, the accept_min stop (the earliest hit
    over every rank, apf_step2.py:300 + the barrier at :338) and the summary.  Every file
    equals a one-process run's byte for byte; the posterior summary (moments summed over
    the ranks) equals it to rtol 1e-12."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = ["--walkers", "7", "--seed", "31", "--burn-in", "20", "--chunk", "60", "-q", "--npy",
            "--checkpoint-every", "2"]
    args += ["--iters", "230"] if mode == "iters" else ["--accept-min", "30"]
    one = step2.main([synth.write_case(str(tmp_path / "one"), 32, 2), *args])
    path2 = synth.write_case(str(tmp_path / "two"), 32, 2)
    env = dict(os.environ)
    for k in [k for pair in step2.MPI_ENV for k in pair]:
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_free_port()), "apf_step2.py", path2, *args,
                        "--share-gpu"], cwd=repo, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    two = pipeline.image_paths(path2)[2]
    for w in range(7):
        for name in (f"{w}_finalarray_mpi.csv", f"{w}_acceptance_rate.csv"):
            with open(one + name, "rb") as f, open(two + name, "rb") as g:
                assert f.read() == g.read(), name
        np.testing.assert_array_equal(np.load(two + f"{w}_chain.npy"), np.load(one + f"{w}_chain.npy"))
    with open(one + "posterior_summary.json") as f, open(two + "posterior_summary.json") as g:
        a, b = json.load(f), json.load(g)
    for name in step3.NAMES_2[:-1]:
        for key in ("mean", "std", "gr_psrf", "gr_rc", "tries", "accepts"):
            np.testing.assert_allclose(b[name][key], a[name][key], rtol=1e-12, err_msg=(name, key))
    assert not [f for f in os.listdir(two) if "checkpoint" in f]
