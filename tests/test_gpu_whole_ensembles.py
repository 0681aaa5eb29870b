"""configs[3] and configs[4] whole, on the one GPU of the test box (round 4).

The multi-GPU runs shard walkers into contiguous ranges with seeds 1000 + global index
and no communication, so rank r of an 8-GPU run computes
exactly what a context holding walkers [r W/8, (r+1) W/8) computes anywhere.  Here the
eight shards of configs[3] (524,288 walkers, 64x64, 2 sources) and of configs[4]
(131,072 walkers, 128x128, 3 sources) run as eight contexts on device 0, and the
whole ensemble as ONE context: chains, final states, counters and RNG state must be
equal bit for bit (the per-GPU and whole launches differ in size, so they take
different launch shapes: walker queue rounds, 16- or 12-wave workgroups, chunking),
the eight shards' moments combined must equal the whole context's, and walkers spread
over the shards must equal the oracle run of their seeds."""
import numpy as np
import pytest

from oracle import olpe_oracle as ora

pytestmark = pytest.mark.gpu


def _setup(n, nsrc):
    from olpefit_amd import synth
    from olpefit_amd.pipeline import initial_parameters
    img, _ = synth.make_image(n, nsrc, 0)
    p0 = initial_parameters(img, synth.guess_values(n, nsrc), nsrc)
    return img, p0


def _run(img, p0, nsrc, w0, W, n_it, launches):
    from olpefit_amd import dist
    from olpefit_amd.core import Sampler
    s = Sampler(img, 1.0, 1, 1, 2, nsrc=nsrc)
    p = p0.copy()
    p[-1] = s.chi_squared(p)
    s.seed(dist.walker_seeds(1000, w0, W))
    s.set_state(np.tile(p, (W, 1)))
    chains = []
    for _ in range(launches):
        chains.append(s.run(n_it, burn_in=0, record_stride=10))
        s.moments_accumulate()
    st, tries, acc = s.get_state()
    mt, g = s.rng_state()
    mom = s.moments_summary()
    s.close()
    return np.concatenate(chains, axis=1), st, tries, acc, mt, g, mom, p


@pytest.mark.parametrize("cfg", ["configs[3]", "configs[4]"])
def test_eight_shards_equal_the_whole_ensemble(lib_loaded, monkeypatch, cfg):
    from olpefit_amd import dist, step3
    for k in ("OLPE_UNITS", "OLPE_NO_QUEUE", "OLPE_WPB", "OLPE_RING"):
        monkeypatch.delenv(k, raising=False)
    n, nsrc, total = (64, 2, 524288) if cfg == "configs[3]" else (128, 3, 131072)
    n_it, launches, world = 100, 2, 8
    img, p0 = _setup(n, nsrc)
    whole = _run(img, p0, nsrc, 0, total, n_it, launches)
    parts = []
    for r in range(world):
        w0, W = dist.shard(total, world, r)
        got = _run(img, p0, nsrc, w0, W, n_it, launches)
        for a, b, what in zip(got[:6], whole[:6], ("chain", "state", "tries", "accepts",
                                                   "mt", "gauss")):
            np.testing.assert_array_equal(a, b[w0:w0 + W], err_msg=f"{cfg} shard {r} {what}")
        parts.append(got[6])
    # the eight shards' moments, combined as the RCCL all-reduce combines them (sums of
    # the per-shard sums; deviations about the pooled mean), equal the whole context's
    comb = step3.combine_moments(parts, [p for p in parts])      # sums only here
    ps = whole[1].shape[1]
    keep = np.r_[0:2 + 2 * ps, 2 + 3 * ps:comb.size]    # n, W, sums, M2, tries, accepts
    np.testing.assert_allclose(comb[keep], whole[6][keep], rtol=1e-12)
    assert comb[1] == total
    # walkers at the shard edges against the oracle
    dm, err, _, _ = ora.noise_model(img, 1.0, 1, 1, 2)
    W8 = total // world
    for w in (0, W8 - 1, W8, 5 * W8 + 17, total - 1):
        ref, _ = ora.Walker(dm, err, whole[7], 1000 + w, nsrc=nsrc).run(n_it * launches,
                                                                         record_stride=10)
        np.testing.assert_allclose(whole[0][w], ref, rtol=1e-8, atol=1e-9,
                                   err_msg=f"{cfg} walker {w}")
