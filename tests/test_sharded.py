"""Within-filter sharding: host algebra and the exchange, on CPU.

The device shard (include/pf_shard.h) needs a GPU (tests/test_gpu_sharded.py); here the
orchestrator in particle_filters_amd/sharded.py drives the NumPy shard of
oracle/shard_oracle.py, in-process (W = 1, 2, 4) and over torch.distributed gloo with world
size 2 on 127.0.0.1.  Claims: the global normaliser / Neff / moments combine exactly; the
systematic slot ranges partition [0, Np) and agree with the positions' own comparisons; a
W-shard filter follows the 1-shard filter to fp64 rounding.
"""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from particle_filters_amd import models as M
from particle_filters_amd import sharded as SH
from oracle import shard_oracle, ssm_oracle


def test_combine_matches_concatenated_weights():
    rng = np.random.default_rng(0)
    W, n, nx = 4, 50, 3
    ls = [rng.normal(size=n) * 3 + 10 * g for g in range(W)]
    xs = [rng.normal(size=(n, nx)) for _ in range(W)]
    lse_g, neff_g, means, covs = [], [], [], []
    for l, x in zip(ls, xs):
        m = l.max()
        e = np.exp(l - m)
        w = e / e.sum()
        lse_g.append(m + np.log(e.sum()))
        neff_g.append(1 / np.sum(w * w))
        means.append(w @ x)
        xc = x - w @ x
        covs.append((xc.T * w) @ xc)
    lse, neff, mean, cov, Wg = SH.combine(np.array(lse_g), np.array(neff_g), np.array(means), np.array(covs))
    L, X = np.concatenate(ls), np.concatenate(xs)
    m = L.max()
    w = np.exp(L - m) / np.exp(L - m).sum()
    np.testing.assert_allclose(lse, m + np.log(np.exp(L - m).sum()), rtol=1e-14)
    np.testing.assert_allclose(neff, 1 / np.sum(w * w), rtol=1e-12)
    np.testing.assert_allclose(mean, w @ X, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(cov, np.cov(X.T, aweights=w, bias=True), rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(Wg.sum(), 1.0, rtol=1e-15)


@pytest.mark.parametrize("seed", range(6))
def test_slot_ranges_partition_and_match_positions(seed):
    rng = np.random.default_rng(seed)
    W, n_total = 5, 4000
    w = rng.dirichlet(np.full(W, 0.3 if seed % 2 else 3.0))
    if seed == 5:
        w[2] = 0.0  # an empty shard
        w /= w.sum()
    B = SH.boundaries(w)
    U = float(rng.random())
    a = SH.slot_starts(B, U, n_total)
    assert a[0] == 0 and a[-1] == n_total and np.all(np.diff(a) >= 0)
    pos = (U + np.arange(n_total)) / n_total
    for g in range(W):  # slots of shard g are exactly the positions in [B_g, B_{g+1})
        own = np.nonzero((pos >= B[g]) & (pos < B[g + 1]))[0] if g < W - 1 else np.nonzero(pos >= B[g])[0]
        np.testing.assert_array_equal(np.arange(a[g], a[g + 1]), own)
    n_loc = n_total // W
    for d in range(W):  # every destination receives exactly n_loc rows, in slot order
        got = []
        for g in range(W):
            lo, n = SH.overlap(a, g, d, n_loc)
            got.extend(range(lo, lo + n))
        assert got == list(range(d * n_loc, (d + 1) * n_loc))


def sv_setup():
    ssm = ssm_oracle.sv_logsq(0.95, 0.2, 1.0)
    g, h = M.SVTransition(0.95), M.SVLogSqObservation(1.0)
    rng = np.random.default_rng(42)
    x = 0.0
    Z = []
    for _ in range(60):
        x = 0.95 * x + 0.2 * rng.standard_normal()
        Z.append(np.log((np.exp(x / 2) * rng.standard_normal()) ** 2))
    return ssm, g, h, np.array(Z)[:, None]


def run_local(W, Np=2000, steps=60):
    ssm, g, h, Z = sv_setup()
    pf = SH.ShardedParticleFilter(g, h, ssm.Q, ssm.R, Np=Np, resample_thresh=0.5, seed=11, n_shards=W,
                                  shard_factory=shard_oracle.factory(ssm))
    pf.initialize([0.0], [[0.5]])
    means, neff, flags = pf.run(Z[:steps])
    parts = np.concatenate([pf.local_particles()[g] for g in range(W)])
    return means, neff, flags, parts


@pytest.mark.parametrize("W", [2, 4])
def test_in_process_shards_follow_one_shard(W):
    m1, n1, f1, x1 = run_local(1)
    mW, nW, fW, xW = run_local(W)
    assert f1.sum() >= 3, "the run must exercise the resample / exchange path"
    np.testing.assert_array_equal(fW, f1)
    np.testing.assert_allclose(mW, m1, rtol=0, atol=1e-10)
    np.testing.assert_allclose(nW, n1, rtol=1e-10)
    np.testing.assert_allclose(xW, x1, rtol=0, atol=1e-10)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ssm, g, h, Z = sv_setup()
        pf = SH.ShardedParticleFilter(g, h, ssm.Q, ssm.R, Np=2000, resample_thresh=0.5, seed=11, comm=SH.DistComm(),
                                      shard_factory=shard_oracle.factory(ssm))
        pf.initialize([0.0], [[0.5]])
        means, neff, flags = pf.run(Z)
        q.put((rank, means, neff, flags, pf.local_particles()[rank]))
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_follow_one_shard():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=180) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m1, n1, f1, x1 = run_local(1)
    for rank, means, neff, flags, parts in out:
        np.testing.assert_array_equal(flags, f1)
        np.testing.assert_allclose(means, m1, rtol=0, atol=1e-10)
        np.testing.assert_allclose(neff, n1, rtol=1e-10)
    np.testing.assert_allclose(np.concatenate([o[4] for o in out]), x1, rtol=0, atol=1e-10)


# ---------------------------------------------------------------------------
# host replay of the reference's draw stream: the sharded filter against the
# reference's own outputs (tests/golden/pf_runs.npz, /root/reference/models/
# particle_filter.py:146-220 for the resample it shards)
# ---------------------------------------------------------------------------
def _sv_models(name):
    if name.startswith("sv_logsq"):
        return M.SVTransition(0.95), M.SVLogSqObservation(1.0)
    return M.L96Transition(8.0, 0.01, 40), M.SelectObservation(np.arange(0, 40, 4), 40)


@pytest.mark.parametrize("name,W", [("sv_logsq_reg", 2), ("sv_logsq_reg", 4), ("sv_logsq", 4), ("l96", 2),
                                    ("l96", 4)])
def test_host_replay_shards_match_reference(name, W, golden_runs, golden_sv, golden_l96, golden_mat):
    """W NumPy shards (fp64) driven by the reference's NumPy draw stream reproduce the
    reference's run: identical decisions, means / Neff within 1e-9 (the shard CDF segments are
    rescaled pieces of the global CDF: ancestors agree except at exact ties)."""
    from tests import pf_cases
    ssm, Z, controls, kw = pf_cases.build(name, golden_sv, golden_l96, golden_mat, golden_runs)
    ref = pf_cases.golden(golden_runs, name)
    g, h = _sv_models(name)
    pf = SH.ShardedParticleFilter(g, h, ssm.Q, ssm.R, Np=kw["Np"], resample_thresh=kw["thresh"],
                                  regularize_after_resample=kw["reg"], n_shards=W, rng_mode="host",
                                  rng=np.random.default_rng(kw["seed"]), shard_factory=shard_oracle.factory(ssm))
    pf.initialize(np.asarray(kw["mean0"], float), np.asarray(kw["cov0"], float))
    means, neff, flags = pf.run(Z)
    assert np.array_equal(flags, ref["flags"])
    np.testing.assert_allclose(means, ref["means"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(neff, ref["neff"], rtol=1e-9)
    parts = np.concatenate([pf.local_particles()[s] for s in range(W)])
    np.testing.assert_allclose(parts, ref["final_particles"], rtol=1e-9, atol=1e-9)


def test_host_replay_across_ranks_needs_a_shared_generator():
    """rng_mode='host' with a communicator: every rank must replay the same draw stream, so an
    implicit unseeded Generator per rank is refused (advisor finding)."""
    class _Comm:
        world, rank = 2, 0

    ssm = ssm_oracle.sv_logsq(0.95, 0.2, 1.0)
    with pytest.raises(ValueError, match="seeded identically"):
        SH.ShardedParticleFilter(M.SVTransition(0.95), M.SVLogSqObservation(1.0), ssm.Q, ssm.R, Np=2000,
                                 comm=_Comm(), rng_mode="host")
