"""Within-filter sharding on the GPU (include/pf_shard.h, -m gpu, MI355X).

W device shards of one SIR filter run in one process on one GPU (the multi-process path is
the same orchestrator over torch.distributed; see tests/test_sharded.py for gloo).  Shards
draw the Philox normals of their global particle indices, so:

* W = 1 equals the unsharded engine (ParticleFilterBatch, same seed): resample decisions
  identical, particles within 1e-12 (fp64);
* W = 2, 4 follow W = 1 to reduction-order rounding: fp64 means / particles within 1e-9,
  Neff rtol 1e-9, decisions identical; fp32 within 2e-4 until the first decision flip.
"""

import numpy as np
import pytest

from particle_filters_amd import models as M
from particle_filters_amd import sharded as SH
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from particle_filters_amd import _native
    assert _native.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def sv(golden_sv, T=60):
    Z = np.log(golden_sv["Y0"][1:T + 1] ** 2)[:, None]
    return M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Z, [0.0], [[0.5]]


def l96(golden_l96, T=20):
    g, h = M.L96Transition(8.0, 0.01, 40), M.SelectObservation(np.arange(0, 40, 4), 40)
    return g, h, 0.01 * np.eye(40), np.eye(10), golden_l96["obs"][1:T + 1], golden_l96["ensemble"][0, 0], 2 * np.eye(40)


def run_sharded(spec, W, Np, precision="fp64", reg=False, seed=11):
    g, h, Q, R, Z, m0, c0 = spec
    pf = SH.ShardedParticleFilter(g, h, Q, R, Np=Np, resample_thresh=0.5, regularize_after_resample=reg, seed=seed,
                                  precision=precision, n_shards=W)
    pf.initialize(m0, c0)
    means, neff, flags = pf.run(Z)
    parts = np.concatenate([pf.local_particles()[k] for k in range(W)])
    pf.close()
    return means, neff, flags, parts


@pytest.mark.parametrize("reg", [False, True])
def test_one_shard_equals_unsharded_engine(golden_sv, reg):
    spec = sv(golden_sv)
    g, h, Q, R, Z, m0, c0 = spec
    b = ParticleFilterBatch(g, h, Q, R, Np=20000, n_replicates=1, seed=11, resample_thresh=0.5,
                            regularize_after_resample=reg, precision="fp64")
    b.initialize(m0, c0)
    res = b.run(Z)
    means, neff, flags, parts = run_sharded(spec, 1, 20000, reg=reg)
    assert flags.sum() >= 3
    np.testing.assert_array_equal(flags, res.flags[:, 0])
    np.testing.assert_allclose(parts, b.particles()[0], rtol=0, atol=1e-12)
    pre = ~flags  # weighted means of non-resample steps are the unsharded update's outputs
    np.testing.assert_allclose(means[pre], res.means[pre, 0], rtol=0, atol=1e-12)


@pytest.mark.parametrize("W", [2, 4])
@pytest.mark.parametrize("reg", [False, True])
def test_shards_follow_one_shard_sv(golden_sv, W, reg):
    spec = sv(golden_sv)
    m1, n1, f1, x1 = run_sharded(spec, 1, 40000, reg=reg)
    mW, nW, fW, xW = run_sharded(spec, W, 40000, reg=reg)
    assert f1.sum() >= 3
    np.testing.assert_array_equal(fW, f1)
    np.testing.assert_allclose(mW, m1, rtol=0, atol=1e-9)
    np.testing.assert_allclose(nW, n1, rtol=1e-9)
    np.testing.assert_allclose(xW, x1, rtol=0, atol=1e-9)


def test_shards_follow_one_shard_l96(golden_l96):
    spec = l96(golden_l96)
    m1, n1, f1, x1 = run_sharded(spec, 1, 8000)
    m2, n2, f2, x2 = run_sharded(spec, 2, 8000)
    assert f1.sum() >= 3
    np.testing.assert_array_equal(f2, f1)
    np.testing.assert_allclose(m2, m1, rtol=0, atol=1e-8)
    np.testing.assert_allclose(x2, x1, rtol=0, atol=1e-8)


def test_fp32_shards(golden_sv):
    spec = sv(golden_sv, T=40)
    m1, n1, f1, _ = run_sharded(spec, 1, 40000, precision="fp32")
    m2, n2, f2, _ = run_sharded(spec, 2, 40000, precision="fp32")
    first = int(np.argmax(f1 != f2)) if np.any(f1 != f2) else len(f1)
    assert first >= 5
    np.testing.assert_allclose(m2[:first], m1[:first], rtol=0, atol=2e-4)


def _gloo_worker(rank, world, port, q):
    import os

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = np.load(os.path.join(os.path.dirname(__file__), "golden", "sv_data.npz"))
        spec = sv({"Y0": d["Y0"]})
        g, h, Q, R, Z, m0, c0 = spec
        pf = SH.ShardedParticleFilter(g, h, Q, R, Np=40000, resample_thresh=0.5, seed=11, precision="fp64",
                                      comm=SH.DistComm(), device=0)
        pf.initialize(m0, c0)
        means, neff, flags = pf.run(Z)
        q.put((rank, means, neff, flags, pf.local_particles()[rank]))
        pf.close()
    finally:
        dist.destroy_process_group()


def test_two_processes_gloo_one_gpu(golden_sv):
    """DistComm (host-staged gloo point-to-point) with two ranks sharing the GPU == the
    in-process two-shard filter."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=100) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m2, n2, f2, x2 = run_sharded(sv(golden_sv), 2, 40000)
    for rank, means, neff, flags, parts in out:
        np.testing.assert_array_equal(flags, f2)
        np.testing.assert_allclose(means, m2, rtol=0, atol=1e-12)
        np.testing.assert_allclose(neff, n2, rtol=1e-12)
    np.testing.assert_allclose(np.concatenate([o[4] for o in out]), x2, rtol=0, atol=1e-12)


@pytest.mark.parametrize("name,W", [("sv_logsq_reg", 2), ("sv_logsq_reg", 4), ("sv_logsq", 4), ("l96", 2),
                                    ("l96", 4)])
def test_host_replay_device_shards_match_reference(name, W, golden_runs, golden_sv, golden_l96, golden_mat):
    """The sharded engine against the REFERENCE (tests/golden/pf_runs.npz, made by importing
    /root/reference/models/particle_filter.py): W fp64 device shards replaying the reference's
    NumPy draw stream (each shard gets its rows of the initial / process / jitter normals, every
    rank the systematic U) reproduce the run at test_replay_fp64_matches_reference's tolerances:
    identical decisions, means rtol 1e-9, Neff rtol 1e-9, final particles 1e-9."""
    from tests import pf_cases
    ssm, Z, controls, kw = pf_cases.build(name, golden_sv, golden_l96, golden_mat, golden_runs)
    ref = pf_cases.golden(golden_runs, name)
    if name.startswith("sv_logsq"):
        g, h = M.SVTransition(0.95), M.SVLogSqObservation(1.0)
    else:
        g, h = M.L96Transition(8.0, 0.01, 40), M.SelectObservation(np.arange(0, 40, 4), 40)
    pf = SH.ShardedParticleFilter(g, h, ssm.Q, ssm.R, Np=kw["Np"], resample_thresh=kw["thresh"],
                                  regularize_after_resample=kw["reg"], precision="fp64", n_shards=W,
                                  rng_mode="host", rng=np.random.default_rng(kw["seed"]))
    pf.initialize(np.asarray(kw["mean0"], float), np.asarray(kw["cov0"], float))
    means, neff, flags = pf.run(Z)
    parts = np.concatenate([pf.local_particles()[k] for k in range(W)])
    pf.close()
    assert np.array_equal(flags, ref["flags"]), f"{name} W={W}: resample decisions differ"
    np.testing.assert_allclose(means, ref["means"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(neff, ref["neff"], rtol=1e-9)
    np.testing.assert_allclose(parts, ref["final_particles"], rtol=1e-9, atol=1e-9)
