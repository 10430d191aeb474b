"""Multi-process (gloo, CPU) tests of the replicate-sharding path.

The engine itself needs a GPU; these cover the host logic that decides which
replicates each rank runs (and hence its Philox ``replicate_base``) and the one
collective of the path, the all-gather of per-replicate summaries, with
world_size 2 (and 3 for ragged shards) over gloo on 127.0.0.1.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from particle_filters_amd import distributed as D
from particle_filters_amd.batch import RunResult


@pytest.mark.parametrize("R", [0, 1, 2, 5, 8, 64, 65])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shards_partition_replicates(R, world):
    ids = []
    for r in range(world):
        base, count = D.shard_replicates(R, world, r)
        assert count >= 0
        ids.extend(range(base, base + count))
    assert ids == list(range(R))  # contiguous, ordered, each exactly once
    counts = [D.shard_replicates(R, world, r)[1] for r in range(world)]
    assert max(counts) - min(counts) <= 1


def test_shard_rejects_bad_requests():
    with pytest.raises(ValueError):
        D.shard_replicates(4, 0, 0)
    with pytest.raises(ValueError):
        D.shard_replicates(4, 2, 2)


def _fake_result(ids, T, nx):
    """Summaries whose every value encodes (replicate id, step, field)."""
    R = len(ids)
    ids = np.asarray(ids, float)
    t = np.arange(T, dtype=float)[:, None]
    means = np.stack([1000 * ids[None, :] + t + 0.1 * d for d in range(nx)], axis=-1)
    neff = 7.0 * ids[None, :] + t
    flags = ((ids[None, :] + t) % 3 == 0)
    lnorm = -ids[None, :] - 0.5 * t
    covs = (means[:, :, :, None] * 0.01 + np.arange(nx * nx, dtype=float).reshape(nx, nx))  # [T][R][nx][nx]
    return RunResult(means.reshape(T, R, nx), covs.reshape(T, R, nx, nx), neff.reshape(T, R), flags.reshape(T, R),
                     lnorm.reshape(T, R), np.where(flags, 50.0, neff).reshape(T, R))


def test_pack_roundtrip():
    r = _fake_result([3, 4, 5], T=6, nx=2)
    u = D.unpack_summaries(D.pack_summaries(r, 2), 2, n_particles=50)
    assert "covs" in D.SUMMARY_FIELDS
    np.testing.assert_array_equal(u.means, r.means)
    np.testing.assert_array_equal(u.covs, r.covs)
    np.testing.assert_array_equal(u.neff, r.neff)
    np.testing.assert_array_equal(u.flags, r.flags)
    np.testing.assert_array_equal(u.log_norm, r.log_norm)
    np.testing.assert_array_equal(u.ess, r.ess)
    r.covs = None  # a run without covariances packs the narrow rows
    u = D.unpack_summaries(D.pack_summaries(r, 2), 2, n_particles=50)
    assert u.covs is None and np.array_equal(u.means, r.means)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, R, T, nx, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        base, count = D.shard_replicates(R, world, rank)
        local = _fake_result(list(range(base, base + count)), T, nx)
        packed = torch.from_numpy(D.pack_summaries(local, nx))
        allp = D.gather_summaries(packed, R)
        res = D.unpack_summaries(allp.numpy(), nx, n_particles=50)
        ref = _fake_result(list(range(R)), T, nx)
        ok = (np.array_equal(res.means, ref.means) and np.array_equal(res.covs, ref.covs)
              and np.array_equal(res.neff, ref.neff)
              and np.array_equal(res.flags, ref.flags) and np.array_equal(res.log_norm, ref.log_norm))
        # the bench's timing reduction: max over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, ok, float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,R", [(2, 4), (2, 5), (3, 7), (2, 1)])
def test_gloo_gather_global_replicate_order(world, R):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, R, 9, 3, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, tmax in out:
        assert ok, f"rank {rank}: gathered summaries out of replicate order"
        assert tmax == float(world)


def _worker_flat(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        local = torch.arange(n, dtype=torch.float64) + 1000.0 * rank  # a rank's flat summary buffer
        out = torch.empty(world * n, dtype=torch.float64)
        D.gather_summary_buffers(out, local)
        ref = torch.cat([torch.arange(n, dtype=torch.float64) + 1000.0 * k for k in range(world)])
        q.put((rank, bool(torch.equal(out, ref))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_flat_summary_buffers_in_rank_order(world):
    """bench.py's timed-region gather: one all_gather_into_tensor of equal flat buffers."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_flat, args=(r, world, port, 37, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok in out:
        assert ok, f"rank {rank}: flat buffers out of rank order"
