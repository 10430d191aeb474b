"""Replicate sharding across GPUs.

The SIR path has no per-step exchange between independent Monte-Carlo
replicates, so multi-GPU is data-parallel over replicates with exactly one
collective at the end: an all-gather of each replicate's posterior summaries
(means, covariances - part of the reference's PFState every update, pf.py:266-268 -, Neff,
resample flags, log normaliser).  One process per GPU;
``torch.distributed`` with backend "nccl" (RCCL over xGMI) on GPUs, "gloo" in the
CPU tests.

Replicate ids are global: rank r runs the contiguous block
``shard_replicates(R, world, r)`` and passes its first id as the engine's
``replicate_base`` (the Philox counter word), so replicate k produces bitwise
the same trajectory whichever rank or world size runs it.
"""

from __future__ import annotations

from typing import List, Tuple

import numpy as np

from .batch import RunResult

SUMMARY_FIELDS = ("means", "covs", "neff", "flags", "log_norm")


def summary_width(nx: int, with_cov: bool = True) -> int:
    """float64 words per replicate and step of a packed summary row."""
    return nx + (nx * nx if with_cov else 0) + 3


def shard_replicates(n_replicates: int, world: int, rank: int) -> Tuple[int, int]:
    """(first global replicate id, count) owned by ``rank``: contiguous blocks, the
    first ``n_replicates % world`` ranks take one extra."""
    if world <= 0 or not 0 <= rank < world or n_replicates < 0:
        raise ValueError(f"bad shard request R={n_replicates} world={world} rank={rank}")
    q, r = divmod(n_replicates, world)
    count = q + (1 if rank < r else 0)
    base = rank * q + min(rank, r)
    return base, count


def pack_summaries(res: RunResult, nx: int) -> np.ndarray:
    """[R_local][T][summary_width] float64: means [nx], covariance [nx * nx] (when the run has
    them), Neff, flag, log normaliser."""
    T, R = res.neff.shape
    wc = res.covs is not None
    out = np.empty((R, T, summary_width(nx, wc)))
    out[:, :, :nx] = np.transpose(res.means, (1, 0, 2))
    o = nx
    if wc:
        out[:, :, nx:nx + nx * nx] = np.transpose(res.covs.reshape(T, R, nx * nx), (1, 0, 2))
        o += nx * nx
    out[:, :, o] = res.neff.T
    out[:, :, o + 1] = res.flags.T.astype(float)
    out[:, :, o + 2] = res.log_norm.T
    return out


def unpack_summaries(packed: np.ndarray, nx: int, n_particles: int) -> RunResult:
    """Inverse of pack_summaries for the gathered [R_total][T][summary_width] block."""
    wc = packed.shape[2] == summary_width(nx, True)
    if not wc and packed.shape[2] != summary_width(nx, False):
        raise ValueError(f"summary rows of width {packed.shape[2]} do not fit nx = {nx}")
    means = np.ascontiguousarray(np.transpose(packed[:, :, :nx], (1, 0, 2)))
    o = nx
    covs = None
    if wc:
        Rt, T = packed.shape[:2]
        covs = np.ascontiguousarray(np.transpose(packed[:, :, nx:nx + nx * nx], (1, 0, 2))).reshape(T, Rt, nx, nx)
        o += nx * nx
    neff = np.ascontiguousarray(packed[:, :, o].T)
    flags = packed[:, :, o + 1].T > 0.5
    lnorm = np.ascontiguousarray(packed[:, :, o + 2].T)
    ess = np.where(flags, float(n_particles), neff)
    return RunResult(means, covs, neff, flags, lnorm, ess)


def gather_summaries(local, n_replicates: int, group=None):
    """All-gather per-replicate summary rows into global replicate order.

    ``local`` is a torch tensor [R_local][...] on the collective's device (CUDA
    for nccl, CPU for gloo).  Ranks may own different counts, so blocks are
    padded to the largest shard for the collective and trimmed afterwards.
    Returns a tensor [n_replicates][...].
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    base, count = shard_replicates(n_replicates, world, rank)
    if local.shape[0] != count:
        raise ValueError(f"rank {rank} holds {local.shape[0]} replicates, shard says {count}")
    width = shard_replicates(n_replicates, world, 0)[1]
    pad = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:count] = local
    blocks: List = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(blocks, pad.contiguous(), group=group)
    parts = [blocks[r][:shard_replicates(n_replicates, world, r)[1]] for r in range(world)]
    return torch.cat(parts, dim=0)


def gather_summary_buffers(out, local, group=None):
    """All-gather equal-sized flat per-rank summary buffers with ONE collective:
    ``out`` [world * local.numel()] receives rank k's ``local`` at block k (RCCL
    all_gather_into_tensor; no padding or packing kernels).  For ranks that own equal
    replicate counts, e.g. bench.py's fixed replicates per rank; ``gather_summaries``
    handles uneven shards."""
    import torch.distributed as dist

    dist.all_gather_into_tensor(out, local, group=group)
    return out


def run_sharded(g, h, Q, R, Z, *, mean0, cov0, n_replicates: int, Np: int, group=None,
                device: int = 0, **pf_kwargs) -> RunResult:
    """Run ``n_replicates`` independent filters sharded over the process group and
    return every replicate's summaries on every rank (global replicate order)."""
    import torch
    import torch.distributed as dist

    from .batch import ParticleFilterBatch

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    base, count = shard_replicates(n_replicates, world, rank)
    nx = np.asarray(Q).shape[0]
    T = np.asarray(Z).shape[0]
    if count > 0:
        pf = ParticleFilterBatch(g, h, Q, R, Np=Np, n_replicates=count, replicate_base=base,
                                 device=device, **pf_kwargs)
        pf.initialize(mean0, cov0)
        packed = pack_summaries(pf.run(Z), nx)
    else:
        packed = np.zeros((0, T, summary_width(nx, True)))
    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", device) if on_gpu else torch.device("cpu")
    allp = gather_summaries(torch.from_numpy(packed).to(dev), n_replicates, group)
    return unpack_summaries(allp.cpu().numpy(), nx, Np)
