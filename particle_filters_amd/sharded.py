"""One SIR particle filter whose particles are sharded over several GPUs.

Mirrors ``ParticleFilter`` (``/root/reference/models/particle_filter.py``, cited ``pf.py:LINE``):
``initialize`` (110-132), ``predict`` (223-237), ``update`` (239-269), ``step`` (271-287),
``effective_sample_size`` (134-144) — for a filter of ``Np`` particles split into W equal
shards (one per rank, or several in one process).  Device work per shard goes through
``include/pf_shard.h``; this module is the host orchestrator:

* **weights** — each shard re-weights with the GLOBAL normaliser of the previous weights and
  reports ``(lse_g, Neff_g, mean_g, cov_g)``; the global ``lse = logsumexp_g lse_g``, shard
  masses ``W_g = e^(lse_g - lse)``, ``Neff = 1 / sum_g W_g^2 / Neff_g`` and the weighted
  moments follow exactly (pf.py:254-267).  One all-gather of ``2 + nx + nx^2`` doubles per
  shard per step — the only collective on non-resample steps.
* **resample** (Neff < thresh * Np, strict, pf.py:198-203; systematic, pf.py:146-171): shard g
  owns the global CDF segment ``[B_g, B_{g+1})``, ``B_g = sum_{h<g} W_h / sum W``, hence the
  positions ``(U + i) / Np`` with ``i`` in ``[a_g, a_{g+1})``.  Rank d must end up with slots
  ``[d N_loc, (d+1) N_loc)``: W rounds of pairwise exchanges (round k: send to ``r + k``,
  receive from ``r - k``) move exactly the overlapping slot ranges, at most N_loc rows per
  round and buffer.  Then the shard adopts its rows (uniform weights, optional
  ``0.001 chol(Q)`` jitter, pf.py:212-218).

Random numbers are the unsharded filter's: a shard draws the Philox normals of its GLOBAL
particle indices and every rank derives the same systematic offset U, so a W-shard filter
follows the 1-shard filter to reduction-order rounding.  Communication: ``comm=None`` runs all
W shards in this process (one GPU, or tests); ``comm=DistComm()`` uses ``torch.distributed``
(RCCL over xGMI with ``nccl``, host-staged with ``gloo``) with one shard per rank.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _native as N
from . import models as M

Array = np.ndarray


@dataclass
class ShardedState:
    """PFState of the whole filter (pf.py:27-49) — the particles stay on their shards."""

    mean: Array
    cov: Array
    t: int
    neff: float
    resampled: bool


# ---------------------------------------------------------------------------- host algebra
def combine(lse: Array, neff: Array, means: Array, covs: Array):
    """Global (lse, Neff, mean, cov, shard masses) from per-shard summaries, in shard order."""
    lse = np.asarray(lse, float)
    m = float(np.max(lse))
    e = np.exp(lse - m)
    tot = float(np.sum(e))
    W = e / tot
    g_lse = m + np.log(tot)
    g_neff = 1.0 / float(np.sum(W * W / np.asarray(neff, float)))
    mean = np.einsum("g,gd->d", W, means)
    dm = means - mean[None, :]
    cov = np.einsum("g,gde->de", W, covs) + np.einsum("g,gd,ge->de", W, dm, dm)
    return g_lse, g_neff, mean, 0.5 * (cov + cov.T), W


def boundaries(W: Array) -> Array:
    """B_0 = 0 <= B_1 <= ... <= B_W = 1: exclusive prefix of the shard masses (fixed order)."""
    c = np.concatenate([[0.0], np.cumsum(np.asarray(W, float))])
    B = c / c[-1]
    B[-1] = 1.0
    return B


def slot_starts(B: Array, U: float, n_total: int) -> Array:
    """a_g = #{i : (U + i) / n_total < B_g}, evaluated with the comparisons the slots are
    defined by (so the W ranges partition [0, n_total) identically on every rank)."""
    a = np.empty(len(B), dtype=np.int64)
    for g, b in enumerate(B):
        if g == 0:
            a[g] = 0
            continue
        if g == len(B) - 1:
            a[g] = n_total
            continue
        k = int(min(max(np.ceil(b * n_total - U), 0), n_total))
        while k > 0 and (U + (k - 1)) / n_total >= b:
            k -= 1
        while k < n_total and (U + k) / n_total < b:
            k += 1
        a[g] = k
    return np.maximum.accumulate(a)


def overlap(a: Array, g: int, d: int, n_loc: int):
    """Global slots of source shard g that destination shard d owns: (start, count)."""
    lo = max(int(a[g]), d * n_loc)
    hi = min(int(a[g + 1]), (d + 1) * n_loc)
    return lo, max(0, hi - lo)


# ---------------------------------------------------------------------------- shards
class HipShard:
    """One shard = one pf_handle (R = 1) on a device; row buffers are torch device tensors."""

    def __init__(self, desc, keep, nx, n_loc, n_total, rank, thresh, regularize, seed, precision, device,
                 kernel_path="auto"):
        import torch

        self._torch = torch
        self._keep = keep
        self.nx = nx
        self.n_loc = n_loc
        self.device = device
        self.dtype = torch.float64 if precision == "fp64" else torch.float32
        lib = N.load()
        opts = N.Opts(n_loc, 1, N.PF_RESAMPLE_SYSTEMATIC, float(thresh), int(bool(regularize)),
                      N.PF_PRECISION_FP64 if precision == "fp64" else N.PF_PRECISION_FP32, int(seed), int(device), 0,
                      M.kernel_path_code(kernel_path))
        self._h = N.C.c_void_p()
        N.check(lib.pf_create(N.C.byref(desc), N.C.byref(opts), N.C.byref(self._h)), "pf_create")
        N.check(lib.pf_shard_configure(self._h, int(n_total), int(rank)), "pf_shard_configure")
        dev = torch.device("cuda", device)
        self.outbox = torch.empty((n_loc, nx), dtype=self.dtype, device=dev)
        self.inbox = torch.empty((n_loc, nx), dtype=self.dtype, device=dev)

    def close(self):
        if N._lib is not None and getattr(self, "_h", None) is not None and self._h.value:
            N._lib.pf_destroy(self._h)
        self._h = None

    def initialize(self, mean, cov, replay=None):
        rp = None if replay is None else np.ascontiguousarray(replay, dtype=float)
        N.check(N.load().pf_initialize(self._h, N.dptr(mean), N.dptr(cov), N.dptr(rp)), "pf_initialize")

    def predict(self, u, replay=None):
        rp = None if replay is None else np.ascontiguousarray(replay, dtype=float)
        N.check(N.load().pf_predict(self._h, N.dptr(u), N.dptr(rp)), "pf_predict")

    def update(self, z, lse_prev):
        st = N.ShardStats()
        mean = np.empty(self.nx)
        cov = np.empty((self.nx, self.nx))
        N.check(N.load().pf_shard_update(self._h, N.dptr(z), float(lse_prev), N.C.byref(st), N.dptr(mean),
                                         N.dptr(cov)), "pf_shard_update")
        return st.lse, st.neff, st.U, mean, cov

    def offspring(self, U, lo, mass, a, n):
        """rows of global slots [a, a + n) in self.outbox[:n] (device)."""
        N.check(N.load().pf_shard_offspring(self._h, float(U), float(lo), float(mass), int(a), int(n),
                                            N.C.c_void_p(self.outbox.data_ptr())), "pf_shard_offspring")
        return self.outbox[:n]

    def adopt(self, jitter=None):
        mean = np.empty(self.nx)
        cov = np.empty((self.nx, self.nx))
        jp = None if jitter is None else np.ascontiguousarray(jitter, dtype=float)
        N.check(N.load().pf_shard_adopt(self._h, N.C.c_void_p(self.inbox.data_ptr()), N.dptr(jp), N.dptr(mean),
                                        N.dptr(cov)), "pf_shard_adopt")
        return mean, cov

    def sync_torch(self):
        self._torch.cuda.synchronize(self.device)

    def particles(self) -> Array:
        out = np.empty((self.n_loc, self.nx))
        N.check(N.load().pf_get_particles(self._h, N.dptr(out)), "pf_get_particles")
        return out

    def log_weights(self) -> Array:
        out = np.empty(self.n_loc)
        N.check(N.load().pf_get_weights(self._h, None, N.dptr(out)), "pf_get_weights")
        return out


class DistComm:
    """torch.distributed process group: one shard per rank (nccl = RCCL on device tensors; gloo
    stages through host memory)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)

    def _dev(self, t):
        return t if self.backend == "nccl" else t.cpu()

    def allgather(self, vec: Array, like) -> Array:
        torch = like._torch if hasattr(like, "_torch") else __import__("torch")
        x = torch.as_tensor(np.asarray(vec, float), dtype=torch.float64)
        if self.backend == "nccl":
            x = x.cuda()
        out = [torch.empty_like(x) for _ in range(self.world)]
        self.dist.all_gather(out, x, group=self.group)
        return np.stack([o.cpu().numpy() for o in out])

    def sendrecv(self, send, dst, recv, src):
        """send rows to dst and receive rows into `recv` from src (either may be None)."""
        ops = []
        s_buf = r_buf = None
        if send is not None and send.shape[0] > 0:
            s_buf = self._dev(send.contiguous())
            ops.append(self.dist.P2POp(self.dist.isend, s_buf, dst, self.group))
        if recv is not None and recv.shape[0] > 0:
            r_buf = recv if self.backend == "nccl" else recv.new_empty(recv.shape, device="cpu")
            ops.append(self.dist.P2POp(self.dist.irecv, r_buf, src, self.group))
        if ops:
            for req in self.dist.batch_isend_irecv(ops):
                req.wait()
        if r_buf is not None and r_buf is not recv:
            recv.copy_(r_buf)


class ShardedParticleFilter:
    """SIR filter of ``Np`` particles in W shards (drop-in for pf.py:53-287 beyond one GPU).

    ``comm=None``: ``n_shards`` shards in this process (``devices`` cycles over the visible
    GPUs, default all on ``device``).  ``comm=DistComm()``: this rank's shard of a
    ``world``-rank filter on ``device``.  ``shard_factory`` builds one shard (default
    :class:`HipShard`); the CPU tests substitute the NumPy shard of ``oracle/``.

    ``rng_mode="host"`` replays the reference's own draw stream (``rng``, a NumPy Generator
    used exactly as pf.py:128,160,217,236 use it): every rank draws the full ``(Np, nx)``
    normals / the systematic U and hands each shard its rows — the parity mode, pinned to the
    reference's outputs (tests/test_gpu_sharded.py).  ``"device"`` draws Philox numbers of
    the global particle indices on the shards."""

    def __init__(self, g, h, Q, R, *, Np: int, resample_thresh: float = 0.5, regularize_after_resample: bool = False,
                 seed: int = 0, precision: str = "fp32", comm: Optional[DistComm] = None, n_shards: int = 1,
                 device: int = 0, devices: Optional[List[int]] = None, shard_factory=None, rng=None,
                 rng_mode: str = "device", kernel_path: str = "auto"):
        if not M.is_device_model(g, h):
            raise NotImplementedError("ShardedParticleFilter needs particle_filters_amd.models g / h")
        self.g, self.h = g, h
        self.Q = np.asarray(Q, float)
        self.R = np.asarray(R, float)
        self.nx, self.nz = self.Q.shape[0], self.R.shape[0]
        self.Np = int(Np)
        self.resample_thresh = float(resample_thresh)
        self.regularize_after_resample = bool(regularize_after_resample)
        self.comm = comm
        self.W = comm.world if comm is not None else int(n_shards)
        if rng_mode not in ("device", "host"):
            raise ValueError("rng_mode must be 'device' or 'host'")
        self.rng_mode = rng_mode
        if rng_mode == "host" and comm is not None and rng is None:
            # every rank replays the SAME reference draw stream (U, normals of all Np rows) and
            # takes its own rows: an unseeded Generator per rank would give the ranks different
            # systematic U / slot ranges and mismatched exchanges
            raise ValueError("rng_mode='host' across ranks needs rng: a Generator seeded identically on every rank")
        self.rng = np.random.default_rng() if rng is None else rng
        if self.Np % self.W:
            raise ValueError("Np must be W * N_loc")
        if rng_mode == "device" and self.nx == 1 and (self.Np // self.W) % 4:
            raise ValueError("device-RNG shards of a scalar state need N_loc % 4 == 0 (Philox groups of 4)")
        self.n_loc = self.Np // self.W
        self.mine = [comm.rank] if comm is not None else list(range(self.W))
        devs = devices or [device]
        self._desc, self._keep = M.describe(g, h, self.Q, self.R)
        make = shard_factory or (lambda **kw: HipShard(**kw))
        self.shards = {}
        for j, r in enumerate(self.mine):
            self.shards[r] = make(desc=self._desc, keep=self._keep, nx=self.nx, n_loc=self.n_loc, n_total=self.Np,
                                  rank=r, thresh=self.resample_thresh, regularize=self.regularize_after_resample,
                                  seed=seed, precision=precision, device=devs[j % len(devs)] if comm is None else device,
                                  kernel_path=kernel_path)
        self.state: Optional[ShardedState] = None
        self._lse_prev = 0.0
        self._neff = float(self.Np)
        self.t = 0

    def close(self):
        for s in self.shards.values():
            s.close()
        self.shards = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ host replay
    def _host_normals(self):
        """The reference's (Np, nx) normal draw (pf.py:128, 217, 236), or None in device mode."""
        if self.rng_mode != "host":
            return None
        return np.asarray(self.rng.standard_normal((self.Np, self.nx)), dtype=float)

    def _rows(self, a, g):
        return None if a is None else a[g * self.n_loc:(g + 1) * self.n_loc]

    # ------------------------------------------------------------------ collectives
    def _gather(self, rows: dict) -> Array:
        """per-shard vectors of every shard, in shard order."""
        if self.comm is None:
            return np.stack([rows[g] for g in range(self.W)])
        (r, v), = rows.items()
        return self.comm.allgather(v, self.shards[r])

    def _resample(self, U: float, W: Array):
        if self.rng_mode == "host":
            U = float(self.rng.random())  # pf.py:160
        B = boundaries(W)
        a = slot_starts(B, U, self.Np)
        mass = np.diff(B)
        if self.comm is None:
            for d in range(self.W):  # destination-major: each shard's outbox is reused per copy
                dst = self.shards[d]
                for g in range(self.W):
                    lo, n = overlap(a, g, d, self.n_loc)
                    if n:
                        rows = self.shards[g].offspring(U, B[g], mass[g], lo, n)
                        dst.inbox[lo - d * self.n_loc: lo - d * self.n_loc + n].copy_(rows)
                        if hasattr(dst, "sync_torch"):
                            dst.sync_torch()
        else:
            r = self.comm.rank
            me = self.shards[r]
            for k in range(self.W):
                dst, src = (r + k) % self.W, (r - k) % self.W
                s_lo, s_n = overlap(a, r, dst, self.n_loc)
                r_lo, r_n = overlap(a, src, r, self.n_loc)
                send = me.offspring(U, B[r], mass[r], s_lo, s_n) if s_n else None
                off = r_lo - r * self.n_loc
                recv = me.inbox[off:off + r_n] if r_n else None
                if k == 0:
                    if r_n:
                        recv.copy_(send)
                else:
                    self.comm.sendrecv(send, dst, recv, src)
                if hasattr(me, "sync_torch"):
                    me.sync_torch()
        jit = self._host_normals() if self.regularize_after_resample else None  # pf.py:212-218
        stats = {}
        for g, s in self.shards.items():
            m, c = s.adopt(self._rows(jit, g))
            stats[g] = np.concatenate([m, c.ravel()])
        allst = self._gather(stats)
        means = allst[:, :self.nx]
        covs = allst[:, self.nx:].reshape(self.W, self.nx, self.nx)
        mean = means.mean(axis=0)  # equal shard sizes, uniform weights
        dm = means - mean[None, :]
        cov = covs.mean(axis=0) + np.einsum("gd,ge->de", dm, dm) / self.W
        return mean, 0.5 * (cov + cov.T)

    # ------------------------------------------------------------------ API (pf.py)
    def initialize(self, mean, cov) -> ShardedState:
        """pf.py:110-132: particles ~ N(mean, cov + 1e-10 I) on every shard, uniform weights."""
        m = np.ascontiguousarray(np.asarray(mean, float).reshape(self.nx))
        c = np.ascontiguousarray(np.asarray(cov, float).reshape(self.nx, self.nx))
        n0 = self._host_normals()
        for g, s in self.shards.items():
            s.initialize(m, c, self._rows(n0, g))
        self.t = 0
        self._lse_prev = 0.0
        self._neff = float(self.Np)
        self.state = ShardedState(m.copy(), c.copy(), 0, float(self.Np), False)
        return self.state

    def _need_init(self):
        if self.state is None:
            raise AssertionError("Filter not initialized.")

    def predict(self, u=None) -> None:
        """pf.py:223-237."""
        self._need_init()
        uu = None if u is None else np.ascontiguousarray(np.asarray(u, float).reshape(self.nx))
        n = self._host_normals()
        for g, s in self.shards.items():
            s.predict(uu, self._rows(n, g))

    def update(self, z) -> ShardedState:
        """pf.py:239-269 over all shards: global weights, Neff, decision, resample, moments."""
        self._need_init()
        zz = np.ascontiguousarray(np.asarray(z, float).reshape(self.nz))
        rows = {}
        U = None
        for g, s in self.shards.items():
            lse, neff, U, mean, cov = s.update(zz, self._lse_prev)
            rows[g] = np.concatenate([[lse, neff], mean, cov.ravel()])
        allv = self._gather(rows)
        lse_g, neff_g = allv[:, 0], allv[:, 1]
        means = allv[:, 2:2 + self.nx]
        covs = allv[:, 2 + self.nx:].reshape(self.W, self.nx, self.nx)
        g_lse, g_neff, mean, cov, W = combine(lse_g, neff_g, means, covs)
        self._neff = g_neff
        resampled = g_neff < self.resample_thresh * self.Np
        if resampled:
            mean, cov = self._resample(U, W)
            self._lse_prev = 0.0
            self._neff = float(self.Np)
        else:
            self._lse_prev = g_lse
        self.t += 1
        self.state = ShardedState(mean, cov, self.t, g_neff, bool(resampled))
        return self.state

    def step(self, z, u=None) -> ShardedState:
        """pf.py:271-287."""
        self.predict(u)
        return self.update(z)

    def effective_sample_size(self) -> float:
        """pf.py:134-144: 1 / sum w^2 of the state weights (Np after a resample)."""
        self._need_init()
        return float(self._neff)

    def run(self, Z, U=None):
        """The driver loop over Z: means [T][nx], Neff of the weights before resampling [T], flags [T]."""
        Z = np.asarray(Z, float).reshape(-1, self.nz)
        T = Z.shape[0]
        means = np.empty((T, self.nx))
        neff = np.empty(T)
        flags = np.zeros(T, dtype=bool)
        for t in range(T):
            st = self.step(Z[t], None if U is None else U[t])
            means[t], neff[t], flags[t] = st.mean, st.neff, st.resampled
        return means, neff, flags

    def local_particles(self) -> dict:
        """{shard: particles [N_loc][nx]} of the shards this process holds."""
        return {g: s.particles() for g, s in self.shards.items()}
