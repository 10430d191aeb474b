"""NumPy shard of a sharded SIR filter — TEST INFRASTRUCTURE ONLY.

The CPU stand-in for ``particle_filters_amd.sharded.HipShard`` (the device shard of
``include/pf_shard.h``), so the host orchestrator and its ``torch.distributed`` exchange
(gloo, world size 2) are tested without a GPU.  Same semantics as the device shard, in fp64:
Philox normals of GLOBAL particle indices (``oracle/philox.py``), the update of
``particle_filter.py:239-263`` with the global normaliser of the previous weights, offspring
rows of global systematic slots (positions mapped into the shard's CDF segment), adoption
with uniform weights and the optional 0.001 chol(Q) jitter; or, in host replay, the
reference's own normals for its rows.  Only ``tests/`` import it.
"""

from __future__ import annotations

import numpy as np
import torch

from oracle import philox


class NumpyShard:
    def __init__(self, ssm, *, nx, n_loc, n_total, rank, thresh, regularize, seed, **_):
        self.regularize = bool(regularize)
        self.ssm = ssm
        self.nx = nx
        self.n_loc = n_loc
        self.n_total = n_total
        self.pbase = rank * n_loc
        self.seed = seed
        self.epoch = 1
        self.ep_res = 0
        self.uniform = True
        self.LQ = np.linalg.cholesky(ssm.Q)
        self.LR = np.linalg.cholesky(ssm.R + 1e-12 * np.eye(ssm.nz))
        self.outbox = torch.empty((n_loc, nx), dtype=torch.float64)
        self.inbox = torch.empty((n_loc, nx), dtype=torch.float64)

    def close(self):
        pass

    def _normals(self, stream, epoch):
        n = philox.normals(self.seed, (self.pbase + self.n_loc) * self.nx, 0, epoch, stream)
        return n[self.pbase * self.nx:].reshape(self.n_loc, self.nx)

    def initialize(self, mean, cov, replay=None):
        L = np.linalg.cholesky(cov + 1e-10 * np.eye(self.nx))
        n = self._normals(philox.STREAM_INIT, self.epoch) if replay is None else np.asarray(replay, float)
        self.x = n @ L.T + mean[None, :]
        self.epoch += 1
        self.l = np.zeros(self.n_loc)
        self.uniform = True

    def predict(self, u, replay=None):
        n = self._normals(philox.STREAM_PROCESS, self.epoch) if replay is None else np.asarray(replay, float)
        self.epoch += 1
        self.x = self.ssm.g_vec(self.x, u) + n @ self.LQ.T

    def _weights(self):
        m = np.max(self.l)
        e = np.exp(self.l - m)
        return e / e.sum(), m + np.log(e.sum())

    def update(self, z, lse_prev):
        y = np.linalg.solve(self.LR, (z[None, :] - self.ssm.h_vec(self.x)).T)
        ll = -0.5 * np.sum(y * y, axis=0)
        prev = np.full(self.n_loc, -np.log(self.n_loc)) if self.uniform else self.l - lse_prev
        self.l = prev + ll
        self.uniform = False
        self.ep_res = self.epoch
        self.epoch += 1
        w, lse = self._weights()
        mean = w @ self.x
        xc = self.x - mean
        cov = (xc.T * w) @ xc
        U = float(philox.uniform53(self.seed, 0, 0, self.ep_res))
        return lse, 1.0 / np.sum(w * w), U, mean, cov

    def offspring(self, U, lo, mass, a, n):
        w, _ = self._weights()
        cdf = np.cumsum(w)
        pos = ((U + np.arange(a, a + n, dtype=np.float64)) / self.n_total - lo) / mass
        j = np.minimum(np.searchsorted(cdf, pos, side="right"), self.n_loc - 1)
        self.outbox[:n] = torch.from_numpy(self.x[j])
        return self.outbox[:n]

    def adopt(self, jitter=None):
        self.x = self.inbox.numpy().copy()
        if self.regularize:  # pf.py:212-218
            try:
                Lq = np.linalg.cholesky(self.ssm.Q)
            except np.linalg.LinAlgError:
                Lq = np.linalg.cholesky(self.ssm.Q + 1e-12 * np.eye(self.nx))
            n = self._normals(philox.STREAM_JITTER, self.ep_res) if jitter is None else np.asarray(jitter, float)
            self.x = self.x + n @ (0.001 * Lq.T)
        self.l = np.zeros(self.n_loc)
        self.uniform = True
        mean = self.x.mean(axis=0)
        xc = self.x - mean
        return mean, xc.T @ xc / self.n_loc

    def particles(self):
        return self.x.copy()


def factory(ssm):
    return lambda **kw: NumpyShard(ssm, **kw)
