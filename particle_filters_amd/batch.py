"""Batched replicates and the device-resident time loop.

``ParticleFilterBatch`` runs R independent copies of one state-space model
(Monte-Carlo replicates, BASELINE config 4) in single launches over
``[R][nx][N]`` state, and drives the whole T-step filter on the GPU with no host
synchronisation inside T (``pf_run`` in include/pf_engine.h).  The per-step
outputs are exactly what the reference's driver loops collect
(tests/integration_tests/test_pf_vs_simulator_sv.py:78-81;
notebooks/PF_VS_experiments.ipynb cell 7): posterior means (post-resample, like
``PFState.mean``), covariances (any nx), pre-resample Neff, resample flags and
the log normaliser.

Replicate r of a batch draws its randomness with Philox counter word
``replicate_base + r``: splitting replicates over GPUs (``distributed.py``)
gives bitwise the same per-replicate results as one GPU.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _native as N
from . import models as M


@dataclass
class RunResult:
    means: np.ndarray      # [T][R][nx]
    covs: Optional[np.ndarray]  # [T][R][nx][nx] (None when run(with_cov=False))
    neff: np.ndarray       # [T][R] pre-resample 1/sum w^2
    flags: np.ndarray      # [T][R] bool, resampled at that step
    log_norm: np.ndarray   # [T][R]
    ess: np.ndarray        # [T][R] effective_sample_size() after each update

    def rmse(self, truth: np.ndarray) -> np.ndarray:
        """Per-replicate RMSE of the posterior means against truth [T][nx] (or [T])."""
        tr = np.asarray(truth, float).reshape(self.means.shape[0], 1, -1)
        return np.sqrt(np.mean((self.means - tr) ** 2, axis=(0, 2)))


def _uniform_ess(n):
    w = np.ones(n) / n
    return 1.0 / np.sum(w ** 2)


class ParticleFilterBatch:
    def __init__(self, g, h, Q, R, *, Np: int, n_replicates: int = 1, replicate_base: int = 0,
                 resample_thresh: float = 0.5, resample_method: str = "systematic",
                 regularize_after_resample: bool = False, seed: int = 0, precision: str = "fp32",
                 device: int = 0, kernel_path: str = "auto"):
        if not M.is_device_model(g, h):
            raise NotImplementedError("ParticleFilterBatch needs particle_filters_amd.models g/h")
        self.Q = np.asarray(Q, float)
        self.R = M.observation_noise(h, R)
        self.nx, self.nz = self.Q.shape[0], self.R.shape[0]
        self.Np = int(Np)
        self.n_replicates = int(n_replicates)
        self.replicate_base = int(replicate_base)
        self.precision = precision
        self._desc, self._keep = M.describe(g, h, self.Q, self.R)
        opts = N.Opts(self.Np, self.n_replicates,
                      N.PF_RESAMPLE_SYSTEMATIC if resample_method == "systematic" else N.PF_RESAMPLE_MULTINOMIAL,
                      float(resample_thresh), int(bool(regularize_after_resample)),
                      N.PF_PRECISION_FP64 if precision == "fp64" else N.PF_PRECISION_FP32,
                      int(seed), int(device), self.replicate_base, M.kernel_path_code(kernel_path))
        self._h = N.C.c_void_p()
        N.check(N.load().pf_create(N.C.byref(self._desc), N.C.byref(opts), N.C.byref(self._h)), "pf_create")

    def close(self) -> None:
        """Release the device state now (also done on garbage collection)."""
        if N._lib is not None and getattr(self, "_h", None) is not None and self._h.value:
            N._lib.pf_destroy(self._h)
        self._h = None

    def __del__(self):
        self.close()

    @property
    def handle(self):
        return self._h

    def _per_rep(self, a, shape):
        a = np.asarray(a, float)
        return np.ascontiguousarray(np.broadcast_to(a, (self.n_replicates,) + shape))

    def initialize(self, mean, cov, replay_normals: Optional[np.ndarray] = None) -> None:
        m = self._per_rep(np.asarray(mean, float).reshape(-1, self.nx) if np.ndim(mean) > 1 else mean, (self.nx,))
        c = self._per_rep(cov, (self.nx, self.nx))
        rn = None if replay_normals is None else np.ascontiguousarray(replay_normals, dtype=float)
        N.check(N.load().pf_initialize(self._h, N.dptr(m), N.dptr(c), N.dptr(rn)), "pf_initialize")

    def run(self, Z, U=None, *, first_update_only: bool = False, with_cov: bool = True) -> RunResult:
        """Filter observations Z ([T][nz], shared by all replicates, or [T][R][nz]).  Every step's
        posterior covariance (pf.py:266-267) is computed on the device for any nx; with_cov=False
        skips it (nx > 4: one MFMA covariance launch pair per step)."""
        Z = np.asarray(Z, float)
        T = Z.shape[0]
        Zr = np.ascontiguousarray(np.broadcast_to(Z.reshape(T, -1, self.nz), (T, self.n_replicates, self.nz)))
        Ur = None
        if U is not None:
            U = np.asarray(U, float)
            Ur = np.ascontiguousarray(np.broadcast_to(U.reshape(T, -1, self.nx), (T, self.n_replicates, self.nx)))
        Rn = self.n_replicates
        means = np.zeros((T, Rn, self.nx))
        covs = np.zeros((T, Rn, self.nx, self.nx)) if with_cov else None
        neff = np.zeros((T, Rn))
        flags = np.zeros((T, Rn), dtype=np.uint8)
        lnorm = np.zeros((T, Rn))
        st = N.load().pf_run(self._h, N.dptr(Zr), N.dptr(Ur), T, int(first_update_only), N.dptr(means),
                             N.dptr(covs), N.dptr(neff), flags.ctypes.data_as(N.C.POINTER(N.C.c_uint8)),
                             N.dptr(lnorm))
        N.check(st, "pf_run")
        fl = flags.astype(bool)
        ess = np.where(fl, _uniform_ess(self.Np), neff)
        return RunResult(means, covs, neff, fl, lnorm, ess)

    def particles(self) -> np.ndarray:
        out = np.empty((self.n_replicates, self.Np, self.nx))
        N.check(N.load().pf_get_particles(self._h, N.dptr(out)), "pf_get_particles")
        return out

    def weights(self) -> np.ndarray:
        out = np.empty((self.n_replicates, self.Np))
        N.check(N.load().pf_get_weights(self._h, N.dptr(out), None), "pf_get_weights")
        return out

    def rng_state(self) -> dict:
        """Philox position of the device RNG (epoch of the next predict)."""
        return N.get_rng_state(self._h)

    def set_rng_state(self, state: dict) -> None:
        N.set_rng_state(self._h, state)

    def checkpoint(self) -> bytes:
        """Bit-exact snapshot at the step boundary: particles, unnormalised log-weights, tile
        records and the Philox position (include/pf_engine.h pf_checkpoint)."""
        return N.checkpoint(self._h)

    def restore(self, blob: bytes) -> None:
        """Continue from a :meth:`checkpoint` of a batch with the same model and options."""
        N.restore(self._h, blob)

    @property
    def last_run_resident(self) -> bool:
        """True if the last run() executed as the register-resident whole-run kernel."""
        return bool(N.load().pf_last_run_resident(self._h))

    def geometry(self):
        G, tile, lds = N.C.c_int32(), N.C.c_int32(), N.C.c_int32()
        N.check(N.load().pf_geometry(self._h, N.C.byref(G), N.C.byref(tile), N.C.byref(lds)), "pf_geometry")
        return G.value, tile.value, lds.value
