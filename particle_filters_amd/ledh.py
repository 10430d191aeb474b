"""Drop-in ``LEDHFlowPF`` backed by the MI355X LEDH flow kernels.

Mirrors ``/root/reference/models/LEDH_particle_filter.py`` (cited ``ledh.py:LINE``):
``LEDHConfig`` (44-49), ``PFState`` with ``diagnostics`` (51-57), ``LEDHFlowPF``
with the same constructor (63-81), ``init_from_gaussian`` (84-91) and
``step(state, z_k, u_km1=None, process_noise_sampler=None)`` (93-214), plus the
module helpers ``systematic_resample`` / ``effective_sample_size`` (25-41).

The per-particle flow (ledh.py:136-179), the weights (186-195), the resampling
(201-206) and the weighted statistics (209, 217-224) run on the GPU through the C
ABI of ``include/pf_ledh.h``.  The Gaussian tracker stays on the host: it is
called exactly as the reference calls it (``predict()`` before the flow,
``update(z)`` after the weights) and only its covariance crosses to the device.

What a user of the reference changes:

* ``g`` / ``h`` are device models (:mod:`particle_filters_amd.models`) — they are
  per-particle callables with the reference's signatures (``g(x, u, v)``,
  ``h(x)``), so the same objects also drive the reference;
* ``jacobian_h`` is ``None`` or ``h.jacobian`` (the analytic Jacobian of the model);
* ``log_trans_pdf`` / ``log_like_pdf`` are
  :class:`~particle_filters_amd.models.GaussianTransitionDensity` /
  :class:`~particle_filters_amd.models.GaussianLikelihood` (callables with the
  reference's semantics);
* ``rng_mode="host"`` (default) draws the initial ensemble and the resampling
  uniform from ``config.rng`` exactly like the reference; ``"device"`` uses Philox.

Arbitrary Python callables raise ``NotImplementedError``: there is no CPU fallback.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from . import _native as N
from . import models as M

Array = np.ndarray


def systematic_resample(weights: Array, rng: np.random.Generator, device: int = 0) -> Array:
    """ledh.py:25-37 on the GPU: renormalise, ``searchsorted(cumsum(w), (U + i)/N, 'right')``
    with ``U = rng.random()``."""
    from .particle_filter import resample_indices

    w = np.asarray(weights, float)
    w = w / np.sum(w)
    return resample_indices(w, "systematic", U=rng.random(), device=device)


def effective_sample_size(weights: Array) -> float:
    """ledh.py:39-41."""
    w = weights / np.sum(weights)
    return 1.0 / float(np.sum(w * w))


@dataclass
class LEDHConfig:
    """ledh.py:44-49 (including the shared default rng of the reference)."""

    n_particles: int = 512
    n_lambda_steps: int = 8
    resample_ess_ratio: float = 0.0
    rng: np.random.Generator = np.random.default_rng(0)


@dataclass
class PFState:
    """ledh.py:51-57."""

    particles: Array
    weights: Array
    mean: Array
    cov: Array
    diagnostics: dict = None


class _DeviceState(PFState):
    """PFState whose particles / weights stay in HBM until read."""

    def __init__(self, pf: "LEDHFlowPF", mean, cov, diagnostics):
        object.__setattr__(self, "_pf", pf)
        object.__setattr__(self, "_version", pf._version)
        object.__setattr__(self, "_particles", None)
        object.__setattr__(self, "_weights", None)
        object.__setattr__(self, "mean", mean)
        object.__setattr__(self, "cov", cov)
        object.__setattr__(self, "diagnostics", diagnostics)

    def _fetch(self, which):
        if self._pf._version != self._version:
            raise RuntimeError("stale PFState: the filter has advanced since this state was returned")
        return self._pf._download(which)

    @property
    def particles(self):  # type: ignore[override]
        if self._particles is None:
            object.__setattr__(self, "_particles", self._fetch("particles"))
        return self._particles

    @particles.setter
    def particles(self, value):
        object.__setattr__(self, "_particles", np.asarray(value, float))

    @property
    def weights(self):  # type: ignore[override]
        if self._weights is None:
            object.__setattr__(self, "_weights", self._fetch("weights"))
        return self._weights

    @weights.setter
    def weights(self, value):
        object.__setattr__(self, "_weights", np.asarray(value, float))

    def __repr__(self):
        return f"PFState(mean={self.mean!r}, cov=<{self.cov.shape}>, particles=<device>, weights=<device>)"


@dataclass
class LEDHRunResult:
    means: Array   # [T][nx]
    covs: Array    # [T][nx][nx]
    ess: Array     # [T] ESS of the flow weights before resampling
    flags: Array   # [T] bool, resampled at that step

    def rmse(self, truth) -> float:
        tr = np.asarray(truth, float).reshape(self.means.shape)
        return float(np.sqrt(np.mean((self.means - tr) ** 2)))


class LEDHFlowPF:
    """EKF/UKF-assisted LEDH particle-flow PF on an MI355X (drop-in for ledh.py:60-224)."""

    def __init__(self, tracker, g, h, jacobian_h, log_trans_pdf, log_like_pdf, R,
                 config: Optional[LEDHConfig] = None, *, rng_mode: str = "host", flow: str = "auto",
                 device: int = 0) -> None:
        self.tracker = tracker
        self.g = g
        self.h = h
        self.Jh = jacobian_h
        self.log_trans_pdf = log_trans_pdf
        self.log_like_pdf = log_like_pdf
        self.R = np.array(R, dtype=float)
        self.cfg = config or LEDHConfig()
        if rng_mode not in ("host", "device"):
            raise ValueError("rng_mode must be 'host' or 'device'")
        if flow not in ("auto", "per_particle"):
            raise ValueError("flow must be 'auto' or 'per_particle'")
        self.rng_mode = rng_mode
        self.device = int(device)
        if not M.is_device_model(g, h):
            raise NotImplementedError("the HIP LEDH flow needs particle_filters_amd.models g / h objects")
        if jacobian_h is not None and getattr(jacobian_h, "__self__", None) is not h:
            raise NotImplementedError("jacobian_h must be None or h.jacobian (the model's analytic Jacobian)")
        if not isinstance(log_trans_pdf, M.GaussianTransitionDensity) or log_trans_pdf.g is not g:
            raise NotImplementedError("log_trans_pdf must be models.GaussianTransitionDensity(g, Q)")
        if not isinstance(log_like_pdf, M.GaussianLikelihood) or log_like_pdf.h is not h:
            raise NotImplementedError("log_like_pdf must be models.GaussianLikelihood(h, R)")
        self.Q = log_trans_pdf.Q
        self.nx, self.nz = self.Q.shape[0], self.R.shape[0]
        self._desc, self._keep = M.describe(g, h, self.Q, self.R)
        self.n = int(self.cfg.n_particles)
        self.L = max(1, int(self.cfg.n_lambda_steps))  # ledh.py:132
        seed = int(self.cfg.rng.integers(0, 2 ** 63 - 1)) if rng_mode == "device" else 0
        opts = N.LedhOpts(self.n, self.L, float(self.cfg.resample_ess_ratio), seed, self.device,
                          N.PF_LEDH_FLOW_AUTO if flow == "auto" else N.PF_LEDH_FLOW_PER_PARTICLE)
        self._h = N.C.c_void_p()
        N.check(N.load().pf_ledh_create(N.C.byref(self._desc), N.C.byref(opts), N.C.byref(self._h)), "pf_ledh_create")
        self._version = 0
        self._state = None
        self.last_ess = float("nan")
        self.last_resampled = False

    # ------------------------------------------------------------------ plumbing
    def close(self):
        if N._lib is not None and getattr(self, "_h", None) is not None and self._h.value:
            N._lib.pf_ledh_destroy(self._h)
        self._h = None

    def __del__(self):
        self.close()

    @property
    def shared_jacobian_path(self) -> bool:
        """True when h is linear and the flow matrices are evaluated once per lambda step."""
        return bool(N.load().pf_ledh_shared_path(self._h))

    def _download(self, which):
        lib = N.load()
        if which == "particles":
            out = np.empty((self.n, self.nx))
            N.check(lib.pf_ledh_get_particles(self._h, N.dptr(out)), "pf_ledh_get_particles")
        else:
            out = np.empty(self.n)
            N.check(lib.pf_ledh_get_weights(self._h, N.dptr(out)), "pf_ledh_get_weights")
        return out

    def _adopt(self, state) -> None:
        """Make ``state`` the device state if it is not the one the engine holds."""
        if state is self._state and self._state is not None:
            return
        p = np.ascontiguousarray(np.asarray(state.particles, float).reshape(self.n, self.nx))
        w = np.ascontiguousarray(np.asarray(state.weights, float).reshape(self.n))
        N.check(N.load().pf_ledh_set_state(self._h, N.dptr(p), N.dptr(w)), "pf_ledh_set_state")

    def _new_state(self, mean, cov, diagnostics):
        self._version += 1
        self._state = _DeviceState(self, mean, cov, diagnostics)
        return self._state

    # ------------------------------------------------------------------ API
    def init_from_gaussian(self, mean0: Array, cov0: Array) -> PFState:
        """ledh.py:84-91: particles = mean0 + eps, uniform weights, weighted stats."""
        mean0 = np.ascontiguousarray(np.asarray(mean0, float).reshape(self.nx))
        cov0 = np.ascontiguousarray(np.asarray(cov0, float).reshape(self.nx, self.nx))
        eps = None
        if self.rng_mode == "host":
            eps = np.ascontiguousarray(self.cfg.rng.multivariate_normal(np.zeros(self.nx), cov0, size=self.n))
        mean = np.empty(self.nx)
        cov = np.empty((self.nx, self.nx))
        N.check(N.load().pf_ledh_init(self._h, N.dptr(mean0), N.dptr(cov0), N.dptr(eps), N.dptr(mean), N.dptr(cov)),
                "pf_ledh_init")
        return self._new_state(mean, cov, {})

    def step(self, state: PFState, z_k: Array, u_km1: Optional[Array] = None,
             process_noise_sampler: Optional[Callable[[int, int], Array]] = None) -> PFState:
        """One LEDH step (ledh.py:93-214)."""
        lib = N.load()
        self._adopt(state)
        _, P = self.tracker.predict()  # ledh.py:105
        P = np.ascontiguousarray(np.asarray(P, float).reshape(self.nx, self.nx))
        z = np.ascontiguousarray(np.asarray(z_k, float).reshape(self.nz))
        u = None if u_km1 is None else np.ascontiguousarray(np.asarray(u_km1, float).reshape(self.nx))
        if process_noise_sampler is None:  # ledh.py:109-110: no noise
            noise, v = N.PF_NOISE_NONE, None
        else:
            noise = N.PF_NOISE_HOST
            v = np.ascontiguousarray(np.asarray(process_noise_sampler(self.n, self.nx), float).reshape(self.n, self.nx))
        info = N.LedhInfo()
        S = np.empty((self.L, self.nz, self.nz))
        N.check(lib.pf_ledh_step(self._h, N.dptr(P), N.dptr(z), N.dptr(u), noise, N.dptr(v), N.C.byref(info),
                                 N.dptr(S)), "pf_ledh_step")
        self.tracker.update(z_k)  # ledh.py:198
        self.last_ess = float(info.ess)
        self.last_resampled = bool(info.resample)
        U = None
        if info.resample and self.rng_mode == "host":
            U = np.array([self.cfg.rng.random()])  # ledh.py:28 (drawn inside systematic_resample)
        mean = np.empty(self.nx)
        cov = np.empty((self.nx, self.nx))
        N.check(lib.pf_ledh_finish(self._h, N.dptr(U), N.dptr(mean), N.dptr(cov)), "pf_ledh_finish")
        conds = []
        for j in range(self.L):  # ledh.py:151-157 (particle 0's S at every lambda step)
            try:
                conds.append(float(np.linalg.cond(S[j])))
            except Exception:
                conds.append(np.nan)
        return self._new_state(mean, cov, {"condition_numbers": conds})

    def _device_tracker(self):
        """(x, P, Qt, Rt) of a trackers.EKFTracker whose EKF runs this filter's own models."""
        from . import trackers as TR

        tr = self.tracker
        if not (isinstance(tr, TR.EKFTracker) and tr.ekf.g is self.g and tr.ekf.h is self.h):
            raise NotImplementedError("tracker='device' needs a trackers.EKFTracker over this filter's g and h")
        if tr.ekf.jitter > 0.0 or tr.ekf.joseph:
            raise NotImplementedError("tracker='device' runs the plain EKF update (no jitter, no Joseph form); "
                                      "use tracker='host' for this ExtendedKalmanFilter")
        c = lambda a: np.ascontiguousarray(np.asarray(a, float))  # noqa: E731
        return c(tr.state.mean).reshape(self.nx), c(tr.state.cov).reshape(self.nx, self.nx), c(tr.ekf.Q), c(tr.ekf.R)

    def tracker_covariances(self, Z: Array) -> Array:
        """The device EKF (analytic Jacobians of the compiled model) over Z from the tracker's
        current state: the symmetrised predicted covariances [T][nx][nx] the flow would use.
        The tracker object is not advanced."""
        x0, P0, Qt, Rt = self._device_tracker()
        Z = np.ascontiguousarray(np.asarray(Z, float).reshape(-1, self.nz))
        Ps = np.empty((Z.shape[0], self.nx, self.nx))
        N.check(N.load().pf_ledh_ekf_sequence(self._h, N.dptr(x0), N.dptr(P0), N.dptr(Qt), N.dptr(Rt), N.dptr(Z),
                                              Z.shape[0], N.dptr(Ps), None, None), "pf_ledh_ekf_sequence")
        return Ps

    def _noise_mode(self, process_noise: str, replay, T: int) -> int:
        """process_noise "device" (Philox), "none", or "host": replay = (V [T][N][nx], U [T]), the
        reference's draws (the process_noise_sampler's per step, and systematic_resample's
        rng.random() at the steps that resample), consumed by the device loop in that order."""
        if process_noise not in ("device", "none", "host"):
            raise ValueError("process_noise must be 'device', 'none' or 'host'")
        if process_noise != "host":
            return N.PF_NOISE_DEVICE if process_noise == "device" else N.PF_NOISE_NONE
        if replay is None:
            raise ValueError("process_noise='host' needs replay=(V [T][N][nx], U [T])")
        V = np.ascontiguousarray(np.asarray(replay[0], float).reshape(T, self.n, self.nx))
        Uu = np.ascontiguousarray(np.asarray(replay[1], float).reshape(T))
        N.check(N.load().pf_ledh_set_run_replay(self._h, N.dptr(V), N.dptr(Uu), T), "pf_ledh_set_run_replay")
        return N.PF_NOISE_HOST

    def run(self, state: PFState, Z: Array, U: Optional[Array] = None, *, process_noise: str = "device",
            tracker_covs: Optional[Array] = None, tracker: str = "host", replay=None) -> LEDHRunResult:
        """The driver loop ``for t: state = step(state, Z[t])`` on the device with no host
        synchronisation inside T.  ``tracker="host"``: the tracker object is run ahead over Z
        (predict/update, the same call sequence as the loop — it never sees the particles)
        unless ``tracker_covs`` [T][nx][nx] is given.  ``tracker="device"``: an EKFTracker over
        this filter's models runs on the GPU (analytic Jacobians), and its object is advanced
        to the final posterior afterwards.  Process noise is Philox times chol(Q)
        (``"device"``, resampling uniforms from Philox), zero (``"none"``, the reference
        default) or replayed (``"host"`` with ``replay=(V, U)``: V [T][N][nx] the
        process_noise_sampler draws of each step, U [T] the systematic-resampling uniforms).
        Replay contract: U[t] is read only on steps that resample, so lay it out with the
        decisions you expect and check the returned flags against them.  A failed launch or
        grid-barrier timeout leaves the filter uninitialised (AssertionError on the next call)."""
        if tracker not in ("host", "device"):
            raise ValueError("tracker must be 'host' or 'device'")
        self._adopt(state)
        Z = np.ascontiguousarray(np.asarray(Z, float).reshape(-1, self.nz))
        T = Z.shape[0]
        noise = self._noise_mode(process_noise, replay, T)
        if tracker == "device":
            from . import trackers as TR

            x0, P0, Qt, Rt = self._device_tracker()
            Uc = None if U is None else np.ascontiguousarray(np.asarray(U, float).reshape(T, self.nx))
            means, covs = np.empty((T, self.nx)), np.empty((T, self.nx, self.nx))
            ess, flags = np.empty(T), np.zeros(T, dtype=np.uint8)
            xf, Pf = np.empty(self.nx), np.empty((self.nx, self.nx))
            N.check(N.load().pf_ledh_run_ekf(self._h, N.dptr(x0), N.dptr(P0), N.dptr(Qt), N.dptr(Rt), N.dptr(Z),
                                             N.dptr(Uc), T, noise, N.dptr(means), N.dptr(covs), N.dptr(ess),
                                             flags.ctypes.data_as(N.C.POINTER(N.C.c_uint8)), N.dptr(xf), N.dptr(Pf)),
                    "pf_ledh_run_ekf")
            tr = self.tracker
            tr.past_mean = xf.copy()  # approximate: the mean before the last predict is not kept
            tr.state = TR.EKFState(mean=xf, cov=Pf, t=tr.state.t + T)
            self._new_state(means[-1], covs[-1], {})
            return LEDHRunResult(means, covs, ess, flags.astype(bool))
        if tracker_covs is None:
            Ps = np.empty((T, self.nx, self.nx))
            for t in range(T):
                _, P = self.tracker.predict()
                Ps[t] = P
                self.tracker.update(Z[t])
        else:
            Ps = np.ascontiguousarray(np.asarray(tracker_covs, float).reshape(T, self.nx, self.nx))
        Uc = None if U is None else np.ascontiguousarray(np.asarray(U, float).reshape(T, self.nx))
        means = np.empty((T, self.nx))
        covs = np.empty((T, self.nx, self.nx))
        ess = np.empty(T)
        flags = np.zeros(T, dtype=np.uint8)
        N.check(N.load().pf_ledh_run(self._h, N.dptr(Ps), N.dptr(Z), N.dptr(Uc), T, noise, N.dptr(means),
                                     N.dptr(covs), N.dptr(ess), flags.ctypes.data_as(N.C.POINTER(N.C.c_uint8))),
                "pf_ledh_run")
        self._new_state(means[-1], covs[-1], {})
        return LEDHRunResult(means, covs, ess, flags.astype(bool))

    @property
    def state(self) -> Optional[PFState]:
        return self._state

    @staticmethod
    def _weighted_stats(x: Array, w: Array):
        """ledh.py:217-224 (host helper kept for API parity)."""
        w = w / np.sum(w)
        mean = np.sum(x * w[:, None], axis=0)
        xc = x - mean[None, :]
        cov = (xc.T * w) @ xc
        return mean, 0.5 * (cov + cov.T)
