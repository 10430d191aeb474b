"""Drop-in ``EDHFlowPF`` backed by the MI355X EDH flow kernels.

Mirrors ``/root/reference/models/EDH_particle_filter.py`` (cited ``edh.py:LINE``):
``rk4_step`` (27-33), ``systematic_resample`` / ``effective_sample_size`` (35-52),
``EDHConfig`` (58-64), ``PFState`` (67-74), ``EKFTracker`` / ``UKFTracker`` with
``get_past_mean`` (77-132), and ``EDHFlowPF`` with the same constructor (138-171),
``init_from_gaussian`` (173-180) and ``step(state, z_k, u_km1=None,
process_noise_sampler=None)`` (182-317).

The exact Daum-Huang flow linearises h once per pseudo-time step at the shared mean
trajectory etabar (edh.py:213-280), so the whole lambda integration of every particle
is one affine map of eta0.  The GPU builds that map per step in one workgroup and
applies it with the weights of edh.py:287-297 in one particle kernel
(``csrc/pf_edh_kernels.h``); resampling and the weighted statistics are the LEDH
engine's (identical code in both reference modules).  The tracker stays on the host,
called exactly as the reference calls it: ``predict()`` before the flow, then
``get_past_mean()`` for etabar, ``update(z)`` after the weights.

What a user of the reference changes is what :mod:`particle_filters_amd.ledh` lists:
device models for ``g`` / ``h``, ``h.jacobian`` for ``jacobian_h``, the Gaussian
density objects, and optionally ``rng_mode="device"``.  There is no CPU fallback.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np

from . import _native as N
from . import models as M
from .ledh import LEDHFlowPF, LEDHRunResult, PFState, effective_sample_size, systematic_resample
from .trackers import EKFTracker

Array = np.ndarray

__all__ = ["EDHConfig", "EDHFlowPF", "PFState", "EKFTracker", "rk4_step", "systematic_resample",
           "effective_sample_size"]


def rk4_step(x: Array, f: Callable[[Array], Array], dt: float) -> Array:
    """edh.py:27-33 (host helper kept for API parity)."""
    k1 = f(x)
    k2 = f(x + 0.5 * dt * k1)
    k3 = f(x + 0.5 * dt * k2)
    k4 = f(x + dt * k3)
    return x + (dt / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)


@dataclass
class EDHConfig:
    """edh.py:58-64 (including the shared default rng of the reference)."""

    n_particles: int = 512
    n_lambda_steps: int = 8
    resample_ess_ratio: float = 0.5
    flow_integrator: str = "rk4"
    rng: np.random.Generator = np.random.default_rng(0)


class EDHFlowPF(LEDHFlowPF):
    """EKF/UKF-assisted EDH particle-flow PF on an MI355X (drop-in for edh.py:135-329)."""

    def __init__(self, tracker, g, h, jacobian_h, log_trans_pdf, log_like_pdf, R,
                 config: Optional[EDHConfig] = None, *, rng_mode: str = "host", device: int = 0) -> None:
        self.tracker = tracker
        self.g = g
        self.h = h
        self.Jh = jacobian_h
        self.log_trans_pdf = log_trans_pdf
        self.log_like_pdf = log_like_pdf
        self.R = np.array(R, dtype=float)
        self.cfg = config or EDHConfig()
        if rng_mode not in ("host", "device"):
            raise ValueError("rng_mode must be 'host' or 'device'")
        self.rng_mode = rng_mode
        self.device = int(device)
        integ = str(self.cfg.flow_integrator).lower()
        # edh.py:271: anything but "euler" integrates with RK4
        self.integrator = "euler" if integ == "euler" else "rk4"
        if not M.is_device_model(g, h):
            raise NotImplementedError("the HIP EDH flow needs particle_filters_amd.models g / h objects")
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
        self.L = max(1, int(self.cfg.n_lambda_steps))  # edh.py:216
        seed = int(self.cfg.rng.integers(0, 2 ** 63 - 1)) if rng_mode == "device" else 0
        opts = N.EdhOpts(self.n, self.L, float(self.cfg.resample_ess_ratio), seed, self.device,
                         N.PF_EDH_EULER if self.integrator == "euler" else N.PF_EDH_RK4)
        self._h = N.C.c_void_p()
        N.check(N.load().pf_edh_create(N.C.byref(self._desc), N.C.byref(opts), N.C.byref(self._h)), "pf_edh_create")
        self._version = 0
        self._state = None
        self.last_ess = float("nan")
        self.last_resampled = False

    def step(self, state: PFState, z_k: Array, u_km1: Optional[Array] = None,
             process_noise_sampler: Optional[Callable[[int, int], Array]] = None) -> PFState:
        """One EDH step (edh.py:182-317)."""
        lib = N.load()
        self._adopt(state)
        _, P = self.tracker.predict()  # edh.py:195
        P = np.ascontiguousarray(np.asarray(P, float).reshape(self.nx, self.nx))
        if process_noise_sampler is None:  # edh.py:200-202: no noise
            noise, v = N.PF_NOISE_NONE, None
        else:
            noise = N.PF_NOISE_HOST
            v = np.ascontiguousarray(np.asarray(process_noise_sampler(self.n, self.nx), float).reshape(self.n, self.nx))
        xbar = np.ascontiguousarray(np.asarray(self.tracker.get_past_mean(), float).reshape(self.nx))  # edh.py:213
        z = np.ascontiguousarray(np.asarray(z_k, float).reshape(self.nz))
        u = None if u_km1 is None else np.ascontiguousarray(np.asarray(u_km1, float).reshape(self.nx))
        info = N.LedhInfo()
        S = np.empty((self.L, self.nz, self.nz))
        N.check(lib.pf_edh_step(self._h, N.dptr(P), N.dptr(xbar), N.dptr(z), N.dptr(u), noise, N.dptr(v),
                                N.C.byref(info), N.dptr(S)), "pf_edh_step")
        self.tracker.update(z_k)  # edh.py:301
        self.last_ess = float(info.ess)
        self.last_resampled = bool(info.resample)
        U = None
        if info.resample and self.rng_mode == "host":
            U = np.array([self.cfg.rng.random()])  # edh.py:41 (drawn inside systematic_resample)
        mean = np.empty(self.nx)
        cov = np.empty((self.nx, self.nx))
        N.check(lib.pf_ledh_finish(self._h, N.dptr(U), N.dptr(mean), N.dptr(cov)), "pf_ledh_finish")
        conds = []
        for j in range(self.L):  # edh.py:238-243
            try:
                conds.append(float(np.linalg.cond(S[j])))
            except Exception:
                conds.append(np.nan)
        return self._new_state(mean, cov, {"condition_numbers": conds})

    def run(self, state: PFState, Z: Array, U: Optional[Array] = None, *, process_noise: str = "device",
            tracker_seq: Optional[tuple] = None, tracker: str = "host", replay=None) -> LEDHRunResult:
        """The driver loop ``for t: state = step(state, Z[t])`` on the device with no host
        synchronisation inside T.  ``tracker="host"``: the tracker object is run ahead over Z
        (predict / get_past_mean / update, the same call sequence as the loop — it never sees
        the particles) unless ``tracker_seq = (Ps [T][nx][nx], Xbars [T][nx])`` is given.
        ``tracker="device"``: an EKFTracker over this filter's models runs on the GPU and
        also yields the past means.  Process noise is Philox times chol(Q) (``"device"``,
        resampling uniforms from Philox), zero (``"none"``) or replayed (``"host"`` with
        ``replay=(V, U)``, the contract of ``LEDHFlowPF.run``: U[t] is read only on steps that
        resample)."""
        if tracker not in ("host", "device"):
            raise ValueError("tracker must be 'host' or 'device'")
        if tracker == "device":
            return super().run(state, Z, U, process_noise=process_noise, tracker="device", replay=replay)
        self._adopt(state)
        Z = np.ascontiguousarray(np.asarray(Z, float).reshape(-1, self.nz))
        T = Z.shape[0]
        noise = self._noise_mode(process_noise, replay, T)
        if tracker_seq is None:
            Ps = np.empty((T, self.nx, self.nx))
            Xb = np.empty((T, self.nx))
            for t in range(T):
                _, P = self.tracker.predict()
                Ps[t] = P
                Xb[t] = self.tracker.get_past_mean()
                self.tracker.update(Z[t])
        else:
            Ps = np.ascontiguousarray(np.asarray(tracker_seq[0], float).reshape(T, self.nx, self.nx))
            Xb = np.ascontiguousarray(np.asarray(tracker_seq[1], float).reshape(T, self.nx))
        Uc = None if U is None else np.ascontiguousarray(np.asarray(U, float).reshape(T, self.nx))
        means = np.empty((T, self.nx))
        covs = np.empty((T, self.nx, self.nx))
        ess = np.empty(T)
        flags = np.zeros(T, dtype=np.uint8)
        N.check(N.load().pf_edh_run(self._h, N.dptr(Ps), N.dptr(Xb), N.dptr(Z), N.dptr(Uc), T, noise, N.dptr(means),
                                    N.dptr(covs), N.dptr(ess), flags.ctypes.data_as(N.C.POINTER(N.C.c_uint8))),
                "pf_edh_run")
        self._new_state(means[-1], covs[-1], {})
        return LEDHRunResult(means, covs, ess, flags.astype(bool))
