"""NumPy restatement of the reference LEDH particle-flow filter — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module; it is the checker for the HIP LEDH engine, never the
thing measured or shipped.

Follows (paths relative to /root/reference):

* ``models/LEDH_particle_filter.py`` (cited ``ledh.py:LINE``):
  ``systematic_resample`` 25-37, ``effective_sample_size`` 39-41,
  ``LEDHConfig`` 44-49, ``PFState`` 51-57, ``LEDHFlowPF.init_from_gaussian``
  84-91, ``step`` 93-214, ``_weighted_stats`` 217-224.
* ``models/extended_kalman_filter.py`` (``ekf.py:LINE``): finite-difference
  Jacobians 43-107, ``predict`` 164-194, ``update`` 196-241.
* the ``EKFTracker`` wrapper of the reference tests
  (``tests/unit_tests/models/test_ledh_flow_pf.py:12-33``) that adapts the EKF
  to the ``GaussianTracker`` protocol (ledh.py:13-16).

Two evaluation modes (like :mod:`oracle.pf_oracle`):

* ``vectorized=False`` (faithful): the reference's per-particle loops and
  per-particle callbacks — the CPU path's cost profile (bench cpu_baseline).
* ``vectorized=True``: the same arithmetic batched over particles with
  ``numpy.linalg`` gufuncs (same LAPACK routines per matrix); plugins take the
  whole particle matrix.  Agrees with the faithful mode to fp64 rounding.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

Array = np.ndarray


# ---------------------------------------------------------------------------
# ledh.py:25-41 utilities
# ---------------------------------------------------------------------------
def systematic_resample(weights: Array, U: float) -> Array:
    """ledh.py:25-37 with the uniform drawn by the caller.  The two-pointer loop over a
    cumsum *without* the cdf[-1] = 1 fix is ``searchsorted(cdf, pos, 'right')``; a
    position past cdf[-1] makes the reference index out of range (IndexError)."""
    n = weights.size
    w = weights / np.sum(weights)
    positions = (U + np.arange(n)) / n
    cdf = np.cumsum(w)
    idx = np.searchsorted(cdf, positions, side="right")
    if np.any(idx >= n):
        raise IndexError("systematic_resample: position beyond cdf[-1] (reference raises here too)")
    return idx.astype(int)


def effective_sample_size(weights: Array) -> float:
    """ledh.py:39-41 (renormalises first)."""
    w = weights / np.sum(weights)
    return 1.0 / float(np.sum(w * w))


def weighted_stats(x: Array, w: Array):
    """ledh.py:217-224."""
    w = w / np.sum(w)
    mean = np.sum(x * w[:, None], axis=0)
    xc = x - mean[None, :]
    cov = (xc.T * w) @ xc
    cov = 0.5 * (cov + cov.T)
    return mean, cov


@dataclass
class LEDHState:
    """ledh.py:51-57."""

    particles: Array
    weights: Array
    mean: Array
    cov: Array
    diagnostics: dict = field(default_factory=dict)


# ---------------------------------------------------------------------------
# ekf.py — the Gaussian tracker that supplies P to the flow
# ---------------------------------------------------------------------------
def numerical_jacobian_g(g, x, u, eps=1e-6):
    """ekf.py:43-75."""
    x = np.asarray(x, dtype=float)
    y0 = np.asarray(g(x, u), dtype=float)
    nx = x.size
    J = np.zeros((y0.size, nx), dtype=float)
    for j in range(nx):
        dx = np.zeros(nx, dtype=float)
        dx[j] = eps
        J[:, j] = (g(x + dx, u) - y0) / eps
    return J


def numerical_jacobian_h(h, x, eps=1e-6):
    """ekf.py:78-107."""
    x = np.asarray(x, dtype=float)
    z0 = np.asarray(h(x), dtype=float)
    nx = x.size
    J = np.zeros((z0.size, nx), dtype=float)
    for j in range(nx):
        dx = np.zeros(nx, dtype=float)
        dx[j] = eps
        J[:, j] = (h(x + dx) - z0) / eps
    return J


@dataclass
class EKFState:
    mean: Array
    cov: Array
    t: int


class EKFOracle:
    """ekf.py:110-241 (additive-noise EKF, optional analytic Jacobians, Joseph form, jitter)."""

    def __init__(self, g, h, Q, R, jac_g=None, jac_h=None, *, joseph=False, jitter=0.0):
        self.g, self.h = g, h
        self.Q = np.asarray(Q, dtype=float)
        self.R = np.asarray(R, dtype=float)
        self.jac_g, self.jac_h = jac_g, jac_h
        self.joseph = bool(joseph)
        self.jitter = float(jitter)

    def predict(self, state: EKFState, u=None) -> EKFState:
        x = np.asarray(state.mean, dtype=float)
        P = np.asarray(state.cov, dtype=float)
        x_pred = np.asarray(self.g(x, u), dtype=float)
        G = self.jac_g(x, u) if self.jac_g is not None else numerical_jacobian_g(self.g, x, u)
        P_pred = G @ P @ G.T + self.Q
        return EKFState(mean=x_pred, cov=P_pred, t=state.t + 1)

    def update(self, pred: EKFState, z) -> EKFState:
        x_pred = np.asarray(pred.mean, dtype=float)
        P_pred = np.asarray(pred.cov, dtype=float)
        z = np.asarray(z, dtype=float)
        nz = z.size
        H = self.jac_h(x_pred) if self.jac_h is not None else numerical_jacobian_h(self.h, x_pred)
        z_pred = np.asarray(self.h(x_pred), dtype=float)
        y = z - z_pred
        S = H @ P_pred @ H.T + self.R
        if self.jitter > 0.0:
            S = S + self.jitter * np.eye(nz)
        K = P_pred @ H.T @ np.linalg.inv(S)
        x_post = x_pred + K @ y
        if self.joseph:
            I = np.eye(P_pred.shape[0])
            A = I - K @ H
            P_post = A @ P_pred @ A.T + K @ self.R @ K.T
        else:
            P_post = (np.eye(P_pred.shape[0]) - K @ H) @ P_pred
        return EKFState(mean=x_post, cov=P_post, t=pred.t)


class EKFTrackerOracle:
    """test_ledh_flow_pf.py:12-33: EKF behind the GaussianTracker protocol (ledh.py:13-16)."""

    def __init__(self, ekf, initial_state: EKFState):
        self.ekf = ekf
        self.state = initial_state
        self.past_mean = initial_state.mean.copy()

    def predict(self):
        self.past_mean = self.state.mean.copy()
        self.state = self.ekf.predict(self.state, u=None)
        return self.state.mean, self.state.cov

    def update(self, z_k):
        self.state = self.ekf.update(self.state, z_k)
        return self.state.mean, self.state.cov

    def get_past_mean(self):
        return self.past_mean


# ---------------------------------------------------------------------------
# LEDH plugins: per-particle callables + vectorised forms
# ---------------------------------------------------------------------------
@dataclass
class LEDHModel:
    nx: int
    nz: int
    Q: Array
    R: Array
    g: Callable            # g(x, u, v) -> (nx,)   (ledh.py:18 GFn)
    h: Callable            # h(x) -> (nz,)
    jac_h: Callable        # (nz, nx)
    log_trans: Callable    # log p(x_k | x_{k-1})
    log_like: Callable     # log p(z | x)
    g_vec: Callable = None         # (N,nx), u, (N,nx) -> (N,nx)
    h_vec: Callable = None         # (N,nx) -> (N,nz)
    jac_vec: Callable = None       # (N,nx) -> (N,nz,nx)
    log_trans_vec: Callable = None  # (N,nx),(N,nx) -> (N,)
    log_like_vec: Callable = None   # z, (N,nx) -> (N,)
    g_ekf: Callable = None          # g(x, u) without noise, for the EKF tracker
    jac_g: Callable = None          # analytic EKF Jacobian of g (None -> finite differences)


def _gauss_logpdf(diff, C):
    """-0.5 (d^T C^{-1} d + log det(2 pi C)) per row, the reference wirings' density."""
    d = np.atleast_2d(diff)
    sol = np.linalg.solve(C, d.T).T
    quad = np.sum(d * sol, axis=1)
    return -0.5 * (quad + np.log(np.linalg.det(2 * np.pi * C)))


def gaussian_model(nx, nz, Q, R, g0, h, jac_h, g0_vec, h_vec, jac_vec, jac_g=None) -> LEDHModel:
    """Additive-noise Gaussian wiring: g(x,u,v) = g0(x,u) + v, log_trans = N(x_k; g0(x_{k-1}), Q),
    log_like = N(z; h(x), R) — the form of every LEDH wiring in the reference tests
    (test_ledh_flow_pf.py:70-100, test_filters_mat_simulator.py:38-73)."""
    Q = np.asarray(Q, float)
    R = np.asarray(R, float)

    def g(x, u=None, v=None):
        y = g0(x, u)
        return y if v is None else y + v

    def log_trans(xk, xkm1):
        diff = xk - g0(xkm1, None)
        return float(-0.5 * (diff.T @ np.linalg.solve(Q, diff) + np.log(np.linalg.det(2 * np.pi * Q))))

    def log_like(z, x):
        diff = z - h(x)
        return float(-0.5 * (diff.T @ np.linalg.solve(R, diff) + np.log(np.linalg.det(2 * np.pi * R))))

    def g_vec(X, u, V):
        return g0_vec(X, u) + V

    def log_trans_vec(XK, XKM1):
        return _gauss_logpdf(XK - g0_vec(XKM1, None), Q)

    def log_like_vec(z, X):
        return _gauss_logpdf(z[None, :] - h_vec(X), R)

    return LEDHModel(nx, nz, Q, R, g, h, jac_h, log_trans, log_like, g_vec, h_vec, jac_vec, log_trans_vec,
                     log_like_vec, g_ekf=g0, jac_g=jac_g)


def linear_1d(alpha=0.9, sigma=0.2, R=0.1) -> LEDHModel:
    """test_ledh_flow_pf.py:62-113 (simple_linear_system)."""
    return gaussian_model(
        1, 1, [[sigma ** 2]], [[R]],
        lambda x, u: np.array([alpha * x[0]]), lambda x: np.array([x[0]]), lambda x: np.array([[1.0]]),
        lambda X, u: alpha * X, lambda X: X.copy(), lambda X: np.ones((X.shape[0], 1, 1)),
        jac_g=lambda x, u: np.array([[alpha]]))


def sv_exp_half(alpha=0.95, sigma=0.2, beta=1.0, R=0.1) -> LEDHModel:
    """1-D SV with the nonlinear test-harness observation h = beta exp(x/2)
    (test_pf_vs_simulator_sv.py:46-56 wiring), Jacobian beta/2 exp(x/2)."""
    return gaussian_model(
        1, 1, [[sigma ** 2]], [[R]],
        lambda x, u: np.array([alpha * x[0]]), lambda x: np.array([beta * np.exp(0.5 * x[0])]),
        lambda x: np.array([[0.5 * beta * np.exp(0.5 * x[0])]]),
        lambda X, u: alpha * X, lambda X: beta * np.exp(0.5 * X),
        lambda X: (0.5 * beta * np.exp(0.5 * X))[:, :, None],
        jac_g=lambda x, u: np.array([[alpha]]))


def acoustic_single(S, psi=10.0, d0=0.1, Q=None, R=None) -> LEDHModel:
    """Per-target acoustic tracking wiring of test_filters_mat_simulator.py:22-73
    (CV g, h = sum over one target of psi/(|p-s|^2+d0), analytic Jacobian)."""
    S = np.asarray(S, float)
    ns = S.shape[0]
    F = np.array([[1.0, 0.0, 1.0, 0.0], [0.0, 1.0, 0.0, 1.0], [0.0, 0.0, 1.0, 0.0], [0.0, 0.0, 0.0, 1.0]])
    if Q is None:
        Q = np.array([[3.0, 0.0, 0.1, 0.0], [0.0, 3.0, 0.0, 0.1], [0.1, 0.0, 0.03, 0.0], [0.0, 0.1, 0.0, 0.03]])
    if R is None:
        R = 0.1 ** 2 * np.eye(ns)

    def h(x):
        pos = x[:2]
        z = np.zeros(ns)
        for s in range(ns):
            z[s] = psi / (np.sum((pos - S[s]) ** 2) + d0)
        return z

    def jac(x):
        pos = x[:2]
        H = np.zeros((ns, 4))
        for s in range(ns):
            diff = pos - S[s]
            denom = (np.sum(diff ** 2) + d0) ** 2
            H[s, 0] = -2.0 * psi * diff[0] / denom
            H[s, 1] = -2.0 * psi * diff[1] / denom
        return H

    def h_vec(X):
        dx = X[:, 0, None] - S[None, :, 0]
        dy = X[:, 1, None] - S[None, :, 1]
        return psi / ((dx ** 2 + dy ** 2) + d0)

    def jac_vec(X):
        dx = X[:, 0, None] - S[None, :, 0]
        dy = X[:, 1, None] - S[None, :, 1]
        den = ((dx ** 2 + dy ** 2) + d0) ** 2
        H = np.zeros((X.shape[0], ns, 4))
        H[:, :, 0] = -2.0 * psi * dx / den
        H[:, :, 1] = -2.0 * psi * dy / den
        return H

    return gaussian_model(4, ns, Q, R, lambda x, u: F @ x, h, jac, lambda X, u: X @ F.T, h_vec, jac_vec,
                          jac_g=lambda x, u: F)


def acoustic_joint(S, psi=10.0, d0=0.1, n_targets=4, Q_single=None, R=None) -> LEDHModel:
    """Joint multi-target acoustic wiring of the MAT notebook (PF_PF_results_reproduction_
    multi_target_acoustic_tracking.ipynb cell 5: ``g_joint`` = CV per [x, y, vx, vy] block,
    ``h_joint`` = sum over targets of psi/(|p_c - s|^2 + d0), ``jac_h_joint`` = per-target
    blocks, ``Q_joint = blockdiag(Q_filter)``, ``R = 0.1^2 I``)."""
    S = np.asarray(S, float)
    ns, C = S.shape[0], int(n_targets)
    nx = 4 * C
    F1 = np.array([[1.0, 0.0, 1.0, 0.0], [0.0, 1.0, 0.0, 1.0], [0.0, 0.0, 1.0, 0.0], [0.0, 0.0, 0.0, 1.0]])
    F = np.kron(np.eye(C), F1)
    if Q_single is None:
        Q_single = np.array([[3.0, 0.0, 0.1, 0.0], [0.0, 3.0, 0.0, 0.1], [0.1, 0.0, 0.03, 0.0],
                             [0.0, 0.1, 0.0, 0.03]])
    Q = np.kron(np.eye(C), np.asarray(Q_single, float))
    if R is None:
        R = 0.1 ** 2 * np.eye(ns)

    def h(x):
        z = np.zeros(ns)
        for c in range(C):
            pos = x[4 * c:4 * c + 2]
            zc = np.zeros(ns)
            for s in range(ns):
                zc[s] = psi / (np.sum((pos - S[s]) ** 2) + d0)
            z += zc
        return z

    def jac(x):
        H = np.zeros((ns, nx))
        for c in range(C):
            pos = x[4 * c:4 * c + 2]
            for s in range(ns):
                diff = pos - S[s]
                denom = (np.sum(diff ** 2) + d0) ** 2
                H[s, 4 * c] = -2.0 * psi * diff[0] / denom
                H[s, 4 * c + 1] = -2.0 * psi * diff[1] / denom
        return H

    def h_vec(X):
        z = np.zeros((X.shape[0], ns))
        for c in range(C):
            dx = X[:, 4 * c, None] - S[None, :, 0]
            dy = X[:, 4 * c + 1, None] - S[None, :, 1]
            z = z + psi / ((dx ** 2 + dy ** 2) + d0)
        return z

    def jac_vec(X):
        H = np.zeros((X.shape[0], ns, nx))
        for c in range(C):
            dx = X[:, 4 * c, None] - S[None, :, 0]
            dy = X[:, 4 * c + 1, None] - S[None, :, 1]
            den = ((dx ** 2 + dy ** 2) + d0) ** 2
            H[:, :, 4 * c] = -2.0 * psi * dx / den
            H[:, :, 4 * c + 1] = -2.0 * psi * dy / den
        return H

    return gaussian_model(nx, ns, Q, R, lambda x, u: F @ x, h, jac, lambda X, u: X @ F.T, h_vec, jac_vec,
                          jac_g=lambda x, u: F)


def lorenz96(nx=40, F=8.0, dt=0.01, obs_fraction=4, obs_error_std=1.0, q_std=0.1) -> LEDHModel:
    """L96 LEDH wiring (BASELINE config 5): g = one RK4 step + v, h = x[H_idx], constant
    selection Jacobian, Q = q_std^2 I (the build's choice, as for the SIR config 3)."""
    from oracle.ssm_oracle import l96_rk4

    H_idx = np.arange(0, nx, obs_fraction)
    nz = H_idx.size
    Hm = np.zeros((nz, nx))
    Hm[np.arange(nz), H_idx] = 1.0
    return gaussian_model(
        nx, nz, q_std ** 2 * np.eye(nx), obs_error_std ** 2 * np.eye(nz),
        lambda x, u: l96_rk4(x, dt, F), lambda x: x[H_idx], lambda x: Hm.copy(),
        lambda X, u: l96_rk4(X, dt, F), lambda X: X[:, H_idx], lambda X: np.broadcast_to(Hm, (X.shape[0], nz, nx)),
        jac_g=None)


# ---------------------------------------------------------------------------
# the filter
# ---------------------------------------------------------------------------
class LEDHOracle:
    """ledh.py:60-224.  ``rng`` is the LEDHConfig rng (ledh.py:49), used for the initial
    draw (ledh.py:87) and the resampling uniform (ledh.py:28)."""

    def __init__(self, tracker, model: LEDHModel, *, n_particles=512, n_lambda_steps=8,
                 resample_ess_ratio=0.0, rng=None, vectorized=True):
        self.tracker = tracker
        self.m = model
        self.R = np.array(model.R, dtype=float)
        self.n_particles = int(n_particles)
        self.n_lambda_steps = int(n_lambda_steps)
        self.resample_ess_ratio = float(resample_ess_ratio)
        self.rng = np.random.default_rng(0) if rng is None else rng
        self.vectorized = vectorized
        self.last_resampled = False
        self.last_ess = float("nan")

    def init_from_gaussian(self, mean0, cov0) -> LEDHState:
        """ledh.py:84-91."""
        mean0 = np.asarray(mean0, float)
        n, nx = self.n_particles, mean0.size
        eps = self.rng.multivariate_normal(np.zeros(nx), cov0, size=n)
        particles = mean0[None, :] + eps
        weights = np.full(n, 1.0 / n)
        mean, cov = weighted_stats(particles, weights)
        return LEDHState(particles, weights, mean, cov, {})

    def step(self, state: LEDHState, z_k, u_km1=None, process_noise_sampler=None) -> LEDHState:
        """ledh.py:93-214."""
        m = self.m
        N, nx = state.particles.shape
        I = np.eye(nx)
        z_k = np.asarray(z_k, float)
        _, P = self.tracker.predict()
        P = 0.5 * (P + P.T)
        v = np.zeros((N, nx)) if process_noise_sampler is None else process_noise_sampler(N, nx)
        if self.vectorized:
            eta0 = m.g_vec(state.particles, u_km1, v)
        else:
            eta0 = np.empty_like(state.particles)
            for i in range(N):
                eta0[i] = m.g(state.particles[i], u_km1, v[i])
        eta = eta0.copy()
        etabar = eta0.copy()
        theta_log = np.zeros(N)
        cond_numbers = []
        n_steps = max(1, int(self.n_lambda_steps))
        dlam = 1.0 / float(n_steps)
        lam = 0.0
        for _ in range(n_steps):
            lam = min(1.0, lam + dlam)
            if self.vectorized:
                Hs = m.jac_vec(eta)                                    # (N, nz, nx)
                e = m.h_vec(eta) - np.matmul(Hs, eta[:, :, None])[:, :, 0]
                HsT = np.swapaxes(Hs, 1, 2)
                S = np.matmul(np.matmul(lam * Hs, P), HsT) + self.R
                try:
                    cond_numbers.append(float(np.linalg.cond(S[0])))
                except Exception:
                    cond_numbers.append(np.nan)
                SinvH = np.linalg.solve(S, Hs)
                A = np.matmul(np.matmul(-0.5 * P, HsT), SinvH)         # (N, nx, nx)
                rin = np.linalg.solve(self.R, (z_k[None, :] - e).T).T   # (N, nz)
                pht = np.matmul(np.matmul(P, HsT), rin[:, :, None])[:, :, 0]
                inner = np.matmul(I + lam * A, pht[:, :, None]) + np.matmul(A, eta0[:, :, None])
                b = np.matmul(I + 2.0 * lam * A, inner)[:, :, 0]
                etabar = etabar + dlam * (np.matmul(A, etabar[:, :, None])[:, :, 0] + b)
                eta = eta + dlam * (np.matmul(A, eta[:, :, None])[:, :, 0] + b)
                Mj = I + dlam * A
                sign, logdet = np.linalg.slogdet(Mj)
                bad = sign <= 0
                if np.any(bad):
                    _, ld2 = np.linalg.slogdet(Mj[bad] + 1e-12 * I)
                    logdet = logdet.copy()
                    logdet[bad] = ld2
                theta_log += logdet
            else:
                for i in range(N):
                    Hi = m.jac_h(eta[i])
                    ei = m.h(eta[i]) - Hi @ eta[i]
                    Si = lam * Hi @ P @ Hi.T + self.R
                    if i == 0:
                        try:
                            cond_numbers.append(float(np.linalg.cond(Si)))
                        except Exception:
                            cond_numbers.append(np.nan)
                    Ai = -0.5 * P @ Hi.T @ np.linalg.solve(Si, Hi)
                    pht = P @ Hi.T @ np.linalg.solve(self.R, (z_k - ei))
                    bi = (I + 2.0 * lam * Ai) @ ((I + lam * Ai) @ pht + Ai @ eta0[i])
                    etabar[i] = etabar[i] + dlam * (Ai @ etabar[i] + bi)
                    eta[i] = eta[i] + dlam * (Ai @ eta[i] + bi)
                    Mj = I + dlam * Ai
                    sign, logdet = np.linalg.slogdet(Mj)
                    if sign <= 0:
                        sign, logdet = np.linalg.slogdet(Mj + 1e-12 * I)
                    theta_log[i] += logdet
        xk = eta
        logw = np.log(state.weights + 1e-300) + theta_log
        if self.vectorized:
            logw = logw + ((m.log_trans_vec(xk, state.particles) + m.log_like_vec(z_k, xk))
                           - m.log_trans_vec(eta0, state.particles))
        else:
            for i in range(N):
                num = m.log_trans(xk[i], state.particles[i]) + m.log_like(z_k, xk[i])
                den = m.log_trans(eta0[i], state.particles[i])
                logw[i] += (num - den)
        logw -= np.max(logw)
        w = np.exp(logw)
        w /= np.sum(w)
        self.tracker.update(z_k)
        self.last_resampled = False
        self.last_ess = effective_sample_size(w)
        if self.resample_ess_ratio > 0.0:
            if self.last_ess < self.resample_ess_ratio * N:
                idx = systematic_resample(w, self.rng.random())
                xk = xk[idx]
                w = np.full_like(w, 1.0 / N)
                self.last_resampled = True
        mean, cov = weighted_stats(xk, w)
        return LEDHState(xk, w, mean, cov, {"condition_numbers": cond_numbers})


def make_ekf_tracker(model: LEDHModel, mean0, cov0) -> EKFTrackerOracle:
    ekf = EKFOracle(model.g_ekf, model.h, model.Q, model.R, jac_g=model.jac_g, jac_h=model.jac_h)
    return EKFTrackerOracle(ekf, EKFState(np.asarray(mean0, float).copy(), np.asarray(cov0, float).copy(), 0))


def run_ledh(model: LEDHModel, Z, *, mean0, cov0, n_particles, n_lambda_steps, ratio, seed, noise=True,
             vectorized=True, tracker_cov0=None, rng=None):
    """Drive the oracle like the reference tests do (test_filters_mat_simulator.py:163-176):
    EKF tracker, ``process_noise_sampler = rng.multivariate_normal(0, Q, N)`` from the
    config rng (or no process noise, the reference default, when ``noise`` is False)."""
    rng = np.random.default_rng(seed) if rng is None else rng
    tracker = make_ekf_tracker(model, mean0, cov0 if tracker_cov0 is None else tracker_cov0)
    pf = LEDHOracle(tracker, model, n_particles=n_particles, n_lambda_steps=n_lambda_steps,
                    resample_ess_ratio=ratio, rng=rng, vectorized=vectorized)
    st = pf.init_from_gaussian(mean0, cov0)
    init = st.particles.copy()
    T = len(Z)
    out = dict(means=np.zeros((T, model.nx)), covs=np.zeros((T, model.nx, model.nx)), ess=np.zeros(T),
               flags=np.zeros(T, dtype=bool), conds=np.zeros((T, max(1, n_lambda_steps))))
    sampler = (lambda N, nx: rng.multivariate_normal(np.zeros(nx), model.Q, size=N)) if noise else None
    for t in range(T):
        st = pf.step(st, np.atleast_1d(Z[t]), process_noise_sampler=sampler)
        out["means"][t] = st.mean
        out["covs"][t] = st.cov
        out["ess"][t] = pf.last_ess
        out["flags"][t] = pf.last_resampled
        out["conds"][t] = st.diagnostics["condition_numbers"]
    out["init_particles"] = init
    out["final_particles"] = st.particles.copy()
    out["final_weights"] = st.weights.copy()
    return out
