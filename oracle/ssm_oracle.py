"""State-space-model plugins (g, h, Q, R) restated for the oracle — TEST INFRASTRUCTURE ONLY.

Each builder returns per-particle callables (the reference's closures) AND
vectorised ``(N, nx)`` forms that are bit-identical to them, so the oracle can
run either the faithful reference cost profile or a fast restatement.

Sources restated (paths relative to /root/reference):

* SV test-harness wiring: ``tests/integration_tests/test_pf_vs_simulator_sv.py:46-56``
  ``g = a*x``, ``h = b*exp(x/2)``, ``Q = s^2``, ``R = 0.1``.
* SV standard wiring: ``notebooks/PF_VS_experiments.ipynb`` cell 3 (``R = b^2``).
* SV log-squared wiring: ``notebooks/PF_VS_experiments.ipynb`` cell 6
  ``z = log y^2``, ``h = log b^2 + x + E[log chi2_1]``, ``R = pi^2/2``.
* Lorenz-96: ``simulator/simulator_Lorenz_96.py:35-84`` (rhs, RK4) and ``:386-389``
  (``H_idx = arange(0, nx, obs_fraction)``, ``R = std^2 I``).
* Multi-target acoustic, joint 16-D wiring: ``notebooks/PF_PF_results_reproduction_
  multi_target_acoustic_tracking.ipynb`` cells 3 and 5 (``g_joint``, ``h_joint``,
  ``Q_joint = blockdiag(article_process_noise_cov())``, ``R = 0.1^2 I``).
* Linear test system: ``tests/unit_tests/models/test_pf_shapes_and_api.py:8-23``.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np

# E[log chi^2_1] = digamma(1/2) - log(1/2) and Var = polygamma(1, 1/2) = pi^2/2,
# computed the way the notebook does (PF_VS_experiments.ipynb cell 6).
try:  # scipy is importable in the build container and on the GPU box
    import scipy.special as _sp

    LOGCHI2_MEAN = float(_sp.digamma(0.5) - np.log(0.5))
    LOGCHI2_VAR = float(_sp.polygamma(1, 0.5))
except Exception:  # pragma: no cover - fallback literal values of the same doubles
    LOGCHI2_MEAN = -1.2703628454614782
    LOGCHI2_VAR = 4.934802200544679


@dataclass
class SSM:
    nx: int
    nz: int
    Q: np.ndarray
    R: np.ndarray
    g: Callable          # per particle: g(x (nx,), u) -> (nx,)
    h: Callable          # per particle: h(x (nx,)) -> (nz,)
    g_vec: Callable      # vectorised:   g(X (N,nx), u) -> (N,nx)
    h_vec: Callable      # vectorised:   h(X (N,nx)) -> (N,nz)
    # optional: J_h(x_i)^T g_i per particle, (X (N,nx), G (N,nz)) -> (N,nx) (test bounds; the
    # analytic Jacobians of the models' h, checked against finite differences by the CPU tests)
    hjt_vec: Optional[Callable] = None


def sv_harness(alpha: float, sigma: float, beta: float, R: float = 0.1) -> SSM:
    """test_pf_vs_simulator_sv.py:46-56 (and the standard notebook wiring with R=beta^2)."""

    def g(x, u):
        return np.array([alpha * x[0]])

    def h(x):
        return np.array([beta * np.exp(0.5 * x[0])])

    return SSM(1, 1, np.array([[sigma ** 2]]), np.array([[R]]), g, h,
               lambda X, u: alpha * X, lambda X: beta * np.exp(0.5 * X))


def sv_logsq(alpha: float, sigma: float, beta: float) -> SSM:
    """PF_VS_experiments.ipynb cell 6: observations must be ``log(Y**2)``."""
    log_beta_sq = np.log(beta ** 2)

    def g(x, u):
        x = np.atleast_1d(x)
        return alpha * x

    def h(x):
        x = np.atleast_1d(x)
        return log_beta_sq + x + LOGCHI2_MEAN

    return SSM(1, 1, np.array([[sigma ** 2]]), np.array([[LOGCHI2_VAR]]), g, h,
               lambda X, u: alpha * X, lambda X: log_beta_sq + X + LOGCHI2_MEAN, lambda X, G: np.array(G, float))


def l96_rhs(x, F):
    """simulator_Lorenz_96.py:35-59 along the last axis: (x[i+1] - x[i-2]) x[i-1] - x[i] + F, cyclic
    (one wrapped copy instead of three np.roll copies; bitwise the same values)."""
    n = x.shape[-1]
    xp = np.concatenate([x[..., -2:], x, x[..., :1]], axis=-1)  # xp[j] = x[j - 2]
    return (xp[..., 3:n + 3] - xp[..., 0:n]) * xp[..., 1:n + 1] - x + F


def l96_rk4(x, dt, F):
    """simulator_Lorenz_96.py:62-84 with f = l96_rhs(., F)."""
    k1 = l96_rhs(x, F)
    k2 = l96_rhs(x + 0.5 * dt * k1, F)
    k3 = l96_rhs(x + 0.5 * dt * k2, F)
    k4 = l96_rhs(x + dt * k3, F)
    return x + (dt / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)


def _scatter_cols(X, G, idx):
    out = np.zeros(np.shape(X))
    out[:, idx] = G
    return out


def lorenz96(nx: int = 40, F: float = 8.0, dt: float = 0.01, obs_fraction: int = 4,
             obs_error_std: float = 1.0, q_std: float = 0.1) -> SSM:
    """L96 SIR wiring: g = one RK4 step, h = x[H_idx], R = std^2 I, Q = q_std^2 I (build's choice)."""
    H_idx = np.arange(0, nx, obs_fraction)
    nz = H_idx.size
    return SSM(nx, nz, (q_std ** 2) * np.eye(nx), (obs_error_std ** 2) * np.eye(nz),
               lambda x, u: l96_rk4(x, dt, F), lambda x: x[H_idx],
               lambda X, u: l96_rk4(X, dt, F), lambda X: X[:, H_idx], lambda X, G: _scatter_cols(X, G, H_idx))


def mat_joint(sensors: np.ndarray, psi: float = 10.0, d0: float = 0.1, n_targets: int = 4,
              meas_noise_std: float = 0.1, Q_single: Optional[np.ndarray] = None) -> SSM:
    """Joint multi-target acoustic wiring (MAT notebook cells 3, 5)."""
    S = np.asarray(sensors, float)
    ns = S.shape[0]
    C = n_targets
    Fcv = np.array([[1.0, 0.0, 1.0, 0.0], [0.0, 1.0, 0.0, 1.0],
                    [0.0, 0.0, 1.0, 0.0], [0.0, 0.0, 0.0, 1.0]])
    if Q_single is None:  # simulator_Multi_acoustic_tracking.py:104-127
        Q_single = (1.0 / 20.0) * np.array([[1.0 / 3.0, 0.0, 0.5, 0.0], [0.0, 1.0 / 3.0, 0.0, 0.5],
                                            [0.5, 0.0, 1.0, 0.0], [0.0, 0.5, 0.0, 1.0]])
    nx = 4 * C
    Q = np.zeros((nx, nx))
    for c in range(C):
        Q[4 * c:4 * c + 4, 4 * c:4 * c + 4] = Q_single
    R = np.eye(ns) * meas_noise_std ** 2

    def g(x, u):
        out = np.zeros(nx)
        for c in range(C):
            out[4 * c:4 * c + 4] = Fcv @ x[4 * c:4 * c + 4]
        return out

    def h(x):
        z = np.zeros(ns)
        for c in range(C):
            pos = x[4 * c:4 * c + 2]
            zc = np.zeros(ns)
            for s in range(ns):
                zc[s] = psi / (np.sum((pos - S[s]) ** 2) + d0)
            z += zc
        return z

    def g_vec(X, u):
        out = np.empty_like(X)
        for c in range(C):
            out[:, 4 * c:4 * c + 4] = X[:, 4 * c:4 * c + 4] @ Fcv.T
        return out

    def h_vec(X):
        z = np.zeros((X.shape[0], ns))
        for c in range(C):
            dx = X[:, 4 * c, None] - S[None, :, 0]
            dy = X[:, 4 * c + 1, None] - S[None, :, 1]
            z += psi / ((dx ** 2 + dy ** 2) + d0)
        return z

    def hjt_vec(X, G):  # d h_s / d p_c = -2 psi (p_c - s) / (|p_c - s|^2 + d0)^2
        out = np.zeros(X.shape)
        for c in range(C):
            dx = X[:, 4 * c, None] - S[None, :, 0]
            dy = X[:, 4 * c + 1, None] - S[None, :, 1]
            k = -2.0 * psi / ((dx ** 2 + dy ** 2) + d0) ** 2 * G
            out[:, 4 * c] = np.sum(k * dx, axis=1)
            out[:, 4 * c + 1] = np.sum(k * dy, axis=1)
        return out

    return SSM(nx, ns, Q, R, g, h, g_vec, h_vec, hjt_vec)


def linear(A: np.ndarray, H: np.ndarray, Q: np.ndarray, R: np.ndarray) -> SSM:
    """test_pf_shapes_and_api.py:8-23 (``g = A x (+u)``, ``h = H x``)."""
    A = np.asarray(A, float)
    H = np.asarray(H, float)

    def g(x, u):
        return A @ x if u is None else A @ x + u

    def g_vec(X, u):
        Y = X @ A.T
        return Y if u is None else Y + np.asarray(u, float)

    return SSM(A.shape[0], H.shape[0], np.asarray(Q, float), np.asarray(R, float),
               g, lambda x: H @ x, g_vec, lambda X: X @ H.T)


def bearings_9d(gamma: float = 1e-2, dt: float = 0.1, q: float = 1e-4, r: float = 1e-6) -> SSM:
    """The 9-D bearings-only SIR of notebooks/SPF_results_reproduction_example2.ipynb:
    cell 1 ``e2_build_system_matrix`` (A = gamma [[-I, I, 0], [0, -I, I], [0, 0, -I]]),
    ``e2_measurement_function`` (azimuth atan2(x, y), elevation atan2(z, |(x, y)|), sensor at
    the origin), ``R = 1e-6 I``; cell 7 ``g_func = x + A x dt``, ``Q = 1e-4 I``."""
    I3, Z3 = np.eye(3), np.zeros((3, 3))
    A = gamma * np.vstack((np.hstack((-I3, I3, Z3)), np.hstack((Z3, -I3, I3)), np.hstack((Z3, Z3, -I3))))

    def g(x, u):
        return x + A @ x * dt

    def h(x):
        r_xy = np.sqrt(x[0] ** 2 + x[1] ** 2)
        return np.array([np.arctan2(x[0], x[1]), np.arctan2(x[2], r_xy)])

    def g_vec(X, u):
        return X + (X @ A.T) * dt

    def h_vec(X):
        r_xy = np.sqrt(X[:, 0] ** 2 + X[:, 1] ** 2)
        return np.stack([np.arctan2(X[:, 0], X[:, 1]), np.arctan2(X[:, 2], r_xy)], axis=1)

    ssm = SSM(9, 2, q * np.eye(9), r * np.eye(2), g, h, g_vec, h_vec)
    ssm.A = A
    ssm.dt = dt
    return ssm
