"""Device state-space-model plugins: the ``g`` / ``h`` arguments of ``ParticleFilter``.

The reference passes arbitrary Python callables ``g(x, u) -> (nx,)`` and
``h(x) -> (nz,)`` (``/root/reference/models/particle_filter.py:20-22``) and calls
them once per particle (``:237``, ``:257``).  A GPU cannot call Python per
particle, so the engine takes *model objects* that

* describe the function to the HIP kernels (a kind + parameters, see
  ``include/pf_engine.h`` ``PF_TRANS_*`` / ``PF_OBS_*``), and
* are still callables with the reference's per-particle semantics, so the very
  same objects can be handed to the reference's own ``ParticleFilter``.

The wirings the reference uses map to one-liners:

======================================================  =========================================
reference closure                                        here
======================================================  =========================================
``lambda x, u: alpha * x`` (SV, test_pf_vs_simulator_sv.py:50)     ``SVTransition(alpha)``
``lambda x: beta*np.exp(0.5*x)`` (:54)                    ``ExpHalfObservation(beta)``
log-squared ``log b^2 + x + E`` (PF_VS notebook cell 6)   ``SVLogSqObservation(beta)``
``A @ x (+u)`` / ``H @ x`` (test_pf_shapes_and_api.py)   ``LinearTransition(A)`` / ``LinearObservation(H)``
``rk4_step(x, dt, l96_rhs)`` / ``x[H_idx]`` (L96)         ``L96Transition(F, dt, nx)`` / ``SelectObservation(H_idx, nx)``
MAT joint ``g_joint`` / ``h_joint``                      ``CVTransition(C, dt)`` / ``AcousticObservation(S, psi, d0, C)``
exact SV ``sv_log_likelihood_fn`` (test_dpf_vs_sv_       ``SVExactObservation(beta)`` (R unused)
simulator.py:60-97)
``x + A @ x * dt`` / ``e2_measurement_function``         ``LinearTransition(I + A dt)`` /
(SPF example 2, 9-D bearings-only SIR)                   ``BearingsObservation(9)``
======================================================  =========================================
"""

from __future__ import annotations

from typing import Optional

import numpy as np

from . import _native as N

# E[log chi^2_1] = digamma(1/2) - log(1/2), Var = polygamma(1, 1/2) = pi^2/2
LOGCHI2_MEAN = -1.2703628454614782
LOGCHI2_VAR = 4.934802200544679


class Transition:
    kind: int
    nx: int

    def params(self) -> np.ndarray:
        raise NotImplementedError

    def __call__(self, x, u=None):  # per particle, reference semantics
        raise NotImplementedError


class Observation:
    kind: int
    nx: int
    nz: int

    def params(self) -> np.ndarray:
        raise NotImplementedError

    def __call__(self, x):
        raise NotImplementedError


# ---------------------------------------------------------------------------
# transitions
# ---------------------------------------------------------------------------
class LinearTransition(Transition):
    """``g(x, u) = A x (+ u)``."""

    kind = N.PF_TRANS_LINEAR

    def __init__(self, A):
        self.A = np.atleast_2d(np.asarray(A, float))
        if self.A.shape[0] != self.A.shape[1]:
            raise ValueError("A must be square")
        self.nx = self.A.shape[0]

    def params(self):
        return np.ascontiguousarray(self.A.ravel())

    def __call__(self, x, u=None, v=None):
        x = np.asarray(x, float)
        y = self.A @ x if u is None else self.A @ x + u
        return y if v is None else y + v

    def jacobian(self, x, u=None):
        """dg/dx = A (the EKF's analytic Jacobian of g)."""
        return self.A.copy()


class SVTransition(LinearTransition):
    """Stochastic-volatility AR(1): ``g(x) = alpha * x`` (elementwise for vector alpha)."""

    def __init__(self, alpha):
        self.alpha = np.atleast_1d(np.asarray(alpha, float))
        super().__init__(np.diag(self.alpha))

    def __call__(self, x, u=None, v=None):
        x = np.atleast_1d(np.asarray(x, float))
        y = self.alpha * x
        y = y if u is None else y + u
        return y if v is None else y + v


class CVTransition(LinearTransition):
    """Joint constant-velocity dynamics of ``n_targets`` ``[x, y, vx, vy]`` blocks
    (simulator_Multi_acoustic_tracking.py:77-101; MAT notebook ``g_joint``)."""

    def __init__(self, n_targets: int = 4, dt: float = 1.0):
        F = np.eye(4)
        F[0, 2] = dt
        F[1, 3] = dt
        self.n_targets = n_targets
        self.F = F
        super().__init__(np.kron(np.eye(n_targets), F))

    def __call__(self, x, u=None, v=None):
        x = np.asarray(x, float)
        out = np.zeros(4 * self.n_targets)
        for c in range(self.n_targets):
            out[4 * c:4 * c + 4] = self.F @ x[4 * c:4 * c + 4]
        out = out if u is None else out + u
        return out if v is None else out + v


class L96Transition(Transition):
    """One RK4 step of Lorenz-96 (simulator_Lorenz_96.py:35-84)."""

    kind = N.PF_TRANS_L96

    def __init__(self, F: float = 8.0, dt: float = 0.01, nx: int = 40):
        self.F = float(F)
        self.dt = float(dt)
        self.nx = int(nx)

    def params(self):
        return np.array([self.F, self.dt])

    def _rhs(self, x):
        return (np.roll(x, -1) - np.roll(x, 2)) * np.roll(x, 1) - x + self.F

    def __call__(self, x, u=None, v=None):
        x = np.asarray(x, float)
        dt = self.dt
        k1 = self._rhs(x)
        k2 = self._rhs(x + 0.5 * dt * k1)
        k3 = self._rhs(x + 0.5 * dt * k2)
        k4 = self._rhs(x + dt * k3)
        y = x + (dt / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)
        y = y if u is None else y + u
        return y if v is None else y + v

    def jacobian(self, x, u=None):
        """Tangent-linear map of one RK4 step at x (analytic EKF Jacobian of g)."""
        x = np.asarray(x, float)
        n, dt, F = self.nx, self.dt, self.F
        idx = np.arange(n)

        def J_rhs(y):  # d/dy of (y[a+1] - y[a-2]) y[a-1] - y[a] + F
            J = -np.eye(n)
            J[idx, (idx + 1) % n] += y[(idx - 1) % n]
            J[idx, (idx - 2) % n] -= y[(idx - 1) % n]
            J[idx, (idx - 1) % n] += y[(idx + 1) % n] - y[(idx - 2) % n]
            return J

        I = np.eye(n)
        k1 = self._rhs(x)
        y2 = x + 0.5 * dt * k1
        k2 = self._rhs(y2)
        y3 = x + 0.5 * dt * k2
        k3 = self._rhs(y3)
        y4 = x + dt * k3
        D1 = J_rhs(x)
        D2 = J_rhs(y2) @ (I + 0.5 * dt * D1)
        D3 = J_rhs(y3) @ (I + 0.5 * dt * D2)
        D4 = J_rhs(y4) @ (I + dt * D3)
        return I + (dt / 6.0) * (D1 + 2 * D2 + 2 * D3 + D4)


# ---------------------------------------------------------------------------
# observations
# ---------------------------------------------------------------------------
class LinearObservation(Observation):
    """``h(x) = H x + c``."""

    kind = N.PF_OBS_LINEAR

    def __init__(self, H, c=None):
        self.H = np.atleast_2d(np.asarray(H, float))
        self.nz, self.nx = self.H.shape
        self.c = np.zeros(self.nz) if c is None else np.atleast_1d(np.asarray(c, float))

    def params(self):
        return np.ascontiguousarray(np.r_[self.H.ravel(), self.c])

    def __call__(self, x):
        return self.H @ np.asarray(x, float) + self.c

    def jacobian(self, x):
        return self.H.copy()


class SVLogSqObservation(LinearObservation):
    """Log-squared SV wiring ``h(x) = log(beta^2) + x + E[log chi^2_1]`` — observations
    must be ``log(Y**2)``, ``R = pi^2/2`` (PF_VS_experiments.ipynb cell 6)."""

    def __init__(self, beta: float):
        self.beta = float(beta)
        self.log_beta_sq = float(np.log(self.beta ** 2))
        super().__init__(np.eye(1), [self.log_beta_sq + LOGCHI2_MEAN])

    def __call__(self, x):
        x = np.atleast_1d(np.asarray(x, float))
        return self.log_beta_sq + x + LOGCHI2_MEAN


class SelectObservation(LinearObservation):
    """Partial observation ``h(x) = x[H_idx]`` (simulator_Lorenz_96.py:147-161)."""

    def __init__(self, H_idx, nx: int):
        self.H_idx = np.asarray(H_idx, dtype=int)
        H = np.zeros((self.H_idx.size, nx))
        H[np.arange(self.H_idx.size), self.H_idx] = 1.0
        super().__init__(H)

    def __call__(self, x):
        return np.asarray(x, float)[self.H_idx]


class ExpHalfObservation(Observation):
    """``h(x) = beta * exp(x / 2)`` elementwise (SV standard / test-harness wiring)."""

    kind = N.PF_OBS_EXP_HALF

    def __init__(self, beta):
        self.beta = np.atleast_1d(np.asarray(beta, float))
        self.nx = self.nz = self.beta.size

    def params(self):
        return np.ascontiguousarray(self.beta)

    def __call__(self, x):
        x = np.atleast_1d(np.asarray(x, float))
        return self.beta * np.exp(0.5 * x)

    def jacobian(self, x):
        x = np.atleast_1d(np.asarray(x, float))
        return np.diag(0.5 * self.beta * np.exp(0.5 * x))


class SVExactObservation(Observation):
    """The exact stochastic-volatility likelihood ``y_k ~ N(0, (beta_k e^{x_k/2})^2)``.

    The reference's ``ParticleFilter`` only takes Gaussian ``h``/``R`` wirings; this one is
    the TensorFlow test's ``sv_log_likelihood_fn``
    (``tests/integration_tests/test_dpf_vs_sv_simulator.py:60-97``):
    ``log p(y|x) = -0.5 log 2pi - log(beta e^{x/2}) - 0.5 (y / (beta e^{x/2}))^2``, evaluated
    on the device without the constants (they cancel in the normalised weights, as pf.py's
    dropped Gaussian constants do; ``log_norm`` outputs differ from the full log-density by
    ``-nz (0.5 log 2pi + log beta)`` per step).  Observations are the raw ``Y`` (not log Y^2).
    ``R`` is not used: pass ``None`` (taken as I) or any positive-definite matrix.
    Calling the object gives the observation scale ``beta e^{x/2}``."""

    kind = N.PF_OBS_SV_EXACT

    def __init__(self, beta):
        self.beta = np.atleast_1d(np.asarray(beta, float))
        self.nx = self.nz = self.beta.size

    def params(self):
        return np.ascontiguousarray(self.beta)

    def __call__(self, x):
        x = np.atleast_1d(np.asarray(x, float))
        return self.beta * np.exp(0.5 * x)

    def log_likelihood(self, y, x):
        """The full log-density of the reference test (with its constants), per particle."""
        sig = self(x)
        y = np.atleast_1d(np.asarray(y, float))
        return float(np.sum(-0.5 * np.log(2 * np.pi) - np.log(sig) - 0.5 * (y / sig) ** 2))


class BearingsObservation(Observation):
    """Azimuth / elevation of the target seen from a sensor at ``s``:
    ``[atan2(x - sx, y - sy), atan2(z - sz, |(x, y) - (sx, sy)|)]`` with the position in the
    first three state components (SPF_results_reproduction_example2.ipynb cell 1
    ``e2_measurement_function``, sensor at the origin; the notebook's 9-D SIR comparison,
    cell 7).  Runs on the runtime-shape kernels (any nx >= 3)."""

    kind = N.PF_OBS_BEARINGS

    def __init__(self, nx: int = 9, sensor=(0.0, 0.0, 0.0)):
        self.nx = int(nx)
        self.nz = 2
        self.sensor = np.asarray(sensor, float).reshape(3)
        if self.nx < 3:
            raise ValueError("bearings need a 3-D position in the state")

    def params(self):
        return np.ascontiguousarray(self.sensor)

    def __call__(self, x):
        x = np.asarray(x, float)
        d = x[:3] - self.sensor
        return np.array([np.arctan2(d[0], d[1]), np.arctan2(d[2], np.sqrt(d[0] ** 2 + d[1] ** 2))])


def observation_noise(h, R):
    """R as the engine takes it: the exact SV likelihood has none (None -> I)."""
    if R is None:
        if getattr(h, "kind", None) == N.PF_OBS_SV_EXACT:
            return np.eye(h.nz)
        raise ValueError("R is required for a Gaussian observation model")
    return np.atleast_2d(np.asarray(R, float))


class AcousticObservation(Observation):
    """Summed acoustic amplitudes ``z_s = sum_c psi / (|p_c - s|^2 + d0)`` of
    ``n_targets`` ``[x, y, vx, vy]`` blocks (simulator_Multi_acoustic_tracking.py:273-309;
    MAT notebook ``h_joint``)."""

    kind = N.PF_OBS_ACOUSTIC

    def __init__(self, sensors, psi: float = 10.0, d0: float = 0.1, n_targets: int = 4):
        self.S = np.asarray(sensors, float).reshape(-1, 2)
        self.psi = float(psi)
        self.d0 = float(d0)
        self.n_targets = int(n_targets)
        self.nz = self.S.shape[0]
        self.nx = 4 * self.n_targets

    def params(self):
        return np.ascontiguousarray(np.r_[self.psi, self.d0, self.S[:, 0], self.S[:, 1]])

    def __call__(self, x):
        x = np.asarray(x, float)
        z = np.zeros(self.nz)
        for c in range(self.n_targets):
            pos = x[4 * c:4 * c + 2]
            zc = np.zeros(self.nz)
            for s in range(self.nz):
                zc[s] = self.psi / (np.sum((pos - self.S[s]) ** 2) + self.d0)
            z += zc
        return z

    def jacobian(self, x):
        """Analytic dh/dx (test_filters_mat_simulator.py:55-64, summed over targets)."""
        x = np.asarray(x, float)
        H = np.zeros((self.nz, self.nx))
        for c in range(self.n_targets):
            pos = x[4 * c:4 * c + 2]
            for s in range(self.nz):
                diff = pos - self.S[s]
                denom = (np.sum(diff ** 2) + self.d0) ** 2
                H[s, 4 * c] = -2.0 * self.psi * diff[0] / denom
                H[s, 4 * c + 1] = -2.0 * self.psi * diff[1] / denom
        return H


# ---------------------------------------------------------------------------
# Gaussian log densities of the LEDH weight (ledh.py:21-22 LogTransPdf / LogLikePdf)
# ---------------------------------------------------------------------------
class GaussianTransitionDensity:
    """``log p(x_k | x_{k-1}) = log N(x_k; g(x_{k-1}), Q)`` — the transition density of every
    LEDH wiring in the reference tests (test_ledh_flow_pf.py:92-95,
    test_filters_mat_simulator.py:66-70).  Callable with the reference's signature; the
    engine evaluates it on the device from (g, Q)."""

    def __init__(self, g: Transition, Q):
        self.g = g
        self.Q = np.atleast_2d(np.asarray(Q, float))

    def __call__(self, xk, xkm1):
        diff = np.atleast_1d(np.asarray(xk, float)) - self.g(xkm1)
        return -0.5 * (diff.T @ np.linalg.solve(self.Q, diff) + np.log(np.linalg.det(2 * np.pi * self.Q)))


class GaussianLikelihood:
    """``log p(z | x) = log N(z; h(x), R)`` (test_ledh_flow_pf.py:97-100,
    test_filters_mat_simulator.py:72-77)."""

    def __init__(self, h: Observation, R):
        self.h = h
        self.R = np.atleast_2d(np.asarray(R, float))

    def __call__(self, z, x):
        diff = np.atleast_1d(np.asarray(z, float)) - self.h(x)
        return -0.5 * (diff.T @ np.linalg.solve(self.R, diff) + np.log(np.linalg.det(2 * np.pi * self.R)))


def is_device_model(g, h) -> bool:
    return isinstance(g, Transition) and isinstance(h, Observation)


def describe(g: Transition, h: Observation, Q: np.ndarray, R: np.ndarray):
    """Validate the pair against Q/R and return (ModelDesc, keepalive arrays)."""
    nx = Q.shape[0]
    nz = R.shape[0]
    if g.nx != nx:
        raise ValueError(f"g has state dimension {g.nx}, Q is {Q.shape}")
    if h.nx != nx:
        raise ValueError(f"h expects state dimension {h.nx}, Q is {Q.shape}")
    if h.nz != nz:
        raise ValueError(f"h has observation dimension {h.nz}, R is {R.shape}")
    tp = np.ascontiguousarray(g.params(), dtype=float)
    op = np.ascontiguousarray(h.params(), dtype=float)
    Qc = np.ascontiguousarray(Q, dtype=float)
    Rc = np.ascontiguousarray(R, dtype=float)
    d = N.ModelDesc(nx, nz, g.kind, h.kind, N.dptr(tp), tp.size, N.dptr(op), op.size, N.dptr(Qc), N.dptr(Rc))
    return d, (tp, op, Qc, Rc)


def supported(g: Transition, h: Observation) -> bool:
    """Can the engine run this pair (any shape whose kinds fit, pf_model_supported)?"""
    return bool(N.load().pf_model_supported(g.nx, h.nz, g.kind, h.kind))


def compiled(g: Transition, h: Observation) -> bool:
    """Is the pair's shape in the compiled register-state list (else the runtime-shape kernels run)?"""
    return bool(N.load().pf_model_compiled(g.nx, h.nz, g.kind, h.kind))


def kernel_path_code(kernel_path: str) -> int:
    """``"auto"``: the compiled shape's register-state kernels when (nx, nz, g, h) is in the
    compiled list, else the runtime-shape kernels (any nx, nz, ``csrc/pf_dyn.h``);
    ``"runtime"``: always the runtime-shape kernels."""
    if kernel_path not in ("auto", "runtime"):
        raise ValueError("kernel_path must be 'auto' or 'runtime'")
    return N.PF_PATH_RUNTIME if kernel_path == "runtime" else N.PF_PATH_AUTO


def sv_logsq_observations(Y) -> np.ndarray:
    """``Z = log(Y^2)`` for :class:`SVLogSqObservation`."""
    return np.log(np.asarray(Y, float) ** 2)
