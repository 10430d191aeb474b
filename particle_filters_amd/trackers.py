"""Gaussian trackers that feed the LEDH flow its prior covariance P_k.

The reference's LEDHFlowPF takes any object with ``predict() -> (m, P)``,
``update(z)`` and ``get_past_mean()`` (``models/LEDH_particle_filter.py:13-16``,
the ``GaussianTracker`` protocol); its tests wrap the EKF
(``models/extended_kalman_filter.py``) in a small adaptor
(``tests/unit_tests/models/test_ledh_flow_pf.py:12-33``).  This module provides the
same pieces for this package:

* :class:`ExtendedKalmanFilter` / :class:`EKFState` — the additive-noise EKF of
  ``extended_kalman_filter.py:110-256`` (analytic or finite-difference Jacobians,
  Joseph form, innovation jitter), host NumPy: nx x nx algebra per step, no particles.
* :class:`EKFTracker` — the GaussianTracker adaptor.

The tracker never sees the particles, so :meth:`particle_filters_amd.ledh.LEDHFlowPF.run`
can run it ahead over the whole observation sequence and hand the device the
stack of covariances in one upload.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import numpy as np

Array = np.ndarray


def numerical_jacobian_g(g: Callable, x: Array, u: Optional[Array], eps: float = 1e-6) -> Array:
    """Forward-difference Jacobian of g(x, u) (extended_kalman_filter.py:43-75)."""
    x = np.asarray(x, dtype=float)
    y0 = np.asarray(g(x, u), dtype=float)
    J = np.zeros((y0.size, x.size))
    for j in range(x.size):
        dx = np.zeros(x.size)
        dx[j] = eps
        J[:, j] = (g(x + dx, u) - y0) / eps
    return J


def numerical_jacobian_h(h: Callable, x: Array, eps: float = 1e-6) -> Array:
    """Forward-difference Jacobian of h(x) (extended_kalman_filter.py:78-107)."""
    x = np.asarray(x, dtype=float)
    z0 = np.asarray(h(x), dtype=float)
    J = np.zeros((z0.size, x.size))
    for j in range(x.size):
        dx = np.zeros(x.size)
        dx[j] = eps
        J[:, j] = (h(x + dx) - z0) / eps
    return J


@dataclass
class EKFState:
    mean: Array
    cov: Array
    t: int


class ExtendedKalmanFilter:
    """x_k = g(x_{k-1}, u) + w, z_k = h(x_k) + v (extended_kalman_filter.py:110-160)."""

    def __init__(self, g, h, Q, R, jac_g=None, jac_h=None, *, joseph: bool = False, jitter: float = 0.0):
        self.g, self.h = g, h
        self.Q = np.asarray(Q, dtype=float)
        self.R = np.asarray(R, dtype=float)
        self.jac_g, self.jac_h = jac_g, jac_h
        self.joseph = bool(joseph)
        self.jitter = float(jitter)
        nx, nz = self.Q.shape[0], self.R.shape[0]
        assert self.Q.shape == (nx, nx), "Q must be square."
        assert self.R.shape == (nz, nz), "R must be square."

    def predict(self, state: EKFState, u: Optional[Array] = None) -> EKFState:
        """extended_kalman_filter.py:164-194."""
        x = np.asarray(state.mean, dtype=float)
        P = np.asarray(state.cov, dtype=float)
        x_pred = np.asarray(self.g(x, u), dtype=float)
        G = self.jac_g(x, u) if self.jac_g is not None else numerical_jacobian_g(self.g, x, u)
        if G.shape != (x.size, x.size):
            raise ValueError("jac_g must return shape (nx, nx).")
        return EKFState(mean=x_pred, cov=G @ P @ G.T + self.Q, t=state.t + 1)

    def update(self, pred: EKFState, z: Array) -> EKFState:
        """extended_kalman_filter.py:196-241."""
        x_pred = np.asarray(pred.mean, dtype=float)
        P_pred = np.asarray(pred.cov, dtype=float)
        z = np.asarray(z, dtype=float)
        H = self.jac_h(x_pred) if self.jac_h is not None else numerical_jacobian_h(self.h, x_pred)
        if H.shape[0] != z.size or H.shape[1] != x_pred.size:
            raise ValueError("jac_h must return shape (nz, nx).")
        y = z - np.asarray(self.h(x_pred), dtype=float)
        S = H @ P_pred @ H.T + self.R
        if self.jitter > 0.0:
            S = S + self.jitter * np.eye(z.size)
        K = P_pred @ H.T @ np.linalg.inv(S)
        x_post = x_pred + K @ y
        I = np.eye(P_pred.shape[0])
        if self.joseph:
            A = I - K @ H
            P_post = A @ P_pred @ A.T + K @ self.R @ K.T
        else:
            P_post = (I - K @ H) @ P_pred
        return EKFState(mean=x_post, cov=P_post, t=pred.t)

    def step(self, state: EKFState, z: Array, u: Optional[Array] = None) -> EKFState:
        return self.update(self.predict(state, u=u), z)


class EKFTracker:
    """GaussianTracker adaptor (LEDH_particle_filter.py:13-16) around an EKF."""

    def __init__(self, ekf: ExtendedKalmanFilter, initial_state: EKFState):
        self.ekf = ekf
        self.state = initial_state
        self.past_mean = np.asarray(initial_state.mean, float).copy()

    def predict(self) -> Tuple[Array, Array]:
        self.past_mean = self.state.mean.copy()
        self.state = self.ekf.predict(self.state, u=None)
        return self.state.mean, self.state.cov

    def update(self, z_k: Array) -> Tuple[Array, Array]:
        self.state = self.ekf.update(self.state, z_k)
        return self.state.mean, self.state.cov

    def get_past_mean(self) -> Array:
        return self.past_mean
