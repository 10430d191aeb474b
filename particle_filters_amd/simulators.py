"""Synthetic-data generators feeding the SIR engine (the ``simulator_*`` surface).

Host-side NumPy, run once per experiment — they are the data sources either
side of the hot path, not the hot path itself.  Each generator reproduces the
reference's draw order and arithmetic so a given seed yields the same arrays
bit-for-bit (pinned by ``tests/test_simulators.py`` against fixtures that the
reference produced, ``tests/golden/{sv,l96,mat}_data.npz``).

Reference surfaces mirrored (paths under ``/root/reference/simulator``):

* ``simulator_sto_volatility_model.py``: ``SV1DResults`` :9-48, ``simulate_sv_1d`` :51-122
* ``simulator_Lorenz_96.py``: ``l96_rhs`` :35-59, ``rk4_step`` :62-84,
  ``l96_integrate`` :87-128, ``ObsModel`` :132-181,
  ``Lorenz96SimulationResult`` (+ ``save``/``load``) :185-295,
  ``simulate_lorenz96`` :299-436, ``compute_rmse`` :440-456,
  ``compute_ensemble_spread`` :459-475
* ``simulator_Multi_acoustic_tracking.py``: configs :29-73,
  ``build_cv_transition`` :77-101, ``article_process_noise_cov`` :104-127,
  ``article_initial_states`` :130-165, ``make_sensor_grid`` :169-192,
  ``simulate_cv_targets`` :196-270, ``acoustic_measurement_model`` :273-309,
  ``simulate_acoustic_dataset`` :312-346
"""

from __future__ import annotations

import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Callable, Dict, Optional, Tuple

import numpy as np

Array = np.ndarray

# ---------------------------------------------------------------------------
# 1-D stochastic volatility
# ---------------------------------------------------------------------------


@dataclass
class SV1DResults:
    """Latent log-volatility ``X`` (n,) and returns ``Y`` (n,) of one SV path."""

    X: Array
    Y: Array
    alpha: float
    sigma: float
    beta: float
    n: int
    seed: Optional[int] = None

    def save(self, filename: str) -> None:
        """``.npz`` with keys X, Y, alpha, sigma, beta, n, seed (reference format)."""
        np.savez(filename, X=self.X, Y=self.Y, alpha=self.alpha, sigma=self.sigma,
                 beta=self.beta, n=self.n, seed=self.seed)


def simulate_sv_1d(n: int, alpha: float, sigma: float, beta: float, *,
                   seed: Optional[int] = None, x0: Optional[float] = None) -> SV1DResults:
    """``X_t = alpha X_{t-1} + sigma V_t``, ``Y_t = beta exp(X_t/2) W_t``.

    Draw order (one ``default_rng(seed)``): X_1 from the stationary law unless
    ``x0`` is given, then all V (n-1), then all W (n).
    """
    if n <= 0:
        raise ValueError("n must be positive.")
    if not np.isfinite(alpha) or abs(alpha) >= 1:
        raise ValueError("alpha must be finite with |alpha| < 1 for stationarity.")
    if not np.isfinite(sigma) or sigma < 0:
        raise ValueError("sigma must be a finite, nonnegative scalar.")
    if not np.isfinite(beta) or beta < 0:
        raise ValueError("beta must be a finite, nonnegative scalar.")
    gen = np.random.default_rng(seed)
    X = np.empty(n, dtype=float)
    if x0 is not None:
        X[0] = float(x0)
    else:
        stationary_var = max(sigma ** 2 / (1.0 - alpha ** 2), 0.0)
        X[0] = gen.normal(0.0, np.sqrt(stationary_var))
    if n > 1:
        shocks = gen.standard_normal(n - 1)
        prev = X[0]
        for t in range(1, n):
            prev = alpha * prev + sigma * shocks[t - 1]
            X[t] = prev
    W = gen.standard_normal(n)
    Y = np.empty(n, dtype=float)
    Y[:] = (beta * np.exp(0.5 * X)) * W
    return SV1DResults(X=X, Y=Y, alpha=alpha, sigma=sigma, beta=beta, n=n, seed=seed)


# ---------------------------------------------------------------------------
# Lorenz-96
# ---------------------------------------------------------------------------


def l96_rhs(x: Array, F: float = 8.0) -> Array:
    """``dx_a/dt = (x_{a+1} - x_{a-2}) x_{a-1} - x_a + F`` with periodic indices."""
    x = np.asarray(x)
    ahead = np.roll(x, -1)
    behind1 = np.roll(x, 1)
    behind2 = np.roll(x, 2)
    return (ahead - behind2) * behind1 - x + F


def rk4_step(x: Array, dt: float, f: Callable[[Array], Array]) -> Array:
    """Classical fourth-order Runge-Kutta step of ``dx/dt = f(x)``."""
    s1 = f(x)
    s2 = f(x + 0.5 * dt * s1)
    s3 = f(x + 0.5 * dt * s2)
    s4 = f(x + dt * s3)
    return x + (dt / 6.0) * (s1 + 2 * s2 + 2 * s3 + s4)


def l96_integrate(x0: Array, dt: float, steps: int, F: float = 8.0, q_std: float = 0.0,
                  rng: Optional[np.random.Generator] = None) -> Array:
    """Trajectory ``(steps+1, nx)`` from ``x0``; optional additive N(0, q_std^2) per step."""
    gen = rng or np.random.default_rng()
    traj = np.empty((steps + 1, x0.size))
    x = x0.copy()
    traj[0] = x
    rhs = lambda z: l96_rhs(z, F)  # noqa: E731
    for t in range(1, steps + 1):
        x = rk4_step(x, dt, rhs)
        if q_std > 0:
            x = x + gen.normal(0.0, q_std, size=x.shape)
        traj[t] = x
    return traj


@dataclass
class ObsModel:
    """Partial linear observation ``y = x[H_idx] + v``, ``v ~ N(0, R)``."""

    H_idx: Array
    R: Array

    def H(self, x: Array) -> Array:
        return x[self.H_idx]

    def JH(self, x: Array) -> Array:
        J = np.zeros((self.H_idx.size, x.size))
        J[np.arange(self.H_idx.size), self.H_idx] = 1.0
        return J


@dataclass
class Lorenz96SimulationResult:
    truth_traj: Array
    ensemble_traj: Array
    observations: Array
    obs_times: Array
    H_idx: Array
    R: Array
    config: Dict[str, Any] = field(default_factory=dict)

    def save(self, filepath: str, overwrite: bool = False) -> None:
        """Arrays to ``<path>.npz`` and ``config`` to ``<path>.json`` (reference layout)."""
        path = Path(filepath)
        if not str(path).endswith(".npz"):
            path = path.with_suffix(".npz")
        if path.exists() and not overwrite:
            raise FileExistsError(f"File already exists: {path}")
        np.savez(path, truth_traj=self.truth_traj, ensemble_traj=self.ensemble_traj,
                 observations=self.observations, obs_times=self.obs_times,
                 H_idx=self.H_idx, R=self.R)
        with open(path.with_suffix(".json"), "w") as fh:
            json.dump(self.config, fh, indent=2)

    @classmethod
    def load(cls, filepath: str) -> "Lorenz96SimulationResult":
        path = Path(filepath)
        if not str(path).endswith(".npz"):
            path = path.with_suffix(".npz")
        arrays = np.load(path)
        cfg_path = path.with_suffix(".json")
        config = json.loads(cfg_path.read_text()) if cfg_path.exists() else {}
        return cls(truth_traj=arrays["truth_traj"], ensemble_traj=arrays["ensemble_traj"],
                   observations=arrays["observations"], obs_times=arrays["obs_times"],
                   H_idx=arrays["H_idx"], R=arrays["R"], config=config)


def simulate_lorenz96(nx: int = 1000, F: float = 8.0, dt: float = 0.01, spinup_steps: int = 1000,
                      total_steps: int = 1500, Np: int = 20, obs_interval: int = 20,
                      obs_fraction: int = 4, obs_error_std: float = 1.0,
                      perturbation_std: Optional[float] = None, x0: Optional[Array] = None,
                      seed: Optional[int] = None) -> Lorenz96SimulationResult:
    """Spin-up, perturbed ensemble, noise-free truth, and noisy partial observations.

    Draw order (one ``default_rng(seed)``): Np ensemble perturbations of size
    nx, then ny observation-noise draws per observation time.
    """
    gen = np.random.default_rng(seed)
    if perturbation_std is None:
        perturbation_std = np.sqrt(2.0)
    if x0 is None:
        start = np.full(nx, F, dtype=float)
        start[np.arange(0, nx, 5)] = F + 1.0
    else:
        start = np.asarray(x0, dtype=float)
        if start.shape != (nx,):
            raise ValueError(f"x0 must have shape ({nx},), got {start.shape}")
    after_spinup = l96_integrate(start, dt, spinup_steps, F=F, q_std=0.0, rng=gen)[-1]
    members = np.empty((Np, nx))
    for i in range(Np):
        members[i] = after_spinup + gen.normal(0.0, perturbation_std, size=nx)
    H_idx = np.arange(0, nx, obs_fraction)
    ny = H_idx.size
    R = obs_error_std ** 2 * np.eye(ny)
    truth = l96_integrate(after_spinup.copy(), dt, total_steps, F=F, q_std=0.0, rng=gen)
    ensemble = np.empty((Np, total_steps + 1, nx))
    for i in range(Np):
        ensemble[i] = l96_integrate(members[i], dt, total_steps, F=F, q_std=0.0, rng=gen)
    obs_times = np.arange(0, total_steps + 1, obs_interval)
    observations = np.empty((len(obs_times), ny))
    for k, t in enumerate(obs_times):
        observations[k] = truth[t][H_idx] + gen.normal(0.0, obs_error_std, size=ny)
    config = {
        "nx": int(nx), "F": float(F), "dt": float(dt), "spinup_steps": int(spinup_steps),
        "total_steps": int(total_steps), "Np": int(Np), "obs_interval": int(obs_interval),
        "obs_fraction": int(obs_fraction), "obs_error_std": float(obs_error_std),
        "perturbation_std": float(perturbation_std), "seed": seed, "ny": int(ny),
        "n_obs_times": int(len(obs_times)),
    }
    return Lorenz96SimulationResult(truth_traj=truth, ensemble_traj=ensemble,
                                    observations=observations, obs_times=obs_times,
                                    H_idx=H_idx, R=R, config=config)


def compute_rmse(forecast: Array, truth: Array) -> float:
    return float(np.sqrt(np.mean((forecast - truth) ** 2)))


def compute_ensemble_spread(ensemble: Array, axis: int = 0) -> Array:
    return np.std(ensemble, axis=axis)


# ---------------------------------------------------------------------------
# Multi-target acoustic tracking
# ---------------------------------------------------------------------------


@dataclass(frozen=True)
class DynamicsConfig:
    dt: float = 1.0


@dataclass(frozen=True)
class ScenarioConfig:
    n_targets: int = 4
    n_steps: int = 100
    area_xy: Tuple[float, float] = (40.0, 40.0)
    sensor_grid_shape: Tuple[int, int] = (5, 5)
    psi: float = 10.0
    d0: float = 0.1
    seed: int = 7
    use_article_init: bool = True


def build_cv_transition(dt: float) -> Array:
    """Constant-velocity transition for state ``[x, y, vx, vy]``."""
    F = np.eye(4)
    F[0, 2] = dt
    F[1, 3] = dt
    return F


def article_process_noise_cov() -> Array:
    """Fixed CV process-noise covariance (independent of dt)."""
    V = np.array([[1.0 / 3.0, 0.0, 0.5, 0.0],
                  [0.0, 1.0 / 3.0, 0.0, 0.5],
                  [0.5, 0.0, 1.0, 0.0],
                  [0.0, 0.5, 0.0, 1.0]])
    return (1.0 / 20.0) * V


def article_initial_states(n_targets: int) -> Array:
    if n_targets != 4:
        raise ValueError("Article initial states are defined for n_targets == 4.")
    return np.array([[12.0, 6.0, 0.001, 0.001],
                     [32.0, 32.0, -0.001, -0.005],
                     [20.0, 13.0, -0.1, 0.01],
                     [15.0, 35.0, 0.002, 0.002]])


def make_sensor_grid(area_xy: Tuple[float, float], grid_shape: Tuple[int, int]) -> Array:
    """Sensors on the (rows, cols) grid intersections of the area, row-major, (S, 2)."""
    width, height = area_xy
    rows, cols = grid_shape
    gx, gy = np.meshgrid(np.linspace(0.0, width, cols), np.linspace(0.0, height, rows))
    return np.column_stack([gx.ravel(), gy.ravel()])


def _reflect(pos: float, vel: float, upper: float, eps: float) -> Tuple[float, float]:
    if pos <= 0:
        return -pos + eps, -vel
    if pos >= upper:
        return 2 * upper - pos - eps, -vel
    return pos, vel


def simulate_cv_targets(n_steps: int, n_targets: int, area_xy: Tuple[float, float],
                        dyn_cfg: DynamicsConfig, rng: np.random.Generator,
                        use_article_init: bool = True, init_vel_std: float = 0.5,
                        enforce_boundaries: bool = True) -> Array:
    """CV trajectories ``(n_steps, n_targets, 4)`` with boundary reflection."""
    F = build_cv_transition(dyn_cfg.dt)
    L = np.linalg.cholesky(article_process_noise_cov() + 1e-12 * np.eye(4))
    width, height = area_xy
    X = np.zeros((n_steps, n_targets, 4), dtype=float)
    if use_article_init and n_targets == 4:
        X[0] = article_initial_states(n_targets)
    else:
        px = rng.uniform(0.25 * width, 0.75 * width, size=(n_targets, 1))
        py = rng.uniform(0.25 * height, 0.75 * height, size=(n_targets, 1))
        vx = rng.normal(0.0, init_vel_std, size=(n_targets, 1))
        vy = rng.normal(0.0, init_vel_std, size=(n_targets, 1))
        X[0] = np.hstack([px, py, vx, vy])
    eps = 1e-6
    for k in range(1, n_steps):
        noise = (L @ rng.normal(size=(4, n_targets))).T
        X[k] = X[k - 1] @ F.T + noise
        if enforce_boundaries:
            for c in range(n_targets):
                X[k, c, 0], X[k, c, 2] = _reflect(X[k, c, 0], X[k, c, 2], width, eps)
                X[k, c, 1], X[k, c, 3] = _reflect(X[k, c, 1], X[k, c, 3], height, eps)
    return X


def acoustic_measurement_model(positions: Array, sensors: Array, psi: float, d0: float) -> Array:
    """Noiseless amplitudes ``Z[t, s] = sum_c psi / (|p_{t,c} - s|^2 + d0)``, (T, S)."""
    diff = positions[:, :, None, :] - sensors[None, None, :, :]
    dist2 = np.sum(diff ** 2, axis=-1)
    return np.sum(psi / (dist2 + d0), axis=1)


def simulate_acoustic_dataset(cfg: ScenarioConfig, dyn_cfg: DynamicsConfig) -> Dict[str, Array]:
    """Dict with X (T,C,4), P (T,C,2), S (S,2), Z (T,S) and meta [W, H, psi, d0, dt]."""
    gen = np.random.default_rng(cfg.seed)
    sensors = make_sensor_grid(cfg.area_xy, cfg.sensor_grid_shape)
    X = simulate_cv_targets(cfg.n_steps, cfg.n_targets, cfg.area_xy, dyn_cfg, gen,
                            use_article_init=cfg.use_article_init)
    P = X[..., :2]
    Z = acoustic_measurement_model(P, sensors, psi=cfg.psi, d0=cfg.d0)
    meta = np.array([cfg.area_xy[0], cfg.area_xy[1], cfg.psi, cfg.d0, dyn_cfg.dt], dtype=float)
    return {"X": X, "P": P, "S": sensors, "Z": Z, "meta": meta}
