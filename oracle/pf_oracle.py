"""NumPy restatement of the reference SIR particle filter — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module.  It is the checker for the HIP engine, never the thing
measured or shipped.

Follows ``/root/reference/models/particle_filter.py`` (cited as ``pf.py:LINE``):

==============================  ==============================================
reference symbol                 restated here
==============================  ==============================================
``PFState``            27-49     :class:`OracleState`
``__init__``           79-107    :meth:`SIROracle.__init__` (LR = chol(R+1e-12 I))
``initialize``        110-132    :meth:`SIROracle.initialize`
``effective_sample_size`` 134-144 :meth:`SIROracle.effective_sample_size`
``_systematic_resample`` 146-171 :func:`systematic_indices` — the two-pointer
                                 loop is ``searchsorted(cdf, pos, 'right')``
``_multinomial_resample`` 173-186 :func:`multinomial_indices` — NumPy's
                                 ``Generator.choice(N, N, p=w)`` draws
                                 ``random(N)`` and searches ``cumsum(w)/cdf[-1]``
``_resample``         188-220    :meth:`SIROracle._resample`
``predict``           223-237    :meth:`SIROracle.predict`
``update``            239-269    :meth:`SIROracle.update`
``step``              271-287    :meth:`SIROracle.step`
==============================  ==============================================

Two evaluation modes of the user plugins:

* ``vectorized=False`` (faithful): ``g``/``h`` are called once per particle
  exactly like ``pf.py:237`` and ``pf.py:257``.  This is the reference CPU
  path's cost profile and is what bench.py times as ``cpu_baseline``.
* ``vectorized=True``: ``g(X, u)`` / ``h(X)`` take the whole ``(N, nx)``
  particle matrix.  Bit-identical for the elementwise models in
  :mod:`oracle.ssm_oracle`, ~100x faster; used for large-N parity references.

The RNG is duck-typed exactly as in the reference (``standard_normal(shape)``,
``random()``, ``choice(n, size, p)``), so :class:`RecordingRNG` can capture the
draw stream and :class:`ReplayRNG` can replay it — that is how the HIP engine's
replay mode is fed identical noise.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, List, Optional, Tuple

import numpy as np

Array = np.ndarray


@dataclass
class OracleState:
    """Posterior container (pf.py:27-49)."""

    particles: Array
    weights: Array
    mean: Array
    cov: Array
    t: int


# ---------------------------------------------------------------------------
# Resampling index kernels (pure functions of weights + uniforms)
# ---------------------------------------------------------------------------
def systematic_indices(weights: Array, U: float) -> Array:
    """Ancestor indices of systematic resampling (pf.py:146-171).

    ``positions = (U + arange(N)) / N``; ``cdf = cumsum(w)`` with
    ``cdf[-1] = 1.0``; the reference while-loop assigns
    ``idx[i] = min{j : positions[i] < cdf[j]}``, i.e.
    ``searchsorted(cdf, positions, side='right')``.  Clamped to ``N-1`` (the
    loop would run off the end only if ``(U+N-1)/N`` rounded to 1.0).
    """
    w = np.asarray(weights, dtype=float)
    N = len(w)
    positions = (U + np.arange(N)) / N
    cdf = np.cumsum(w)
    cdf[-1] = 1.0
    idx = np.searchsorted(cdf, positions, side="right")
    return np.minimum(idx, N - 1).astype(int)


def multinomial_indices(weights: Array, uniforms: Array) -> Array:
    """Ancestor indices of multinomial resampling (pf.py:173-186).

    ``Generator.choice(N, size=N, p=w)`` with replacement is
    ``searchsorted(cumsum(w)/cumsum(w)[-1], random(N), side='right')``.
    """
    w = np.asarray(weights, dtype=float)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.searchsorted(cdf, np.asarray(uniforms, float), side="right").astype(np.int64)


def effective_sample_size(weights: Array) -> float:
    """``1 / sum(w^2)`` (pf.py:144, pf.py:203)."""
    w = np.asarray(weights, dtype=float)
    return 1.0 / np.sum(w ** 2)


# ---------------------------------------------------------------------------
# RNG recording / replay (duck-typed like numpy.random.Generator)
# ---------------------------------------------------------------------------
class RecordingRNG:
    """Wraps a ``numpy.random.Generator`` and records every draw in order.

    The SIR path uses only ``standard_normal(shape)`` (pf.py:128, 217, 236),
    ``random()`` (pf.py:160) and ``choice(N, size=N, p=w)`` (pf.py:186).
    ``choice`` is restated as ``random(N)`` + search so the uniforms can be
    recorded; tests/test_oracle_golden.py pins that this consumes the stream
    exactly like ``Generator.choice``.
    """

    def __init__(self, gen: np.random.Generator):
        self.gen = gen
        self.log: List[Tuple[str, Any]] = []

    def standard_normal(self, size=None):
        v = self.gen.standard_normal(size)
        self.log.append(("normal", np.array(v, dtype=float)))
        return v

    def random(self, size=None):
        v = self.gen.random(size)
        self.log.append(("uniform", np.array(v, dtype=float) if size is not None else float(v)))
        return v

    def choice(self, a, size=None, replace=True, p=None):
        if p is None or not replace:
            raise NotImplementedError("only choice(n, size, p=w) with replacement is on the SIR path")
        u = self.random(size)
        return multinomial_indices(p, u)


class ReplayRNG:
    """Replays a :class:`RecordingRNG` log; raises if the call pattern diverges."""

    def __init__(self, log: List[Tuple[str, Any]]):
        self.log = list(log)
        self.pos = 0

    def _next(self, kind: str, size):
        if self.pos >= len(self.log):
            raise RuntimeError("replay log exhausted")
        k, v = self.log[self.pos]
        if k != kind:
            raise RuntimeError(f"replay mismatch at draw {self.pos}: wanted {kind}, log has {k}")
        if size is not None and np.shape(v) != tuple(np.atleast_1d(size)):
            raise RuntimeError(f"replay shape mismatch at draw {self.pos}: {np.shape(v)} vs {size}")
        self.pos += 1
        return np.array(v) if size is not None else float(v)

    def standard_normal(self, size=None):
        return self._next("normal", size)

    def random(self, size=None):
        return self._next("uniform", size)

    def choice(self, a, size=None, replace=True, p=None):
        return multinomial_indices(p, self.random(size))


# ---------------------------------------------------------------------------
# The filter
# ---------------------------------------------------------------------------
class SIROracle:
    """Restatement of ``ParticleFilter`` (pf.py:53-287).

    Extra instrumentation (not in the reference, read-only): ``last_neff`` is
    the pre-resample Neff of the last update, ``last_resampled`` whether
    ``_resample`` fired (pf.py:203-204) and ``last_lse`` the update's log
    normaliser ``m + log sum exp(logw - m)`` (pf.py:261-262).
    """

    def __init__(
        self,
        g: Callable,
        h: Callable,
        Q: Array,
        R: Array,
        *,
        Np: int = 1000,
        resample_thresh: float = 0.5,
        resample_method: str = "systematic",
        regularize_after_resample: bool = False,
        rng=None,
        vectorized: bool = False,
    ) -> None:
        self.g = g
        self.h = h
        self.Q = np.asarray(Q, float)
        self.R = np.asarray(R, float)
        self.Np = int(Np)
        self.resample_thresh = float(resample_thresh)
        self.resample_method = resample_method
        self.regularize_after_resample = regularize_after_resample
        self.rng = np.random.default_rng() if rng is None else rng
        self.vectorized = vectorized
        self.nx = self.Q.shape[0]
        self.nz = self.R.shape[0]
        self.state: Optional[OracleState] = None
        self.LR = np.linalg.cholesky(self.R + 1e-12 * np.eye(self.nz))  # pf.py:107
        self.last_neff = float("nan")
        self.last_resampled = False
        self.last_lse = float("nan")

    # pf.py:110-132
    def initialize(self, mean: Array, cov: Array) -> OracleState:
        mean = np.asarray(mean, float)
        cov = np.asarray(cov, float)
        Lc = np.linalg.cholesky(cov + 1e-10 * np.eye(len(mean)))
        particles = self.rng.standard_normal((self.Np, len(mean))) @ Lc.T + mean
        weights = np.ones(self.Np) / self.Np
        self.state = OracleState(particles, weights, mean, np.atleast_2d(cov), 0)
        return self.state

    # pf.py:134-144
    def effective_sample_size(self) -> float:
        assert self.state is not None, "Filter not initialized."
        return effective_sample_size(self.state.weights)

    # pf.py:146-171
    def _systematic_resample(self, weights: Array) -> Array:
        return systematic_indices(weights, self.rng.random())

    # pf.py:173-186
    def _multinomial_resample(self, weights: Array) -> Array:
        return self.rng.choice(len(weights), size=len(weights), p=weights)

    # pf.py:188-220
    def _resample(self, particles: Array, weights: Array) -> Tuple[Array, Array]:
        neff = 1.0 / np.sum(weights ** 2)
        self.last_neff = float(neff)
        self.last_resampled = bool(neff < self.resample_thresh * self.Np)
        if self.last_resampled:
            if self.resample_method == "systematic":
                idx = self._systematic_resample(weights)
            else:  # any other string is multinomial (pf.py:207-208)
                idx = self._multinomial_resample(weights)
            particles = particles[idx]
            weights = np.ones_like(weights) / len(weights)
            if self.regularize_after_resample:
                try:
                    Lq = np.linalg.cholesky(self.Q)
                except np.linalg.LinAlgError:
                    Lq = np.linalg.cholesky(self.Q + 1e-12 * np.eye(self.nx))
                particles += self.rng.standard_normal(particles.shape) @ (0.001 * Lq.T)
        return particles, weights

    # pf.py:223-237
    def predict(self, u: Optional[Array] = None) -> None:
        assert self.state is not None, "Filter not initialized."
        try:
            Lq = np.linalg.cholesky(self.Q)
        except np.linalg.LinAlgError:
            Lq = np.linalg.cholesky(self.Q + 1e-10 * np.eye(self.nx))
        noise = self.rng.standard_normal((self.Np, self.nx)) @ Lq.T
        if self.vectorized:
            moved = np.asarray(self.g(self.state.particles, u), float)
        else:
            moved = np.array([self.g(x, u) for x in self.state.particles])
        self.state.particles = moved + noise

    # pf.py:239-269
    def update(self, z: Array) -> OracleState:
        assert self.state is not None, "Filter not initialized."
        z = np.asarray(z, float)
        particles = self.state.particles
        weights = self.state.weights
        if self.vectorized:
            z_pred = np.asarray(self.h(particles), float).reshape(self.Np, self.nz)
        else:
            z_pred = np.array([self.h(x) for x in particles])
        diffs = (z - z_pred).T
        y = np.linalg.solve(self.LR, diffs)
        quad = np.sum(y * y, axis=0)
        logw = np.log(weights + 1e-300) - 0.5 * quad
        m = np.max(logw)
        lse = m + np.log(np.sum(np.exp(logw - m)))
        self.last_lse = float(lse)  # the log-normaliser (marginal-likelihood increment), read-only
        w = np.exp(logw - lse)
        particles, w = self._resample(particles, w)
        mean = np.average(particles, axis=0, weights=w)
        cov = np.atleast_2d(np.cov(particles.T, aweights=w, bias=True))
        self.state = OracleState(particles, w, mean, cov, self.state.t + 1)
        return self.state

    # pf.py:271-287
    def step(self, z: Array, u: Optional[Array] = None) -> OracleState:
        self.predict(u)
        return self.update(z)


def run_filter(pf: SIROracle, Z: Array, *, first_update_only: bool = False,
               controls: Optional[Array] = None) -> dict:
    """Drive a filter over observations ``Z`` (T, nz) the way the reference's
    drivers do (tests/integration_tests/test_pf_vs_simulator_sv.py:78-81 with
    ``step``; notebooks/PF_VS_experiments.ipynb cell 7 when
    ``first_update_only``: update(Z[0]) then predict+update).

    Returns per-step posterior means, post-update ESS (what
    ``effective_sample_size()`` reports), pre-resample Neff and resample flags.
    """
    Z = np.asarray(Z, float)
    T = Z.shape[0]
    means = np.zeros((T, pf.nx))
    covs = np.zeros((T, pf.nx, pf.nx))
    ess = np.zeros(T)
    neff = np.zeros(T)
    lse = np.zeros(T)
    flags = np.zeros(T, dtype=bool)
    for t in range(T):
        z = np.atleast_1d(Z[t])
        if first_update_only and t == 0:
            st = pf.update(z)
        else:
            st = pf.step(z, None if controls is None else controls[t])
        means[t] = st.mean
        covs[t] = st.cov
        ess[t] = pf.effective_sample_size()
        neff[t] = pf.last_neff
        lse[t] = pf.last_lse
        flags[t] = pf.last_resampled
    return dict(means=means, covs=covs, ess=ess, neff=neff, lse=lse, flags=flags,
                final_particles=pf.state.particles.copy(), final_weights=pf.state.weights.copy(),
                t_final=pf.state.t)


def build_and_run(ssm, Z, *, Np, seed, mean0, cov0, method="systematic", reg=False, thresh=0.5,
                  first_update_only=False, controls=None, vectorized=True, rng=None):
    """Construct a :class:`SIROracle` for ``ssm`` (oracle.ssm_oracle.SSM), initialise it and run."""
    pf = SIROracle(ssm.g_vec if vectorized else ssm.g, ssm.h_vec if vectorized else ssm.h,
                   ssm.Q, ssm.R, Np=Np, resample_thresh=thresh, resample_method=method,
                   regularize_after_resample=reg,
                   rng=np.random.default_rng(seed) if rng is None else rng, vectorized=vectorized)
    pf.initialize(np.asarray(mean0, float), np.asarray(cov0, float))
    init = pf.state.particles.copy()
    out = run_filter(pf, Z, first_update_only=first_update_only, controls=controls)
    out["init_particles"] = init
    return out
