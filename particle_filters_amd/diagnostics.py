"""Particle-degeneracy diagnostics on the GPU.

Mirrors the diagnostic functions of the reference's degeneracy study
(``/root/reference/notebooks/particle_filter_NLNGSSM.ipynb`` cell 5, cited ``diag:LINE``):
``compute_weight_entropy`` (5-19), ``compute_gini_coefficient`` (22-36),
``count_unique_particles`` (39-58) and ``compute_diagnostics(pf, resampled)`` (61-91), with
the same names, arguments and return values.

The array functions upload their arguments and reduce them on the device (``pf_diagnostics_host``);
``compute_diagnostics`` reads an engine filter's state where it lives in HBM
(``pf_state_diagnostics`` / ``pf_ledh_diagnostics``): the weights are never normalised on or
copied to the host.  ``filter_diagnostics`` returns the record of every replicate of a
:class:`~particle_filters_amd.batch.ParticleFilterBatch`.  There is no CPU fallback.
"""

from __future__ import annotations

import numpy as np

from . import _native as N

__all__ = ["compute_weight_entropy", "compute_gini_coefficient", "count_unique_particles", "compute_diagnostics",
           "filter_diagnostics"]


def _host(weights, particles=None, tol=1e-10, cov=None, device=0) -> N.Diagnostics:
    w = np.ascontiguousarray(np.asarray(weights, float).reshape(-1))
    x = None
    nx = 0
    if particles is not None:
        x = np.asarray(particles, float)
        x = np.ascontiguousarray(x.reshape(len(w), -1))
        nx = x.shape[1]
    c = None
    if cov is not None:
        c = np.ascontiguousarray(np.atleast_2d(np.asarray(cov, float)))
        nx = nx or c.shape[0]
    out = N.Diagnostics()
    N.check(N.load().pf_diagnostics_host(int(device), N.dptr(w), N.dptr(x), len(w), nx, float(tol), N.dptr(c),
                                         N.C.byref(out)), "pf_diagnostics_host")
    return out


def compute_weight_entropy(weights: np.ndarray, normalized: bool = True, *, device: int = 0) -> float:
    """diag:5-19: Shannon entropy of the weights (+1e-300), normalised by log(N) to [0, 1]."""
    d = _host(weights, device=device)
    return float(d.entropy if normalized else d.entropy_raw)


def compute_gini_coefficient(weights: np.ndarray, *, device: int = 0) -> float:
    """diag:22-36: Gini coefficient of the weights (0 equal, 1 one particle holds all)."""
    return float(_host(weights, device=device).gini)


def count_unique_particles(particles: np.ndarray, weights: np.ndarray, tol: float = 1e-10, *, device: int = 0) -> int:
    """diag:39-58: number of distinct rows of round(particles / tol) * tol."""
    x = np.asarray(particles, float)
    if len(x) <= 1:  # diag:52-53
        return len(x)
    return int(_host(weights, x, tol, device=device).n_unique)


def _as_dict(d: N.Diagnostics, resampled: bool) -> dict:
    return {
        "ess": float(d.ess),
        "entropy": float(d.entropy),
        "gini": float(d.gini),
        "max_weight": float(d.max_weight),
        "n_unique": int(d.n_unique),
        "resampled": resampled,
        "posterior_spread": float(d.posterior_spread),
    }


def filter_diagnostics(pf, tol: float = 1e-10) -> list:
    """diag:61-91 for every replicate of an engine filter, from its device state."""
    from .batch import ParticleFilterBatch
    from .ledh import LEDHFlowPF
    from .particle_filter import ParticleFilter

    lib = N.load()
    if isinstance(pf, (ParticleFilter, ParticleFilterBatch)):  # SIR engine
        handle = pf._handle if isinstance(pf, ParticleFilter) else pf.handle
        R = 1 if isinstance(pf, ParticleFilter) else pf.n_replicates
        out = (N.Diagnostics * R)()
        N.check(lib.pf_state_diagnostics(handle, float(tol), out), "pf_state_diagnostics")
        return [out[r] for r in range(R)]
    if isinstance(pf, LEDHFlowPF):  # LEDHFlowPF / EDHFlowPF
        out = N.Diagnostics()
        N.check(lib.pf_ledh_diagnostics(pf._h, float(tol), N.C.byref(out)), "pf_ledh_diagnostics")
        return [out]
    raise NotImplementedError("compute_diagnostics needs a particle_filters_amd filter")


def compute_diagnostics(pf, resampled: bool, tol: float = 1e-10) -> dict:
    """diag:61-91: ESS, normalised entropy, Gini, max weight, unique particles, the resample
    flag passed in and trace(state covariance), for the filter's current state.

    For an engine filter the ESS is ``pf.effective_sample_size()`` of the state weights
    (particle_filter.py:134-144) and the spread is the weighted covariance trace of the
    particles (the state covariance of particle_filter.py:264-266), both from HBM."""
    return _as_dict(filter_diagnostics(pf, tol)[0], resampled)
