"""NumPy restatement of the reference's particle-degeneracy diagnostics — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import
this module; it is the checker for the HIP diagnostics kernels (``csrc/pf_diag.hip``),
never the thing measured or shipped.

Follows ``/root/reference/notebooks/particle_filter_NLNGSSM.ipynb`` cell 5 ("diag:LINE" =
line within that cell's source): ``compute_weight_entropy`` 5-19, ``compute_gini_coefficient``
22-36, ``count_unique_particles`` 39-58, ``compute_diagnostics`` 61-91 (ESS from
``pf.effective_sample_size()``, ``particle_filter.py:134-144``; posterior spread = trace of the
state covariance).  Pinned bit-for-bit by ``tests/golden/diag_cases.npz``, which
``tests/golden/make_golden_diag.py`` produced by executing the notebook cell itself.
"""

from __future__ import annotations

import numpy as np


def weight_entropy(weights, normalized=True) -> float:
    """diag:5-19: -sum (w + 1e-300) log(w + 1e-300), / log N when normalised and N > 1."""
    w = np.asarray(weights, float) + 1e-300
    ent = -np.sum(w * np.log(w))
    if normalized and len(w) > 1:
        ent /= np.log(len(w))
    return ent


def gini_coefficient(weights) -> float:
    """diag:22-36: (2 sum_i i w_(i)) / (N sum w) - (N + 1) / N over ascending weights, i = 1..N."""
    s = np.sort(np.asarray(weights, float))
    n = len(s)
    idx = np.arange(1, n + 1)
    return (2 * np.sum(idx * s)) / (n * np.sum(s)) - (n + 1) / n


def unique_particles(particles, tol=1e-10) -> int:
    """diag:39-58: distinct rows of round(x / tol) * tol."""
    x = np.asarray(particles, float)
    if len(x) <= 1:
        return len(x)
    xr = np.round(x / tol) * tol
    return len(np.unique(xr, axis=0))


def diagnostics(weights, particles, cov, tol=1e-10) -> dict:
    """diag:61-91 on a state (weights (N,), particles (N, nx), cov (nx, nx))."""
    w = np.asarray(weights, float)
    return {
        "ess": 1.0 / float(np.sum(w ** 2)),
        "entropy": weight_entropy(w, True),
        "gini": gini_coefficient(w),
        "max_weight": float(np.max(w)),
        "n_unique": unique_particles(np.asarray(particles, float).reshape(len(w), -1), tol),
        "posterior_spread": float(np.trace(np.atleast_2d(cov))),
    }
