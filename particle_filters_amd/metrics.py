"""Tracking accuracy of the multi-target configuration (BASELINE config 4).

``omat`` is the OMAT distance the reference evaluates its joint acoustic-tracking filter with
(/root/reference/notebooks/PF_PF_results_reproduction_multi_target_acoustic_tracking.ipynb,
``compute_omat`` at lines 175-206 of the .ipynb, per time step at 728-737): the optimal
one-to-one assignment of the C estimated target positions to the C true ones under Euclidean
distance, and ``(1 / C) * (sum of assigned distances ** p) ** (1 / p)``.  It runs on the host over
the posterior means the device loop returns (C = 4 targets: the 24 assignments are enumerated,
the exact optimum the notebook's Hungarian solver finds; larger C falls back to SciPy's solver).
"""

from __future__ import annotations

from itertools import permutations

import numpy as np

_PERMS = {}


def _perms(C):
    if C not in _PERMS:
        _PERMS[C] = np.array(list(permutations(range(C))), dtype=np.int64)
    return _PERMS[C]


def omat(X_true_t, X_est_t, p: float = 1) -> float:
    """OMAT between true positions [C][2] and estimated positions [C][2] (notebook compute_omat)."""
    X_true_t = np.asarray(X_true_t, float)
    X_est_t = np.asarray(X_est_t, float)
    C = X_true_t.shape[0]
    if X_est_t.shape != X_true_t.shape:
        raise ValueError("true and estimated positions must have the same shape")
    d = np.sqrt(np.sum((X_true_t[:, None, :] - X_est_t[None, :, :]) ** 2, axis=-1))  # [C][C]
    if C <= 7:
        P = _perms(C)
        cost = d[np.arange(C)[None, :], P]  # [C!][C]: row i assigned to column P[k, i]
        best = cost[np.argmin(cost.sum(axis=1))]
    else:
        from scipy.optimize import linear_sum_assignment

        r, c = linear_sum_assignment(d)
        best = d[r, c]
    s = 0.0
    for v in best:  # row order, as the notebook sums d[row_ind, col_ind]
        s += v ** p
    return (1.0 / C) * s ** (1.0 / p)


def omat_series(truth, means, n_targets: int, p: float = 1, dims_per_target: int = 4) -> np.ndarray:
    """Per-step OMAT of a joint multi-target run: truth / means [T][C * dims_per_target] with each
    target's block [x, y, vx, vy] (the joint 16-D state of config 4); positions are a block's
    first two components (notebook: ``state.mean[c*4:c*4+2]``)."""
    truth = np.asarray(truth, float).reshape(-1, n_targets, dims_per_target)[:, :, :2]
    means = np.asarray(means, float).reshape(-1, n_targets, dims_per_target)[:, :, :2]
    if truth.shape != means.shape:
        raise ValueError("truth and means must cover the same steps")
    return np.array([omat(truth[t], means[t], p) for t in range(truth.shape[0])])
