"""OMAT (optimal mean assignment) distance of BASELINE config 4 — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` and ``bench.py``'s checks may use this module, as the checker.

Restates ``compute_omat`` of the reference notebook
/root/reference/notebooks/PF_PF_results_reproduction_multi_target_acoustic_tracking.ipynb
(lines 175-206 of the .ipynb; evaluated per time step on the joint filter's posterior mean at
728-737 and averaged over T at 785, "Average OMAT: 10.6974"): the C x C matrix of Euclidean
distances between true and estimated target positions, an optimal assignment (the Hungarian
method: scipy.optimize.linear_sum_assignment, as the notebook uses it), and
``(1 / C) * (sum of assigned distances ** p) ** (1 / p)``.  Pinned to the notebook function's
own outputs by tests/test_omat.py (tests/golden/omat_cases.npz, make_golden_omat.py).
"""

from __future__ import annotations

import numpy as np
from scipy.optimize import linear_sum_assignment


def compute_omat(X_true_t, X_est_t, p=1):
    X_true_t = np.asarray(X_true_t, float)
    X_est_t = np.asarray(X_est_t, float)
    C = X_true_t.shape[0]
    d = np.zeros((C, C))
    for i in range(C):
        for j in range(C):
            d[i, j] = np.linalg.norm(X_true_t[i] - X_est_t[j])
    r, c = linear_sum_assignment(d)
    return (1.0 / C) * np.sum(d[r, c] ** p) ** (1.0 / p)
