"""OMAT of BASELINE config 4 (CPU tests).

The oracle (oracle/omat_oracle.py) is pinned to the reference notebook's own compute_omat outputs
(tests/golden/omat_cases.npz, produced by executing the notebook function: make_golden_omat.py)
bit for bit; the product metric (particle_filters_amd/metrics.py: exhaustive assignment for C <= 7)
equals the oracle to 1e-14 relative on the same cases and on random ones, including ties.
"""

import os

import numpy as np
import pytest

from oracle import omat_oracle as OO
from particle_filters_amd import metrics as MT

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "omat_cases.npz"))
CASES = sorted({k.split("__")[0] + "__" + k.split("__")[1] for k in GOLD.files if k.endswith("__est")})


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("p", [1, 2])
def test_oracle_equals_notebook(case, p):
    key = case.split("__")[0]
    P, E = GOLD[f"{key}__truth"], GOLD[f"{case}__est"]
    want = GOLD[f"{case}__omat_p{p}"]
    got = np.array([OO.compute_omat(P[t], E[t], p=p) for t in range(P.shape[0])])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("p", [1, 2])
def test_metric_equals_oracle(case, p):
    key = case.split("__")[0]
    P, E = GOLD[f"{key}__truth"], GOLD[f"{case}__est"]
    want = GOLD[f"{case}__omat_p{p}"]
    got = np.array([MT.omat(P[t], E[t], p=p) for t in range(P.shape[0])])
    np.testing.assert_allclose(got, want, rtol=1e-14, atol=0)


def test_series_and_random_cases():
    rng = np.random.default_rng(3)
    for C in (1, 2, 4, 6, 9):
        for _ in range(20):
            P = rng.standard_normal((C, 2)) * 10
            E = rng.standard_normal((C, 2)) * 10
            E[rng.integers(0, C)] = E[0]  # ties in the assignment
            np.testing.assert_allclose(MT.omat(P, E), OO.compute_omat(P, E), rtol=1e-14)
    T, C = 7, 4
    X = rng.standard_normal((T, C, 4))
    M = X + 0.5 * rng.standard_normal((T, C, 4))
    s = MT.omat_series(X.reshape(T, 16), M.reshape(T, 16), C)
    want = [OO.compute_omat(X[t, :, :2], M[t, :, :2]) for t in range(T)]
    np.testing.assert_allclose(s, want, rtol=1e-14)
