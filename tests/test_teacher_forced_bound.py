"""CPU check of the teacher-forced parity's particle-rounding term (tests/teacher_forced.py
``ll_rounding_bound``): the oracle-gradient bound covers the likelihood change of random
perturbations within the particle tolerance, for the SV, L96 and joint acoustic models."""

import numpy as np
import pytest

from oracle import ssm_oracle
from tests.teacher_forced import ll_rounding_bound


def _mat():
    g = np.linspace(0.0, 40.0, 5)
    S = np.array([[x, y] for x in g for y in g])
    return ssm_oracle.mat_joint(S)


@pytest.mark.parametrize("make,scale", [(lambda: ssm_oracle.sv_logsq(0.95, 0.2, 1.0), 1.0),
                                        (lambda: ssm_oracle.lorenz96(40), 8.0), (_mat, 40.0)])
def test_bound_covers_perturbations(make, scale):
    ssm = make()
    rs = np.random.default_rng(1)
    N = 2000
    X = rs.normal(0.0, 1.0, (N, ssm.nx)) * (scale / 2) + (scale / 2)
    z = np.asarray(ssm.h_vec(X[:1]), float)[0] + rs.normal(0, 1.0, ssm.nz)
    LR = np.linalg.cholesky(ssm.R + 1e-12 * np.eye(ssm.nz))

    def ll(Y):
        r = np.linalg.solve(LR, (z - np.asarray(ssm.h_vec(Y), float).reshape(N, -1)).T)
        return 0.5 * np.sum(r * r, axis=0)

    r0 = np.linalg.solve(LR, (z - np.asarray(ssm.h_vec(X), float).reshape(N, -1)).T)
    gz = np.linalg.solve(LR.T, r0)
    dx = 2e-6 * scale
    b = ll_rounding_bound(ssm.h_vec, X, gz, dx, ssm.hjt_vec)
    worst = np.zeros(N)
    for _ in range(8):
        d = rs.choice([-dx, dx], size=X.shape)  # corners of the tolerance box
        worst = np.maximum(worst, np.abs(ll(X + d) - ll(X)))
    assert np.all(worst <= b + 1e-12 * (1 + np.abs(ll(X)))), float(np.max(worst / np.maximum(b, 1e-300)))
    assert np.median(worst / np.maximum(b, 1e-300)) > 0.05  # not vacuous


@pytest.mark.parametrize("make,scale", [(lambda: ssm_oracle.sv_logsq(0.95, 0.2, 1.0), 1.0),
                                        (lambda: ssm_oracle.lorenz96(40), 8.0), (_mat, 40.0)])
def test_analytic_jacobian_matches_differences(make, scale):
    """The models' analytic J_h^T g (ssm.hjt_vec, used by the GPU tests) equals the central
    differences of g . h(x)."""
    ssm = make()
    assert ssm.hjt_vec is not None
    rs = np.random.default_rng(2)
    X = rs.normal(0.0, 1.0, (500, ssm.nx)) * (scale / 2) + (scale / 2)
    gz = rs.normal(0.0, 1.0, (ssm.nz, 500))
    a = ll_rounding_bound(ssm.h_vec, X, gz, 1e-6, ssm.hjt_vec)
    b = ll_rounding_bound(ssm.h_vec, X, gz, 1e-6)
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-12)
