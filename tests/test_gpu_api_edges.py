"""Reference edge cases re-expressed on the engine (run on an MI355X: -m gpu).

* Np = 1 (/root/reference/tests/unit_tests/models/test_pf_resampling.py:338-360): a
  one-particle filter initialises and steps; the state has shape (1, 1), weights sum to 1.
  Also through the device T-loop (``run``), both precisions.
* predict / update / effective_sample_size before initialize raise AssertionError through
  the real class (test_pf_shapes_and_api.py:298-310), not only at the status-code level.
* Assigning ``state.particles`` keeps the (non-uniform) weights and the ESS, as assigning an
  attribute of the reference's PFState does (particle_filter.py:27-49).
"""

import numpy as np
import pytest

import particle_filters_amd as pfa
from particle_filters_amd import _native as NV, models as M

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def _simple(Np, precision="fp32", **kw):
    # test_pf_resampling.py:9-21: g = 0.9 x, h = x, Q = 0.1, R = 0.5
    return pfa.ParticleFilter(M.SVTransition(0.9), M.LinearObservation([[1.0]]), [[0.1]], [[0.5]], Np=Np,
                              resample_method="systematic", resample_thresh=0.5, precision=precision,
                              rng=np.random.default_rng(0), **kw)


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_single_particle_filter(precision):
    pf = _simple(1, precision)
    pf.initialize(np.array([0.0]), np.array([[1.0]]))
    st = pf.step(np.array([1.0]))
    assert st.particles.shape == (1, 1)
    assert np.isclose(np.sum(st.weights), 1.0)
    assert np.all(np.isfinite(st.mean)) and st.cov.shape == (1, 1)
    assert pf.effective_sample_size() == pytest.approx(1.0)
    res = pf.run(np.array([[0.5], [0.2], [-0.3]]))
    assert res.means.shape == (3, 1, 1) and np.all(np.isfinite(res.means))
    assert np.isclose(np.sum(pf.state.weights), 1.0)


def test_operations_before_initialize_raise():
    # test_pf_shapes_and_api.py:298-310 (simple_linear_system)
    pf = pfa.ParticleFilter(M.LinearTransition([[0.9, 0.2], [0.0, 0.7]]), M.LinearObservation([[1.0, 0.5]]),
                            np.diag([0.05, 0.02]), [[0.10]], Np=500)
    with pytest.raises(AssertionError):
        pf.predict()
    with pytest.raises(AssertionError):
        pf.update(np.array([1.0]))
    with pytest.raises(AssertionError):
        pf.effective_sample_size()
    with pytest.raises(AssertionError):
        pf.step(np.array([1.0]))


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_assigning_particles_keeps_weights(precision):
    pf2 = pfa.ParticleFilter(M.SVTransition(0.9), M.LinearObservation([[1.0]]), [[0.1]], [[0.5]], Np=4000,
                             resample_thresh=0.0, precision=precision, rng=np.random.default_rng(0))  # never resample
    pf2.initialize(np.array([0.0]), np.array([[1.0]]))
    st = pf2.step(np.array([1.3]))
    ess0 = pf2.effective_sample_size()
    assert ess0 < 3999  # non-uniform weights
    w_before = st.weights.copy()
    st2 = pf2.state
    fresh = pf2.state.particles + 0.5
    # a fresh handle on the state whose weights were never read: the setter must fetch them
    pf3 = pfa.ParticleFilter(M.SVTransition(0.9), M.LinearObservation([[1.0]]), [[0.1]], [[0.5]], Np=4000,
                             resample_thresh=0.0, precision=precision, rng=np.random.default_rng(0))
    pf3.initialize(np.array([0.0]), np.array([[1.0]]))
    s3 = pf3.step(np.array([1.3]))
    s3.particles = s3.particles + 0.5  # weights not read before the assignment
    np.testing.assert_allclose(pf3.state.weights, w_before, rtol=1e-6 if precision == "fp32" else 1e-12)
    assert pf3.effective_sample_size() == pytest.approx(ess0, rel=1e-6)
    st2.particles = fresh
    np.testing.assert_allclose(pf2.state.weights, w_before, rtol=1e-6 if precision == "fp32" else 1e-12)
    np.testing.assert_allclose(pf2.state.particles, fresh, rtol=1e-6)
