"""HIP degeneracy diagnostics (csrc/pf_diag.hip) vs the reference's own outputs (-m gpu).

tests/golden/diag_cases.npz holds the reference notebook functions' results
(tests/golden/make_golden_diag.py), including compute_diagnostics on a reference
ParticleFilter state.  Tolerances: the reductions run in a different (fixed) order than
NumPy's pairwise sums, so entropy / ESS / spread agree to rtol 1e-12, Gini (a difference of
two O(1) terms) to atol 1e-12; the unique count is exact.
"""

import os

import numpy as np
import pytest

import particle_filters_amd as pfa
from particle_filters_amd import diagnostics as DG
from particle_filters_amd import models as M
from particle_filters_amd.batch import ParticleFilterBatch
from oracle import diag_oracle as DO

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(__file__)
GOLD = np.load(os.path.join(HERE, "golden", "diag_cases.npz"))
NAMES = [str(n) for n in GOLD["names"]]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from particle_filters_amd import _native
    assert _native.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def gcase(name):
    return {k.split("__", 1)[1]: GOLD[k] for k in GOLD.files if k.startswith(name + "__")}


def close(a, b, rtol=1e-12, atol=0.0):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


@pytest.mark.parametrize("name", NAMES)
def test_array_functions_match_reference(name):
    g = gcase(name)
    w, x = g["w"], g["x"]
    close(DG.compute_weight_entropy(w, True), g["entropy"], atol=1e-15)
    if "entropy_raw" in g:
        close(DG.compute_weight_entropy(w, False), g["entropy_raw"], atol=1e-15)
    close(DG.compute_gini_coefficient(w), g["gini"], rtol=0, atol=1e-12)
    assert DG.count_unique_particles(x, w) == int(g["n_unique"])


def sv_filter(precision="fp64", rng_mode="host", Np=2000, seed=7):
    return pfa.ParticleFilter(M.SVTransition(0.95), M.ExpHalfObservation(1.0), [[0.04]], [[0.1]], Np=Np,
                              resample_thresh=0.5, regularize_after_resample=False, rng=np.random.default_rng(seed),
                              precision=precision, rng_mode=rng_mode)


def test_compute_diagnostics_on_replayed_reference_state():
    """The engine replaying the reference's draws reaches the reference's states; the
    device diagnostics of those states match the notebook's compute_diagnostics."""
    sv = np.load(os.path.join(HERE, "golden", "sv_data.npz"))
    X, Y = sv["X0"], sv["Y0"]
    pf = sv_filter()
    pf.initialize([X[0]], [[0.5]])
    for k in range(1, 26):
        pf.predict()
        st = pf.update(np.array([Y[k]]))
        if k in (5, 12, 25):
            g = gcase(f"pfstate{k}")
            d = DG.compute_diagnostics(pf, resampled=False)
            for key in ("ess", "entropy", "max_weight", "posterior_spread"):
                close(d[key], g[key], rtol=1e-9)
            close(d["gini"], g["gini"], rtol=0, atol=1e-9)
            assert abs(d["n_unique"] - int(g["n_unique"])) <= 1
            # exact against the oracle on the engine's own state
            assert d["n_unique"] == DO.unique_particles(st.particles)
            o = DO.diagnostics(st.weights, st.particles, st.cov)
            close(d["entropy"], o["entropy"], atol=1e-15)
            close(d["ess"], o["ess"])
            close(d["posterior_spread"], o["posterior_spread"], rtol=1e-10)


@pytest.mark.parametrize("precision", ["fp32", "fp64"])
def test_batch_state_diagnostics_per_replicate(precision):
    """filter_diagnostics reads every replicate's state from HBM (log weights + normaliser,
    fp32 or fp64 storage) and agrees with the oracle on the downloaded state."""
    sv = np.load(os.path.join(HERE, "golden", "sv_data.npz"))
    Z = np.log(sv["Y0"][1:41] ** 2)[:, None]
    b = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=20000,
                            n_replicates=3, seed=5, precision=precision)
    b.initialize([sv["X0"][0]], [[0.5]])
    b.run(Z)
    recs = DG.filter_diagnostics(b)
    xs, ws = b.particles(), b.weights()
    for r in range(3):
        o = DO.diagnostics(ws[r], xs[r], np.atleast_2d(np.cov(xs[r].T, aweights=ws[r], bias=True)))
        close(recs[r].ess, o["ess"], rtol=1e-9)
        close(recs[r].entropy, o["entropy"], rtol=1e-9)
        close(recs[r].gini, o["gini"], rtol=0, atol=1e-9)
        close(recs[r].max_weight, o["max_weight"], rtol=1e-9)
        close(recs[r].posterior_spread, o["posterior_spread"], rtol=1e-6)
        assert recs[r].n_unique == o["n_unique"]


def test_large_state_unique_and_gini():
    """N = 1e6: exact unique count after resampling and the Gini sum of the sorted weights."""
    rng = np.random.default_rng(3)
    n = 1_000_000
    w = rng.gamma(0.5, size=n)
    w /= w.sum()
    base = rng.standard_normal((n, 2))
    x = base[rng.integers(0, n, n)]
    d = DG._host(w, x)
    assert d.n_unique == DO.unique_particles(x)
    close(d.gini, DO.gini_coefficient(w), rtol=0, atol=1e-11)
    close(d.entropy, DO.weight_entropy(w), rtol=1e-11)
    close(d.ess, 1.0 / np.sum(w ** 2), rtol=1e-11)


def test_flow_filter_state_diagnostics():
    """pf_ledh_diagnostics on an EDH / LEDH handle's state (fp64 weights + SoA particles)."""
    from tests.test_gpu_edh import make_filter

    pf, cfg, om, g = make_filter("acoustic", n_particles=3000, ratio=0.0)
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    sampler = lambda n, nx: cfg.rng.multivariate_normal(np.zeros(nx), om.Q, size=n)  # noqa: E731
    for t in range(3):
        st = pf.step(st, g["Z"][t], process_noise_sampler=sampler)
    d = DG.compute_diagnostics(pf, resampled=pf.last_resampled)
    o = DO.diagnostics(st.weights, st.particles, st.cov)
    for key in ("ess", "entropy", "max_weight"):
        close(d[key], o[key], rtol=1e-10)
    close(d["gini"], o["gini"], rtol=0, atol=1e-10)
    close(d["posterior_spread"], o["posterior_spread"], rtol=1e-9)
    assert d["n_unique"] == o["n_unique"] == 3000
