"""The exact SV likelihood and the all-dead guard (-m gpu).

The wiring is the reference test's ``sv_log_likelihood_fn``
(/root/reference/tests/integration_tests/test_dpf_vs_sv_simulator.py:60-97): it lives
in a TensorFlow test that is not importable here, so its parity is **unpinned** against
reference outputs; it is pinned against the formula instead — the C oracle's exact
mode (oracle/sir_philox.c, obs 3) is checked against a direct NumPy statement of the
formula in tests/test_sir_philox.py, and the engine against that oracle here, on the
engine's own Philox draws.  Tolerances:

* fp64 engine (launch-per-step k_step) vs the fp64 oracle: identical decisions, means
  within 1e-9 abs, Neff rel 1e-9;
* fp32 resident kernel at BASELINE config 2's size (N = 1e6, T = 999) vs the oracle:
  teacher-forced as in tests/oracle_compare.py (1e-5 / rel 1e-4 before the first resample,
  well inside the filter's own Monte-Carlo error after it), free-run |dRMSE| <= 1e-4 (the
  survey measured 4.3e-6 for this wiring);
* fp32 vs fp64 engine, same Philox noise, N = 1e6: |dRMSE| <= 1e-4.

All-dead steps (every weight zero or NaN — e.g. a NaN observation):
the reference would carry NaN weights on silently; the engine reports PF_E_NAN
(FloatingPointError) on every path and, for the resident kernel, poisons the handle.
"""

import numpy as np
import pytest

import particle_filters_amd as pfa
from particle_filters_amd import _native as NV, models as M
from particle_filters_amd.batch import ParticleFilterBatch
from oracle import sir_philox as SP
from tests.oracle_compare import check_forced, forced_compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def _model():
    return SP.scalar_model(0.95, 0.04, SP.OBS_SV_EXACT, hc=1.0)


def _batch(N, precision, seed=42, reg=False):
    b = ParticleFilterBatch(M.SVTransition(0.95), M.SVExactObservation(1.0), [[0.04]], None, Np=N, seed=seed,
                            precision=precision, regularize_after_resample=reg)
    return b


def test_exact_fp64_step_path_matches_oracle(golden_sv):
    X, Y = golden_sv["X0"], golden_sv["Y0"]
    Y = Y[1:301]
    N = 100_003
    b = _batch(N, "fp64", seed=11, reg=True)
    b.initialize([X[0]], [[0.5]])
    r = b.run(Y[:, None])
    assert not NV.load().pf_last_run_resident(b.handle)
    b.close()
    o = SP.run_scalar(_model(), Y, N=N, seed=11, mean0=X[0], var0=0.5, bm24=False, regularize=True)
    assert o["flags"].sum() >= 5
    assert np.array_equal(r.flags[:, 0], o["flags"])
    np.testing.assert_allclose(r.means[:, 0, 0], o["means"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(r.neff[:, 0], o["neff"], rtol=1e-9)


def test_exact_fp32_resident_vs_oracle_and_fp64(golden_sv):
    X, Y = golden_sv["X0"], golden_sv["Y0"]
    Y = Y[1:]
    N = 1_000_000
    runs = {}
    for prec in ("fp32", "fp64"):
        b = _batch(N, prec)
        b.initialize([X[0]], [[0.5]])
        runs[prec] = b.run(Y[:, None])
        runs[prec + "_resident"] = bool(NV.load().pf_last_run_resident(b.handle))
        b.close()
    assert runs["fp32_resident"]
    r = runs["fp32"]
    c = forced_compare(r.means[:, 0, 0], r.neff[:, 0], r.flags[:, 0], _model(), Y, N=N, seed=42, mean0=X[0],
                       var0=0.5)
    free = SP.run_scalar(_model(), Y, N=N, seed=42, mean0=X[0], var0=0.5, bm24=True)
    truth = X[1:]
    r_e = float(np.sqrt(np.mean((r.means[:, 0, 0] - truth) ** 2)))
    r_o = float(np.sqrt(np.mean((free["means"] - truth) ** 2)))
    r_64 = float(np.sqrt(np.mean((runs["fp64"].means[:, 0, 0] - truth) ** 2)))
    print(f"exact SV N=1e6: {c['summary']}; RMSE fp32 {r_e:.9f} oracle {r_o:.9f} fp64 {r_64:.9f}")
    check_forced(c)
    assert abs(r_e - r_o) <= 1e-4
    assert abs(r_e - r_64) <= 1e-4
    assert r_o < 0.6  # the survey's fp64 RMSE for this wiring: 0.4456 (different noise)


@pytest.mark.parametrize("path", ["resident", "step"])
def test_all_dead_step_raises(path, golden_sv, monkeypatch):
    if path == "step":
        monkeypatch.setenv("PF_RESIDENT", "0")
    Y = golden_sv["Y0"][1:40].copy()
    Y[17] = np.nan
    b = _batch(20_000, "fp32")
    b.initialize([0.0], [[0.5]])
    with pytest.raises(FloatingPointError):
        b.run(Y[:, None])
    # the state has moved past the dead step on either path: the handle is poisoned until re-initialised
    with pytest.raises(AssertionError, match="Filter not initialized"):
        b.run(Y[:5, None])
    b.initialize([0.0], [[0.5]])
    r = b.run(Y[:10, None])
    assert np.all(np.isfinite(r.means))
    b.close()


def test_all_dead_update_api_raises(golden_sv):
    pf = pfa.ParticleFilter(M.SVTransition(0.95), M.SVExactObservation(1.0), [[0.04]], None, Np=5000,
                            rng=np.random.default_rng(3))
    pf.initialize([0.0], [[0.5]])
    pf.step(np.array([0.4]))
    with pytest.raises(FloatingPointError):
        pf.step(np.array([np.nan]))
    with pytest.raises(AssertionError, match="Filter not initialized"):
        pf.step(np.array([0.4]))


@pytest.mark.parametrize("path", ["resident", "step"])
def test_one_dead_replicate_poisons_the_batch(path, golden_sv, monkeypatch):
    """R = 2, only replicate 1 sees the NaN observation: the batch reports FloatingPointError and
    refuses to continue (the live replicate's step has advanced with the dead one's)."""
    if path == "step":
        monkeypatch.setenv("PF_RESIDENT", "0")
    Y = golden_sv["Y0"][1:30].copy()
    Zr = np.stack([Y, Y], axis=1)[:, :, None]
    Zr[11, 1, 0] = np.nan
    b = ParticleFilterBatch(M.SVTransition(0.95), M.SVExactObservation(1.0), [[0.04]], None, Np=20_000, n_replicates=2,
                            seed=4)
    b.initialize([0.0], [[0.5]])
    with pytest.raises(FloatingPointError):
        b.run(Zr)
    with pytest.raises(AssertionError, match="Filter not initialized"):
        b.run(Zr[:3])
    b.initialize([0.0], [[0.5]])
    assert np.all(np.isfinite(b.run(Zr[:10]).means))
    b.close()
