"""The Philox-driven SIR oracle (oracle/sir_philox.*) — CPU tests.

* Philox4x32-10 against Random123's published known-answer vectors, in both the
  NumPy restatement (oracle/philox.py) and the C one (oracle/sir_philox.c).
* The C scalar-state SIR run against :class:`oracle.sir_philox.PhiloxSIROracle`
  (= oracle/pf_oracle.SIROracle, pinned bit for bit to the reference's outputs by
  tests/test_oracle_golden.py, fed the engine's draws): fp64, rel 1e-11, identical
  decisions, for systematic / multinomial / regularised and teacher-forced runs.
* The exact SV likelihood against a direct NumPy
  statement of the formula of the reference's test wiring
  (tests/integration_tests/test_dpf_vs_sv_simulator.py:60-97).
"""

import numpy as np
import pytest

from oracle import philox, ssm_oracle, sir_philox as SP
from oracle.pf_oracle import run_filter

# Random123 kat_vectors, philox4x32 with 10 rounds: (counter, key, expected)
KAT = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
       ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
       ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
        (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_known_answers(ctr, key, want):
    got_np = [int(v[0]) for v in philox.philox4x32_10(*[np.array([c]) for c in ctr], *key)]
    assert got_np == list(want)
    assert [int(v) for v in SP.philox4x32_10(ctr, key)] == list(want)


@pytest.mark.parametrize("bm24", [True, False])
def test_c_normals_match_numpy(bm24):
    a = SP.normals(42, 4099, 3, 7, philox.STREAM_PROCESS, bm24)
    b = philox.normals(42, 4099, 3, 7, philox.STREAM_PROCESS, dtype=np.float32 if bm24 else np.float64)
    np.testing.assert_allclose(a, b, rtol=1e-14, atol=1e-15)
    assert float(SP.load().pfo_uniform53(42, 5, 3, 9)) == float(philox.uniform53(42, np.array([5]), 3, 9)[0])


def _numpy_run(Z, X0, method, reg, N, forced=None, fo=False):
    ssm = ssm_oracle.sv_logsq(0.95, 0.2, 1.0)
    o = SP.PhiloxSIROracle(ssm.g_vec, ssm.h_vec, ssm.Q, ssm.R, seed=42, Np=N, vectorized=True,
                           resample_method=method, regularize_after_resample=reg)
    o.initialize(np.array([X0]), np.array([[0.5]]))
    if forced is not None:
        o.forced = list(forced)
    r = run_filter(o, Z[:, None], first_update_only=fo)
    return r


@pytest.mark.parametrize("method,reg,fo", [("systematic", False, False), ("systematic", True, False),
                                           ("multinomial", True, False), ("systematic", True, True)])
def test_c_oracle_equals_numpy_oracle(method, reg, fo, golden_sv):
    X, Y = golden_sv["X0"], golden_sv["Y0"]
    Z = np.log(Y[1:160] ** 2)
    N = 3001
    r = _numpy_run(Z, X[0], method, reg, N, fo=fo)
    c = SP.run_scalar(SP.sv_logsq_model(0.95, 0.2, 1.0), Z, N=N, seed=42, mean0=X[0], var0=0.5, method=method,
                      regularize=reg, first_update_only=fo)
    assert r["flags"].sum() >= 5
    assert np.array_equal(r["flags"], c["flags"])
    np.testing.assert_allclose(c["means"], r["means"][:, 0], rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose(c["vars"], r["covs"][:, 0, 0], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(c["neff"], r["neff"], rtol=1e-11)
    np.testing.assert_allclose(c["x"], r["final_particles"][:, 0], rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose(c["w"], r["final_weights"], rtol=1e-10, atol=1e-18)


def test_forced_decisions(golden_sv):
    """Teacher forcing: the C oracle takes exactly the decisions it is given and reports
    its own Neff; the NumPy oracle forced the same way agrees."""
    X, Y = golden_sv["X0"], golden_sv["Y0"]
    Z = np.log(Y[1:80] ** 2)
    N = 2003
    forced = np.zeros(len(Z), np.int32)
    forced[[3, 10, 11, 40, 41, 42]] = 1
    c = SP.run_scalar(SP.sv_logsq_model(0.95, 0.2, 1.0), Z, N=N, seed=42, mean0=X[0], var0=0.5, regularize=True,
                      forced=forced)
    assert np.array_equal(c["flags"], forced.astype(bool))
    r = _numpy_run(Z, X[0], "systematic", True, N, forced=forced)
    assert np.array_equal(r["flags"], forced.astype(bool))
    np.testing.assert_allclose(c["means"], r["means"][:, 0], rtol=1e-11, atol=1e-12)


def test_exact_sv_likelihood_formula(golden_sv):
    """SV_EXACT: log p(y|x) = -x/2 - y^2 e^{-x} / (2 beta^2) + const
    (test_dpf_vs_sv_simulator.py:60-97: -0.5 log 2pi - log(beta e^{x/2}) - 0.5 (y / (beta e^{x/2}))^2).
    One step from a known state, against NumPy."""
    X, Y = golden_sv["X0"], golden_sv["Y0"]
    N, beta = 5000, 1.3
    m = SP.scalar_model(0.95, 0.04, SP.OBS_SV_EXACT, hc=beta)
    x0 = np.linspace(-2.0, 2.0, N)
    c = SP.run_scalar(m, Y[1:2], N=N, seed=9, x0=x0, w0=np.full(N, 1.0 / N), thresh=0.0)
    x1 = 0.95 * x0 + 0.2 * philox.normals(9, N, 0, 2, philox.STREAM_PROCESS, dtype=np.float32)
    sig = beta * np.exp(0.5 * x1)
    ll = -0.5 * np.log(2 * np.pi) - np.log(sig) - 0.5 * (Y[1] / sig) ** 2  # the reference test's formula
    lw = np.log(1.0 / N + 1e-300) + ll
    w = np.exp(lw - lw.max())
    w /= w.sum()
    np.testing.assert_allclose(c["x"], x1, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(c["w"], w, rtol=1e-9)
    np.testing.assert_allclose(c["means"][0], np.sum(w * x1), rtol=1e-10)
    np.testing.assert_allclose(c["neff"][0], 1.0 / np.sum(w ** 2), rtol=1e-9)


def _engine_like_step(x0, w0, z, N, epoch, thresh=0.5, reg=False):
    """The NumPy oracle's step (pinned to the reference) recorded the way the resident kernel's
    trace records it: fp32 predicted particles and log-weights, int32 ancestors."""
    from tests.teacher_forced import StepOracle
    from oracle.pf_oracle import OracleState

    ssm = ssm_oracle.sv_logsq(0.95, 0.2, 1.0)
    o = StepOracle(ssm.g_vec, ssm.h_vec, ssm.Q, ssm.R, seed=42, rep=0, bm24=True, epoch=epoch, Np=N,
                   resample_thresh=thresh, resample_method="systematic", regularize_after_resample=reg,
                   vectorized=True)
    o.state = OracleState(x0[:, None].copy(), w0.copy(), np.zeros(1), np.eye(1), 0)
    st = o.step(np.array([z]))
    anc = None if o.idx is None else o.idx.astype(np.int32)
    rec = dict(xe=o.pre_x[:, 0].astype(np.float32), le=np.log(o.pre_w).astype(np.float32), anc=anc,
               neff_e=o.last_neff, flag_e=o.last_resampled, mean_e=float(st.mean[0]), var_e=float(st.cov[0, 0]))
    return o, st, rec


@pytest.mark.parametrize("reg", [False, True])
def test_check_step_against_numpy_oracle(golden_sv, reg):
    """oracle/sir_philox.c pfo_sir_scalar_check_step (the trace checker of the resident kernel's
    in-launch steps, tests/test_gpu_resident_trace.py) reproduces the NumPy oracle's step: fed the
    oracle's own step as the 'engine' record it measures fp32 rounding only, ancestors equal, and
    its fp64 reference quantities (Neff, decision, moments) equal the NumPy oracle's."""
    X, Y = golden_sv["X0"], golden_sv["Y0"]
    N = 20000
    rs = np.random.default_rng(5)
    x0 = X[0] + 0.7 * rs.standard_normal(N)
    w0 = rs.random(N) ** 8
    w0 /= w0.sum()  # Neff well below N / 2: the step resamples
    z = float(np.log(Y[3] ** 2))
    o, st, rec = _engine_like_step(x0, w0, z, N, epoch=6, reg=reg)
    assert o.last_resampled
    c = SP.check_step(SP.sv_logsq_model(0.95, 0.2, 1.0), seed=42, rep=0, epoch=6, thresh=0.5, x0=x0, w0=w0, z=z,
                      regularize=reg, **rec)
    assert c["dx_pre"] <= 1e-6 and c["tv_w"] <= 1e-5 and c["dcdf"] <= 1e-5
    np.testing.assert_allclose(c["neff_o"], o.last_neff, rtol=1e-12)
    assert c["flag_o"] and c["n_anc_bad"] == 0 and c["n_anc_oracle_diff"] == 0
    assert c["n_anc_self_diff"] <= 3 and c["max_margin_self"] <= 1e-6  # the fp32-rounded weights' own CDF
    np.testing.assert_allclose(c["mean_o"], st.mean[0], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(c["var_o"], st.cov[0, 0], rtol=1e-9)
    assert c["dmean"] <= 1e-13 and c["eps_w"] < 1e-4
    # tampering: an ancestor moved to the next index, a non-monotone slot
    bad = rec["anc"].copy()
    bad[N // 2] += 1
    c2 = SP.check_step(SP.sv_logsq_model(0.95, 0.2, 1.0), seed=42, rep=0, epoch=6, thresh=0.5, x0=x0, w0=w0, z=z,
                       regularize=reg, **dict(rec, anc=bad))
    assert c2["n_anc_oracle_diff"] >= 1 and c2["max_margin_oracle"] > 0.0
    bad[N // 2 + 1] = 0
    c3 = SP.check_step(SP.sv_logsq_model(0.95, 0.2, 1.0), seed=42, rep=0, epoch=6, thresh=0.5, x0=x0, w0=w0, z=z,
                       regularize=reg, **dict(rec, anc=bad))
    assert c3["n_anc_bad"] >= 1


def test_check_step_no_resample(golden_sv):
    X, Y = golden_sv["X0"], golden_sv["Y0"]
    N = 8192
    x0 = X[0] + 0.3 * np.random.default_rng(1).standard_normal(N)
    w0 = np.full(N, 1.0 / N)
    z = float(np.log(Y[2] ** 2))
    o, st, rec = _engine_like_step(x0, w0, z, N, epoch=4, thresh=0.01)
    assert not o.last_resampled
    c = SP.check_step(SP.sv_logsq_model(0.95, 0.2, 1.0), seed=42, rep=0, epoch=4, thresh=0.01, x0=x0, w0=w0, z=z,
                      **rec)
    assert not c["flag_o"] and c["n_anc_oracle_diff"] == 0
    np.testing.assert_allclose(c["mean_o"], st.mean[0], rtol=1e-12)
    np.testing.assert_allclose(c["var_o"], st.cov[0, 0], rtol=1e-10)
    assert c["dmean"] <= 1e-13
