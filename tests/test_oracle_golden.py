"""Pin the CPU oracle to the reference: every golden fixture was produced by the
reference itself (tests/golden/make_golden.py); the oracle must reproduce it
bit-for-bit in fp64 before it is trusted as the checker of the HIP engine."""

import numpy as np
import pytest

from oracle import pf_oracle, ssm_oracle
from tests import pf_cases

EXACT_KEYS = ["means", "covs", "ess", "neff", "flags", "final_particles", "final_weights",
              "init_particles"]


@pytest.mark.parametrize("name", pf_cases.RUN_NAMES)
def test_vectorized_oracle_matches_reference_bitwise(name, golden_runs, golden_sv, golden_l96,
                                                     golden_mat):
    ssm, Z, controls, kw = pf_cases.build(name, golden_sv, golden_l96, golden_mat, golden_runs)
    ref = pf_cases.golden(golden_runs, name)
    out = pf_oracle.build_and_run(ssm, Z, controls=controls, vectorized=True, **kw)
    if name == "linear_sys" or name == "linear_multi_reg":
        # X @ A.T (gemm) vs A @ x (gemv) may round differently: 1e-12, not bitwise
        for k in EXACT_KEYS:
            np.testing.assert_allclose(out[k], ref[k], rtol=1e-10, atol=1e-12, err_msg=k)
    else:
        for k in EXACT_KEYS:
            assert np.array_equal(out[k], ref[k]), f"{name}:{k} differs from reference"
    assert out["t_final"] == int(ref["t_final"])


@pytest.mark.parametrize("name", ["sv_harness", "sv_logsq_multi_reg", "linear_multi_reg", "mat"])
def test_faithful_oracle_matches_reference_bitwise(name, golden_runs, golden_sv, golden_l96,
                                                   golden_mat):
    """Per-particle callbacks exactly like particle_filter.py:237,257."""
    ssm, Z, controls, kw = pf_cases.build(name, golden_sv, golden_l96, golden_mat, golden_runs)
    ref = pf_cases.golden(golden_runs, name)
    if name in ("sv_harness", "sv_logsq_multi_reg"):
        Z = Z[:200]
        for k in ("means", "ess", "flags"):
            ref[k] = ref[k][:200]
    out = pf_oracle.build_and_run(ssm, Z, controls=controls, vectorized=False, **kw)
    for k in ("means", "ess", "flags", "neff"):
        if name.startswith("linear"):
            np.testing.assert_allclose(out[k], ref[k][: len(out[k])], rtol=1e-10, atol=1e-12)
        else:
            assert np.array_equal(out[k], ref[k][: len(out[k])]), f"{name}:{k}"


def test_resample_indices_match_reference(golden_resample):
    """systematic == searchsorted(cdf, (U+i)/N, 'right'); choice(p=w) == random(N) + search."""
    for name in golden_resample["names"]:
        w = golden_resample[f"{name}_w"]
        U = float(golden_resample[f"{name}_U"])
        assert np.array_equal(pf_oracle.systematic_indices(w, U), golden_resample[f"{name}_sys"]), name
        u = golden_resample[f"{name}_u"]
        assert np.array_equal(pf_oracle.multinomial_indices(w, u), golden_resample[f"{name}_multi"]), name


def test_recording_choice_consumes_like_generator_choice():
    w = np.random.default_rng(1).random(777)
    w /= w.sum()
    a = np.random.default_rng(9).choice(777, size=777, p=w)
    rec = pf_oracle.RecordingRNG(np.random.default_rng(9))
    b = rec.choice(777, size=777, p=w)
    assert np.array_equal(a, b)
    # and the next draw of both streams agrees
    g = np.random.default_rng(9)
    g.choice(777, size=777, p=w)
    assert g.standard_normal() == rec.standard_normal()


def test_replay_rng_reproduces_run(golden_runs, golden_sv, golden_l96, golden_mat):
    ssm, Z, controls, kw = pf_cases.build("sv_logsq_multi_reg", golden_sv, golden_l96, golden_mat,
                                          golden_runs)
    rec = pf_oracle.RecordingRNG(np.random.default_rng(kw["seed"]))
    a = pf_oracle.build_and_run(ssm, Z[:50], rng=rec, **kw)
    b = pf_oracle.build_and_run(ssm, Z[:50], rng=pf_oracle.ReplayRNG(rec.log), **kw)
    assert np.array_equal(a["means"], b["means"])
    kinds = {k for k, _ in rec.log}
    assert kinds == {"normal", "uniform"}


def test_logchi2_constants():
    assert ssm_oracle.LOGCHI2_MEAN == pytest.approx(-1.2703628454614782, abs=1e-15)
    assert ssm_oracle.LOGCHI2_VAR == pytest.approx(np.pi ** 2 / 2, abs=1e-14)


def test_sv_integration_rmse_bound(golden_runs, golden_sv):
    """test_pf_vs_simulator_sv.py:99-148: RMSE < 1.5 (reference outputs pinned)."""
    ref = pf_cases.golden(golden_runs, "sv_it")
    est = np.r_[golden_sv["X1"][0], ref["means"][:, 0]]
    rmse = np.sqrt(np.mean((est - golden_sv["X1"]) ** 2))
    assert rmse < 1.5
