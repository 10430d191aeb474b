"""HIP LEDH flow filter vs the reference's own outputs and the oracle (-m gpu, MI355X).

tests/golden/ledh_runs.npz holds the reference LEDHFlowPF + EKF run on fixed seeds
(tests/golden/make_golden_ledh.py).  The engine in rng_mode="host" consumes the
identical random stream (initial multivariate_normal, the process_noise_sampler's
draws, the resampling uniform), so its outputs are compared per step.

Tolerances (fp64 engine): the flow is evaluated in observation space (matrix
determinant lemma, A v = Gm (H v); see pf_ledh_kernels.h) and reductions run in a
different order, so agreement is to rounding amplified by the flow: posterior
means within 1e-9 (relative to the state scale), covariances within 1e-8,
condition-number diagnostics within rtol 1e-6; resample decisions identical.
"""

import os

import numpy as np
import pytest

from particle_filters_amd import ledh as LD
from particle_filters_amd import models as M
from particle_filters_amd import trackers as TR
from oracle import ledh_oracle as LO

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "ledh_runs.npz"))
MAT = np.load(os.path.join(os.path.dirname(__file__), "golden", "mat_data.npz"))
L96 = np.load(os.path.join(os.path.dirname(__file__), "golden", "l96_data.npz"))
NAMES = [str(n) for n in GOLD["names"]]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from particle_filters_amd import _native
    assert _native.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def case(name):
    g = {k.split("__", 1)[1]: GOLD[k] for k in GOLD.files if k.startswith(name + "__")}
    psi, d0 = float(MAT["meta2"][2]), float(MAT["meta2"][3])
    if name.startswith("lin1d"):
        om = LO.linear_1d()
        gm, hm = M.SVTransition(0.9), M.LinearObservation([[1.0]])
    elif name == "sv_exp":
        om = LO.sv_exp_half(0.95, 0.2, 1.0, 0.1)
        gm, hm = M.SVTransition(0.95), M.ExpHalfObservation(1.0)
    elif name == "acoustic":
        om = LO.acoustic_single(MAT["S2"], psi=psi, d0=d0)
        gm, hm = M.CVTransition(1, 1.0), M.AcousticObservation(MAT["S2"], psi, d0, 1)
    elif name == "l96":
        om = LO.lorenz96(40)
        gm, hm = M.L96Transition(8.0, 0.01, 40), M.SelectObservation(np.arange(0, 40, 4), 40)
    elif name == "mat_joint":  # the MAT notebook's joint 16-D / 25-sensor wiring (nz = 25, per-particle flow)
        from particle_filters_amd.simulators import article_process_noise_cov
        pj, dj = float(MAT["meta"][2]), float(MAT["meta"][3])
        om = LO.acoustic_joint(MAT["S"], psi=pj, d0=dj, n_targets=4, Q_single=article_process_noise_cov())
        gm, hm = M.CVTransition(4, 1.0), M.AcousticObservation(MAT["S"], pj, dj, 4)
    else:
        raise KeyError(name)
    return om, gm, hm, g


def make_filter(name, flow="auto", rng_mode="host", n_particles=None, ratio=None, seed=None):
    om, gm, hm, g = case(name)
    ekf = TR.ExtendedKalmanFilter(om.g_ekf, om.h, om.Q, om.R, jac_g=om.jac_g, jac_h=om.jac_h)
    tracker = TR.EKFTracker(ekf, TR.EKFState(np.asarray(g["mean0"], float).copy(),
                                             np.asarray(g["cov0"], float).copy(), 0))
    cfg = LD.LEDHConfig(n_particles=int(g["n_particles"]) if n_particles is None else n_particles,
                        n_lambda_steps=int(g["n_lambda"]),
                        resample_ess_ratio=float(g["ratio"]) if ratio is None else ratio,
                        rng=np.random.default_rng(int(g["seed"]) if seed is None else seed))
    pf = LD.LEDHFlowPF(tracker, gm, hm, hm.jacobian, M.GaussianTransitionDensity(gm, om.Q),
                       M.GaussianLikelihood(hm, om.R), om.R, cfg, rng_mode=rng_mode, flow=flow)
    return pf, cfg, om, g


@pytest.mark.parametrize("flow", ["auto", "per_particle"])
@pytest.mark.parametrize("name", NAMES)
def test_step_matches_reference(name, flow):
    pf, cfg, om, g = make_filter(name, flow=flow)
    if flow == "auto":
        assert pf.shared_jacobian_path == (name in ("lin1d", "lin1d_nonoise", "l96"))
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    np.testing.assert_array_equal(st.particles, g["init_particles"])
    np.testing.assert_allclose(st.mean, g["init_mean"], rtol=0, atol=1e-12 * max(1.0, np.abs(g["init_mean"]).max()))
    np.testing.assert_allclose(st.cov, g["init_cov"], rtol=1e-10, atol=1e-12)
    noise = bool(g["noise"]) if "noise" in g else True
    sampler = (lambda n, nx: cfg.rng.multivariate_normal(np.zeros(nx), om.Q, size=n)) if noise else None
    scale = max(1.0, float(np.abs(g["means"]).max()))
    for t in range(len(g["Z"])):
        st = pf.step(st, g["Z"][t], process_noise_sampler=sampler)
        assert pf.last_resampled == bool(g["flags"][t]), f"resample decision differs at step {t}"
        np.testing.assert_allclose(st.mean, g["means"][t], rtol=0, atol=1e-9 * scale, err_msg=f"mean t={t}")
        cs = max(1.0, float(np.abs(g["covs"][t]).max()))
        np.testing.assert_allclose(st.cov, g["covs"][t], rtol=0, atol=1e-8 * cs, err_msg=f"cov t={t}")
        np.testing.assert_allclose(st.weights, g["weights"][t], rtol=1e-7, atol=1e-13, err_msg=f"w t={t}")
        np.testing.assert_allclose(st.particles, g["particles"][t], rtol=0, atol=1e-9 * scale, err_msg=f"x t={t}")
        np.testing.assert_allclose(st.diagnostics["condition_numbers"], g["conds"][t], rtol=1e-6)


def test_run_equals_step_without_noise():
    """pf_ledh_run (device-resident loop, tracker covariances uploaded up front) reproduces
    the step API when nothing random happens after the initial draw (no process noise,
    no resampling)."""
    name = "l96"
    pf1, cfg1, om, g = make_filter(name, ratio=0.0)
    st1 = pf1.init_from_gaussian(g["mean0"], g["cov0"])
    means = []
    for t in range(len(g["Z"])):
        st1 = pf1.step(st1, g["Z"][t])
        means.append(st1.mean)
    pf2, _, _, _ = make_filter(name, ratio=0.0)
    st2 = pf2.init_from_gaussian(g["mean0"], g["cov0"])
    res = pf2.run(st2, g["Z"], process_noise="none")
    np.testing.assert_allclose(res.means, np.array(means), rtol=0, atol=1e-12 * 10)
    np.testing.assert_allclose(pf2.state.particles, st1.particles, rtol=0, atol=1e-11)
    assert not res.flags.any()


def truth(name, T):
    if name == "l96":
        return L96["truth"][1:T + 1]
    if name == "acoustic":
        return MAT["X2"][1:T + 1, 0]
    sv = np.load(os.path.join(os.path.dirname(__file__), "golden", "sv_data.npz"))
    return sv["X0"][1:T + 1, None]


@pytest.mark.parametrize("name", ["l96", "acoustic", "sv_exp"])
def test_device_rng_run_statistics(name):
    """Device noise + device resampling (Philox) vs the oracle with NumPy noise: the
    RMSE of the posterior means against the simulator's truth agrees (independent
    Monte-Carlo draws, so within a band, not to rounding)."""
    om, gm, hm, g = case(name)
    n = 2000
    pf, cfg, _, _ = make_filter(name, rng_mode="device", n_particles=n, seed=11)
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    res = pf.run(st, g["Z"], process_noise="device")
    assert np.all(np.isfinite(res.means)) and np.all(np.isfinite(res.covs))
    assert np.all(res.ess > 0) and np.all(res.ess <= n * (1 + 1e-9))
    tr = truth(name, len(g["Z"]))
    rm_e = res.rmse(tr)
    rm_o = []
    for seed in (11, 12, 13):
        o = LO.run_ledh(om, g["Z"], mean0=g["mean0"], cov0=g["cov0"], n_particles=n,
                        n_lambda_steps=int(g["n_lambda"]), ratio=float(g["ratio"]), seed=seed, vectorized=True)
        rm_o.append(float(np.sqrt(np.mean((o["means"] - tr.reshape(o["means"].shape)) ** 2))))
    lo, hi = min(rm_o), max(rm_o)
    assert 0.5 * lo - 0.05 <= rm_e <= 1.5 * hi + 0.05, (rm_e, rm_o)


def test_large_l96_shared_vs_per_particle():
    """The shared-Jacobian flow and the per-particle flow agree for a linear h at N = 4096."""
    name = "l96"
    out = {}
    for flow in ("auto", "per_particle"):
        pf, cfg, om, g = make_filter(name, flow=flow, n_particles=4096, seed=5)
        st = pf.init_from_gaussian(g["mean0"], g["cov0"])
        sampler = lambda n, nx: cfg.rng.multivariate_normal(np.zeros(nx), om.Q, size=n)  # noqa: E731
        ms = []
        for t in range(len(g["Z"])):
            st = pf.step(st, g["Z"][t], process_noise_sampler=sampler)
            ms.append(st.mean)
        out[flow] = np.array(ms)
    np.testing.assert_allclose(out["auto"], out["per_particle"], rtol=0, atol=1e-8)


def device_tracked_filter(name, n_particles=2000, seed=11, rng_mode="device"):
    """A filter whose EKFTracker runs the engine's own device models (analytic Jacobians)."""
    om, gm, hm, g = case(name)
    ekf = TR.ExtendedKalmanFilter(gm, hm, om.Q, om.R, jac_g=gm.jacobian, jac_h=hm.jacobian)
    tracker = TR.EKFTracker(ekf, TR.EKFState(np.asarray(g["mean0"], float).copy(),
                                             np.asarray(g["cov0"], float).copy(), 0))
    cfg = LD.LEDHConfig(n_particles=n_particles, n_lambda_steps=int(g["n_lambda"]),
                        resample_ess_ratio=float(g["ratio"]), rng=np.random.default_rng(seed))
    pf = LD.LEDHFlowPF(tracker, gm, hm, hm.jacobian, M.GaussianTransitionDensity(gm, om.Q),
                       M.GaussianLikelihood(hm, om.R), om.R, cfg, rng_mode=rng_mode)
    return pf, tracker, ekf, g


@pytest.mark.parametrize("name", NAMES)
def test_device_ekf_matches_host_ekf(name):
    """k_ekf_seq (the EKF of extended_kalman_filter.py:164-241 on the device) reproduces the
    host EKF with the same analytic Jacobians: every symmetrised predicted covariance."""
    pf, tracker, ekf, g = device_tracked_filter(name, n_particles=64)
    Ps = pf.tracker_covariances(g["Z"])
    host = TR.EKFTracker(ekf, TR.EKFState(np.asarray(g["mean0"], float).copy(),
                                          np.asarray(g["cov0"], float).copy(), 0))
    for t in range(len(g["Z"])):
        _, P = host.predict()
        ref = 0.5 * (P + P.T)
        np.testing.assert_allclose(Ps[t], ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max(), err_msg=f"t={t}")
        host.update(np.atleast_1d(g["Z"][t]))


@pytest.mark.parametrize("name", ["l96", "acoustic"])
def test_run_with_device_tracker_equals_host_tracker(name):
    """run(tracker='device') == run(tracker_covs=<host EKF covariances>) on identical Philox
    draws, to the rounding of the two EKF evaluations."""
    pf1, tr1, ekf, g = device_tracked_filter(name)
    st1 = pf1.init_from_gaussian(g["mean0"], g["cov0"])
    r1 = pf1.run(st1, g["Z"], tracker="device")
    pf2, tr2, _, _ = device_tracked_filter(name)
    st2 = pf2.init_from_gaussian(g["mean0"], g["cov0"])
    r2 = pf2.run(st2, g["Z"], tracker="host")
    scale = max(1.0, float(np.abs(r2.means).max()))
    np.testing.assert_array_equal(r1.flags, r2.flags)
    np.testing.assert_allclose(r1.means, r2.means, rtol=0, atol=1e-8 * scale)
    np.testing.assert_allclose(tr1.state.cov, tr2.state.cov, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("variant", ["jitter", "joseph"])
def test_device_tracker_rejects_other_ekf_updates(variant):
    """The device EKF runs the plain update (extended_kalman_filter.py:208-239 without jitter or
    the Joseph form): an EKF configured otherwise is refused, not silently run differently."""
    pf, tracker, ekf, g = device_tracked_filter("l96", n_particles=64)
    if variant == "jitter":
        ekf.jitter = 1e-9
    else:
        ekf.joseph = True
    with pytest.raises(NotImplementedError, match="tracker='host'"):
        pf.tracker_covariances(g["Z"])


@pytest.mark.parametrize("algo", ["ledh", "edh"])
def test_fused_step_equals_kernel_chain(algo, monkeypatch):
    """run() on the shared path uses the one-launch fused step (pf_ledh_fused.h); with
    PF_LEDH_FUSED=0 it runs the five-kernel chain.  Same Philox noise and offsets: same
    resample decisions, posterior means within 1e-9 of the state scale (workgroup-order sums)."""
    from particle_filters_amd import edh as ED

    om, gm, hm, g = case("l96")
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PF_LEDH_FUSED", flag)
        ekf = TR.ExtendedKalmanFilter(gm, hm, om.Q, om.R, jac_g=gm.jacobian, jac_h=hm.jacobian)
        tracker = TR.EKFTracker(ekf, TR.EKFState(np.asarray(g["mean0"], float).copy(),
                                                 np.asarray(g["cov0"], float).copy(), 0))
        args = (tracker, gm, hm, hm.jacobian, M.GaussianTransitionDensity(gm, om.Q), M.GaussianLikelihood(hm, om.R),
                om.R)
        if algo == "edh":
            cfg = ED.EDHConfig(n_particles=10000, n_lambda_steps=8, resample_ess_ratio=0.5,
                               rng=np.random.default_rng(3))
            pf = ED.EDHFlowPF(*args, cfg, rng_mode="device")
        else:
            cfg = LD.LEDHConfig(n_particles=10000, n_lambda_steps=8, resample_ess_ratio=0.5,
                                rng=np.random.default_rng(3))
            pf = LD.LEDHFlowPF(*args, cfg, rng_mode="device")
        st = pf.init_from_gaussian(g["mean0"], g["cov0"])
        Z = np.concatenate([g["Z"], L96["obs"][5:25]])
        res = pf.run(st, Z, tracker="device")
        out[flag] = (res, pf.state.particles, pf.state.weights)
    (r1, x1, w1), (r0, x0, w0) = out["1"], out["0"]
    assert r1.flags.sum() >= 2, "the run must exercise the resample path"
    np.testing.assert_array_equal(r1.flags, r0.flags)
    np.testing.assert_allclose(r1.ess, r0.ess, rtol=1e-9)
    scale = max(1.0, float(np.abs(r0.means).max()))
    np.testing.assert_allclose(r1.means, r0.means, rtol=0, atol=1e-9 * scale)
    np.testing.assert_allclose(r1.covs, r0.covs, rtol=0, atol=1e-8 * max(1.0, float(np.abs(r0.covs).max())))
    np.testing.assert_allclose(x1, x0, rtol=0, atol=1e-9 * scale)
    np.testing.assert_allclose(w1, w0, rtol=1e-9, atol=1e-15)


def test_fused_run_failure_poisons_handle(monkeypatch):
    """A fused run whose grid barrier reports a timeout (hook PF_TEST_LEDH_FAIL=1) leaves its state
    part-advanced: the handle must then refuse to continue (AssertionError 'Filter not initialized.'
    from the next call) instead of filtering on from a corrupt state."""
    om, gm, hm, g = case("l96")
    ekf = TR.ExtendedKalmanFilter(gm, hm, om.Q, om.R, jac_g=gm.jacobian, jac_h=hm.jacobian)
    tracker = TR.EKFTracker(ekf, TR.EKFState(np.asarray(g["mean0"], float).copy(),
                                             np.asarray(g["cov0"], float).copy(), 0))
    cfg = LD.LEDHConfig(n_particles=4096, n_lambda_steps=4, resample_ess_ratio=0.5, rng=np.random.default_rng(3))
    pf = LD.LEDHFlowPF(tracker, gm, hm, hm.jacobian, M.GaussianTransitionDensity(gm, om.Q),
                       M.GaussianLikelihood(hm, om.R), om.R, cfg, rng_mode="device")
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    Z = np.asarray(g["Z"], float)
    pf.run(st, Z[:3], tracker="device")  # a good run first
    monkeypatch.setenv("PF_TEST_HOOKS", "1")
    monkeypatch.setenv("PF_TEST_LEDH_FAIL", "1")
    with pytest.raises(Exception) as e:
        pf.run(pf.state, Z[3:6], tracker="device")
    assert "timed out" in str(e.value)
    monkeypatch.delenv("PF_TEST_LEDH_FAIL")
    with pytest.raises(AssertionError, match="Filter not initialized"):
        pf.run(pf.state, Z[6:8], tracker="device")
    # a fresh initialize makes the handle usable again
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    res = pf.run(st, Z[:3], tracker="device")
    assert np.all(np.isfinite(res.means))


def _mat_joint_steps(monkeypatch, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    pf, cfg, om, g = make_filter("mat_joint")
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    sampler = lambda n, nx: cfg.rng.multivariate_normal(np.zeros(nx), om.Q, size=n)  # noqa: E731
    steps = []
    for t in range(len(g["Z"])):
        st = pf.step(st, g["Z"][t], process_noise_sampler=sampler)
        steps.append((st.particles.copy(), st.weights.copy(), st.mean.copy(), pf.last_resampled))
    for k in env:
        monkeypatch.delenv(k, raising=False)
    return steps, max(1.0, float(np.abs(g["means"]).max()))


@pytest.mark.parametrize("force", [1, 2, 4, 7])
def test_flow_lr_fallbacks_equal_primary(monkeypatch, force):
    """Advisor (round 5): k_flow_wave_lr's fallback branches, forced by a test hook
    (PF_TEST_FLOW_LR_FORCE, FlowParams::lr_force) on the MAT joint case with the reference's recorded
    noise - bit 0 the Householder QR instead of the Gram's Cholesky factor, bit 1 the separate pivoted
    determinants (lr_logdet) instead of the Gauss-Jordan pair, bit 2 the reference's +1e-12 I retry
    (ledh.py:174-179) - against the primary path: the same flow to rounding (particles 1e-9 scale,
    weights rtol 1e-7, decisions equal); with the QR the particles are not bitwise the primary
    path's (the forced branch did run).  The separate eliminations (bit 1) repeat the Gauss-Jordan
    pair's pivoted arithmetic per matrix and give its determinants bit for bit, and the retry (bit 2)
    moves every particle's log-weight by the same ~1e-9 (NX log(1 + 1e-12) per pseudo-time step),
    which the normalised weights do not see (measured: the outputs stay bitwise equal)."""
    ref, scale = _mat_joint_steps(monkeypatch, {})
    got, _ = _mat_joint_steps(monkeypatch, {"PF_TEST_HOOKS": "1", "PF_TEST_FLOW_LR_FORCE": str(force)})
    differs = False
    for t, (a, b) in enumerate(zip(ref, got)):
        assert a[3] == b[3], f"resample decision differs at step {t}"
        np.testing.assert_allclose(b[0], a[0], rtol=0, atol=1e-9 * scale, err_msg=f"x t={t}")
        np.testing.assert_allclose(b[1], a[1], rtol=1e-7, atol=1e-13, err_msg=f"w t={t}")
        np.testing.assert_allclose(b[2], a[2], rtol=0, atol=1e-9 * scale, err_msg=f"mean t={t}")
        differs |= not (np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]))
    if force & 1:
        assert differs, "the forced QR left every output bitwise unchanged (hook not taken?)"


def test_flow_lr_equals_dense_flow(monkeypatch):
    """Advisor (round 5): the position-space acoustic flow k_flow_wave_lr against the dense
    observation-space k_flow_wave (PF_FLOW_LR=0, read per launch) on the same inputs - the MAT
    notebook's joint 16-D / 25-sensor case with the reference's recorded noise: particles, weights,
    means and the flow's condition numbers step by step to ~1e-9 (both are fp64 evaluations of
    ledh.py:136-179; they differ only by rounding)."""
    out = {}
    for lr in ("1", "0"):
        monkeypatch.setenv("PF_FLOW_LR", lr)
        pf, cfg, om, g = make_filter("mat_joint")
        st = pf.init_from_gaussian(g["mean0"], g["cov0"])
        sampler = lambda n, nx: cfg.rng.multivariate_normal(np.zeros(nx), om.Q, size=n)  # noqa: E731
        steps = []
        for t in range(len(g["Z"])):
            st = pf.step(st, g["Z"][t], process_noise_sampler=sampler)
            steps.append((st.particles.copy(), st.weights.copy(), st.mean.copy(), pf.last_resampled,
                          np.asarray(st.diagnostics["condition_numbers"]).copy()))
        out[lr] = steps
    scale = max(1.0, float(np.abs(g["means"]).max()))
    for t, (a, b) in enumerate(zip(out["1"], out["0"])):
        assert a[3] == b[3], f"resample decision differs at step {t}"
        np.testing.assert_allclose(a[0], b[0], rtol=0, atol=1e-9 * scale, err_msg=f"x t={t}")
        np.testing.assert_allclose(a[1], b[1], rtol=1e-7, atol=1e-13, err_msg=f"w t={t}")
        np.testing.assert_allclose(a[2], b[2], rtol=0, atol=1e-9 * scale, err_msg=f"mean t={t}")
        np.testing.assert_allclose(a[4], b[4], rtol=1e-6, err_msg=f"cond t={t}")
