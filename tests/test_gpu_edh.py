"""HIP EDH flow filter vs the reference's own outputs and the oracle (-m gpu, MI355X).

tests/golden/edh_runs.npz holds the reference EDHFlowPF + EKF run on fixed seeds
(tests/golden/make_golden_edh.py).  The engine in rng_mode="host" consumes the identical
random stream (initial multivariate_normal, the process_noise_sampler's draws, the
resampling uniform), so its outputs are compared per step.

Tolerances (fp64 engine): the per-particle RK4 / Euler integration of the shared affine
field is applied as ONE composed affine map (pf_edh_kernels.h), and reductions run in a
different order, so agreement is to rounding amplified by the flow: posterior means and
particles within 1e-9 of the state scale, covariances within 1e-8, weights rtol 1e-7,
condition-number diagnostics rtol 1e-6; resample decisions identical.
"""

import os

import numpy as np
import pytest

from particle_filters_amd import edh as ED
from particle_filters_amd import models as M
from particle_filters_amd import trackers as TR
from oracle import edh_oracle as EO
from oracle import ledh_oracle as LO

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(__file__)
GOLD = np.load(os.path.join(HERE, "golden", "edh_runs.npz"))
MAT = np.load(os.path.join(HERE, "golden", "mat_data.npz"))
L96 = np.load(os.path.join(HERE, "golden", "l96_data.npz"))
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
    elif name.startswith("l96"):
        om = LO.lorenz96(40)
        gm, hm = M.L96Transition(8.0, 0.01, 40), M.SelectObservation(np.arange(0, 40, 4), 40)
    else:
        raise KeyError(name)
    return om, gm, hm, g


def make_filter(name, rng_mode="host", n_particles=None, ratio=None, seed=None, device_models_tracker=False):
    om, gm, hm, g = case(name)
    if device_models_tracker:
        ekf = TR.ExtendedKalmanFilter(gm, hm, om.Q, om.R, jac_g=gm.jacobian, jac_h=hm.jacobian)
    else:
        ekf = TR.ExtendedKalmanFilter(om.g_ekf, om.h, om.Q, om.R, jac_g=om.jac_g, jac_h=om.jac_h)
    tracker = TR.EKFTracker(ekf, TR.EKFState(np.asarray(g["mean0"], float).copy(),
                                             np.asarray(g["cov0"], float).copy(), 0))
    cfg = ED.EDHConfig(n_particles=int(g["n_particles"]) if n_particles is None else n_particles,
                       n_lambda_steps=int(g["n_lambda"]),
                       resample_ess_ratio=float(g["ratio"]) if ratio is None else ratio,
                       flow_integrator=str(g["integrator"]),
                       rng=np.random.default_rng(int(g["seed"]) if seed is None else seed))
    pf = ED.EDHFlowPF(tracker, gm, hm, hm.jacobian, M.GaussianTransitionDensity(gm, om.Q),
                      M.GaussianLikelihood(hm, om.R), om.R, cfg, rng_mode=rng_mode)
    return pf, cfg, om, g


@pytest.mark.parametrize("name", NAMES)
def test_step_matches_reference(name):
    pf, cfg, om, g = make_filter(name)
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    np.testing.assert_array_equal(st.particles, g["init_particles"])
    np.testing.assert_allclose(st.mean, g["init_mean"], rtol=0, atol=1e-12 * max(1.0, np.abs(g["init_mean"]).max()))
    sampler = lambda n, nx: cfg.rng.multivariate_normal(np.zeros(nx), om.Q, size=n)  # noqa: E731
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


def test_edh_handle_refuses_ledh_step():
    pf, cfg, om, g = make_filter("l96_rk4")
    from particle_filters_amd import _native as N
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    P = np.eye(40)
    z = np.ascontiguousarray(g["Z"][0], float)
    rc = N.load().pf_ledh_step(pf._h, N.dptr(P), N.dptr(z), None, N.PF_NOISE_NONE, None, None, None)
    assert rc == N.PF_E_ARG
    del st


@pytest.mark.parametrize("name", ["l96_rk4", "l96_euler", "acoustic"])
def test_run_equals_step_without_noise(name):
    """pf_edh_run (device-resident loop, tracker sequence uploaded up front, all flow maps built
    in one batched launch) reproduces the step API when nothing random happens after the
    initial draw (no process noise, no resampling)."""
    pf1, _, om, g = make_filter(name, ratio=0.0)
    st1 = pf1.init_from_gaussian(g["mean0"], g["cov0"])
    means = []
    for t in range(len(g["Z"])):
        st1 = pf1.step(st1, g["Z"][t])
        means.append(st1.mean)
    pf2, _, _, _ = make_filter(name, ratio=0.0)
    st2 = pf2.init_from_gaussian(g["mean0"], g["cov0"])
    res = pf2.run(st2, g["Z"], process_noise="none")
    scale = max(1.0, float(np.abs(np.array(means)).max()))
    np.testing.assert_allclose(res.means, np.array(means), rtol=0, atol=1e-12 * scale)
    np.testing.assert_allclose(pf2.state.particles, st1.particles, rtol=0, atol=1e-11 * scale)
    assert not res.flags.any()


def truth(name, T):
    if name.startswith("l96"):
        return L96["truth"][1:T + 1]
    if name == "acoustic":
        return MAT["X2"][1:T + 1, 0]
    sv = np.load(os.path.join(HERE, "golden", "sv_data.npz"))
    return sv["X0"][1:T + 1, None]


@pytest.mark.parametrize("name", ["l96_rk4", "acoustic", "sv_exp"])
def test_device_rng_run_statistics(name):
    """Device noise + device resampling (Philox) vs the oracle with NumPy noise: the RMSE of
    the posterior means against the simulator's truth agrees within a Monte-Carlo band."""
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
        o = EO.run_edh(om, g["Z"], mean0=g["mean0"], cov0=g["cov0"], n_particles=n,
                       n_lambda_steps=int(g["n_lambda"]), ratio=float(g["ratio"]), seed=seed,
                       integrator=str(g["integrator"]), vectorized=True)
        rm_o.append(float(np.sqrt(np.mean((o["means"] - tr.reshape(o["means"].shape)) ** 2))))
    lo, hi = min(rm_o), max(rm_o)
    assert 0.5 * lo - 0.05 <= rm_e <= 1.5 * hi + 0.05, (rm_e, rm_o)


@pytest.mark.parametrize("name", ["l96_rk4", "acoustic"])
def test_run_with_device_tracker_equals_host_tracker(name):
    """run(tracker='device') (device EKF also emitting the past means x_{k-1|k-1}) ==
    run(tracker='host') on identical Philox draws, to the rounding of the two EKFs."""
    pf1, _, _, g = make_filter(name, rng_mode="device", n_particles=2000, seed=11, device_models_tracker=True)
    st1 = pf1.init_from_gaussian(g["mean0"], g["cov0"])
    r1 = pf1.run(st1, g["Z"], tracker="device")
    pf2, _, _, _ = make_filter(name, rng_mode="device", n_particles=2000, seed=11, device_models_tracker=True)
    st2 = pf2.init_from_gaussian(g["mean0"], g["cov0"])
    r2 = pf2.run(st2, g["Z"], tracker="host")
    scale = max(1.0, float(np.abs(r2.means).max()))
    np.testing.assert_array_equal(r1.flags, r2.flags)
    np.testing.assert_allclose(r1.means, r2.means, rtol=0, atol=1e-8 * scale)
