"""Runtime-shape kernels (csrc/pf_dyn.h) on an MI355X (-m gpu).

Models outside the compiled (nx, nz, g, h) list run on kernels that take nx / nz as arguments.
Parity, stated per test:

* every golden reference run (tests/golden/pf_runs.npz) forced onto the runtime path, fp64
  replay (the reference's own draws): the tolerances of test_replay_fp64_matches_reference
  (means rtol 1e-9, covariances 1e-8, identical resample decisions);
* shapes no reference run covers — L96 with nx = 12 (the builder's second L96 golden case,
  tests/golden/l96_data.npz ``*2``), the 9-D bearings-only SIR of
  SPF_results_reproduction_example2.ipynb, a 5-D linear system with a dense non-diagonal R —
  against the oracle (oracle/pf_oracle.py, pinned bit-for-bit to the reference) on the same
  replayed draws: same tolerances.  Parity against the reference's own outputs for these shapes
  is unpinned (no reference run of them exists); the oracle carries the pin;
* device RNG: the run() device loop equals the step API bitwise; a replicate batch equals its
  single replicates bitwise; nx = 1000 (simulate_lorenz96's default) runs and tracks.
"""

import numpy as np
import pytest

import particle_filters_amd as pfa
from particle_filters_amd import models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch
from oracle import pf_oracle, ssm_oracle
from tests import pf_cases
from tests.test_gpu_parity import run_engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from particle_filters_amd import _native
    assert _native.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def check_fp64(out, ref, name):
    assert np.array_equal(out["flags"], ref["flags"]), f"{name}: resample decisions differ"
    np.testing.assert_allclose(out["init_particles"], ref["init_particles"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(out["means"], ref["means"], rtol=1e-9, atol=1e-9, err_msg=name)
    np.testing.assert_allclose(out["covs"], ref["covs"], rtol=1e-8, atol=1e-9, err_msg=name)
    np.testing.assert_allclose(out["ess"], ref["ess"], rtol=1e-9, err_msg=name)
    np.testing.assert_allclose(out["neff"], ref["neff"], rtol=1e-9, err_msg=name)
    np.testing.assert_allclose(out["final_particles"], ref["final_particles"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(out["final_weights"], ref["final_weights"], rtol=1e-8, atol=1e-15)


@pytest.mark.parametrize("name", pf_cases.RUN_NAMES)
def test_runtime_path_replays_reference(name, golden_runs, golden_sv, golden_l96, golden_mat):
    ref = pf_cases.golden(golden_runs, name)
    out, _ = run_engine(name, golden_sv, golden_l96, golden_mat, golden_runs, "fp64", kernel_path="runtime")
    check_fp64(out, ref, name)


def engine_replay(g, h, ssm, Z, *, Np, seed, mean0, cov0, method="systematic", reg=False, thresh=0.5,
                  precision="fp64"):
    pf = pfa.ParticleFilter(g, h, ssm.Q, ssm.R, Np=Np, resample_thresh=thresh, resample_method=method,
                            regularize_after_resample=reg, rng=np.random.default_rng(seed), rng_mode="host",
                            precision=precision)
    assert pf.kernel_path_used == "runtime"
    st0 = pf.initialize(np.asarray(mean0, float), np.asarray(cov0, float))
    T = Z.shape[0]
    out = dict(init_particles=st0.particles.copy(), means=np.zeros((T, pf.nx)), covs=np.zeros((T, pf.nx, pf.nx)),
               ess=np.zeros(T), neff=np.zeros(T), flags=np.zeros(T, bool))
    for t in range(T):
        st = pf.step(Z[t])
        out["means"][t] = st.mean
        out["covs"][t] = st.cov
        out["ess"][t] = pf.effective_sample_size()
        out["neff"][t] = pf.last_neff
        out["flags"][t] = pf.last_resampled
    out["final_particles"] = pf.state.particles
    out["final_weights"] = pf.state.weights
    return out


def l96_12_case(golden_l96):
    """L96, nx = 12, F = 6, dt = 0.02, every 3rd component observed (the builder's second
    golden trajectory, observed every step with seeded N(0, 0.5^2) noise)."""
    truth = golden_l96["truth2"]
    H_idx = golden_l96["H_idx2"]
    rng = np.random.default_rng(5)
    Z = truth[1:, H_idx] + 0.5 * rng.standard_normal((truth.shape[0] - 1, H_idx.size))
    ssm = ssm_oracle.lorenz96(nx=12, F=6.0, dt=0.02, obs_fraction=3, obs_error_std=0.5, q_std=0.1)
    g, h = M.L96Transition(6.0, 0.02, 12), M.SelectObservation(H_idx, 12)
    return ssm, g, h, Z, truth


@pytest.mark.parametrize("method,reg", [("systematic", True), ("multinomial", False)])
def test_l96_nx12_replay_vs_oracle(golden_l96, method, reg):
    ssm, g, h, Z, truth = l96_12_case(golden_l96)
    kw = dict(Np=700, seed=11, mean0=truth[0] + 0.3, cov0=np.eye(12), method=method, reg=reg)
    ref = pf_oracle.build_and_run(ssm, Z, **kw)
    assert ref["flags"].any()
    out = engine_replay(g, h, ssm, Z, **kw)
    check_fp64(out, ref, f"l96_12_{method}")


def test_bearings_9d_replay_vs_oracle():
    """The notebook's 9-D SIR comparison (cell 7): x + A x dt, azimuth / elevation, R = 1e-6 I,
    prior N(s_prior0, P_prior0) (cell 1 e2_build_config), on a simulated trajectory."""
    ssm = ssm_oracle.bearings_9d()
    s_true = np.array([40.0, 40.0, 40.0, 8.0, 0.0, -3.0, 0.0, 0.0, 0.0])
    rng = np.random.default_rng(42)
    Z = []
    for _ in range(15):
        s_true = ssm.g(s_true, None)
        Z.append(ssm.h(s_true) + rng.multivariate_normal(np.zeros(2), ssm.R))
    Z = np.array(Z)
    mean0 = np.array([50.0, 50.0, 10.0, 10.0, 40.0, 0.0, 0.0, 0.0, 0.0])
    cov0 = np.diag([10.0, 10.0, 10.0, 1e4, 1e4, 1e4, 10.0, 10.0, 10.0])
    g = M.LinearTransition(np.eye(9) + ssm.A * ssm.dt)
    h = M.BearingsObservation(9)
    kw = dict(Np=2000, seed=42, mean0=mean0, cov0=cov0, reg=True)
    ref = pf_oracle.build_and_run(ssm, Z, **kw)
    out = engine_replay(g, h, ssm, Z, **kw)
    # g = (I + A dt) x on the device vs x + (A x) dt in the oracle: ~1e-16 relative per step
    assert np.array_equal(out["flags"], ref["flags"])
    np.testing.assert_allclose(out["means"], ref["means"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(out["neff"], ref["neff"], rtol=1e-7)
    np.testing.assert_allclose(out["final_particles"], ref["final_particles"], rtol=1e-9, atol=1e-9)


def test_linear_5d_dense_R_replay_vs_oracle():
    """A dense 5-D linear system with a dense Q, a 3-D dense H and a non-diagonal R (the
    forward substitution and the dense noise factors of the runtime kernels)."""
    rng = np.random.default_rng(3)
    A = 0.9 * np.eye(5) + 0.05 * rng.standard_normal((5, 5))
    H = rng.standard_normal((3, 5))
    B = rng.standard_normal((5, 5))
    Q = 0.05 * (B @ B.T / 5 + np.eye(5))
    C = rng.standard_normal((3, 3))
    R = 0.2 * (C @ C.T / 3 + np.eye(3))
    ssm = ssm_oracle.linear(A, H, Q, R)
    x = np.zeros(5)
    Z = []
    for _ in range(25):
        x = A @ x + np.linalg.cholesky(Q) @ rng.standard_normal(5)
        Z.append(H @ x + np.linalg.cholesky(R) @ rng.standard_normal(3))
    Z = np.array(Z)
    kw = dict(Np=1500, seed=9, mean0=np.zeros(5), cov0=np.eye(5), reg=True, thresh=0.8)
    ref = pf_oracle.build_and_run(ssm, Z, **kw)
    assert ref["flags"].any()
    out = engine_replay(M.LinearTransition(A), M.LinearObservation(H), ssm, Z, **kw)
    check_fp64(out, ref, "linear_5d")


def test_runtime_run_equals_step_api():
    """Device RNG: the whole-run device loop and the step API draw the same Philox numbers."""
    g, h = M.L96Transition(8.0, 0.01, 24), M.SelectObservation(np.arange(0, 24, 4), 24)
    Q, R = 0.01 * np.eye(24), np.eye(6)
    Z = np.random.default_rng(1).standard_normal((12, 6))
    mean0, cov0 = np.full(24, 1.0), np.eye(24)
    means = []
    for mode in ("step", "run"):
        pf = pfa.ParticleFilter(g, h, Q, R, Np=3000, regularize_after_resample=True, precision="fp64",
                                rng=np.random.default_rng(4))
        assert pf.kernel_path_used == "runtime"
        pf.initialize(mean0, cov0)
        if mode == "step":
            means.append(np.array([pf.step(z).mean for z in Z]))
        else:
            means.append(pf.run(Z).means[:, 0, :])
    np.testing.assert_array_equal(means[0], means[1])


def test_runtime_batch_equals_single_replicates():
    g, h = M.LinearTransition(0.95 * np.eye(6)), M.LinearObservation(np.eye(6)[:2])
    Q, R = 0.04 * np.eye(6), 0.5 * np.eye(2)
    Z = np.random.default_rng(2).standard_normal((10, 2))
    kw = dict(Np=2500, regularize_after_resample=True, seed=77, precision="fp32")
    b = ParticleFilterBatch(g, h, Q, R, n_replicates=3, **kw)
    b.initialize(np.zeros(6), np.eye(6))
    allm = b.run(Z).means
    for r in range(3):
        s = ParticleFilterBatch(g, h, Q, R, n_replicates=1, replicate_base=r, **kw)
        s.initialize(np.zeros(6), np.eye(6))
        np.testing.assert_array_equal(s.run(Z).means[:, 0], allm[:, r])


def test_runtime_moments_match_state():
    """PFState.cov (nx > 4: the two-pass moment kernels) equals np.cov of the downloaded state."""
    g, h = M.LinearTransition(0.9 * np.eye(7)), M.LinearObservation(np.ones((1, 7)))
    pf = pfa.ParticleFilter(g, h, 0.1 * np.eye(7), [[0.3]], Np=4000, precision="fp64",
                            rng=np.random.default_rng(3))
    pf.initialize(np.zeros(7), np.eye(7))
    pf.predict()
    st = pf.update([0.7])
    x, w = pf.state.particles, pf.state.weights
    np.testing.assert_allclose(st.mean, np.average(x, weights=w, axis=0), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(st.cov, np.cov(x, rowvar=False, aweights=w, bias=True), rtol=1e-9, atol=1e-12)


def test_l96_nx1000_runs_and_tracks():
    """simulate_lorenz96's default dimension (nx = 1000, every 4th observed): the runtime kernels
    track the truth from a spread prior (RMSE well below the prior's)."""
    sim = S.simulate_lorenz96(nx=1000, F=8.0, dt=0.01, spinup_steps=200, total_steps=10, Np=1, seed=3)
    truth = sim.truth_traj
    H_idx = sim.H_idx
    rng = np.random.default_rng(0)
    Z = truth[1:, H_idx] + rng.standard_normal((truth.shape[0] - 1, H_idx.size))
    g, h = M.L96Transition(8.0, 0.01, 1000), M.SelectObservation(H_idx, 1000)
    pf = pfa.ParticleFilter(g, h, 0.01 * np.eye(1000), np.eye(H_idx.size), Np=2048, precision="fp32",
                            regularize_after_resample=True, rng=np.random.default_rng(1))
    assert pf.kernel_path_used == "runtime"
    pf.initialize(truth[0], 0.25 * np.eye(1000))
    res = pf.run(Z)
    m = res.means[:, 0, :]
    assert np.all(np.isfinite(m))
    rmse = np.sqrt(np.mean((m - truth[1:]) ** 2))
    assert rmse < 1.0, rmse  # prior spread 0.5; 250 unit-noise observations per step
