"""The benchmarked LEDH / EDH device loop (``run()``: the fused one-launch step k_ledh_fused on the
linear-h path, the kernel chain otherwise) against the reference's own runs, head on (-m gpu).

tests/golden/ledh_runs.npz and edh_runs.npz hold the reference LEDHFlowPF / EDHFlowPF runs
(LEDH_particle_filter.py:93-214, EDH_particle_filter.py:182-317) with process noise and
resampling.  Their random stream is replayed into the device loop: after the initial draw,
step t's process_noise_sampler draw (rng.multivariate_normal(0, Q, N)) and - at the steps the
reference resampled - systematic_resample's rng.random() (ledh.py:28), laid out per step
(``run(..., process_noise="host", replay=(V, U))``, include/pf_ledh.h pf_ledh_set_run_replay).
The loop then takes its own decisions: they must equal the reference's.  Tolerances are those
of the step-API tests (tests/test_gpu_ledh.py, test_gpu_edh.py): every step's posterior mean
within 1e-9 x the state scale, covariance within 1e-8 x its scale, ESS rtol 1e-9 where no resample
reset it; the final particles within 1e-9 x scale and weights rtol 1e-7.
"""

import os

import numpy as np
import pytest

from particle_filters_amd import _native as NV
from tests import test_gpu_edh as TE
from tests import test_gpu_ledh as TL

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def replay_stream(cfg, Q, N, nx, flags):
    """The reference's draws after init_from_gaussian, in its order: noise every step, U on
    resample steps (NaN elsewhere: never read)."""
    T = len(flags)
    V = np.empty((T, N, nx))
    U = np.full(T, np.nan)
    for t in range(T):
        V[t] = cfg.rng.multivariate_normal(np.zeros(nx), Q, size=N)
        if flags[t]:
            U[t] = cfg.rng.random()
    return V, U


def check_run(pf, cfg, om, g, fused_expected=None):
    st = pf.init_from_gaussian(g["mean0"], g["cov0"])
    np.testing.assert_array_equal(st.particles, g["init_particles"])
    N, nx = g["init_particles"].shape
    flags = np.asarray(g["flags"], bool)
    V, U = replay_stream(cfg, om.Q, N, nx, flags)
    res = pf.run(st, g["Z"], process_noise="host", replay=(V, U))
    assert np.array_equal(res.flags, flags), f"decisions {res.flags.astype(int)} vs reference {flags.astype(int)}"
    scale = max(1.0, float(np.abs(g["means"]).max()))
    np.testing.assert_allclose(res.means, g["means"], rtol=0, atol=1e-9 * scale)
    cs = np.maximum(1.0, np.abs(g["covs"]).max(axis=(1, 2)))[:, None, None]
    assert np.all(np.abs(res.covs - g["covs"]) <= 1e-8 * cs)
    fin = pf.state
    np.testing.assert_allclose(fin.particles, g["particles"][-1], rtol=0, atol=1e-9 * scale)
    np.testing.assert_allclose(fin.weights, g["weights"][-1], rtol=1e-7, atol=1e-13)
    print(f"{g.get('name', '')}: T={len(flags)} N={N} resamples {int(flags.sum())}, max|dmean|/scale "
          f"{np.max(np.abs(res.means - g['means'])) / scale:.2e}")


@pytest.mark.parametrize("name", [n for n in TL.NAMES if n != "lin1d_nonoise"])
def test_ledh_run_replays_reference(name):
    pf, cfg, om, g = TL.make_filter(name)
    g = dict(g, name=f"LEDH {name} ({'fused step' if pf.shared_jacobian_path else 'kernel chain'})")
    check_run(pf, cfg, om, g)


@pytest.mark.parametrize("name", TE.NAMES)
def test_edh_run_replays_reference(name):
    pf, cfg, om, g = TE.make_filter(name)
    g = dict(g, name=f"EDH {name}")
    check_run(pf, cfg, om, g)


# ---------------------------------------------------------------------------------------------
# BASELINE config 5 at its benchmarked size: N = 1e4 particles (157 workgroups of the fused step:
# the cross-workgroup combine, the source-driven slot partition over CDF slices and the offspring-
# count moments), L = 8, Lorenz-96 d = 40, the reference's LEDH and EDH runs of
# tests/golden/flow_c5.npz (make_golden_flow_c5.py).  The fixture keeps the runs' outputs and a
# summary of every draw; the draws themselves are regenerated here from the seed with the same
# NumPy calls in the same order, and checked against that summary before they are replayed.
# ---------------------------------------------------------------------------------------------
C5 = np.load(os.path.join(os.path.dirname(__file__), "golden", "flow_c5.npz"))


def _c5_filter(algo):
    from particle_filters_amd import edh as ED, ledh as LD, models as M, trackers as TR
    from oracle import ledh_oracle as LO

    om = LO.lorenz96(40, q_std=0.1)
    gm, hm = M.L96Transition(8.0, 0.01, 40), M.SelectObservation(np.asarray(C5["H_idx"]), 40)
    ekf = TR.ExtendedKalmanFilter(om.g_ekf, om.h, om.Q, om.R, jac_g=om.jac_g, jac_h=om.jac_h)
    tracker = TR.EKFTracker(ekf, TR.EKFState(np.asarray(C5["mean0"], float).copy(),
                                             np.asarray(C5["cov0"], float).copy(), 0))
    N, L = int(C5["n_particles"]), int(C5["n_lambda"])
    args = (tracker, gm, hm, hm.jacobian, M.GaussianTransitionDensity(gm, om.Q), M.GaussianLikelihood(hm, om.R), om.R)
    if algo == "edh":
        cfg = ED.EDHConfig(n_particles=N, n_lambda_steps=L, resample_ess_ratio=float(C5["ratio"]), flow_integrator="rk4",
                           rng=np.random.default_rng(int(C5["seed"])))
        return ED.EDHFlowPF(*args, cfg, rng_mode="host"), cfg, om
    cfg = LD.LEDHConfig(n_particles=N, n_lambda_steps=L, resample_ess_ratio=float(C5["ratio"]),
                        rng=np.random.default_rng(int(C5["seed"])))
    return LD.LEDHFlowPF(*args, cfg, rng_mode="host"), cfg, om


def _summary_row(kind, a):
    a = np.asarray(a, float).reshape(-1)
    head = np.zeros(8)
    head[:min(8, a.size)] = a[:8]
    return np.concatenate([[kind, a.size, a.sum(), (a * a).sum()], head])


@pytest.mark.parametrize("algo", ["ledh", "edh"])
def test_config5_run_replays_reference(algo):
    pf, cfg, om = _c5_filter(algo)
    assert pf.shared_jacobian_path, "config 5 runs the fused shared-Jacobian step"
    N, nx = int(C5["n_particles"]), 40
    st = pf.init_from_gaussian(np.asarray(C5["mean0"], float), np.asarray(C5["cov0"], float))
    np.testing.assert_array_equal(np.asarray(st.particles)[:256], C5[f"{algo}__init_particles_head"])
    flags = np.asarray(C5[f"{algo}__flags"], bool)
    V, U = replay_stream(cfg, om.Q, N, nx, flags)
    # the regenerated stream is the reference's: every draw's size, sum, sum of squares, first values
    rows = [None]  # row 0: the initial draw (checked through the particles above)
    for t in range(len(flags)):
        rows.append(_summary_row(0.0, V[t]))
        if flags[t]:
            rows.append(_summary_row(1.0, U[t]))
    want = C5[f"{algo}__stream"]
    assert want.shape[0] == len(rows)
    np.testing.assert_array_equal(np.array(rows[1:]), want[1:])
    Z = np.asarray(C5["Z"], float)
    res = pf.run(st, Z, process_noise="host", replay=(V, U))
    assert np.array_equal(res.flags, flags), f"decisions {res.flags.astype(int)} vs reference {flags.astype(int)}"
    means, covs = C5[f"{algo}__means"], C5[f"{algo}__covs"]
    scale = max(1.0, float(np.abs(means).max()))
    dm = float(np.max(np.abs(res.means - means)))
    cs = np.maximum(1.0, np.abs(covs).max(axis=(1, 2)))[:, None, None]
    dc = float(np.max(np.abs(res.covs - covs) / cs))
    print(f"{algo.upper()} config 5 (N = {N}, L = {int(C5['n_lambda'])}, T = {len(flags)}, {int(flags.sum())} resamples): "
          f"max|dmean|/scale {dm / scale:.2e}, max|dcov|/scale {dc:.2e}")
    assert dm <= 1e-9 * scale
    assert dc <= 1e-8
    fin = pf.state
    np.testing.assert_allclose(np.asarray(fin.particles)[:256], C5[f"{algo}__final_particles_head"], rtol=0,
                               atol=1e-9 * scale)
    np.testing.assert_allclose(fin.weights, C5[f"{algo}__final_weights"], rtol=1e-7, atol=1e-13)
