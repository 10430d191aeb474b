"""Restated simulators (particle_filters_amd.simulators) vs arrays the reference produced,
plus the reference's own property pins (tests/unit_tests/simulator/test_sv_*,
test_lorenz96_*, test_mat_*)."""

import numpy as np
import pytest

from particle_filters_amd import simulators as sim


def test_sv_bitwise_vs_reference(golden_sv):
    for k in range(int(golden_sv["nspecs"])):
        n, a, s, b, seed, x0 = golden_sv[f"spec{k}"]
        r = sim.simulate_sv_1d(int(n), a, s, b, seed=int(seed), x0=None if np.isnan(x0) else x0)
        assert np.array_equal(r.X, golden_sv[f"X{k}"]), k
        assert np.array_equal(r.Y, golden_sv[f"Y{k}"]), k


@pytest.mark.parametrize("bad,match", [
    (dict(n=0), "n must be positive"), (dict(n=-3), "n must be positive"),
    (dict(alpha=1.0), "alpha.*< 1"), (dict(alpha=np.nan), "alpha.*< 1"),
    (dict(sigma=-0.1), "sigma.*nonnegative"), (dict(beta=-1.0), "beta.*nonnegative"),
])
def test_sv_validation(bad, match):
    args = dict(n=10, alpha=0.9, sigma=0.2, beta=1.0)
    args.update(bad)
    with pytest.raises(ValueError, match=match):
        sim.simulate_sv_1d(args["n"], args["alpha"], args["sigma"], args["beta"], seed=0)


def test_sv_sigma_zero_closed_form():
    r = sim.simulate_sv_1d(30, 0.8, 0.0, 1.0, seed=1, x0=2.0)
    np.testing.assert_allclose(r.X, 2.0 * 0.8 ** np.arange(30), rtol=1e-12)


def test_sv_stationary_stats():
    r = sim.simulate_sv_1d(200000, 0.9, 0.3, 1.0, seed=5)
    assert np.var(r.X) == pytest.approx(0.09 / (1 - 0.81), rel=0.05)
    x = r.X - r.X.mean()
    assert np.dot(x[1:], x[:-1]) / np.dot(x, x) == pytest.approx(0.9, abs=0.01)


def test_sv_save_roundtrip(tmp_path):
    r = sim.simulate_sv_1d(20, 0.9, 0.2, 1.0, seed=3)
    r.save(str(tmp_path / "sv.npz"))
    d = np.load(tmp_path / "sv.npz")
    assert np.array_equal(d["X"], r.X) and float(d["alpha"]) == 0.9


def test_l96_bitwise_vs_reference(golden_l96):
    g = golden_l96
    r = sim.simulate_lorenz96(nx=40, F=8.0, dt=0.01, spinup_steps=1000, total_steps=15, Np=3,
                              obs_interval=1, obs_fraction=4, obs_error_std=1.0, seed=42)
    for a, b in [("truth_traj", "truth"), ("ensemble_traj", "ensemble"), ("observations", "obs"),
                 ("obs_times", "obs_times"), ("H_idx", "H_idx"), ("R", "R")]:
        assert np.array_equal(getattr(r, a), g[b]), a
    r2 = sim.simulate_lorenz96(nx=12, F=6.0, dt=0.02, spinup_steps=50, total_steps=20, Np=2,
                               obs_interval=5, obs_fraction=3, obs_error_std=0.5,
                               perturbation_std=0.3, seed=5)
    assert np.array_equal(r2.truth_traj, g["truth2"])
    assert np.array_equal(r2.observations, g["obs2"])
    assert np.array_equal(r2.ensemble_traj, g["ensemble2"])
    rhs = np.stack([sim.l96_rhs(x, 8.0) for x in g["rhs_in"]])
    rk4 = np.stack([sim.rk4_step(x, 0.01, lambda z: sim.l96_rhs(z, 8.0)) for x in g["rhs_in"]])
    assert np.array_equal(rhs, g["rhs_out"]) and np.array_equal(rk4, g["rk4_out"])


def test_l96_forcing_shift_and_periodicity():
    """test_lorenz96_dynamics.py:24-52: +1 on F shifts the RHS by exactly +1... per unit."""
    x = np.random.default_rng(0).normal(size=40)
    np.testing.assert_allclose(sim.l96_rhs(x, 10.0) - sim.l96_rhs(x, 8.0), 2.0, atol=1e-12)
    np.testing.assert_allclose(np.roll(sim.l96_rhs(x, 8.0), 3), sim.l96_rhs(np.roll(x, 3), 8.0),
                               atol=1e-12)


def test_l96_invalid_x0():
    with pytest.raises(ValueError, match="x0 must have shape"):
        sim.simulate_lorenz96(nx=10, x0=np.zeros(9), total_steps=2, spinup_steps=1)


def test_l96_io_roundtrip(tmp_path):
    r = sim.simulate_lorenz96(nx=8, spinup_steps=5, total_steps=6, Np=2, obs_interval=2, seed=1)
    p = tmp_path / "l96.npz"
    r.save(str(p))
    with pytest.raises(FileExistsError):
        r.save(str(p))
    r2 = sim.Lorenz96SimulationResult.load(str(p))
    assert np.array_equal(r2.truth_traj, r.truth_traj) and r2.config == r.config


def test_mat_bitwise_vs_reference(golden_mat):
    g = golden_mat
    d = sim.simulate_acoustic_dataset(sim.ScenarioConfig(n_targets=4, n_steps=40, seed=56),
                                      sim.DynamicsConfig(dt=1.0))
    for k in ("X", "P", "S", "Z", "meta"):
        assert np.array_equal(d[k], g[k]), k
    cfg2 = sim.ScenarioConfig(n_targets=3, n_steps=25, area_xy=(30.0, 20.0), sensor_grid_shape=(3, 4),
                              psi=5.0, d0=0.2, seed=7, use_article_init=False)
    d2 = sim.simulate_acoustic_dataset(cfg2, sim.DynamicsConfig(dt=0.5))
    for k in ("X", "P", "S", "Z", "meta"):
        assert np.array_equal(d2[k], g[k + "2"]), k


def test_mat_vectorized_matches_naive():
    """test_mat_measurement.py:29-51."""
    rng = np.random.default_rng(3)
    P = rng.uniform(0, 40, size=(7, 4, 2))
    S = sim.make_sensor_grid((40.0, 40.0), (5, 5))
    Z = sim.acoustic_measurement_model(P, S, 10.0, 0.1)
    naive = np.zeros((7, 25))
    for t in range(7):
        for s in range(25):
            naive[t, s] = sum(10.0 / (np.sum((P[t, c] - S[s]) ** 2) + 0.1) for c in range(4))
    np.testing.assert_allclose(Z, naive, rtol=1e-12)


def test_mat_article_init_requires_four():
    with pytest.raises(ValueError):
        sim.article_initial_states(3)
