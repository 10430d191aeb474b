#!/usr/bin/env python
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports ``/root/reference`` (models/particle_filter.py and simulator/*),
runs the reference's own ``ParticleFilter`` and simulators on fixed seeds and
stores inputs + outputs as small ``.npz`` data files.  Nothing from the
reference's source is stored — only numbers it produced.

Instrumentation: the reference ``ParticleFilter`` is subclassed here only to
*observe* ``_resample`` (pre-resample Neff and whether it fired); the call is
forwarded unchanged to the reference implementation.
"""

from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
REF = os.environ.get("PF_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from models.particle_filter import ParticleFilter  # noqa: E402  (reference)
from simulator.simulator_sto_volatility_model import simulate_sv_1d  # noqa: E402
from simulator import simulator_Lorenz_96 as ref_l96  # noqa: E402
from simulator import simulator_Multi_acoustic_tracking as ref_mat  # noqa: E402

from oracle.pf_oracle import RecordingRNG  # noqa: E402
from oracle import ssm_oracle  # noqa: E402


class ObservedPF(ParticleFilter):
    """Reference ParticleFilter with read-only observation of _resample."""

    def _resample(self, particles, weights):
        self.last_neff = float(1.0 / np.sum(weights ** 2))
        self.last_resampled = bool(self.last_neff < self.resample_thresh * self.Np)
        return super()._resample(particles, weights)


def run_ref(ssm, Z, *, Np, seed, mean0, cov0, method="systematic", reg=False, thresh=0.5,
            first_update_only=False, controls=None):
    pf = ObservedPF(ssm.g, ssm.h, ssm.Q, ssm.R, Np=Np, resample_thresh=thresh,
                    resample_method=method, regularize_after_resample=reg,
                    rng=np.random.default_rng(seed))
    pf.initialize(np.asarray(mean0, float), np.asarray(cov0, float))
    init_particles = pf.state.particles.copy()
    T = Z.shape[0]
    out = dict(means=np.zeros((T, pf.nx)), covs=np.zeros((T, pf.nx, pf.nx)), ess=np.zeros(T),
               neff=np.zeros(T), flags=np.zeros(T, dtype=bool))
    for t in range(T):
        z = np.atleast_1d(Z[t])
        u = None if controls is None else controls[t]
        st = pf.update(z) if (first_update_only and t == 0) else pf.step(z, u)
        out["means"][t] = st.mean
        out["covs"][t] = st.cov
        out["ess"][t] = pf.effective_sample_size()
        out["neff"][t] = pf.last_neff
        out["flags"][t] = pf.last_resampled
    out["final_particles"] = pf.state.particles.copy()
    out["final_weights"] = pf.state.weights.copy()
    out["init_particles"] = init_particles
    out["t_final"] = pf.state.t
    return out


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


def gen_sv():
    cases = {}
    specs = [  # (n, alpha, sigma, beta, seed, x0)
        (1000, 0.95, 0.2, 1.0, 42, None),   # BASELINE config 1/2 data
        (200, 0.9, 0.2, 1.0, 42, None),     # integration-test data
        (64, 0.5, 0.0, 2.0, 3, 1.5),        # sigma = 0 closed form x0*alpha^t
        (1, 0.3, 0.7, 0.5, 11, None),       # n = 1 edge
        (2000, 0.91, 1.0, 0.5, 7, None),    # notebook-like parameters
    ]
    for k, (n, a, s, b, seed, x0) in enumerate(specs):
        r = simulate_sv_1d(n, a, s, b, seed=seed, x0=x0)
        cases[f"X{k}"] = r.X
        cases[f"Y{k}"] = r.Y
        cases[f"spec{k}"] = np.array([n, a, s, b, seed, np.nan if x0 is None else x0])
    cases["nspecs"] = np.array(len(specs))
    save("sv_data", **cases)
    return simulate_sv_1d(1000, 0.95, 0.2, 1.0, seed=42), simulate_sv_1d(200, 0.9, 0.2, 1.0, seed=42)


def gen_l96():
    res = ref_l96.simulate_lorenz96(nx=40, F=8.0, dt=0.01, spinup_steps=1000, total_steps=15, Np=3,
                                    obs_interval=1, obs_fraction=4, obs_error_std=1.0, seed=42)
    res2 = ref_l96.simulate_lorenz96(nx=12, F=6.0, dt=0.02, spinup_steps=50, total_steps=20, Np=2,
                                     obs_interval=5, obs_fraction=3, obs_error_std=0.5,
                                     perturbation_std=0.3, seed=5)
    rng = np.random.default_rng(0)
    xr = rng.normal(size=(5, 40)) * 3 + 8
    rhs = np.stack([ref_l96.l96_rhs(x, 8.0) for x in xr])
    rk4 = np.stack([ref_l96.rk4_step(x, 0.01, lambda z: ref_l96.l96_rhs(z, 8.0)) for x in xr])
    save("l96_data", truth=res.truth_traj, ensemble=res.ensemble_traj, obs=res.observations,
         obs_times=res.obs_times, H_idx=res.H_idx, R=res.R,
         truth2=res2.truth_traj, ensemble2=res2.ensemble_traj, obs2=res2.observations,
         obs_times2=res2.obs_times, H_idx2=res2.H_idx, R2=res2.R,
         rhs_in=xr, rhs_out=rhs, rk4_out=rk4)
    return res


def gen_mat():
    cfg = ref_mat.ScenarioConfig(n_targets=4, n_steps=40, area_xy=(40.0, 40.0),
                                 sensor_grid_shape=(5, 5), psi=10.0, d0=0.1, seed=56,
                                 use_article_init=True)
    d = ref_mat.simulate_acoustic_dataset(cfg, ref_mat.DynamicsConfig(dt=1.0))
    cfg2 = ref_mat.ScenarioConfig(n_targets=3, n_steps=25, area_xy=(30.0, 20.0),
                                  sensor_grid_shape=(3, 4), psi=5.0, d0=0.2, seed=7,
                                  use_article_init=False)
    d2 = ref_mat.simulate_acoustic_dataset(cfg2, ref_mat.DynamicsConfig(dt=0.5))
    save("mat_data", X=d["X"], P=d["P"], S=d["S"], Z=d["Z"], meta=d["meta"],
         X2=d2["X"], P2=d2["P"], S2=d2["S"], Z2=d2["Z"], meta2=d2["meta"])
    return d


def gen_resample():
    """Reference _systematic_resample / _multinomial_resample on fixed weights."""
    out = {}
    dummy = ssm_oracle.sv_harness(0.9, 0.2, 1.0)
    rng_w = np.random.default_rng(2024)
    wsets = {
        "rand1000": rng_w.random(1000),
        "one": np.ones(1),
        "ragged7": rng_w.random(7),
        "onehot": np.eye(1, 513, 200).ravel() + 0.0,
        "uniform": np.ones(4096),
        "sparse": np.where(rng_w.random(3000) < 0.01, rng_w.random(3000), 0.0),
        "skewed": np.exp(-0.5 * (rng_w.normal(size=5000) * 6) ** 2),
        "dominant": np.r_[0.9, np.full(999, 0.1 / 999)],
    }
    for k, (name, w) in enumerate(wsets.items()):
        w = np.asarray(w, float)
        w = w / np.sum(w)
        # systematic: record the single U drawn by the reference (pf.py:160)
        rec = RecordingRNG(np.random.default_rng(100 + k))
        pf = ParticleFilter(dummy.g, dummy.h, dummy.Q, dummy.R, Np=len(w), rng=rec)
        idx_s = pf._systematic_resample(w)
        U = rec.log[0][1]
        # multinomial: the REAL Generator.choice path of the reference (pf.py:186)
        pf2 = ParticleFilter(dummy.g, dummy.h, dummy.Q, dummy.R, Np=len(w),
                             rng=np.random.default_rng(200 + k))
        idx_m = pf2._multinomial_resample(w)
        u_m = np.random.default_rng(200 + k).random(len(w))  # the uniforms choice() consumed
        out[f"{name}_w"] = w
        out[f"{name}_U"] = np.array(U)
        out[f"{name}_sys"] = idx_s.astype(np.int64)
        out[f"{name}_u"] = u_m
        out[f"{name}_multi"] = np.asarray(idx_m, np.int64)
    out["names"] = np.array(list(wsets.keys()))
    save("resample_idx", **out)


def gen_pf_runs(sv_c1, sv_it, l96, mat):
    runs = {}
    X, Y = sv_c1.X, sv_c1.Y
    Zh = Y[1:, None]
    Zl = np.log(Y[1:] ** 2)[:, None]
    base = dict(Np=1000, seed=42, mean0=[X[0]], cov0=[[0.5]])
    runs["sv_harness"] = run_ref(ssm_oracle.sv_harness(0.95, 0.2, 1.0), Zh, **base)
    runs["sv_logsq"] = run_ref(ssm_oracle.sv_logsq(0.95, 0.2, 1.0), Zl, **base)
    runs["sv_logsq_reg"] = run_ref(ssm_oracle.sv_logsq(0.95, 0.2, 1.0), Zl, reg=True, **base)
    runs["sv_logsq_multi_reg"] = run_ref(ssm_oracle.sv_logsq(0.95, 0.2, 1.0), Zl, reg=True,
                                         method="multinomial", **base)
    # notebook driver: update(Z[0]) first, then predict+update (PF_VS_experiments.ipynb cell 7)
    runs["sv_logsq_nb"] = run_ref(ssm_oracle.sv_logsq(0.95, 0.2, 1.0), np.log(Y[:300] ** 2)[:, None],
                                  Np=1000, seed=7, mean0=[0.0], cov0=[[0.2 ** 2 / (1 - 0.95 ** 2)]],
                                  reg=True, first_update_only=True)
    # integration test (test_pf_vs_simulator_sv.py:99-148)
    runs["sv_it"] = run_ref(ssm_oracle.sv_harness(0.9, 0.2, 1.0), sv_it.Y[1:, None], Np=3000,
                            seed=123, mean0=[sv_it.X[0]], cov0=[[0.3]], reg=True)
    # Lorenz-96 d=40, short run
    l96m = ssm_oracle.lorenz96(nx=40, q_std=0.1)
    # plugins from the reference simulator itself (simulator_Lorenz_96.py:35-84, 147-161)
    obs_model = ref_l96.ObsModel(H_idx=l96.H_idx, R=l96.R)
    l96m.g = lambda x, u: ref_l96.rk4_step(x, 0.01, lambda z: ref_l96.l96_rhs(z, 8.0))
    l96m.h = obs_model.H
    runs["l96"] = run_ref(l96m, l96.observations[1:], Np=500, seed=42,
                          mean0=l96.ensemble_traj[0, 0], cov0=2.0 * np.eye(40))
    # MAT joint 16-D, short run
    matm = ssm_oracle.mat_joint(mat["S"])
    P0 = np.kron(np.eye(4), np.diag([100.0, 100.0, 1.0, 1.0]))
    runs["mat"] = run_ref(matm, mat["Z"][1:11], Np=500, seed=42, mean0=mat["X"][0].ravel(), cov0=P0)
    # linear 2-D system (test_pf_shapes_and_api.py:8-23), controls on, both methods
    A = np.array([[0.9, 0.2], [0.0, 0.7]])
    H = np.array([[1.0, 0.5]])
    lin = ssm_oracle.linear(A, H, np.diag([0.05, 0.02]), np.array([[0.10]]))
    Zlin = np.random.default_rng(123).normal(size=(12, 1))
    U = np.random.default_rng(321).normal(size=(12, 2)) * 0.1
    runs["linear_sys"] = run_ref(lin, Zlin, Np=1000, seed=42, mean0=[0.0, 0.0], cov0=np.eye(2),
                                 controls=U, thresh=0.9)
    runs["linear_multi_reg"] = run_ref(lin, Zlin, Np=1000, seed=43, mean0=[0.0, 0.0],
                                       cov0=np.eye(2), controls=U, thresh=0.9,
                                       method="multinomial", reg=True)
    flat = {}
    for name, r in runs.items():
        for k, v in r.items():
            flat[f"{name}__{k}"] = np.asarray(v)
    flat["lin_Z"] = Zlin
    flat["lin_U"] = U
    save("pf_runs", **flat)
    for name, r in runs.items():
        print(f"  {name}: resample rate {np.mean(r['flags']):.3f}")


def main():
    sv_c1, sv_it = gen_sv()
    l96 = gen_l96()
    mat = gen_mat()
    gen_resample()
    gen_pf_runs(sv_c1, sv_it, l96, mat)


if __name__ == "__main__":
    main()
