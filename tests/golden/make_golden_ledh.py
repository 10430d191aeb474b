#!/usr/bin/env python
"""Generate tests/golden/ledh_runs.npz by running the REFERENCE LEDH filter itself.

Build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ledh.py

Imports /root/reference's ``models.LEDH_particle_filter.LEDHFlowPF`` and
``models.extended_kalman_filter.ExtendedKalmanFilter``, drives them the way the
reference's own tests do (EKF tracker behind the GaussianTracker protocol,
``process_noise_sampler = cfg.rng.multivariate_normal(0, Q, N)``), and stores the
inputs, every random draw the filter consumed (so the HIP engine's host-replay
mode can be fed the identical stream) and the per-step outputs.  Only numbers
are stored.  The plugin wirings (g, h, Jacobian, log densities) are the
restatements in oracle/ledh_oracle.py of the reference tests' closures.
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

from models.LEDH_particle_filter import LEDHFlowPF, LEDHConfig  # noqa: E402  (reference)
from models.extended_kalman_filter import ExtendedKalmanFilter, EKFState  # noqa: E402  (reference)

from oracle import ledh_oracle as LO  # noqa: E402


class RecordingGenerator:
    """Forwards to a numpy Generator and logs what multivariate_normal / random returned."""

    def __init__(self, gen):
        self.gen = gen
        self.log = []

    def multivariate_normal(self, mean, cov, size=None):
        out = self.gen.multivariate_normal(mean, cov, size=size)
        self.log.append(("mvn", np.array(out)))
        return out

    def random(self, size=None):
        out = self.gen.random(size)
        self.log.append(("random", np.array(out)))
        return out


class Tracker:
    """EKF behind the GaussianTracker protocol (ledh.py:13-16), as the reference tests wrap it."""

    def __init__(self, ekf, st):
        self.ekf, self.state, self.past_mean = ekf, st, st.mean.copy()

    def predict(self):
        self.past_mean = self.state.mean.copy()
        self.state = self.ekf.predict(self.state, u=None)
        return self.state.mean, self.state.cov

    def update(self, z):
        self.state = self.ekf.update(self.state, z)
        return self.state.mean, self.state.cov

    def get_past_mean(self):
        return self.past_mean


def run_ref(model: LO.LEDHModel, Z, *, mean0, cov0, n_particles, n_lambda, ratio, seed, noise=True):
    rec = RecordingGenerator(np.random.default_rng(seed))
    ekf = ExtendedKalmanFilter(g=model.g_ekf, h=model.h, Q=model.Q, R=model.R, jac_g=model.jac_g,
                               jac_h=model.jac_h)
    tracker = Tracker(ekf, EKFState(mean=np.asarray(mean0, float).copy(), cov=np.asarray(cov0, float).copy(), t=0))
    cfg = LEDHConfig(n_particles=n_particles, n_lambda_steps=n_lambda, resample_ess_ratio=ratio, rng=rec)
    pf = LEDHFlowPF(tracker=tracker, g=model.g, h=model.h, jacobian_h=model.jac_h,
                    log_trans_pdf=model.log_trans, log_like_pdf=model.log_like, R=model.R, config=cfg)
    st = pf.init_from_gaussian(np.asarray(mean0, float), np.asarray(cov0, float))
    out = {"init_particles": st.particles.copy(), "init_mean": st.mean.copy(), "init_cov": st.cov.copy()}
    sampler = (lambda N, nx: rec.multivariate_normal(np.zeros(nx), model.Q, size=N)) if noise else None
    T = len(Z)
    nx = model.nx
    out.update(means=np.zeros((T, nx)), covs=np.zeros((T, nx, nx)), weights=np.zeros((T, n_particles)),
               particles=np.zeros((T, n_particles, nx)), conds=np.zeros((T, max(1, n_lambda))),
               tracker_P=np.zeros((T, nx, nx)))
    for t in range(T):
        st = pf.step(st, np.atleast_1d(Z[t]), process_noise_sampler=sampler)
        out["means"][t] = st.mean
        out["covs"][t] = st.cov
        out["weights"][t] = st.weights
        out["particles"][t] = st.particles
        out["conds"][t] = st.diagnostics["condition_numbers"]
    # the random stream: init draw, then per step [noise draw], [resample uniform]
    mvn = [a for k, a in rec.log if k == "mvn"]
    out["rng_init"] = mvn[0]
    out["rng_noise"] = np.stack(mvn[1:]) if noise else np.zeros((0, n_particles, nx))
    unif = [float(a) for k, a in rec.log if k == "random"]
    out["rng_unif"] = np.array(unif)
    out["flags"] = np.all(out["weights"] == 1.0 / n_particles, axis=1)
    # the tracker's predicted covariances as the flow saw them (replayed through a twin EKF)
    twin = Tracker(ExtendedKalmanFilter(g=model.g_ekf, h=model.h, Q=model.Q, R=model.R, jac_g=model.jac_g,
                                        jac_h=model.jac_h),
                   EKFState(mean=np.asarray(mean0, float).copy(), cov=np.asarray(cov0, float).copy(), t=0))
    for t in range(T):
        _, P = twin.predict()
        out["tracker_P"][t] = 0.5 * (P + P.T)
        twin.update(np.atleast_1d(Z[t]))
    return out


def main():
    runs = {}
    # 1-D linear system of the reference unit tests (test_ledh_flow_pf.py:62-126)
    rng = np.random.default_rng(5)
    Zlin = 0.6 + 0.3 * rng.standard_normal(12)
    runs["lin1d"] = dict(model=LO.linear_1d(), Z=Zlin[:, None], mean0=[0.5], cov0=[[0.3]], n_particles=100,
                         n_lambda=4, ratio=0.5, seed=123)
    runs["lin1d_nonoise"] = dict(model=LO.linear_1d(), Z=Zlin[:5, None], mean0=[0.5], cov0=[[0.3]],
                                 n_particles=50, n_lambda=8, ratio=0.0, seed=7, noise=False)
    # 1-D SV, nonlinear h = beta exp(x/2): per-particle Jacobians
    sv = np.load(os.path.join(HERE, "sv_data.npz"))
    runs["sv_exp"] = dict(model=LO.sv_exp_half(0.95, 0.2, 1.0, 0.1), Z=sv["Y0"][1:21, None], mean0=[sv["X0"][0]],
                          cov0=[[0.5]], n_particles=200, n_lambda=8, ratio=0.5, seed=42)
    # per-target acoustic tracking (test_filters_mat_simulator.py:120-176), 3x3 sensor grid
    mat = np.load(os.path.join(HERE, "mat_data.npz"))
    S2 = mat["S2"]
    runs["acoustic"] = dict(model=LO.acoustic_single(S2, psi=float(mat["meta2"][2]), d0=float(mat["meta2"][3])),
                            Z=mat["Z2"][1:7], mean0=mat["X2"][0, 0], cov0=np.diag([100.0, 100.0, 1.0, 1.0]),
                            n_particles=100, n_lambda=3, ratio=0.5, seed=100)
    # joint 4-target acoustic tracking, 16-D state, 5x5 sensors (the MAT notebook's h_joint wiring, the
    # reference's only published LEDH run: PF_PF_results_reproduction_multi_target_acoustic_tracking.ipynb)
    from simulator.simulator_Multi_acoustic_tracking import article_process_noise_cov  # reference
    Xj = mat["X"]
    m0 = Xj[0].reshape(-1) + np.tile([1.5, -1.0, 0.1, -0.1], Xj.shape[1])
    runs["mat_joint"] = dict(model=LO.acoustic_joint(mat["S"], psi=float(mat["meta"][2]), d0=float(mat["meta"][3]),
                                                     n_targets=Xj.shape[1], Q_single=article_process_noise_cov()),
                             Z=mat["Z"][1:5], mean0=m0, cov0=np.kron(np.eye(Xj.shape[1]), np.diag([100.0, 100.0, 1.0, 1.0])),
                             n_particles=96, n_lambda=8, ratio=0.5, seed=56)
    # Lorenz-96 d=40 (BASELINE config 5 wiring), short
    l96 = np.load(os.path.join(HERE, "l96_data.npz"))
    runs["l96"] = dict(model=LO.lorenz96(40), Z=l96["obs"][1:5], mean0=l96["ensemble"][0, 0], cov0=2.0 * np.eye(40),
                       n_particles=64, n_lambda=8, ratio=0.5, seed=42)
    arrays = {}
    for name, spec in runs.items():
        model = spec.pop("model")
        Z = np.asarray(spec.pop("Z"), float)
        out = run_ref(model, Z, **spec)
        # the oracle must reproduce the reference (fp64 rounding level)
        for vec in (True, False):
            o = LO.run_ledh(model, Z, mean0=spec["mean0"], cov0=spec["cov0"], n_particles=spec["n_particles"],
                            n_lambda_steps=spec["n_lambda"], ratio=spec["ratio"], seed=spec["seed"],
                            noise=spec.get("noise", True), vectorized=vec)
            err = np.max(np.abs(o["means"] - out["means"]))
            print(f"  oracle(vectorized={vec}) vs reference {name}: max|dmean| = {err:.3e}")
        arrays[f"{name}__Z"] = Z
        for k, v in spec.items():
            arrays[f"{name}__{k}"] = np.asarray(v)
        for k, v in out.items():
            arrays[f"{name}__{k}"] = np.asarray(v)
    arrays["names"] = np.array(list(runs.keys()))
    path = os.path.join(HERE, "ledh_runs.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


if __name__ == "__main__":
    main()
