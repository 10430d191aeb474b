#!/usr/bin/env python
"""Generate tests/golden/edh_runs.npz by running the REFERENCE EDH filter itself.

Build container only:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_edh.py

Imports /root/reference's ``models.EDH_particle_filter.EDHFlowPF`` and its EKF, drives them
like the reference tests (test_filters_mat_simulator.py:155-186: EKF tracker, process noise
``cfg.rng.multivariate_normal(0, Q, N)``) and stores inputs, the random stream it consumed and
the per-step outputs.  Only numbers are stored; the plugin wirings are oracle/ledh_oracle.py's.
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
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from models.EDH_particle_filter import EDHFlowPF, EDHConfig  # noqa: E402  (reference)
from models.extended_kalman_filter import ExtendedKalmanFilter, EKFState  # noqa: E402  (reference)

from oracle import ledh_oracle as LO, edh_oracle as EO  # noqa: E402
from make_golden_ledh import RecordingGenerator, Tracker  # noqa: E402


def run_ref(model, Z, *, mean0, cov0, n_particles, n_lambda, ratio, seed, integrator, noise=True):
    rec = RecordingGenerator(np.random.default_rng(seed))
    ekf = ExtendedKalmanFilter(g=model.g_ekf, h=model.h, Q=model.Q, R=model.R, jac_g=model.jac_g, jac_h=model.jac_h)
    tracker = Tracker(ekf, EKFState(mean=np.asarray(mean0, float).copy(), cov=np.asarray(cov0, float).copy(), t=0))
    cfg = EDHConfig(n_particles=n_particles, n_lambda_steps=n_lambda, resample_ess_ratio=ratio,
                    flow_integrator=integrator, rng=rec)
    pf = EDHFlowPF(tracker=tracker, g=model.g, h=model.h, jacobian_h=model.jac_h, log_trans_pdf=model.log_trans,
                   log_like_pdf=model.log_like, R=model.R, config=cfg)
    st = pf.init_from_gaussian(np.asarray(mean0, float), np.asarray(cov0, float))
    out = {"init_particles": st.particles.copy(), "init_mean": st.mean.copy(), "init_cov": st.cov.copy()}
    sampler = (lambda N, nx: rec.multivariate_normal(np.zeros(nx), model.Q, size=N)) if noise else None
    T, nx = len(Z), model.nx
    out.update(means=np.zeros((T, nx)), covs=np.zeros((T, nx, nx)), weights=np.zeros((T, n_particles)),
               particles=np.zeros((T, n_particles, nx)), conds=np.zeros((T, max(1, n_lambda))))
    for t in range(T):
        st = pf.step(st, np.atleast_1d(Z[t]), process_noise_sampler=sampler)
        out["means"][t] = st.mean
        out["covs"][t] = st.cov
        out["weights"][t] = st.weights
        out["particles"][t] = st.particles
        out["conds"][t] = st.diagnostics["condition_numbers"]
    out["flags"] = np.all(out["weights"] == 1.0 / n_particles, axis=1)
    return out


def main():
    rng = np.random.default_rng(5)
    Zlin = 0.6 + 0.3 * rng.standard_normal(12)
    sv = np.load(os.path.join(HERE, "sv_data.npz"))
    mat = np.load(os.path.join(HERE, "mat_data.npz"))
    l96 = np.load(os.path.join(HERE, "l96_data.npz"))
    psi, d0 = float(mat["meta2"][2]), float(mat["meta2"][3])
    runs = {
        "lin1d_rk4": dict(model=LO.linear_1d(), Z=Zlin[:, None], mean0=[0.5], cov0=[[0.3]], n_particles=100,
                          n_lambda=4, ratio=0.5, seed=123, integrator="rk4"),
        "lin1d_euler": dict(model=LO.linear_1d(), Z=Zlin[:, None], mean0=[0.5], cov0=[[0.3]], n_particles=100,
                            n_lambda=4, ratio=0.5, seed=124, integrator="euler"),
        "sv_exp": dict(model=LO.sv_exp_half(0.95, 0.2, 1.0, 0.1), Z=sv["Y0"][1:21, None], mean0=[sv["X0"][0]],
                       cov0=[[0.5]], n_particles=200, n_lambda=8, ratio=0.5, seed=42, integrator="rk4"),
        "acoustic": dict(model=LO.acoustic_single(mat["S2"], psi=psi, d0=d0), Z=mat["Z2"][1:7], mean0=mat["X2"][0, 0],
                         cov0=np.diag([100.0, 100.0, 1.0, 1.0]), n_particles=100, n_lambda=3, ratio=0.5, seed=200,
                         integrator="rk4"),
        "l96_rk4": dict(model=LO.lorenz96(40), Z=l96["obs"][1:5], mean0=l96["ensemble"][0, 0], cov0=2.0 * np.eye(40),
                        n_particles=64, n_lambda=8, ratio=0.5, seed=42, integrator="rk4"),
        "l96_euler": dict(model=LO.lorenz96(40), Z=l96["obs"][1:5], mean0=l96["ensemble"][0, 0],
                          cov0=2.0 * np.eye(40), n_particles=64, n_lambda=8, ratio=0.0, seed=43, integrator="euler"),
    }
    arrays = {}
    for name, spec in runs.items():
        model = spec.pop("model")
        Z = np.asarray(spec.pop("Z"), float)
        out = run_ref(model, Z, **spec)
        for vec in (True, False):
            o = EO.run_edh(model, Z, mean0=spec["mean0"], cov0=spec["cov0"], n_particles=spec["n_particles"],
                           n_lambda_steps=spec["n_lambda"], ratio=spec["ratio"], seed=spec["seed"],
                           integrator=spec["integrator"], vectorized=vec)
            print(f"  oracle(vectorized={vec}) vs reference {name}: max|dmean| = "
                  f"{np.max(np.abs(o['means'] - out['means'])):.3e}")
        arrays[f"{name}__Z"] = Z
        for k, v in spec.items():
            arrays[f"{name}__{k}"] = np.asarray(v)
        for k, v in out.items():
            arrays[f"{name}__{k}"] = np.asarray(v)
    arrays["names"] = np.array(list(runs.keys()))
    path = os.path.join(HERE, "edh_runs.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


if __name__ == "__main__":
    main()
