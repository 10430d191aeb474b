"""The PF runs pinned by tests/golden/pf_runs.npz, described once.

``make_golden.py`` produced each run with the reference's ``ParticleFilter``;
the oracle test and the GPU parity tests rebuild the same inputs from here.
"""

from __future__ import annotations

import numpy as np

from oracle import ssm_oracle

SV_LOGSQ_P0 = 0.2 ** 2 / (1 - 0.95 ** 2)
LIN_A = np.array([[0.9, 0.2], [0.0, 0.7]])
LIN_H = np.array([[1.0, 0.5]])
LIN_Q = np.diag([0.05, 0.02])
LIN_R = np.array([[0.10]])

RUN_NAMES = ["sv_harness", "sv_logsq", "sv_logsq_reg", "sv_logsq_multi_reg", "sv_logsq_nb",
             "sv_it", "l96", "mat", "linear_sys", "linear_multi_reg"]


def build(name, sv, l96, mat, runs):
    """Return (ssm, Z, controls, kwargs) where kwargs hold Np, seed, mean0, cov0,
    method, reg, thresh, first_update_only."""
    X, Y = sv["X0"], sv["Y0"]
    kw = dict(method="systematic", reg=False, thresh=0.5, first_update_only=False)
    controls = None
    if name.startswith("sv_") and name not in ("sv_it", "sv_logsq_nb"):
        kw.update(Np=1000, seed=42, mean0=[X[0]], cov0=[[0.5]])
        if name == "sv_harness":
            ssm, Z = ssm_oracle.sv_harness(0.95, 0.2, 1.0), Y[1:, None]
        else:
            ssm, Z = ssm_oracle.sv_logsq(0.95, 0.2, 1.0), np.log(Y[1:] ** 2)[:, None]
            kw["reg"] = name != "sv_logsq"
            if name == "sv_logsq_multi_reg":
                kw["method"] = "multinomial"
    elif name == "sv_logsq_nb":
        ssm, Z = ssm_oracle.sv_logsq(0.95, 0.2, 1.0), np.log(Y[:300] ** 2)[:, None]
        kw.update(Np=1000, seed=7, mean0=[0.0], cov0=[[SV_LOGSQ_P0]], reg=True,
                  first_update_only=True)
    elif name == "sv_it":
        ssm, Z = ssm_oracle.sv_harness(0.9, 0.2, 1.0), sv["Y1"][1:, None]
        kw.update(Np=3000, seed=123, mean0=[sv["X1"][0]], cov0=[[0.3]], reg=True)
    elif name == "l96":
        ssm, Z = ssm_oracle.lorenz96(nx=40, q_std=0.1), l96["obs"][1:]
        kw.update(Np=500, seed=42, mean0=l96["ensemble"][0, 0], cov0=2.0 * np.eye(40))
    elif name == "mat":
        ssm, Z = ssm_oracle.mat_joint(mat["S"]), mat["Z"][1:11]
        kw.update(Np=500, seed=42, mean0=mat["X"][0].ravel(),
                  cov0=np.kron(np.eye(4), np.diag([100.0, 100.0, 1.0, 1.0])))
    elif name in ("linear_sys", "linear_multi_reg"):
        ssm = ssm_oracle.linear(LIN_A, LIN_H, LIN_Q, LIN_R)
        Z, controls = runs["lin_Z"], runs["lin_U"]
        kw.update(Np=1000, seed=42 if name == "linear_sys" else 43, mean0=[0.0, 0.0],
                  cov0=np.eye(2), thresh=0.9)
        if name == "linear_multi_reg":
            kw.update(method="multinomial", reg=True)
    else:
        raise KeyError(name)
    return ssm, np.asarray(Z, float), controls, kw


def golden(runs, name):
    keys = ["means", "covs", "ess", "neff", "flags", "final_particles", "final_weights",
            "init_particles", "t_final"]
    return {k: runs[f"{name}__{k}"] for k in keys}
