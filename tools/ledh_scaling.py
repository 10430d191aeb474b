"""LEDH/EDH config-5 job at one N (for per-kernel scaling under rocprofv3).
usage: python tools/ledh_scaling.py N [ledh|edh]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particle_filters_amd import edh as ED, ledh as LD, models as M, simulators as S, trackers as TR  # noqa: E402

Np = int(sys.argv[1])
algo = sys.argv[2] if len(sys.argv) > 2 else "ledh"
sim = S.simulate_lorenz96(nx=40, F=8.0, dt=0.01, spinup_steps=1000, total_steps=120, Np=1, obs_interval=1,
                          obs_fraction=4, obs_error_std=1.0, seed=42)
g, h = M.L96Transition(8.0, 0.01, 40), M.SelectObservation(sim.H_idx, 40)
Q, R = 0.1 ** 2 * np.eye(40), sim.R
m0, c0 = sim.ensemble_traj[0, 0], 2.0 * np.eye(40)
ekf = TR.ExtendedKalmanFilter(g, h, Q, R, jac_g=g.jacobian, jac_h=h.jacobian)
tr = TR.EKFTracker(ekf, TR.EKFState(m0.copy(), c0.copy(), 0))
args = (tr, g, h, h.jacobian, M.GaussianTransitionDensity(g, Q), M.GaussianLikelihood(h, R), R)
if algo == "edh":
    pf = ED.EDHFlowPF(*args, ED.EDHConfig(n_particles=Np, n_lambda_steps=8, resample_ess_ratio=0.5,
                                          rng=np.random.default_rng(1)), rng_mode="device")
else:
    pf = LD.LEDHFlowPF(*args, LD.LEDHConfig(n_particles=Np, n_lambda_steps=8, resample_ess_ratio=0.5,
                                            rng=np.random.default_rng(1)), rng_mode="device")
st = pf.init_from_gaussian(m0, c0)
res = pf.run(st, sim.observations[1:101], tracker="device")
print(Np, algo, "resample rate", res.flags.mean())
