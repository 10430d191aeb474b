"""Device-RNG L96 / MAT SIR runs (fp32, fp64) vs the vectorised NumPy oracle: RMSE vs truth."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particle_filters_amd import models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch
from oracle import pf_oracle, ssm_oracle

T = int(sys.argv[1]) if len(sys.argv) > 1 else 100
N = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
sim = S.simulate_lorenz96(nx=40, F=8.0, dt=0.01, spinup_steps=1000, total_steps=T, Np=1, obs_interval=1,
                          obs_fraction=4, obs_error_std=1.0, seed=42)
Z, X = sim.observations[1:], sim.truth_traj[1:]
g, h = M.L96Transition(8.0, 0.01, 40), M.SelectObservation(sim.H_idx, 40)
Q = 0.01 * np.eye(40)
for prec in ("fp32", "fp64"):
    pf = ParticleFilterBatch(g, h, Q, sim.R, Np=N, seed=42, precision=prec)
    pf.initialize(sim.ensemble_traj[0, 0], 2.0 * np.eye(40))
    res = pf.run(Z)
    print(prec, "rmse", float(res.rmse(X)[0]), "resample", res.flags.mean(), flush=True)
t0 = time.time()
o = pf_oracle.build_and_run(ssm_oracle.lorenz96(nx=40, q_std=0.1), Z, Np=N, seed=1, mean0=sim.ensemble_traj[0, 0],
                            cov0=2.0 * np.eye(40))
print("oracle rmse", float(np.sqrt(np.mean((o["means"] - X) ** 2))), "resample", o["flags"].mean(), time.time() - t0)
