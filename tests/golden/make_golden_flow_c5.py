#!/usr/bin/env python
"""Generate tests/golden/flow_c5.npz: the REFERENCE LEDH and EDH filters at BASELINE config 5's size.

Build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_flow_c5.py

Config 5 is the LEDH particle-flow filter on Lorenz-96 d = 40 with N = 1e4 particles and L = 8
pseudo-time steps (the bench's ``--workload ledh``: simulate_lorenz96(nx=40, spinup 1000,
obs_interval 1, obs_fraction 4, seed 42), Q = 0.1^2 I, x0 ~ N(ensemble[0, 0], 2 I), resampling at
ESS < N / 2).  At N = 1e4 the fused device step spreads the particles over 157 workgroups: the
cross-workgroup combine, the source-driven slot partition over CDF slices and the offspring-count
moments all run, which the N = 64 golden of make_golden_ledh.py (one workgroup) never reaches.

Stored (numbers only, ~0.6 MB): the observations, the per-step posterior means and covariances,
the resample flags, the final weights, the first 256 final particles, and per draw of the random
stream its length, sum, sum of squares and first values, so that the test can regenerate the stream
from the seed with NumPy on the GPU box (the draws themselves are 64 MB) and prove it regenerated
the reference's.  The runs are driven exactly as make_golden_ledh.py / make_golden_edh.py drive the
reference (EKF tracker, process_noise_sampler = rng.multivariate_normal(0, Q, N)).
"""

from __future__ import annotations

import os
import sys
import time

sys.dont_write_bytecode = True
REF = os.environ.get("PF_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from simulator.simulator_Lorenz_96 import simulate_lorenz96  # noqa: E402  (reference)

from oracle import ledh_oracle as LO  # noqa: E402
import make_golden_ledh as GL  # noqa: E402
import make_golden_edh as GE  # noqa: E402

T_STEPS = 20
N_PART = 10_000
N_LAMBDA = 8
N_KEEP = 256


def stream_summary(log):
    """Per draw: kind (0 mvn, 1 random), size, sum, sum of squares, first 8 values."""
    rows = []
    for kind, a in log:
        a = np.asarray(a, float).reshape(-1)
        head = np.zeros(8)
        head[:min(8, a.size)] = a[:8]
        rows.append(np.concatenate([[0.0 if kind == "mvn" else 1.0, a.size, a.sum(), (a * a).sum()], head]))
    return np.array(rows)



def main():
    sim = simulate_lorenz96(nx=40, F=8.0, dt=0.01, spinup_steps=1000, total_steps=T_STEPS, Np=1, obs_interval=1,
                            obs_fraction=4, obs_error_std=1.0, seed=42)
    Z = np.asarray(sim.observations, float)[1:T_STEPS + 1]
    model = LO.lorenz96(40, q_std=0.1)
    assert np.allclose(model.Q, 0.01 * np.eye(40)), "config 5 uses Q = 0.1^2 I"
    mean0 = np.asarray(sim.ensemble_traj[0, 0], float)
    cov0 = 2.0 * np.eye(40)
    arrays = {"Z": Z, "mean0": mean0, "cov0": cov0, "R": np.asarray(sim.R, float), "H_idx": np.asarray(sim.H_idx),
              "n_particles": N_PART, "n_lambda": N_LAMBDA, "ratio": 0.5, "seed": 42}
    for algo in ("ledh", "edh"):
        t0 = time.time()
        seen = {}
        orig = GL.RecordingGenerator.__init__

        def init(self, gen, _orig=orig):  # keep a handle on the run's recording generator
            _orig(self, gen)
            seen["rec"] = self

        GL.RecordingGenerator.__init__ = init
        try:
            if algo == "ledh":
                out = GL.run_ref(model, Z, mean0=mean0, cov0=cov0, n_particles=N_PART, n_lambda=N_LAMBDA, ratio=0.5,
                                 seed=42)
            else:
                out = GE.run_ref(model, Z, mean0=mean0, cov0=cov0, n_particles=N_PART, n_lambda=N_LAMBDA, ratio=0.5,
                                 seed=42, integrator="rk4")
        finally:
            GL.RecordingGenerator.__init__ = orig
        arrays[f"{algo}__means"] = out["means"]
        arrays[f"{algo}__covs"] = out["covs"]
        arrays[f"{algo}__flags"] = out["flags"]
        arrays[f"{algo}__final_weights"] = out["weights"][-1]
        arrays[f"{algo}__final_particles_head"] = out["particles"][-1][:N_KEEP]
        arrays[f"{algo}__init_particles_head"] = out["init_particles"][:N_KEEP]
        arrays[f"{algo}__init_mean"] = out["init_mean"]
        arrays[f"{algo}__stream"] = stream_summary(seen["rec"].log)
        print(f"{algo}: T={T_STEPS} N={N_PART} L={N_LAMBDA}: resamples {int(out['flags'].sum())} at "
              f"{np.nonzero(out['flags'])[0].tolist()}, {time.time() - t0:.0f} s")
    path = os.path.join(HERE, "flow_c5.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


if __name__ == "__main__":
    main()
