"""Per-phase timing of the fused LEDH step (k_ledh_fused) from s_memrealtime stamps.
usage: PF_LIB=build/libpf_hip_stamps.so python tools/diag_stamps_ledh.py [N]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particle_filters_amd import _native as NV, ledh as LD, models as M, simulators as S, trackers as TR  # noqa: E402

lib = NV.load()
lib.pf_debug_stamps_ledh.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
Np = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
noise = sys.argv[2] if len(sys.argv) > 2 else "device"
sim = S.simulate_lorenz96(nx=40, F=8.0, dt=0.01, spinup_steps=1000, total_steps=60, Np=1, obs_interval=1,
                          obs_fraction=4, obs_error_std=1.0, seed=42)
g, h = M.L96Transition(8.0, 0.01, 40), M.SelectObservation(sim.H_idx, 40)
Q, R = 0.01 * np.eye(40), sim.R
m0, c0 = sim.ensemble_traj[0, 0], 2.0 * np.eye(40)
ekf = TR.ExtendedKalmanFilter(g, h, Q, R, jac_g=g.jacobian, jac_h=h.jacobian)
tr = TR.EKFTracker(ekf, TR.EKFState(m0.copy(), c0.copy(), 0))
pf = LD.LEDHFlowPF(tr, g, h, h.jacobian, M.GaussianTransitionDensity(g, Q), M.GaussianLikelihood(h, R), R,
                   LD.LEDHConfig(n_particles=Np, n_lambda_steps=8, resample_ess_ratio=0.5,
                                 rng=np.random.default_rng(1)), rng_mode="device")
st = pf.init_from_gaussian(m0, c0)
names = {0: "entry", 1: "params staged (first prior under it)", 6: " flow: x loaded", 7: " flow: RK4", 8: " flow: noise", 9: " flow: H eta0", 10: " flow: eta_L", 11: " flow: weight", 12: " P1 rows out + wg max", 13: " P2 exp + scan", 2: "P1+P2 flow/exp", 3: "B1", 14: " P3 partials loaded", 15: " P3 combine + decision", 4: "P3 decide", 18: " P4 setup + chunk barrier", 19: " P4 weights staged", 16: " P4 MFMA Gram accumulate", 17: " P4 partial stores", 5: "P4 rows+moments"}
FST = 20
for T in (10, 30, 50):
    res = pf.run(pf.state, sim.observations[1:T + 1], tracker="device", process_noise=noise)
    nb = 256
    buf = (C.c_ulonglong * (nb * FST))()
    assert lib.pf_debug_stamps_ledh(buf, nb * FST) == 0
    a = np.array(buf[:], dtype=np.float64).reshape(nb, FST)
    live = a[:, 0] > 0
    a = a[live]
    rel = (a - a[:, 0].min()) / 100.0
    print(f"noise={noise} N={Np} T={T} workgroups={live.sum()} last flag={res.flags[-1]}")
    for k, nm in names.items():
        col = rel[:, k]
        col = col[col > -1e6]
        print(f"  {nm:12s} min {col.min():8.2f} med {np.median(col):8.2f} max {col.max():8.2f} us")
