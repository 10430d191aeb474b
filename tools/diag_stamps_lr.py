"""Phase accounting of the acoustic per-particle flow k_flow_wave_lr (LEDH-MAT, bench.py --workload
ledh_mat's model: joint 16-D / 25 sensors, N = 500, L = 64).  Workgroup 0 accumulates s_memrealtime
ticks (10 ns) per phase over its particles and pseudo-time steps.
usage: PF_LIB=build/libpf_hip_stamps.so python tools/diag_stamps_lr.py [T]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particle_filters_amd import _native as NV, ledh as LD, models as M, simulators as S, trackers as TR  # noqa: E402

lib = NV.load()
lib.pf_debug_lr_acc.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
T = int(sys.argv[1]) if len(sys.argv) > 1 else 5
Np, L = 500, 64
cfg_s = S.ScenarioConfig(n_targets=4, n_steps=max(40, T + 1), sensor_grid_shape=(5, 5), psi=10.0, d0=0.1, seed=56,
                         use_article_init=True)
data = S.simulate_acoustic_dataset(cfg_s, S.DynamicsConfig())
g, h = M.CVTransition(4, 1.0), M.AcousticObservation(data["S"], 10.0, 0.1, 4)
Q, R = np.kron(np.eye(4), S.article_process_noise_cov()), 0.1 ** 2 * np.eye(25)
Xt = data["X"].reshape(data["X"].shape[0], 16)
mean0 = Xt[0] + np.tile([1.5, -1.0, 0.1, -0.1], 4)
cov0 = np.kron(np.eye(4), np.diag([100.0, 100.0, 1.0, 1.0]))
ekf = TR.ExtendedKalmanFilter(g, h, Q, R, jac_g=g.jacobian, jac_h=h.jacobian)
tr = TR.EKFTracker(ekf, TR.EKFState(mean0.copy(), cov0.copy(), 0))
pf = LD.LEDHFlowPF(tr, g, h, h.jacobian, M.GaussianTransitionDensity(g, Q), M.GaussianLikelihood(h, R), R,
                   LD.LEDHConfig(n_particles=Np, n_lambda_steps=L, resample_ess_ratio=0.5,
                                 rng=np.random.default_rng(42)), rng_mode="device")
st = pf.init_from_gaussian(mean0, cov0)
buf = (C.c_ulonglong * 16)()
assert lib.pf_debug_lr_acc(buf, 16, 1) == 0
pf.run(st, data["Z"][1:T + 1], tracker="device")
assert lib.pf_debug_lr_acc(buf, 16, 1) == 0
a = np.array(buf[:10], dtype=np.float64) / 100.0  # us
names = ["H8 rows, h, R^-1 (z - e)", "Rq: Gram (MFMA) + Cholesky", "M = Rq P_pp Rq^T (MFMA) (+ S of particle 0)",
         "Gauss-Jordan [D | Rq | C], log-dets", "K = -1/2 Rq^T D^-1 Rq", "(unused)",
         "position-space flow update", "prior (g, noise) per particle", "weight + store per particle", "[D | Rq | C] columns"]
per = T * L  # pseudo-time steps of workgroup 0's first particle per filter step... (one particle per workgroup)
tot = a.sum()
print(f"k_flow_wave_lr workgroup 0: T={T} filter steps x L={L}, total {tot:.1f} us")
for k, nm in enumerate(names):
    scale = T if k in (7, 8) else per
    print(f"  {nm:40s} {a[k]:9.1f} us  {a[k] / scale:7.3f} us per {'particle' if k in (7, 8) else 'lambda step'}"
          f"  ({100 * a[k] / tot:5.1f} %)")
