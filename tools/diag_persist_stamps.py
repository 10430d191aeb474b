"""Phase accounting of k_persist (the fp64 whole-run kernel) on bench.py's fp64 window (diagnostic
stamps build: PF_LIB=build/libpf_hip_<stamps variant>.so): a W-step warm-up run, then the K-step run
whose stamps (thread 0 of workgroup PF_PSTAMP_B) are printed per step.

    python tools/diag_persist_stamps.py [K=20] [W=5] [N=1e6]
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particle_filters_amd import _native as NV, models as M, simulators as S  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402

lib = NV.load()
K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
N = int(float(sys.argv[3])) if len(sys.argv) > 3 else 1_000_000
d = S.simulate_sv_1d(W + K + 1, 0.95, 0.2, 1.0, seed=42)
Z = np.log(d.Y[1:] ** 2)[:, None]
pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=N, seed=42,
                         precision="fp64")
pf.initialize([d.X[0]], [[0.5]])
if W:
    pf.run(Z[:W])
lib.pf_debug_stamps_sv_zero(8)
r = pf.run(Z[W:W + K])
assert lib.pf_last_run_persistent(pf.handle) == 1
buf = (C.c_ulonglong * 8)()
lib.pf_debug_stamps_sv(buf, 8)
v = np.array(buf[:], dtype=float)
steps = max(v[7], 1)
names = ["speculation (normals, predict, loglik)", "data flag (store drain + barrier)", "record poll (wait)",
         "prologue reduce", "weights / gather + stores", "record merge + publish", "outputs (workgroup 0)"]
print(f"K={K} W={W} N={N}: steps {int(v[7])}, resample steps {np.nonzero(r.flags[:, 0])[0].tolist()}")
for k, n in enumerate(names):
    print(f"  {n:40s} {v[k] / 100 / steps:8.3f} us/step")
print(f"  {'total':40s} {v[:7].sum() / 100 / steps:8.3f} us/step")
pf.close()
