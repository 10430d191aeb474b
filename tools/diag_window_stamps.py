"""Phase accounting of k_resident in bench.py's driver window (diagnostic stamps build:
PF_LIB=build/libpf_hip_stamps.so): the same data series (simulate_sv_1d over W + max(K, 30)
steps, seed 42), a W-step warm-up launch, then the K-step launch whose stamps are printed,
with the step of every resample in the window.

    python tools/diag_window_stamps.py [K=20] [W=5] [N=1e6]
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from particle_filters_amd import _native as NV, models as M, simulators as S  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402

lib = NV.load()
K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
N = int(float(sys.argv[3])) if len(sys.argv) > 3 else 1_000_000
T_data = W + max(K, 30)
d = S.simulate_sv_1d(T_data + 1, 0.95, 0.2, 1.0, seed=42)
Z = np.log(d.Y[1:] ** 2)
pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=N, seed=42)
pf.initialize([d.X[0]], [[0.5]])
dev = torch.device("cuda", 0)
names = ["loop top (prefetch, decision tail)", "compute", "barrier wait", "publish", "verify combine",
         "rollback (total)"]
rb_names = {6: "rb: own tile CDF", 7: "rb: offspring counts", 8: "rb: global prefix", 9: "rb: offspring scatter",
            10: "rb: gathered hand-off", 11: "rb: read+jitter", 12: "slow polls"}


def run(z, T):
    dZ = torch.tensor(z[:T, None], dtype=torch.float32, device=dev).contiguous()
    outs = [torch.zeros((T, 1), dtype=torch.float64, device=dev) for _ in range(4)]
    fl = torch.zeros((T, 1), dtype=torch.int32, device=dev)
    NV.check(lib.pf_run_device(pf.handle, C.c_void_p(dZ.data_ptr()), None, T, 0, C.c_void_p(outs[0].data_ptr()),
                               C.c_void_p(outs[1].data_ptr()), C.c_void_p(outs[2].data_ptr()),
                               C.c_void_p(fl.data_ptr()), C.c_void_p(outs[3].data_ptr())))
    NV.check(lib.pf_synchronize(pf.handle))
    return fl.cpu().numpy()[:, 0], outs[2].cpu().numpy()[:, 0]


if W > 0:
    run(Z[:W], W)
lib.pf_debug_stamps_sv_zero(24)
flags, neff = run(Z[W:W + K], K)
ms = C.c_float()
lib.pf_last_run_ms(pf.handle, C.byref(ms))
buf = (C.c_ulonglong * 24)()
lib.pf_debug_stamps_sv(buf, 24)
v = np.array(buf[:], dtype=float)
steps = max(v[14], 1)
tot = v[:6].sum() + v[22] + v[23]
print(f"window W={W} K={K} N={N}: resample steps {np.nonzero(flags)[0].tolist()}, Neff/N "
      f"{np.round(neff / N, 3).tolist()}")
print(f"launch phases (workgroup 0): entry {(v[17] - v[16]) / 100:.2f} us (prologue "
      f"{(v[20] - v[16]) / 100:.2f}), loop {(v[18] - v[17]) / 100:.2f} us, exit {(v[19] - v[18]) / 100:.2f} us "
      f"(state stores {(v[21] - v[18]) / 100:.2f}); engine events {ms.value * 1e3:.1f} us")
print(f"steps computed {int(v[14])} rollbacks {int(v[13])} failed polls {int(v[15])} "
      f"total {tot / 100 / K:.2f} us per filter step")
for k, n in enumerate(names):
    print(f"   {n:34s} {v[k] / 100 / steps:8.3f} us/computed-step ({v[k] / 100:7.2f} us)")
for k, n in {22: "  of which: own wave partials", 23: "  of which: verification summary"}.items():
    print(f"   {n:34s} {v[k] / 100 / steps:8.3f} us/computed-step ({v[k] / 100:7.2f} us)")
for k, n in rb_names.items():
    per = v[k] / 100 / max(v[13], 1) if k < 12 else v[k] / 100 / steps
    print(f"   {n:34s} {per:8.3f} us/{'rollback' if k < 12 else 'computed-step'}")
pf.close()
