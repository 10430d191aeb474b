"""Phase accounting of k_resident (diagnostic stamps build: PF_LIB=build/libpf_hip_stamps.so).
Workgroup 0 accumulates s_memrealtime ticks (10 ns) per phase over a whole run."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from particle_filters_amd import _native as NV, models as M, simulators as S  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402

lib = NV.load()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
Z = np.log(d.Y[1:] ** 2)
pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=N, seed=42)
pf.initialize([d.X[0]], [[0.5]])
dev = torch.device("cuda", 0)
dZ = torch.tensor(Z[:T, None], dtype=torch.float32, device=dev).contiguous()
outs = [torch.zeros((T, 1), dtype=torch.float64, device=dev) for _ in range(4)]
fl = torch.zeros((T, 1), dtype=torch.int32, device=dev)
names = ["loop top (prefetch, decision tail)", "compute", "wave partials + barrier", "publish", "verify combine",
         "rollback (total)"]
rb_names = {6: "rb: own tile CDF", 7: "rb: offspring counts", 8: "rb: global prefix", 9: "rb: offspring scatter",
            10: "rb: gathered hand-off", 11: "rb: read+jitter", 12: "slow polls"}
for rep in range(2):
    lib.pf_debug_stamps_sv_zero(24)
    NV.check(lib.pf_run_device(pf.handle, C.c_void_p(dZ.data_ptr()), None, T, 0, C.c_void_p(outs[0].data_ptr()),
                               C.c_void_p(outs[1].data_ptr()), C.c_void_p(outs[2].data_ptr()),
                               C.c_void_p(fl.data_ptr()), C.c_void_p(outs[3].data_ptr())))
    NV.check(lib.pf_synchronize(pf.handle))
    buf = (C.c_ulonglong * 24)()
    lib.pf_debug_stamps_sv(buf, 24)
    v = np.array(buf[:], dtype=float)
    steps = max(v[14], 1)
    tot = v[:6].sum()
    print(f"run {rep}: launch phases (workgroup 0): entry {(v[17] - v[16]) / 100:.2f} us (prologue "
          f"{(v[20] - v[16]) / 100:.2f}), loop {(v[18] - v[17]) / 100:.2f} us, exit {(v[19] - v[18]) / 100:.2f} us "
          f"(state stores {(v[21] - v[18]) / 100:.2f})")
    print(f"run {rep}: steps computed {int(v[14])} rollbacks {int(v[13])} failed polls {int(v[15])} "
          f"total {tot / 100 / T:.2f} us per filter step")
    for k, n in enumerate(names):
        print(f"   {n:34s} {v[k] / 100 / steps:8.3f} us/computed-step")
    for k, n in rb_names.items():
        per = v[k] / 100 / max(v[13], 1) if k < 12 else v[k] / 100 / steps
        print(f"   {n:34s} {per:8.3f} us/{'rollback' if k < 12 else 'computed-step'}")
