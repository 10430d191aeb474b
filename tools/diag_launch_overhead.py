"""Host-side cost of one pf_run_device call (the launch API) vs its device interval, for the
resident SV kernel at N = 1e6: plain vs cooperative launch (PF_COOP, read once per process).
    python tools/diag_launch_overhead.py T reps"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from particle_filters_amd import _native as NV, models as M, simulators as S  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
lib = NV.load()
d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=1_000_000,
                         seed=42)
pf.initialize([d.X[0]], [[0.5]])
NV.check(lib.pf_set_timing(pf.handle, 1))
dev = torch.device("cuda", 0)
dZ = torch.tensor(np.log(d.Y[1:T + 1] ** 2)[:, None], dtype=torch.float32, device=dev).contiguous()
o = [torch.zeros((T, 1), dtype=torch.float64, device=dev) for _ in range(3)]
fl = torch.zeros((T, 1), dtype=torch.int32, device=dev)
host, devi, wall = [], [], []
for k in range(reps):
    NV.check(lib.pf_synchronize(pf.handle))
    t0 = time.perf_counter()
    NV.check(lib.pf_run_device(pf.handle, C.c_void_p(dZ.data_ptr()), None, T, 0, C.c_void_p(o[0].data_ptr()), None,
                               C.c_void_p(o[1].data_ptr()), C.c_void_p(fl.data_ptr()), C.c_void_p(o[2].data_ptr())))
    t1 = time.perf_counter()
    NV.check(lib.pf_synchronize(pf.handle))
    t2 = time.perf_counter()
    ms = C.c_float()
    NV.check(lib.pf_last_run_ms(pf.handle, C.byref(ms)))
    if k >= 3:
        host.append((t1 - t0) * 1e6)
        wall.append((t2 - t0) * 1e6)
        devi.append(ms.value * 1e3)
print(f"PF_COOP={os.environ.get('PF_COOP', '1')} T={T}: host call {np.median(host):.1f} us, device events "
      f"{np.median(devi):.1f} us ({np.median(devi) / T:.2f} us/step), call+sync wall {np.median(wall):.1f} us")
pf.close()
