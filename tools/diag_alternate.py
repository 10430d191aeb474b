"""Device time of consecutive K=20 resident runs on one handle, outputs preallocated; prints
each run (is every other run slower, and why).  python tools/diag_alternate.py [T] [runs]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from particle_filters_amd import _native as NV, models as M, simulators as S  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 20
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 12
lib = NV.load()
d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
dev = torch.device("cuda", 0)
dZ = torch.tensor(np.log(d.Y[1:T + 1] ** 2)[:, None], dtype=torch.float32, device=dev).contiguous()
o = [torch.zeros((T, 1), dtype=torch.float64, device=dev) for _ in range(3)]
fl = torch.zeros((T, 1), dtype=torch.int32, device=dev)
torch.cuda.synchronize()
pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=1_000_000,
                         seed=42)
pf.initialize([d.X[0]], [[0.5]])
NV.check(lib.pf_set_timing(pf.handle, 1))
res = []
for k in range(runs):
    NV.check(lib.pf_run_device(pf.handle, C.c_void_p(dZ.data_ptr()), None, T, 0, C.c_void_p(o[0].data_ptr()), None,
                               C.c_void_p(o[1].data_ptr()), C.c_void_p(fl.data_ptr()), C.c_void_p(o[2].data_ptr())))
    NV.check(lib.pf_synchronize(pf.handle))
    ms = C.c_float()
    NV.check(lib.pf_last_run_ms(pf.handle, C.byref(ms)))
    res.append((ms.value * 1e3, int(fl.cpu().numpy().sum()), int(fl.cpu().numpy()[-1, 0])))
print(f"T={T} PF_COOP={os.environ.get('PF_COOP', '-')}: " + ", ".join(f"{u:.1f}us(res {n}, last {l})" for u, n, l in res))
pf.close()
