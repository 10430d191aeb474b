"""Why the first timed K=20 resident run after a 5-step warm-up is slower than later ones:
device time of the first run after different untimed preludes (fresh process each).
    python tools/diag_warmup.py none|matmul|filter"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from particle_filters_amd import _native as NV, models as M, simulators as S  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "none"
lib = NV.load()
W, K = 5, 20
d = S.simulate_sv_1d(W + K + 1, 0.95, 0.2, 1.0, seed=42)
Z = np.log(d.Y[1:] ** 2)[:, None]
dev = torch.device("cuda", 0)


def mk():
    pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                             Np=1_000_000, seed=42)
    pf.initialize([d.X[0]], [[0.5]])
    NV.check(lib.pf_set_timing(pf.handle, 1))
    return pf


def run(pf, dz, T):
    o = [torch.zeros((T, 1), dtype=torch.float64, device=dev) for _ in range(3)]
    fl = torch.zeros((T, 1), dtype=torch.int32, device=dev)
    NV.check(lib.pf_run_device(pf.handle, C.c_void_p(dz.data_ptr()), None, T, 0, C.c_void_p(o[0].data_ptr()), None,
                               C.c_void_p(o[1].data_ptr()), C.c_void_p(fl.data_ptr()), C.c_void_p(o[2].data_ptr())))
    NV.check(lib.pf_synchronize(pf.handle))
    ms = C.c_float()
    NV.check(lib.pf_last_run_ms(pf.handle, C.byref(ms)))
    return ms.value * 1e3


pf = mk()
dzw = torch.tensor(Z[:W], dtype=torch.float32, device=dev).contiguous()
dzk = torch.tensor(Z[W:W + K], dtype=torch.float32, device=dev).contiguous()
run(pf, dzw, W)
if mode == "matmul":
    a = torch.randn(4096, 4096, device=dev)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.005:
        a = a @ a
        a = a / a.norm()
    torch.cuda.synchronize()
elif mode == "filter":
    pf2 = mk()
    dz2 = torch.tensor(np.tile(Z[:20], (50, 1)), dtype=torch.float32, device=dev).contiguous()
    run(pf2, dz2, 1000)
    pf2.close()
torch.cuda.synchronize()
first = run(pf, dzk, K)
later = [run(pf, dzk, K) for _ in range(5)]
print(f"prelude={mode}: first timed K={K} run {first:.1f} us, next runs {np.round(later, 1).tolist()} us")
pf.close()
