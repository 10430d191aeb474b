"""Diagnostic: does having torch initialised in-process slow the engine's launches?"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1]
import torch
if mode in ("init", "tensors"):
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
import ctypes as C
from particle_filters_amd import _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch
lib = NV.load()
pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=1000000, seed=1)
pf.initialize([0.0], [[0.5]])
T = 1000
d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
Z = np.log(d.Y[1:] ** 2).astype(np.float32)
if mode == "tensors":
    dZ = torch.tensor(Z, device="cuda")
    outs = [torch.zeros(T, dtype=torch.float64, device="cuda") for _ in range(4)]
    ptrs = [C.c_void_p(dZ.data_ptr())] + [C.c_void_p(o.data_ptr()) for o in outs]
else:
    hip = C.CDLL("libamdhip64.so")
    ptrs = []
    for nb in (Z.nbytes, T * 8, T * 8, T * 8, T * 8):
        p = C.c_void_p(); hip.hipMalloc(C.byref(p), C.c_size_t(nb)); ptrs.append(p)
    hip.hipMemcpy(ptrs[0], Z.ctypes.data_as(C.c_void_p), C.c_size_t(Z.nbytes), 1)
torch.cuda.synchronize() if mode != "import" else None
for rep in range(3):
    t0 = time.perf_counter()
    lib.pf_run_device(pf.handle, ptrs[0], None, T, 0, ptrs[1], None, ptrs[2], ptrs[3], ptrs[4])
    t1 = time.perf_counter()
    lib.pf_synchronize(pf.handle)
    t2 = time.perf_counter()
    print(f"{mode}: enqueue {1e6*(t1-t0)/T:.1f} us/step, total {1e6*(t2-t0)/T:.1f} us/step", flush=True)
print(mode, {k: v for k, v in os.environ.items() if k.startswith(("HIP", "HSA", "AMD", "GPU"))})
