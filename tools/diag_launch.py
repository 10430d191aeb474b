"""Diagnostic: where does the wall time of the device-resident loop go?
Times host enqueue of pf_run_device vs total, for several step counts."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C
from particle_filters_amd import _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch

lib = NV.load()
Np = int(os.environ.get("NP", "1000000"))
pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=Np, seed=1)
pf.initialize([0.0], [[0.5]])
T = 1000
d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
Z = np.log(d.Y[1:] ** 2).astype(np.float32)

def dalloc(nbytes):
    p = C.c_void_p()
    lib_hip = C.CDLL("libamdhip64.so")
    assert lib_hip.hipMalloc(C.byref(p), C.c_size_t(nbytes)) == 0
    return p, lib_hip
dZ, hip = dalloc(Z.nbytes)
hip.hipMemcpy(dZ, Z.ctypes.data_as(C.c_void_p), C.c_size_t(Z.nbytes), 1)
outs = [dalloc(T * 8)[0] for _ in range(4)]
for rep in range(3):
    for steps in (10, 100, 1000):
        t0 = time.perf_counter()
        st = lib.pf_run_device(pf.handle, dZ, None, steps, 0, outs[0], None, outs[1], outs[2], outs[3])
        t1 = time.perf_counter()
        lib.pf_synchronize(pf.handle)
        t2 = time.perf_counter()
        print(f"steps {steps}: enqueue {1e6*(t1-t0)/steps:.1f} us/step, total {1e6*(t2-t0)/steps:.1f} us/step", flush=True)
