"""Per-phase timing of k_step from s_memrealtime stamps (PF_STAMPS build).
usage: PF_LIB=build/libpf_hip_stamps.so python tools/diag_stamps.py [N] [fp32|fp64]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C
from particle_filters_amd import _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch
lib = NV.load()
lib.pf_debug_stamps_sv.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
Np = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=Np, seed=1,
                         precision=prec)
pf.initialize([0.0], [[0.5]])
G, tile, lds = pf.geometry()
d = S.simulate_sv_1d(400, 0.95, 0.2, 1.0, seed=42)
Z = np.log(d.Y[1:] ** 2)
SL = 10
for rep in range(3):
    res = pf.run(Z[:50 + rep])
    buf = (C.c_ulonglong * (G * SL))()
    assert lib.pf_debug_stamps_sv(buf, G * SL) == 0
    a = np.array(buf[:], dtype=np.float64).reshape(G, SL)[:, :8]
    t0 = a[:, 0].min()
    rel = (a - t0) / 100.0  # us (100 MHz)
    print(f"N={Np} G={G} tile={tile} last-step flag={res.flags[-1,0]}")
    names = ["entry", "prologue", "outputs", "ancestors", "chunks", "record", "-", "-"]
    for k, nm in enumerate(names):
        col = rel[:, k]
        print(f"  {nm:11s} min {col.min():7.2f}  med {np.median(col):7.2f}  max {col.max():7.2f} us")
