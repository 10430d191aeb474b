"""Many-replicate SV timing probe: 64 x N=1e6 filters, device loop, with / without resampling.
usage: python tools/sv64_probe.py [R] [N] [T]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particle_filters_amd import models as M, simulators as S  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402
from particle_filters_amd import _native as NV  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 64
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
T = int(sys.argv[3]) if len(sys.argv) > 3 else 40
d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=42)
Z = np.log(d.Y[1:] ** 2)[:, None]
for thresh in (0.0, 0.5, 1.01):
    pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=N,
                             n_replicates=R, seed=42, resample_thresh=thresh)
    pf.initialize([d.X[0]], [[0.5]])
    pf.run(Z[:5])
    NV.check(NV.load().pf_synchronize(pf.handle))
    t0 = time.perf_counter()
    res = pf.run(Z[:T])
    NV.check(NV.load().pf_synchronize(pf.handle))
    dt = time.perf_counter() - t0
    print(f"R={R} N={N} thresh={thresh}: {dt / T * 1e6:.1f} us/step, {R * N * T / dt:.3g} particle-steps/s, "
          f"resample rate {res.flags.mean():.3f}, geometry {pf.geometry()}", flush=True)
    pf.close()
