"""Diagnostic: device-loop covariance (pf_cov.h) per replicate and step against the exact two-pass
moments of the same state (pf_moments), run as a chain of one-step runs.
    python tools/diag_cov.py [workload] [R] [N] [precision] [T]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from particle_filters_amd import _native as NV  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "mat"
R = int(sys.argv[2]) if len(sys.argv) > 2 else 2
N = int(sys.argv[3]) if len(sys.argv) > 3 else 1500
prec = sys.argv[4] if len(sys.argv) > 4 else "fp64"
T = int(sys.argv[5]) if len(sys.argv) > 5 else 10
wl = bench.WORKLOADS[name]()
g, h, Q, R_, Z, truth, mean0, cov0 = wl.build(T, 0)
Z = np.asarray(Z, float)
b = ParticleFilterBatch(g, h, Q, R_, Np=N, n_replicates=R, seed=5, precision=prec)
b.initialize(mean0, cov0)
nx = b.nx
for t in range(T):
    r = b.run(Z[t:t + 1])
    m = np.empty((R, nx))
    c = np.empty((R, nx, nx))
    NV.check(NV.load().pf_moments(b.handle, NV.dptr(m), NV.dptr(c)))
    for k in range(R):
        sc = np.max(np.abs(c[k]))
        print(f"t={t} rep {k} flag {int(r.flags[0, k])}: |dcov|/max|cov| {np.max(np.abs(r.covs[0, k] - c[k])) / sc:.2e} "
              f"|dmean| {np.max(np.abs(r.means[0, k] - m[k])):.2e} max|cov| {sc:.3e} engine max|cov| "
              f"{np.max(np.abs(r.covs[0, k])):.3e}")
b.close()
