"""fp32 within-filter sharding: W = 1 vs W = 2 step by step (tests/test_gpu_sharded.py::test_fp32_shards).
usage: [PF_LIB=...] python tools/diag_shards.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particle_filters_amd import models as M
from particle_filters_amd import sharded as SH

d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "sv_data.npz"))
T = 40
Z = np.log(d["Y0"][1:T + 1] ** 2)[:, None]


def run(W, prec):
    pf = SH.ShardedParticleFilter(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                                  Np=40000, resample_thresh=0.5, seed=11, precision=prec, n_shards=W)
    pf.initialize([0.0], [[0.5]])
    m, n, f = pf.run(Z)
    pf.close()
    return m[:, 0], n, f


for prec in ("fp32", "fp64"):
    m1, n1, f1 = run(1, prec)
    m2, n2, f2 = run(2, prec)
    print(f"{prec} ({os.environ.get('PF_LIB', 'default lib')})")
    for t in range(T):
        print(f"  t={t:2d} f {int(f1[t])}{int(f2[t])} neff {n1[t]:10.2f} {n2[t]:10.2f}  mean {m1[t]: .7f} {m2[t]: .7f}  "
              f"d {m2[t] - m1[t]: .2e}", flush=True)
