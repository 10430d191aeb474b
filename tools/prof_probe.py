"""Minimal resident-kernel run without torch (profiler exit-path probe)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from particle_filters_amd import models as M, simulators as S  # noqa: E402
from particle_filters_amd.batch import ParticleFilterBatch  # noqa: E402

d = S.simulate_sv_1d(201, 0.95, 0.2, 1.0, seed=42)
pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=1_000_000,
                         seed=42)
pf.initialize([d.X[0]], [[0.5]])
r = pf.run(np.log(d.Y[1:] ** 2))
print("resident", pf.last_run_resident, "rmse", float(r.rmse(d.X[1:])[0]))
pf.close()
