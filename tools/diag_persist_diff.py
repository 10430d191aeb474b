"""Where k_persist and the launch-per-step loop first differ on one case of tests/test_gpu_persist.py
(and whether each path repeats itself bitwise).   python tools/diag_persist_diff.py [case index]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_gpu_persist as TP  # noqa: E402


class MP:  # the monkeypatch calls _run makes
    def setenv(self, k, v):
        os.environ[k] = v

    def delenv(self, k, raising=False):
        os.environ.pop(k, None)


CASES = [dict(N=1_000_000, T=40), dict(N=1_000_000, T=40, fo=True), dict(N=1_000_003, T=20, thresh=0.8),
         dict(N=5_000, T=30, reps=3, regularize=True, thresh=0.8), dict(N=200_000, T=25, pre_update=True, thresh=0.999),
         dict(N=300_000, T=30, segments=(7, 8, 19, None), thresh=0.8)]
case = CASES[int(sys.argv[1]) if len(sys.argv) > 1 else 2]
runs = {k: TP._run(MP(), p, **case) for k, p in (("step", False), ("persist", True), ("persist2", True),
                                                   ("step2", False))}
for a, b in (("step", "step2"), ("persist", "persist2"), ("step", "persist")):
    bad = []
    for key in ("means", "covs", "neff", "flags", "log_norm", "x", "w"):
        x, y = np.asarray(runs[a][key], float), np.asarray(runs[b][key], float)
        if not np.array_equal(x, y, equal_nan=True):
            d = np.argwhere(~((x == y) | (np.isnan(x) & np.isnan(y))))
            bad.append(f"{key}: {len(d)} differ, first at {d[0].tolist()} ({x[tuple(d[0])]!r} vs {y[tuple(d[0])]!r})")
    print(f"{a} vs {b}: " + ("bitwise equal" if not bad else "; ".join(bad)))
print("flags (step):", np.nonzero(np.asarray(runs["step"]["flags"])[:, 0])[0].tolist())
