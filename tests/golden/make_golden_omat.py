#!/usr/bin/env python
"""Generate tests/golden/omat_cases.npz by running the REFERENCE OMAT metric.

Build container only:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_omat.py

The OMAT distance of BASELINE config 4 lives in a notebook, not a module:
/root/reference/notebooks/PF_PF_results_reproduction_multi_target_acoustic_tracking.ipynb
(``compute_omat``, lines 175-206 of the .ipynb; used per time step at 728-737, "Average OMAT"
at 785).  This script executes that function's source as it stands in the notebook (with
scipy's linear_sum_assignment, as the notebook imports it) and records inputs and outputs on
the committed MAT fixtures (tests/golden/mat_data.npz: true positions P [T][C][2]) against
perturbed, permuted, far and collapsed estimates, for p = 1 (the notebook's) and p = 2.  Only
numbers are stored.
"""

from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True
REF = os.environ.get("PF_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402
from scipy.optimize import linear_sum_assignment  # noqa: E402

NB = "PF_PF_results_reproduction_multi_target_acoustic_tracking.ipynb"


def load_compute_omat():
    nb = json.load(open(os.path.join(REF, "notebooks", NB)))
    for cell in nb["cells"]:
        src = "".join(cell["source"])
        if "def compute_omat(" in src:
            a = src.index("def compute_omat(")
            b = src.index("return omat", a) + len("return omat")
            ns = {"np": np, "linear_sum_assignment": linear_sum_assignment}
            exec(compile(src[a:b] + "\n", f"{NB}:compute_omat", "exec"), ns)  # noqa: S102
            return ns["compute_omat"]
    raise RuntimeError("compute_omat not found in the notebook")


def main():
    f = load_compute_omat()
    mat = np.load(os.path.join(HERE, "mat_data.npz"))
    rng = np.random.default_rng(11)
    arrays = {}
    for key, P in (("c4", mat["P"]), ("c3", mat["P2"])):
        T, C, _ = P.shape
        ests = {
            "near": P + rng.standard_normal(P.shape),
            "permuted": P[:, rng.permutation(C)] + 3.0 * rng.standard_normal(P.shape),
            "far": P + 20.0 * rng.standard_normal(P.shape),
            "collapsed": np.repeat(P.mean(axis=1, keepdims=True), C, axis=1) + 0.1 * rng.standard_normal(P.shape),
            "exact": P.copy(),
        }
        for name, E in ests.items():
            arrays[f"{key}__{name}__est"] = E
            for p in (1, 2):
                arrays[f"{key}__{name}__omat_p{p}"] = np.array([f(P[t], E[t], p=p) for t in range(T)])
        arrays[f"{key}__truth"] = P
    np.savez_compressed(os.path.join(HERE, "omat_cases.npz"), **arrays)
    print(f"wrote omat_cases.npz: {len(arrays)} arrays; c4 near p=1 average OMAT "
          f"{arrays['c4__near__omat_p1'].mean():.6f}")


if __name__ == "__main__":
    main()
