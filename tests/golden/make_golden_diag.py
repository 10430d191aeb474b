#!/usr/bin/env python
"""Generate tests/golden/diag_cases.npz by running the REFERENCE degeneracy diagnostics.

Build container only:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_diag.py

The diagnostics live in a notebook, not a module: cell 5 of
/root/reference/notebooks/particle_filter_NLNGSSM.ipynb defines compute_weight_entropy,
compute_gini_coefficient, count_unique_particles and compute_diagnostics.  This script
executes that cell's source as-is (with the reference ParticleFilter importable for its
annotations) and records inputs and outputs on synthetic states plus the state of a
reference ParticleFilter run.  Only numbers are stored.
"""

from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True
REF = os.environ.get("PF_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402

from models.particle_filter import ParticleFilter  # noqa: E402  (reference)


def load_cell():
    nb = json.load(open(os.path.join(REF, "notebooks", "particle_filter_NLNGSSM.ipynb")))
    src = "".join(nb["cells"][5]["source"])
    ns = {"np": np, "ParticleFilter": ParticleFilter}
    exec(compile(src, "particle_filter_NLNGSSM.ipynb:cell5", "exec"), ns)  # noqa: S102
    return ns


def cases(rng):
    out = {}
    # ragged random weights, resampled duplicates in 2-D
    N = 1000
    w = rng.gamma(0.3, size=N)
    w /= w.sum()
    base = rng.standard_normal((N, 2))
    out["random2d"] = (w, base[rng.integers(0, N, N)])
    # uniform weights after a resample, 1-D, heavy duplication
    idx = np.sort(rng.integers(0, 50, N))
    out["uniform1d"] = (np.full(N, 1.0 / N), rng.standard_normal((N, 1))[idx])
    # near-degenerate: one weight dominates, others underflow to 0
    w = np.zeros(N)
    w[17] = 1.0 - 1e-12
    w[3] = 1e-12
    out["degenerate"] = (w, rng.standard_normal((N, 3)))
    # single particle
    out["single"] = (np.array([1.0]), np.array([[0.25, -1.0]]))
    # signed zeros, values on and near the 1e-10 rounding grid, exact duplicates
    x = np.array([[0.0], [-0.0], [1e-10], [1.5e-10], [2.5e-10], [-2.5e-10], [3e-10 + 1e-26], [1.0], [1.0],
                  [np.nextafter(1.0, 2.0)]])
    w = rng.random(len(x))
    out["grid"] = (w / w.sum(), x)
    # Lorenz-96-sized rows (nx = 40), partial duplication
    N = 500
    base = rng.standard_normal((N, 40)) * 3.0
    anc = np.concatenate([np.arange(300), rng.integers(0, 300, 200)])
    w = rng.dirichlet(np.full(N, 0.5))
    out["l96"] = (w, base[anc])
    return out


def main():
    ns = load_cell()
    rng = np.random.default_rng(2024)
    arrays = {}
    names = []
    for name, (w, x) in cases(rng).items():
        names.append(name)
        arrays[f"{name}__w"] = w
        arrays[f"{name}__x"] = x
        arrays[f"{name}__entropy"] = np.float64(ns["compute_weight_entropy"](w, normalized=True))
        arrays[f"{name}__entropy_raw"] = np.float64(ns["compute_weight_entropy"](w, normalized=False))
        arrays[f"{name}__gini"] = np.float64(ns["compute_gini_coefficient"](w))
        arrays[f"{name}__n_unique"] = np.int64(ns["count_unique_particles"](x, w))
    # compute_diagnostics on a reference ParticleFilter state (SV harness wiring, N = 2000)
    sv = np.load(os.path.join(HERE, "sv_data.npz"))
    X, Y = sv["X0"], sv["Y0"]
    pf = ParticleFilter(lambda x, u=None: 0.95 * x, lambda x: 1.0 * np.exp(0.5 * x), np.array([[0.04]]),
                        np.array([[0.1]]), Np=2000, resample_thresh=0.5, regularize_after_resample=False,
                        rng=np.random.default_rng(7))
    pf.initialize(mean=np.array([X[0]]), cov=np.array([[0.5]]))
    snaps = []
    for k in range(1, 26):
        pf.predict()
        st = pf.update(np.array([Y[k]]))
        if k in (5, 12, 25):
            d = ns["compute_diagnostics"](pf, resampled=False)
            snaps.append((k, st.weights.copy(), st.particles.copy(), st.cov.copy(), d))
    for k, w, x, c, d in snaps:
        name = f"pfstate{k}"
        names.append(name)
        arrays[f"{name}__w"] = w
        arrays[f"{name}__x"] = x
        arrays[f"{name}__cov"] = c
        for key in ("ess", "entropy", "gini", "max_weight", "n_unique", "posterior_spread"):
            arrays[f"{name}__{key}"] = np.asarray(d[key])
    arrays["names"] = np.array(names)
    path = os.path.join(HERE, "diag_cases.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


if __name__ == "__main__":
    main()
