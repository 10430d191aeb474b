"""BASELINE config 5 fixture (tests/golden/flow_c5.npz: the reference's LEDH and EDH runs at N = 1e4,
L = 8, Lorenz-96 d = 40; make_golden_flow_c5.py) - CPU tests.

* The draw stream the GPU replay test regenerates from the seed (NumPy, same calls in the same
  order) is the reference's: every draw's size, sum, sum of squares and first values.
* The vectorised NumPy oracles (oracle/ledh_oracle.py, oracle/edh_oracle.py), pinned bit for bit to
  the reference at small N by tests/test_ledh_oracle.py / test_edh_oracle.py, reproduce the
  reference at this size too: means within 1e-9 x scale and covariances within 1e-8 (LEDH over the
  first 4 steps - its per-particle flow costs ~7 s a step in NumPy -, EDH over all 20).
"""

import os

import numpy as np
import pytest

from oracle import edh_oracle as EO, ledh_oracle as LO

C5 = np.load(os.path.join(os.path.dirname(__file__), "golden", "flow_c5.npz"))


def _row(kind, a):
    a = np.asarray(a, float).reshape(-1)
    head = np.zeros(8)
    head[:min(8, a.size)] = a[:8]
    return np.concatenate([[kind, a.size, a.sum(), (a * a).sum()], head])


@pytest.mark.parametrize("algo", ["ledh", "edh"])
def test_regenerated_stream_is_the_references(algo):
    rng = np.random.default_rng(int(C5["seed"]))
    N = int(C5["n_particles"])
    Q = 0.01 * np.eye(40)
    rows = [_row(0.0, rng.multivariate_normal(np.zeros(40), np.asarray(C5["cov0"], float), size=N))]
    for f in np.asarray(C5[f"{algo}__flags"], bool):
        rows.append(_row(0.0, rng.multivariate_normal(np.zeros(40), Q, size=N)))
        if f:
            rows.append(_row(1.0, rng.random()))
    np.testing.assert_array_equal(np.array(rows), C5[f"{algo}__stream"])


@pytest.mark.parametrize("algo", ["ledh", "edh"])
def test_vectorised_oracle_reproduces_reference_at_config5(algo):
    model = LO.lorenz96(40, q_std=0.1)
    Z = np.asarray(C5["Z"], float)
    T = 4 if algo == "ledh" else len(Z)
    Z = Z[:T]
    kw = dict(mean0=np.asarray(C5["mean0"], float), cov0=np.asarray(C5["cov0"], float),
              n_particles=int(C5["n_particles"]), n_lambda_steps=int(C5["n_lambda"]), ratio=float(C5["ratio"]),
              seed=int(C5["seed"]))
    o = LO.run_ledh(model, Z, vectorized=True, **kw) if algo == "ledh" else EO.run_edh(model, Z, **kw)
    means = C5[f"{algo}__means"][:T]
    scale = max(1.0, float(np.abs(means).max()))
    assert np.max(np.abs(o["means"] - means)) <= 1e-9 * scale
    covs = C5[f"{algo}__covs"][:T]
    cs = np.maximum(1.0, np.abs(covs).max(axis=(1, 2)))[:, None, None]
    assert np.max(np.abs(o["covs"] - covs) / cs) <= 1e-8
