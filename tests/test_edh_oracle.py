"""The EDH oracle (oracle/edh_oracle.py) against the reference's own outputs.

tests/golden/edh_runs.npz was produced by running the reference EDHFlowPF + EKF
(tests/golden/make_golden_edh.py).  The faithful oracle must reproduce it bit-for-bit,
the vectorised one to fp64 rounding.
"""

import os

import numpy as np
import pytest

from oracle import edh_oracle as EO
from oracle import ledh_oracle as LO

HERE = os.path.dirname(__file__)
GOLD = np.load(os.path.join(HERE, "golden", "edh_runs.npz"))
NAMES = [str(n) for n in GOLD["names"]]


def edh_case(name):
    g = {k.split("__", 1)[1]: GOLD[k] for k in GOLD.files if k.startswith(name + "__")}
    mat = np.load(os.path.join(HERE, "golden", "mat_data.npz"))
    if name.startswith("lin1d"):
        model = LO.linear_1d()
    elif name == "sv_exp":
        model = LO.sv_exp_half(0.95, 0.2, 1.0, 0.1)
    elif name == "acoustic":
        model = LO.acoustic_single(mat["S2"], psi=float(mat["meta2"][2]), d0=float(mat["meta2"][3]))
    else:
        model = LO.lorenz96(40)
    return model, g


def run(model, g, vectorized):
    return EO.run_edh(model, g["Z"], mean0=g["mean0"], cov0=g["cov0"], n_particles=int(g["n_particles"]),
                      n_lambda_steps=int(g["n_lambda"]), ratio=float(g["ratio"]), seed=int(g["seed"]),
                      integrator=str(g["integrator"]), vectorized=vectorized)


@pytest.mark.parametrize("name", NAMES)
def test_faithful_edh_oracle_bitwise(name):
    model, g = edh_case(name)
    o = run(model, g, vectorized=False)
    np.testing.assert_array_equal(o["init_particles"], g["init_particles"])
    np.testing.assert_array_equal(o["means"], g["means"])
    np.testing.assert_array_equal(o["covs"], g["covs"])
    np.testing.assert_array_equal(o["final_particles"], g["particles"][-1])
    np.testing.assert_array_equal(o["flags"], g["flags"])
    np.testing.assert_array_equal(o["conds"], g["conds"])


@pytest.mark.parametrize("name", NAMES)
def test_vectorized_edh_oracle_close(name):
    model, g = edh_case(name)
    o = run(model, g, vectorized=True)
    scale = max(1.0, float(np.max(np.abs(g["means"]))))
    np.testing.assert_allclose(o["means"], g["means"], rtol=0, atol=1e-9 * scale)
    np.testing.assert_array_equal(o["flags"], g["flags"])
