"""The diagnostics oracle (oracle/diag_oracle.py) against the reference's own outputs.

tests/golden/diag_cases.npz was produced by executing the reference notebook's diagnostic
functions (tests/golden/make_golden_diag.py); the restatement must reproduce them bit-for-bit.
"""

import os

import numpy as np
import pytest

from oracle import diag_oracle as DO

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "diag_cases.npz"))
NAMES = [str(n) for n in GOLD["names"]]


def gcase(name):
    return {k.split("__", 1)[1]: GOLD[k] for k in GOLD.files if k.startswith(name + "__")}


@pytest.mark.parametrize("name", NAMES)
def test_diag_oracle_bitwise(name):
    g = gcase(name)
    w, x = g["w"], g["x"]
    assert DO.weight_entropy(w, True) == g["entropy"]
    if "entropy_raw" in g:
        assert DO.weight_entropy(w, False) == g["entropy_raw"]
    assert DO.gini_coefficient(w) == g["gini"]
    assert DO.unique_particles(x) == int(g["n_unique"])
    if "cov" in g:
        d = DO.diagnostics(w, x, g["cov"])
        for key in ("ess", "max_weight", "posterior_spread"):
            assert d[key] == g[key], key
