"""Paired multi-replicate free-run parity of the large-state configurations.

BASELINE config 3 (Lorenz-96 d = 40, N = 1e5, ``k_step_grp<float,40,10>``) and config 4 (joint
16-D / 25-sensor acoustic tracking, N = 1e5, ``k_step_grp<float,16,25>``): R replicates of the
engine's native-Philox free run from initialize (seed 42, replicate ids 0..R-1, one batch launch
per step) against the fp64 oracle — the reference algorithm
(/root/reference/models/particle_filter.py:223-269, restated in oracle/pf_oracle.py and pinned to
the reference by tests/test_oracle_golden.py) on exactly the same Philox draws
(oracle/sir_philox.PhiloxSIROracle), committed as numbers in tests/golden/free_run_pairs.npz.

Per replicate: RMSE of the posterior means against the truth, the summed log normaliser (the
marginal-likelihood estimate), the resample rate and, for config 4, the notebook's OMAT.  Past the
first fp32-vs-fp64 resample-decision or ancestor flip the engine's and the oracle's replicate r
are different Monte-Carlo draws of the same filter, so the check is statistical: for every
statistic the mean of the paired differences (engine_r - oracle_r) lies within 3 standard
errors of those differences AND within the stated relative equivalence margin
(oracle/free_run.MARGINS: L96 RMSE 16 %, log-likelihood 22 %, resample rate 2 %; MAT RMSE and
OMAT 6.5 %, log-likelihood 3 %, resample rate 1.5 %), and the replicates resolve a bias of the
margin's size (3 SE / |oracle mean| <= margin).  L96: 64 replicates over config 3's T = 500; MAT:
512 replicates over the bench window.  The per-replicate pairs go to $PF_EVIDENCE_DIR (default
gpurun_out/evidence) as JSON; the round's copy is kept under profiles/.
"""

import json
import os

import numpy as np
import pytest

import bench
from oracle import free_run as FR

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fixture():
    from tests.conftest import load_golden

    return load_golden("free_run_pairs")


@pytest.mark.parametrize("name", ["l96", "mat"])
def test_paired_free_run(name, fixture):
    verdict, eng, ora = bench.paired_free_run(name, fixture=fixture)
    d = os.environ.get("PF_EVIDENCE_DIR", os.path.join("gpurun_out", "evidence"))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"free_run_pairs_{name}.json"), "w") as f:
        json.dump({"verdict": verdict, "engine": {k: v.tolist() for k, v in eng.items()},
                   "oracle": {k: v.tolist() for k, v in ora.items()}}, f, indent=1, default=float)
    for k in FR.STATS:
        if k in verdict:
            v = verdict[k]
            print(f"{name} {k}: engine {v['engine_mean']:.6g} oracle {v['oracle_mean']:.6g} "
                  f"paired diff {v['mean_paired_diff']:.3g} +- {v['se_paired_diff']:.3g} (z {v['z']:.2f}); "
                  f"relative {v['relative_diff']:.4f}, detectable {v['detectable_bias_rel']:.4f}, "
                  f"margin {v['margin_rel']}")
    assert verdict["replicates"] >= 64
    bad = [k for k in FR.STATS if k in verdict and not verdict[k]["ok"]]
    assert not bad, {k: verdict[k] for k in bad}
