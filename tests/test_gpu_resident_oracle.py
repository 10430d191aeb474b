"""The benchmarked kernel against the oracle, head-on (run on an MI355X: -m gpu).

BASELINE config 2 — SV log-squared wiring, N = 1e6, T = 999, seed 42 — run by the
register-resident whole-run kernel (``k_resident``, the kernel bench.py times), and
the fp64 oracle (oracle/sir_philox.c: the reference algorithm, particle_filter.py
:110-269, pinned to the NumPy oracle and through it to the reference's own outputs)
fed the SAME Philox draws (oracle/sir_philox.py restates the engine's counter /
epoch mapping).  Stated tolerances (SURVEY 8c "stated tolerance proposal"):

* teacher-forced (the oracle takes the engine's resample decisions): before the first
  resample every step's posterior mean within 1e-5 abs and Neff within rel 1e-4 (fp32
  arithmetic only); from then on fp32 rounding moves a few systematic-resampling slots to
  neighbouring ancestors (tests/oracle_compare.py), so the per-step differences are held to
  the filter's own Monte-Carlo error, measured by an independent-seed oracle run (RMS at
  most 0.75 of it), Neff within rel 5e-2; a decision the oracle would have taken
  differently is legitimate only where its Neff is within 1e-3 N of the 0.5 N threshold
  (SURVEY 8c(iv));
* free run (the oracle decides itself): RMSE vs truth within 1e-4 of the engine's
  over all 999 steps at N = 1e6 (the BASELINE.json north-star tolerance).
"""

import numpy as np
import pytest

from particle_filters_amd import _native as NV, models as M
from particle_filters_amd.batch import ParticleFilterBatch
from oracle import sir_philox as SP
from tests.oracle_compare import check_forced, forced_compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def _engine_run(Z, X0, N, seed=42, reg=False):
    b = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=N,
                            seed=seed, precision="fp32", regularize_after_resample=reg)
    b.initialize([X0], [[0.5]])
    r = b.run(Z[:, None])
    resident = bool(NV.load().pf_last_run_resident(b.handle))
    b.close()
    return r, resident


def _compare(r, Z, X, N, seed=42, reg=False, check_rmse=True):
    m = SP.sv_logsq_model(0.95, 0.2, 1.0)
    c = forced_compare(r.means[:, 0, 0], r.neff[:, 0], r.flags[:, 0], m, Z, N=N, seed=seed, mean0=X[0], var0=0.5,
                       reg=reg)
    free = SP.run_scalar(m, Z, N=N, seed=seed, mean0=X[0], var0=0.5, bm24=True, regularize=reg)
    truth = X[1:len(Z) + 1]
    r_e = float(np.sqrt(np.mean((r.means[:, 0, 0] - truth) ** 2)))
    r_o = float(np.sqrt(np.mean((free["means"] - truth) ** 2)))
    print(f"N={N} T={len(Z)}: {c['summary']}; free run RMSE engine {r_e:.9f} oracle {r_o:.9f} "
          f"|d| {abs(r_e - r_o):.2e}, free-run decision flips {int(np.sum(free['flags'] != r.flags[:, 0]))}")
    check_forced(c)
    if check_rmse:
        assert abs(r_e - r_o) <= 1e-4


def test_resident_kernel_vs_oracle_bench_config(golden_sv):
    X, Y = golden_sv["X0"], golden_sv["Y0"]
    Z = np.log(Y[1:] ** 2)
    N = 1_000_000
    r, resident = _engine_run(Z, X[0], N)
    assert resident, "BASELINE config 2 must run on the register-resident kernel"
    _compare(r, Z, X, N)


def test_resident_kernel_vs_oracle_regularised_small(golden_sv):
    """Jitter after resampling (pf.py:212-218) and a partial last workgroup tile."""
    X, Y = golden_sv["X0"], golden_sv["Y0"]
    Z = np.log(Y[1:400] ** 2)
    N = 300_001
    r, resident = _engine_run(Z, X[0], N, seed=7, reg=True)
    assert resident
    _compare(r, Z, X, N, seed=7, reg=True, check_rmse=False)  # the 1e-4 RMSE target is stated at N = 1e6
