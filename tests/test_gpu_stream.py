"""The persistent many-replicate fused step (k_step_stream, pf_step_stream.h) against the
one-workgroup-per-tile k_step (PF_STREAM=0) on the same filters and Philox draws.

Per tile both kernels compute the same slots from the same operands in the same order (the fast path
and the gather-fast block of k_step, weighed against the workgroup maximum, merged by
block_sum_lds), so the runs are expected bitwise equal: decisions, means, covariances, Neff,
particles and weights.  The shapes put several tiles on every workgroup of the persistent grid, a
partial last tile, replicates that resample while others do not (different observation sequences),
jitter after resampling, the EXP_HALF and exact-SV observation kinds, a control input, and the
fallback conditions (R * G below the head threshold).
"""

import numpy as np
import pytest

from particle_filters_amd import _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def _run(monkeypatch, stream, N, R, T, reg=False, seed=7, obs="logsq", control=False):
    monkeypatch.setenv("PF_STREAM", "1" if stream else "0")
    d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=seed)
    if obs == "logsq":
        Z, h, Rm = np.log(d.Y[1:] ** 2)[:, None], M.SVLogSqObservation(1.0), [[M.LOGCHI2_VAR]]
    elif obs == "exp_half":  # the test-harness wiring h = beta e^{x/2}, R = 0.1 (EXP_HALF kernels)
        Z, h, Rm = (np.exp(0.5 * d.X[1:]) + 0.3 * d.Y[1:])[:, None], M.ExpHalfObservation(1.0), [[0.1]]
    else:  # the exact SV likelihood on the raw Y (SV_EXACT kernels)
        Z, h, Rm = d.Y[1:, None], M.SVExactObservation(1.0), None
    # per-replicate observation shifts: the replicates resample at different steps
    Zr = np.repeat(Z[:, None, :], R, axis=1) + 0.3 * np.sin(np.arange(R))[None, :, None]
    # a control input u_t (g(x, u) = alpha x + u, pf.py:237), different per replicate and step
    U = (0.05 * np.cos(0.3 * np.arange(T)[:, None, None] + np.arange(R)[None, :, None])) if control else None
    pf = ParticleFilterBatch(M.SVTransition(0.95), h, [[0.04]], Rm, Np=N,
                             n_replicates=R, seed=seed, resample_thresh=0.5, regularize_after_resample=reg)
    pf.initialize([float(d.X[0])], [[0.5]])
    res = pf.run(Zr, U)
    streamed = bool(NV.load().pf_last_step_streamed(pf.handle))
    out = dict(means=res.means.copy(), covs=res.covs.copy(), neff=res.neff.copy(), flags=res.flags.copy(),
               x=pf.particles().copy(), w=pf.weights().copy(), streamed=streamed)
    pf.close()
    return out


@pytest.mark.parametrize("N,R,reg", [(16384 - 1000, 300, False), (6000, 1024, True)])
def test_stream_equals_tile_grid(monkeypatch, N, R, reg):
    T = 40
    a = _run(monkeypatch, True, N, R, T, reg)
    b = _run(monkeypatch, False, N, R, T, reg)
    assert a["streamed"] and not b["streamed"]
    fl = a["flags"]
    assert (fl.any(axis=1) & ~fl.all(axis=1)).any(), "want steps where some replicates resample and others not"
    for k in ("flags", "means", "covs", "neff", "x", "w"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("obs,control", [("exp_half", True), ("exact", False), ("logsq", True)])
def test_stream_equals_tile_grid_models(monkeypatch, obs, control):
    """The other observation kinds the persistent kernel is instantiated for, and a control input.
    (Host-replayed noise / uniforms never reach it: pf_predict with replay normals is a predict-only
    launch, and k_step_stream runs only fused predict + update steps.)"""
    N, R, T = 6000, 1024, 30  # R x G >= 2048: the per-replicate heads, hence the persistent kernel
    a = _run(monkeypatch, True, N, R, T, obs=obs, control=control)
    b = _run(monkeypatch, False, N, R, T, obs=obs, control=control)
    assert a["streamed"] and not b["streamed"]
    assert a["flags"].any()
    for k in ("flags", "means", "covs", "neff", "x", "w"):
        assert np.array_equal(a[k], b[k]), k


def test_stream_not_used_below_head_threshold(monkeypatch):
    a = _run(monkeypatch, True, 4096, 4, 6)  # R G = 8 < 2048: no per-replicate heads, k_step
    assert not a["streamed"]
