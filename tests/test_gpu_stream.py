"""The persistent many-replicate fused step (k_step_stream, pf_step_stream.h) against the
one-workgroup-per-tile k_step (PF_STREAM=0) on the same filters and Philox draws.

Per tile both kernels compute the same slots from the same operands in the same order (the fast path
and the gather-fast block of k_step, weighed against the workgroup maximum, merged by
block_sum_lds), so the runs are expected bitwise equal: decisions, means, covariances, Neff,
particles and weights.  The shapes put several tiles on every workgroup of the persistent grid, a
partial last tile, replicates that resample while others do not (different observation sequences),
jitter after resampling, and the fallback conditions (R * G below the head threshold).
"""

import numpy as np
import pytest

from particle_filters_amd import _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def _run(monkeypatch, stream, N, R, T, reg=False, seed=7):
    monkeypatch.setenv("PF_STREAM", "1" if stream else "0")
    d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=seed)
    Z = np.log(d.Y[1:] ** 2)[:, None]
    # per-replicate observation shifts: the replicates resample at different steps
    Zr = np.repeat(Z[:, None, :], R, axis=1) + 0.3 * np.sin(np.arange(R))[None, :, None]
    pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=N,
                             n_replicates=R, seed=seed, resample_thresh=0.5, regularize_after_resample=reg)
    pf.initialize([float(d.X[0])], [[0.5]])
    res = pf.run(Zr)
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


def test_stream_not_used_below_head_threshold(monkeypatch):
    a = _run(monkeypatch, True, 4096, 4, 6)  # R G = 8 < 2048: no per-replicate heads, k_step
    assert not a["streamed"]
