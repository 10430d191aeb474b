"""The register-resident whole-run kernel (k_resident, pf_resident.h) vs the
launch-per-step loop (k_step, PF_RESIDENT=0) on identical Philox noise.

Both run the same filter with the same counter-based draws; they differ only in
how the reductions are grouped (4096- vs 1024-particle tiles, a lagged uniform
renormalisation) — fp32 rounding.  Tolerances (fp32 engine):

* until the first resample: means / covariances within 1e-5 abs (x ~ O(1)),
  Neff rel 1e-5, log-normaliser 1e-5 abs, decisions identical;
* after it: an fp32 weight moves by ~1e-7, which at N=1e5..1e6 hands a few of the
  N slots to a neighbouring ancestor and the trajectories then decorrelate at the
  Monte-Carlo level, so the whole run is compared statistically: resample
  decisions agree on >= 97% of steps and RMSE vs truth within 3x the MC floor;
* the exit state (particles, weights, records) hands over to the step API.
"""

import numpy as np
import pytest

from particle_filters_amd import models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    from particle_filters_amd import _native
    assert _native.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def sv_data(T, seed=42):
    d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=seed)
    return d.X, np.log(d.Y[1:] ** 2)[:, None]


def make(N, R=1, reg=False, thresh=0.5, h=None, seed=42, precision="fp32"):
    h = h or M.SVLogSqObservation(1.0)
    Rm = [[M.LOGCHI2_VAR]] if isinstance(h, M.SVLogSqObservation) else [[0.1]]
    return ParticleFilterBatch(M.SVTransition(0.95), h, [[0.04]], Rm, Np=N, n_replicates=R, seed=seed,
                               regularize_after_resample=reg, resample_thresh=thresh, precision=precision)


def both(monkeypatch, N, Z, X0, U=None, fo=False, **kw):
    out = {}
    for resident in (True, False):
        monkeypatch.setenv("PF_RESIDENT", "1" if resident else "0")
        pf = make(N, **kw)
        pf.initialize([X0], [[0.5]])
        res = pf.run(Z, U, first_update_only=fo)
        assert pf.last_run_resident == resident
        out[resident] = (pf, res)
    return out


def check_prefix(a, b, label):
    """a, b: RunResult.  Exact-path agreement up to the first resample."""
    fa, fb = a.flags[:, 0], b.flags[:, 0]
    assert fa.any(), f"{label}: no resample in the run"
    first = int(np.argmax(fa | fb))
    assert fa[first] == fb[first], f"{label}: first decision differs at step {first}"
    k = first  # steps strictly before the first resample
    dm = np.max(np.abs(a.means[:k] - b.means[:k]), initial=0.0)
    dc = np.max(np.abs(a.covs[:k] - b.covs[:k]), initial=0.0)
    dn = np.max(np.abs(a.neff[:k + 1] / b.neff[:k + 1] - 1))
    dl = np.max(np.abs(a.log_norm[:k + 1] - b.log_norm[:k + 1]))
    print(f"{label}: first resample {first}; max|dmean| {dm:.2e} |dcov| {dc:.2e} rel dNeff {dn:.2e} |dlse| {dl:.2e}")
    assert dm <= 1e-5 and dc <= 1e-5 and dn <= 1e-5 and dl <= 1e-5
    return first


@pytest.mark.parametrize("N,reg", [(200_003, False), (200_003, True), (4096 * 3 + 5, False), (1000, True)])
def test_resident_matches_launch_per_step(monkeypatch, N, reg):
    X, Z = sv_data(300)
    o = both(monkeypatch, N, Z, X[0], reg=reg, thresh=0.7)
    a, b = o[True][1], o[False][1]
    check_prefix(a, b, f"N={N} reg={reg}")
    agree = np.mean(a.flags == b.flags)
    ra, rb = float(a.rmse(X[1:])[0]), float(b.rmse(X[1:])[0])
    print(f"N={N}: decisions agree {agree:.4f}; resamples {a.flags.sum()} / {b.flags.sum()}; RMSE {ra:.6f} {rb:.6f}")
    assert agree >= 0.97
    assert abs(ra - rb) <= 3 * 1.1e-4 * np.sqrt(1e6 / N)  # 3x the seed-to-seed RMSE spread at this N
    # exit state: normalised weights, particles on the same support
    pa, pb = o[True][0], o[False][0]
    wa = pa.weights()[0]
    assert abs(wa.sum() - 1.0) < 1e-6 and np.all(wa >= 0)
    xa = pa.particles()[0, :, 0]
    assert np.all(np.isfinite(xa))
    ma, mb = np.sum(wa * xa), np.sum(pb.weights()[0] * pb.particles()[0, :, 0])
    assert abs(ma - mb) < 0.2


def test_resident_replicates_and_partial_tile(monkeypatch):
    """R replicates in one launch (grid y), N not a multiple of the 4096-particle tile."""
    X, Z = sv_data(200)
    o = both(monkeypatch, 50_001, Z, X[0], R=3, thresh=0.7)
    a, b = o[True][1], o[False][1]
    for r in range(3):
        ar = type(a)(a.means[:, r:r + 1], a.covs[:, r:r + 1], a.neff[:, r:r + 1], a.flags[:, r:r + 1],
                     a.log_norm[:, r:r + 1], a.ess[:, r:r + 1])
        br = type(b)(b.means[:, r:r + 1], b.covs[:, r:r + 1], b.neff[:, r:r + 1], b.flags[:, r:r + 1],
                     b.log_norm[:, r:r + 1], b.ess[:, r:r + 1])
        check_prefix(ar, br, f"replicate {r}")
    assert not np.array_equal(a.means[:, 0], a.means[:, 1])


def test_resident_first_update_only_and_controls(monkeypatch):
    """The notebook driver (update(Z[0]) first, no predict) and additive controls u."""
    X, Z = sv_data(150)
    U = 0.01 * np.sin(np.arange(150))[:, None]
    for fo, u in ((True, None), (False, U), (True, U)):
        o = both(monkeypatch, 100_000, Z, X[0], U=u, fo=fo, thresh=0.7)
        check_prefix(o[True][1], o[False][1], f"first_update_only={fo} controls={u is not None}")


def test_resident_exp_half_wiring(monkeypatch):
    """The test-harness wiring h = beta exp(x/2), R = 0.1 (frequent resampling)."""
    X, Z0 = sv_data(200)
    d = S.simulate_sv_1d(201, 0.95, 0.2, 1.0, seed=42)
    Z = d.Y[1:, None]
    o = both(monkeypatch, 100_000, Z, X[0], h=M.ExpHalfObservation(1.0), thresh=0.2)
    a, b = o[True][1], o[False][1]
    check_prefix(a, b, "exp-half")
    assert np.mean(a.flags == b.flags) >= 0.95


def test_resident_hands_state_to_step_api(monkeypatch):
    """After a resident run, the step API continues from the exit state (records in
    the launch-per-step layout): same decisions and moments as after a
    launch-per-step run, to fp32 rounding, for the steps before any resample."""
    X, Z = sv_data(120)
    means = {}
    for resident in (True, False):
        monkeypatch.setenv("PF_RESIDENT", "1" if resident else "0")
        pf = make(100_000, thresh=0.3)
        pf.initialize([X[0]], [[0.5]])
        r1 = pf.run(Z[:20])
        monkeypatch.setenv("PF_RESIDENT", "0")
        r2 = pf.run(Z[20:40])  # launch-per-step continuation reads the exit records
        means[resident] = (r1, r2)
    a1, b1 = means[True][0], means[False][0]
    a2, b2 = means[True][1], means[False][1]
    assert not a1.flags.any() and not b1.flags.any(), "pick a window without resampling"
    np.testing.assert_allclose(a1.means, b1.means, atol=1e-5)
    k = int(np.argmax(a2.flags[:, 0] | b2.flags[:, 0])) if (a2.flags.any() or b2.flags.any()) else 20
    np.testing.assert_allclose(a2.means[:k], b2.means[:k], atol=1e-5)
    np.testing.assert_allclose(a2.neff[:k + 1], b2.neff[:k + 1], rtol=1e-5)


def test_resident_bench_config(monkeypatch):
    """BASELINE config 2 (N=1e6, T=999): the resident path runs, and its RMSE vs truth
    is within 1e-4 of the launch-per-step path's on the same noise."""
    from tests.conftest import load_golden
    g = load_golden("sv_data")
    X, Y = g["X0"], g["Y0"]
    Z = np.log(Y[1:] ** 2)[:, None]
    o = both(monkeypatch, 1_000_000, Z, X[0])
    a, b = o[True][1], o[False][1]
    ra, rb = float(a.rmse(X[1:])[0]), float(b.rmse(X[1:])[0])
    print(f"N=1e6: RMSE resident {ra:.7f} launch-per-step {rb:.7f}; decisions agree {np.mean(a.flags == b.flags):.4f}")
    assert abs(ra - rb) <= 1e-4
    assert np.mean(a.flags == b.flags) >= 0.99


def test_resident_replicate_groups_are_bitwise_single_replicates(golden_sv):
    """R replicates whose grids do not all fit co-resident run as sequential groups of the
    resident kernel: every replicate is bitwise the single-replicate run with the same Philox
    replicate id (the path does not depend on R or on the multi-GPU sharding)."""
    from particle_filters_amd import _native as NV
    Z = np.log(golden_sv["Y0"][1:150] ** 2)[:, None]
    kw = dict(Np=200_000, seed=31, resample_thresh=0.5)
    big = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                              n_replicates=8, **kw)  # 8 x 49 workgroups > 256 co-resident
    big.initialize([0.0], [[0.5]])
    rb = big.run(Z)
    assert NV.load().pf_last_run_resident(big.handle)
    for r in (0, 5, 7):
        one = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                                  n_replicates=1, replicate_base=r, **kw)
        one.initialize([0.0], [[0.5]])
        ro = one.run(Z)
        assert NV.load().pf_last_run_resident(one.handle)
        assert np.array_equal(ro.means[:, 0], rb.means[:, r])
        assert np.array_equal(ro.neff[:, 0], rb.neff[:, r])
        assert np.array_equal(ro.flags[:, 0], rb.flags[:, r])
        assert np.array_equal(one.particles()[0], big.particles()[r])
        one.close()
    assert rb.flags.sum() >= 8
    big.close()
