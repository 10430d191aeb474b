"""The persistent fp64 whole-run kernel (k_persist, particle_filters_amd/csrc/pf_persist.h) against the
launch-per-step k_step<double> loop it replaces: bitwise.

k_persist runs the T fused steps, the tail (the last update's resample) and the finalize of one
pf_run / pf_run_device call in one launch, with k_step's geometry and arithmetic: the records, the
systematic ancestors, the decisions and every output must be the bits the launch-per-step loop produces
(the reported Neff to a few ulps: the same square and division, rounded by two kernels' code)
(the default; PF_PERSIST=1 selects k_persist).  The launch-per-step loop is pinned against the
reference by the fp64 parity tests (tests/test_gpu_parity.py's replay goldens,
tests/test_gpu_teacher_forced.py::test_step_fp64_sv_config2 at 1e-12); here the cases cover what
the kernel does differently from k_step: the state carried across steps in LDS, the record granules instead of a kernel boundary, the
data flags + acquire before a gather, the in-kernel tail and finalize, a resample decided before the run
(pending), update-only first steps, partial chunks (N not a multiple of 4), several replicates, jitter.
Reference semantics: /root/reference/models/particle_filter.py:223-269 (step), 146-171 (systematic),
188-218 (resample + regularisation).
"""

import numpy as np
import pytest

import bench
from particle_filters_amd import _native as NV
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu


def _sv(T):
    wl = bench.WORKLOADS["sv"]()
    g, h, Q, R, Z, truth, mean0, cov0 = wl.build(T, 0)
    return g, h, Q, R, np.asarray(Z, float), mean0, cov0


def _run(monkeypatch, persist, *, N, T, reps=1, regularize=False, fo=False, pre_update=False, segments=(None,),
         Z=None, thresh=0.5):
    monkeypatch.setenv("PF_PERSIST", "1" if persist else "0")
    g, h, Q, R, Zs, mean0, cov0 = _sv(T)
    if Z is None:
        Z = Zs
    pf = ParticleFilterBatch(g, h, Q, R, Np=N, n_replicates=reps, seed=7, precision="fp64",
                             regularize_after_resample=regularize, resample_thresh=thresh)
    try:
        pf.initialize(mean0, cov0)
        lib = NV.load()
        out = {}
        if pre_update:  # a decision taken before the run: the run's step 0 applies it
            NV.check(lib.pf_predict(pf.handle, None, None), "pf_predict")
            info = (NV.UpdateInfo * reps)()
            z0 = np.ascontiguousarray(np.broadcast_to(Z[0], (reps, 1)), dtype=float)
            NV.check(lib.pf_update(pf.handle, NV.dptr(z0), info, None, None), "pf_update")
            out["pre_resample"] = np.array([i.resample for i in info])
            Z = Z[1:]
        t0, runs = 0, []
        for seg in segments:
            t1 = len(Z) if seg is None else seg
            r = pf.run(Z[t0:t1], first_update_only=fo and t0 == 0)
            runs.append(r)
            assert bool(lib.pf_last_run_persistent(pf.handle)) == persist
            t0 = t1
        for k in ("means", "covs", "neff", "flags", "log_norm"):
            out[k] = np.concatenate([getattr(r, k) for r in runs])
        out["x"], out["w"] = pf.particles(), pf.weights()
        out["rng"] = pf.rng_state()
    finally:
        pf.close()
    return out


def _same(a, b):
    for k in a:
        if k == "rng":
            assert a[k] == b[k]
            continue
        x, y = np.asarray(a[k]), np.asarray(b[k])
        assert x.shape == y.shape, k
        if k == "neff":
            # the reported Neff = S^2 / S2 of bitwise-equal sums: the two kernels' code generation
            # rounds that square and division differently in rare steps (<= 2 ulp measured on
            # N = 1e6 + 3, N = 5000 x 3 and N = 3e5: tools/diag_persist_diff.py,
            # profiles/r06/persist); the decisions are the flags, compared bitwise
            assert np.all(np.abs(x - y) <= 4 * np.spacing(np.abs(x))), (k, np.max(np.abs(x - y)))
            continue
        assert np.array_equal(x, y, equal_nan=True), (k, np.max(np.abs(x.astype(float) - y.astype(float))))


@pytest.mark.parametrize("case", [
    dict(N=1_000_000, T=40),                                   # config 2, fp64 line
    dict(N=1_000_000, T=40, fo=True),                          # update-only first step
    dict(N=1_000_003, T=20, thresh=0.8),                       # partial last chunk
    dict(N=5_000, T=30, reps=3, regularize=True, thresh=0.8),  # 3 tiles, replicates, jitter
    dict(N=200_000, T=25, pre_update=True, thresh=0.999),      # a resample decided before the run
    dict(N=300_000, T=30, segments=(7, 8, 19, None), thresh=0.8),  # runs back to back (tags, ring, flags)
])
def test_persist_equals_launch_per_step(monkeypatch, case):
    ref = _run(monkeypatch, False, **case)
    got = _run(monkeypatch, True, **case)
    assert np.asarray(ref["flags"]).any(), "the window should hold a resample"
    if case.get("pre_update"):
        assert ref["pre_resample"].all(), "step 0 of the run should apply a pending resample"
    _same(ref, got)


def test_persist_is_opt_in_and_uses_the_grid(monkeypatch):
    """The default fp64 run is the launch-per-step loop (k_persist is not faster at N = 1e6); with
    PF_PERSIST=1 config 2's G x R grid (k_step's 489 tiles of 2048 particles) runs co-resident."""
    g, h, Q, R, Z, mean0, cov0 = _sv(5)
    pf = ParticleFilterBatch(g, h, Q, R, Np=1_000_000, seed=7, precision="fp64")
    try:
        pf.initialize(mean0, cov0)
        monkeypatch.delenv("PF_PERSIST", raising=False)
        pf.run(Z)
        assert NV.load().pf_last_run_persistent(pf.handle) == 0
        monkeypatch.setenv("PF_PERSIST", "1")
        pf.run(Z)
        assert NV.load().pf_last_run_persistent(pf.handle) == 1
        G, tile, _ = pf.geometry()
        assert (G, tile) == (489, 2048)
    finally:
        pf.close()
