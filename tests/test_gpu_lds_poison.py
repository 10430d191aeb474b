"""Uninitialised-LDS regression (round-5 verdict item 2).

A kernel that reads an LDS word it did not write gets whatever the previous kernel on that CU left
there.  Round 5 found one such read in the fused LEDH step (P4 multiplied LDS rows past a
workgroup's last particle by a zero weight: 0 x NaN = NaN when the leftover happened to be a NaN);
a green run does not show such a read is gone, because the leftovers are usually finite.

Here the leftovers are made hostile: with PF_TEST_HOOKS=1 and PF_TEST_LDS_POISON=1 the engine
launches ``k_lds_poison`` (0xFFFFFFFF - a NaN as fp32 and fp64 - over the whole 160 KB of LDS of
every CU) on the stream right before every launch of the kernels that stage data in LDS:
``k_step_grp`` (L96, MAT; also ``k_step`` for the small states), ``k_cov_part``,
``k_ledh_fused`` (LEDH and EDH device loop), ``k_flow_wave_lr`` / ``k_flow_wave`` (per-particle
flow) and ``k_ekf_seq`` (device tracker).  Each run uses a particle count that is not a multiple
of the kernel's per-workgroup particle count, so partial tiles exist, and must give finite outputs
bitwise equal to the same run without the poison (reference semantics: weights and statistics over
the valid particles only, /root/reference/models/LEDH_particle_filter.py:191-209,
models/particle_filter.py:239-269).
"""

import numpy as np
import pytest

import bench
from particle_filters_amd import _native as NV
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu


@pytest.fixture
def poison(monkeypatch):
    def on():
        monkeypatch.setenv("PF_TEST_HOOKS", "1")
        monkeypatch.setenv("PF_TEST_LDS_POISON", "1")

    def off():
        monkeypatch.delenv("PF_TEST_LDS_POISON", raising=False)

    off()
    return on, off


def test_poison_reaches_every_cu():
    """The mechanism itself: after k_lds_poison, workgroups of a new launch find the pattern in their
    uninitialised LDS on every CU (4 workgroups per CU, whole 160 KB allocations)."""
    lib = NV.load()
    NV.check(lib.pf_test_lds_poison(None), "pf_test_lds_poison")
    nb = lib.pf_test_lds_probe_blocks()
    out = np.full(nb, -1, dtype=np.int32)
    NV.check(lib.pf_test_lds_probe(None, out.ctypes.data_as(NV.C.POINTER(NV.C.c_int32))), "pf_test_lds_probe")
    assert nb >= 4 * 256 - 64
    assert np.all(out == 0), f"{np.count_nonzero(out)} of {nb} workgroups saw non-poisoned LDS words"


def _poisoned(fn):
    """fn() with the hook on; asserts the engine did launch the poison in front of its kernels."""
    lib = NV.load()
    c0 = lib.pf_test_lds_poison_count()
    out = fn()
    assert lib.pf_test_lds_poison_count() > c0, "the poison hook never fired"
    return out


def _same(a, b):
    for k in a:
        x, y = np.asarray(a[k]), np.asarray(b[k])
        if x.dtype.kind == "f":
            assert np.all(np.isfinite(x)), k
        assert np.array_equal(x, y), (k, np.max(np.abs(x.astype(float) - y.astype(float))))


@pytest.mark.parametrize("name", ["l96", "mat"])
def test_group_step_and_covariance_poisoned(name, poison):
    """k_step_grp (8 lanes per particle for L96, 4 for MAT) and k_cov_part over N = 1001 particles
    (partial last tile), with resampling and the per-step covariance."""
    on, off = poison
    wl = bench.WORKLOADS[name]()
    T = 12
    g, h, Q, R, Z, truth, mean0, cov0 = wl.build(T, 0)
    reps = 1 if name == "l96" else 2

    def run():
        pf = ParticleFilterBatch(g, h, Q, R, Np=1001, n_replicates=reps, seed=7)
        try:
            pf.initialize(mean0, cov0)
            r = pf.run(np.asarray(Z[:T], float), with_cov=True)
            x, w = pf.particles(), pf.weights()
        finally:
            pf.close()
        return {"means": r.means, "covs": r.covs, "neff": r.neff, "flags": r.flags, "lnorm": r.log_norm,
                "x": x, "w": w}

    off()
    lib = NV.load()
    c0 = lib.pf_test_lds_poison_count()
    ref = run()
    assert lib.pf_test_lds_poison_count() == c0
    on()
    got = _poisoned(run)
    off()
    assert np.asarray(ref["flags"]).any(), "the window should hold a resample"
    _same(ref, got)


def _flow_run(algo, name, n, tracker):
    from tests import test_gpu_edh as TE
    from tests import test_gpu_ledh as TL

    if tracker == "device":  # the tracker on the engine's own models (analytic Jacobians)
        pf, _, _, gd = TL.device_tracked_filter(name, n_particles=n, seed=11)
    else:
        make = TL.make_filter if algo == "ledh" else TE.make_filter
        pf, _, _, gd = make(name, rng_mode="device", n_particles=n, seed=11)
    st = pf.init_from_gaussian(gd["mean0"], gd["cov0"])
    res = pf.run(st, gd["Z"], process_noise="device", tracker=tracker)
    return {"means": res.means, "covs": res.covs, "ess": res.ess, "flags": res.flags}


@pytest.mark.parametrize("algo,name,n,tracker", [
    ("ledh", "l96", 1000, "host"),      # k_ledh_fused (LEDH), 64-slot workgroups: 15 full + 40
    ("ledh", "l96", 1000, "device"),    # + k_ekf_seq
    ("edh", "l96_rk4", 1000, "host"),   # k_ledh_fused (EDH composed flow)
    ("ledh", "acoustic", 100, "host"),  # k_flow_wave_lr (acoustic h, one particle per wave)
])
def test_flow_kernels_poisoned(algo, name, n, tracker, poison):
    on, off = poison
    off()
    ref = _flow_run(algo, name, n, tracker)
    on()
    got = _poisoned(lambda: _flow_run(algo, name, n, tracker))
    off()
    _same(ref, got)
