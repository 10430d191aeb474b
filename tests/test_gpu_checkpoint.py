"""Checkpoint / resume and the Philox position, -m gpu.

``pf_checkpoint`` snapshots the whole filter state at a step boundary (particles and unnormalised
log-weights in the engine precision, tile records, the systematic-CDF prefix, the resident
kernel's entry header, the Philox position); ``pf_restore`` into a fresh handle of the same
configuration must continue BIT FOR BIT as the original handle does - on every step path:
the register-resident kernel (SV), the large-state lane-group step (L96, with its CDF prefix),
replicate batches (MAT), fp64, multinomial resampling with jitter, and the step API.
"""

import numpy as np
import pytest

import bench
from particle_filters_amd import ParticleFilter, _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


def _same(a, b):
    for f in ("means", "covs", "neff", "flags", "log_norm"):
        va, vb = getattr(a, f), getattr(b, f)
        if va is None and vb is None:
            continue
        assert np.array_equal(va, vb), f


def _resume_case(make, init, Z, cut):
    ref = make()
    init(ref)
    ref.run(Z[:cut])
    rest_ref = ref.run(Z[cut:])
    a = make()
    init(a)
    a.run(Z[:cut])
    blob = a.checkpoint()
    st_a = a.rng_state()
    a.close()
    b = make()
    b.restore(blob)
    assert b.rng_state()["epoch"] == st_a["epoch"]
    rest = b.run(Z[cut:])
    _same(rest_ref, rest)
    assert np.array_equal(ref.particles(), b.particles())
    ref.close()
    b.close()
    return rest


@pytest.mark.parametrize("name,T,cut,kw", [
    ("sv", 60, 23, {}),
    ("sv", 60, 23, dict(precision="fp64")),
    ("sv", 40, 17, dict(resample_method="multinomial", regularize_after_resample=True, resample_thresh=0.9)),
    ("l96", 30, 11, {}),
    ("mat", 12, 5, {}),
])
def test_checkpoint_resume_is_bitwise(name, T, cut, kw):
    wl = bench.WORKLOADS[name]()
    g, h, Q, R, Z, truth, mean0, cov0 = wl.build(T, 0)
    Np = min(wl.n_particles, 300_000)
    Z = np.asarray(Z, float).reshape(T, -1)

    def make():
        return ParticleFilterBatch(g, h, Q, R, Np=Np, n_replicates=wl.replicates, seed=42, **kw)

    rest = _resume_case(make, lambda pf: pf.initialize(mean0, cov0), Z, cut)
    assert rest.flags.any()


def test_resident_resume_uses_the_entry_header():
    """The SV resident kernel: resumed run == continued run bitwise (the restored exit header),
    and the epoch bookkeeping: initialize draws at 1, a T-step run advances 2T."""
    d = S.simulate_sv_1d(61, 0.95, 0.2, 1.0, seed=7)
    Z = np.log(d.Y[1:] ** 2)[:, None]

    def make():
        return ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                                   Np=300_000, seed=42)

    pf = make()
    pf.initialize([d.X[0]], [[0.5]])
    assert pf.rng_state()["epoch"] == 2
    pf.run(Z[:10])
    assert pf.last_run_resident
    assert pf.rng_state()["epoch"] == 22
    pf.close()
    _resume_case(make, lambda p: p.initialize([d.X[0]], [[0.5]]), Z, 23)


def test_step_api_checkpoint_and_host_rng():
    """ParticleFilter.checkpoint() also carries the host Generator (rng_mode='host'): a restored
    filter replays the reference's draw stream from the same position."""
    d = S.simulate_sv_1d(41, 0.95, 0.2, 1.0, seed=3)
    Z = np.log(d.Y[1:] ** 2)[:, None]

    def make(seed):
        return ParticleFilter(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=2000,
                              rng=np.random.default_rng(seed), rng_mode="host", precision="fp64",
                              regularize_after_resample=True)

    a = make(5)
    a.initialize([d.X[0]], [[0.5]])
    for z in Z[:15]:
        a.step(z)
    ck = a.checkpoint()
    ref = [a.step(z).mean.copy() for z in Z[15:]]
    b = make(99)  # a different generator: restore must bring the checkpoint's position
    b.restore(ck)
    assert b.state.t == 15
    got = [b.step(z).mean.copy() for z in Z[15:]]
    assert np.array_equal(np.array(ref), np.array(got))


def test_restore_rejects_another_configuration():
    wl = bench.WORKLOADS["sv"]()
    g, h, Q, R, Z, truth, mean0, cov0 = wl.build(5, 0)
    a = ParticleFilterBatch(g, h, Q, R, Np=4096, seed=1)
    a.initialize(mean0, cov0)
    blob = a.checkpoint()
    for kw in (dict(Np=8192), dict(Np=4096, precision="fp64"), dict(Np=4096, n_replicates=2)):
        b = ParticleFilterBatch(g, h, Q, R, seed=1, **kw)
        with pytest.raises(ValueError):
            b.restore(blob)
        b.close()
    with pytest.raises(ValueError):
        a.restore(blob[:100])
    a.close()


def test_set_rng_state_moves_the_draws():
    """Two handles at the same state and Philox position draw identically; a moved epoch does not."""
    wl = bench.WORKLOADS["sv"]()
    g, h, Q, R, Z, truth, mean0, cov0 = wl.build(8, 0)
    a = ParticleFilterBatch(g, h, Q, R, Np=8192, seed=5)
    b = ParticleFilterBatch(g, h, Q, R, Np=8192, seed=6)
    a.initialize(mean0, cov0)
    blob = a.checkpoint()
    b.restore(blob)  # also takes seed 5
    ra, rb = a.run(Z), b.run(Z)
    assert np.array_equal(ra.means, rb.means)
    b.restore(blob)
    st = b.rng_state()
    st["epoch"] += 2
    b.set_rng_state(st)
    rc = b.run(Z)
    assert not np.array_equal(ra.means, rc.means)
    a.close()
    b.close()
