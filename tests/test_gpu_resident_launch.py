"""How k_resident is launched (-m gpu): a plain launch that verifies its own co-residency, the
cooperative launch, the abort path, and resident runs of several handles on one device.

Every workgroup of k_resident waits for the others' records, so the whole grid must be
resident at once.  A plain launch (the default: ~17 us cheaper than hipLaunchCooperativeKernel)
counts its workgroups in before touching any state and aborts if the grid does not arrive
within 1 ms (pf_resident.h, res_arrival).  The test hook PF_TEST_ABORT=1 makes the check await
one workgroup more than the grid has, i.e. forces that abort.

* plain and cooperative launches compute the same thing: bitwise equal outputs;
* pf_run (host API) repeats an aborted run cooperatively: bitwise equal to an undisturbed run;
* pf_run_device reports the abort at pf_synchronize (PFRetry) with the state unchanged; the
  next run (now cooperative) continues as if the aborted one never happened;
* two handles' resident runs issued back to back on their own streams are serialised on the
  device (two partial grids would wait for each other) and equal their one-at-a-time results,
  also when both grids fill the device and their launches alternate.
"""

import ctypes as C

import numpy as np
import pytest

from particle_filters_amd import _native as NV, models as M, simulators as S
from particle_filters_amd.batch import ParticleFilterBatch

pytestmark = pytest.mark.gpu

N = 300_000
T = 60


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert NV.device_count() > 0, "no HIP device visible: -m gpu tests must run on an MI355X"


@pytest.fixture(scope="module")
def data():
    d = S.simulate_sv_1d(T + 1, 0.95, 0.2, 1.0, seed=7)
    return d.X[0], np.log(d.Y[1:] ** 2)[:, None]


def make(seed=42):
    return ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]], Np=N,
                               seed=seed)


def host_run(x0, Z, seed=42):
    pf = make(seed)
    pf.initialize([x0], [[0.5]])
    r = pf.run(Z)
    assert pf.last_run_resident
    pf.close()
    return r


def same(a, b):
    for f in ("means", "covs", "neff", "flags", "log_norm"):
        va, vb = getattr(a, f, None), getattr(b, f, None)
        if va is None and vb is None:
            continue
        assert np.array_equal(np.asarray(va), np.asarray(vb)), f


def test_plain_and_cooperative_are_bitwise_equal(data, monkeypatch):
    x0, Z = data
    monkeypatch.delenv("PF_COOP", raising=False)
    plain = host_run(x0, Z)
    monkeypatch.setenv("PF_COOP", "1")
    coop = host_run(x0, Z)
    assert plain.flags.any()
    same(plain, coop)


def test_host_run_repeats_an_aborted_launch(data, monkeypatch):
    x0, Z = data
    ref = host_run(x0, Z)
    monkeypatch.setenv("PF_TEST_HOOKS", "1")
    monkeypatch.setenv("PF_TEST_ABORT", "1")
    got = host_run(x0, Z)
    same(ref, got)


def test_abort_with_two_replicates_repeats_bitwise(data, monkeypatch):
    """Two replicates in one plain launch (advisor finding): a verified step of one replicate does
    not prove that the other replicate's workgroups arrived, so nothing is written in place until
    the whole grid has counted in.  Forced abort (the last workgroup of replicate 0 arrives late):
    pf_run repeats the run cooperatively, bitwise equal to an undisturbed run."""
    x0, Z = data

    def run():
        pf = ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                                 Np=N, n_replicates=2, seed=42)
        pf.initialize([x0], [[0.5]])
        r = pf.run(Z)
        assert pf.last_run_resident
        pf.close()
        return r

    monkeypatch.delenv("PF_TEST_ABORT", raising=False)
    ref = run()
    monkeypatch.setenv("PF_TEST_HOOKS", "1")
    monkeypatch.setenv("PF_TEST_ABORT", "1")
    got = run()
    same(ref, got)
    assert not np.array_equal(ref.means[:, 0], ref.means[:, 1])


class DeviceRun:
    """pf_run_device on torch buffers (async), outputs fetched after pf_synchronize."""

    def __init__(self, pf, Z):
        import torch
        self.torch = torch
        self.pf, self.T = pf, Z.shape[0]
        dev = torch.device("cuda", 0)
        self.dZ = torch.tensor(Z, dtype=torch.float32, device=dev).contiguous()
        self.o = [torch.zeros((self.T, 1), dtype=torch.float64, device=dev) for _ in range(3)]
        self.fl = torch.zeros((self.T, 1), dtype=torch.int32, device=dev)

    def launch(self, lo=0, hi=None):
        hi = self.T if hi is None else hi
        lib = NV.load()
        off8, off4 = lo * 8, lo * 4
        NV.check(lib.pf_run_device(self.pf.handle, C.c_void_p(self.dZ.data_ptr() + off4), None, hi - lo, 0,
                                   C.c_void_p(self.o[0].data_ptr() + off8), None,
                                   C.c_void_p(self.o[1].data_ptr() + off8), C.c_void_p(self.fl.data_ptr() + off4),
                                   C.c_void_p(self.o[2].data_ptr() + off8)))

    def sync(self):
        NV.check(NV.load().pf_synchronize(self.pf.handle))

    def result(self):
        self.torch.cuda.synchronize()
        return (self.o[0].cpu().numpy(), self.o[1].cpu().numpy(), self.fl.cpu().numpy(), self.o[2].cpu().numpy())


def test_device_run_abort_leaves_the_state_unchanged(data, monkeypatch):
    x0, Z = data
    ref_pf = make()  # the same two runs (steps [0, 20) and [20, T)) undisturbed
    ref_pf.initialize([x0], [[0.5]])
    ref_pf.run(Z[:20])
    ref = ref_pf.run(Z[20:])
    ref_pf.close()
    pf = make()
    pf.initialize([x0], [[0.5]])
    run = DeviceRun(pf, Z)
    run.launch(0, 20)  # a clean first part
    run.sync()
    monkeypatch.setenv("PF_TEST_HOOKS", "1")
    monkeypatch.setenv("PF_TEST_ABORT", "1")
    run.launch(20, T)
    with pytest.raises(NV.PFRetry):
        run.sync()
    monkeypatch.delenv("PF_TEST_ABORT")
    run.launch(20, T)  # the same steps again, now cooperatively, from the unchanged state
    run.sync()
    means, neff, flags, lse = run.result()
    assert np.array_equal(means[20:, 0], ref.means[:, 0, 0])
    assert np.array_equal(neff[20:, 0], ref.neff[:, 0])
    assert np.array_equal(flags[20:, 0] != 0, ref.flags[:, 0])
    pf.close()


def test_two_handles_back_to_back(data):
    x0, Z = data
    refs = [host_run(x0, Z, seed=s) for s in (42, 43)]
    pfs = [make(s) for s in (42, 43)]
    runs = []
    for pf in pfs:
        pf.initialize([x0], [[0.5]])
        runs.append(DeviceRun(pf, Z))
    for run in runs:  # both enqueued before either is waited for
        run.launch()
    for run in runs:
        run.sync()
    for run, ref in zip(runs, refs):
        means, neff, flags, _ = run.result()
        assert np.array_equal(means[:, 0], ref.means[:, 0, 0])
        assert np.array_equal(neff[:, 0], ref.neff[:, 0])
    for pf in pfs:
        pf.close()


def test_two_full_grids_interleaved(data):
    """Two handles whose grids each fill the device (N = 1e6: 245 workgroups, one per CU), their
    20-step device runs enqueued alternately (A, B, A, B) before any wait.  Each launch that
    follows the other stream's grid waits for it on the device through the grid-order event, which
    is recorded lazily on the previous stream at the switch (pf_order.h); two partially resident
    grids would wait for each other until the co-residency check aborts them (PFRetry).  Both runs
    equal their one-at-a-time results bitwise."""
    x0, Z = data
    Z = Z[:40]

    def mk(seed):
        return ParticleFilterBatch(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[M.LOGCHI2_VAR]],
                                   Np=1_000_000, seed=seed)

    lib = NV.load()
    refs = {}
    for s in (42, 43):
        pf = mk(s)
        pf.initialize([x0], [[0.5]])
        run = DeviceRun(pf, Z)
        for lo, hi in ((0, 20), (20, 40)):
            run.launch(lo, hi)
            run.sync()
        assert lib.pf_last_run_resident(pf.handle)
        refs[s] = run.result()
        pf.close()
    pfs = [mk(s) for s in (42, 43)]
    runs = []
    for pf in pfs:
        pf.initialize([x0], [[0.5]])
        runs.append(DeviceRun(pf, Z))
    for lo, hi in ((0, 20), (20, 40)):
        for run in runs:
            run.launch(lo, hi)
    for run in runs:
        run.sync()
    for run, s in zip(runs, (42, 43)):
        for a, b in zip(run.result(), refs[s]):
            assert np.array_equal(a, b)
    assert refs[42][2].any(), "want resample steps in the window"
    for pf in pfs:
        pf.close()


def test_entry_header_matches_the_records_prologue(data, monkeypatch):
    """A resident run that follows a resident run takes the previous exit's header (log sum of
    the exit weights = the last verified mass in the exit frame) instead of reducing the
    records; PF_RES_HDR=0 forces the prologue.  Both describe the same normaliser up to fp32
    rounding of the log-weights: same decisions, means within 1e-5, Neff rel 1e-5."""
    x0, Z = data
    out = {}
    for hdr in ("1", "0"):
        monkeypatch.setenv("PF_RES_HDR", hdr)
        pf = make()
        pf.initialize([x0], [[0.5]])
        pf.run(Z[:23])
        out[hdr] = pf.run(Z[23:])
        pf.close()
    a, b = out["1"], out["0"]
    assert np.array_equal(a.flags, b.flags)
    np.testing.assert_allclose(a.means, b.means, rtol=0, atol=1e-5)
    np.testing.assert_allclose(a.neff, b.neff, rtol=1e-5)
    np.testing.assert_allclose(a.log_norm, b.log_norm, rtol=0, atol=1e-5)
