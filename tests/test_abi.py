"""CPU checks of the C-ABI boundary (no GPU, no compute calls).

* libpf_hip.so loads and exports every function include/pf_engine.h declares,
  and the ctypes binding (particle_filters_amd/_native.py) covers exactly that set;
* host-only entry points (version, model registry, argument validation in
  pf_create) answer without a device;
* the status -> exception mapping mirrors the reference's error behaviour
  (particle_filter.py:142,231,252 AssertionError; LinAlgError for non-PD).
"""

import ctypes as C
import os
import re

import numpy as np
import pytest

from particle_filters_amd import _native as NV
from particle_filters_amd import models as M

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h) for h in ("pf_engine.h", "pf_ledh.h", "pf_edh.h", "pf_diag.h", "pf_shard.h")]


def header_functions():
    names = []
    for hdr in HEADERS:
        src = open(hdr).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(pf_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_parses_all_entry_points():
    names = header_functions()
    assert len(names) >= 30
    for must in ("pf_create", "pf_destroy", "pf_initialize", "pf_predict", "pf_update", "pf_resample",
                 "pf_run", "pf_run_device", "pf_resample_indices", "pf_last_error",
                 "pf_ledh_create", "pf_ledh_init", "pf_ledh_step", "pf_ledh_finish", "pf_ledh_run"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(NV.LIB_PATH)
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, f"declared in include/*.h but not exported: {missing}"


def test_binding_covers_header_exactly():
    assert sorted(NV.SIGNATURES) == header_functions()
    lib = NV.load()
    for n in NV.SIGNATURES:
        assert getattr(lib, n).argtypes is not None or NV.SIGNATURES[n][1] == []


def test_exports_are_plain_c_symbols():
    # extern "C": no C++ mangling on the ABI surface
    lib = C.CDLL(NV.LIB_PATH)
    for n in header_functions():
        assert C.cast(getattr(lib, n), C.c_void_p).value


def test_version_string():
    v = NV.load().pf_version().decode()
    assert re.search(r"\d+\.\d+", v) and "gfx950" in v, v


def test_model_registry():
    lib = NV.load()
    # compiled instantiations (pf_inst_*.hip)
    assert lib.pf_model_supported(1, 1, NV.PF_TRANS_LINEAR, NV.PF_OBS_LINEAR)
    assert lib.pf_model_supported(1, 1, NV.PF_TRANS_LINEAR, NV.PF_OBS_EXP_HALF)
    assert lib.pf_model_supported(3, 3, NV.PF_TRANS_LINEAR, NV.PF_OBS_EXP_HALF)
    assert lib.pf_model_supported(40, 10, NV.PF_TRANS_L96, NV.PF_OBS_LINEAR)
    assert lib.pf_model_supported(16, 25, NV.PF_TRANS_LINEAR, NV.PF_OBS_ACOUSTIC)
    assert not lib.pf_model_supported(7, 3, NV.PF_TRANS_L96, NV.PF_OBS_ACOUSTIC)
    assert M.supported(M.SVTransition(0.95), M.SVLogSqObservation(1.0))
    assert M.supported(M.L96Transition(8.0, 0.01, 40), M.SelectObservation(np.arange(0, 40, 4), 40))


def _create(g, h, Q, R, **kw):
    d, keep = M.describe(g, h, np.asarray(Q, float), np.asarray(R, float))
    o = dict(n_particles=100, n_replicates=1, resample_method=0, resample_thresh=0.5, regularize=0,
             precision=0, seed=1, device=0, replicate_base=0, kernel_path=0)
    o.update(kw)
    opts = NV.Opts(**o)
    h_ = C.c_void_p()
    st = NV.load().pf_create(C.byref(d), C.byref(opts), C.byref(h_))
    return st, h_


def test_create_rejects_bad_arguments_before_touching_a_device():
    g, h = M.SVTransition(0.95), M.SVLogSqObservation(1.0)
    st, hd = _create(g, h, [[0.04]], [[1.0]], n_particles=0)
    assert st == NV.PF_E_ARG and not hd.value
    assert "n_particles" in NV.load().pf_last_error().decode()
    st, _ = _create(g, h, [[0.04]], [[1.0]], n_replicates=0)
    assert st == NV.PF_E_ARG
    st, _ = _create(g, h, [[0.04]], [[1.0]], precision=7)
    assert st == NV.PF_E_ARG
    with pytest.raises(ValueError):
        NV.check(st)


def test_create_unsupported_model():
    # kinds that do not fit the shape (EXP_HALF observes every component: nz must equal nx)
    Q, R, beta = np.eye(5), np.eye(3), np.ones(3)
    d = NV.ModelDesc(5, 3, NV.PF_TRANS_LINEAR, NV.PF_OBS_EXP_HALF, NV.dptr(np.eye(5).ravel()), 25,
                     NV.dptr(beta), 3, NV.dptr(Q), NV.dptr(R))
    opts = NV.Opts(100, 1, 0, 0.5, 0, 0, 1, 0, 0, 0)
    h_ = C.c_void_p()
    st = NV.load().pf_create(C.byref(d), C.byref(opts), C.byref(h_))
    assert st == NV.PF_E_UNSUPPORTED and not h_.value
    with pytest.raises(NotImplementedError):
        NV.check(st)


def test_runtime_shape_registry():
    """Shapes outside the compiled list run on the runtime-shape kernels (pf_dyn.h)."""
    lib = NV.load()
    L96, LIN = NV.PF_TRANS_L96, NV.PF_TRANS_LINEAR
    # the builder's second L96 golden case (nx = 12) and the simulator's default nx = 1000
    for nx, nz in ((12, 3), (1000, 250), (40, 10)):
        assert lib.pf_model_supported(nx, nz, L96, NV.PF_OBS_LINEAR)
    assert lib.pf_model_compiled(40, 10, L96, NV.PF_OBS_LINEAR)
    assert not lib.pf_model_compiled(12, 3, L96, NV.PF_OBS_LINEAR)
    # the 9-D bearings-only SIR (SPF example 2)
    assert lib.pf_model_supported(9, 2, LIN, NV.PF_OBS_BEARINGS)
    assert not lib.pf_model_supported(9, 3, LIN, NV.PF_OBS_BEARINGS)
    assert not lib.pf_model_supported(2, 2, LIN, NV.PF_OBS_BEARINGS)
    assert lib.pf_model_supported(8, 25, LIN, NV.PF_OBS_ACOUSTIC)
    assert not lib.pf_model_supported(6, 25, LIN, NV.PF_OBS_ACOUSTIC)
    assert lib.pf_model_supported(5, 5, LIN, NV.PF_OBS_SV_EXACT)
    assert not lib.pf_model_supported(5, 4, LIN, NV.PF_OBS_EXP_HALF)
    assert M.supported(M.LinearTransition(np.eye(9)), M.BearingsObservation(9))
    assert not M.compiled(M.LinearTransition(np.eye(9)), M.BearingsObservation(9))
    assert M.kernel_path_code("runtime") == NV.PF_PATH_RUNTIME
    with pytest.raises(ValueError):
        M.kernel_path_code("jit")
    st, _ = _create(M.SVTransition(0.95), M.SVLogSqObservation(1.0), [[0.04]], [[1.0]], kernel_path=5)
    assert st == NV.PF_E_ARG


def test_bearings_observation_matches_notebook_formula():
    h = M.BearingsObservation(9)
    s = np.array([40.0, 40.0, 40.0, 8.0, 0.0, -3.0, 0.0, 0.0, 0.0])
    r = np.sqrt(s[0] ** 2 + s[1] ** 2)
    np.testing.assert_array_equal(h(s), [np.arctan2(s[0], s[1]), np.arctan2(s[2], r)])


def test_status_exception_mapping():
    with pytest.raises(AssertionError, match="Filter not initialized."):
        NV.check(NV.PF_E_NOT_INITIALIZED)
    with pytest.raises(np.linalg.LinAlgError):
        NV.check(NV.PF_E_NOT_PD)
    with pytest.raises(NV.PFError):
        NV.check(NV.PF_E_HIP)
    NV.check(NV.PF_OK)


def test_describe_validates_shapes():
    with pytest.raises(ValueError):
        M.describe(M.SVTransition(0.95), M.SVLogSqObservation(1.0), np.eye(2), np.eye(1))
    with pytest.raises(ValueError):
        M.describe(M.SVTransition(0.95), M.SVLogSqObservation(1.0), np.eye(1), np.eye(2))


def test_ledh_model_registry_and_validation():
    lib = NV.load()
    assert lib.pf_ledh_model_supported(40, 10, NV.PF_TRANS_L96, NV.PF_OBS_LINEAR)
    assert lib.pf_ledh_model_supported(1, 1, NV.PF_TRANS_LINEAR, NV.PF_OBS_EXP_HALF)
    assert lib.pf_ledh_model_supported(4, 9, NV.PF_TRANS_LINEAR, NV.PF_OBS_ACOUSTIC)
    assert not lib.pf_ledh_model_supported(7, 3, NV.PF_TRANS_L96, NV.PF_OBS_ACOUSTIC)
    d, keep = M.describe(M.SVTransition(0.9), M.LinearObservation([[1.0]]), np.eye(1) * 0.04, np.eye(1) * 0.1)
    h_ = C.c_void_p()
    opts = NV.LedhOpts(0, 8, 0.5, 1, 0, 0)
    assert lib.pf_ledh_create(C.byref(d), C.byref(opts), C.byref(h_)) == NV.PF_E_ARG and not h_.value
    d2, keep2 = M.describe(M.LinearTransition(np.eye(5)), M.LinearObservation(np.ones((1, 5))), np.eye(5), np.eye(1))
    opts = NV.LedhOpts(10, 8, 0.5, 1, 0, 0)
    assert lib.pf_ledh_create(C.byref(d2), C.byref(opts), C.byref(h_)) == NV.PF_E_UNSUPPORTED


def test_checkpoint_api_validates_arguments_without_a_device():
    lib = NV.load()
    st = NV.RngState()
    assert lib.pf_get_rng_state(None, C.byref(st)) == NV.PF_E_ARG
    assert lib.pf_set_rng_state(None, C.byref(st)) == NV.PF_E_ARG
    assert lib.pf_checkpoint_bytes(None) == -1
    buf = C.create_string_buffer(256)
    assert lib.pf_checkpoint(None, C.cast(buf, C.c_void_p), 256) == NV.PF_E_ARG
    assert lib.pf_restore(None, C.cast(buf, C.c_void_p), 256) == NV.PF_E_ARG
