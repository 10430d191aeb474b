"""ctypes binding of ``libpf_hip.so`` (the C ABI declared in ``include/pf_engine.h``,
``include/pf_ledh.h``, ``include/pf_edh.h``, ``include/pf_diag.h`` and ``include/pf_shard.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C
particle_filters_amd/csrc``).  There is no fallback: if the library is missing
or cannot be loaded, importing the engine raises.
"""

from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PF_LIB", os.path.join(_HERE, "libpf_hip.so"))

PF_OK = 0
PF_E_NOT_INITIALIZED = 1
PF_E_ARG = 2
PF_E_NOT_PD = 3
PF_E_HIP = 4
PF_E_UNSUPPORTED = 5
PF_E_NAN = 6
PF_E_RETRY = 7

PF_TRANS_LINEAR = 0
PF_TRANS_L96 = 1
PF_OBS_LINEAR = 0
PF_OBS_EXP_HALF = 1
PF_OBS_ACOUSTIC = 2
PF_OBS_SV_EXACT = 3
PF_OBS_BEARINGS = 4
PF_PATH_AUTO = 0
PF_PATH_RUNTIME = 1
PF_RESAMPLE_SYSTEMATIC = 0
PF_RESAMPLE_MULTINOMIAL = 1
PF_PRECISION_FP32 = 0
PF_PRECISION_FP64 = 1
PF_NOISE_NONE = 0
PF_NOISE_HOST = 1
PF_NOISE_DEVICE = 2
PF_LEDH_FLOW_AUTO = 0
PF_LEDH_FLOW_PER_PARTICLE = 1
PF_EDH_RK4 = 0
PF_EDH_EULER = 1

_dp = C.POINTER(C.c_double)
_vp = C.c_void_p


class ModelDesc(C.Structure):
    _fields_ = [("nx", C.c_int32), ("nz", C.c_int32), ("trans_kind", C.c_int32), ("obs_kind", C.c_int32),
                ("trans_params", _dp), ("n_trans_params", C.c_int64),
                ("obs_params", _dp), ("n_obs_params", C.c_int64),
                ("Q", _dp), ("R", _dp)]


class Opts(C.Structure):
    _fields_ = [("n_particles", C.c_int64), ("n_replicates", C.c_int32), ("resample_method", C.c_int32),
                ("resample_thresh", C.c_double), ("regularize", C.c_int32), ("precision", C.c_int32),
                ("seed", C.c_uint64), ("device", C.c_int32), ("replicate_base", C.c_int32),
                ("kernel_path", C.c_int32)]


class LedhOpts(C.Structure):
    _fields_ = [("n_particles", C.c_int64), ("n_lambda", C.c_int32), ("resample_ess_ratio", C.c_double),
                ("seed", C.c_uint64), ("device", C.c_int32), ("flow_mode", C.c_int32)]


class EdhOpts(C.Structure):
    _fields_ = [("n_particles", C.c_int64), ("n_lambda", C.c_int32), ("resample_ess_ratio", C.c_double),
                ("seed", C.c_uint64), ("device", C.c_int32), ("integrator", C.c_int32)]


class Diagnostics(C.Structure):
    _fields_ = [("ess", C.c_double), ("entropy", C.c_double), ("entropy_raw", C.c_double), ("gini", C.c_double),
                ("max_weight", C.c_double), ("posterior_spread", C.c_double), ("n_unique", C.c_int64)]


class ShardStats(C.Structure):
    _fields_ = [("lse", C.c_double), ("neff", C.c_double), ("U", C.c_double)]


class LedhInfo(C.Structure):
    _fields_ = [("ess", C.c_double), ("resample", C.c_int32), ("_pad", C.c_int32)]


class RngState(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("epoch", C.c_uint32), ("ep_res", C.c_uint32), ("replicate_base", C.c_int32),
                ("pending", C.c_int32)]


class UpdateInfo(C.Structure):
    _fields_ = [("neff", C.c_double), ("log_norm", C.c_double), ("resample", C.c_int32), ("_pad", C.c_int32)]


# name -> (restype, argtypes); every symbol declared in include/pf_engine.h
SIGNATURES = {
    "pf_last_error": (C.c_char_p, []),
    "pf_version": (C.c_char_p, []),
    "pf_device_count": (C.c_int32, []),
    "pf_model_supported": (C.c_int32, [C.c_int32] * 4),
    "pf_model_compiled": (C.c_int32, [C.c_int32] * 4),
    "pf_kernel_path": (C.c_int32, [_vp]),
    "pf_last_step_streamed": (C.c_int32, [_vp]),
    "pf_create": (C.c_int32, [C.POINTER(ModelDesc), C.POINTER(Opts), C.POINTER(_vp)]),
    "pf_destroy": (None, [_vp]),
    "pf_initialize": (C.c_int32, [_vp, _dp, _dp, _dp]),
    "pf_predict": (C.c_int32, [_vp, _dp, _dp]),
    "pf_update": (C.c_int32, [_vp, _dp, C.POINTER(UpdateInfo), _dp, _dp]),
    "pf_resample": (C.c_int32, [_vp, _dp, _dp, _dp, _dp]),
    "pf_resample_state": (C.c_int32, [_vp, _dp, _dp]),
    "pf_run": (C.c_int32, [_vp, _dp, _dp, C.c_int64, C.c_int32, _dp, _dp, _dp, C.POINTER(C.c_uint8), _dp]),
    "pf_run_device": (C.c_int32, [_vp, _vp, _vp, C.c_int64, C.c_int32, _vp, _vp, _vp, _vp, _vp]),
    "pf_get_particles": (C.c_int32, [_vp, _dp]),
    "pf_get_weights": (C.c_int32, [_vp, _dp, _dp]),
    "pf_set_state": (C.c_int32, [_vp, _dp, _dp]),
    "pf_weights_uniform": (C.c_int32, [_vp]),
    "pf_moments": (C.c_int32, [_vp, _dp, _dp]),
    "pf_get_rng_state": (C.c_int32, [_vp, C.POINTER(RngState)]),
    "pf_set_rng_state": (C.c_int32, [_vp, C.POINTER(RngState)]),
    "pf_checkpoint_bytes": (C.c_int64, [_vp]),
    "pf_checkpoint": (C.c_int32, [_vp, _vp, C.c_int64]),
    "pf_restore": (C.c_int32, [_vp, _vp, C.c_int64]),
    "pf_resample_indices": (C.c_int32, [C.c_int32, C.c_int32, _dp, C.c_int64, C.c_double, _dp,
                                        C.POINTER(C.c_int64)]),
    "pf_stream": (_vp, [_vp]),
    "pf_synchronize": (C.c_int32, [_vp]),
    "pf_profile_steps": (C.c_int32, [_vp, _vp, C.c_int64, C.POINTER(C.c_float)]),
    "pf_geometry": (C.c_int32, [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "pf_last_run_resident": (C.c_int32, [_vp]),
    "pf_last_run_persistent": (C.c_int32, [_vp]),
    "pf_test_lds_poison": (C.c_int32, [_vp]),
    "pf_test_lds_probe_blocks": (C.c_int32, []),
    "pf_test_lds_poison_count": (C.c_int64, []),
    "pf_test_lds_probe": (C.c_int32, [_vp, C.POINTER(C.c_int32)]),
    "pf_set_timing": (C.c_int32, [_vp, C.c_int32]),
    "pf_last_run_ms": (C.c_int32, [_vp, C.POINTER(C.c_float)]),
    "pf_set_trace": (C.c_int32, [_vp, C.c_int64]),
    "pf_get_trace": (C.c_int32, [_vp, C.c_int64, C.c_int32, _vp, _vp, _vp]),
    # include/pf_ledh.h
    "pf_ledh_create": (C.c_int32, [C.POINTER(ModelDesc), C.POINTER(LedhOpts), C.POINTER(_vp)]),
    "pf_ledh_destroy": (None, [_vp]),
    "pf_ledh_model_supported": (C.c_int32, [C.c_int32] * 4),
    "pf_ledh_init": (C.c_int32, [_vp, _dp, _dp, _dp, _dp, _dp]),
    "pf_ledh_step": (C.c_int32, [_vp, _dp, _dp, _dp, C.c_int32, _dp, C.POINTER(LedhInfo), _dp]),
    "pf_ledh_finish": (C.c_int32, [_vp, _dp, _dp, _dp]),
    "pf_ledh_get_particles": (C.c_int32, [_vp, _dp]),
    "pf_ledh_get_weights": (C.c_int32, [_vp, _dp]),
    "pf_ledh_set_state": (C.c_int32, [_vp, _dp, _dp]),
    "pf_ledh_run": (C.c_int32, [_vp, _dp, _dp, _dp, C.c_int64, C.c_int32, _dp, _dp, _dp, C.POINTER(C.c_uint8)]),
    "pf_ledh_ekf_sequence": (C.c_int32, [_vp, _dp, _dp, _dp, _dp, _dp, C.c_int64, _dp, _dp, _dp]),
    "pf_ledh_run_ekf": (C.c_int32, [_vp, _dp, _dp, _dp, _dp, _dp, _dp, C.c_int64, C.c_int32, _dp, _dp, _dp,
                                    C.POINTER(C.c_uint8), _dp, _dp]),
    "pf_ledh_set_run_replay": (C.c_int32, [_vp, _dp, _dp, C.c_int64]),
    "pf_ledh_stream": (_vp, [_vp]),
    "pf_ledh_synchronize": (C.c_int32, [_vp]),
    "pf_ledh_shared_path": (C.c_int32, [_vp]),
    # include/pf_edh.h
    "pf_edh_create": (C.c_int32, [C.POINTER(ModelDesc), C.POINTER(EdhOpts), C.POINTER(_vp)]),
    "pf_edh_step": (C.c_int32, [_vp, _dp, _dp, _dp, _dp, C.c_int32, _dp, C.POINTER(LedhInfo), _dp]),
    "pf_edh_run": (C.c_int32, [_vp, _dp, _dp, _dp, _dp, C.c_int64, C.c_int32, _dp, _dp, _dp, C.POINTER(C.c_uint8)]),
    "pf_edh_is_edh": (C.c_int32, [_vp]),
    # include/pf_diag.h
    "pf_diagnostics_host": (C.c_int32, [C.c_int32, _dp, _dp, C.c_int64, C.c_int32, C.c_double, _dp,
                                        C.POINTER(Diagnostics)]),
    "pf_state_diagnostics": (C.c_int32, [_vp, C.c_double, C.POINTER(Diagnostics)]),
    "pf_ledh_diagnostics": (C.c_int32, [_vp, C.c_double, C.POINTER(Diagnostics)]),
    # include/pf_shard.h
    "pf_shard_configure": (C.c_int32, [_vp, C.c_int64, C.c_int32]),
    "pf_shard_update": (C.c_int32, [_vp, _dp, C.c_double, C.POINTER(ShardStats), _dp, _dp]),
    "pf_shard_offspring": (C.c_int32, [_vp, C.c_double, C.c_double, C.c_double, C.c_int64, C.c_int64, _vp]),
    "pf_shard_adopt": (C.c_int32, [_vp, _vp, _dp, _dp, _dp]),
}

_lib = None
_lock = threading.Lock()


def load() -> C.CDLL:
    """Load libpf_hip.so (raises ImportError if it was not built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: build the HIP engine first "
                "(python -c 'import __graft_entry__ as g; g.build()' or make -C particle_filters_amd/csrc)")
        lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            if "PF_LIB" in os.environ and not hasattr(lib, name):
                continue  # an experiment variant built from an older tree (tools/gpu_ab.sh)
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


class PFError(RuntimeError):
    pass


class PFRetry(PFError):
    """PF_E_RETRY: a resident launch found its grid not co-resident and computed nothing; the
    state is unchanged and the next run launches cooperatively."""


def check(status: int, what: str = "") -> None:
    """Map a pf_status to the reference's exception types (particle_filter.py)."""
    if status == PF_OK:
        return
    msg = load().pf_last_error().decode(errors="replace")
    if what:
        msg = f"{what}: {msg}"
    if status == PF_E_NOT_INITIALIZED:
        raise AssertionError("Filter not initialized.")
    if status == PF_E_NOT_PD:
        raise np.linalg.LinAlgError(msg)
    if status == PF_E_ARG:
        raise ValueError(msg)
    if status == PF_E_UNSUPPORTED:
        raise NotImplementedError(msg)
    if status == PF_E_NAN:
        raise FloatingPointError(msg)
    if status == PF_E_RETRY:
        raise PFRetry(msg)
    raise PFError(msg)


def dptr(a):
    """double* of a C-contiguous float64 array (or NULL for None)."""
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def device_count() -> int:
    return int(load().pf_device_count())


# ---------------------------------------------------------------- Philox position / checkpoints
def get_rng_state(handle) -> dict:
    """The handle's Philox position (pf_get_rng_state): seed, epoch, ep_res, replicate_base,
    pending."""
    st = RngState()
    check(load().pf_get_rng_state(handle, C.byref(st)), "pf_get_rng_state")
    return dict(seed=int(st.seed), epoch=int(st.epoch), ep_res=int(st.ep_res),
                replicate_base=int(st.replicate_base), pending=bool(st.pending))


def set_rng_state(handle, state: dict) -> None:
    st = RngState(int(state["seed"]), int(state["epoch"]), int(state["ep_res"]), int(state["replicate_base"]), 0)
    check(load().pf_set_rng_state(handle, C.byref(st)), "pf_set_rng_state")


def checkpoint(handle) -> bytes:
    """Bit-exact snapshot of the filter state (pf_checkpoint): opaque bytes."""
    lib = load()
    n = int(lib.pf_checkpoint_bytes(handle))
    if n <= 0:
        raise PFError("pf_checkpoint_bytes failed")
    buf = C.create_string_buffer(n)
    check(lib.pf_checkpoint(handle, C.cast(buf, C.c_void_p), n), "pf_checkpoint")
    return buf.raw


def restore(handle, blob: bytes) -> None:
    b = bytes(blob)
    buf = C.create_string_buffer(b, len(b))
    check(load().pf_restore(handle, C.cast(buf, C.c_void_p), len(b)), "pf_restore")
