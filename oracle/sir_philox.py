"""The SIR oracle on the engine's Philox draw stream — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` /
``rmse_vs_ref`` legs may use this module, as the checker.

The reference (``/root/reference/models/particle_filter.py``) draws from NumPy's
PCG64 generator; the HIP engine's device RNG is counter-based Philox4x32-10
(``particle_filters_amd/csrc/philox.h``).  To compare the engine's *device-RNG*
runs (the benchmarked register-resident kernel has no host replay mode) with the
reference algorithm on identical noise, the oracle is driven by the engine's
draws instead of PCG64:

* :class:`PhiloxRNG` — a duck-typed ``numpy.random.Generator`` (the SIR path uses
  only ``standard_normal(shape)``, ``random()`` and ``choice(n, n, p)``,
  pf.py:128,160,186,217,236) serving the draws of one (epoch, stream);
* :class:`PhiloxSIROracle` — :class:`oracle.pf_oracle.SIROracle` (bit-identical to
  the reference on its own draws) with the engine's epoch bookkeeping: initialize
  at epoch e, step t predicts at e + 1 + 2t and resamples at e + 2 + 2t;
* :func:`run_scalar` — the same filter for scalar-state models in C
  (``oracle/sir_philox.c``, OpenMP, fp64), fast enough for the BASELINE config-2
  size (N = 1e6, T = 999); pinned to :class:`PhiloxSIROracle` by
  ``tests/test_sir_philox.py``.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional

import numpy as np

from . import philox
from .pf_oracle import SIROracle, multinomial_indices

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsir_oracle.so")

OBS_LINEAR, OBS_EXP_HALF, OBS_SV_EXACT = 0, 1, 3


class PhiloxRNG:
    """Serves the engine's device draws for the (epoch, stream) set by the caller."""

    def __init__(self, seed: int, rep: int = 0, bm24: bool = True, c_normals: bool = False):
        self.seed = int(seed)
        self.rep = int(rep)
        self.bm24 = bool(bm24)
        # c_normals: the same draws from the C restatement (pfo_normals, ~20x faster; its libm
        # sin / cos differ from NumPy's in the last ulp on ~0.2 % of the values) - used by the
        # statistical free-run pairs (oracle/free_run.py), where one ulp is immaterial
        self.c_normals = bool(c_normals)
        self.epoch: Optional[int] = None
        self.stream: Optional[int] = None

    def at(self, epoch: int, stream: int) -> "PhiloxRNG":
        self.epoch, self.stream = int(epoch), int(stream)
        return self

    def standard_normal(self, size=None):
        shape = () if size is None else tuple(np.atleast_1d(size))
        n = int(np.prod(shape)) if shape else 1
        if self.c_normals:
            v = normals(self.seed, n, self.rep, self.epoch, self.stream, bm24=self.bm24)
        else:
            v = philox.normals(self.seed, n, self.rep, self.epoch, self.stream,
                               dtype=np.float32 if self.bm24 else np.float64)
        return v.reshape(shape) if shape else float(v[0])

    def random(self, size=None):
        if size is None:
            return float(philox.uniform53(self.seed, 0, self.rep, self.epoch))
        return philox.uniform53(self.seed, np.arange(int(size), dtype=np.uint64), self.rep, self.epoch)

    def choice(self, a, size=None, replace=True, p=None):
        return multinomial_indices(p, self.random(size))


class PhiloxSIROracle(SIROracle):
    """``SIROracle`` on the engine's Philox draws (epochs of pf_engine.hip: one per
    initialize / predict / update)."""

    def __init__(self, g, h, Q, R, *, seed: int, rep: int = 0, bm24: bool = True, epoch: int = 1,
                 c_normals: bool = False, **kw):
        self.prng = PhiloxRNG(seed, rep, bm24, c_normals)
        super().__init__(g, h, Q, R, rng=self.prng, **kw)
        self.epoch = int(epoch)
        self.forced = None  # optional per-step decisions (teacher forcing), consumed in order
        self.own_decision = False

    def initialize(self, mean, cov):
        self.prng.at(self.epoch, philox.STREAM_INIT)
        self.epoch += 1
        return super().initialize(mean, cov)

    def predict(self, u=None):
        self.prng.at(self.epoch, philox.STREAM_PROCESS)
        self.epoch += 1
        return super().predict(u)

    def update(self, z):
        # the resample's uniforms (STREAM_RESAMPLE, via random()) and jitter normals share the epoch
        self.prng.at(self.epoch, philox.STREAM_JITTER)
        self.epoch += 1
        return super().update(z)

    def _resample(self, particles, weights):
        if self.forced is None:
            return super()._resample(particles, weights)
        want = bool(self.forced.pop(0))
        neff = 1.0 / np.sum(weights ** 2)
        self.own_decision = bool(neff < self.resample_thresh * self.Np)
        thresh = self.resample_thresh
        # force the decision by moving the threshold past Neff (the rest of _resample unchanged)
        self.resample_thresh = (2.0 * neff / self.Np + 1.0) if want else 0.0
        try:
            return super()._resample(particles, weights)
        finally:
            self.resample_thresh = thresh


# ---------------------------------------------------------------------------
# C restatement (scalar state)
# ---------------------------------------------------------------------------
class _Model(C.Structure):
    _fields_ = [("a", C.c_double), ("lq", C.c_double), ("lj", C.c_double), ("obs", C.c_int32),
                ("_pad", C.c_int32), ("hH", C.c_double), ("hc", C.c_double), ("lr", C.c_double)]


class _Opts(C.Structure):
    _fields_ = [("N", C.c_int64), ("T", C.c_int64), ("seed", C.c_uint64), ("rep", C.c_uint32),
                ("ep0", C.c_uint32), ("thresh", C.c_double), ("method", C.c_int32), ("regularize", C.c_int32),
                ("bm24", C.c_int32), ("first_update_only", C.c_int32), ("init", C.c_int32), ("_pad", C.c_int32),
                ("mean0", C.c_double), ("var0", C.c_double)]


class _StepCheck(C.Structure):
    _fields_ = [("N", C.c_int64), ("seed", C.c_uint64), ("rep", C.c_uint32), ("epoch", C.c_uint32),
                ("thresh", C.c_double), ("bm24", C.c_int32), ("regularize", C.c_int32), ("u", C.c_double),
                ("z", C.c_double), ("neff_e", C.c_double), ("mean_e", C.c_double), ("var_e", C.c_double),
                ("flag_e", C.c_int32), ("_pad0", C.c_int32),
                ("dx_pre", C.c_double), ("mean_abs_x", C.c_double), ("tv_w", C.c_double), ("dcdf", C.c_double),
                ("lmag", C.c_double), ("eps_w", C.c_double), ("neff_o", C.c_double), ("neff_rel", C.c_double),
                ("flag_o", C.c_int32), ("near_threshold", C.c_int32), ("U", C.c_double),
                ("n_anc_bad", C.c_int64), ("n_anc_self_diff", C.c_int64), ("n_anc_oracle_diff", C.c_int64),
                ("max_margin_self", C.c_double), ("max_margin_oracle", C.c_double),
                ("dmean", C.c_double), ("dvar", C.c_double), ("dmean_oracle", C.c_double),
                ("mean_o", C.c_double), ("var_o", C.c_double)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
                os.path.join(HERE, "sir_philox.c")):
            build()
        lib = C.CDLL(LIB_PATH)
        d = C.POINTER(C.c_double)
        lib.pfo_sir_scalar_run.restype = C.c_int64
        lib.pfo_sir_scalar_run.argtypes = [C.POINTER(_Model), C.POINTER(_Opts), d, d, C.POINTER(C.c_int32), d, d, d,
                                           d, d, C.POINTER(C.c_int32), d]
        lib.pfo_normals.restype = None
        lib.pfo_normals.argtypes = [C.c_uint64, C.c_int64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, d]
        lib.pfo_uniform53.restype = C.c_double
        lib.pfo_uniform53.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        lib.pfo_sir_scalar_check_step.restype = C.c_int
        lib.pfo_sir_scalar_check_step.argtypes = [C.POINTER(_Model), C.POINTER(_StepCheck), d, d,
                                                  C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_int32)]
        lib.pfo_philox4x32_10.restype = None
        lib.pfo_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        _lib = lib
    return _lib


def _p(a, t=C.c_double):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


def philox4x32_10(ctr, key):
    lib = load()
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, np.uint32)
    lib.pfo_philox4x32_10(_p(c, C.c_uint32), _p(k, C.c_uint32), _p(out, C.c_uint32))
    return out


def normals(seed, n, rep, epoch, stream, bm24=True):
    out = np.empty(int(n))
    load().pfo_normals(int(seed), int(n), int(rep), int(epoch), int(stream), int(bool(bm24)), _p(out))
    return out


def scalar_model(alpha, q_var, obs, *, hH=1.0, hc=0.0, r_var=1.0):
    """Scalar SSM: g = alpha x, Q = q_var; obs LINEAR (h = hH x + hc), EXP_HALF (h = hc e^{x/2})
    or SV_EXACT (beta = hc).  chol factors as the engine / reference take them."""
    lq = np.sqrt(q_var) if q_var > 0 else np.sqrt(q_var + 1e-10)
    lj = 0.001 * (np.sqrt(q_var) if q_var > 0 else np.sqrt(q_var + 1e-12))
    return _Model(a=float(alpha), lq=float(lq), lj=float(lj), obs=int(obs), _pad=0, hH=float(hH), hc=float(hc),
                  lr=float(np.sqrt(r_var + 1e-12)))


def sv_logsq_model(alpha, sigma, beta):
    from .ssm_oracle import LOGCHI2_MEAN, LOGCHI2_VAR
    return scalar_model(alpha, sigma ** 2, OBS_LINEAR, hH=1.0, hc=float(np.log(beta ** 2)) + LOGCHI2_MEAN,
                        r_var=LOGCHI2_VAR)


def run_scalar(model: _Model, Z, *, N, seed, rep=0, ep0=2, thresh=0.5, method="systematic", regularize=False,
               bm24=True, first_update_only=False, mean0=None, var0=None, x0=None, w0=None, U=None, forced=None):
    """Run the C oracle; returns dict(means, vars, neff, flags, lse, x, w).

    ``ep0`` is the engine handle's epoch at the first step (a fresh handle initialises
    at epoch 1, so its first run starts at 2).  Give ``mean0``/``var0`` to initialise at
    ``ep0 - 1``, or ``x0``/``w0`` to start from a given state."""
    lib = load()
    Z = np.ascontiguousarray(np.asarray(Z, float).reshape(-1))
    T = Z.size
    init = mean0 is not None
    x = np.zeros(N) if x0 is None else np.array(x0, dtype=float).reshape(-1)
    w = np.full(N, 1.0 / N) if w0 is None else np.array(w0, dtype=float).reshape(-1)
    o = _Opts(N=int(N), T=T, seed=int(seed), rep=int(rep), ep0=int(ep0), thresh=float(thresh),
              method=0 if method == "systematic" else 1, regularize=int(bool(regularize)), bm24=int(bool(bm24)),
              first_update_only=int(bool(first_update_only)), init=int(init), _pad=0,
              mean0=float(np.asarray(mean0).reshape(-1)[0]) if init else 0.0,
              var0=float(np.asarray(var0).reshape(-1)[0]) if init else 0.0)
    out = dict(means=np.zeros(T), vars=np.zeros(T), neff=np.zeros(T), flags=np.zeros(T, np.int32), lse=np.zeros(T))
    Uc = None if U is None else np.ascontiguousarray(np.asarray(U, float).reshape(-1))
    Fc = None if forced is None else np.ascontiguousarray(np.asarray(forced).reshape(-1).astype(np.int32))
    st = lib.pfo_sir_scalar_run(C.byref(model), C.byref(o), _p(Z), _p(Uc), _p(Fc, C.c_int32), _p(x), _p(w),
                                _p(out["means"]), _p(out["vars"]), _p(out["neff"]), _p(out["flags"], C.c_int32),
                                _p(out["lse"]))
    if st < 0:
        raise MemoryError("sir_philox: allocation failed")
    out["dead_step"] = int(st) - 1 if st > 0 else -1
    out["flags"] = out["flags"].astype(bool)
    out["x"], out["w"] = x, w
    return out


def check_step(model: _Model, *, seed, rep, epoch, thresh, x0, w0, z, xe, le, anc, neff_e, flag_e, mean_e, var_e,
               bm24=True, regularize=False, u=0.0) -> dict:
    """One oracle step from the state (x0, w0) against an engine's record of the same step
    (``pfo_sir_scalar_check_step`` in sir_philox.c): returns the measured quantities as a dict.
    ``anc`` is the engine's ancestor of every slot (int32) when it resampled, else None."""
    N = int(np.asarray(xe).size)
    c = _StepCheck(N=N, seed=int(seed), rep=int(rep), epoch=int(epoch), thresh=float(thresh), bm24=int(bool(bm24)),
                   regularize=int(bool(regularize)), u=float(u), z=float(np.asarray(z).reshape(-1)[0]),
                   neff_e=float(neff_e), mean_e=float(mean_e), var_e=float(var_e), flag_e=int(bool(flag_e)))
    x0 = np.ascontiguousarray(np.asarray(x0, float).reshape(-1))
    w0 = np.ascontiguousarray(np.asarray(w0, float).reshape(-1))
    xe = np.ascontiguousarray(np.asarray(xe, np.float32).reshape(-1))
    le = np.ascontiguousarray(np.asarray(le, np.float32).reshape(-1))
    a = None if anc is None else np.ascontiguousarray(np.asarray(anc, np.int32).reshape(-1))
    if x0.size != N or w0.size != N or le.size != N or (a is not None and a.size != N):
        raise ValueError("check_step: arrays of different lengths")
    if load().pfo_sir_scalar_check_step(C.byref(model), C.byref(c), _p(x0), _p(w0), _p(xe, C.c_float),
                                        _p(le, C.c_float), _p(a, C.c_int32)) != 0:
        raise MemoryError("check_step: allocation failed")
    out = {k: getattr(c, k) for k, _ in _StepCheck._fields_ if not k.startswith("_")}
    for k in ("flag_e", "flag_o", "near_threshold"):
        out[k] = bool(out[k])
    return out
