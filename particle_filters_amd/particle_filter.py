"""Drop-in ``ParticleFilter`` / ``PFState`` backed by the MI355X HIP engine.

Mirrors ``/root/reference/models/particle_filter.py`` (cited ``pf.py:LINE``):
same constructor keywords and defaults (``:79-107``), same methods
(``initialize`` ``:110``, ``predict`` ``:223``, ``update`` ``:239``, ``step``
``:271``, ``effective_sample_size`` ``:134``, and the private
``_systematic_resample`` / ``_multinomial_resample`` / ``_resample`` that the
reference's tests call), same public attributes (``Np, nx, nz, Q, R, LR,
resample_thresh, resample_method, regularize_after_resample, rng, state``) and
the same errors (``AssertionError("Filter not initialized.")``,
``numpy.linalg.LinAlgError`` for non-PD covariances).

Differences a user sees:

* ``g`` / ``h`` must be device models from :mod:`particle_filters_amd.models`
  (which are themselves per-particle callables, so the same objects work with
  the reference).  Arbitrary Python callables raise ``NotImplementedError`` —
  there is no CPU fallback.
* Randomness: ``rng_mode="device"`` (default) draws every normal/uniform on the
  GPU with counter-based Philox4x32-10 seeded from ``rng`` (the seed is one
  ``rng.integers`` draw at construction).  ``rng_mode="host"`` draws exactly the
  reference's stream from ``rng`` (``pf.py:128,160,186,217,236``) and ships it
  to the GPU — the replay mode used to prove parity with the reference.
* ``precision="fp32"`` (default, particle storage and per-particle arithmetic) or
  ``"fp64"``.  The resampling CDF and the tile masses that place it are fp64 on every
  path; the launch-per-step kernels combine tiles in fp64, while the whole-run fp32
  kernel (``k_resident``, scalar state) sums within a 512-particle wave in fp32 and
  carries the per-tile W2 / moment sums as fp32 (the tile mass S0 as fp64), so its
  Neff decision and moments are fp32-reduced per tile.
* ``state`` arrays live on the GPU and are fetched lazily on attribute access.
* Any (nx, nz): shapes in the compiled list keep the particle in registers; any other shape
  (or ``kernel_path="runtime"``) runs the runtime-shape kernels (``csrc/pf_dyn.h``);
  ``kernel_path_used`` says which.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from . import _native as N
from . import models as M

Array = np.ndarray


@dataclass
class PFState:
    """Posterior container (pf.py:27-49)."""

    particles: Array
    weights: Array
    mean: Array
    cov: Array
    t: int


class _DeviceState(PFState):
    """PFState whose particles / weights stay on the GPU until read."""

    def __init__(self, pf: "ParticleFilter", mean: Array, cov: Array, t: int):  # noqa: D401
        object.__setattr__(self, "_pf", pf)
        object.__setattr__(self, "_version", pf._version)
        object.__setattr__(self, "_particles", None)
        object.__setattr__(self, "_weights", None)
        object.__setattr__(self, "mean", mean)
        object.__setattr__(self, "cov", cov)
        object.__setattr__(self, "t", t)

    def _fresh(self) -> bool:
        return self._pf._version == self._version

    @property
    def particles(self) -> Array:  # type: ignore[override]
        if self._particles is None:
            if not self._fresh():
                raise RuntimeError("stale PFState: the filter has advanced since this state was returned")
            object.__setattr__(self, "_particles", self._pf._download_particles())
        return self._particles

    @particles.setter
    def particles(self, value) -> None:
        value = np.asarray(value, float)
        if self._fresh():
            # the weights stay what they are (pf.py keeps state.weights when particles are
            # assigned): fetch them first unless the device says they are uniform
            w = self._weights
            if w is None and not N.load().pf_weights_uniform(self._pf._handle):
                w = self.weights
            object.__setattr__(self, "_particles", value)
            self._pf._upload_state(value, w)
            object.__setattr__(self, "_version", self._pf._version)
        else:
            object.__setattr__(self, "_particles", value)

    @property
    def weights(self) -> Array:  # type: ignore[override]
        if self._weights is None:
            if not self._fresh():
                raise RuntimeError("stale PFState: the filter has advanced since this state was returned")
            object.__setattr__(self, "_weights", self._pf._download_weights())
        return self._weights

    @weights.setter
    def weights(self, value) -> None:
        value = np.asarray(value, float)
        object.__setattr__(self, "_weights", value)
        if self._fresh():
            self._pf._upload_state(self.particles, value)
            object.__setattr__(self, "_version", self._pf._version)

    def __repr__(self) -> str:
        return f"PFState(mean={self.mean!r}, cov={self.cov!r}, t={self.t}, particles=<device>, weights=<device>)"


_UNIFORM_ESS_CACHE = {}


def _uniform_ess(n: int) -> float:
    """1/sum((1/n)^2) evaluated like the reference (pf.py:144 after pf.py:210)."""
    v = _UNIFORM_ESS_CACHE.get(n)
    if v is None:
        w = np.ones(n) / n
        v = 1.0 / np.sum(w ** 2)
        _UNIFORM_ESS_CACHE[n] = v
    return v


class ParticleFilter:
    """SIR particle filter on an MI355X (drop-in for pf.py:53-287)."""

    def __init__(
        self,
        g,
        h,
        Q: Array,
        R: Array,
        *,
        Np: int = 1000,
        resample_thresh: float = 0.5,
        resample_method: str = "systematic",
        regularize_after_resample: bool = False,
        rng: Optional[np.random.Generator] = None,
        precision: str = "fp32",
        rng_mode: str = "device",
        device: int = 0,
        kernel_path: str = "auto",
    ) -> None:
        self.g = g
        self.h = h
        self.Q = np.asarray(Q, float)
        self.R = M.observation_noise(h, R)
        self.Np = int(Np)
        self.resample_thresh = float(resample_thresh)
        self.resample_method = resample_method
        self.regularize_after_resample = regularize_after_resample
        self.rng = np.random.default_rng() if rng is None else rng
        self.nx = self.Q.shape[0]
        self.nz = self.R.shape[0]
        self.state: Optional[PFState] = None
        self.LR = np.linalg.cholesky(self.R + 1e-12 * np.eye(self.nz))  # pf.py:107 (LinAlgError if not PD)
        if precision not in ("fp32", "fp64"):
            raise ValueError("precision must be 'fp32' or 'fp64'")
        if rng_mode not in ("device", "host"):
            raise ValueError("rng_mode must be 'device' or 'host'")
        self.precision = precision
        self.rng_mode = rng_mode
        self.device = int(device)
        self.kernel_path = kernel_path
        self._path = M.kernel_path_code(kernel_path)
        if not M.is_device_model(g, h):
            raise NotImplementedError(
                "the HIP engine runs g/h on the GPU: pass particle_filters_amd.models objects "
                "(e.g. SVTransition(alpha), ExpHalfObservation(beta)); arbitrary Python callables "
                "cannot be evaluated per particle on the device")
        self._method = N.PF_RESAMPLE_SYSTEMATIC if resample_method == "systematic" else N.PF_RESAMPLE_MULTINOMIAL
        self._desc, self._keep = M.describe(g, h, self.Q, self.R)
        seed = int(self.rng.integers(0, 2 ** 63 - 1)) if rng_mode == "device" else 0
        self._handle = self._create(self.Np, seed)
        self._version = 0
        self._scratch = None

    # ------------------------------------------------------------------ plumbing
    def _create(self, n: int, seed: int):
        lib = N.load()
        opts = N.Opts(n, 1, self._method, self.resample_thresh, int(bool(self.regularize_after_resample)),
                      N.PF_PRECISION_FP64 if self.precision == "fp64" else N.PF_PRECISION_FP32,
                      seed, self.device, 0, self._path)
        h = N.C.c_void_p()
        N.check(lib.pf_create(N.C.byref(self._desc), N.C.byref(opts), N.C.byref(h)), "pf_create")
        return h

    @property
    def kernel_path_used(self) -> str:
        """``"runtime"`` when this filter runs the runtime-shape kernels (pf_dyn.h), else
        ``"compiled"`` (the compiled shape's register-state kernels)."""
        return "runtime" if N.load().pf_kernel_path(self._handle) == N.PF_PATH_RUNTIME else "compiled"

    def __del__(self):
        lib = N._lib
        for name in ("_handle", "_scratch"):
            hnd = getattr(self, name, None)
            if lib is not None and hnd is not None and hnd.value:
                lib.pf_destroy(hnd)
                setattr(self, name, None)

    def _normals(self, n: int) -> Optional[Array]:
        if self.rng_mode != "host":
            return None
        return np.ascontiguousarray(self.rng.standard_normal((n, self.nx)), dtype=float)

    def _download_particles(self) -> Array:
        out = np.empty((self.Np, self.nx))
        N.check(N.load().pf_get_particles(self._handle, N.dptr(out)), "pf_get_particles")
        return out

    def _download_weights(self) -> Array:
        lib = N.load()
        if lib.pf_weights_uniform(self._handle):
            return np.ones(self.Np) / self.Np  # pf.py:210
        out = np.empty(self.Np)
        N.check(lib.pf_get_weights(self._handle, N.dptr(out), None), "pf_get_weights")
        return out

    def _upload_state(self, particles: Array, weights: Optional[Array]) -> None:
        p = np.ascontiguousarray(np.asarray(particles, float).reshape(self.Np, self.nx))
        w = None if weights is None else np.ascontiguousarray(np.asarray(weights, float).reshape(self.Np))
        N.check(N.load().pf_set_state(self._handle, N.dptr(p), N.dptr(w)), "pf_set_state")
        self._version += 1
        self._ess = _uniform_ess(self.Np) if w is None else 1.0 / np.sum(w ** 2)

    # ------------------------------------------------------------------ API
    def initialize(self, mean: Array, cov: Array) -> PFState:
        """Particles ~ N(mean, cov), uniform weights (pf.py:110-132)."""
        mean = np.asarray(mean, float)
        cov = np.asarray(cov, float)
        if mean.shape != (self.nx,):
            raise ValueError(f"mean must have shape ({self.nx},), got {mean.shape}")
        cov2 = np.atleast_2d(cov)
        np.linalg.cholesky(cov2 + 1e-10 * np.eye(len(mean)))  # LinAlgError like pf.py:127
        normals = self._normals(self.Np)
        m = np.ascontiguousarray(mean)
        c = np.ascontiguousarray(cov2)
        N.check(N.load().pf_initialize(self._handle, N.dptr(m), N.dptr(c), N.dptr(normals)), "pf_initialize")
        self._version += 1
        self._ess = _uniform_ess(self.Np)
        self.state = _DeviceState(self, mean, cov2, 0)
        return self.state

    def effective_sample_size(self) -> float:
        """1 / sum(w^2) of the state weights (pf.py:134-144)."""
        assert self.state is not None, "Filter not initialized."
        return float(self._ess)

    def predict(self, u: Optional[Array] = None) -> None:
        """x <- g(x, u) + chol(Q) n (pf.py:223-237); weights unchanged."""
        assert self.state is not None, "Filter not initialized."
        uu = None if u is None else np.ascontiguousarray(np.broadcast_to(np.asarray(u, float), (self.nx,)))
        normals = self._normals(self.Np)
        N.check(N.load().pf_predict(self._handle, N.dptr(uu), N.dptr(normals)), "pf_predict")
        self._version += 1
        self.state = _DeviceState(self, self.state.mean, self.state.cov, self.state.t)

    def update(self, z: Array) -> PFState:
        """Reweight by p(z | x), resample if Neff < thresh*Np, report mean/cov (pf.py:239-269)."""
        assert self.state is not None, "Filter not initialized."
        z = np.ascontiguousarray(np.asarray(z, float).reshape(self.nz))
        lib = N.load()
        info = N.UpdateInfo()
        mean = np.empty(self.nx)
        cov = np.empty((self.nx, self.nx))
        N.check(lib.pf_update(self._handle, N.dptr(z), N.C.byref(info), N.dptr(mean), N.dptr(cov)), "pf_update")
        self.last_neff = float(info.neff)
        self.last_resampled = bool(info.resample)
        self.last_log_norm = float(info.log_norm)
        if info.resample:
            uniforms = jitter = None
            if self.rng_mode == "host":  # the reference's draw order inside _resample (pf.py:160/186, 217)
                if self._method == N.PF_RESAMPLE_SYSTEMATIC:
                    uniforms = np.array([self.rng.random()])
                else:
                    uniforms = np.ascontiguousarray(self.rng.random(self.Np))
                if self.regularize_after_resample:
                    jitter = self._normals(self.Np)
            N.check(lib.pf_resample(self._handle, N.dptr(uniforms), N.dptr(jitter), N.dptr(mean), N.dptr(cov)),
                    "pf_resample")
            self._ess = _uniform_ess(self.Np)
        else:
            self._ess = float(info.neff)
        self._version += 1
        self.state = _DeviceState(self, mean, cov, self.state.t + 1)
        return self.state

    def step(self, z: Array, u: Optional[Array] = None) -> PFState:
        """predict(u) then update(z) (pf.py:271-287)."""
        self.predict(u)
        return self.update(z)

    def run(self, Z, U=None, *, first_update_only: bool = False, with_cov: bool = True):
        """The reference driver loop ``for t: state = step(Z[t], U[t])`` (or ``update(Z[0])``
        first when ``first_update_only``) executed on the GPU with no host sync inside T.
        Device RNG only (host replay needs the per-step resample decisions on the host).
        Returns a :class:`particle_filters_amd.batch.RunResult` with R = 1."""
        assert self.state is not None, "Filter not initialized."
        if self.rng_mode != "device":
            raise ValueError("run() draws on the device; use step() in rng_mode='host'")
        from .batch import RunResult, _uniform_ess as _uess
        Z = np.ascontiguousarray(np.asarray(Z, float).reshape(-1, self.nz))
        T = Z.shape[0]
        Uc = None if U is None else np.ascontiguousarray(np.asarray(U, float).reshape(T, self.nx))
        means = np.zeros((T, 1, self.nx))
        covs = np.zeros((T, 1, self.nx, self.nx)) if with_cov else None
        neff = np.zeros((T, 1))
        flags = np.zeros((T, 1), dtype=np.uint8)
        lnorm = np.zeros((T, 1))
        st = N.load().pf_run(self._handle, N.dptr(Z), N.dptr(Uc), T, int(first_update_only), N.dptr(means),
                             N.dptr(covs), N.dptr(neff), flags.ctypes.data_as(N.C.POINTER(N.C.c_uint8)),
                             N.dptr(lnorm))
        N.check(st, "pf_run")
        fl = flags.astype(bool)
        res = RunResult(means, covs, neff, fl, lnorm, np.where(fl, _uess(self.Np), neff))
        self._version += 1
        self._ess = float(res.ess[-1, 0])
        cov = covs[-1, 0] if covs is not None else None
        self.state = _DeviceState(self, means[-1, 0], cov, self.state.t + T)
        if cov is None:
            c = np.empty((self.nx, self.nx))
            N.check(N.load().pf_moments(self._handle, None, N.dptr(c)), "pf_moments")
            self.state.cov = c
        return res

    # ------------------------------------------------------ checkpoint / resume
    def rng_state(self) -> dict:
        """Philox position of the device RNG (epoch of the next predict)."""
        return N.get_rng_state(self._handle)

    def set_rng_state(self, state: dict) -> None:
        N.set_rng_state(self._handle, state)

    def checkpoint(self) -> dict:
        """Bit-exact snapshot at the step boundary: the engine blob (particles, unnormalised
        log-weights, tile records, Philox position) plus the host side (step count, ESS, the
        host Generator's state for rng_mode='host')."""
        assert self.state is not None, "Filter not initialized."
        blob = N.checkpoint(self._handle)
        return dict(engine=blob, t=int(self.state.t), ess=float(self._ess),
                    rng=self.rng.bit_generator.state if hasattr(self.rng, "bit_generator") else None)

    def restore(self, ckpt: dict) -> PFState:
        """Continue from :meth:`checkpoint` of a filter with the same model and options."""
        N.restore(self._handle, ckpt["engine"])
        if ckpt.get("rng") is not None and hasattr(self.rng, "bit_generator"):
            self.rng.bit_generator.state = ckpt["rng"]
        self._version += 1
        self._ess = float(ckpt["ess"])
        mean = np.empty(self.nx)
        cov = np.empty((self.nx, self.nx))
        N.check(N.load().pf_moments(self._handle, N.dptr(mean), N.dptr(cov)), "pf_moments")
        self.state = _DeviceState(self, mean, cov, int(ckpt["t"]))
        return self.state

    # ------------------------------------------------- reference private helpers
    def _systematic_resample(self, weights: Array) -> Array:
        """Ancestor indices of systematic resampling (pf.py:146-171), computed on the GPU
        with U drawn from ``self.rng`` exactly like the reference."""
        w = np.ascontiguousarray(np.asarray(weights, float))
        U = self.rng.random()
        return resample_indices(w, "systematic", U=U, device=self.device)

    def _multinomial_resample(self, weights: Array) -> Array:
        """``rng.choice(N, N, p=w)`` (pf.py:173-186) on the GPU: the same uniforms
        (``rng.random(N)``, after NumPy's probability checks) and the same search."""
        w = np.ascontiguousarray(np.asarray(weights, float))
        if np.any(w < 0):
            raise ValueError("probabilities are not non-negative")
        if abs(float(np.sum(w)) - 1.0) > np.sqrt(np.finfo(np.float64).eps):
            raise ValueError("probabilities do not sum to 1")
        u = self.rng.random(len(w))
        return resample_indices(w, "multinomial", uniforms=u, device=self.device)

    def _resample(self, particles: Array, weights: Array) -> Tuple[Array, Array]:
        """Neff-gated resampling + optional jitter of caller arrays (pf.py:188-220),
        executed by the engine on a scratch device state."""
        particles = np.asarray(particles, float)
        weights = np.asarray(weights, float)
        n = len(weights)
        if particles.shape != (n, self.nx):
            raise ValueError(f"particles must have shape ({n}, {self.nx})")
        neff = 1.0 / np.sum(weights ** 2)
        if not neff < self.resample_thresh * self.Np:
            return particles, weights
        lib = N.load()
        if self._scratch is None or self._scratch_n != n:
            if self._scratch is not None:
                lib.pf_destroy(self._scratch)
            self._scratch = self._create_scratch(n)
            self._scratch_n = n
        p = np.ascontiguousarray(particles)
        w = np.ascontiguousarray(weights)
        N.check(lib.pf_set_state(self._scratch, N.dptr(p), N.dptr(w)), "pf_set_state")
        # decision on the device from the same weights: force it by a zero-likelihood update
        if self._method == N.PF_RESAMPLE_SYSTEMATIC:
            uniforms = np.array([self.rng.random()])
        else:
            uniforms = np.ascontiguousarray(self.rng.random(n))
        jitter = (np.ascontiguousarray(self.rng.standard_normal((n, self.nx)))
                  if self.regularize_after_resample else None)
        N.check(lib.pf_resample_state(self._scratch, N.dptr(uniforms), N.dptr(jitter)), "pf_resample_state")
        out = np.empty((n, self.nx))
        N.check(lib.pf_get_particles(self._scratch, N.dptr(out)), "pf_get_particles")
        return out, np.ones_like(weights) / len(weights)

    def _create_scratch(self, n: int):
        lib = N.load()
        opts = N.Opts(n, 1, self._method, self.resample_thresh, int(bool(self.regularize_after_resample)),
                      N.PF_PRECISION_FP64, 0, self.device, 0, self._path)
        h = N.C.c_void_p()
        N.check(lib.pf_create(N.C.byref(self._desc), N.C.byref(opts), N.C.byref(h)), "pf_create")
        return h


def resample_indices(weights: Array, method: str = "systematic", *, U: Optional[float] = None,
                     uniforms: Optional[Array] = None, device: int = 0) -> Array:
    """Resampling ancestor indices of normalised ``weights`` on the GPU.

    ``systematic``: ``searchsorted(cumsum(w) with cdf[-1]=1, (U + arange(N))/N, 'right')``
    (pf.py:146-171); ``multinomial``: ``searchsorted(cumsum(w)/cdf[-1], uniforms, 'right')``
    (pf.py:173-186 via ``Generator.choice``).  Returns int64 indices.
    """
    w = np.ascontiguousarray(np.asarray(weights, float))
    n = len(w)
    idx = np.empty(n, dtype=np.int64)
    if method == "systematic":
        if U is None:
            raise ValueError("systematic resampling needs U")
        st = N.load().pf_resample_indices(device, N.PF_RESAMPLE_SYSTEMATIC, N.dptr(w), n, float(U), None,
                                          idx.ctypes.data_as(N.C.POINTER(N.C.c_int64)))
    else:
        u = np.ascontiguousarray(np.asarray(uniforms, float))
        if u.shape != (n,):
            raise ValueError("multinomial resampling needs N uniforms")
        st = N.load().pf_resample_indices(device, N.PF_RESAMPLE_MULTINOMIAL, N.dptr(w), n, 0.0, N.dptr(u),
                                          idx.ctypes.data_as(N.C.POINTER(N.C.c_int64)))
    N.check(st, "pf_resample_indices")
    return idx.astype(int)
