"""NumPy Philox4x32-10 + the engine's Box-Muller mapping — TEST INFRASTRUCTURE ONLY.

The reference draws from NumPy's PCG64 (not reproducible on a GPU); the engine's
device RNG is counter-based Philox4x32-10 (Salmon et al., SC'11, as in Random123).
This restatement lets tests check device-drawn numbers exactly: it is pinned to
Random123's published known-answer vectors (tests/test_philox.py) and mirrors
``particle_filters_amd/csrc/philox.h`` (counter = (group, replicate, epoch,
stream), key = seed).
"""

from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)

STREAM_INIT, STREAM_PROCESS, STREAM_JITTER, STREAM_RESAMPLE = 1, 2, 3, 4


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Vectorised Philox4x32-10 over uint32 counter arrays; returns 4 uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & MASK for c in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return [c.astype(np.uint32) for c in (c0, c1, c2, c3)]


def normals(seed: int, n_flat: int, rep: int, epoch: int, stream: int, dtype=np.float64) -> np.ndarray:
    """The first ``n_flat`` normals of (rep, epoch, stream) in flat (particle, dim) order,
    mapped exactly as philox.h's Box-Muller (24-bit uniforms, radius from u01)."""
    groups = (n_flat + 3) // 4
    g = np.arange(groups, dtype=np.uint64)
    x, y, z, w = philox4x32_10(g, rep, epoch, stream, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    f = np.float64 if dtype == np.float64 else np.float32

    def radius(a):
        if f == np.float32:
            u = ((a >> np.uint32(8)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)
        else:
            u = (a.astype(np.float64) + 1.0) * (1.0 / 4294967296.0)
        return np.sqrt(-2.0 * np.log(u.astype(np.float64)))

    def angle(b):
        return (b >> np.uint32(8)).astype(np.float64) * (2.0 / 16777216.0) * np.pi

    r0, r1 = radius(x), radius(z)
    t0, t1 = angle(y), angle(w)
    out = np.stack([r0 * np.cos(t0), r0 * np.sin(t0), r1 * np.cos(t1), r1 * np.sin(t1)], axis=1).ravel()
    return out[:n_flat]


def uniform53(seed: int, index, rep: int, epoch: int) -> np.ndarray:
    """philox.h ``uniform53``: systematic U (index 0) / multinomial u_i on STREAM_RESAMPLE."""
    x, y, _, _ = philox4x32_10(np.asarray(index, dtype=np.uint64), rep, epoch, STREAM_RESAMPLE,
                               seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    a = (x >> np.uint32(5)).astype(np.uint64)
    b = (y >> np.uint32(6)).astype(np.uint64)
    return ((a << np.uint64(26)) | b).astype(np.float64) * (1.0 / 9007199254740992.0)
