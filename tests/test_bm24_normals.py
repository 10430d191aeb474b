"""The flow filters' device-RNG process noise (advisor, round 5): ``normal4_bm24d`` in
particle_filters_amd/csrc/philox.h is the SIR engine's fp32 Box-Muller on 24-bit uniforms, widened
to double.  Its normals have 24-bit resolution and a hard tail cut where the uniform bottoms out:
u >= 2^-24 gives |n| <= sqrt(-2 ln 2^-24) = 5.768 sigma (a two-sided mass of 8e-9 of N(0, 1) is
never drawn).  This checks, on the CPU restatement of the mapping (oracle/philox.py, the same counters
and bit fields), that the draws are N(0, 1) to Monte-Carlo precision: moments, tail masses out to
5 sigma, the truncation point, and that the fp32 evaluation the device does differs from the fp64
evaluation of the same 24-bit uniforms only by fp32 rounding."""

import math

import numpy as np

from oracle import philox

N_DRAWS = 1 << 22


def _draws(bm24=True):
    return philox.normals(1234567, N_DRAWS, 3, 17, philox.STREAM_PROCESS,
                          dtype=np.float32 if bm24 else np.float64)


def test_moments_match_standard_normal():
    n = _draws()
    se = 1.0 / math.sqrt(N_DRAWS)
    assert abs(n.mean()) < 5 * se
    assert abs(n.var() - 1.0) < 5 * math.sqrt(2.0) * se
    z = n / n.std()
    assert abs(np.mean(z ** 3)) < 5 * math.sqrt(6.0) * se          # skewness
    assert abs(np.mean(z ** 4) - 3.0) < 5 * math.sqrt(96.0) * se   # kurtosis


def test_tail_masses_and_truncation():
    n = np.abs(_draws())
    cut = math.sqrt(-2.0 * math.log(2.0 ** -24))
    assert n.max() <= cut * (1 + 1e-12)
    for k in (2.0, 3.0, 4.0, 5.0):
        p = math.erfc(k / math.sqrt(2.0))  # two-sided N(0, 1) tail
        cnt = int(np.count_nonzero(n > k))
        sd = math.sqrt(N_DRAWS * p * (1 - p))
        assert abs(cnt - N_DRAWS * p) <= 5 * sd + 3, (k, cnt, N_DRAWS * p)


def test_fp32_evaluation_is_rounding_of_the_fp64_one():
    """philox.h box_muller4: radius sqrt(-2 ln2 log2 u) and cos/sin of 2 pi a, all in fp32, on the same
    24-bit fields as the fp64 evaluation of the restatement."""
    g = np.arange(N_DRAWS // 4, dtype=np.uint64)
    x, y, z, w = philox.philox4x32_10(g, 3, 17, philox.STREAM_PROCESS, 1234567, 0)
    u = ((x >> np.uint32(8)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)
    a = (y >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    r32 = np.sqrt(np.float32(-1.3862943611198906) * np.log2(u))
    n32 = (r32 * np.cos(np.float32(2.0 * np.pi) * a)).astype(np.float64)
    n64 = _draws()[0::4]
    # a few fp32 ulps of the radius and of the angle (2 pi a rounded to fp32: ~5e-7 absolute)
    r64 = np.sqrt(-2.0 * np.log(u.astype(np.float64)))
    assert np.max(np.abs(n32 - n64)) < 1e-5
    assert np.max(np.abs(n32 - n64) / (1.0 + r64)) < 1e-6
