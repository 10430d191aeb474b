"""The fused LEDH step's source-driven systematic resampling (csrc/pf_ledh_fused.h, P3) restated in
NumPy and checked against the destination-side search it replaced, on the CPU.

Workgroup b owns particles [b*ppb, (b+1)*ppb); its CDF slice is c_j = (O_b + f_b scan_j) / S (c = 1
for the global last particle) and its last value last_b.  The destination search (the round-2 kernel,
= the reference's searchsorted(cdf, (U+i)/N, 'right') over monotone slices, ledh.py:25-37) finds for
slot i the first workgroup with pos_i < last_k, then the first j of that slice with pos_i < c_j
(the slice's last particle if none).  The source-driven form gives particle j the slots
{i : max(last_{b-1}, c_{j-1}) <= pos_i < c_j}, the last particle of the last workgroup also every
position past the end, counting positions below a value with the kernel's fast path
(y = x N - U, floor + 1) and its exact fallback near integers.  Both must give the same ancestor of
every slot, bit for bit, for any weights - degenerate ones and exact ties included.
"""

import math
import zlib

import numpy as np
import pytest


def count_below(x, U, N):
    """fcount_below: #{i in [0, N) : (U + i) / N < x}, the kernel's arithmetic."""
    if not x > -math.inf:
        return 0
    if x == math.inf:
        return N
    # the kernel rounds x N - U once (fma); Python < 3.13 has no math.fma, and the product's extra
    # rounding (~1e-12 at these N) stays far inside the 1e-7 band of the exact fallback
    y = math.fma(x, float(N), -U) if hasattr(math, "fma") else x * float(N) - U
    fl = math.floor(y)
    d = y - fl
    c = min(max(int(fl) + 1, 0), N)
    if 1e-7 < d < 1.0 - 1e-7:
        return c
    while c > 0 and (U + float(c - 1)) / float(N) >= x:
        c -= 1
    while c < N and (U + float(c)) / float(N) < x:
        c += 1
    return c


def slices(e, ppb):
    """Per-workgroup scans and the combined prefix, in the kernel's fixed order (fp64)."""
    N = e.size
    nbk = (N + ppb - 1) // ppb
    scans, sums, lasts = [], [], []
    for b in range(nbk):
        s = np.cumsum(e[b * ppb:(b + 1) * ppb])  # the in-workgroup inclusive scan
        scans.append(s)
        sums.append(float(np.sum(e[b * ppb:(b + 1) * ppb])))
        lasts.append(float(s[-1]))
    boff = np.concatenate([[0.0], np.cumsum(sums)[:-1]])
    S = float(np.sum(sums))
    return scans, boff, S, lasts, nbk


def cdf_of(scans, boff, S, N, ppb, b, j):
    g = b * ppb + j
    return 1.0 if g == N - 1 else (boff[b] + scans[b][j]) / S


def destination(e, U, ppb):
    N = e.size
    scans, boff, S, lasts, nbk = slices(e, ppb)
    last = [1.0 if b == nbk - 1 else (boff[b] + lasts[b]) / S for b in range(nbk)]
    anc = np.empty(N, np.int64)
    for i in range(N):
        pos = (U + float(i)) / float(N)
        k = next((b for b in range(nbk) if pos < last[b]), nbk - 1)
        n = scans[k].size
        j = next((jj for jj in range(n) if pos < cdf_of(scans, boff, S, N, ppb, k, jj)), n - 1)
        anc[i] = k * ppb + j
    return anc


def source(e, U, ppb):
    N = e.size
    scans, boff, S, lasts, nbk = slices(e, ppb)
    last = [1.0 if b == nbk - 1 else (boff[b] + lasts[b]) / S for b in range(nbk)]
    anc = np.full(N, -1, np.int64)
    for b in range(nbk):
        n = scans[b].size
        shi = [N if (b == nbk - 1 and j == n - 1) else count_below(cdf_of(scans, boff, S, N, ppb, b, j), U, N)
               for j in range(n)]
        slo0 = count_below(last[b - 1] if b > 0 else -math.inf, U, N)
        j = 0
        for s in range(slo0, shi[n - 1]):
            while shi[j] <= s:
                j += 1
            assert anc[s] == -1, "slot written twice"
            anc[s] = b * ppb + j
    return anc


CASES = [
    ("smooth", lambda rs, N: rs.random(N)),
    ("lognormal", lambda rs, N: np.exp(3.0 * rs.standard_normal(N))),
    ("degenerate", lambda rs, N: np.exp(-40.0 * rs.random(N)) * (rs.random(N) < 0.02)),
    ("one_particle", lambda rs, N: np.eye(1, N, rs.integers(N)).ravel()),
    ("zeros_tail", lambda rs, N: np.concatenate([rs.random(N // 2), np.zeros(N - N // 2)])),
    ("equal", lambda rs, N: np.ones(N)),
]


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("N,ppb", [(1000, 64), (777, 64), (300, 128), (64, 64)])
def test_source_driven_equals_destination_search(name, make, N, ppb):
    rs = np.random.default_rng(zlib.crc32(f"{name}-{N}-{ppb}".encode()))
    for trial in range(3):
        e = np.asarray(make(rs, N), float)
        if e.sum() == 0.0:
            e[rs.integers(N)] = 1.0
        for U in (rs.random(), 0.0, 1.0 - 2.0 ** -53, 0.5):
            a = destination(e, U, ppb)
            b = source(e, U, ppb)
            assert (b >= 0).all(), "a slot got no ancestor"
            np.testing.assert_array_equal(a, b)


def test_equal_weights_hit_exact_boundaries():
    """Equal weights and U = 0 put every position exactly on a CDF value (the fallback path)."""
    N, ppb = 256, 64
    e = np.ones(N)
    np.testing.assert_array_equal(destination(e, 0.0, ppb), source(e, 0.0, ppb))
