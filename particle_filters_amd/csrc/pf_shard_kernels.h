// Within-filter sharding kernels (include/pf_shard.h): the offspring rows one shard owes the
// global systematic resample, and the adoption of the rows a shard receives.
#pragma once
#include "pf_kernels.h"

namespace pf {

// Rows of global systematic slots [a, a + n) (particle_filter.py:146-171 with positions
// (U + i) / Ntot): the position mapped into this shard's segment [lo, lo + mass) of the global
// CDF, then the first j with pos < cdf[j] in the shard's own normalised CDF (k_cdf).
template <typename Real, int NX>
__global__ void __launch_bounds__(BLOCK) k_shard_offspring(const Real* __restrict__ x, int64_t N, int64_t Npad,
                                                           const double* __restrict__ cdf, double U, double lo,
                                                           double mass, int64_t Ntot, int64_t a, int64_t n,
                                                           Real* __restrict__ out) {
  const int64_t s = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (s >= n) return;
  const double pos = ((U + (double)(a + s)) / (double)Ntot - lo) / mass;
  int64_t l = 0, hi = N;
  while (l < hi) {
    const int64_t mid = (l + hi) >> 1;
    if (pos < cdf[mid]) hi = mid; else l = mid + 1;
  }
  const int64_t j = l < N ? l : N - 1;
#pragma unroll
  for (int d = 0; d < NX; ++d) out[s * NX + d] = x[(int64_t)d * Npad + j];
}

// Received rows -> SoA state (+ the 0.001 chol(Q) jitter of particle_filter.py:212-218 drawn for
// the GLOBAL slot, as the unsharded filter draws it), records -> uniform weights.
template <typename Real, int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(BLOCK) k_shard_adopt(const Real* __restrict__ rows, Real* __restrict__ x, int64_t N,
                                                       int64_t Npad, double* rec, int G, const Real* __restrict__ P,
                                                       int jitter, const double* __restrict__ rp_jit, uint64_t seed,
                                                       uint32_t rep, uint32_t ep, int64_t pbase) {
  using M = Model<Real, NX, NZ, TK, OK>;
  using RC = Rec<NX>;
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i < N) {
    Real v[NX];
#pragma unroll
    for (int d = 0; d < NX; ++d) v[d] = rows[i * NX + d];
    if (jitter) {
      Real nj[NX];
      fill_normals<NX, Real>(seed, i, 0u, rep, ep, STREAM_JITTER, rp_jit, N, nj, pbase);  // replay: [N][NX]
      M::add_lower(v, nj, P, M::L::LJ);
    }
#pragma unroll
    for (int d = 0; d < NX; ++d) x[(int64_t)d * Npad + i] = v[d];
  }
  if (i < G) {
    for (int q = 0; q < RC::SIZE; ++q) rec[(int64_t)q * G + i] = 0.0;
    rec[(int64_t)RC::UNI * G + i] = 1.0;
  }
}

}  // namespace pf
