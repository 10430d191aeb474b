// Standalone resampling of caller-supplied weights (pf_resample_indices):
// the reference's _systematic_resample / _multinomial_resample as pure functions
// (particle_filter.py:146-186).  Included by pf_engine.hip only.
#pragma once
#include "pf_kernels.h"

namespace pf {

// ---------------------------------------------------------------------------
// Standalone resampling of given weights (ParticleFilter._systematic_resample /
// _multinomial_resample): tile sums -> CDF -> search.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(BLOCK) k_w_tile_sums(const double* w, int64_t N, int tile, double* sums) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int64_t s = (int64_t)blockIdx.x * tile;
  const int len = (int)min((int64_t)tile, N - s);
  const int per = (len + BLOCK - 1) / BLOCK;
  const int j0 = threadIdx.x * per;
  double acc = 0.0;
  for (int j = j0; j < j0 + per && j < len; ++j) acc += w[s + j];
  double tot;
  block_excl_scan(acc, smem, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK) k_w_cdf(const double* w, int64_t N, int tile, int G,
                                                 const double* sums, double* cdf, int force_last_one) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  // prefix of tile sums before this tile (same fixed order in every block)
  double run = 0.0;
  {
    double v[4], tsum = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 4 * threadIdx.x + j;
      v[j] = (k < G && k < (int)blockIdx.x) ? sums[k] : 0.0;
      tsum += v[j];
    }
    double tot;
    block_excl_scan(tsum, red, &tot);
    run = tot;
  }
  const int64_t s = (int64_t)blockIdx.x * tile;
  const int len = (int)min((int64_t)tile, N - s);
  const int per = (len + BLOCK - 1) / BLOCK;
  const int j0 = threadIdx.x * per;
  double acc = 0.0;
  for (int j = j0; j < j0 + per && j < len; ++j) acc += w[s + j];
  double tot;
  double off = block_excl_scan(acc, red, &tot) + run;
  for (int j = j0; j < j0 + per && j < len; ++j) {
    off += w[s + j];
    cdf[s + j] = off;
  }
  if (force_last_one && s + len == N && threadIdx.x == 0) {
    // cumsum[-1] = 1.0 (particle_filter.py:163); written after this block's own stores below
  }
  __syncthreads();
  if (force_last_one && s + len == N && (int64_t)(j0 + per) >= len && j0 < len) cdf[N - 1] = 1.0;
}

__global__ void __launch_bounds__(BLOCK) k_w_search(const double* cdf, int64_t N, int method, double U,
                                                    const double* unif, int64_t* idx) {
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= N) return;
  double key;
  double last = 1.0;
  if (method == 0) {
    key = (U + (double)i) / (double)N;
  } else {
    key = unif[i];
    last = cdf[N - 1];
  }
  int64_t lo = 0, hi = N;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const double c = method == 0 ? cdf[mid] : cdf[mid] / last;
    if (key < c) hi = mid; else lo = mid + 1;
  }
  idx[i] = lo < N ? lo : N - 1;
}

}  // namespace pf
