// SIR particle-filter kernels for gfx950 (CDNA4, wave64).
//
// One launch of k_step = one pass over the particle set, fusing, in order:
//   (0) prologue   every workgroup reduces the previous update's per-tile
//                  partial records (tiny, L2-resident) to the global
//                  log-normaliser, Neff, resample decision, systematic U and the
//                  per-tile weight prefix.  All workgroups run the identical
//                  fixed-order reduction, so they agree bit-for-bit and no
//                  inter-workgroup communication is ever needed inside a launch;
//                  workgroup 0 additionally writes that step's posterior outputs.
//   (1) gather     if the previous update decided to resample: each output slot
//                  finds its ancestor (systematic: walk only the input tiles its
//                  positions land in, scanning each tile's weights in LDS in fp64;
//                  multinomial: binary search of a materialised fp64 CDF), reads
//                  the ancestor and adds the regularisation jitter
//                  (particle_filter.py:188-220).
//   (2) predict    x <- g(x, u) + chol(Q) n   (particle_filter.py:223-237)
//   (3) update     l <- (l_prev - lse_prev) + loglik(z | x)  (particle_filter.py:239-263)
//                  and the tile's online (max, sum e^(l-m), sum e^2(l-m), sum e^(l-m) x, ...)
//                  partial record for the next launch's prologue.
//
// Layout in HBM (replicate-major, structure-of-arrays):
//   x   [R][NX][Npad]  Real     particles (ping-pong pair)
//   lw  [R][Npad]      Real     unnormalised log weights (ping-pong pair)
//   rec [R][G][RS]     double   per-tile partial records (ping-pong pair)
//   cdf [R][N]         double   materialised CDF (multinomial only)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "philox.h"
#include "pf_models.h"

namespace pf {

constexpr int BLOCK = 256;
constexpr int NWAVES = BLOCK / 64;
constexpr int MAXG = 1024;  // tiles per replicate (prologue holds 4 records per thread)

// ---------------------------------------------------------------------------
// Partial record layout (doubles), one per (replicate, tile)
// ---------------------------------------------------------------------------
template <int NX>
struct Rec {
  static constexpr bool COV = NX <= 4;  // in-kernel weighted covariance for small state
  static constexpr int NC = COV ? NX * (NX + 1) / 2 : 0;
  static constexpr int M = 0;        // tile max of l (or -inf)
  static constexpr int S0 = 1;       // sum e^(l-m)
  static constexpr int S00 = 2;      // sum e^(2(l-m))
  static constexpr int UNI = 3;      // 1.0: weights are uniform (after init / resample), head unused
  static constexpr int CNT = 4;      // aux: number of freshly resampled particles in tile (0: aux invalid)
  static constexpr int S1 = 5;       // NX   sum e^(l-m) x_d
  static constexpr int S2 = S1 + NX; // NC   sum e^(l-m) x_d x_e (d<=e)
  static constexpr int A1 = S2 + NC; // NX   aux: sum x_d of resampled particles
  static constexpr int A2 = A1 + NX; // NC   aux: sum x_d x_e
  static constexpr int SIZE = A2 + NC;
};

template <typename Real>
__device__ __forceinline__ Real exp_r(Real v);
template <>
__device__ __forceinline__ float exp_r<float>(float v) { return __expf(v); }
template <>
__device__ __forceinline__ double exp_r<double>(double v) { return exp(v); }

// ---------------------------------------------------------------------------
// Wave / block collectives (fixed combination order -> deterministic)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double wave_incl_scan(double v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

// every thread returns the block total; `red` holds NWAVES doubles
__device__ __forceinline__ double block_sum(double v, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < NWAVES; ++i) s += red[i];
  return s;
}
__device__ __forceinline__ double block_max(double v, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < NWAVES; ++i) s = fmax(s, red[i]);
  return s;
}
__device__ __forceinline__ int block_min_i(int v, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_min_i(v);
  __syncthreads();
  if (lane == 0) ((int*)red)[w] = v;
  __syncthreads();
  int s = ((int*)red)[0];
#pragma unroll
  for (int i = 1; i < NWAVES; ++i) s = min(s, ((int*)red)[i]);
  return s;
}
// exclusive block scan; returns this thread's offset, *total = block total
__device__ __forceinline__ double block_excl_scan(double v, double* red, double* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double incl = wave_incl_scan(v, lane);
  __syncthreads();
  if (lane == 63) red[w] = incl;
  __syncthreads();
  double off = 0.0, tot = 0.0;
#pragma unroll
  for (int i = 0; i < NWAVES; ++i) {
    if (i < w) off += red[i];
    tot += red[i];
  }
  *total = tot;
  return off + incl - v;
}

// ---------------------------------------------------------------------------
// Online weighted accumulator (per thread), combined across lanes/waves
// ---------------------------------------------------------------------------
template <typename Real, int NX>
struct WAcc {
  using RC = Rec<NX>;
  double m;  // running max of l (exact value of some l)
  double s0, s00;
  double s1[NX];
  double s2[RC::NC > 0 ? RC::NC : 1];

  __device__ __forceinline__ void init() {
    m = -INFINITY;
    s0 = s00 = 0.0;
#pragma unroll
    for (int d = 0; d < NX; ++d) s1[d] = 0.0;
#pragma unroll
    for (int c = 0; c < RC::NC; ++c) s2[c] = 0.0;
  }
  __device__ __forceinline__ void scale(double f) {
    s0 *= f;
    s00 *= f * f;
#pragma unroll
    for (int d = 0; d < NX; ++d) s1[d] *= f;
#pragma unroll
    for (int c = 0; c < RC::NC; ++c) s2[c] *= f;
  }
  __device__ __forceinline__ void add(Real l, const Real* x) {
    if (!(l > -INFINITY)) return;  // zero weight (l = -inf); NaN also skipped here, caught by neff
    if ((double)l > m) {
      if (m > -INFINITY) scale((double)exp_r<Real>((Real)(m - (double)l)));
      m = (double)l;
    }
    const double e = (double)exp_r<Real>(l - (Real)m);
    s0 += e;
    s00 += e * e;
#pragma unroll
    for (int d = 0; d < NX; ++d) s1[d] += e * (double)x[d];
    if constexpr (RC::COV) {
      int c = 0;
#pragma unroll
      for (int d = 0; d < NX; ++d)
#pragma unroll
        for (int f = d; f < NX; ++f) s2[c++] += e * (double)x[d] * (double)x[f];
    }
  }
  __device__ __forceinline__ void merge(double om, double os0, double os00, const double* os1,
                                        const double* os2) {
    if (!(om > -INFINITY)) return;
    if (!(m > -INFINITY)) {
      m = om;
      s0 = os0;
      s00 = os00;
#pragma unroll
      for (int d = 0; d < NX; ++d) s1[d] = os1[d];
#pragma unroll
      for (int c = 0; c < RC::NC; ++c) s2[c] = os2[c];
      return;
    }
    const double M = fmax(m, om);
    const double fa = exp(m - M), fb = exp(om - M);
    s0 = s0 * fa + os0 * fb;
    s00 = s00 * fa * fa + os00 * fb * fb;
#pragma unroll
    for (int d = 0; d < NX; ++d) s1[d] = s1[d] * fa + os1[d] * fb;
#pragma unroll
    for (int c = 0; c < RC::NC; ++c) s2[c] = s2[c] * fa + os2[c] * fb;
    m = M;
  }
  __device__ __forceinline__ void wave_reduce() {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      double om = __shfl_xor(m, o), os0 = __shfl_xor(s0, o), os00 = __shfl_xor(s00, o);
      double os1[NX], os2[RC::NC > 0 ? RC::NC : 1];
#pragma unroll
      for (int d = 0; d < NX; ++d) os1[d] = __shfl_xor(s1[d], o);
#pragma unroll
      for (int c = 0; c < RC::NC; ++c) os2[c] = __shfl_xor(s2[c], o);
      merge(om, os0, os00, os1, os2);
    }
  }
};

// ---------------------------------------------------------------------------
// Kernel parameters (by value)
// ---------------------------------------------------------------------------
struct StepParams {
  const void* x_in;
  void* x_out;
  const void* lw_in;
  void* lw_out;
  const double* rec_in;
  double* rec_out;
  const void* P;          // Real[PSIZE] model parameters (shared by replicates)
  const void* z;          // Real[R][NZ] (stride z_rs)
  const void* u;          // Real[R][NX] control or null
  const double* rp_noise; // replay process normals [R][N][NX] or null
  const double* rp_jit;   // replay jitter normals [R][N][NX] or null
  const double* rp_unif;  // replay resample uniforms: [R] (systematic) / [R][N] (multinomial) or null
  const double* cdf;      // [R][N] materialised CDF (multinomial) or null
  double* o_mean;         // [.][R][NX]
  double* o_cov;          // [.][R][NX][NX] (NX <= 4) or null
  double* o_neff;         // [.][R]
  double* o_lse;          // [.][R]
  int32_t* o_flag;        // [.][R]
  int64_t out_step;       // index for the weighted stats of the update in rec_in (-1: none)
  int64_t out_post_step;  // index for the post-resample stats in rec_in's aux (-1: none)
  int64_t N, Npad;
  int64_t z_rs, u_rs;
  int G, tile;
  uint64_t seed;
  uint32_t ep_predict, ep_resample;
  double thresh;
  int method;             // 0 systematic, 1 multinomial
  int do_predict, do_update, allow_gather, regularize, r_diag;
  int force_gather;       // resample regardless of Neff (ParticleFilter._resample after its own test)
  int rep_base;           // global id of replicate 0 of this launch (Philox counter word)
};

struct Head {
  double M, S, S2, lse, neff, U;
  int uniform, resample;
};

// Reduce the weight heads of rec (this replicate): M, S, S2, lse, Neff, decision,
// and (if want_prefix) the normalised exclusive tile prefix P[0..G] into `Pl`.
// Identical instruction stream in every workgroup -> identical results.
__device__ __forceinline__ Head reduce_heads(const double* rec, int RS, int G, int64_t N, double thresh,
                                             bool allow, double* red, double* Pl, bool want_prefix,
                                             bool force = false) {
  Head h;
  h.uniform = rec[3] != 0.0;  // same in every record of a launch
  h.resample = 0;
  h.U = 0.0;
  if (h.uniform) {
    h.M = 0.0;
    h.S = 1.0;
    h.S2 = 1.0 / (double)N;
    h.lse = 0.0;
    h.neff = (double)N;
    return h;
  }
  const int t = threadIdx.x;
  double mk[4], s0k[4], s00k[4];
  double lmax = -INFINITY;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 4 * t + j;
    if (k < G) {
      mk[j] = rec[(int64_t)k * RS + 0];
      s0k[j] = rec[(int64_t)k * RS + 1];
      s00k[j] = rec[(int64_t)k * RS + 2];
      if (s0k[j] > 0.0) lmax = fmax(lmax, mk[j]);
    } else {
      mk[j] = -INFINITY;
      s0k[j] = s00k[j] = 0.0;
    }
  }
  const double M = block_max(lmax, red);
  double wk[4], v2 = 0.0, tsum = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double f = (s0k[j] > 0.0) ? exp(mk[j] - M) : 0.0;
    wk[j] = s0k[j] * f;
    v2 += s00k[j] * f * f;
    tsum += wk[j];
  }
  double S;
  const double off = block_excl_scan(tsum, red, &S);
  const double S2 = block_sum(v2, red);
  h.M = M;
  h.S = S;
  h.S2 = S2;
  h.lse = M + log(S);
  h.neff = (S * S) / S2;
  h.resample = allow && (force || h.neff < thresh * (double)N);
  if (want_prefix) {
    double run = off;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 4 * t + j;
      if (k < G) Pl[k] = run / S;
      run += wk[j];
    }
    if (t == 0) Pl[G] = 1.0;
    __syncthreads();
  }
  return h;
}

// Block 0 only: posterior outputs of the update whose records are in `rec`
// (weighted mean/cov, Neff, lse, decision) and of a resample whose fresh particles
// were summarised in rec's aux part (uniform-weight mean/cov).
template <int NX>
__device__ void write_outputs(const StepParams& p, const double* rec, const Head& h, int r, int R,
                              double* red) {
  using RC = Rec<NX>;
  const int t = threadIdx.x;
  if (p.out_step >= 0 && !h.uniform) {
    const int64_t o = p.out_step * R + r;
    for (int q = 0; q < NX + RC::NC; ++q) {
      double acc = 0.0;
      for (int k = 4 * t; k < 4 * t + 4 && k < p.G; ++k) {
        const double s0 = rec[(int64_t)k * RC::SIZE + RC::S0];
        if (s0 > 0.0) acc += rec[(int64_t)k * RC::SIZE + RC::S1 + q] * exp(rec[(int64_t)k * RC::SIZE] - h.M);
      }
      const double tot = block_sum(acc, red) / h.S;
      if (t == 0) red[8 + q] = tot;  // stash E[x_d], E[x_d x_e]
    }
    __syncthreads();
    if (t == 0) {
      for (int d = 0; d < NX; ++d) p.o_mean[o * NX + d] = red[8 + d];
      if (RC::COV && p.o_cov) {
        int c = 0;
        for (int d = 0; d < NX; ++d)
          for (int f = d; f < NX; ++f, ++c) {
            const double v = red[8 + NX + c] - red[8 + d] * red[8 + f];
            p.o_cov[o * NX * NX + d * NX + f] = v;
            p.o_cov[o * NX * NX + f * NX + d] = v;
          }
      }
      p.o_neff[o] = h.neff;
      p.o_lse[o] = h.lse;
      p.o_flag[o] = h.resample;
    }
    __syncthreads();
  }
  if (p.out_post_step >= 0) {
    double cnt = 0.0;
    for (int k = 4 * t; k < 4 * t + 4 && k < p.G; ++k) cnt += rec[(int64_t)k * RC::SIZE + RC::CNT];
    cnt = block_sum(cnt, red);
    if (cnt > 0.0) {
      const int64_t o = p.out_post_step * R + r;
      for (int q = 0; q < NX + RC::NC; ++q) {
        double acc = 0.0;
        for (int k = 4 * t; k < 4 * t + 4 && k < p.G; ++k) acc += rec[(int64_t)k * RC::SIZE + RC::A1 + q];
        const double tot = block_sum(acc, red) / cnt;
        if (t == 0) red[8 + q] = tot;
      }
      __syncthreads();
      if (t == 0) {
        for (int d = 0; d < NX; ++d) p.o_mean[o * NX + d] = red[8 + d];
        if (RC::COV && p.o_cov) {
          int c = 0;
          for (int d = 0; d < NX; ++d)
            for (int f = d; f < NX; ++f, ++c) {
              const double v = red[8 + NX + c] - red[8 + d] * red[8 + f];
              p.o_cov[o * NX * NX + d * NX + f] = v;
              p.o_cov[o * NX * NX + f * NX + d] = v;
            }
        }
      }
      __syncthreads();
    }
  }
}

// Build the global CDF values of input tile k in LDS:
//   cdf[j] = P_k + (e^(m_k - M) / S) * sum_{j' <= j} e^(l_j' - m_k)
// (the same per-element weights the update's partial records summed).
template <typename Real>
__device__ __forceinline__ int tile_cdf(const Real* __restrict__ lw, int64_t N, int tile, int k,
                                        double mk, const Head& h, const double* Pl, double* cdf,
                                        double* red) {
  const int64_t s = (int64_t)k * tile;
  const int len = (int)min((int64_t)tile, N - s);
  const int per = (len + BLOCK - 1) / BLOCK;
  const int j0 = threadIdx.x * per;
  const Real m = (Real)mk;
  double acc = 0.0;
  for (int j = j0; j < j0 + per && j < len; ++j) {
    const Real l = lw[s + j];
    acc += (l > -INFINITY) ? (double)exp_r<Real>(l - m) : 0.0;
  }
  double tot;
  double off = block_excl_scan(acc, red, &tot);
  const double c = exp(mk - h.M) / h.S;
  const double base = Pl[k];
  for (int j = j0; j < j0 + per && j < len; ++j) {
    const Real l = lw[s + j];
    off += (l > -INFINITY) ? (double)exp_r<Real>(l - m) : 0.0;
    cdf[j] = base + c * off;
  }
  __syncthreads();
  return len;
}

// first j in [0, len) with pos < cdf[j]; len-1 if none
__device__ __forceinline__ int lds_upper(const double* cdf, int len, double pos) {
  int lo = 0, hi = len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (pos < cdf[mid]) hi = mid; else lo = mid + 1;
  }
  return lo < len ? lo : len - 1;
}
__device__ __forceinline__ int prefix_tile(const double* Pl, int G, double pos) {
  // first k with pos < P[k+1]
  int lo = 0, hi = G;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (pos < Pl[mid + 1]) hi = mid; else lo = mid + 1;
  }
  return lo < G ? lo : G - 1;
}

template <int NX>
__device__ __forceinline__ void fill_normals(uint64_t seed, int64_t i, uint32_t lrep, uint32_t rep, uint32_t ep,
                                             uint32_t stream, const double* replay, int64_t N,
                                             float* n) {
  if (replay) {
#pragma unroll
    for (int d = 0; d < NX; ++d) n[d] = (float)replay[((int64_t)lrep * N + i) * NX + d];
    return;
  }
  const int64_t f0 = i * NX, f1 = f0 + NX - 1;
  constexpr int GMAX = (NX % 4 == 0) ? NX / 4 : NX / 4 + 2;
#pragma unroll
  for (int gg = 0; gg < GMAX; ++gg) {
    const int64_t g = (f0 >> 2) + gg;
    if (g > (f1 >> 2)) break;
    const Normal4<float> q = normal4<float>(seed, (uint32_t)g, rep, ep, stream);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t f = 4 * g + e;
      if (f >= f0 && f <= f1) n[f - f0] = q.v[e];
    }
  }
}
template <int NX>
__device__ __forceinline__ void fill_normals(uint64_t seed, int64_t i, uint32_t lrep, uint32_t rep, uint32_t ep,
                                             uint32_t stream, const double* replay, int64_t N,
                                             double* n) {
  if (replay) {
#pragma unroll
    for (int d = 0; d < NX; ++d) n[d] = replay[((int64_t)lrep * N + i) * NX + d];
    return;
  }
  const int64_t f0 = i * NX, f1 = f0 + NX - 1;
  constexpr int GMAX = (NX % 4 == 0) ? NX / 4 : NX / 4 + 2;
#pragma unroll
  for (int gg = 0; gg < GMAX; ++gg) {
    const int64_t g = (f0 >> 2) + gg;
    if (g > (f1 >> 2)) break;
    const Normal4<double> q = normal4<double>(seed, (uint32_t)g, rep, ep, stream);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t f = 4 * g + e;
      if (f >= f0 && f <= f1) n[f - f0] = q.v[e];
    }
  }
}

// 16-byte (fp32) / 2x16-byte (fp64) vector moves of 4 consecutive slots
template <typename Real>
__device__ __forceinline__ void load4(const Real* src, Real& a, Real& b, Real& c, Real& d) {
  if constexpr (sizeof(Real) == 4) {
    const float4 v = *(const float4*)src;
    a = v.x; b = v.y; c = v.z; d = v.w;
  } else {
    const double2 v0 = *(const double2*)src;
    const double2 v1 = *(const double2*)(src + 2);
    a = v0.x; b = v0.y; c = v1.x; d = v1.y;
  }
}
template <typename Real>
__device__ __forceinline__ void store4(Real* dst, Real a, Real b, Real c, Real d) {
  if constexpr (sizeof(Real) == 4) {
    *(float4*)dst = make_float4(a, b, c, d);
  } else {
    *(double2*)dst = make_double2(a, b);
    *(double2*)(dst + 2) = make_double2(c, d);
  }
}
// normals of particles i0..i0+3 of a scalar state (flat indices i0..i0+3 = one group)
template <typename Real>
__device__ __forceinline__ void chunk_normals4(uint64_t seed, int64_t i0, uint32_t lrep, uint32_t rep, uint32_t ep,
                                               uint32_t stream, const double* replay, int64_t N,
                                               Real* n) {
  if (replay) {
#pragma unroll
    for (int e = 0; e < 4; ++e) n[e] = (i0 + e < N) ? (Real)replay[(int64_t)lrep * N + i0 + e] : Real(0);
    return;
  }
  const Normal4<Real> q = normal4<Real>(seed, (uint32_t)(i0 >> 2), rep, ep, stream);
#pragma unroll
  for (int e = 0; e < 4; ++e) n[e] = q.v[e];
}

// ---------------------------------------------------------------------------
// The fused step kernel
// ---------------------------------------------------------------------------
// Work split: workgroup (b, r) owns particle slots [b*tile, (b+1)*tile) of
// replicate r.  A thread owns "chunks" of CH consecutive slots (CH = 4 for the
// scalar state so x/lw move as 16-byte vectors), at most MAXC chunks.
template <typename Real, int NX, int NZ, int TK, int OK>
struct StepTraits {
  static constexpr int CH = (NX == 1) ? 4 : 1;
  static constexpr int MAXC = (NX == 1) ? 8 : 4;
  static constexpr int TILE_MAX = BLOCK * CH * MAXC;
};

template <typename Real, int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(BLOCK) k_step(StepParams p) {
  using M = Model<Real, NX, NZ, TK, OK>;
  using RC = Rec<NX>;
  using TR = StepTraits<Real, NX, NZ, TK, OK>;
  constexpr int CH = TR::CH, MAXC = TR::MAXC;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;                   // 64 doubles scratch
  double* Pl = smem + 64;               // G + 1 prefix
  double* cdf = smem + 64 + MAXG + 8;   // tile doubles

  const int b = blockIdx.x, r = blockIdx.y, R = gridDim.y;
  const int t = threadIdx.x;
  const Real* __restrict__ P = (const Real*)p.P;
  const Real* x_in = (const Real*)p.x_in + (int64_t)r * NX * p.Npad;
  Real* x_out = (Real*)p.x_out + (int64_t)r * NX * p.Npad;
  const Real* lw_in = (const Real*)p.lw_in + (int64_t)r * p.Npad;
  Real* lw_out = (Real*)p.lw_out + (int64_t)r * p.Npad;
  const double* rec_in = p.rec_in + (int64_t)r * p.G * RC::SIZE;
  const int64_t o0 = (int64_t)b * p.tile;
  const int64_t o1 = min(o0 + (int64_t)p.tile, p.N);
  const int nchunks = (int)((o1 - o0 + CH - 1) / CH);

  // ---- (0) prologue -------------------------------------------------------
  const bool need_gather_info = p.allow_gather != 0;
  Head h = reduce_heads(rec_in, RC::SIZE, p.G, p.N, p.thresh, p.allow_gather != 0, red, Pl,
                        need_gather_info && p.method == 0, p.force_gather != 0);
  if (b == 0) write_outputs<NX>(p, rec_in, h, r, R, red);
  const bool gather = h.resample != 0;
  if (gather && p.method == 0)
    h.U = p.rp_unif ? p.rp_unif[r] : uniform53(p.seed, 0, (uint32_t)(r + p.rep_base), p.ep_resample);
  const double lprev_uniform = -log((double)p.N);

  // ---- (1) ancestors -----------------------------------------------------
  int anc[MAXC][CH];
  if (gather) {
    if (p.method == 0) {
      int kk[MAXC][CH];
      int nextk = p.G;
      for (int q = 0; q < MAXC; ++q) {
        const int c = t + q * BLOCK;
#pragma unroll
        for (int e = 0; e < CH; ++e) {
          kk[q][e] = p.G;
          anc[q][e] = -1;
          const int64_t i = o0 + (int64_t)c * CH + e;
          if (c < nchunks && i < o1) {
            const double pos = (h.U + (double)i) / (double)p.N;
            kk[q][e] = prefix_tile(Pl, p.G, pos);
            nextk = min(nextk, kk[q][e]);
          }
        }
      }
      int k = block_min_i(nextk, red);
      while (k < p.G) {
        const double mk = rec_in[(int64_t)k * RC::SIZE + RC::M];
        const int len = tile_cdf<Real>(lw_in, p.N, p.tile, k, mk, h, Pl, cdf, red);
        nextk = p.G;
        for (int q = 0; q < MAXC; ++q) {
#pragma unroll
          for (int e = 0; e < CH; ++e) {
            if (kk[q][e] == k) {
              const int64_t i = o0 + (int64_t)(t + q * BLOCK) * CH + e;
              const double pos = (h.U + (double)i) / (double)p.N;
              anc[q][e] = (int)((int64_t)k * p.tile + lds_upper(cdf, len, pos));
              kk[q][e] = p.G;
            } else if (kk[q][e] < p.G) {
              nextk = min(nextk, kk[q][e]);
            }
          }
        }
        __syncthreads();  // cdf reused by the next tile
        k = block_min_i(nextk, red);
      }
    } else {  // multinomial: binary search in the materialised CDF (cdf /= cdf[-1])
      const double* C = p.cdf + (int64_t)r * p.N;
      const double last = C[p.N - 1];
      for (int q = 0; q < MAXC; ++q) {
        const int c = t + q * BLOCK;
#pragma unroll
        for (int e = 0; e < CH; ++e) {
          const int64_t i = o0 + (int64_t)c * CH + e;
          anc[q][e] = -1;
          if (c < nchunks && i < o1) {
            const double uu = p.rp_unif ? p.rp_unif[(int64_t)r * p.N + i]
                                        : uniform53(p.seed, (uint32_t)i, (uint32_t)(r + p.rep_base), p.ep_resample);
            int64_t lo = 0, hi = p.N;
            while (lo < hi) {
              const int64_t mid = (lo + hi) >> 1;
              if (uu < C[mid] / last) hi = mid; else lo = mid + 1;
            }
            anc[q][e] = (int)(lo < p.N ? lo : p.N - 1);
          }
        }
      }
    }
  }

  // ---- (2)+(3) per particle -----------------------------------------------
  WAcc<Real, NX> acc;
  acc.init();
  double aux_cnt = 0.0, aux1[NX], aux2[RC::NC > 0 ? RC::NC : 1];
#pragma unroll
  for (int d = 0; d < NX; ++d) aux1[d] = 0.0;
#pragma unroll
  for (int c = 0; c < RC::NC; ++c) aux2[c] = 0.0;

  Real z[NZ];
  if (p.do_update) {
#pragma unroll
    for (int k = 0; k < NZ; ++k) z[k] = ((const Real*)p.z)[(int64_t)r * p.z_rs + k];
  }
  const Real* u = p.u ? (const Real*)p.u + (int64_t)r * p.u_rs : nullptr;
  const double lse_prev = h.uniform ? 0.0 : h.lse;

  const bool write_x = p.do_predict || p.allow_gather;  // gather launches always produce x_out
  for (int q = 0; q < MAXC; ++q) {
    const int c = t + q * BLOCK;
    if (c >= nchunks) break;
    const int64_t i0 = o0 + (int64_t)c * CH;
    Real xs[CH][NX];
    Real lp[CH];
    // load (or gather) the particle(s) and their normalised previous log weight
    if (gather) {
#pragma unroll
      for (int e = 0; e < CH; ++e) {
        const int a = anc[q][e] < 0 ? 0 : anc[q][e];
#pragma unroll
        for (int d = 0; d < NX; ++d) xs[e][d] = x_in[(int64_t)d * p.Npad + a];
        lp[e] = (Real)lprev_uniform;
      }
    } else if constexpr (CH == 4) {
      load4<Real>(x_in + i0, xs[0][0], xs[1][0], xs[2][0], xs[3][0]);
      if (p.do_update) {
        if (h.uniform) {
#pragma unroll
          for (int e = 0; e < 4; ++e) lp[e] = (Real)lprev_uniform;
        } else {
          Real l0, l1, l2, l3;
          load4<Real>(lw_in + i0, l0, l1, l2, l3);
          lp[0] = (Real)((double)l0 - lse_prev); lp[1] = (Real)((double)l1 - lse_prev);
          lp[2] = (Real)((double)l2 - lse_prev); lp[3] = (Real)((double)l3 - lse_prev);
        }
      }
    } else {
#pragma unroll
      for (int d = 0; d < NX; ++d) xs[0][d] = x_in[(int64_t)d * p.Npad + i0];
      if (p.do_update)
        lp[0] = h.uniform ? (Real)lprev_uniform : (Real)((double)lw_in[i0] - lse_prev);
    }

    // scalar state: one Philox call yields the normals of the chunk's 4 particles
    Real nj4[CH], np4[CH];
    if constexpr (CH == 4) {
      if (gather && p.regularize) chunk_normals4<Real>(p.seed, i0, (uint32_t)r, (uint32_t)(r + p.rep_base), p.ep_resample, STREAM_JITTER, p.rp_jit, p.N, nj4);
      if (p.do_predict) chunk_normals4<Real>(p.seed, i0, (uint32_t)r, (uint32_t)(r + p.rep_base), p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, np4);
    }

#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const int64_t i = i0 + e;
      const bool live = i < o1;
      Real* x = xs[e];
      if (gather && live) {
        if (p.regularize) {
          Real n[NX];
          if constexpr (CH == 4) n[0] = nj4[e];
          else fill_normals<NX>(p.seed, i, (uint32_t)r, (uint32_t)(r + p.rep_base), p.ep_resample, STREAM_JITTER, p.rp_jit, p.N, n);
          M::add_lower(x, n, P, M::L::LJ);
        }
        aux_cnt += 1.0;
#pragma unroll
        for (int d = 0; d < NX; ++d) aux1[d] += (double)x[d];
        if constexpr (RC::COV) {
          int cc = 0;
#pragma unroll
          for (int d = 0; d < NX; ++d)
#pragma unroll
            for (int f = d; f < NX; ++f) aux2[cc++] += (double)x[d] * (double)x[f];
        }
      }
      if (p.do_predict && live) {
        Real n[NX];
        if constexpr (CH == 4) n[0] = np4[e];
        else fill_normals<NX>(p.seed, i, (uint32_t)r, (uint32_t)(r + p.rep_base), p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, n);
        M::transition(x, P, u);
        M::add_lower(x, n, P, M::L::LQ);
      }
      if (p.do_update && live) {
        if (p.do_update == 1) lp[e] = lp[e] + M::loglik(x, z, P, p.r_diag != 0);  // 2: reweigh only
        acc.add(lp[e], x);
      }
    }
    // store
    if constexpr (CH == 4) {
      if (i0 + 3 < o1) {
        if (write_x) store4<Real>(x_out + i0, xs[0][0], xs[1][0], xs[2][0], xs[3][0]);
        if (p.do_update) store4<Real>(lw_out + i0, lp[0], lp[1], lp[2], lp[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (i0 + e < o1) {
            if (write_x) x_out[i0 + e] = xs[e][0];
            if (p.do_update) lw_out[i0 + e] = lp[e];
          }
        }
      }
    } else {
      if (write_x)
#pragma unroll
        for (int d = 0; d < NX; ++d) x_out[(int64_t)d * p.Npad + i0] = xs[0][d];
      if (p.do_update) lw_out[i0] = lp[0];
    }
  }

  // ---- partial record ------------------------------------------------------
  // (written only by launches that produce records: updates and gathers)
  if (!(p.do_update || p.allow_gather)) return;
  double* rec_out = p.rec_out + ((int64_t)r * p.G + b) * RC::SIZE;
  double* wsm = smem + 64 + MAXG + 8;  // reuse cdf area: NWAVES x (RC::SIZE) doubles
  __syncthreads();
  if (p.do_update) {
    acc.wave_reduce();
    if ((t & 63) == 0) {
      double* o = wsm + (t >> 6) * RC::SIZE;
      o[RC::M] = acc.m; o[RC::S0] = acc.s0; o[RC::S00] = acc.s00;
#pragma unroll
      for (int d = 0; d < NX; ++d) o[RC::S1 + d] = acc.s1[d];
#pragma unroll
      for (int c = 0; c < RC::NC; ++c) o[RC::S2 + c] = acc.s2[c];
    }
  }
  // aux sums (plain adds)
  if (gather) {
    aux_cnt = wave_sum(aux_cnt);
#pragma unroll
    for (int d = 0; d < NX; ++d) aux1[d] = wave_sum(aux1[d]);
#pragma unroll
    for (int c = 0; c < RC::NC; ++c) aux2[c] = wave_sum(aux2[c]);
    if ((t & 63) == 0) {
      double* o = wsm + (t >> 6) * RC::SIZE;
      o[RC::CNT] = aux_cnt;
#pragma unroll
      for (int d = 0; d < NX; ++d) o[RC::A1 + d] = aux1[d];
#pragma unroll
      for (int c = 0; c < RC::NC; ++c) o[RC::A2 + c] = aux2[c];
    }
  }
  __syncthreads();
  if (t == 0) {
    if (p.do_update) {
      WAcc<Real, NX> tot;
      tot.init();
      for (int w = 0; w < NWAVES; ++w) {
        const double* o = wsm + w * RC::SIZE;
        tot.merge(o[RC::M], o[RC::S0], o[RC::S00], o + RC::S1, o + RC::S2);
      }
      rec_out[RC::M] = tot.m; rec_out[RC::S0] = tot.s0; rec_out[RC::S00] = tot.s00;
      rec_out[RC::UNI] = 0.0;
      for (int d = 0; d < NX; ++d) rec_out[RC::S1 + d] = tot.s1[d];
      for (int c = 0; c < RC::NC; ++c) rec_out[RC::S2 + c] = tot.s2[c];
    } else if (gather) {  // gather-only launch: weights become uniform
      rec_out[RC::M] = 0.0; rec_out[RC::S0] = 0.0; rec_out[RC::S00] = 0.0;
      rec_out[RC::UNI] = 1.0;
    } else {  // gather-only launch that did not resample: carry the update's head over
      const double* ri = rec_in + (int64_t)b * RC::SIZE;
      for (int q = 0; q < RC::A1; ++q) rec_out[q] = ri[q];
    }
    if (gather) {
      double cnt = 0.0;
      for (int w = 0; w < NWAVES; ++w) cnt += wsm[w * RC::SIZE + RC::CNT];
      rec_out[RC::CNT] = cnt;
      for (int q = 0; q < NX + RC::NC; ++q) {
        double s = 0.0;
        for (int w = 0; w < NWAVES; ++w) s += wsm[w * RC::SIZE + RC::A1 + q];
        rec_out[RC::A1 + q] = s;
      }
    } else {
      rec_out[RC::CNT] = 0.0;
    }
  }
}

// ---------------------------------------------------------------------------
// Finalize: posterior outputs of the records in rec (one workgroup per replicate)
// ---------------------------------------------------------------------------
template <int NX>
__global__ void __launch_bounds__(BLOCK) k_finalize(StepParams p) {
  using RC = Rec<NX>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  const int r = blockIdx.x, R = gridDim.x;
  const double* rec = p.rec_in + (int64_t)r * p.G * RC::SIZE;
  Head h = reduce_heads(rec, RC::SIZE, p.G, p.N, p.thresh, p.allow_gather != 0, red, nullptr, false);
  write_outputs<NX>(p, rec, h, r, R, red);
}

// ---------------------------------------------------------------------------
// Multinomial: materialise the CDF of the update in rec_in (if it resamples)
// ---------------------------------------------------------------------------
template <typename Real, int NX>
__global__ void __launch_bounds__(BLOCK) k_cdf(StepParams p, double* cdf_out) {
  using RC = Rec<NX>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  double* Pl = smem + 64;
  double* cdf = smem + 64 + MAXG + 8;
  const int b = blockIdx.x, r = blockIdx.y;
  const double* rec = p.rec_in + (int64_t)r * p.G * RC::SIZE;
  Head h = reduce_heads(rec, RC::SIZE, p.G, p.N, p.thresh, true, red, Pl, true, p.force_gather != 0);
  if (!h.resample) return;
  const Real* lw = (const Real*)p.lw_in + (int64_t)r * p.Npad;
  const double mk = rec[(int64_t)b * RC::SIZE + RC::M];
  const int len = tile_cdf<Real>(lw, p.N, p.tile, b, mk, h, Pl, cdf, red);
  for (int j = threadIdx.x; j < len; j += BLOCK) cdf_out[(int64_t)r * p.N + (int64_t)b * p.tile + j] = cdf[j];
}

// ---------------------------------------------------------------------------
// initialize(): x = mean + chol(cov) n, records -> uniform weights
// ---------------------------------------------------------------------------
template <typename Real, int NX>
__global__ void __launch_bounds__(BLOCK) k_init(Real* x, double* rec, const Real* mean /*[R][NX]*/,
                                                const Real* Lc /*[R][NX][NX]*/, const double* replay,
                                                int64_t N, int64_t Npad, int G, uint64_t seed,
                                                uint32_t epoch, int rep_base) {
  using RC = Rec<NX>;
  const int r = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i < N) {
    Real n[NX];
    fill_normals<NX>(seed, i, (uint32_t)r, (uint32_t)(r + rep_base), epoch, STREAM_INIT, replay, N, n);
    const Real* L = Lc + (int64_t)r * NX * NX;
#pragma unroll
    for (int d = 0; d < NX; ++d) {
      Real acc = Real(0);
#pragma unroll
      for (int e = 0; e <= d; ++e) acc += n[e] * L[d * NX + e];
      x[((int64_t)r * NX + d) * Npad + i] = acc + mean[r * NX + d];
    }
  }
  const int64_t k = i;  // one record per tile
  if (k < G) {
    double* o = rec + ((int64_t)r * G + k) * RC::SIZE;
    for (int q = 0; q < RC::SIZE; ++q) o[q] = 0.0;
    o[RC::UNI] = 1.0;
  }
}

// ---------------------------------------------------------------------------
// Exact two-pass weighted moments of the current state (np.average / np.cov with
// aweights, bias=True; particle_filter.py:266-267) for any NX — the PFState.cov
// readout when NX is too large for the in-kernel one-pass covariance.
// w_i = exp(l_i - lse) (or 1/N when uniform); lse per replicate in `lse`.
// ---------------------------------------------------------------------------
template <typename Real>
__device__ __forceinline__ double mom_weight(const Real* lw, int64_t i, bool uni, double lse) {
  if (uni) return 1.0;
  const Real l = lw[i];
  return (l > -INFINITY) ? exp((double)l - lse) : 0.0;
}

template <typename Real, int NX>
__global__ void __launch_bounds__(BLOCK) k_mom_mean(const Real* x, const Real* lw, const double* rec, int RS, int G,
                                                    const double* lse, int64_t N, int64_t Npad, double* mean) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int d = blockIdx.x, r = blockIdx.y;
  const bool uni = rec[(int64_t)r * G * RS + 3] != 0.0;
  const Real* xr = x + ((int64_t)r * NX + d) * Npad;
  const Real* lr = lw + (int64_t)r * Npad;
  double sw = 0.0, sx = 0.0;
  for (int64_t i = threadIdx.x; i < N; i += BLOCK) {
    const double w = mom_weight<Real>(lr, i, uni, lse[r]);
    sw += w;
    sx += w * (double)xr[i];
  }
  sw = block_sum(sw, smem);
  sx = block_sum(sx, smem);
  if (threadIdx.x == 0) mean[(int64_t)r * NX + d] = sx / sw;
}

template <typename Real, int NX>
__global__ void __launch_bounds__(BLOCK) k_mom_cov(const Real* x, const Real* lw, const double* rec, int RS, int G,
                                                   const double* lse, int64_t N, int64_t Npad, const double* mean,
                                                   double* cov) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int d = blockIdx.x / NX, e = blockIdx.x % NX, r = blockIdx.y;
  if (e < d) return;
  const bool uni = rec[(int64_t)r * G * RS + 3] != 0.0;
  const Real* xd = x + ((int64_t)r * NX + d) * Npad;
  const Real* xe = x + ((int64_t)r * NX + e) * Npad;
  const Real* lr = lw + (int64_t)r * Npad;
  const double md = mean[(int64_t)r * NX + d], me = mean[(int64_t)r * NX + e];
  double sw = 0.0, sc = 0.0;
  for (int64_t i = threadIdx.x; i < N; i += BLOCK) {
    const double w = mom_weight<Real>(lr, i, uni, lse[r]);
    sw += w;
    sc += w * ((double)xd[i] - md) * ((double)xe[i] - me);
  }
  sw = block_sum(sw, smem);
  sc = block_sum(sc, smem);
  if (threadIdx.x == 0) {
    cov[(int64_t)r * NX * NX + d * NX + e] = sc / sw;
    cov[(int64_t)r * NX * NX + e * NX + d] = sc / sw;
  }
}

}  // namespace pf
