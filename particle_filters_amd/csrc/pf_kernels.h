// SIR particle-filter kernels for gfx950 (CDNA4, wave64).
//
// One launch of k_step = one pass over the particle set, fusing, in order:
//   (0) prologue   every workgroup reduces the previous update's per-tile
//                  partial records (field-major, L2-resident) to the global log
//                  normaliser, Neff, resample decision and — on resample steps —
//                  the per-tile weight prefix.  All workgroups run the identical
//                  fixed-order reduction (max first, then one exp per record, then
//                  plain sums), so they agree bit-for-bit and no inter-workgroup
//                  communication is needed inside a launch; workgroup 0 also
//                  writes that step's posterior outputs.
//   (1) gather     if the previous update decided to resample: each output slot
//                  finds its ancestor (systematic: walk only the input tiles its
//                  positions land in, scanning each tile's weights in LDS in fp64;
//                  multinomial: binary search of a materialised fp64 CDF), reads
//                  the ancestor and adds the regularisation jitter
//                  (particle_filter.py:188-220).
//   (2) predict    x <- g(x, u) + chol(Q) n   (particle_filter.py:223-237)
//   (3) update     l <- (l_prev - lse_prev) + loglik(z | x)  (particle_filter.py:239-263)
//                  and the tile's (max, sum e^(l-m), sum e^2(l-m), sum e^(l-m) x, ...)
//                  partial record for the next launch's prologue.
//
// Occupancy is the design driver: a tile is one 4-particle chunk per thread
// (16-byte vector loads/stores), several workgroups per CU, a rolled chunk loop
// and no per-thread arrays, so that several waves per SIMD hide the latency of
// the per-particle dependency chain (Philox -> Box-Muller -> g -> h -> weight).
//
// Layout in HBM (replicate-major, structure-of-arrays):
//   x   [R][NX][Npad]  Real     particles (ping-pong pair)
//   lw  [R][Npad]      Real     unnormalised log weights (ping-pong pair)
//   rec [R][F][G]      double   per-tile partial records, field-major (ping-pong pair)
//   cdf [R][N]         double   materialised CDF (multinomial only)
#pragma once
#include "pf_dpp.h"
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "philox.h"
#include "pf_models.h"

namespace pf {

constexpr int BLOCK = 256;
constexpr int NWAVES = BLOCK / 64;
#ifndef PF_MAXG
#define PF_MAXG 1024
#endif
constexpr int MAXG = PF_MAXG;      // tiles per replicate

// Diagnostic phase stamps (PF_STAMPS builds only; never in the product library):
// per workgroup, thread 0 records s_memrealtime (100 MHz) at phase boundaries.
#ifdef PF_STAMPS
constexpr int STAMP_SLOTS = 10;
constexpr int STAMP_WG = 65536;  // workgroups stamped: linear id y * gridDim.x + x (replicate-major)
__device__ unsigned long long g_pf_stamps[STAMP_WG * STAMP_SLOTS];
#define PF_STAMP(k)                                                                                     \
  do {                                                                                                  \
    const unsigned wid_ = blockIdx.y * gridDim.x + blockIdx.x;                                          \
    if (stamp_on && threadIdx.x == 0 && wid_ < (unsigned)STAMP_WG)                                      \
      g_pf_stamps[wid_ * STAMP_SLOTS + (k)] = __builtin_amdgcn_s_memrealtime();                         \
  } while (0)
#else
#define PF_STAMP(k) \
  do {              \
  } while (0)
#endif

// ---------------------------------------------------------------------------
// Partial record layout (doubles), field-major: rec[f * G + tile]
// ---------------------------------------------------------------------------
template <int NX>
struct Rec {
  static constexpr bool COV = NX <= 4;  // in-kernel weighted covariance for small state
  static constexpr int NC = COV ? NX * (NX + 1) / 2 : 0;
  static constexpr int M = 0;        // tile max of l (or -inf)
  static constexpr int S0 = 1;       // sum e^(l-m)
  static constexpr int S00 = 2;      // sum e^(2(l-m))
  static constexpr int UNI = 3;      // 1.0: weights are uniform (after init / resample)
  static constexpr int CNT = 4;      // aux: freshly resampled particles in tile (0: aux invalid)
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
// Wave / block collectives (fixed combination order -> deterministic; an xor
// butterfly gives every lane the bitwise-same result since + and max commute)
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

// The prologue's block reductions on the DPP network (uniform wave results, no LDS-crossbar
// shuffles; a fixed combination tree, identical in every workgroup and every kernel that
// reduces a replicate's records: k_step, k_step_grp, k_cdf, k_head, k_finalize, k_dyn_*).
template <int BS>
__device__ __forceinline__ double pblock_max(double v, double* red) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max_ud(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) s = fmax(s, red[i]);
  return s;
}
template <int K, int BS>
__device__ __forceinline__ void pblock_sum_k(double (&v)[K], double* red) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < K; ++i) v[i] = wave_sum_ud(v[i]);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < K; ++i) red[w * K + i] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K; ++i) {
    double s = red[i];
#pragma unroll
    for (int j = 1; j < NW; ++j) s += red[j * K + i];
    v[i] = s;
  }
}
template <int BS>
__device__ __forceinline__ double pblock_excl_scan(double v, double* red, double* total) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double incl = wave_incl_scan_dpp(v);
  __syncthreads();
  if (lane == 63) red[w] = incl;
  __syncthreads();
  double off = 0.0, tot = 0.0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    if (i < w) off += red[i];
    tot += red[i];
  }
  *total = tot;
  return off + incl - v;
}

// Block reductions (BS threads) over K values at once; `red` needs (BS/64)*K doubles.
template <int K, int BS = BLOCK>
__device__ __forceinline__ void block_sum_k(double (&v)[K], double* red) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < K; ++i) v[i] = wave_sum(v[i]);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < K; ++i) red[w * K + i] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K; ++i) {
    double s = red[i];
#pragma unroll
    for (int j = 1; j < NW; ++j) s += red[j * K + i];
    v[i] = s;
  }
}
template <int BS = BLOCK>
__device__ __forceinline__ double block_sum(double v, double* red) {
  double a[1] = {v};
  block_sum_k<1, BS>(a, red);
  return a[0];
}
template <int BS = BLOCK>
__device__ __forceinline__ double block_max(double v, double* red) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) s = fmax(s, red[i]);
  return s;
}
template <int BS = BLOCK>
__device__ __forceinline__ int block_min_i(int v, double* red) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_min_i(v);
  __syncthreads();
  if (lane == 0) ((int*)red)[w] = v;
  __syncthreads();
  int s = ((int*)red)[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) s = min(s, ((int*)red)[i]);
  return s;
}
// exclusive block scan; returns this thread's offset, *total = block total
template <int BS = BLOCK>
__device__ __forceinline__ double block_excl_scan(double v, double* red, double* total) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double incl = wave_incl_scan(v, lane);
  __syncthreads();
  if (lane == 63) red[w] = incl;
  __syncthreads();
  double off = 0.0, tot = 0.0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    if (i < w) off += red[i];
    tot += red[i];
  }
  *total = tot;
  return off + incl - v;
}

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
  int lq_local, lj_local; // chol(Q) / jitter factor block-diagonal in the lane blocks of k_step_grp
  int sys_cdf;            // systematic ancestors searched in the materialised CDF `cdf` (k_step_grp)
  // k_step_grp, systematic: the in-tile inclusive prefix sum_{j' <= j} e^(l_j' - m_k) of the weights
  // in rec_in, written by the launch that produced them (lcum_out, tile_cdf's summation order) and
  // read by the next gather (lcum_in) as cdf[j] = P_k + c_k lcum[j] — tile_cdf's values without the
  // k_cdf launch.  Null: not available (k_cdf materialises `cdf` instead).
  const double* lcum_in;
  double* lcum_out;
  // within-filter sharding (pf_shard.h): global index of local particle 0 (Philox counters) and
  // the global log normaliser of the previous weights (replaces the local one when use_lse_ext)
  int64_t pbase;
  double lse_ext;
  int use_lse_ext;
  // LINEAR h that selects components (every row of H one 1, e.g. L96's x[::4]): the large-state
  // kernel reads the observed component instead of the H row (h_sel != 0); hcol2k[c] = the
  // observation of component c or -1
  int h_sel;
  int32_t hcol2k[64];
  // many-replicate launches: the summary of rec_in computed once per replicate by k_head
  // ([R][HEAD_STRIDE] doubles); k_step / k_step_grp / k_cdf then read it instead of every
  // workgroup re-reducing all G records (O(R G^2) -> O(R G) record reads).  Null: in-kernel prologue.
  const double* head;
  // runtime-shape kernels (pf_dyn.h): the model's dimensions, the per-replicate scratch
  // [R][wrows][Npad] and whether A / chol(Q) / 0.001 chol(Q) are diagonal
  int dnx, dnz;
  void* wbuf;
  int64_t wrows;
  int a_diag, lq_diag, lj_diag;
  // device-loop covariance for nx > 4 (pf_cov.h): a gathering launch also writes its post-resample
  // (post-jitter) rows here, [R][NX][Npad]; null: not wanted
  void* xr_out;
  // ... or, without jitter (the post-resample row of slot i IS predicted row anc[i]), only the
  // ancestor index of every slot, [R][N] (4 bytes instead of 4 nx per slot); null: not wanted
  int32_t* anc_out;
};

struct Head {
  double M, S, S2, Sscan, lse, neff;
  int uniform, resample;
};

// ---------------------------------------------------------------------------
// Prologue: the summary of the previous launch's records.  Thread t owns the
// contiguous records [t*RPT, t*RPT + RPT).  Max first, then per-record factors,
// then plain sums: a short dependency chain with one parallel exp per record.
// ---------------------------------------------------------------------------
// The summary from the record heads already in registers (thread t: records [t RPT, t RPT + RPT),
// -inf / 0 past G) and the uniform flag: prologue() after its loads, and the persistent fp64 step
// (pf_persist.h), which reads the heads from its record granules - the same arithmetic, bit for bit.
template <int NX, int BS>
__device__ __forceinline__ Head prologue_reduce(const double (&mk)[MAXG / BS], const double (&s0k)[MAXG / BS],
                                                const double (&s00k)[MAXG / BS], double uni, int G, int64_t N,
                                                double thresh, bool allow, bool force, bool want_prefix, double* red,
                                                double* Pl) {
  constexpr int RPT = MAXG / BS;  // records per thread
  const int t = threadIdx.x;
  const int k0 = t * RPT;
  Head h;
  h.uniform = uni != 0.0;  // a launch-wide property
  h.resample = 0;
  if (h.uniform) {
    h.M = 0.0; h.S = h.S2 = h.Sscan = 1.0; h.lse = 0.0; h.neff = (double)N;
    return h;
  }
  double lmax = -INFINITY;
#pragma unroll
  for (int j = 0; j < RPT; ++j)
    if (s0k[j] > 0.0) lmax = fmax(lmax, mk[j]);
  const double M = pblock_max<BS>(lmax, red);
  double s[2] = {0.0, 0.0};
  double wk[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const double f = (s0k[j] > 0.0) ? exp(mk[j] - M) : 0.0;
    wk[j] = s0k[j] * f;
    s[0] += wk[j];
    s[1] += s00k[j] * f * f;
  }
  const double tsum = s[0];
  pblock_sum_k<2, BS>(s, red);
  h.M = M;
  h.S = s[0];
  h.S2 = s[1];
  h.Sscan = h.S;
  h.lse = M + log(h.S);
  h.neff = (h.S * h.S) / h.S2;
  h.resample = allow && (force || h.neff < thresh * (double)N);
  if (want_prefix && h.resample) {  // normalised exclusive prefix of the tile weights
    double S;
    double run = pblock_excl_scan<BS>(tsum, red, &S);
    h.Sscan = S;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int k = k0 + j;
      if (k < G) Pl[k] = run / S;
      run += wk[j];
    }
    if (t == 0) Pl[G] = 1.0;
    __syncthreads();
  }
  return h;
}

template <int NX, int BS>
__device__ __forceinline__ Head prologue(const double* rec, int G, int64_t N, double thresh, bool allow, bool force,
                                         bool want_prefix, double* red, double* Pl) {
  using RC = Rec<NX>;
  constexpr int RPT = MAXG / BS;  // records per thread
  const int k0 = threadIdx.x * RPT;
  // one round of loads: the uniform flag and this thread's record heads
  double mk[RPT], s0k[RPT], s00k[RPT];
  const double uni = rec[RC::UNI * G];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int k = k0 + j;
    const bool in = k < G;
    mk[j] = in ? rec[RC::M * G + k] : -INFINITY;
    s0k[j] = in ? rec[RC::S0 * G + k] : 0.0;
    s00k[j] = in ? rec[RC::S00 * G + k] : 0.0;
  }
  return prologue_reduce<NX, BS>(mk, s0k, s00k, uni, G, N, thresh, allow, force, want_prefix, red, Pl);
}

// Head of a replicate as k_head stored it (same fields prologue() returns; the
// prefix Pl[0..G] staged into LDS when this kernel searches it).  want_prefix must
// be what the caller's own prologue call would have passed.
constexpr int HEAD_F = 8;  // M, S, S2, Sscan (with prefix), lse, neff, uniform, resample
constexpr int HEAD_STRIDE = HEAD_F + MAXG + 8;
template <int BS>
__device__ __forceinline__ Head load_head(const double* head, int r, int G, bool want_prefix, double* Pl) {
  const double* o = head + (int64_t)r * HEAD_STRIDE;
  Head h;
  h.M = o[0];
  h.S = o[1];
  h.S2 = o[2];
  h.lse = o[4];
  h.neff = o[5];
  h.uniform = o[6] != 0.0;
  h.resample = o[7] != 0.0;
  const bool pre = want_prefix && h.resample;
  h.Sscan = pre ? o[3] : h.S;
  if (pre) {
    for (int k = threadIdx.x; k <= G; k += BS) Pl[k] = o[HEAD_F + k];
    __syncthreads();
  }
  return h;
}

// Outputs of the update / resample summarised by `rec`: weighted mean/cov, Neff,
// log normaliser, decision (out_step) and the uniform-weight mean/cov of freshly
// resampled particles (out_post_step).  Field f of the output vector is reduced
// by workgroup f mod nblk (spreads the work when NX is large).
// rec(f, k): field f of tile k's record (plain memory, or the persistent step's granules)
template <int NX, int BS, class RecF>
__device__ void write_outputs_f(const StepParams& p, int64_t out_step, int64_t out_post_step, RecF&& rec_at,
                                const Head& h, int r, int R, int blk, int nblk, double* red) {
  using RC = Rec<NX>;
  const int t = threadIdx.x;
  const int G = p.G;
  const bool pre = out_step >= 0 && !h.uniform;
  const bool want_post = out_post_step >= 0;
  if (!pre && !want_post) return;
  if (pre && blk == 0 && t == 0) {
    const int64_t o = out_step * R + r;
    p.o_neff[o] = h.neff;
    p.o_lse[o] = h.lse;
    p.o_flag[o] = h.resample;
  }
  constexpr int NF = NX + RC::NC;  // means + (small NX) second moments
  if constexpr (RC::COV) {
    if (blk != 0) return;
    double v[2 * NF + 1];
#pragma unroll
    for (int f = 0; f < 2 * NF + 1; ++f) v[f] = 0.0;
    for (int k = t; k < G; k += BS) {
      if (pre) {
        const double s0 = rec_at(RC::S0, k);
        if (s0 > 0.0) {
          const double fk = exp(rec_at(RC::M, k) - h.M);
#pragma unroll
          for (int f = 0; f < NF; ++f) v[f] += rec_at(RC::S1 + f, k) * fk;
        }
      }
      if (want_post) {
        v[2 * NF] += rec_at(RC::CNT, k);
#pragma unroll
        for (int f = 0; f < NF; ++f) v[NF + f] += rec_at(RC::A1 + f, k);
      }
    }
    block_sum_k<2 * NF + 1, BS>(v, red);
    if (t != 0) return;
    const double cnt = v[2 * NF];
    for (int pass = 0; pass < 2; ++pass) {
      if (pass == 0 ? !pre : !(want_post && cnt > 0.0)) continue;
      const int64_t o = (pass == 0 ? out_step : out_post_step) * R + r;
      const double* m = v + pass * NF;
      const double den = pass == 0 ? h.S : cnt;
      for (int d = 0; d < NX; ++d) p.o_mean[o * NX + d] = m[d] / den;
      if (p.o_cov) {
        int c = 0;
        for (int d = 0; d < NX; ++d)
          for (int e = d; e < NX; ++e, ++c) {
            const double val = m[NX + c] / den - (m[d] / den) * (m[e] / den);
            p.o_cov[o * NX * NX + d * NX + e] = val;
            p.o_cov[o * NX * NX + e * NX + d] = val;
          }
      }
    }
  } else {
    if (blk >= 2 * NX) return;  // no field of this workgroup (field f is reduced by workgroup f mod nblk)
    double cnt = 0.0;
    if (want_post) {
      for (int k = t; k < G; k += BS) cnt += rec_at(RC::CNT, k);
      cnt = block_sum<BS>(cnt, red);
    }
    const bool post = want_post && cnt > 0.0;
    for (int f = blk; f < 2 * NX; f += nblk) {
      const bool is_post = f >= NX;
      if (is_post ? !post : !pre) continue;
      const int d = is_post ? f - NX : f;
      double acc = 0.0;
      for (int k = t; k < G; k += BS) {
        if (is_post) {
          acc += rec_at(RC::A1 + d, k);
        } else {
          const double s0 = rec_at(RC::S0, k);
          if (s0 > 0.0) acc += rec_at(RC::S1 + d, k) * exp(rec_at(RC::M, k) - h.M);
        }
      }
      acc = block_sum<BS>(acc, red);
      if (t == 0) {
        const int64_t o = (is_post ? out_post_step : out_step) * R + r;
        p.o_mean[o * NX + d] = acc / (is_post ? cnt : h.S);
      }
    }
  }
}

template <int NX, int BS>
__device__ void write_outputs(const StepParams& p, const double* rec, const Head& h, int r, int R, int blk, int nblk,
                              double* red) {
  const int G = p.G;
  write_outputs_f<NX, BS>(p, p.out_step, p.out_post_step, [rec, G](int f, int k) { return rec[f * G + k]; }, h, r, R, blk,
                          nblk, red);
}

// Global CDF values of input tile k, in LDS:
//   cdf[j] = P_k + (e^(m_k - M) / S) * sum_{j' <= j} e^(l_j' - m_k)
// (the same per-element weights the update's records summed).
template <typename Real, int NX, int BS>
__device__ __forceinline__ int tile_cdf(const Real* __restrict__ lw, const double* rec, int G, int64_t N, int tile,
                                        int k, const Head& h, const double* Pl, double* cdf, double* red) {
  const int64_t s = (int64_t)k * tile;
  const int len = (int)min((int64_t)tile, N - s);
  const int per = (len + BS - 1) / BS;
  const int j0 = threadIdx.x * per;
  const double mk = rec[Rec<NX>::M * G + k];
  const Real m = (Real)mk;
  double acc = 0.0;
  for (int j = j0; j < j0 + per && j < len; ++j) {
    const Real l = lw[s + j];
    acc += (l > -INFINITY) ? (double)exp_r<Real>(l - m) : 0.0;
  }
  double tot;
  double off = block_excl_scan<BS>(acc, red, &tot);
  const double c = (mk > -INFINITY) ? exp(mk - h.M) / h.Sscan : 0.0;
  const double base = Pl[k];
  for (int j = j0; j < j0 + per && j < len; ++j) {
    const Real l = lw[s + j];
    off += (l > -INFINITY) ? (double)exp_r<Real>(l - m) : 0.0;
    cdf[j] = base + c * off;
  }
  __syncthreads();
  return len;
}

// tile_cdf from log-weights the caller already holds in registers (thread t: elements
// [t per, t per + per) of tile k, loaded one source tile ahead by load_tile_lw): the same
// partition, exponentials and summation order, so exactly tile_cdf's doubles
template <typename Real, int PM>
__device__ __forceinline__ void load_tile_lw(const Real* __restrict__ lw, int64_t N, int tile, int k, int BS,
                                             Real (&lv)[PM]) {
  const int64_t s = (int64_t)k * tile;
  const int len = (int)min((int64_t)tile, N - s);
  const int per = (len + BS - 1) / BS;
  const int j0 = threadIdx.x * per;
#pragma unroll
  for (int q = 0; q < PM; ++q)
    if (q < per && j0 + q < len) lv[q] = lw[s + j0 + q];
}
template <typename Real, int NX, int BS, int PM>
__device__ __forceinline__ int tile_cdf_regs(const Real (&lv)[PM], const double* rec, int G, int64_t N, int tile, int k,
                                             const Head& h, const double* Pl, double* cdf, double* red) {
  const int64_t s = (int64_t)k * tile;
  const int len = (int)min((int64_t)tile, N - s);
  const int per = (len + BS - 1) / BS;
  const int j0 = threadIdx.x * per;
  const double mk = rec[Rec<NX>::M * G + k];
  const Real m = (Real)mk;
  double acc = 0.0;
#pragma unroll
  for (int q = 0; q < PM; ++q)
    if (q < per && j0 + q < len) acc += (lv[q] > -INFINITY) ? (double)exp_r<Real>(lv[q] - m) : 0.0;
  double tot;
  double off = block_excl_scan<BS>(acc, red, &tot);
  const double c = (mk > -INFINITY) ? exp(mk - h.M) / h.Sscan : 0.0;
  const double base = Pl[k];
#pragma unroll
  for (int q = 0; q < PM; ++q)
    if (q < per && j0 + q < len) {
      off += (lv[q] > -INFINITY) ? (double)exp_r<Real>(lv[q] - m) : 0.0;
      cdf[j0 + q] = base + c * off;
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
// first k with pos < P[k+1] (the tile whose CDF range holds pos); G-1 if none
__device__ __forceinline__ int prefix_tile(const double* Pl, int G, double pos) {
  int lo = 0, hi = G;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (pos < Pl[mid + 1]) hi = mid; else lo = mid + 1;
  }
  return lo < G ? lo : G - 1;
}

// Number of systematic positions below x: #{ i in [0, N) : (U + i) / N < x } (pf.py:146-171 compares
// pos = (U + arange(N)) / N < cdf[j] in fp64).  Exactly, (U + i) / N < x <=> i < y = x N - U; the fp64
// division can disagree only when y is within ~1e-10 of an integer, and only then are the candidate
// positions evaluated the reference's way.  32-bit slot indices (k_step: N < 2^31).
__device__ __forceinline__ int sys_count_exact(double x, double U, int N, int c) {
  const double Nd = (double)N;
  while (c > 0 && (U + (double)(c - 1)) / Nd >= x) --c;
  while (c < N && (U + (double)c) / Nd < x) ++c;
  return c;
}
__device__ __forceinline__ int sys_count_below(double x, double U, int N) {
  const double y = fma(x, (double)N, -U);
  const double fl = floor(y), d = y - fl;
  const int c = (int)fmin(fmax(fl + 1.0, 0.0), (double)N);
  if (d > 1e-7 && d < 1.0 - 1e-7) return c;
  return sys_count_exact(x, U, N, c);
}

template <typename Real>
__device__ __forceinline__ Real rmax(Real a, Real b) {
  if constexpr (sizeof(Real) == 4) return fmaxf(a, b);
  else return fmax(a, b);
}

// block maximum of floats (every thread gets it); redf >= BS / 64 floats, free on entry
template <int BS>
__device__ __forceinline__ float block_max_f(float v, float* redf) {
  constexpr int NW = BS / 64;
  const float wm = wave_max_u(v);
  if ((threadIdx.x & 63) == 0) redf[threadIdx.x >> 6] = wm;
  __syncthreads();
  float M = redf[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) M = fmaxf(M, redf[i]);
  return M;
}

// block maximum in the engine precision (fp32: block_max_f on the staging floats; fp64: block_max)
template <int BS, typename Real>
__device__ __forceinline__ Real block_max_r(Real v, double* stage) {
  if constexpr (sizeof(Real) == 4) return block_max_f<BS>(v, (float*)stage);
  else return block_max<BS>(v, stage);
}

// exclusive block max-scan of ints (-1 below thread 0); redi >= BS / 64 ints
template <int BS>
__device__ __forceinline__ int block_excl_max_i(int v, int* redi) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o);
    if (lane >= o) incl = max(incl, u);
  }
  int ex = __shfl_up(incl, 1);
  if (lane == 0) ex = -1;
  __syncthreads();
  if (lane == 63) redi[w] = incl;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NW; ++i)
    if (i < w) ex = max(ex, redi[i]);
  return ex;
}

// Systematic ancestors of slots [o0, o1) of a replicate (pf.py:146-171: the ancestor of slot i is the
// first j with (U + i) / N < cdf[j], the last particle if none), source-driven and search-free.  The
// source tiles k whose prefix ranges [Pl[k], Pl[k+1]) hold some of the slots (the tile of a position
// as prefix_tile finds it) each build their fp64 CDF segment cdf[j] = Pl[k] + c_k sum_{j' <= j}
// e^(l_j' - m_k), c_k = e^(m_k - M) / S (thread t: elements [t per, t per + per), a DPP block scan of
// the thread sums), and particle j's offspring start at slot L_j = C(cdf[j - 1]) (cdf[-1] = Pl[k];
// C = sys_count_below): the owner of slot i is the last particle with L_j <= i.  Each particle marks
// its first slot in anc_l with an LDS max (particles starting before this workgroup's slots mark the
// first slot, one max per thread), and an inclusive max-scan over the slots fills the runs (ancestor
// indices increase with the slot).  The tile's slot range is [C(Pl[k]), C(Pl[k+1])): L_0 = C(Pl[k])
// by construction, so consecutive tiles meet exactly.
template <typename Real, int NX, int BS, int PM>
__device__ __forceinline__ void sys_ancestors(const Real* __restrict__ lw_in, const double* rec_in, int G, int64_t N,
                                              int tile, int64_t o0, int64_t o1, double U, const Head& h,
                                              const double* Pl, int* anc_l, double* red, bool stamp_on) {
  (void)stamp_on;
  const int t = threadIdx.x;
  const int N32 = (int)N, w0 = (int)o0, w1 = (int)o1, nsl = w1 - w0;
  for (int s = t; s < nsl; s += BS) anc_l[s] = -1;  // ordered before the marks by the scans' barriers
  const double Nd = (double)N;
  const int klo = prefix_tile(Pl, G, (U + (double)w0) / Nd);
  const int khi = prefix_tile(Pl, G, (U + (double)(w1 - 1)) / Nd);
  PF_STAMP(6);
  int ntiles = 0;
  // log-weights of <= PM per thread in registers (loaded once per tile, read by both passes)
  const bool regs = PM > 1 && (tile + BS - 1) / BS <= PM;
  int A0 = klo == 0 ? 0 : sys_count_below(Pl[klo], U, N32);
  for (int k = klo; k <= khi; ++k) {
    const int A1 = k == G - 1 ? N32 : sys_count_below(Pl[k + 1], U, N32);
    const int lo_w = max(A0, w0), hi_w = min(A1, w1);
    if (lo_w < hi_w) {  // uniform
      const int64_t s0 = (int64_t)k * tile;
      const int len = (int)min((int64_t)tile, N - s0);
      const int per = (len + BS - 1) / BS, j0 = t * per;
      const double mk = rec_in[Rec<NX>::M * G + k];
      const Real m = (Real)mk;
      Real lv[PM];
      double part = 0.0;
      if (regs) {
        load_tile_lw<Real, PM>(lw_in, N, tile, k, BS, lv);
#pragma unroll
        for (int q = 0; q < PM; ++q)
          if (q < per && j0 + q < len) part += (lv[q] > -INFINITY) ? (double)exp_r<Real>(lv[q] - m) : 0.0;
      } else {
        for (int q = 0; q < per && j0 + q < len; ++q) {
          const Real l = lw_in[s0 + j0 + q];
          part += (l > -INFINITY) ? (double)exp_r<Real>(l - m) : 0.0;
        }
      }
      double tot;
      double run = pblock_excl_scan<BS>(part, red, &tot);
      if (ntiles++ == 0) PF_STAMP(7);
      const double c = (mk > -INFINITY) ? exp(mk - h.M) / h.Sscan : 0.0;
      const double base = Pl[k];
      int before = -1;  // the last of this thread's particles that starts before slot lo_w
      if (regs) {
#pragma unroll
        for (int q = 0; q < PM; ++q) {
          if (q < per && j0 + q < len) {
            const int L = sys_count_below(base + c * run, U, N32);
            const int j = (int)s0 + j0 + q;
            if (L < lo_w) before = j;
            else if (L < hi_w) atomicMax(&anc_l[L - w0], j);
            run += (lv[q] > -INFINITY) ? (double)exp_r<Real>(lv[q] - m) : 0.0;
          }
        }
      } else {
        for (int q = 0; q < per && j0 + q < len; ++q) {
          const Real l = lw_in[s0 + j0 + q];
          const int L = sys_count_below(base + c * run, U, N32);
          const int j = (int)s0 + j0 + q;
          if (L < lo_w) before = j;
          else if (L < hi_w) atomicMax(&anc_l[L - w0], j);
          run += (l > -INFINITY) ? (double)exp_r<Real>(l - m) : 0.0;
        }
      }
      if (before >= 0) atomicMax(&anc_l[lo_w - w0], before);
    }
    A0 = A1;
  }
  PF_STAMP(8);
#ifdef PF_STAMPS
  if (stamp_on && t == 0 && blockIdx.y * gridDim.x + blockIdx.x < (unsigned)STAMP_WG)
    g_pf_stamps[(blockIdx.y * gridDim.x + blockIdx.x) * STAMP_SLOTS + 9] = (unsigned long long)ntiles;
#endif
  __syncthreads();
  // fill: thread t owns slots [t pp, t pp + pp)
  const int pp = (nsl + BS - 1) / BS, s0 = t * pp, s1 = min(s0 + pp, nsl);
  int mx = -1;
  for (int s = s0; s < s1; ++s) mx = max(mx, anc_l[s]);
  mx = block_excl_max_i<BS>(mx, (int*)red);
  for (int s = s0; s < s1; ++s) {
    mx = max(mx, anc_l[s]);
    anc_l[s] = mx;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Normals
// ---------------------------------------------------------------------------
// NX normals of particle i (flat indices i*NX .. i*NX+NX-1) from Philox, or replay
template <int NX, typename Real>
__device__ __forceinline__ void fill_normals(uint64_t seed, int64_t i, uint32_t lrep, uint32_t rep, uint32_t ep,
                                             uint32_t stream, const double* replay, int64_t N, Real* n,
                                             int64_t pbase = 0) {
  if (replay) {
#pragma unroll
    for (int d = 0; d < NX; ++d) n[d] = (Real)replay[((int64_t)lrep * N + i) * NX + d];
    return;
  }
  const int64_t f0 = (i + pbase) * NX, f1 = f0 + NX - 1;  // pbase: global index of local particle 0 (shards)
  constexpr int GMAX = (NX % 4 == 0) ? NX / 4 : NX / 4 + 2;
#pragma unroll
  for (int gg = 0; gg < GMAX; ++gg) {
    const int64_t g = (f0 >> 2) + gg;
    if (g > (f1 >> 2)) break;
    const Normal4<Real> q = normal4<Real>(seed, (uint32_t)g, rep, ep, stream);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t f = 4 * g + e;
      if (f >= f0 && f <= f1) n[f - f0] = q.v[e];
    }
  }
}
// normals of scalar particles i0..i0+3 (flat indices i0..i0+3 = one Philox group)
template <typename Real>
__device__ __forceinline__ void chunk_normals4(uint64_t seed, int64_t i0, uint32_t lrep, uint32_t rep, uint32_t ep,
                                               uint32_t stream, const double* replay, int64_t N, Real* n,
                                               int64_t pbase = 0) {
  if (replay) {
#pragma unroll
    for (int e = 0; e < 4; ++e) n[e] = (i0 + e < N) ? (Real)replay[(int64_t)lrep * N + i0 + e] : Real(0);
    return;
  }
  const Normal4<Real> q = normal4<Real>(seed, (uint32_t)((i0 + pbase) >> 2), rep, ep, stream);  // pbase % 4 == 0
#pragma unroll
  for (int e = 0; e < 4; ++e) n[e] = q.v[e];
}

// 16-byte (fp32) / 2x16-byte (fp64) vector moves of 4 consecutive slots
template <typename Real>
__device__ __forceinline__ void load4(const Real* src, Real* v) {
  if constexpr (sizeof(Real) == 4) {
    const float4 a = *(const float4*)src;
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  } else {
    const double2 a = *(const double2*)src;
    const double2 b = *(const double2*)(src + 2);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
}
template <typename Real>
__device__ __forceinline__ void store4(Real* dst, const Real* v) {
  if constexpr (sizeof(Real) == 4) {
    *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    *(double2*)dst = make_double2(v[0], v[1]);
    *(double2*)(dst + 2) = make_double2(v[2], v[3]);
  }
}

// ---------------------------------------------------------------------------
// Per-thread weighted accumulator: running max + scaled sums (online, per thread
// only a few particles), merged max-first across lanes and waves.
// ---------------------------------------------------------------------------
template <typename Real, int NX>
struct WAcc {
  using RC = Rec<NX>;
  static constexpr int NS = 2 + NX + RC::NC;  // s0, s00, s1[NX], s2[NC]
  // a thread sums only a few particles: accumulate in the engine precision,
  // combine across lanes and waves in fp64
  Real m;
  Real s[NS];

  __device__ __forceinline__ void init() {
    m = -INFINITY;
#pragma unroll
    for (int i = 0; i < NS; ++i) s[i] = Real(0);
  }
  __device__ __forceinline__ void add(Real l, const Real* x) {
    if (!(l > -INFINITY)) return;  // zero weight (l = -inf); NaN also skipped
    if (l > m) {
      if (m > -INFINITY) {
        const Real f = exp_r<Real>(m - l);
        s[0] *= f;
        s[1] *= f * f;
#pragma unroll
        for (int i = 2; i < NS; ++i) s[i] *= f;
      }
      m = l;
    }
    const Real e = exp_r<Real>(l - m);
    s[0] += e;
    s[1] += e * e;
#pragma unroll
    for (int d = 0; d < NX; ++d) s[2 + d] += e * x[d];
    if constexpr (RC::COV) {
      int c = 2 + NX;
#pragma unroll
      for (int d = 0; d < NX; ++d)
#pragma unroll
        for (int f = d; f < NX; ++f) s[c++] += e * x[d] * x[f];
    }
  }
  // The thread's particles (fp32 scalar state, 8 particles: chunk t, then chunk t + BS) relative to
  // the workgroup's maximum M (block_max_f): every thread's sums share one reference, so the record
  // merge is a plain sum (block_sum_lds) - no rescale factors, nothing rounded in fp32 beyond the
  // per-particle exponentials.  Slots past the tile carry l = -inf, x = 0.
  __device__ __forceinline__ void add_ref8(const Real (&l)[8], const Real (&x)[8], Real M) {
    static_assert(NX == 1, "scalar state");
    m = M;
    if (!(M > -INFINITY)) return;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const Real we = (l[e] > -INFINITY) ? exp_r<Real>(l[e] - M) : Real(0);
      s[0] += we;
      s[1] += we * we;
      s[2] += we * x[e];
      s[3] += we * x[e] * x[e];
    }
  }
  // Block merge (max first): result (m, s...) in out[0..NS] of thread 0 only.
  // red >= (BS/64)*(NS+1) doubles.
  template <int BS>
  __device__ __forceinline__ void block_merge(double* red, double* out) {
    constexpr int NW = BS / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // wave partials on the DPP network (row reductions + row broadcasts, lane 63 read back as a
    // uniform value): no LDS-crossbar shuffles on the record's critical path
    const double md = (double)m;
    // fp32 engine: the maxima are floats, so the fp32 DPP max is the same value in fewer issues
    const double Mw = sizeof(Real) == 4 ? (double)wave_max_u((float)m) : wave_max_ud(md);
    const double f = (md > -INFINITY) ? exp(md - Mw) : 0.0;
    double v[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) v[i] = wave_sum_ud((double)s[i] * (i == 1 ? f * f : f));
    __syncthreads();
    if (lane == 0) {
      red[w * (NS + 1)] = Mw;
#pragma unroll
      for (int i = 0; i < NS; ++i) red[w * (NS + 1) + 1 + i] = v[i];
    }
    __syncthreads();
    if (w != 0) return;
    // wave 0: lane j < NW holds wave j's partial; one exp per lane, then DPP sums
    const double mj = lane < NW ? red[lane * (NS + 1)] : -INFINITY;
    const double M = sizeof(Real) == 4 ? (double)wave_max_u((float)mj) : wave_max_ud(mj);
    const double fj = (mj > -INFINITY) ? exp(mj - M) : 0.0;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const double vi = lane < NW ? red[lane * (NS + 1) + 1 + i] * (i == 1 ? fj * fj : fj) : 0.0;
      out[1 + i] = wave_sum_ud(vi);
    }
    out[0] = M;
  }
  // The same merge with one wave instead of all: every thread stages (m, s...) in LDS (stage:
  // [NS + 1][BS] floats), then wave 0 alone rescales and sums them - lane l takes threads l, l + 64,
  // ... with fp64 factors e^(m_t - M) relative to the wave's (= the workgroup's) maximum M and fp64
  // sums, then one DPP sum per field.  The other waves do no reduction arithmetic at all.  The
  // factors are fp64 exponentials (as in block_merge): with fp32 ones (~1e-7 relative) the tile
  // records - the resampling CDF's tile masses - would carry fp32 rounding and a filter's ancestors
  // would depend on how its particles are cut into tiles and shards.  The fp32 scalar step's default
  // (PF_MERGE_LDS): sv64 306 -> 279 us/step in a same-box A/B (profiles/r04/ab).
  template <int BS>
  __device__ __forceinline__ void block_merge_lds(float* stage, double* out) {
    static_assert(sizeof(Real) == 4, "fp32 engine");
    constexpr int K = BS / 64;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    stage[t] = m;
#pragma unroll
    for (int i = 0; i < NS; ++i) stage[(1 + i) * BS + t] = s[i];
    __syncthreads();
    if (w != 0) return;
    float mk[K];
    float Ml = -INFINITY;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      mk[k] = stage[k * 64 + lane];
      Ml = fmaxf(Ml, mk[k]);
    }
    const float Mw = wave_max_u(Ml);
    double acc[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) acc[i] = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double f = (mk[k] > -INFINITY) ? exp((double)mk[k] - (double)Mw) : 0.0;
#pragma unroll
      for (int i = 0; i < NS; ++i) acc[i] = fma((double)stage[(1 + i) * BS + k * 64 + lane], i == 1 ? f * f : f, acc[i]);
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) out[1 + i] = wave_sum_ud(acc[i]);
    out[0] = Mw;
  }
  // Merge of add_ref8 sums in fp64 (fp64 engine: every thread's sums share the workgroup maximum, so the
  // record is their plain block sum; out[0..NS] in every thread)
  template <int BS>
  __device__ __forceinline__ void block_sum_ref(double* red, double* out) {
    double v[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) v[i] = (double)s[i];
    block_sum_k<NS, BS>(v, red);
#pragma unroll
    for (int i = 0; i < NS; ++i) out[1 + i] = v[i];
    out[0] = m;
  }
  // Merge of add_ref8 sums (one reference M for the whole workgroup): the partials staged in LDS,
  // wave 0 sums them in fp64 (lane l: threads l, l + 64, ...), then one DPP sum per field.
  template <int BS>
  __device__ __forceinline__ void block_sum_lds(float* stage, double* out) {
    static_assert(sizeof(Real) == 4, "fp32 engine");
    constexpr int K = BS / 64;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
    for (int i = 0; i < NS; ++i) stage[i * BS + t] = s[i];
    __syncthreads();
    if (w != 0) return;
    double acc[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      acc[i] = 0.0;
#pragma unroll
      for (int k = 0; k < K; ++k) acc[i] += (double)stage[i * BS + k * 64 + lane];
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) out[1 + i] = wave_sum_ud(acc[i]);
    out[0] = m;
  }
};

// ---------------------------------------------------------------------------
// The fused step kernel
// ---------------------------------------------------------------------------
// Work split: workgroup (b, r) owns particle slots [b*tile, (b+1)*tile) of
// replicate r.  A thread owns "chunks" of CH consecutive slots (CH = 4 for the
// scalar state so x / lw move as 16-byte vectors): chunk c = t, t+BLOCK, ...
#ifndef PF_SMALL_BS
#define PF_SMALL_BS 256
#endif
template <int NX>
constexpr int step_bs = (NX == 1) ? PF_SMALL_BS : 256;

template <typename Real, int NX, int NZ, int TK, int OK>
struct StepTraits {
  static constexpr int CH = (NX == 1) ? 4 : 1;
  // Workgroup size: PF_SMALL_BS for the small-state models (bigger workgroups ->
  // fewer tiles -> less O(tiles^2) prologue redundancy, but a lower VGPR cap);
  // register-heavy large-state models (L96, MAT) keep 256.
  static constexpr int BS = step_bs<NX>;
  static constexpr int TILE_MAX = BS * CH * 16;  // at most 16 chunks per thread
};

// LDS carve (doubles): [0, LDS_RED) scratch | Pl[G+1] | tile area (cdf doubles + anc ints, or
// the staged epilogue record, and for the fp32 scalar state the record merge's staging after it)
#ifndef PF_MERGE_LDS
#define PF_MERGE_LDS 1
#endif
constexpr int MERGE_LDS_BYTES = 32 * 8 + 5 * 256 * 4;  // record slots + [NS + 1][BS] floats (NX = 1, BS = 256)
constexpr int LDS_RED = 512;
constexpr int LDS_PL = LDS_RED;
__host__ __device__ constexpr int lds_tile(int G) { return LDS_PL + ((G + 8) & ~7); }

// waves per SIMD the fp32 scalar-state step is compiled for (its VGPR cap; LDS allows 5 workgroups
// per CU with the gather area of a 2048-particle tile)
#ifndef PF_STEP_WPE
#define PF_STEP_WPE 4
#endif
// fp64 scalar state: >= 2 waves per SIMD (its 170 VGPRs; capped at 168 for 3 waves it spills 144 B per
// lane and runs 23.5 instead of 21.0 us/step, profiles/r06/fp64): 512 workgroups resident, config 2's
// 489 tiles of 2048 particles in one round
#ifndef PF_STEP_WPE_D
#define PF_STEP_WPE_D 2
#endif
template <typename Real, int NX>
constexpr int step_wpe = NX == 1 ? (sizeof(Real) == 4 ? PF_STEP_WPE : PF_STEP_WPE_D) : 1;
template <typename Real, int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(step_bs<NX>) __attribute__((amdgpu_waves_per_eu(step_wpe<Real, NX>)))
k_step(StepParams p) {
  using M = Model<Real, NX, NZ, TK, OK>;
  using RC = Rec<NX>;
  using WA = WAcc<Real, NX>;
  constexpr int CH = StepTraits<Real, NX, NZ, TK, OK>::CH;
  constexpr int BS = StepTraits<Real, NX, NZ, TK, OK>::BS;
  static_assert((BS / 64) * (WA::NS + 1) <= LDS_RED, "scratch too small");
  static_assert((BS / 64) * (2 * (NX + Rec<NX>::NC) + 1) <= LDS_RED, "scratch too small");
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  double* Pl = smem + LDS_PL;
  double* cdf = smem + lds_tile(p.G);
  int* anc_l = (int*)(cdf + p.tile);

  const int b = blockIdx.x, r = blockIdx.y, R = gridDim.y;
  const int t = threadIdx.x;
  const Real* __restrict__ P = (const Real*)p.P;
  const Real* x_in = (const Real*)p.x_in + (int64_t)r * NX * p.Npad;
  Real* x_out = (Real*)p.x_out + (int64_t)r * NX * p.Npad;
  const Real* lw_in = (const Real*)p.lw_in + (int64_t)r * p.Npad;
  Real* lw_out = (Real*)p.lw_out + (int64_t)r * p.Npad;
  const double* rec_in = p.rec_in + (int64_t)r * RC::SIZE * p.G;
  const int64_t o0 = (int64_t)b * p.tile;
  const int64_t o1 = min(o0 + (int64_t)p.tile, p.N);
  const int nchunks = (int)((o1 - o0 + CH - 1) / CH);
  const uint32_t rep = (uint32_t)(r + p.rep_base);
  const bool stamp_on = p.do_predict && p.do_update;  // stamps: fused steps only
  (void)stamp_on;
  PF_STAMP(0);

  // ---- (S) speculative first chunk --------------------------------------------
  // Loads, normals, g and h of this thread's first chunk on the no-resample path do
  // not depend on the prologue: computing them first overlaps the prologue's record
  // loads.  On a resample step the chunk is redone from the gathered ancestors with
  // the same (counter-based) normals.
  constexpr bool PRE = NX <= 4;
  constexpr int SC = PRE ? CH : 1;
  Real sx[SC][NX], sl[SC], sll[SC], sn[SC][NX];
  Real px[4], pl[4];  // scalar state: the thread's second chunk, loaded with the first
  bool pre1 = false;
  // fp32 scalar state (the sv64 roofline run): the second chunk is speculated too (qx, qll), and a
  // launch that does not gather finishes both chunks straight from registers (straight-line code,
  // no per-chunk reloads, bounds tests or pointer bookkeeping) instead of the generic chunk loop
#ifndef PF_STEP_FAST
#define PF_STEP_FAST 1
#endif
  constexpr bool FAST2 = PF_STEP_FAST && NX == 1 && CH == 4 && sizeof(Real) == 4;
  // fp64 scalar state (the reference's precision, BASELINE config 2's fp64 line): the same straight-
  // line finish - both chunks speculated under the prologue, one exponential per slot against the
  // workgroup maximum (add_ref8) instead of the online max (up to two per slot, lane-divergent), the
  // record's sums merged as plain fp64 sums
#ifndef PF_STEP_FAST_D
#define PF_STEP_FAST_D 1
#endif
  constexpr bool FASTD = PF_STEP_FAST_D && NX == 1 && CH == 4 && sizeof(Real) == 8;
  constexpr bool FASTX = FAST2 || FASTD;
  constexpr int QC = FASTX ? 4 : 1;
  Real qx[QC], qll[QC];
  bool spec1 = false;  // qx / qll hold the second chunk's predicted particles and log-likelihoods
  Real z[NZ];
  if (p.do_update) {
#pragma unroll
    for (int k = 0; k < NZ; ++k) z[k] = ((const Real*)p.z)[(int64_t)r * p.z_rs + k];
  }
  const Real* u = p.u ? (const Real*)p.u + (int64_t)r * p.u_rs : nullptr;
  if constexpr (PRE) {
    if (t < nchunks) {
      const int64_t i0 = o0 + (int64_t)t * CH;
      if constexpr (CH == 4) {
        Real v[4];
        load4<Real>(x_in + i0, v);
#pragma unroll
        for (int e = 0; e < 4; ++e) sx[e][0] = v[e];
        if (p.do_update) load4<Real>(lw_in + i0, sl);
#ifndef PF_NO_PRE1
        if (t + BS < nchunks)  // two-pass tiles: the second chunk's loads overlap the first's work
#else
        if (false)
#endif
        {
          const int64_t i1 = o0 + (int64_t)(t + BS) * CH;
          load4<Real>(x_in + i1, px);
          if (p.do_update) load4<Real>(lw_in + i1, pl);
          pre1 = true;
        }
        if (p.do_predict) {
          Real n4[4];
          chunk_normals4<Real>(p.seed, i0, (uint32_t)r, rep, p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, n4,
                               p.pbase);
#pragma unroll
          for (int e = 0; e < 4; ++e) sn[e][0] = n4[e];
        }
      } else {
#pragma unroll
        for (int d = 0; d < NX; ++d) sx[0][d] = x_in[(int64_t)d * p.Npad + i0];
        if (p.do_update) sl[0] = lw_in[i0];
        if (p.do_predict)
          fill_normals<NX, Real>(p.seed, i0, (uint32_t)r, rep, p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, sn[0],
                                 p.pbase);
      }
#pragma unroll
      for (int e = 0; e < SC; ++e) {
        if (CH == 4 || i0 + e < o1) {  // scalar state: slots past the tile computed too (padding, never used) - no per-slot branches
          if (p.do_predict) {
            M::transition(sx[e], P, u);
            M::add_lower(sx[e], sn[e], P, M::L::LQ);
          }
          sll[e] = (p.do_update == 1) ? M::loglik(sx[e], z, P, p.r_diag != 0) : Real(0);
        }
      }
      if constexpr (FASTX) {
        if (pre1 && p.do_update == 1) {
          const int64_t i1 = o0 + (int64_t)(t + BS) * CH;
          Real n4[4];
          if (p.do_predict)
            chunk_normals4<Real>(p.seed, i1, (uint32_t)r, rep, p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, n4,
                                 p.pbase);
#pragma unroll
          for (int e = 0; e < 4; ++e) {  // slots past o1 are never stored nor weighed
            Real xe[1] = {px[e]};
            if (p.do_predict) {
              M::transition(xe, P, u);
              Real ne[1] = {n4[e]};
              M::add_lower(xe, ne, P, M::L::LQ);
            }
            qx[e] = xe[0];
            qll[e] = M::loglik(xe, z, P, p.r_diag != 0);
          }
          spec1 = true;
        }
      }
    }
  }

  // ---- (0) prologue ---------------------------------------------------------
  Head h;
  if (p.head) {
    h = load_head<BS>(p.head, r, p.G, p.allow_gather != 0 && p.method == 0, Pl);
    PF_STAMP(1);
  } else {
    h = prologue<NX, BS>(rec_in, p.G, p.N, p.thresh, p.allow_gather != 0, p.force_gather != 0,
                         p.allow_gather != 0 && p.method == 0, red, Pl);
    PF_STAMP(1);
    write_outputs<NX, BS>(p, rec_in, h, r, R, b, p.G, red);
  }
  PF_STAMP(2);
  const bool gather = h.resample != 0;
  const double lprev_uniform = -log((double)p.N);

  // ---- (2)+(3) per chunk: [gather + jitter] -> [predict] -> [weight] -> store
  WA acc;
  acc.init();
  constexpr int NA = 1 + NX + RC::NC;  // aux: cnt, sum x, sum x x^T
  double aux[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) aux[i] = 0.0;
  const double lse_prev = h.uniform ? 0.0 : (p.use_lse_ext ? p.lse_ext : h.lse);  // shards: the global lse
  const Real lse_r = (Real)lse_prev;
  const bool write_x = p.do_predict || p.allow_gather;  // gather launches always produce x_out

  bool fast = false, gfast = false;
  // the generic chunk loop, instantiated for gathering and non-gathering workgroups apart: in the
  // gathering one the speculated chunks are dead (fewer live registers through the ancestors)
  auto chunk_loop = [&](auto gather_tag) {
    constexpr bool gather_c = decltype(gather_tag)::value;
    for (int c = t; c < nchunks; c += BS) {
      const int64_t i0 = o0 + (int64_t)c * CH;
      const bool first = PRE && c == t;
      const bool spec = first && !gather_c;  // predicted x and loglik already computed
      Real x[CH][NX];
      Real lp[CH];
      Real ll[CH];
      if (gather_c) {
#pragma unroll
        for (int e = 0; e < CH; ++e) {
          const int a = (i0 + e < o1) ? anc_l[c * CH + e] : 0;
#pragma unroll
          for (int d = 0; d < NX; ++d) x[e][d] = x_in[(int64_t)d * p.Npad + a];
          lp[e] = (Real)lprev_uniform;
        }
      } else {
        Real lraw[CH];
        if (spec) {
#pragma unroll
          for (int e = 0; e < CH; ++e) {
#pragma unroll
            for (int d = 0; d < NX; ++d) x[e][d] = sx[SC == CH ? e : 0][d];
            lraw[e] = sl[SC == CH ? e : 0];
            ll[e] = sll[SC == CH ? e : 0];
          }
        } else if constexpr (CH == 4) {
          if (pre1 && c == t + BS) {  // prefetched before the prologue
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              x[e][0] = px[e];
              lraw[e] = pl[e];
            }
          } else {
            Real v[4];
            load4<Real>(x_in + i0, v);
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e][0] = v[e];
            if (p.do_update && !h.uniform) load4<Real>(lw_in + i0, lraw);
          }
        } else {
#pragma unroll
          for (int d = 0; d < NX; ++d) x[0][d] = x_in[(int64_t)d * p.Npad + i0];
          if (p.do_update && !h.uniform) lraw[0] = lw_in[i0];
        }
        if (p.do_update) {
#pragma unroll
          for (int e = 0; e < CH; ++e)
            lp[e] = h.uniform ? (Real)lprev_uniform : lraw[e] - lse_r;
        }
      }

      Real nj4[CH], np4[CH];
      if constexpr (CH == 4) {  // one Philox call covers the chunk's 4 scalar particles
        if (gather_c && p.regularize)
          chunk_normals4<Real>(p.seed, i0, (uint32_t)r, rep, p.ep_resample, STREAM_JITTER, p.rp_jit, p.N, nj4, p.pbase);
        if (p.do_predict) {
          if (first) {
#pragma unroll
            for (int e = 0; e < 4; ++e) np4[e] = sn[e][0];
          } else {
            chunk_normals4<Real>(p.seed, i0, (uint32_t)r, rep, p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, np4,
                                 p.pbase);
          }
        }
      }
#pragma unroll
      for (int e = 0; e < CH; ++e) {
        const int64_t i = i0 + e;
        if (i >= o1) break;
        Real* xe = x[e];
        if (gather_c) {
          if (p.regularize) {
            Real n[NX];
            if constexpr (CH == 4) n[0] = nj4[e];
            else fill_normals<NX, Real>(p.seed, i, (uint32_t)r, rep, p.ep_resample, STREAM_JITTER, p.rp_jit, p.N, n,
                                        p.pbase);
            M::add_lower(xe, n, P, M::L::LJ);
          }
          aux[0] += 1.0;
#pragma unroll
          for (int d = 0; d < NX; ++d) aux[1 + d] += (double)xe[d];
          if constexpr (RC::COV) {
            int cc = 1 + NX;
#pragma unroll
            for (int d = 0; d < NX; ++d)
#pragma unroll
              for (int f = d; f < NX; ++f) aux[cc++] += (double)xe[d] * (double)xe[f];
          }
        }
        if (!spec) {
          if (p.do_predict) {
            Real n[NX];
            if constexpr (CH == 4) {
              n[0] = np4[e];
            } else if (first) {
#pragma unroll
              for (int d = 0; d < NX; ++d) n[d] = sn[0][d];
            } else {
              fill_normals<NX, Real>(p.seed, i, (uint32_t)r, rep, p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, n,
                                     p.pbase);
            }
            M::transition(xe, P, u);
            M::add_lower(xe, n, P, M::L::LQ);
          }
          ll[e] = (p.do_update == 1) ? M::loglik(xe, z, P, p.r_diag != 0) : Real(0);
        }
        if (p.do_update) {
          lp[e] = lp[e] + ll[e];  // log(w_prev) - quad/2  (do_update == 2: reweigh only, ll = 0)
          acc.add(lp[e], xe);
        }
      }
      if constexpr (CH == 4) {
        if (i0 + 3 < o1) {
          if (write_x) {
            Real v[4] = {x[0][0], x[1][0], x[2][0], x[3][0]};
            store4<Real>(x_out + i0, v);
          }
          if (p.do_update) store4<Real>(lw_out + i0, lp);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (i0 + e < o1) {
              if (write_x) x_out[i0 + e] = x[e][0];
              if (p.do_update) lw_out[i0 + e] = lp[e];
            }
          }
        }
      } else {
        if (write_x)
#pragma unroll
          for (int d = 0; d < NX; ++d) x_out[(int64_t)d * p.Npad + i0] = x[0][d];
        if (p.do_update) lw_out[i0] = lp[0];
      }
    }
  };

  // ---- (1) ancestors of this thread's slots (LDS), then the chunks ----------
  if (gather) {
    if (p.method == 0) {
      const double U = p.rp_unif ? p.rp_unif[r] : uniform53(p.seed, 0, rep, p.ep_resample);
      constexpr int PM = sizeof(Real) == 4 ? 8 : 1;  // fp64: reloaded from L2 (registers)
      sys_ancestors<Real, NX, BS, PM>(lw_in, rec_in, p.G, p.N, p.tile, o0, o1, U, h, Pl, anc_l, red, stamp_on);
    } else {  // multinomial: binary search of the materialised CDF (cdf /= cdf[-1])
      const double* C = p.cdf + (int64_t)r * p.N;
      const double last = C[p.N - 1];
      for (int c = t; c < nchunks; c += BS) {
#pragma unroll
        for (int e = 0; e < CH; ++e) {
          const int64_t i = o0 + (int64_t)c * CH + e;
          if (i < o1) {
            const double uu = p.rp_unif ? p.rp_unif[(int64_t)r * p.N + i] : uniform53(p.seed, (uint32_t)i, rep, p.ep_resample);
            int64_t lo = 0, hi = p.N;
            while (lo < hi) {
              const int64_t mid = (lo + hi) >> 1;
              if (uu < C[mid] / last) hi = mid; else lo = mid + 1;
            }
            anc_l[c * CH + e] = (int)(lo < p.N ? lo : p.N - 1);
          }
        }
      }
    }
    PF_STAMP(3);
    // gather-fast (fp32 scalar, <= 2 chunks per thread, fused predict + update after a resample): the
    // thread's 8 gathered slots straight through, weighed against the workgroup maximum as the fast
    // path does - so this step and the same step run as a gather-only launch followed by a fast launch
    // (a run cut at a resample) give bitwise the same records
    if constexpr (FASTX) {
#ifndef PF_GFAST
#define PF_GFAST 1
#endif
      gfast = PF_GFAST && gather && p.do_predict && p.do_update == 1 && nchunks <= 2 * BS;
      Real xv[8], lp[8];
      Real mt = -INFINITY;  // this thread's maximum log-weight
      if (gfast && t < nchunks) {
        const int ca = t, cb = t + BS;
        const int64_t ia = o0 + (int64_t)ca * CH, ib = o0 + (int64_t)cb * CH;
        const int na = (int)min((int64_t)4, o1 - ia), nb = cb < nchunks ? (int)min((int64_t)4, o1 - ib) : 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xv[e] = e < na ? x_in[anc_l[ca * CH + e]] : Real(0);
          xv[4 + e] = e < nb ? x_in[anc_l[cb * CH + e]] : Real(0);
        }
        if (p.regularize) {
          Real ja[4], jb[4];
          chunk_normals4<Real>(p.seed, ia, (uint32_t)r, rep, p.ep_resample, STREAM_JITTER, p.rp_jit, p.N, ja, p.pbase);
          if (nb > 0)
            chunk_normals4<Real>(p.seed, ib, (uint32_t)r, rep, p.ep_resample, STREAM_JITTER, p.rp_jit, p.N, jb, p.pbase);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            Real xa[1] = {xv[e]}, na1[1] = {ja[e]};
            M::add_lower(xa, na1, P, M::L::LJ);
            xv[e] = xa[0];
            if (nb > 0) {
              Real xb[1] = {xv[4 + e]}, nb1[1] = {jb[e]};
              M::add_lower(xb, nb1, P, M::L::LJ);
              xv[4 + e] = xb[0];
            }
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // the generic loop's order: chunk t's slots, then chunk t + BS's
          if (e < na || (e >= 4 && e - 4 < nb)) {
            aux[0] += 1.0;
            aux[1] += (double)xv[e];
            if constexpr (RC::COV) aux[2] += (double)xv[e] * (double)xv[e];
          }
        }
        Real pb[4];
        if (nb > 0)
          chunk_normals4<Real>(p.seed, ib, (uint32_t)r, rep, p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, pb, p.pbase);
        const Real lu = (Real)lprev_uniform;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool in = e < 4 ? e < na : e - 4 < nb;
          Real xe[1] = {xv[e]};
          Real ne[1] = {e < 4 ? sn[e][0] : pb[e - 4]};
          M::transition(xe, P, u);
          M::add_lower(xe, ne, P, M::L::LQ);
          xv[e] = in ? xe[0] : Real(0);
          lp[e] = in ? lu + M::loglik(xe, z, P, p.r_diag != 0) : -INFINITY;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) mt = rmax<Real>(mt, lp[e]);
        if (na == 4) {
          store4<Real>(x_out + ia, xv);
          store4<Real>(lw_out + ia, lp);
        } else {
          for (int e = 0; e < na; ++e) {
            x_out[ia + e] = xv[e];
            lw_out[ia + e] = lp[e];
          }
        }
        if (nb == 4) {
          store4<Real>(x_out + ib, xv + 4);
          store4<Real>(lw_out + ib, lp + 4);
        } else {
          for (int e = 0; e < nb; ++e) {
            x_out[ib + e] = xv[4 + e];
            lw_out[ib + e] = lp[4 + e];
          }
        }
      }
      if (gfast) {  // uniform: the workgroup's reference maximum, then the thread's sums against it
        const Real Mb = block_max_r<BS>(mt, cdf + 32);  // the merge staging area: free here
        if (t < nchunks) acc.add_ref8(lp, xv, Mb);
      }
    }
    if (!gfast) chunk_loop(std::true_type{});
  } else {
    PF_STAMP(3);
    // fast finish of the fp32 scalar step (uniform per workgroup): every chunk of the thread was
    // speculated and nothing is gathered
    if constexpr (FASTX) {
#ifndef PF_NO_PRE1
      constexpr int SPEC_CHUNKS = 2;
#else
      constexpr int SPEC_CHUNKS = 1;
#endif
      fast = !gather && p.do_update == 1 && nchunks <= SPEC_CHUNKS * BS;  // fused step, or update only
      Real lp[8], xv[8];
      Real mt = -INFINITY;  // this thread's maximum log-weight
      if (fast && t < nchunks) {
        const Real lu = (Real)lprev_uniform;
        const int64_t ia = o0 + (int64_t)t * CH, ib = o0 + (int64_t)(t + BS) * CH;
        const int na = (int)min((int64_t)4, o1 - ia), nb = spec1 ? (int)min((int64_t)4, o1 - ib) : 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // arithmetic on every slot, then selects (no per-slot branches)
          const Real va = (h.uniform ? lu : sl[e] - lse_r) + sll[e];
          const Real vb = (h.uniform ? lu : pl[e] - lse_r) + qll[e];
          xv[e] = e < na ? sx[e][0] : Real(0);  // slots past the tile: zero weight, finite value
          lp[e] = e < na ? va : -INFINITY;
          xv[4 + e] = e < nb ? qx[e] : Real(0);
          lp[4 + e] = e < nb ? vb : -INFINITY;
        }
        // the weights against the workgroup's maximum (add_ref8) - the same pass the gather-fast block
        // makes, so a step after a gather-only launch (a run cut at a resample) and the same step fused
        // with its gather give bitwise the same records: a run cut into segments stays the uninterrupted run
#pragma unroll
        for (int e = 0; e < 8; ++e) mt = rmax<Real>(mt, lp[e]);
        if (na == 4) {
          if (write_x) store4<Real>(x_out + ia, xv);
          store4<Real>(lw_out + ia, lp);
        } else {
          for (int e = 0; e < na; ++e) {
            if (write_x) x_out[ia + e] = xv[e];
            lw_out[ia + e] = lp[e];
          }
        }
        if (nb == 4) {
          if (write_x) store4<Real>(x_out + ib, xv + 4);
          store4<Real>(lw_out + ib, lp + 4);
        } else {
          for (int e = 0; e < nb; ++e) {
            if (write_x) x_out[ib + e] = xv[4 + e];
            lw_out[ib + e] = lp[4 + e];
          }
        }
      }
      if (fast) {  // uniform
        const Real Mb = block_max_r<BS>(mt, cdf + 32);  // the merge staging area: free here
        if (t < nchunks) acc.add_ref8(lp, xv, Mb);
      }
    }

    if (!fast) chunk_loop(std::false_type{});
  }
  PF_STAMP(4);

  // ---- (4) this tile's partial record (field-major) --------------------------
  if (!(p.do_update || p.allow_gather)) return;
  double* rec_out = p.rec_out + (int64_t)r * RC::SIZE * p.G;
  double* fin = cdf;  // staged record: RC::SIZE doubles (tile area is free again)
  __syncthreads();    // all tile-CDF / ancestor reads are done
  if (p.do_update) {
    double w[1 + WA::NS];
#if PF_MERGE_LDS
    if constexpr (NX == 1 && sizeof(Real) == 4) {  // staged after the record's slots (step_lds: MERGE_LDS_BYTES)
      static_assert((WA::NS + 1) * BS * 4 + 32 * 8 <= MERGE_LDS_BYTES && RC::SIZE <= 32, "merge staging");
      if (fast || gfast) acc.template block_sum_lds<BS>((float*)(cdf + 32), w);  // one reference maximum
      else acc.template block_merge_lds<BS>((float*)(cdf + 32), w);
    }
    else
#endif
    if constexpr (FASTD) {
      if (fast || gfast) acc.template block_sum_ref<BS>(red, w);  // one reference maximum: plain sums
      else acc.template block_merge<BS>(red, w);
    } else
      acc.template block_merge<BS>(red, w);
    if (t == 0) {
      fin[RC::M] = w[0];
      fin[RC::S0] = w[1];
      fin[RC::S00] = w[2];
      fin[RC::UNI] = 0.0;
      for (int i = 0; i < NX + RC::NC; ++i) fin[RC::S1 + i] = w[3 + i];
    }
  } else if (t == 0) {
    if (gather) {  // gather-only launch: weights become uniform
      fin[RC::M] = 0.0; fin[RC::S0] = 0.0; fin[RC::S00] = 0.0; fin[RC::UNI] = 1.0;
      for (int q = RC::S1; q < RC::A1; ++q) fin[q] = 0.0;
    } else {  // gather-only launch that did not resample: carry the update's record over
      for (int q = 0; q < RC::A1; ++q) fin[q] = rec_in[q * p.G + b];
    }
  }
  if (gather) {
    block_sum_k<NA, BS>(aux, red);
    if (t == 0) {
      fin[RC::CNT] = aux[0];
      for (int i = 0; i < NX + RC::NC; ++i) fin[RC::A1 + i] = aux[1 + i];
    }
  } else if (t == 0) {
    fin[RC::CNT] = 0.0;
    for (int q = RC::A1; q < RC::SIZE; ++q) fin[q] = 0.0;
  }
  __syncthreads();
  PF_STAMP(5);
  for (int q = t; q < RC::SIZE; q += BS) rec_out[q * p.G + b] = fin[q];
}

// ---------------------------------------------------------------------------
// Finalize: posterior outputs of the records in rec_in (one workgroup per replicate)
// ---------------------------------------------------------------------------
// (same block size and reduction tree as k_step's prologue -> bitwise the same decision)
template <int NX, int BS>
__global__ void __launch_bounds__(BS) k_finalize(StepParams p) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int r = blockIdx.x, R = gridDim.x;
  const double* rec = p.rec_in + (int64_t)r * Rec<NX>::SIZE * p.G;
  const Head h = prologue<NX, BS>(rec, p.G, p.N, p.thresh, p.allow_gather != 0, false, false, smem, nullptr);
  write_outputs<NX, BS>(p, rec, h, r, R, 0, 1, smem);
}

// ---------------------------------------------------------------------------
// Multinomial: materialise the CDF of the update in rec_in (if it resamples)
// ---------------------------------------------------------------------------
template <typename Real, int NX, int BS>
__global__ void __launch_bounds__(BS) k_cdf(StepParams p, double* cdf_out) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  double* Pl = smem + LDS_PL;
  double* cdf = smem + lds_tile(p.G);
  const int b = blockIdx.x, r = blockIdx.y;
  const double* rec = p.rec_in + (int64_t)r * Rec<NX>::SIZE * p.G;
  const Head h = p.head ? load_head<BS>(p.head, r, p.G, true, Pl)
                        : prologue<NX, BS>(rec, p.G, p.N, p.thresh, true, p.force_gather != 0, true, red, Pl);
  if (!h.resample) return;
  const Real* lw = (const Real*)p.lw_in + (int64_t)r * p.Npad;
  const int len = tile_cdf<Real, NX, BS>(lw, rec, p.G, p.N, p.tile, b, h, Pl, cdf, red);
  for (int j = threadIdx.x; j < len; j += BS) cdf_out[(int64_t)r * p.N + (int64_t)b * p.tile + j] = cdf[j];
}

// ---------------------------------------------------------------------------
// Head: the summary of rec_in for every replicate (grid H x R), once per step, for
// the many-replicate launches (StepParams::head).  The same prologue() and block
// size as the kernels that read it -> bitwise the decision they would compute.
// Also writes the step's outputs (write_outputs over the H workgroups).
// ---------------------------------------------------------------------------
template <int NX, int BS>
__global__ void __launch_bounds__(BS) k_head(StepParams p, double* head) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  double* Pl = smem + LDS_PL;
  const int b = blockIdx.x, r = blockIdx.y, R = gridDim.y;
  const double* rec = p.rec_in + (int64_t)r * Rec<NX>::SIZE * p.G;
  const bool allow = p.allow_gather != 0;
  const Head h = prologue<NX, BS>(rec, p.G, p.N, p.thresh, allow, p.force_gather != 0, allow, red, Pl);
  write_outputs<NX, BS>(p, rec, h, r, R, b, gridDim.x, red);
  if (b != 0) return;
  double* o = head + (int64_t)r * HEAD_STRIDE;
  if (threadIdx.x == 0) {
    o[0] = h.M;
    o[1] = h.S;
    o[2] = h.S2;
    o[3] = h.Sscan;
    o[4] = h.lse;
    o[5] = h.neff;
    o[6] = h.uniform ? 1.0 : 0.0;
    o[7] = h.resample ? 1.0 : 0.0;
  }
  if (allow && h.resample)
    for (int k = threadIdx.x; k <= p.G; k += BS) o[HEAD_F + k] = Pl[k];
}

// ---------------------------------------------------------------------------
// initialize(): x = mean + chol(cov) n, records -> uniform weights
// ---------------------------------------------------------------------------
template <typename Real, int NX>
__global__ void __launch_bounds__(BLOCK) k_init(Real* x, double* rec, const Real* mean /*[R][NX]*/,
                                                const Real* Lc /*[R][NX][NX]*/, const double* replay,
                                                int64_t N, int64_t Npad, int G, uint64_t seed,
                                                uint32_t epoch, int rep_base, int64_t pbase) {
  using RC = Rec<NX>;
  const int r = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i < N) {
    Real n[NX];
    fill_normals<NX, Real>(seed, i, (uint32_t)r, (uint32_t)(r + rep_base), epoch, STREAM_INIT, replay, N, n, pbase);
    const Real* L = Lc + (int64_t)r * NX * NX;
#pragma unroll
    for (int d = 0; d < NX; ++d) {
      Real acc = Real(0);
#pragma unroll
      for (int e = 0; e <= d; ++e) acc += n[e] * L[d * NX + e];
      x[((int64_t)r * NX + d) * Npad + i] = acc + mean[r * NX + d];
    }
  }
  const int64_t k = i;  // one record per tile (field q at [q*G + k])
  if (k < G) {
    double* o = rec + (int64_t)r * RC::SIZE * G;
    for (int q = 0; q < RC::SIZE; ++q) o[(int64_t)q * G + k] = 0.0;
    o[(int64_t)RC::UNI * G + k] = 1.0;
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
  const bool uni = rec[(int64_t)r * G * RS + 3 * (int64_t)G] != 0.0;
  const Real* xr = x + ((int64_t)r * NX + d) * Npad;
  const Real* lr = lw + (int64_t)r * Npad;
  double v[2] = {0.0, 0.0};
  for (int64_t i = threadIdx.x; i < N; i += BLOCK) {
    const double w = mom_weight<Real>(lr, i, uni, lse[r]);
    v[0] += w;
    v[1] += w * (double)xr[i];
  }
  block_sum_k<2>(v, smem);
  if (threadIdx.x == 0) mean[(int64_t)r * NX + d] = v[1] / v[0];
}

template <typename Real, int NX>
__global__ void __launch_bounds__(BLOCK) k_mom_cov(const Real* x, const Real* lw, const double* rec, int RS, int G,
                                                   const double* lse, int64_t N, int64_t Npad, const double* mean,
                                                   double* cov) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int d = blockIdx.x / NX, e = blockIdx.x % NX, r = blockIdx.y;
  if (e < d) return;
  const bool uni = rec[(int64_t)r * G * RS + 3 * (int64_t)G] != 0.0;
  const Real* xd = x + ((int64_t)r * NX + d) * Npad;
  const Real* xe = x + ((int64_t)r * NX + e) * Npad;
  const Real* lr = lw + (int64_t)r * Npad;
  const double md = mean[(int64_t)r * NX + d], me = mean[(int64_t)r * NX + e];
  double v[2] = {0.0, 0.0};
  for (int64_t i = threadIdx.x; i < N; i += BLOCK) {
    const double w = mom_weight<Real>(lr, i, uni, lse[r]);
    v[0] += w;
    v[1] += w * ((double)xd[i] - md) * ((double)xe[i] - me);
  }
  block_sum_k<2>(v, smem);
  if (threadIdx.x == 0) {
    cov[(int64_t)r * NX * NX + d * NX + e] = v[1] / v[0];
    cov[(int64_t)r * NX * NX + e * NX + d] = v[1] / v[0];
  }
}

}  // namespace pf
