// Posterior covariance of the reported state, every step of the device loop, any nx
// (pf.py:266-267: cov = np.cov(particles.T, aweights=w, bias=True) on the state update() returns).
//
// The reported state of step s is the post-resample particle set (uniform weights) when step s
// resampled, else the predicted particles with their normalised weights w_i = e^(l_i - lse).
// The step kernels cover nx <= 4 in their tile records; for larger states the record would need
// nx(nx+1)/2 sums per tile, so the device loop computes it here instead, as the GEMM it is.
//
// Numerics follow np.cov (centre, then multiply): each wave first takes its particles' weighted
// mean c_w (about its first particle; a resampled set of copies gives exactly zero spread, as
// np.cov does), then accumulates
//   W_w = sum w_i,  S1_w = sum w_i (x_i - c_w),  S2_w = Y^T Y with Y[i][d] = sqrt(w_i) (x_id - c_wd)
// (S2 by MFMA in 16x16 blocks over the upper block triangle: v_mfma_f32_16x16x4_f32 for the fp32
// engine, fp32 partials over one wave's particles and fp64 from there on; v_mfma_f64_16x16x4 for
// the fp64 engine; S1 / W by fp64 VALU), so m_w = c_w + S1_w / W_w and M2_w = S2_w - S1_w S1_w^T / W_w.
// Waves, then blocks, then the whole set combine exactly (Chan et al.):
//   W = sum W_b,  m = sum W_b m_b / W,  M2 = sum_b [M2_b + W_b (m_b - m)(m_b - m)^T],  cov = M2 / W.
// Rows: the post-resample rows the gather wrote (StepParams::xr_out) or the predicted rows.  Fixed
// reduction orders throughout (deterministic).
//
//   k_cov_part  grid (nblk, R, npz), 4 waves per block, wave w takes particles
//               [(4 b + w) per_wave, +per_wave); NB > 0: every block pair of the upper triangle in one
//               wave (nx <= 48); NB == 0: the block pair blockIdx.z (any nx).  -> block partials
//               [pairs][256] M2_b | [nb][16] m_b | W_b
//   k_cov_sum   grid (ceil(npairs 256 / 16), R), 16 entries x 16 lanes per workgroup: the lanes of an
//               entry split the blocks; the last workgroup to finish (per replicate) writes cov.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pf {

struct CovParams {
  const void* xs;       // [R][nx][Npad] predicted particles of the step (Real)
  const void* xr;       // [R][nx][Npad] post-resample rows of the step (written by the next gather)
  const void* lw;       // [R][Npad] unnormalised log-weights of the step (Real)
  int64_t N, Npad;
  int nx, nb, npairs, P;   // blocks of 16 components, block pairs (upper triangle), partial size
  int nblk, per_wave;      // blocks per replicate, particles per wave (multiple of 4)
  const int32_t* flag;     // [R] resampled at this step
  const double* lse;       // [R] log normaliser of lw
  double* part;            // [R][nblk][P]
  double* tot;             // [R][P]
  unsigned int* cnt;       // [R] workgroups of k_cov_sum done (the last one resets it)
  double* cov;             // [R][nx][nx]
};

__host__ __device__ inline int cov_pair_index(int bi, int bj, int nb) { return bi * nb - bi * (bi - 1) / 2 + (bj - bi); }
__host__ __device__ inline void cov_pair_blocks(int pr, int nb, int* bi, int* bj) {
  int i = 0;
  while (pr >= nb - i) {
    pr -= nb - i;
    ++i;
  }
  *bi = i;
  *bj = i + pr;
}

typedef float cov_f4 __attribute__((ext_vector_type(4)));
typedef double cov_d4 __attribute__((ext_vector_type(4)));

template <typename Real>
struct CovMfma;
template <>
struct CovMfma<float> {  // C/D: col = lane & 15, row = 4 (lane >> 4) + reg
  typedef cov_f4 acc_t;
  __device__ static acc_t zero() { return acc_t{0.f, 0.f, 0.f, 0.f}; }
  __device__ static acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32((float)a, (float)b, c, 0, 0, 0);
  }
  __device__ static int row(int lane, int reg) { return 4 * (lane >> 4) + reg; }
};
template <>
struct CovMfma<double> {  // C/D: col = lane & 15, row = (lane >> 4) + 4 reg
  typedef cov_d4 acc_t;
  __device__ static acc_t zero() { return acc_t{0.0, 0.0, 0.0, 0.0}; }
  __device__ static acc_t mma(double a, double b, acc_t c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
  __device__ static int row(int lane, int reg) { return (lane >> 4) + 4 * reg; }
};

// LDS per workgroup: 4 waves x (NPW 256 M2 | NBL 16 mean | W) doubles
template <int NB>
__host__ __device__ constexpr int cov_wave_slots(int npw_runtime) {
  return (NB > 0 ? NB * (NB + 1) / 2 : npw_runtime) * 256 + (NB > 0 ? NB : 2) * 16 + 1;
}

// NB > 0: nb == NB, all NB (NB + 1) / 2 pairs per wave.  NB == 0: the pair blockIdx.z.
template <typename Real, int NB>
__global__ void __launch_bounds__(256) k_cov_part(CovParams p) {
  using MF = CovMfma<Real>;
  constexpr int NBL = NB > 0 ? NB : 2;                 // row blocks a wave loads
  constexpr int NPW = NB > 0 ? NB * (NB + 1) / 2 : 1;  // pairs a wave accumulates
  constexpr int WS = cov_wave_slots<NB>(1);            // LDS doubles per wave
  constexpr int OM = NPW * 256, OW = OM + NBL * 16;    // offsets of the means and W in a wave's slots
  extern __shared__ __attribute__((aligned(16))) double cs[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, kq = lane >> 4;
  const int b = blockIdx.x, r = blockIdx.y;
  int blk[NBL];  // the row blocks this wave loads
  int pair0 = 0;
  if constexpr (NB > 0) {
#pragma unroll
    for (int k = 0; k < NB; ++k) blk[k] = k;
  } else {
    cov_pair_blocks(blockIdx.z, p.nb, &blk[0], &blk[1]);
    pair0 = blockIdx.z;
  }
  const bool res = p.flag[r] != 0;
  const Real* X = (const Real*)(res ? p.xr : p.xs) + (int64_t)r * p.nx * p.Npad;
  const Real* L = (const Real*)p.lw + (int64_t)r * p.Npad;
  const double lse = p.lse[r], swu = sqrt(1.0 / (double)p.N);  // uniform weights: sqrt(1/N)
  const int64_t i0 = ((int64_t)b * 4 + w) * p.per_wave;
  const int64_t i1 = min(i0 + (int64_t)p.per_wave, p.N);
  int dd[NBL];
  double cd[NBL];  // the wave's centre: its weighted mean (pass 1, about its first particle)
#pragma unroll
  for (int k = 0; k < NBL; ++k) {
    dd[k] = blk[k] * 16 + col;
    cd[k] = (i0 < i1 && dd[k] < p.nx) ? (double)X[(int64_t)dd[k] * p.Npad + i0] : 0.0;
  }
  auto weight_root = [&](int64_t i) -> double {  // sqrt(w_i) of this lane's particle (0 past the range)
    if (i >= i1) return 0.0;
    if (res) return swu;
    const Real l = L[i];
    return (l > -INFINITY) ? sqrt(exp((double)l - lse)) : 0.0;
  };
  {
    double m1[NBL], w1 = 0.0;
#pragma unroll
    for (int k = 0; k < NBL; ++k) m1[k] = 0.0;
    for (int64_t ib = i0; ib < i1; ib += 4) {
      const int64_t i = ib + kq;
      const double sw = weight_root(i);
      const double wi = sw * sw;
      w1 += wi;
#pragma unroll
      for (int k = 0; k < NBL; ++k)
        if (i < i1 && dd[k] < p.nx) m1[k] += wi * ((double)X[(int64_t)dd[k] * p.Npad + i] - cd[k]);
    }
    w1 += __shfl_xor(w1, 16);
    w1 += __shfl_xor(w1, 32);
#pragma unroll
    for (int k = 0; k < NBL; ++k) {
      m1[k] += __shfl_xor(m1[k], 16);
      m1[k] += __shfl_xor(m1[k], 32);
      if (w1 > 0.0) cd[k] += m1[k] / w1;
    }
  }
  typename MF::acc_t acc[NPW];
#pragma unroll
  for (int q = 0; q < NPW; ++q) acc[q] = MF::zero();
  double s1[NBL], wsum = 0.0;
#pragma unroll
  for (int k = 0; k < NBL; ++k) s1[k] = 0.0;
  for (int64_t ib = i0; ib < i1; ib += 4) {
    const int64_t i = ib + kq;  // this lane's particle (k index of the MFMA)
    const double sw = weight_root(i);
    double y[NBL];
#pragma unroll
    for (int k = 0; k < NBL; ++k) {
      const bool in = i < i1 && dd[k] < p.nx;
      y[k] = in ? sw * ((double)X[(int64_t)dd[k] * p.Npad + i] - cd[k]) : 0.0;
      s1[k] += sw * y[k];
    }
    if (col == 0) wsum += sw * sw;
    if constexpr (NB > 0) {
      int q = 0;
#pragma unroll
      for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int bj = bi; bj < NB; ++bj, ++q) acc[q] = MF::mma(y[bi], y[bj], acc[q]);
    } else {
      acc[0] = MF::mma(y[0], y[1], acc[0]);
    }
  }
  // S1 / W over the four k lanes of each column
#pragma unroll
  for (int k = 0; k < NBL; ++k) {
    s1[k] += __shfl_xor(s1[k], 16);
    s1[k] += __shfl_xor(s1[k], 32);
  }
  wsum += __shfl_xor(wsum, 16);
  wsum += __shfl_xor(wsum, 32);
  wsum = __shfl(wsum, 0);
  // this wave's mean and S1 (LDS, for the rows of its MFMA tiles), then M2_w = S2 - S1 S1^T / W
  double* mine = cs + (int64_t)w * WS;
  if (kq == 0) {
#pragma unroll
    for (int k = 0; k < NBL; ++k) {
      mine[OM + k * 16 + col] = s1[k];  // S1 for now, the mean below
    }
    if (col == 0) mine[OW] = wsum;
  }
  __syncthreads();
  const double iw = wsum > 0.0 ? 1.0 / wsum : 0.0;
#pragma unroll
  for (int q = 0; q < NPW; ++q) {
    int a = 0, c2 = 1;  // the wave-local block indices of pair q
    if constexpr (NB > 0) {
      int bi = 0, bj = 0;
      cov_pair_blocks(q, NB, &bi, &bj);
      a = bi;
      c2 = bj;
    } else {
      a = 0;
      c2 = 1;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int rw = MF::row(lane, g);
      const double m2 = (double)acc[q][g] - mine[OM + a * 16 + rw] * mine[OM + c2 * 16 + col] * iw;
      mine[q * 256 + rw * 16 + col] = m2;
    }
  }
  __syncthreads();
  if (kq == 0) {
#pragma unroll
    for (int k = 0; k < NBL; ++k) mine[OM + k * 16 + col] = cd[k] + mine[OM + k * 16 + col] * iw;  // m_w
  }
  __syncthreads();
  // the block's 4 waves combined (Chan): W_b, m_b, M2_b
  double* out = p.part + ((int64_t)r * p.nblk + b) * p.P;
  double Wb = 0.0;
  for (int v = 0; v < 4; ++v) Wb += cs[v * WS + OW];
  const double iWb = Wb > 0.0 ? 1.0 / Wb : 0.0;
  __shared__ double mb[NBL * 16];
  for (int e = threadIdx.x; e < NBL * 16; e += 256) {
    double s = 0.0;
    for (int v = 0; v < 4; ++v) s += cs[v * WS + OW] * cs[v * WS + OM + e];
    mb[e] = s * iWb;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NPW * 256; e += 256) {
    const int q = e >> 8, rw = (e >> 4) & 15, cl = e & 15;
    int a = 0, c2 = 1;
    if constexpr (NB > 0) cov_pair_blocks(q, NB, &a, &c2);
    double s = 0.0;
    for (int v = 0; v < 4; ++v) {
      const double* wv = cs + v * WS;
      const double da = wv[OM + a * 16 + rw] - mb[a * 16 + rw], dc = wv[OM + c2 * 16 + cl] - mb[c2 * 16 + cl];
      s += wv[e] + wv[OW] * da * dc;
    }
    out[(NB > 0 ? 0 : pair0 * 256) + e] = s;
  }
  const int nbl = NB > 0 ? NB : 1;  // mean blocks this workgroup owns (diagonal pairs only for NB == 0)
  if (NB > 0 || blk[0] == blk[1]) {
    for (int e = threadIdx.x; e < nbl * 16; e += 256) out[p.npairs * 256 + blk[0] * 16 * (NB > 0 ? 0 : 1) + e] = mb[e];
  }
  if (threadIdx.x == 0 && (NB > 0 || pair0 == 0)) out[p.npairs * 256 + p.nb * 16] = Wb;
}

// M2 entries over the blocks (Chan), 16 lanes per entry splitting the blocks; the last workgroup
// to finish per replicate writes cov = M2 / W (symmetric).
__global__ void __launch_bounds__(256) k_cov_sum(CovParams p) {
  const int r = blockIdx.y, t = threadIdx.x, sub = t & 15;
  const int e = blockIdx.x * 16 + (t >> 4);  // M2 slot: pair e >> 8, row (e >> 4) & 15, col e & 15
  const double* base = p.part + (int64_t)r * p.nblk * p.P;
  const int OM = p.npairs * 256, OW = OM + p.nb * 16;
  double* T = p.tot + (int64_t)r * p.P;
  if (e < p.npairs * 256) {
    int bi = 0, bj = 0;
    cov_pair_blocks(e >> 8, p.nb, &bi, &bj);
    const int d = bi * 16 + ((e >> 4) & 15), f = bj * 16 + (e & 15);
    double W = 0.0, md = 0.0, mf = 0.0;
    for (int k = sub; k < p.nblk; k += 16) {
      const double* q = base + (int64_t)k * p.P;
      const double wk = q[OW];
      W += wk;
      md += wk * q[OM + d];
      mf += wk * q[OM + f];
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      W += __shfl_xor(W, o);
      md += __shfl_xor(md, o);
      mf += __shfl_xor(mf, o);
    }
    const double iW = W > 0.0 ? 1.0 / W : 0.0;
    md *= iW;
    mf *= iW;
    double s = 0.0;
    for (int k = sub; k < p.nblk; k += 16) {
      const double* q = base + (int64_t)k * p.P;
      s += q[e] + q[OW] * (q[OM + d] - md) * (q[OM + f] - mf);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (sub == 0) {
      T[e] = s;
      if (e == 0) T[OW] = W;
    }
  }
  __threadfence();
  __shared__ int last;
  __syncthreads();
  if (t == 0) last = atomicAdd(p.cnt + r, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  // the other workgroups' sums: device-coherent loads (never a line this CU's L1 may hold)
  auto ld = [](const double* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const double W = ld(T + OW);
  const double iW = W > 0.0 ? 1.0 / W : 0.0;
  double* cov = p.cov + (int64_t)r * p.nx * p.nx;
  for (int g = t; g < p.nx * p.nx; g += 256) {
    const int d0 = g / p.nx, f0 = g % p.nx;
    const int d = min(d0, f0), f = max(d0, f0);  // the upper-triangle entry for both: exactly symmetric
    const double m2 = ld(T + cov_pair_index(d >> 4, f >> 4, p.nb) * 256 + (d & 15) * 16 + (f & 15));
    cov[g] = m2 * iW;
  }
  if (t == 0) p.cnt[r] = 0u;
}

}  // namespace pf
