// Posterior covariance of the reported state, every step of the device loop, any nx
// (pf.py:266-267: cov = np.cov(particles.T, aweights=w, bias=True) on the state update() returns).
//
// The reported state of step s is the post-resample particle set (uniform weights) when step s
// resampled, else the predicted particles with their normalised weights w_i = e^(l_i - lse).
// The step kernels cover nx <= 4 in their tile records; for larger states the record would need
// nx(nx+1)/2 sums per tile, so the device loop computes it here instead, as the GEMM it is:
//
//   S2 = Y^T Y,  Y[i][d] = sqrt(w_i) (x_id - c_d),   S1 = sum_i w_i (x_i - c),  W = sum_i w_i
//   cov = S2 / W - (S1 / W)(S1 / W)^T
//
// with c the step's weighted mean (pre-resample, already an output of the loop) as the shift.
// S2 is accumulated by MFMA in 16x16 blocks over the upper block triangle (v_mfma_f32_16x16x4_f32 for
// the fp32 engine: fp32 partial sums over one wave's particles, fp64 from there on; v_mfma_f64_16x16x4
// for the fp64 engine); S1 and W by fp64 VALU.  Rows: the post-resample rows the gather wrote
// (StepParams::xr_out) or the predicted rows.  Fixed reduction order throughout (deterministic).
//
//   k_cov_part  grid (nblk, R, npz): 4 waves per block, wave w takes particles
//               [(4 b + w) per_wave, +per_wave); NB > 0: every block pair of the upper triangle in one
//               wave (nx <= 48); NB == 0: one pair per blockIdx.z (any nx).  The 4 waves' sums are
//               combined in LDS into one partial per block.
//   k_cov_sum   grid (ceil(P / 256), R): partials summed over blocks in block order; the last block to
//               finish (per replicate) writes cov.
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
  const double* mean;      // [R][nx] weighted (pre-resample) mean: the shift
  double* part;            // [R][nblk][P]
  double* tot;             // [R][P]
  unsigned int* cnt;       // [R] blocks of k_cov_sum done (the last one resets it)
  double* cov;             // [R][nx][nx]
};

__host__ __device__ inline int cov_pair_index(int bi, int bj, int nb) { return bi * nb - bi * (bi - 1) / 2 + (bj - bi); }

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

// NB > 0: nb == NB, all NB (NB + 1) / 2 pairs per wave.  NB == 0: the pair blockIdx.z.
template <typename Real, int NB>
__global__ void __launch_bounds__(256) k_cov_part(CovParams p) {
  using MF = CovMfma<Real>;
  constexpr int NBL = NB > 0 ? NB : 2;                 // row blocks a wave loads
  constexpr int NPW = NB > 0 ? NB * (NB + 1) / 2 : 1;  // pairs a wave accumulates
  extern __shared__ __attribute__((aligned(16))) double cs[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, col = lane & 15, kq = lane >> 4;
  const int b = blockIdx.x, r = blockIdx.y;
  int blk[NBL];  // the row blocks this wave loads
  int pair0 = 0;
  if constexpr (NB > 0) {
#pragma unroll
    for (int k = 0; k < NB; ++k) blk[k] = k;
  } else {  // pair z of the upper triangle -> (bi, bj)
    int z = blockIdx.z, bi = 0;
    while (z >= p.nb - bi) {
      z -= p.nb - bi;
      ++bi;
    }
    blk[0] = bi;
    blk[1] = bi + z;
    pair0 = blockIdx.z;
  }
  const bool res = p.flag[r] != 0;
  const Real* X = (const Real*)(res ? p.xr : p.xs) + (int64_t)r * p.nx * p.Npad;
  const Real* L = (const Real*)p.lw + (int64_t)r * p.Npad;
  const double lse = p.lse[r], invN = 1.0 / (double)p.N, swu = sqrt(invN);
  const double* c = p.mean + (int64_t)r * p.nx;
  int dd[NBL];
  double cd[NBL];
#pragma unroll
  for (int k = 0; k < NBL; ++k) {
    dd[k] = blk[k] * 16 + col;
    cd[k] = dd[k] < p.nx ? c[dd[k]] : 0.0;
  }
  typename MF::acc_t acc[NPW];
#pragma unroll
  for (int q = 0; q < NPW; ++q) acc[q] = MF::zero();
  double s1[NBL], wsum = 0.0;
#pragma unroll
  for (int k = 0; k < NBL; ++k) s1[k] = 0.0;
  const int64_t i0 = ((int64_t)b * 4 + w) * p.per_wave;
  const int64_t i1 = min(i0 + (int64_t)p.per_wave, p.N);
  for (int64_t ib = i0; ib < i1; ib += 4) {
    const int64_t i = ib + kq;  // this lane's particle (k index of the MFMA)
    double sw = 0.0;
    if (i < i1) {
      if (res) {
        sw = swu;
      } else {
        const Real l = L[i];
        sw = (l > -INFINITY) ? sqrt(exp((double)l - lse)) : 0.0;
      }
    }
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
  // per-wave sums -> LDS [4][P'] (P' = this block's slots), combined in wave order
  const int Pw = NB > 0 ? p.P : 256 + 16 + 1;
  double* mine = cs + (int64_t)w * Pw;
#pragma unroll
  for (int q = 0; q < NPW; ++q)
#pragma unroll
    for (int g = 0; g < 4; ++g) mine[q * 256 + MF::row(lane, g) * 16 + col] = (double)acc[q][g];
  if (kq == 0) {
    const int nbl = NB > 0 ? NB : 1;
#pragma unroll
    for (int k = 0; k < NBL; ++k)
      if (k < nbl) mine[NPW * 256 + k * 16 + col] = s1[k];
    if (col == 0) mine[NPW * 256 + nbl * 16] = wsum;
  }
  __syncthreads();
  double* out = p.part + ((int64_t)r * p.nblk + b) * p.P;
  for (int e = threadIdx.x; e < Pw; e += 256) {
    const double v = cs[e] + cs[Pw + e] + cs[2 * Pw + e] + cs[3 * Pw + e];
    if constexpr (NB > 0) {
      out[e] = v;
    } else {  // this pair's block, its S1 block (diagonal pairs) and W (pair 0)
      const int bi = blk[0], bj = blk[1];
      if (e < 256) out[pair0 * 256 + e] = v;
      else if (e < 256 + 16) { if (bi == bj) out[p.npairs * 256 + bi * 16 + (e - 256)] = v; }
      else if (pair0 == 0) out[p.npairs * 256 + p.nb * 16] = v;
    }
  }
}

// partials summed over blocks (block order), then cov from the sums by the last block per replicate
__global__ void __launch_bounds__(256) k_cov_sum(CovParams p) {
  const int r = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e < p.P) {
    const double* src = p.part + (int64_t)r * p.nblk * p.P + e;
    double s = 0.0;
    for (int k = 0; k < p.nblk; ++k) s += src[(int64_t)k * p.P];
    p.tot[(int64_t)r * p.P + e] = s;
  }
  __threadfence();
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(p.cnt + r, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  // the other blocks' sums: device-coherent loads (never a line this CU's L1 may hold)
  const double* T = p.tot + (int64_t)r * p.P;
  auto ld = [](const double* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const double W = ld(T + p.npairs * 256 + p.nb * 16);
  const double* S1 = T + p.npairs * 256;
  double* cov = p.cov + (int64_t)r * p.nx * p.nx;
  for (int f = threadIdx.x; f < p.nx * p.nx; f += 256) {
    const int d = f / p.nx, e2 = f % p.nx;
    const int bd = d >> 4, be = e2 >> 4;
    const double s2 = bd <= be ? ld(T + cov_pair_index(bd, be, p.nb) * 256 + (d & 15) * 16 + (e2 & 15))
                               : ld(T + cov_pair_index(be, bd, p.nb) * 256 + (e2 & 15) * 16 + (d & 15));
    const double md = ld(S1 + d) / W, me = ld(S1 + e2) / W;
    cov[f] = s2 / W - md * me;
  }
  if (threadIdx.x == 0) p.cnt[r] = 0u;
}

}  // namespace pf
