// Posterior covariance of the reported state, every step of the device loop, any nx
// (pf.py:266-267: cov = np.cov(particles.T, aweights=w, bias=True) on the state update() returns).
//
// The reported state of step s is the post-resample particle set (uniform weights) when step s
// resampled, else the predicted particles with their normalised weights w_i = e^(l_i - lse).
// The step kernels cover nx <= 4 in their tile records; for larger states the record would need
// nx(nx+1)/2 sums per tile, so the device loop computes it here instead, as the GEMM it is:
//
//   Y[i][d] = sqrt(w_i) (x_id - c_d),  S2 = Y^T Y,  S1 = sum_i w_i (x_i - c),  W = sum_i w_i
//   cov = S2 / W - (S1 / W)(S1 / W)^T
//
// with c the step's weighted (pre-resample) mean, already an output of the loop: the set is
// centred before the products, so S1 / W is O(sampling noise) and nothing cancels.  Each workgroup
// stages 256 particles' centred, weighted rows in LDS with coalesced loads (component-major, rows
// padded so the MFMA operand reads are bank-conflict-free), then each of its 4 waves runs 16 MFMA
// k-steps over 64 of them: S2 in 16x16 blocks over the upper block triangle (v_mfma_f32_16x16x4_f32
// for the fp32 engine - fp32 sums over 64 particles, fp64 from there on - v_mfma_f64_16x16x4 for the
// fp64 engine), S1 / W in fp64.  Rows: the predicted rows, or on a resample step the post-resample
// rows - read through the ancestor indices the next gather wrote (StepParams::anc_out: without
// jitter post-resample row i is predicted row anc[i]), or, with jitter, the rows it wrote
// (StepParams::xr_out).  Fixed reduction orders throughout (deterministic).
//
//   k_cov_part  grid (ceil(N / (256 cpb)), R, npz): NB > 0: every block pair of the upper triangle
//               (nx <= 48); NB == 0: the block pair blockIdx.z (any nx).  -> block partials
//               [pairs][256] S2 | [nb][16] S1 | W
//               into a ring slot: the partials of up to Tc steps (Tc from a memory budget) wait
//               there, so a step costs this one launch;
//   k_cov_fin_sum / k_cov_fin_out  once per Tc steps (and at the end of the run): every entry's
//               block sum in block order, then the chunk's covariances (symmetric).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pf {

struct CovParams {
  const void* xs;       // [R][nx][Npad] predicted particles of the step (Real)
  const void* xr;       // [R][nx][Npad] post-resample (jittered) rows of the step (written by the next gather)
  const int32_t* anc;   // [R][N] or null: the next gather's ancestors (no jitter: post-resample row i = xs row anc[i])
  const void* lw;       // [R][Npad] unnormalised log-weights of the step (Real)
  int64_t N, Npad;
  int nx, nb, npairs, P;   // blocks of 16 components, block pairs (upper triangle), partial size
  int nblk;                // workgroups per replicate (cpb chunks of 256 particles each)
  int cpb;                 // 256-particle chunks per workgroup
  const int32_t* flag;     // [R] resampled at this step
  const double* lse;       // [R] log normaliser of lw
  const double* mean;      // [R][nx] the step's weighted (pre-resample) mean: the centre
  void* part;              // [R][nblk][P] doubles: this step's ring slot
  int diag;                // experiment knob (PF_COV_DIAG): 1 no staging loads, 2 no MFMA loop, 4 no output
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
  __device__ static acc_t mma(float a, float b, acc_t c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
  __device__ static int row(int lane, int reg) { return 4 * (lane >> 4) + reg; }
};
template <>
struct CovMfma<double> {  // C/D: col = lane & 15, row = (lane >> 4) + 4 reg
  typedef cov_d4 acc_t;
  __device__ static acc_t zero() { return acc_t{0.0, 0.0, 0.0, 0.0}; }
  __device__ static acc_t mma(double a, double b, acc_t c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
  __device__ static int row(int lane, int reg) { return (lane >> 4) + 4 * reg; }
};

constexpr int COV_BLK = 256;  // particles per chunk (64 per wave: 16 MFMA k-steps)
constexpr int COV_YS = COV_BLK + 4;  // LDS row stride (elements): lanes (col, kq) read 64 distinct banks
constexpr int COV_CPB_MAX = 8;       // chunks per workgroup

// chunks per workgroup.  One: every workgroup's load -> products -> store chain runs once and the
// grid is a single round (measured, profiles/r03/cov: L96 1e5 16.7 vs 19.7 us at two chunks, MAT
// 8 x 1e5 19.6 vs 27.2 at eight; the smaller partial ring does not pay for the longer chain).
__host__ inline int cov_chunks_per_block(int64_t, int) { return 1; }

// LDS bytes of k_cov_part: the staged rows (reused for the waves' sums) + sqrt weights
template <typename Real, int NB>
__host__ __device__ constexpr size_t cov_part_lds() {
  constexpr int NBL = NB > 0 ? NB : 2, NPW = NB > 0 ? NB * (NB + 1) / 2 : 1;
  constexpr size_t ys = (size_t)NBL * 16 * COV_YS * sizeof(Real);
  constexpr size_t comb = 4 * ((size_t)NPW * 256 + NBL * 16 + 1) * sizeof(double);
  return (ys > comb ? ys : comb) + (COV_BLK + NBL * 16) * sizeof(double);
}

// NB > 0: nb == NB, all NB (NB + 1) / 2 pairs per wave.  NB == 0: the pair blockIdx.z.
// A workgroup runs cpb chunks of 256 particles into the same MFMA accumulators; the next chunk's
// rows are loaded into registers while the current chunk's products run (its ancestors one chunk
// earlier still), so the row stream is not serialised behind the products.
template <typename Real, int NB>
__global__ void __launch_bounds__(256) k_cov_part(CovParams p) {
  using MF = CovMfma<Real>;
  constexpr int NBL = NB > 0 ? NB : 2;                 // row blocks staged
  constexpr int NPW = NB > 0 ? NB * (NB + 1) / 2 : 1;  // pairs per wave
  constexpr int WS = NPW * 256 + NBL * 16 + 1;         // one wave's sums (doubles)
  extern __shared__ __attribute__((aligned(16))) double cs[];
  constexpr size_t YB = (size_t)NBL * 16 * COV_YS * sizeof(Real);
  constexpr size_t CB = 4 * (size_t)WS * sizeof(double);
  Real* ys = (Real*)cs;                                               // [NBL * 16][COV_YS]
  double* sws = cs + (YB > CB ? YB : CB) / sizeof(double);            // [256] sqrt weights
  double* cl = sws + COV_BLK;                                         // [NBL * 16] the centre
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, col = lane & 15, kq = lane >> 4;
  const int b = blockIdx.x, r = blockIdx.y;
  if (p.diag & 32) return;
  int blk[NBL];
  int pair0 = 0;
  if constexpr (NB > 0) {
#pragma unroll
    for (int k = 0; k < NB; ++k) blk[k] = k;
  } else {
    cov_pair_blocks(blockIdx.z, p.nb, &blk[0], &blk[1]);
    pair0 = blockIdx.z;
  }
  const bool res = p.flag[r] != 0;
  const bool by_anc = res && p.anc != nullptr;
  const Real* X = (const Real*)((res && !by_anc) ? p.xr : p.xs) + (int64_t)r * p.nx * p.Npad;
  const int32_t* A = p.anc ? p.anc + (int64_t)r * p.N : nullptr;
  const Real* LW = (const Real*)p.lw + (int64_t)r * p.Npad;
  const double lse = p.lse[r];
  const double* c = p.mean + (int64_t)r * p.nx;
  const int64_t wg0 = (int64_t)b * p.cpb * COV_BLK;
  const int nch = (int)min((int64_t)p.cpb, (p.N - wg0 + COV_BLK - 1) / COV_BLK);  // chunks of this workgroup (>= 1)
  if (t < NBL * 16) {  // the centre through LDS: one vector load instead of a serial scalar-load chain
    const int d = blk[t >> 4] * 16 + (t & 15);
    cl[t] = d < p.nx ? c[d] : 0.0;
  }
  // ---- per chunk: thread t = particle base + t (coalesced rows); unconditional loads from
  //      clamped addresses (all issued before the first use), masked when staged ----
  Real xv[NBL][16];
  Real lv = Real(0);
  int an = 0;  // ancestor of the next chunk's slot (by_anc)
  auto issue_rows = [&](int64_t base, int col_i) {
#pragma unroll
    for (int k = 0; k < NBL; ++k)
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) xv[k][cc] = X[(int64_t)min(blk[k] * 16 + cc, p.nx - 1) * p.Npad + col_i];
    if (!res) lv = LW[col_i];
    (void)base;
  };
  auto slot_col = [&](int64_t base) -> int { return base + t < p.N ? (int)(base + t) : 0; };
  // the ancestors are loaded whether or not this step resampled (not behind the flag's load)
  if (A) an = A[slot_col(wg0)];
  issue_rows(wg0, by_anc ? an : slot_col(wg0));
  if (by_anc && nch > 1) an = A[slot_col(wg0 + COV_BLK)];
  double accd[NPW][4];  // the chunks' MFMA sums in fp64 (fp32 MFMA sums span 64 particles only)
#pragma unroll
  for (int q = 0; q < NPW; ++q)
#pragma unroll
    for (int g = 0; g < 4; ++g) accd[q][g] = 0.0;
  double s1[NBL], wsum = 0.0;
#pragma unroll
  for (int k = 0; k < NBL; ++k) s1[k] = 0.0;
  for (int ch = 0; ch < nch; ++ch) {
    const int64_t base = wg0 + (int64_t)ch * COV_BLK;
    const bool live = base + t < p.N;
    double sw = 0.0;
    if (live) sw = res ? sqrt(1.0 / (double)p.N) : ((lv > -INFINITY) ? sqrt(exp((double)lv - lse)) : 0.0);
    __syncthreads();  // the previous chunk's rows are consumed; cl is written (first chunk)
    sws[t] = sw;
#pragma unroll
    for (int k = 0; k < NBL; ++k)
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) {
        const int d = blk[k] * 16 + cc;
        const double v = (d < p.nx && !(p.diag & 1)) ? sw * ((double)xv[k][cc] - cl[k * 16 + cc]) : 0.0;
        ys[(k * 16 + cc) * COV_YS + t] = (Real)v;
      }
    __syncthreads();
    if (ch + 1 < nch) {  // the next chunk's rows (and the ancestors of the one after) in flight
      const int64_t nb_ = base + COV_BLK;
      issue_rows(nb_, by_anc ? an : slot_col(nb_));
      if (by_anc && ch + 2 < nch) an = A[slot_col(nb_ + COV_BLK)];
    }
    // ---- this wave's 64 particles: 16 MFMA k-steps per pair, S1 / W in fp64 ----
    typename MF::acc_t acc[NPW];
#pragma unroll
    for (int q = 0; q < NPW; ++q) acc[q] = MF::zero();
#pragma unroll 4
    for (int st = 0; st < ((p.diag & 2) ? 0 : 16); ++st) {
      const int i = w * 64 + 4 * st + kq;
      const double swi = sws[i];
      Real y[NBL];
#pragma unroll
      for (int k = 0; k < NBL; ++k) {
        y[k] = ys[(k * 16 + col) * COV_YS + i];
        s1[k] += swi * (double)y[k];
      }
      if (col == 0) wsum += swi * swi;
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
#pragma unroll
    for (int q = 0; q < NPW; ++q)
#pragma unroll
      for (int g = 0; g < 4; ++g) accd[q][g] += (double)acc[q][g];
  }
#pragma unroll
  for (int k = 0; k < NBL; ++k) {
    s1[k] += __shfl_xor(s1[k], 16);
    s1[k] += __shfl_xor(s1[k], 32);
  }
  wsum += __shfl_xor(wsum, 16);
  wsum += __shfl_xor(wsum, 32);
  __syncthreads();  // the staged rows are consumed: their LDS now takes the waves' sums
  double* mine = cs + (int64_t)w * WS;
#pragma unroll
  for (int q = 0; q < NPW; ++q)
#pragma unroll
    for (int g = 0; g < 4; ++g) mine[q * 256 + MF::row(lane, g) * 16 + col] = accd[q][g];
  if (kq == 0) {
#pragma unroll
    for (int k = 0; k < NBL; ++k) mine[NPW * 256 + k * 16 + col] = s1[k];
    if (col == 0) mine[NPW * 256 + NBL * 16] = wsum;
  }
  __syncthreads();
  double* out = (double*)p.part + ((int64_t)r * p.nblk + b) * p.P;
  for (int e = t; e < ((p.diag & 4) ? 0 : WS); e += 256) {
    const double v = ((cs[e] + cs[WS + e]) + cs[2 * WS + e]) + cs[3 * WS + e];
    if constexpr (NB > 0) {
      out[e] = v;
    } else {  // this pair's block, its S1 block (diagonal pairs) and W (pair 0)
      if (e < 256) out[pair0 * 256 + e] = v;
      else if (e < 256 + 16) { if (blk[0] == blk[1]) out[p.npairs * 256 + blk[0] * 16 + (e - 256)] = v; }
      else if (e == 256 + 32 && pair0 == 0) out[p.npairs * 256 + p.nb * 16] = v;
    }
  }
}

// The blocks' partials of n consecutive steps (a chunk of the ring the k_cov_part launches fill)
// summed per entry in block order - one lane per entry, 16 independent loads in flight - then
// cov = S2 / W - (S1 / W)(S1 / W)^T per step, exactly symmetric.  Two launches per chunk.
struct CovFin {
  const void* part;    // [n][R][nblk][P], float when part_f32
  int part_f32;
  double* tot;         // [n][R][P]
  double* cov;         // [n][R][nx][nx]: the chunk's first step
  int R, nblk, P, nx, nb, npairs;
};

// grid (ceil(P / 256), n R), 256 threads; PT: the partials' type (double; fp32 partials were tried:
// the 4-byte strided reads of this kernel took 98 instead of 23 us per 32-step chunk)
template <typename PT>
__global__ void __launch_bounds__(256) k_cov_fin_sum(CovFin f) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int64_t jr = blockIdx.y;  // step-in-chunk * R + replicate
  if (e >= f.P) return;
  const PT* src = (const PT*)f.part + jr * f.nblk * f.P + e;
  double s = 0.0;
  for (int k0 = 0; k0 < f.nblk; k0 += 16) {
    double v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = k0 + k < f.nblk ? (double)src[(int64_t)(k0 + k) * f.P] : 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += v[k];
  }
  f.tot[jr * f.P + e] = s;
}

// grid (ceil(nx^2 / 256), n R), 256 threads
__global__ void __launch_bounds__(256) k_cov_fin_out(CovFin f) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  const int64_t jr = blockIdx.y;
  if (g >= f.nx * f.nx) return;
  const double* T = f.tot + jr * f.P;
  const int OM = f.npairs * 256;
  const double W = T[OM + f.nb * 16];
  const double iW = W > 0.0 ? 1.0 / W : 0.0;
  const int d0 = g / f.nx, f0 = g % f.nx;
  const int d = min(d0, f0), c = max(d0, f0);  // the upper-triangle entry for both: exactly symmetric
  const double s2 = T[cov_pair_index(d >> 4, c >> 4, f.nb) * 256 + (d & 15) * 16 + (c & 15)];
  f.cov[jr * f.nx * f.nx + g] = s2 * iW - (T[OM + d] * iW) * (T[OM + c] * iW);
}

}  // namespace pf
