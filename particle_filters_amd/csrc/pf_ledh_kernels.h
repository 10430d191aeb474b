// LEDH particle-flow kernels for gfx950 (fp64, wave64).
//
// The reference's LEDHFlowPF.step (/root/reference/models/LEDH_particle_filter.py,
// "ledh.py:LINE") linearises h at every particle for every pseudo-time step
// lambda_j and forms dense nx x nx matrices per particle:
//   S = lam H P H^T + R,  A = -1/2 P H^T S^{-1} H,  b = (I + 2 lam A)[(I + lam A) P H^T R^{-1}(z - e) + A eta0]
//   eta += dlam (A eta + b),  theta += log|det(I + dlam A)|                        (ledh.py:136-179)
// Here the same quantities are evaluated in observation space, never forming A:
//   K = P H^T (nx x nz), M = H K, Gm = -1/2 K S^{-1}  =>  A v = Gm (H v),
//   det(I + dlam A) = det(S - dlam/2 M) / det(S)      (matrix-determinant lemma;
//   the reference's +1e-12 I retry becomes (1+eps)^nx det(S - dlam/(2(1+eps)) M) / det(S)).
// That is O(nx nz^2 + nz^3) per particle and lambda instead of O(nx^3).
//
// Two flow kernels:
//   k_flow_affine  h linear (L96 x[::k], linear test systems): H, e = c, and hence K, M, S, Gm,
//                  the logdets and P H^T R^{-1}(z - e) are the SAME for every particle, so
//                  the whole lambda integration is an affine map of eta0.  k_setup builds the
//                  per-lambda_j matrices (one workgroup per j), k_compose folds the L steps
//                  into eta_L = eta0 + d0 + D (H eta0); a particle then costs g, its noise,
//                  two small mat-vecs and the weight.  4 lanes per particle (L96: 10
//                  contiguous components per lane, RK4 neighbours by lane shuffles).
//   k_flow_wave    any h with an analytic Jacobian (EXP_HALF, ACOUSTIC): one 64-lane
//                  workgroup per particle (persistent over particles), the small dense
//                  algebra in LDS with lanes over matrix entries.
// Both end in the weight of ledh.py:186-190:
//   l_i = log(w_i + 1e-300) + theta_i + log N(eta_i; g(x_i), Q) + log N(z; h(eta_i), R) - log N(eta0_i; g(x_i), Q)
// (the Gaussian normalising constants cancel between numerator and denominator, and
// across particles in the normalisation, so they are not evaluated).
//
// Then the weight pipeline (tiles of LT particles, fixed-order reductions so every
// workgroup derives bit-identical global scalars):
//   k_tile_max -> k_exp_sum -> k_normalise (w, tile sums of w, w^2, w x) -> k_decide (ESS,
//   resample flag) -> [k_cdf -> k_gather] (systematic, ledh.py:25-37, 204-206) ->
//   k_mean_part -> k_mean -> k_cov_part -> k_cov (ledh.py:217-224).
//
// Layout in HBM: particles SoA x[nx][Npad] (fp64), weights w[N] (normalised, ledh.py:195).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pf_ledh.h"
#include "pf_dpp.h"
#include "philox.h"

namespace pf {
namespace ledh {

// diagnostic phase stamps (PF_STAMPS builds only): s_memrealtime (100 MHz) per workgroup, slots
// 0-5 the fused step's phases (pf_ledh_fused.h), 6-11 the first flow round's sub-phases, 12-19 the
// sub-phases of P2-P4
#ifdef PF_STAMPS
constexpr int FST = 20;
__device__ unsigned long long g_ledh_stamps[256 * FST];
#define LF_STAMP(k)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 256) g_ledh_stamps[blockIdx.x * FST + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// k_flow_wave_lr phase accumulators (workgroup 0, thread 0): ticks of 10 ns per phase over a launch
__device__ unsigned long long g_lr_acc[16];
#define LR_MARK(k)                                                          \
  do {                                                                      \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                              \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();     \
      g_lr_acc[k] += now_ - lr_last_;                                       \
      lr_last_ = now_;                                                      \
    }                                                                       \
  } while (0)
#else
#define LF_STAMP(k) \
  do {              \
  } while (0)
#define LR_MARK(k) \
  do {             \
  } while (0)
#endif

constexpr int TB = 256;    // block of the per-particle-thread and reduction kernels
constexpr int LT = 1024;   // particles per reduction tile
constexpr int MAXT = 1024; // tiles (N <= LT * MAXT)
constexpr int CT = 128;    // particles per covariance sub-tile (staged in LDS)
constexpr int CTS = 1;     // sub-tiles per moments workgroup

// ---------------------------------------------------------------------------
// parameter layout (doubles)
// ---------------------------------------------------------------------------
template <int NX, int NZ>
struct Lay {
  static constexpr int A = 0;                 // NX*NX transition matrix (LINEAR g)
  static constexpr int EX = A + NX * NX;      // F, dt (L96 g)
  static constexpr int H = EX + 2;            // NZ*NX observation matrix (LINEAR h)
  static constexpr int C = H + NZ * NX;       // NZ offset (LINEAR) / beta (EXP_HALF)
  static constexpr int AC = C + NZ;           // psi, d0, sx[NZ], sy[NZ] (ACOUSTIC)
  static constexpr int LQ = AC + 2 + 2 * NZ;  // NX*NX chol(Q) (device noise)
  static constexpr int QI = LQ + NX * NX;     // NX*NX Q^{-1}
  static constexpr int R = QI + NX * NX;      // NZ*NZ R
  static constexpr int RI = R + NZ * NZ;      // NZ*NZ R^{-1}
  static constexpr int SIZE = RI + NZ * NZ;
};

// shared-path flow table (doubles)
template <int NX, int NZ>
struct TLay {
  static constexpr int Cv = 0;               // NX  c = K R^{-1}(z - e)   (= P H^T R^{-1}(z - e), ledh.py:163-164)
  static constexpr int HC = Cv + NX;         // NZ  H c
  static constexpr int HEAD = HC + NZ;
  static constexpr int GM = 0;               // NX*NZ  Gm_j = -1/2 K S_j^{-1}
  static constexpr int HGM = GM + NX * NZ;   // NZ*NZ  H Gm_j
  static constexpr int AC = HGM + NZ * NZ;   // NX     A_j c = Gm_j H c
  static constexpr int HAC = AC + NX;        // NZ     H A_j c
  static constexpr int LD = HAC + NZ;        // 1      log|det(I + dlam A_j)|
  static constexpr int PJ = LD + 1;
  // the composed flow (k_compose): eta_L = eta0 + d0 + D (H eta0), H eta_L = pL + QL (H eta0)
  static constexpr int aff(int L) { return HEAD + L * PJ; }
  static constexpr int D0 = 0;               // NX
  static constexpr int DM = D0 + NX;         // NX*NZ
  static constexpr int PL = DM + NX * NZ;    // NZ
  static constexpr int QL = PL + NZ;         // NZ*NZ
  static constexpr int TH = QL + NZ * NZ;    // 1  theta = sum_j log|det(I + dlam A_j)|
  static constexpr int AFF_SIZE = TH + 1;
  static constexpr int size(int L) { return aff(L) + AFF_SIZE; }
};

struct FlowParams {
  const double* x_in;   // [NX][Npad]
  double* x_out;        // [NX][Npad]
  const double* w_in;   // [N] normalised weights
  double* lw;           // [N] unnormalised log weights (out)
  const double* Pm;     // Lay
  const double* Pk;     // [NX][NX] symmetrised tracker covariance
  const double* z;      // [NZ]
  const double* u;      // [NX] or null
  const double* v_host; // [N][NX] or null
  const double* table;  // TLay (shared path)
  int64_t pk_stride, z_stride, table_stride;  // batched k_setup / k_compose over steps (blockIdx.y / .x)
  const double* lams;   // [L]
  double* diagS;        // [L][NZ][NZ] or null (S of particle 0)
  int64_t N, Npad;
  int L;
  double dlam;
  int noise;
  uint64_t seed;
  uint32_t epoch;
  int q_diag, r_diag;
  // EDH (pf_edh_kernels.h): tracker past means x_{k-1|k-1} [nx] per step, u per step, integrator
  const double* xbar;
  int64_t xbar_stride, u_stride;
  int integ;
  // test hook (pf_hooks.h, PF_TEST_FLOW_LR_FORCE): k_flow_wave_lr's fallbacks forced - bit 0 the
  // Householder QR instead of the Gram's Cholesky factor, bit 1 the separate pivoted determinants,
  // bit 2 the +1e-12 I retry; 0 in every product launch
  int lr_force;
};

// ---------------------------------------------------------------------------
// model pieces
// ---------------------------------------------------------------------------
template <int NX>
__device__ __forceinline__ double l96_rhs_at(const double* x, int a, double F) {
  return (x[(a + 1) % NX] - x[(a + NX - 2) % NX]) * x[(a + NX - 1) % NX] - x[a] + F;
}

// g(x, u) for one particle in registers (thread path)
template <int NX, int NZ, int TK>
__device__ __forceinline__ void g_thread(double* x, const double* __restrict__ Pm, const double* u) {
  using L = Lay<NX, NZ>;
  if constexpr (TK == PF_TRANS_LINEAR) {
    double y[NX];
#pragma unroll
    for (int d = 0; d < NX; ++d) {
      double acc = 0.0;
#pragma unroll
      for (int e = 0; e < NX; ++e) acc += Pm[L::A + d * NX + e] * x[e];
      y[d] = acc;
    }
#pragma unroll
    for (int d = 0; d < NX; ++d) x[d] = u ? y[d] + u[d] : y[d];
  } else {  // L96: x + dt/6 (k1 + 2 k2 + 2 k3 + k4)  (simulator_Lorenz_96.py:62-84)
    const double F = Pm[L::EX], dt = Pm[L::EX + 1];
    double k[NX], acc[NX], tmp[NX];
#pragma unroll
    for (int a = 0; a < NX; ++a) k[a] = l96_rhs_at<NX>(x, a, F);
#pragma unroll
    for (int a = 0; a < NX; ++a) { acc[a] = k[a]; tmp[a] = x[a] + 0.5 * dt * k[a]; }
#pragma unroll
    for (int a = 0; a < NX; ++a) k[a] = l96_rhs_at<NX>(tmp, a, F);
#pragma unroll
    for (int a = 0; a < NX; ++a) { acc[a] += 2.0 * k[a]; }
#pragma unroll
    for (int a = 0; a < NX; ++a) tmp[a] = x[a] + 0.5 * dt * k[a];
#pragma unroll
    for (int a = 0; a < NX; ++a) k[a] = l96_rhs_at<NX>(tmp, a, F);
#pragma unroll
    for (int a = 0; a < NX; ++a) { acc[a] += 2.0 * k[a]; tmp[a] = x[a] + dt * k[a]; }
#pragma unroll
    for (int a = 0; a < NX; ++a) k[a] = l96_rhs_at<NX>(tmp, a, F);
    const double h6 = dt / 6.0;
#pragma unroll
    for (int a = 0; a < NX; ++a) x[a] = x[a] + h6 * (acc[a] + k[a]);
    if (u) {
#pragma unroll
      for (int a = 0; a < NX; ++a) x[a] += u[a];
    }
  }
}

// normals of the flat indices f0 .. f0+PER-1 (NumPy row-major order of an (N, nx) draw):
// one Philox call per group of 4 consecutive flat indices
template <int PER>
__device__ __forceinline__ void normals_range(uint64_t seed, int64_t f0, uint32_t epoch, uint32_t stream, double* n) {
  constexpr int GMAX = PER / 4 + 2;
  const int64_t g0 = f0 >> 2, g1 = (f0 + PER - 1) >> 2;
#pragma unroll
  for (int gg = 0; gg < GMAX; ++gg) {
    const int64_t g = g0 + gg;
    if (g <= g1) {
      const Normal4<double> q4 = normal4_bm24d(seed, (uint32_t)g, 0u, epoch, stream);
      // flat index 4g + e lands in slot 4g + e - f0 = 4 gg + e - (f0 & 3)
      const int sh = (int)(f0 & 3);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int j = 0; j < PER; ++j)
          if (4 * gg + e - sh == j) n[j] = q4.v[e];
      }
    }
  }
}

// process noise of particle i (thread path): v = chol(Q) n, n ~ Philox, or the host draw
template <int NX, int NZ>
__device__ __forceinline__ void noise_thread(const FlowParams& p, int64_t i, double* v) {
  using L = Lay<NX, NZ>;
  if (p.noise == PF_NOISE_HOST) {
#pragma unroll
    for (int d = 0; d < NX; ++d) v[d] = p.v_host[i * NX + d];
  } else if (p.noise == PF_NOISE_DEVICE) {
    double n[NX];
#pragma unroll
    for (int d = 0; d < NX; ++d) {
      const int64_t f = i * NX + d;
      n[d] = pick4(normal4_bm24d(p.seed, (uint32_t)(f >> 2), 0u, p.epoch, STREAM_PROCESS), (int)(f & 3));
    }
#pragma unroll
    for (int d = 0; d < NX; ++d) {
      double acc = 0.0;
#pragma unroll
      for (int e = 0; e <= d; ++e) acc += p.Pm[L::LQ + d * NX + e] * n[e];
      v[d] = acc;
    }
  } else {
#pragma unroll
    for (int d = 0; d < NX; ++d) v[d] = 0.0;
  }
}

// d^T C d for C = Q^{-1} (NX) or R^{-1} (NZ), row-major at Pm[off]
template <int D>
__device__ __forceinline__ double quad_form(const double* d, const double* __restrict__ C, bool diag) {
  double q = 0.0;
  if (diag) {
#pragma unroll
    for (int a = 0; a < D; ++a) q += d[a] * (C[a * D + a] * d[a]);
  } else {
#pragma unroll
    for (int a = 0; a < D; ++a) {
      double t = 0.0;
#pragma unroll
      for (int b = 0; b < D; ++b) t += C[a * D + b] * d[b];
      q += d[a] * t;
    }
  }
  return q;
}

// ---------------------------------------------------------------------------
// block-level small dense algebra in LDS (row-major, no pivoting: S, S - c M are SPD)
// ---------------------------------------------------------------------------
// Sum of log|pivot| in pivot order.  pv null: each log in its pivot step (one wave-wide fp64 log per
// pivot on the serial chain).  pv (N doubles of LDS scratch, written at pv[p] by lane 0 during the
// elimination): the N logs at once, one per lane, then the same sequential sum - identical value.
template <int N>
__device__ __forceinline__ double pivot_logsum(double* pv) {
  const int t = threadIdx.x, nt = blockDim.x;
  for (int r = t; r < N; r += nt) pv[r] = log(fabs(pv[r]));
  __syncthreads();
  double la = 0.0;
#pragma unroll
  for (int p = 0; p < N; ++p) la += pv[p];
  return la;
}

// Gauss-Jordan on aug [N][2N] = [S | I] -> [I | S^{-1}]; returns log|det S| and its sign.
// Eliminations run column per lane over all N rows (rows unrolled): each lane's loads of its column
// are independent of its stores, so they issue together instead of one LDS round trip per element
// (a flattened row x column loop with a runtime stride serialised them).  Every element gets the
// same expression as before, a - f * b with the row's factor and the pivot row's entry.
template <int N>
__device__ __forceinline__ void block_gauss_jordan(double* aug, double* fac, double* logabs, int* sign,
                                                   double* pv = nullptr) {
  const int t = threadIdx.x, nt = blockDim.x;
  constexpr int w = 2 * N;
  double la = 0.0;
  int sg = 1;
  for (int p = 0; p < N; ++p) {
    const double piv = aug[p * w + p];
    if (pv) {
      if (t == 0) pv[p] = piv;
    } else {
      la += log(fabs(piv));
    }
    if (piv < 0.0) sg = -sg;
    if (piv == 0.0) sg = 0;
    for (int r = t; r < N; r += nt) fac[r] = aug[r * w + p];
    __syncthreads();
    // the lane that scales column c of the pivot row is the lane that eliminates column c: no
    // barrier between the two (fac is read-only until the next pivot)
    for (int c = t; c < w; c += nt) {
      const double bp = aug[p * w + c] / piv;
      aug[p * w + c] = bp;
#pragma unroll
      for (int r = 0; r < N; ++r)
        if (r != p) aug[r * w + c] = aug[r * w + c] - fac[r] * bp;
    }
    __syncthreads();
  }
  *logabs = pv ? pivot_logsum<N>(pv) : la;
  *sign = sg;
}

// LU elimination (no pivoting) of T [N][N] in place; log|det| and sign.  Trailing updates column
// per lane over the rows below the pivot (unrolled, predicated), as in block_gauss_jordan.
template <int N>
__device__ __forceinline__ void block_logdet(double* T, double* fac, double* logabs, int* sign, double* pv = nullptr) {
  const int t = threadIdx.x, nt = blockDim.x;
  double la = 0.0;
  int sg = 1;
  for (int p = 0; p < N; ++p) {
    const double piv = T[p * N + p];
    if (pv) {
      if (t == 0) pv[p] = piv;
    } else {
      la += log(fabs(piv));
    }
    if (piv < 0.0) sg = -sg;
    if (piv == 0.0) sg = 0;
    for (int r = p + 1 + t; r < N; r += nt) fac[r] = T[r * N + p] / piv;
    __syncthreads();
    for (int c = p + 1 + t; c < N; c += nt) {
      const double bp = T[p * N + c];
#pragma unroll
      for (int r = 0; r < N; ++r)
        if (r > p) T[r * N + c] = T[r * N + c] - fac[r] * bp;
    }
    __syncthreads();
  }
  *logabs = pv ? pivot_logsum<N>(pv) : la;
  *sign = sg;
}

// log|det(I + dlam A)| = log|det(S - dlam/2 M)| - log|det S|, with the reference's
// +1e-12 I retry (ledh.py:174-179) when that determinant is not positive.
// S_ld/S_sg: log|det S| and sign; M, R: LDS matrices; T, fac scratch.
template <int NX, int NZ>
__device__ __forceinline__ double flow_logdet(const double* M, const double* R, double lam, double dlam, double S_ld,
                                              int S_sg, double* T, double* fac, double* pv = nullptr) {
  const int t = threadIdx.x, nt = blockDim.x;
  const double c1 = lam - 0.5 * dlam;
  for (int q = t; q < NZ * NZ; q += nt) T[q] = c1 * M[q] + R[q];
  __syncthreads();
  double ld;
  int sg;
  block_logdet<NZ>(T, fac, &ld, &sg, pv);
  if (sg * S_sg > 0) return ld - S_ld;
  const double eps = 1e-12;
  const double c2 = lam - dlam / (2.0 * (1.0 + eps));
  for (int q = t; q < NZ * NZ; q += nt) T[q] = c2 * M[q] + R[q];
  __syncthreads();
  block_logdet<NZ>(T, fac, &ld, &sg, pv);
  return (double)NX * log1p(eps) + ld - S_ld;
}

// ---------------------------------------------------------------------------
// k_setup: the shared-path table, one workgroup per lambda step j
// ---------------------------------------------------------------------------
template <int NX, int NZ>
struct SetupSmem {
  static constexpr int P = 0;                 // NX*NX
  static constexpr int H = P + NX * NX;       // NZ*NX
  static constexpr int K = H + NZ * NX;       // NX*NZ
  static constexpr int M = K + NX * NZ;       // NZ*NZ
  static constexpr int R = M + NZ * NZ;       // NZ*NZ
  static constexpr int AUG = R + NZ * NZ;     // NZ*2NZ
  static constexpr int T = AUG + 2 * NZ * NZ; // NZ*NZ
  static constexpr int GM = T + NZ * NZ;      // NX*NZ
  static constexpr int RV = GM + NX * NZ;     // NZ   R^{-1}(z - e)
  static constexpr int CV = RV + NZ;          // NX   c
  static constexpr int HC = CV + NX;          // NZ
  static constexpr int AC = HC + NZ;          // NX
  static constexpr int FAC = AC + NX;         // NZ
  static constexpr int SIZE = FAC + NZ;
};

constexpr int SB = 256;  // setup / compose workgroup
template <int NX, int NZ>
__global__ void __launch_bounds__(SB) k_setup(FlowParams p, double* table) {
  using L = Lay<NX, NZ>;
  using T = TLay<NX, NZ>;
  using SM = SetupSmem<NX, NZ>;
  __shared__ double sm[SM::SIZE];
  const int t = threadIdx.x, j = blockIdx.x;
  const int64_t step = blockIdx.y;  // batched over time steps (pf_ledh_run): P_k, z_k, table_k
  const double* Pk = p.Pk + step * p.pk_stride;
  const double* zk = p.z + step * p.z_stride;
  table += step * p.table_stride;
  double* diagS = gridDim.y == 1 ? p.diagS : nullptr;
  const double* __restrict__ Pm = p.Pm;
  for (int q = t; q < NX * NX; q += SB) sm[SM::P + q] = Pk[q];
  for (int q = t; q < NZ * NX; q += SB) sm[SM::H + q] = Pm[L::H + q];
  for (int q = t; q < NZ * NZ; q += SB) sm[SM::R + q] = Pm[L::R + q];
  __syncthreads();
  // K = P H^T
  for (int q = t; q < NX * NZ; q += SB) {
    const int d = q / NZ, k = q - d * NZ;
    double acc = 0.0;
    for (int e = 0; e < NX; ++e) acc += sm[SM::P + d * NX + e] * sm[SM::H + k * NX + e];
    sm[SM::K + q] = acc;
  }
  // r = R^{-1} (z - e), e = h(eta) - H eta = c for a linear h
  for (int k = t; k < NZ; k += SB) {
    double acc = 0.0;
    for (int l = 0; l < NZ; ++l) acc += Pm[L::RI + k * NZ + l] * (zk[l] - Pm[L::C + l]);
    sm[SM::RV + k] = acc;
  }
  __syncthreads();
  // M = H K ; c = K r
  for (int q = t; q < NZ * NZ; q += SB) {
    const int k = q / NZ, l = q - k * NZ;
    double acc = 0.0;
    for (int d = 0; d < NX; ++d) acc += sm[SM::H + k * NX + d] * sm[SM::K + d * NZ + l];
    sm[SM::M + q] = acc;
  }
  for (int d = t; d < NX; d += SB) {
    double acc = 0.0;
    for (int k = 0; k < NZ; ++k) acc += sm[SM::K + d * NZ + k] * sm[SM::RV + k];
    sm[SM::CV + d] = acc;
  }
  __syncthreads();
  for (int k = t; k < NZ; k += SB) {
    double acc = 0.0;
    for (int d = 0; d < NX; ++d) acc += sm[SM::H + k * NX + d] * sm[SM::CV + d];
    sm[SM::HC + k] = acc;
  }
  const double lam = p.lams[j];
  // S = lam M + R -> [S | I]
  for (int q = t; q < NZ * 2 * NZ; q += SB) {
    const int r = q / (2 * NZ), c = q - r * 2 * NZ;
    sm[SM::AUG + q] = c < NZ ? lam * sm[SM::M + r * NZ + c] + sm[SM::R + r * NZ + c] : (c - NZ == r ? 1.0 : 0.0);
  }
  __syncthreads();
  if (diagS)
    for (int q = t; q < NZ * NZ; q += SB) diagS[(int64_t)j * NZ * NZ + q] = sm[SM::AUG + (q / NZ) * 2 * NZ + q % NZ];
  __syncthreads();
  double S_ld;
  int S_sg;
  block_gauss_jordan<NZ>(sm + SM::AUG, sm + SM::FAC, &S_ld, &S_sg);
  const double ld = flow_logdet<NX, NZ>(sm + SM::M, sm + SM::R, lam, p.dlam, S_ld, S_sg, sm + SM::T, sm + SM::FAC);
  // Gm = -1/2 K S^{-1}
  for (int q = t; q < NX * NZ; q += SB) {
    const int d = q / NZ, l = q - d * NZ;
    double acc = 0.0;
    for (int k = 0; k < NZ; ++k) acc += sm[SM::K + d * NZ + k] * sm[SM::AUG + k * 2 * NZ + NZ + l];
    sm[SM::GM + q] = -0.5 * acc;
  }
  __syncthreads();
  double* tj = table + T::HEAD + (int64_t)j * T::PJ;
  for (int d = t; d < NX; d += SB) {
    double acc = 0.0;
    for (int l = 0; l < NZ; ++l) acc += sm[SM::GM + d * NZ + l] * sm[SM::HC + l];
    sm[SM::AC + d] = acc;
    tj[T::AC + d] = acc;
  }
  for (int q = t; q < NX * NZ; q += SB) tj[T::GM + q] = sm[SM::GM + q];
  __syncthreads();
  for (int q = t; q < NZ * NZ; q += SB) {
    const int k = q / NZ, l = q - k * NZ;
    double acc = 0.0;
    for (int d = 0; d < NX; ++d) acc += sm[SM::H + k * NX + d] * sm[SM::GM + d * NZ + l];
    tj[T::HGM + q] = acc;
  }
  for (int k = t; k < NZ; k += SB) {
    double acc = 0.0;
    for (int d = 0; d < NX; ++d) acc += sm[SM::H + k * NX + d] * sm[SM::AC + d];
    tj[T::HAC + k] = acc;
  }
  if (t == 0) tj[T::LD] = ld;
  if (j == 0) {
    for (int d = t; d < NX; d += SB) table[T::Cv + d] = sm[SM::CV + d];
    for (int k = t; k < NZ; k += SB) table[T::HC + k] = sm[SM::HC + k];
  }
}

// ---------------------------------------------------------------------------
// k_compose: with a linear h the flow ODE d eta / d lambda = A(lambda) eta + b(lambda; eta0)
// has particle-independent coefficients, so lambda-stepping it (ledh.py:136-171) is an
// affine map of eta0.  In observation space (y = H eta, y0 = H eta0), with per-step
//   Hw_j = Hc + lam_j HAc_j + HGm_j y0,   s_j = y_j + y0 + 2 lam_j Hw_j,
//   y_{j+1} = y_j + dlam (Hc + lam_j HAc_j + HGm_j s_j),
//   eta_{j+1} = eta_j + dlam (c + lam_j Ac_j + Gm_j s_j),
// every s_j = a_j + B_j y0 and y_j = p_j + Q_j y0 with shared a_j, B_j, p_j, Q_j, hence
//   eta_L = eta0 + d0 + D y0,   y_L = pL + QL y0.
// One workgroup composes the L steps (NZ^3 + NX NZ^2 per step).
// ---------------------------------------------------------------------------
template <int NX, int NZ>
__global__ void __launch_bounds__(SB) k_compose(double* table, const double* lams, int L, double dlam,
                                                int64_t table_stride) {
  using T = TLay<NX, NZ>;
  table += (int64_t)blockIdx.x * table_stride;  // batched over time steps
  __shared__ double Qm[NZ * NZ], B[NZ * NZ], D[NX * NZ], pv[NZ], a[NZ], d0[NX], hd[T::HEAD];
  extern __shared__ double tall[];  // [L][PJ]: the whole per-lambda table, staged once
  const int t = threadIdx.x;
  double* af = table + T::aff(L);
  for (int q = t; q < NZ * NZ; q += SB) Qm[q] = (q / NZ == q % NZ) ? 1.0 : 0.0;
  for (int q = t; q < NX * NZ; q += SB) D[q] = 0.0;
  for (int k = t; k < NZ; k += SB) pv[k] = 0.0;
  for (int d = t; d < NX; d += SB) d0[d] = 0.0;
  for (int q = t; q < T::HEAD; q += SB) hd[q] = table[q];
  for (int q = t; q < L * T::PJ; q += SB) tall[q] = table[T::HEAD + q];
  double theta = 0.0;
  __syncthreads();
  for (int j = 0; j < L; ++j) {
    const double lam = lams[j];
    const double* tjs = tall + (int64_t)j * T::PJ;
    // a = p + 2 lam hw_a ; B = Q + I + 2 lam HGm
    for (int k = t; k < NZ; k += SB) a[k] = pv[k] + 2.0 * lam * (hd[T::HC + k] + lam * tjs[T::HAC + k]);
    for (int q = t; q < NZ * NZ; q += SB)
      B[q] = (Qm[q] + ((q / NZ == q % NZ) ? 1.0 : 0.0)) + 2.0 * lam * tjs[T::HGM + q];
    __syncthreads();
    // p += dlam (hw_a + HGm a) ; Q += dlam HGm B ; d0 += dlam (c + lam Ac + Gm a) ; D += dlam Gm B
    for (int k = t; k < NZ; k += SB) {
      double acc = hd[T::HC + k] + lam * tjs[T::HAC + k];
      for (int l = 0; l < NZ; ++l) acc += tjs[T::HGM + k * NZ + l] * a[l];
      pv[k] += dlam * acc;
    }
    for (int q = t; q < NZ * NZ; q += SB) {
      const int k = q / NZ, m = q - k * NZ;
      double acc = 0.0;
      for (int l = 0; l < NZ; ++l) acc += tjs[T::HGM + k * NZ + l] * B[l * NZ + m];
      Qm[q] += dlam * acc;
    }
    for (int d = t; d < NX; d += SB) {
      double acc = hd[T::Cv + d] + lam * tjs[T::AC + d];
      for (int l = 0; l < NZ; ++l) acc += tjs[T::GM + d * NZ + l] * a[l];
      d0[d] += dlam * acc;
    }
    for (int q = t; q < NX * NZ; q += SB) {
      const int d = q / NZ, m = q - d * NZ;
      double acc = 0.0;
      for (int l = 0; l < NZ; ++l) acc += tjs[T::GM + d * NZ + l] * B[l * NZ + m];
      D[q] += dlam * acc;
    }
    theta += tjs[T::LD];
    __syncthreads();
  }
  for (int d = t; d < NX; d += SB) af[T::D0 + d] = d0[d];
  for (int q = t; q < NX * NZ; q += SB) af[T::DM + q] = D[q];
  for (int k = t; k < NZ; k += SB) af[T::PL + k] = pv[k];
  for (int q = t; q < NZ * NZ; q += SB) af[T::QL + q] = Qm[q];
  if (t == 0) af[T::TH] = theta;
}

// ---------------------------------------------------------------------------
// k_flow_affine: GL lanes per particle (PER = NX / GL components each), linear h
// ---------------------------------------------------------------------------
template <int NX>
struct Grp {
  // lanes per particle (8 for L96 d = 40 was tried: inside k_ledh_fused it needs ~540 registers
  // against the 256 of two waves per SIMD and spilled ~290 VGPRs to scratch)
  static constexpr int GL = NX >= 16 ? 4 : 1;
  static constexpr int PER = (NX + GL - 1) / GL;
};

// acc[j] += sum_e C[a_j][e] vec_e over the group-distributed vector (e <= a_j if lower),
// streaming the components through lane shuffles instead of materialising the vector
template <int NX>
__device__ __forceinline__ void group_rows(const double* loc, const double* __restrict__ C, int q, int base,
                                           double* acc, bool lower) {
  constexpr int GL = Grp<NX>::GL, PER = Grp<NX>::PER;
#pragma unroll
  for (int r = 0; r < GL; ++r) {
#pragma unroll
    for (int jj = 0; jj < PER; ++jj) {
      const double val = (GL == 1) ? loc[jj] : __shfl(loc[jj], base + r);
      const int e = r * PER + jj;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int a = q * PER + j;
        if (a < NX && e < NX && (!lower || e <= a)) acc[j] += C[a * NX + e] * val;
      }
    }
  }
}

template <int GL>
__device__ __forceinline__ double group_sum(double v) {
  if constexpr (GL == 4) return quad_sum_d(v);  // xor 1, xor 2 on the DPP network: the same sums
#pragma unroll
  for (int o = 1; o < GL; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// eta0 = g(x_{k-1}, u) + v of particle i over a lane group (ledh.py:104-115): gx = g(x) and v
// (PER components per lane, lane q of the group holds components q*PER ..)
template <int NX, int NZ, int TK>
// (src: the row of x_in the particle in slot i starts from - i itself, or its resampling ancestor
// when the previous step's resample is applied here, k_ledh_fused)
// (xpre: the lane's PER components of that row, already loaded by the caller, or null)
__device__ __forceinline__ void group_prior(const FlowParams& p, const double* __restrict__ Pm, int64_t i, int64_t src,
                                            int q, int base, double* gx, double* v, const double* xpre = nullptr,
                                            bool use_pre = false) {
  using L = Lay<NX, NZ>;
  constexpr int GL = Grp<NX>::GL, PER = Grp<NX>::PER;
  // the process noise's normals depend on (particle, epoch) only: drawn first, so the Philox
  // arithmetic runs while the row loads are in flight
  double nrm[PER];
  if (p.noise == PF_NOISE_DEVICE) normals_range<PER>(p.seed, i * NX + q * PER, p.epoch, STREAM_PROCESS, nrm);
  // xpre (when given) always points at the caller's register array and use_pre picks its values:
  // a pointer chosen at run time between that array and null would force the array into scratch
  double x[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int a = q * PER + j;
    const double xm = (a < NX && !(xpre && use_pre)) ? p.x_in[(int64_t)a * p.Npad + src] : 0.0;
    x[j] = (xpre && use_pre) ? xpre[j] : xm;
  }
#ifdef PF_STAMPS
  asm volatile("" ::"v"(x[0]));
  LF_STAMP(6);
#endif
  // ---- g(x_{k-1}, u) ------------------------------------------------------------
  if constexpr (TK == PF_TRANS_L96) {
    static_assert(NX % GL == 0 && PER >= 2, "L96 lane groups hold >= 2 contiguous components each");
    const double F = Pm[L::EX], dt = Pm[L::EX + 1];
    const int nxt = base + (q + 1) % GL, prv = base + (q + GL - 1) % GL;
    auto rhs = [&](const double* y, double* k) {
      // neighbours across the lane boundary: y[a+1] from the next lane, y[a-1], y[a-2] from the previous
      double nx0, pv1, pv2;
      if constexpr (GL == 1) {
        nx0 = y[0];
        pv1 = y[PER - 1];
        pv2 = y[PER - 2];
      } else if constexpr (GL == 4) {  // quad rotations on the DPP network (no LDS crossbar)
        nx0 = dpp_d<DPP_QP_ROT1>(0.0, y[0]);
        pv1 = dpp_d<DPP_QP_ROT3>(0.0, y[PER - 1]);
        pv2 = dpp_d<DPP_QP_ROT3>(0.0, y[PER - 2]);
      } else {
        nx0 = __shfl(y[0], nxt);
        pv1 = __shfl(y[PER - 1], prv);
        pv2 = __shfl(y[PER - 2], prv);
      }
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const double yp1 = j + 1 < PER ? y[j + 1] : nx0;
        const double ym1 = j >= 1 ? y[j - 1] : pv1;
        const double ym2 = j >= 2 ? y[j - 2] : (j == 1 ? pv1 : pv2);
        k[j] = (yp1 - ym2) * ym1 - y[j] + F;
      }
    };
    double k[PER], acc[PER], tmp[PER];
    rhs(x, k);
#pragma unroll
    for (int j = 0; j < PER; ++j) { acc[j] = k[j]; tmp[j] = x[j] + 0.5 * dt * k[j]; }
    rhs(tmp, k);
#pragma unroll
    for (int j = 0; j < PER; ++j) { acc[j] += 2.0 * k[j]; tmp[j] = x[j] + 0.5 * dt * k[j]; }
    rhs(tmp, k);
#pragma unroll
    for (int j = 0; j < PER; ++j) { acc[j] += 2.0 * k[j]; tmp[j] = x[j] + dt * k[j]; }
    rhs(tmp, k);
    const double h6 = dt / 6.0;
#pragma unroll
    for (int j = 0; j < PER; ++j) gx[j] = x[j] + h6 * (acc[j] + k[j]);
#ifdef PF_STAMPS
    asm volatile("" ::"v"(gx[PER - 1]));
    LF_STAMP(7);
#endif
  } else {
#pragma unroll
    for (int j = 0; j < PER; ++j) gx[j] = 0.0;
    group_rows<NX>(x, Pm + L::A, q, base, gx, false);
  }
  if (p.u) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int a = q * PER + j;
      if (a < NX) gx[j] += p.u[a];
    }
  }
  // ---- process noise v ------------------------------------------------------------
  if (p.noise == PF_NOISE_HOST) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int a = q * PER + j;
      v[j] = a < NX ? p.v_host[i * NX + a] : 0.0;
    }
  } else if (p.noise == PF_NOISE_DEVICE) {
    const double* n = nrm;
    if (p.q_diag) {
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int a = q * PER + j;
        v[j] = a < NX ? Pm[L::LQ + a * NX + a] * n[j] : 0.0;
      }
    } else {
#pragma unroll
      for (int j = 0; j < PER; ++j) v[j] = 0.0;
      group_rows<NX>(n, Pm + L::LQ, q, base, v, true);
    }
  } else {
#pragma unroll
    for (int j = 0; j < PER; ++j) v[j] = 0.0;
  }
}

// log N(eta; g(x), Q) - log N(eta0; g(x), Q) up to the cancelling constant (ledh.py:186-190),
// dd = eta - g(x), v = eta0 - g(x); summed over the lane group
template <int NX, int NZ>
__device__ __forceinline__ double group_trans_part(const FlowParams& p, const double* __restrict__ Pm, int q, int base,
                                                   const double* dd, const double* v) {
  using L = Lay<NX, NZ>;
  constexpr int GL = Grp<NX>::GL, PER = Grp<NX>::PER;
  double part = 0.0;
  if (p.q_diag) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int a = q * PER + j;
      if (a < NX) {
        const double qi = Pm[L::QI + a * NX + a];
        part += (-0.5 * (dd[j] * (qi * dd[j]))) - (-0.5 * (v[j] * (qi * v[j])));
      }
    }
  } else {
    double ta[PER], tb[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) ta[j] = tb[j] = 0.0;
    group_rows<NX>(dd, Pm + L::QI, q, base, ta, false);
    group_rows<NX>(v, Pm + L::QI, q, base, tb, false);
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if (q * PER + j < NX) part += (-0.5 * (dd[j] * ta[j])) - (-0.5 * (v[j] * tb[j]));
  }
  return group_sum<GL>(part);
}

// write-through (agent-coherent) fp64 store / load: data handed between workgroups of one launch
// that may sit on different XCDs (each with its own L2), as in k_resident
__device__ __forceinline__ void wt_store(double* p, double v) {
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double wt_load(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// The affine flow of particle i by its lane group (lane q of GL): eta_L -> eta[PER] (this lane's
// components q*PER ..), returns the unnormalised log weight (valid in every lane of the group);
// w_i = w_in[i], loaded by the caller ahead of the chain.
// Pm: the parameter block (Lay), af: the composed flow (TLay::aff) - p.Pm / p.table in HBM, or
// copies staged in LDS (k_ledh_fused).
// The part after the prior (gx = g(x), v its process noise): split from flow_affine_particle so that
// k_ledh_fused can run the prior while its LDS staging loads are in flight.
template <int NX, int NZ, int TK>
__device__ __forceinline__ double flow_affine_post(const FlowParams& p, const double* __restrict__ Pm,
                                                  const double* __restrict__ af, int q, int base, const double* gx,
                                                  const double* v, double* eta, double w_i,
                                                  const double* zz = nullptr) {
  using L = Lay<NX, NZ>;
  using T = TLay<NX, NZ>;
  constexpr int GL = Grp<NX>::GL, PER = Grp<NX>::PER;
#ifdef PF_STAMPS
  asm volatile("" ::"v"(v[PER - 1]), "v"(gx[PER - 1]));
  LF_STAMP(8);
#endif
  // ---- eta0, y0 = H eta0 (group all-reduce), the composed flow ----------------------
  double e0[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) e0[j] = gx[j] + v[j];
  double y0[NZ];
#pragma unroll
  for (int k = 0; k < NZ; ++k) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int a = q * PER + j;
      if (a < NX) acc += Pm[L::H + k * NX + a] * e0[j];
    }
    y0[k] = group_sum<GL>(acc);
  }
#ifdef PF_STAMPS
  asm volatile("" ::"v"(y0[NZ - 1]));
  LF_STAMP(9);
#endif
  double dd[PER];  // eta - g(x) = v + delta
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int a = q * PER + j;
    if (a < NX) {
      double acc = af[T::D0 + a];
#pragma unroll
      for (int k = 0; k < NZ; ++k) acc += af[T::DM + a * NZ + k] * y0[k];
      eta[j] = e0[j] + acc;
      dd[j] = v[j] + acc;
    } else {
      eta[j] = 0.0;
      dd[j] = 0.0;
    }
  }
  // ---- log weight (ledh.py:186-190) -----------------------------------------------
#ifdef PF_STAMPS
  asm volatile("" ::"v"(dd[PER - 1]));
  LF_STAMP(10);
#endif
  const double part = group_trans_part<NX, NZ>(p, Pm, q, base, dd, v);
  const double* __restrict__ z = zz ? zz : p.z;
  double like;
  if (GL > 1 && p.r_diag) {
    // lane q of the group takes the observation components k = GL j + q: its share of the residual
    // z - h(eta_L) and of the diagonal quadratic form, then the group sum (a quarter of the
    // residual's QL y0 products per lane instead of all of them)
    double lq = 0.0;
#pragma unroll
    for (int j = 0; j < (NZ + GL - 1) / GL; ++j) {
      const int k = GL * j + q;
      const int kc = k < NZ ? k : NZ - 1;
      double yl = af[T::PL + kc];
#pragma unroll
      for (int l = 0; l < NZ; ++l) yl += af[T::QL + kc * NZ + l] * y0[l];
      const double e = z[kc] - (yl + Pm[L::C + kc]);
      const double v = e * (Pm[L::RI + kc * NZ + kc] * e);
      lq += k < NZ ? v : 0.0;
    }
    like = group_sum<GL>(lq);
  } else {
    double ez[NZ];
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
      double yl = af[T::PL + k];
#pragma unroll
      for (int l = 0; l < NZ; ++l) yl += af[T::QL + k * NZ + l] * y0[l];
      ez[k] = z[k] - (yl + Pm[L::C + k]);
    }
    like = quad_form<NZ>(ez, Pm + L::RI, p.r_diag != 0);
  }
  return (log(w_i + 1e-300) + af[T::TH]) + (part + (-0.5 * like));
}

template <int NX, int NZ, int TK>
__device__ __forceinline__ double flow_affine_particle(const FlowParams& p, const double* __restrict__ Pm,
                                                      const double* __restrict__ af, int64_t i, int64_t src, int q,
                                                      int base, double* eta, double w_i) {
  constexpr int PER = Grp<NX>::PER;
  double gx[PER], v[PER];
  group_prior<NX, NZ, TK>(p, Pm, i, src, q, base, gx, v);
  return flow_affine_post<NX, NZ, TK>(p, Pm, af, q, base, gx, v, eta, w_i);
}

template <int NX, int NZ, int TK>
__global__ void __launch_bounds__(TB) k_flow_affine(FlowParams p) {
  constexpr int GL = Grp<NX>::GL;
  const int64_t tid = (int64_t)blockIdx.x * TB + threadIdx.x;
  const int64_t i = tid / GL;
  if (i >= p.N) return;  // whole groups leave together
  const int q = (int)(tid % GL);
  const int base = (threadIdx.x & 63) - q;
  constexpr int PER = Grp<NX>::PER;
  double eta[PER];
  const double l =
      flow_affine_particle<NX, NZ, TK>(p, p.Pm, p.table + TLay<NX, NZ>::aff(p.L), i, i, q, base, eta, p.w_in[i]);
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (q * PER + j < NX) p.x_out[(int64_t)(q * PER + j) * p.Npad + i] = eta[j];
  if (q == 0) p.lw[i] = l;
}

// ---------------------------------------------------------------------------
// k_flow_wave: one 64-lane workgroup per particle, any h with a Jacobian
// ---------------------------------------------------------------------------
template <int NX, int NZ>
struct WaveSmem {
  static constexpr int P = 0;                 // NX*NX
  static constexpr int R = P + NX * NX;       // NZ*NZ
  static constexpr int XP = R + NZ * NZ;      // NX  x_{k-1}
  static constexpr int GX = XP + NX;          // NX  g(x)
  static constexpr int V = GX + NX;           // NX  v (noise), later scratch
  static constexpr int E0 = V + NX;           // NX  eta0
  static constexpr int ET = E0 + NX;          // NX  eta
  static constexpr int T1 = ET + NX;          // NX
  static constexpr int T2 = T1 + NX;          // NX
  static constexpr int CV = T2 + NX;          // NX  c
  static constexpr int H = CV + NX;           // NZ*NX
  static constexpr int K = H + NZ * NX;       // NX*NZ
  static constexpr int M = K + NX * NZ;       // NZ*NZ
  static constexpr int AUG = M + NZ * NZ;     // NZ*2NZ
  static constexpr int TT = AUG + 2 * NZ * NZ;// NZ*NZ
  static constexpr int GM = TT + NZ * NZ;     // NX*NZ
  static constexpr int HV = GM + NX * NZ;     // NZ  h(eta)
  static constexpr int ZE = HV + NZ;          // NZ  e / scratch
  static constexpr int ZT = ZE + NZ;          // NZ  scratch
  static constexpr int FAC = ZT + NZ;         // NZ
  static constexpr int RED = FAC + NZ;        // 64
  static constexpr int SIZE = RED + 64;
};

template <int NX, int NZ, int TK>
__device__ __forceinline__ void g_block(const double* x, double* out, double* tmp, double* kk, const double* __restrict__ Pm,
                                        const double* u) {
  using L = Lay<NX, NZ>;
  const int t = threadIdx.x;
  if constexpr (TK == PF_TRANS_LINEAR) {
    for (int d = t; d < NX; d += blockDim.x) {
      double acc = 0.0;
      for (int e = 0; e < NX; ++e) acc += Pm[L::A + d * NX + e] * x[e];
      out[d] = u ? acc + u[d] : acc;
    }
    __syncthreads();
  } else {
    const double F = Pm[L::EX], dt = Pm[L::EX + 1];
    // out accumulates k1 + 2k2 + 2k3; kk holds the current stage slope
    for (int a = t; a < NX; a += blockDim.x) { kk[a] = l96_rhs_at<NX>(x, a, F); out[a] = kk[a]; tmp[a] = x[a] + 0.5 * dt * kk[a]; }
    __syncthreads();
    for (int a = t; a < NX; a += blockDim.x) kk[a] = l96_rhs_at<NX>(tmp, a, F);
    __syncthreads();
    for (int a = t; a < NX; a += blockDim.x) { out[a] += 2.0 * kk[a]; tmp[a] = x[a] + 0.5 * dt * kk[a]; }
    __syncthreads();
    for (int a = t; a < NX; a += blockDim.x) kk[a] = l96_rhs_at<NX>(tmp, a, F);
    __syncthreads();
    for (int a = t; a < NX; a += blockDim.x) { out[a] += 2.0 * kk[a]; tmp[a] = x[a] + dt * kk[a]; }
    __syncthreads();
    for (int a = t; a < NX; a += blockDim.x) kk[a] = l96_rhs_at<NX>(tmp, a, F);
    __syncthreads();
    const double h6 = dt / 6.0;
    for (int a = t; a < NX; a += blockDim.x) {
      const double r = x[a] + h6 * (out[a] + kk[a]);
      out[a] = u ? r + u[a] : r;
    }
    __syncthreads();
  }
}

// H = dh/deta and h(eta) at eta (LDS), lanes over entries
template <int NX, int NZ, int OK>
__device__ __forceinline__ void obs_jac_block(const double* eta, double* H, double* hv, const double* __restrict__ Pm) {
  using L = Lay<NX, NZ>;
  const int t = threadIdx.x;
  if constexpr (OK == PF_OBS_LINEAR) {
    for (int q = t; q < NZ * NX; q += blockDim.x) H[q] = Pm[L::H + q];
    for (int k = t; k < NZ; k += blockDim.x) {
      double acc = 0.0;
      for (int e = 0; e < NX; ++e) acc += Pm[L::H + k * NX + e] * eta[e];
      hv[k] = acc + Pm[L::C + k];
    }
  } else if constexpr (OK == PF_OBS_EXP_HALF) {
    static_assert(NX == NZ, "EXP_HALF observes every component");
    for (int q = t; q < NZ * NX; q += blockDim.x) {
      const int k = q / NX, e = q - k * NX;
      H[q] = (k == e) ? 0.5 * Pm[L::C + k] * exp(0.5 * eta[k]) : 0.0;
    }
    for (int k = t; k < NZ; k += blockDim.x) hv[k] = Pm[L::C + k] * exp(0.5 * eta[k]);
  } else {  // ACOUSTIC: z_s = sum_c psi / (|p_c - s|^2 + d0)
    static_assert(NX % 4 == 0, "acoustic state is 4 per target");
    const double psi = Pm[L::AC], d0 = Pm[L::AC + 1];
    for (int k = t; k < NZ; k += blockDim.x) {
      const double sx = Pm[L::AC + 2 + k], sy = Pm[L::AC + 2 + NZ + k];
      double acc = 0.0;
      for (int c = 0; c < NX / 4; ++c) {
        const double dx = eta[4 * c] - sx, dy = eta[4 * c + 1] - sy;
        const double den = (dx * dx + dy * dy) + d0;
        acc += psi / den;
        const double den2 = den * den;
        H[k * NX + 4 * c] = (-2.0 * psi * dx) / den2;
        H[k * NX + 4 * c + 1] = (-2.0 * psi * dy) / den2;
        H[k * NX + 4 * c + 2] = 0.0;
        H[k * NX + 4 * c + 3] = 0.0;
      }
      hv[k] = acc;
    }
  }
  __syncthreads();
}

// Columns of the observation Jacobian that are zero by the model's form: the acoustic h depends on
// the target positions only, so its velocity columns (4c + 2, 4c + 3) are exact zeros.  Dot products
// over H skip them at compile time: a finite x times 0.0 adds a signed zero to a sum that never is
// -0.0 here, so the sums are bitwise those of the dense loops.  That equality assumes finite operands:
// a NaN / Inf in a skipped velocity entry no longer poisons these sums (NaN * 0 would).  A diverged
// particle still shows up as NaN: the non-finite entry stays in its own flow components (eta += dlam
// (A eta + b) keeps it), and the transition density of its weight reads every component.
template <int OK>
__device__ __forceinline__ constexpr bool h_zero_col(int e) {
  return OK == PF_OBS_ACOUSTIC && (e & 2) != 0;
}

// out = Gm (H v): zt scratch (NZ)
template <int NX, int NZ, int OK = -1>
__device__ __forceinline__ void apply_A(const double* H, const double* Gm, const double* v, double* zt, double* out) {
  const int t = threadIdx.x;
  for (int k = t; k < NZ; k += blockDim.x) {
    double acc = 0.0;
#pragma unroll
    for (int e = 0; e < NX; ++e)
      if (!h_zero_col<OK>(e)) acc += H[k * NX + e] * v[e];
    zt[k] = acc;
  }
  __syncthreads();
  for (int d = t; d < NX; d += blockDim.x) {
    double acc = 0.0;
    for (int l = 0; l < NZ; ++l) acc += Gm[d * NZ + l] * zt[l];
    out[d] = acc;
  }
  __syncthreads();
}

// sum over the block of one value per thread (block = 64 lanes = one wave)
__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(64) k_flow_wave(FlowParams p) {
  static_assert(NX <= 64 && NZ <= 64, "one lane per state / observation component");
  using L = Lay<NX, NZ>;
  using SM = WaveSmem<NX, NZ>;
  __shared__ double sm[SM::SIZE];
  const int t = threadIdx.x;
  const double* __restrict__ Pm = p.Pm;
  for (int q = t; q < NX * NX; q += 64) sm[SM::P + q] = p.Pk[q];
  for (int q = t; q < NZ * NZ; q += 64) sm[SM::R + q] = Pm[L::R + q];
  __syncthreads();
  double* H = sm + SM::H;
  double* K = sm + SM::K;
  double* Mm = sm + SM::M;
  double* aug = sm + SM::AUG;
  double* Gm = sm + SM::GM;
  double* eta = sm + SM::ET;
  double* eta0 = sm + SM::E0;
  double* t1 = sm + SM::T1;
  double* t2 = sm + SM::T2;
  double* cv = sm + SM::CV;
  double* zt = sm + SM::ZT;
  const double dlam = p.dlam;
  for (int64_t i = blockIdx.x; i < p.N; i += gridDim.x) {
    // ---- eta0 = g(x_{k-1}, u) + v -------------------------------------------
    for (int d = t; d < NX; d += 64) sm[SM::XP + d] = p.x_in[(int64_t)d * p.Npad + i];
    __syncthreads();
    g_block<NX, NZ, TK>(sm + SM::XP, sm + SM::GX, t1, t2, Pm, p.u);
    for (int d = t; d < NX; d += 64) {
      double vd = 0.0;
      if (p.noise == PF_NOISE_HOST) {
        vd = p.v_host[i * NX + d];
      } else if (p.noise == PF_NOISE_DEVICE) {
        const int64_t f = i * NX + d;
        t1[d] = pick4(normal4_bm24d(p.seed, (uint32_t)(f >> 2), 0u, p.epoch, STREAM_PROCESS), (int)(f & 3));
      }
      sm[SM::V + d] = vd;
    }
    __syncthreads();
    if (p.noise == PF_NOISE_DEVICE) {
      for (int d = t; d < NX; d += 64) {
        double acc = 0.0;
        for (int e = 0; e <= d; ++e) acc += Pm[L::LQ + d * NX + e] * t1[e];
        sm[SM::V + d] = acc;
      }
      __syncthreads();
    }
    for (int d = t; d < NX; d += 64) {
      const double e0 = sm[SM::GX + d] + sm[SM::V + d];
      eta0[d] = e0;
      eta[d] = e0;
    }
    __syncthreads();
    double theta = 0.0;
    for (int j = 0; j < p.L; ++j) {
      const double lam = p.lams[j];
      // linearise at eta (ledh.py:143-145)
      obs_jac_block<NX, NZ, OK>(eta, H, sm + SM::HV, Pm);
      for (int k = t; k < NZ; k += 64) {
        double acc = 0.0;
#pragma unroll
        for (int e = 0; e < NX; ++e)
          if (!h_zero_col<OK>(e)) acc += H[k * NX + e] * eta[e];
        sm[SM::ZE + k] = sm[SM::HV + k] - acc;  // e = h(eta) - H eta
      }
      // K = P H^T
      for (int q = t; q < NX * NZ; q += 64) {
        const int d = q / NZ, k = q - d * NZ;
        double acc = 0.0;
#pragma unroll
        for (int e = 0; e < NX; ++e)
          if (!h_zero_col<OK>(e)) acc += sm[SM::P + d * NX + e] * H[k * NX + e];
        K[q] = acc;
      }
      __syncthreads();
      // M = H K, S = lam M + R -> [S | I]; r = R^{-1}(z - e) into zt
      for (int q = t; q < NZ * NZ; q += 64) {
        const int k = q / NZ, l = q - k * NZ;
        double acc = 0.0;
#pragma unroll
        for (int d = 0; d < NX; ++d)
          if (!h_zero_col<OK>(d)) acc += H[k * NX + d] * K[d * NZ + l];
        Mm[q] = acc;
        aug[k * 2 * NZ + l] = lam * acc + sm[SM::R + q];
        aug[k * 2 * NZ + NZ + l] = (k == l) ? 1.0 : 0.0;
      }
      for (int k = t; k < NZ; k += 64) {
        double acc = 0.0;
        for (int l = 0; l < NZ; ++l) acc += Pm[L::RI + k * NZ + l] * (p.z[l] - sm[SM::ZE + l]);
        zt[k] = acc;
      }
      __syncthreads();
      if (i == 0 && p.diagS)
        for (int q = t; q < NZ * NZ; q += 64) p.diagS[(int64_t)j * NZ * NZ + q] = aug[(q / NZ) * 2 * NZ + q % NZ];
      // c = K r  (= P H^T R^{-1}(z - e))
      for (int d = t; d < NX; d += 64) {
        double acc = 0.0;
        for (int k = 0; k < NZ; ++k) acc += K[d * NZ + k] * zt[k];
        cv[d] = acc;
      }
      __syncthreads();
      double S_ld;
      int S_sg;
      // zt (R^{-1}(z - e), consumed by c above) is free until apply_A: the pivots' log scratch
      block_gauss_jordan<NZ>(aug, sm + SM::FAC, &S_ld, &S_sg, zt);
      theta += flow_logdet<NX, NZ>(Mm, sm + SM::R, lam, dlam, S_ld, S_sg, sm + SM::TT, sm + SM::FAC, zt);
      // Gm = -1/2 K S^{-1}
      for (int q = t; q < NX * NZ; q += 64) {
        const int d = q / NZ, l = q - d * NZ;
        double acc = 0.0;
        for (int k = 0; k < NZ; ++k) acc += K[d * NZ + k] * aug[k * 2 * NZ + NZ + l];
        Gm[q] = -0.5 * acc;
      }
      __syncthreads();
      // b = (I + 2 lam A)[(I + lam A) c + A eta0]   (ledh.py:165)
      apply_A<NX, NZ, OK>(H, Gm, eta0, zt, t1);   // t1 = A eta0
      apply_A<NX, NZ, OK>(H, Gm, cv, zt, t2);     // t2 = A c
      for (int d = t; d < NX; d += 64) t1[d] = (cv[d] + lam * t2[d]) + t1[d];  // w
      __syncthreads();
      apply_A<NX, NZ, OK>(H, Gm, t1, zt, t2);     // t2 = A w
      for (int d = t; d < NX; d += 64) t1[d] = t1[d] + 2.0 * lam * t2[d];      // b
      __syncthreads();
      apply_A<NX, NZ, OK>(H, Gm, eta, zt, t2);    // t2 = A eta
      for (int d = t; d < NX; d += 64) eta[d] = eta[d] + dlam * (t2[d] + t1[d]);  // ledh.py:171
      __syncthreads();
    }
    // ---- weight (ledh.py:186-190) ---------------------------------------------
    obs_jac_block<NX, NZ, OK>(eta, H, sm + SM::HV, Pm);
    double part = 0.0;
    for (int d = t; d < NX; d += 64) {  // (eta - gx)^T Q^{-1} (eta - gx) - v^T Q^{-1} v
      double a = 0.0, b = 0.0;
      for (int e = 0; e < NX; ++e) {
        const double qi = Pm[L::QI + d * NX + e];
        a += qi * (eta[e] - sm[SM::GX + e]);
        b += qi * sm[SM::V + e];
      }
      part += (-0.5 * ((eta[d] - sm[SM::GX + d]) * a)) - (-0.5 * (sm[SM::V + d] * b));
    }
    for (int k = t; k < NZ; k += 64) {
      double a = 0.0;
      for (int l = 0; l < NZ; ++l) a += Pm[L::RI + k * NZ + l] * (p.z[l] - sm[SM::HV + l]);
      part += -0.5 * ((p.z[k] - sm[SM::HV + k]) * a);
    }
    const double tot = wave_sum64(part);
    if (t == 0) p.lw[i] = (log(p.w_in[i] + 1e-300) + theta) + tot;
    for (int d = t; d < NX; d += 64) p.x_out[(int64_t)d * p.Npad + i] = eta[d];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_flow_wave_lr: the per-particle flow of the acoustic h in the NR = NX / 2 dimensional space of
// the targets' positions (one 64-lane workgroup per particle, persistent over particles).
//
// The acoustic h reads the positions only, so H = H8 E with E the NR x NX position selection and
// H8 = dh/d(positions) (NZ x NR, NR = 8 for the joint 4-target model against NZ = 25 sensors).  With
// R diagonal, U = R^{-1/2} H8 and Rq the NR x NR upper-triangular factor with Rq^T Rq = U^T U (= W, the
// Gram): the Cholesky factor of W, W formed on the fp64 matrix cores; where W is not numerically
// positive definite (a pivot below 1e-12 of its diagonal) the thin Householder QR U = Q Rq over the
// wave instead (lane k holds row k; the fallback, FlowParams::lr_force bit 0 forces it in tests), and
//   H8^T S^{-1} H8 = Rq^T D^{-1} Rq,  D = I + lam Rq P_pp Rq^T   (NR x NR, symmetric, eigenvalues >= 1)
// (S = R^{1/2} (I + lam U P_pp U^T) R^{1/2}; Q^T (I + Q M Q^T)^{-1} Q = (I + M)^{-1}), so
//   A v  = -1/2 P H^T S^{-1} H v = G v_pos,  G = -1/2 P_{:,pos} Rq^T D^{-1} Rq          (NX x NR)
//   c    = P H^T R^{-1}(z - e) = P_{:,pos} H8^T R^{-1} (z - e)
//   det(I + dlam A) = det(S - dlam/2 M) / det(S) = det(I + c1 Rq P_pp Rq^T) / det(D),  c1 = lam - dlam/2
// (Sylvester; the reference's +1e-12 I retry is flow_logdet's c2 = lam - dlam / (2 (1 + eps)) form).
// Per pseudo-time step the dense algebra is NR x NR: the Gram and its Cholesky factor (or the QR:
// sensor rows mirrored in both half-waves, each half summing half of a reflector's reductions),
// M = Rq P_pp Rq^T as two fp64 MFMA products,
// and one Gauss-Jordan elimination of [D | Rq | C] in registers (column per lane, pivot columns by
// DPP row_newbcast) that gives D^{-1} Rq and both determinants; the flow update then runs in the
// position space (K = -1/2 Rq^T D^{-1} Rq, 8-vectors between lanes by readlane) - instead of
// k_flow_wave's NZ x 2NZ Gauss-Jordan through LDS.  A Woodbury form solving with W itself squares
// the condition of H8 (W spans 1e-4 .. 4e5 next to a sensor) and lost 2e-4 of the flow; the factor
// Rq does not (only Rq^T D^{-1} Rq enters the flow, D's eigenvalues are >= 1): a 40-digit
// recomputation of the MAT golden's most ill-conditioned particle (cond S = 5e6) puts this algebra at
// 2.4e-9 of the exact flow and the reference's own fp64 path at 3.1e-8 (tools/flow_accuracy.py).  The
// determinant pair comes from the one Gauss-Jordan (lr_gj_pair); when a sign there is not positive,
// separate pivoted eliminations (lr_logdet) and then the reference's +1e-12 I retry (FlowParams::
// lr_force bits 1 and 2 force those paths in tests).  The flow's
// reciprocals (Jacobian rows, reflector scales, pivots) are v_rcp_f64 + two Newton steps (within an
// ulp of the division); h and the weight terms evaluate as in k_flow_wave (identical expressions).
// Diagonal R only (the host takes k_flow_wave otherwise).
template <int NX, int NZ>
struct LrSmem {
  static constexpr int NR = NX / 2;             // position components: x, y of each target
  static constexpr int P = 0;                   // NX*NX  tracker covariance
  static constexpr int XP = P + NX * NX;        // NX  x_{k-1}
  static constexpr int GX = XP + NX;            // NX  g(x)
  static constexpr int V = GX + NX;             // NX  v
  static constexpr int E0 = V + NX;             // NX  eta0
  static constexpr int ET = E0 + NX;            // NX  eta
  static constexpr int T1 = ET + NX;            // NX
  static constexpr int T2 = T1 + NX;            // NX
  static constexpr int CV = T2 + NX;            // NX  c
  static constexpr int H8 = CV + NX;            // NZ*NR  dh/d(positions)
  static constexpr int HV = H8 + NZ * NR;       // NZ  h(eta)
  static constexpr int ZE = HV + NZ;            // NZ  e = h(eta) - H eta
  static constexpr int RU = ZE + NZ;            // NZ  R^{-1}(z - e)
  static constexpr int RQ = RU + NZ;            // NR*NR  Rq (row-major, upper triangular)
  static constexpr int R8 = RQ + NR * NR;       // NR  H8^T R^{-1}(z - e)
  static constexpr int TT = R8 + NR;            // NR*NR  Rq P_pp
  static constexpr int X = TT + NR * NR;        // NR*NR  D^{-1} Rq
  static constexpr int MC = X + NR * NR;        // NR*NR  M = Rq P_pp Rq^T, column-major
  static constexpr int KS = MC + NR * NR;       // NR*NZ  P_pp H8^T (S of particle 0, diagnostics)
  static constexpr int UT = KS + NR * NZ;       // NZ*NR  U = R^{-1/2} H8 (the Gram's operand)
  static constexpr int WC = UT + NZ * NR;       // NR*NR  W = U^T U, column-major
  static constexpr int RED = WC + NR * NR;      // 64
  static constexpr int SIZE = RED + 64;
};

// state index of position component a (x, y of target a / 2)
__device__ __forceinline__ constexpr int lr_pos(int a) { return 4 * (a >> 1) + (a & 1); }

// k_flow_wave_lr's LDS hand-offs inside the lambda loop: the workgroup is one wave, and a wave's LDS
// operations complete in issue order, so a compiler barrier orders a write before the reads that
// follow it - no s_waitcnt drain and no s_barrier between the phases
__device__ __forceinline__ void lr_wave_sync() { asm volatile("" ::: "memory"); }

// 1 / x from v_rcp_f64 and two Newton steps (within an ulp; a third of the dependent instructions of
// a correctly rounded division, which sits on the flow's serial chain)
__device__ __forceinline__ double lr_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// 1 / sqrt(x) from v_rsq_f64 and two Newton steps (for the Cholesky pivots: one short chain instead of
// a correctly rounded square root and a reciprocal)
__device__ __forceinline__ double lr_rsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  double e = fma(-x * y, y, 1.0);
  y = fma(0.5 * y, e, y);
  e = fma(-x * y, y, 1.0);
  return fma(0.5 * y, e, y);
}

// Right-looking Cholesky W = R^T R, column per lane (lane c < NR of row 0 holds column c of the trailing
// matrix; pivot columns by DPP row_newbcast): lane c ends with column c of R in rr.  ok turns false
// when a pivot is not above 1e-12 of its original diagonal dg (or is NaN).
template <int NR, int P>
__device__ __forceinline__ void lr_chol_pivot(double (&a)[NR], double (&rr)[NR], double dg, bool& ok, int c) {
  double f[NR];
#pragma unroll
  for (int r = P; r < NR; ++r) f[r] = dpp_mov_d<0x150 + P>(a[r]);
  const double d0 = dpp_mov_d<0x150 + P>(dg);
  const double d = f[P];
  ok = ok && (d > 1e-12 * d0);
  const double ri = lr_rsq(d);  // 1 / R[P][P]
  const double rpc = c >= P ? a[P] * ri : 0.0;  // R[P][c]
  rr[P] = rpc;
#pragma unroll
  for (int r = P + 1; r < NR; ++r) a[r] = a[r] - (f[r] * ri) * rpc;
  if constexpr (P + 1 < NR) lr_chol_pivot<NR, P + 1>(a, rr, dg, ok, c);
}

// out[a] = x of lane NR + a, in every lane of each 16-lane row (row 0 holds the flow update's lanes):
// DPP row_newbcast, no scalar round trip
template <int NR, int A = 0>
__device__ __forceinline__ void lr_row_gather(double x, double (&out)[NR]) {
  out[A] = dpp_mov_d<0x150 + NR + A>(x);
  if constexpr (A + 1 < NR) lr_row_gather<NR, A + 1>(x, out);
}

// sums over the lanes of the sensor rows of N values at once, level by level (each DPP move reads a
// register written several instructions earlier: no DPP hazard stalls).  NZ <= 32: the sensor rows
// are mirrored in the upper half of the wave (lane 32 + k holds row k too), so the lower 32 lanes sum
// the first ceil(N/2) values and the upper 32 the rest - half the DPP work, one level less than a wave
// sum.  Otherwise the whole wave sums every value.  Every lane ends with the N sums.
template <int NZ, int N>
__device__ __forceinline__ void lr_row_sums(double (&v)[N]) {
  constexpr bool SPLIT = NZ <= 32;
  constexpr int H = SPLIT ? (N + 1) / 2 : N;
  double w[H];
  // the upper half's values by a bit mask (a select of two array elements becomes an indexed scratch
  // load otherwise)
  const long long up = (threadIdx.x & 63) >= 32 ? -1LL : 0LL;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    if (SPLIT && H + j < N) {
      const long long a = __double_as_longlong(v[j]), b = __double_as_longlong(v[H + j]);
      w[j] = __longlong_as_double((a & ~up) | (b & up));
    } else {
      w[j] = v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < H; ++j) w[j] += dpp_mov_d<DPP_QP_1032>(w[j]);
#pragma unroll
  for (int j = 0; j < H; ++j) w[j] += dpp_mov_d<DPP_QP_2301>(w[j]);
#pragma unroll
  for (int j = 0; j < H; ++j) w[j] += dpp_mov_d<DPP_ROW_HMIRROR>(w[j]);
#pragma unroll
  for (int j = 0; j < H; ++j) w[j] += dpp_mov_d<DPP_ROW_MIRROR>(w[j]);
#pragma unroll
  for (int j = 0; j < H; ++j) w[j] += dpp_mov_d<DPP_ROW_BCAST15, 0xa>(w[j]);  // rows 0, 2 not read
  if constexpr (SPLIT) {
#pragma unroll
    for (int j = 0; j < H; ++j) {
      v[j] = readlane_d(w[j], 31);
      if (H + j < N) v[H + j] = readlane_d(w[j], 63);
    }
  } else {
#pragma unroll
    for (int j = 0; j < H; ++j) w[j] += dpp_mov_d<DPP_ROW_BCAST31, 0xc>(w[j]);
#pragma unroll
    for (int j = 0; j < H; ++j) v[j] = readlane_d(w[j], 63);
  }
}

// Householder reflector PC of the QR of U over the wave (lane k holds row k): v = x - alpha e_PC
// (x = column PC's rows >= PC, alpha = -sign(x_PC) |x|).  Every reduction of the step is issued at
// once - |x|^2 and x^T u_c of the trailing columns - since v^T v = 2 alpha (alpha - x_PC) and
// v^T u_c = x^T u_c - alpha u_{PC,c} (LAPACK's dlarfg / dlarf algebra): one wave-sum level per column.
template <int NR, int NZ, int PC>
__device__ __forceinline__ void lr_qr_col(double (&u)[NR], int t) {
  constexpr int N = NR - PC;  // |x|^2, then x^T u_c for c > PC
  const double xk = t >= PC ? u[PC] : 0.0;
  double sv[N];
  sv[0] = xk * xk;
#pragma unroll
  for (int c = PC + 1; c < NR; ++c) sv[c - PC] = xk * u[c];
  lr_row_sums<NZ, N>(sv);
  const double xp = readlane_d(u[PC], PC);
  const double alpha = xp >= 0.0 ? -sqrt(sv[0]) : sqrt(sv[0]);
  const double vk = t == PC ? xp - alpha : xk;  // the reflector v (rows >= PC)
  const double vtv = 2.0 * alpha * (alpha - xp);
  const double beta = vtv > 0.0 ? 2.0 * lr_rcp(vtv) : 0.0;  // no branch: one basic block per QR
#pragma unroll
  for (int c = PC + 1; c < NR; ++c) {
    const double sc = sv[c - PC] - alpha * readlane_d(u[c], PC);
    u[c] = u[c] - beta * vk * sc;
  }
  u[PC] = t == PC ? alpha : (t > PC ? 0.0 : u[PC]);
  if constexpr (PC + 1 < NR) lr_qr_col<NR, NZ, PC + 1>(u, t);
}

// |det| as mantissa x 2^exponent: the pivots' product renormalised after every factor (no overflow, and
// one log per determinant - or per ratio of two - instead of one per pivot)
struct DetAcc {
  double m = 1.0;
  int e = 0;
  __device__ __forceinline__ void mul(double a) {
    int k;
    m = frexp(m * a, &k);
    e += k;
  }
};
// log(|det A| / |det B|)
__device__ __forceinline__ double det_log_ratio(const DetAcc& a, const DetAcc& b) {
  return log(a.m / b.m) + (double)(a.e - b.e) * 0.69314718055994530942;
}

// Gauss-Jordan with partial pivoting on the NR x 2NR matrix [B | I] held column per lane (lane c < 2NR:
// col[r] = row r of column c): -> [I | B^{-1}] (lanes NR .. 2NR - 1), |det B|, sign.  One wave.
template <int NR>
__device__ __forceinline__ void lr_gauss_jordan(double (&col)[NR], DetAcc* det, int* sign) {
  DetAcc dacc;
  int sg = 1;
#pragma unroll
  for (int p = 0; p < NR; ++p) {
    double f[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) f[r] = readlane_d(col[r], p);  // the pivot column, in every lane
    int rp = p;
    double best = fabs(f[p]);
#pragma unroll
    for (int r = p + 1; r < NR; ++r)
      if (fabs(f[r]) > best) {
        best = fabs(f[r]);
        rp = r;
      }
    if (rp != p) sg = -sg;
#pragma unroll
    for (int r = p + 1; r < NR; ++r)
      if (r == rp) {  // swap rows p and rp (uniform branch)
        const double a = col[p], fa = f[p];
        col[p] = col[r];
        col[r] = a;
        f[p] = f[r];
        f[r] = fa;
      }
    const double piv = f[p];
    dacc.mul(fabs(piv));
    if (piv < 0.0) sg = -sg;
    if (piv == 0.0) sg = 0;
    const double bp = col[p] / piv;
    col[p] = bp;
#pragma unroll
    for (int r = 0; r < NR; ++r)
      if (r != p) col[r] = col[r] - f[r] * bp;
  }
  *det = dacc;
  *sign = sg;
}

// |det T| and its sign by LU with partial pivoting, T NR x NR column per lane (lanes c < NR)
template <int NR>
__device__ __forceinline__ void lr_logdet(double (&col)[NR], DetAcc* det, int* sign) {
  const int c = threadIdx.x & 63;
  DetAcc dacc;
  int sg = 1;
#pragma unroll
  for (int p = 0; p < NR; ++p) {
    double f[NR];
#pragma unroll
    for (int r = p; r < NR; ++r) f[r] = readlane_d(col[r], p);
    int rp = p;
    double best = fabs(f[p]);
#pragma unroll
    for (int r = p + 1; r < NR; ++r)
      if (fabs(f[r]) > best) {
        best = fabs(f[r]);
        rp = r;
      }
    if (rp != p) sg = -sg;
#pragma unroll
    for (int r = p + 1; r < NR; ++r)
      if (r == rp) {
        const double a = col[p], fa = f[p];
        col[p] = col[r];
        col[r] = a;
        f[p] = f[r];
        f[r] = fa;
      }
    const double piv = f[p];
    dacc.mul(fabs(piv));
    if (piv < 0.0) sg = -sg;
    if (piv == 0.0) sg = 0;
    if (c > p) {
      const double bp = col[p] / piv;
#pragma unroll
      for (int r = p + 1; r < NR; ++r) col[r] = col[r] - f[r] * bp;
    }
  }
  *det = dacc;
  *sign = sg;
}

// Gauss-Jordan on [D | B | C] without pivoting, column per lane: D in lanes 0..NR-1 and B in NR..2NR-1
// (row 0 of the wave), C in lanes LR_CB..LR_CB+NR-1 (row 1); D and C symmetric positive definite with
// eigenvalues >= 1, so no pivot is small.  Lanes NR..2NR-1 end with D^{-1} B, and |det D|, |det C| come
// from the pivots.  Each 16-lane row takes its pivot column with DPP row_newbcast (one v_mov_dpp per
// dword, no scalar round trip), so the two eliminations share one instruction stream: row 0
// eliminates with D's pivot column, row 1 with C's.
constexpr int LR_CB = 16;
template <int NR, int P>
__device__ __forceinline__ void lr_gj_pivot(double (&col)[NR], DetAcc& det, bool& ok) {
  double f[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) f[r] = dpp_mov_d<0x150 + P>(col[r]);  // row_newbcast: lane P of this row
  det.mul(fabs(f[P]));
  ok = ok && (f[P] > 0.0);  // not positive definite after all (NaN, ...)
  const double bp = col[P] * lr_rcp(f[P]);
  col[P] = bp;
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (r != P) col[r] = col[r] - f[r] * bp;
  if constexpr (P + 1 < NR) lr_gj_pivot<NR, P + 1>(col, det, ok);
}
template <int NR>
__device__ __forceinline__ void lr_gj_pair(double (&col)[NR], DetAcc* detD, DetAcc* detC, int* sign) {
  static_assert(2 * NR <= LR_CB, "D and B in one 16-lane row");
  DetAcc det;  // this row's pivots: D's in row 0, C's in row 1
  bool ok = true;
  lr_gj_pivot<NR, 0>(col, det, ok);
  detD->m = readlane_d(det.m, 0);
  detD->e = __builtin_amdgcn_readlane(det.e, 0);
  detC->m = readlane_d(det.m, LR_CB);
  detC->e = __builtin_amdgcn_readlane(det.e, LR_CB);
  const int okv = ok ? 1 : 0;
  *sign = (__builtin_amdgcn_readlane(okv, 0) & __builtin_amdgcn_readlane(okv, LR_CB)) ? 1 : 0;
}

template <int NX, int NZ, int TK>
__global__ void __launch_bounds__(64) k_flow_wave_lr(FlowParams p) {
  static_assert(NX % 4 == 0 && NX / 2 <= 32 && NZ <= 64, "acoustic: 4 components per target, 2NR <= 64 lanes");
  using L = Lay<NX, NZ>;
  using SM = LrSmem<NX, NZ>;
  constexpr int NR = SM::NR, NT = NX / 4;
  __shared__ double sm[SM::SIZE];
  const int t = threadIdx.x;
  const double* __restrict__ Pm = p.Pm;
  for (int q = t; q < NX * NX; q += 64) sm[SM::P + q] = p.Pk[q];
  __syncthreads();
  const double* P = sm + SM::P;
  double* eta = sm + SM::ET;
  double* eta0 = sm + SM::E0;
  double* t1 = sm + SM::T1;
  double* t2 = sm + SM::T2;
  double* H8 = sm + SM::H8;
  const double psi = Pm[L::AC], d0 = Pm[L::AC + 1];
  const double dlam = p.dlam;
  // lane k < NZ: sensor k's position, R_kk^{-1/2}, R_kk^{-1} (this kernel runs for a diagonal R only) and
  // z_k, loaded once instead of per pseudo-time step
  // this lane's sensor row: NZ <= 32 mirrors the rows in the upper half of the wave (lr_row_sums)
  const int tr = NZ <= 32 ? (t & 31) : t;
  const int kz = tr < NZ ? tr : 0;
  const double sxk = Pm[L::AC + 2 + kz], syk = Pm[L::AC + 2 + NZ + kz];
  const double rsk = tr < NZ ? 1.0 / sqrt(Pm[L::R + kz * NZ + kz]) : 0.0;
  const double rik = Pm[L::RI + kz * NZ + kz], zk = p.z[kz];
  // lane NR + a: row a of P_pp; lane d < NX: row d of P_{:,pos} (the flow update's operands)
  const bool in_b = t >= NR && t < 2 * NR, in_c = t >= LR_CB && t < LR_CB + NR;
  typedef double dbl4 __attribute__((ext_vector_type(4)));
  constexpr int KS = (NR + 3) / 4;         // k-steps of the 8 x 8 MFMA products
  const int r16 = t & 15, kq = t >> 4;
  double pb[KS];                           // P_pp(4 ks + kq, r16): B of Rq P_pp
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = 4 * ks + kq;
    pb[ks] = (r16 < NR && k < NR) ? P[lr_pos(k) * NX + lr_pos(r16 < NR ? r16 : 0)] : 0.0;
  }
  double pp[NR], prow[NR];
  {
    const int a = in_b ? t - NR : 0, d = t < NX ? t : 0;
#pragma unroll
    for (int b = 0; b < NR; ++b) {
      pp[b] = P[lr_pos(a) * NX + lr_pos(b)];
      prow[b] = P[d * NX + lr_pos(b)];
    }
  }
#ifdef PF_STAMPS
  unsigned long long lr_last_ = __builtin_amdgcn_s_memrealtime();
#endif
  for (int64_t i = blockIdx.x; i < p.N; i += gridDim.x) {
    // ---- eta0 = g(x_{k-1}, u) + v (as k_flow_wave) ----------------------------
    for (int d = t; d < NX; d += 64) sm[SM::XP + d] = p.x_in[(int64_t)d * p.Npad + i];
    __syncthreads();
    g_block<NX, NZ, TK>(sm + SM::XP, sm + SM::GX, t1, t2, Pm, p.u);
    for (int d = t; d < NX; d += 64) {
      double vd = 0.0;
      if (p.noise == PF_NOISE_HOST) {
        vd = p.v_host[i * NX + d];
      } else if (p.noise == PF_NOISE_DEVICE) {
        const int64_t f = i * NX + d;
        t1[d] = pick4(normal4_bm24d(p.seed, (uint32_t)(f >> 2), 0u, p.epoch, STREAM_PROCESS), (int)(f & 3));
      }
      sm[SM::V + d] = vd;
    }
    __syncthreads();
    if (p.noise == PF_NOISE_DEVICE) {
      for (int d = t; d < NX; d += 64) {
        double acc = 0.0;
        for (int e = 0; e <= d; ++e) acc += Pm[L::LQ + d * NX + e] * t1[e];
        sm[SM::V + d] = acc;
      }
      __syncthreads();
    }
    for (int d = t; d < NX; d += 64) {
      const double e0 = sm[SM::GX + d] + sm[SM::V + d];
      eta0[d] = e0;
      eta[d] = e0;
    }
    __syncthreads();
    double e0p[NR];  // eta0's position components (uniform)
#pragma unroll
    for (int a = 0; a < NR; ++a) e0p[a] = eta0[lr_pos(a)];
    LR_MARK(7);
    double theta = 0.0;
    for (int j = 0; j < p.L; ++j) {
      const double lam = p.lams[j];
      double etap[NR];  // eta's position components (uniform)
#pragma unroll
      for (int a = 0; a < NR; ++a) etap[a] = eta[lr_pos(a)];
      // ---- H8 = dh/d(positions) and h at eta (ledh.py:143-145; obs_jac_block's expressions) ----
      // lane k < NZ: row k of H8, h_k(eta), and R^{-1}(z - e) with e = h(eta) - H eta (diagonal R)
      double h8[NR];
      double ru = 0.0;
      if (tr < NZ) {
        double acc = 0.0;
#pragma unroll
        for (int c = 0; c < NT; ++c) {
          const double dx = etap[2 * c] - sxk, dy = etap[2 * c + 1] - syk;
          const double den = (dx * dx + dy * dy) + d0;
          const double rd = lr_rcp(den), rd2 = rd * rd;
          acc += psi * rd;
          h8[2 * c] = (-2.0 * psi * dx) * rd2;
          h8[2 * c + 1] = (-2.0 * psi * dy) * rd2;
        }
        double he = 0.0;  // H eta over the nonzero columns, in column order
#pragma unroll
        for (int a = 0; a < NR; ++a) {
          if (t < NZ) H8[t * NR + a] = h8[a];
          he += h8[a] * etap[a];
        }
        ru = rik * (zk - (acc - he));
      } else {
#pragma unroll
        for (int a = 0; a < NR; ++a) h8[a] = 0.0;
      }
      LR_MARK(0);
      if (t < NZ)
#pragma unroll
        for (int a = 0; a < NR; ++a) sm[SM::UT + t * NR + a] = h8[a] * rsk;
      // r8 = H8^T R^{-1}(z - e) (uniform)
      double r8[NR];
#pragma unroll
      for (int a = 0; a < NR; ++a) r8[a] = h8[a] * ru;
      lr_row_sums<NZ, NR>(r8);
      lr_wave_sync();
      // ---- Rq with Rq^T Rq = U^T U (U = R^{-1/2} H8): the Cholesky factor of the Gram W = U^T U, W on
      // the fp64 matrix cores over the sensor rows, the factorisation column per lane (row 0).  Where W
      // is not numerically positive definite (a pivot below 1e-12 of its diagonal), the Householder QR.
      {
        constexpr int KZ = (NZ + 3) / 4;
        dbl4 g = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < KZ; ++ks) {
          const int k = 4 * ks + kq;
          const double v = (r16 < NR && k < NZ) ? sm[SM::UT + k * NR + r16] : 0.0;  // U(k, r16)
          g = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, g, 0, 0, 0);               // W += U^T U
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (r16 < NR && kq + 4 * q < NR) sm[SM::WC + r16 * NR + (kq + 4 * q)] = g[q];
        lr_wave_sync();
        double wa[NR], rr[NR];
        const int cw = r16 < NR ? r16 : 0;
#pragma unroll
        for (int r = 0; r < NR; ++r) wa[r] = sm[SM::WC + cw * NR + r];
        bool okc = true;
        lr_chol_pivot<NR, 0>(wa, rr, sm[SM::WC + cw * NR + cw], okc, r16);  // dg: W(c, c)
        if (!(p.lr_force & 1) && __builtin_amdgcn_readlane(okc ? 1 : 0, 0)) {
          if (t < NR)
#pragma unroll
            for (int pr = 0; pr < NR; ++pr) sm[SM::RQ + pr * NR + t] = rr[pr];
        } else {
          double u[NR];
#pragma unroll
          for (int a = 0; a < NR; ++a) u[a] = tr < NZ ? sm[SM::UT + tr * NR + a] : 0.0;
          lr_qr_col<NR, NZ, 0>(u, tr);
          if (t < NR)
#pragma unroll
            for (int c = 0; c < NR; ++c) sm[SM::RQ + t * NR + c] = c >= t ? u[c] : 0.0;
        }
      }
      lr_wave_sync();
      LR_MARK(1);
      if (i == 0 && p.diagS) {  // S = lam H8 P_pp H8^T + R of particle 0 (the condition-number diagnostic)
        for (int q = t; q < NR * NZ; q += 64) {
          const int a = q / NZ, l = q - a * NZ;
          double acc = 0.0;
          for (int m = 0; m < NR; ++m) acc += P[lr_pos(a) * NX + lr_pos(m)] * H8[l * NR + m];
          sm[SM::KS + q] = acc;
        }
        __syncthreads();
        for (int q = t; q < NZ * NZ; q += 64) {
          const int k = q / NZ, l = q - k * NZ;
          double acc = 0.0;
          for (int a = 0; a < NR; ++a) acc += H8[k * NR + a] * sm[SM::KS + a * NZ + l];
          p.diagS[(int64_t)j * NZ * NZ + q] = lam * acc + Pm[L::R + q];
        }
      }
      // ---- M = Rq P_pp Rq^T on the fp64 matrix cores: TT = Rq P_pp, then M = TT Rq^T ------------------
      // (v_mfma_f64_16x16x4f64 operands: A(r16, 4 ks + kq), B(4 ks + kq, r16); D(kq + 4 i, r16))
      {
        const bool rv = r16 < NR;
        double ra[KS];  // Rq(r16, 4 ks + kq): A of Rq P_pp and B of TT Rq^T
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int k = 4 * ks + kq;
          ra[ks] = (rv && k < NR) ? sm[SM::RQ + r16 * NR + k] : 0.0;
        }
        dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ra[ks], pb[ks], acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (rv && kq + 4 * q < NR) sm[SM::TT + (kq + 4 * q) * NR + r16] = acc[q];
        lr_wave_sync();
        double ta[KS];  // TT(r16, 4 ks + kq)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int k = 4 * ks + kq;
          ta[ks] = (rv && k < NR) ? sm[SM::TT + r16 * NR + k] : 0.0;
        }
        acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ta[ks], ra[ks], acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q)  // column r16 of M, contiguous
          if (rv && kq + 4 * q < NR) sm[SM::MC + r16 * NR + (kq + 4 * q)] = acc[q];
      }
      lr_wave_sync();
      LR_MARK(2);
      // ---- D = I + lam Rq P_pp Rq^T, D1 = I + c1 (..), column per lane: [D | Rq] -> [I | D^{-1} Rq] ----
      const double c1 = lam - 0.5 * dlam;
      // column cc of M = Rq P_pp Rq^T (lanes < NR and LR_CB .. LR_CB + NR - 1), or of Rq (lanes NR .. 2NR - 1)
      double m2[NR];
      {
        const int cc = t < NR ? t : (in_b ? t - NR : (in_c ? t - LR_CB : 0));
#pragma unroll
        for (int r = 0; r < NR; ++r) m2[r] = in_b ? sm[SM::RQ + r * NR + cc] : sm[SM::MC + cc * NR + r];
      }
      // [D | Rq | C], D = I + lam M, C = I + c1 M (det(I + dlam A) = det C / det D)
      double colD[NR];
      {
        const double sc = t < NR ? lam : (in_b ? 1.0 : (in_c ? c1 : 0.0));
        const int dr = t < NR ? t : (in_c ? t - LR_CB : -1);
#pragma unroll
        for (int r = 0; r < NR; ++r) colD[r] = (r == dr ? 1.0 : 0.0) + sc * m2[r];
      }
      LR_MARK(9);
      DetAcc D_d, C_d;
      int DC_sg;
      lr_gj_pair<NR>(colD, &D_d, &C_d, &DC_sg);
      if (DC_sg > 0 && !(p.lr_force & 6)) {
        theta += det_log_ratio(C_d, D_d);
      } else {  // the reference's +1e-12 I retry (ledh.py:174-179), as flow_logdet
        double colC[NR];
        int C_sg, D_sg = 1;
#pragma unroll
        for (int r = 0; r < NR; ++r) colC[r] = ((t < NR && r == t) ? 1.0 : 0.0) + c1 * m2[r];
        lr_logdet<NR>(colC, &C_d, &C_sg);
        {
          double colE[NR];
#pragma unroll
          for (int r = 0; r < NR; ++r) colE[r] = ((t < NR && r == t) ? 1.0 : 0.0) + lam * m2[r];
          lr_logdet<NR>(colE, &D_d, &D_sg);
        }
        if (C_sg * D_sg > 0 && !(p.lr_force & 4)) {
          theta += det_log_ratio(C_d, D_d);
        } else {
          const double eps = 1e-12;
          const double c2 = lam - dlam / (2.0 * (1.0 + eps));
#pragma unroll
          for (int r = 0; r < NR; ++r) colC[r] = ((t < NR && r == t) ? 1.0 : 0.0) + c2 * m2[r];
          lr_logdet<NR>(colC, &C_d, &C_sg);
          theta += (double)NX * log1p(eps) + det_log_ratio(C_d, D_d);
        }
      }
      if (in_b)
#pragma unroll
        for (int r = 0; r < NR; ++r) sm[SM::X + r * NR + (t - NR)] = colD[r];  // D^{-1} Rq
      lr_wave_sync();
      LR_MARK(3);
      // ---- the flow update in the position space (ledh.py:165-171) ------------------------------
      // A v = P_{:,pos} K v_pos with K = -1/2 Rq^T D^{-1} Rq (8 x 8) and c = P_{:,pos} r8, so
      //   w = c + lam A c + A eta0 = P_{:,pos} om,        om = r8 + K (lam P_pp r8 + eta0_pos)
      //   b = (I + 2 lam A) w     = P_{:,pos} (om + 2 lam K P_pp om)
      //   eta += dlam (A eta + b) = eta + dlam P_{:,pos} (om + 2 lam K P_pp om + K eta_pos)
      // lane NR + a holds row a of K and of P_pp; the 8-vectors pass between steps by readlane
      double kr[NR];  // lane NR + a: K[a][b] = -1/2 sum_r Rq[r][a] (D^{-1} Rq)[r][b]
      {
        // Rq^T (D^{-1} Rq) on the fp64 matrix cores: A(r16, k) = Rq(k, r16), B(k, r16) = X(k, r16)
        const bool rv = r16 < NR;
        dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int k = 4 * ks + kq;
          const bool v = rv && k < NR;
          const double av = v ? sm[SM::RQ + k * NR + r16] : 0.0, bv = v ? sm[SM::X + k * NR + r16] : 0.0;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)  // K row-major (the TT buffer is free again)
          if (rv && kq + 4 * q < NR) sm[SM::TT + (kq + 4 * q) * NR + r16] = -0.5 * acc[q];
        lr_wave_sync();
        const int a = in_b ? t - NR : 0;
#pragma unroll
        for (int b = 0; b < NR; ++b) kr[b] = sm[SM::TT + a * NR + b];
      }
      LR_MARK(4);
      auto dot8 = [](const double (&x)[NR], const double (&y)[NR]) {
        double acc = 0.0;
#pragma unroll
        for (int b = 0; b < NR; ++b) acc += x[b] * y[b];
        return acc;
      };
      double v1[NR], om_u[NR], v2[NR], dl[NR];
      double r8a = 0.0;  // lane NR + a: r8[a]
#pragma unroll
      for (int a = 0; a < NR; ++a) r8a = (t == NR + a) ? r8[a] : r8a;
      const double pr = dot8(pp, r8);
      lr_row_gather<NR>(pr, v1);
#pragma unroll
      for (int a = 0; a < NR; ++a) v1[a] = lam * v1[a] + e0p[a];
      const double ke = dot8(kr, etap);
      const double om = r8a + dot8(kr, v1);
      lr_row_gather<NR>(om, om_u);
      const double po = dot8(pp, om_u);
      lr_row_gather<NR>(po, v2);
      const double del = (om + 2.0 * lam * dot8(kr, v2)) + ke;
      lr_row_gather<NR>(del, dl);
      if (t < NX) eta[t] = eta[t] + dlam * dot8(prow, dl);  // lanes < NX <= 16: row 0
      lr_wave_sync();
      LR_MARK(6);
    }
    // ---- weight (ledh.py:186-190), as k_flow_wave ---------------------------------
    for (int k = t; k < NZ; k += 64) {
      const double sx = Pm[L::AC + 2 + k], sy = Pm[L::AC + 2 + NZ + k];
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        const double dx = eta[4 * c] - sx, dy = eta[4 * c + 1] - sy;
        acc += psi / ((dx * dx + dy * dy) + d0);
      }
      sm[SM::HV + k] = acc;
    }
    __syncthreads();
    double part = 0.0;
    for (int d = t; d < NX; d += 64) {  // (eta - gx)^T Q^{-1} (eta - gx) - v^T Q^{-1} v
      double a = 0.0, b = 0.0;
      for (int e = 0; e < NX; ++e) {
        const double qi = Pm[L::QI + d * NX + e];
        a += qi * (eta[e] - sm[SM::GX + e]);
        b += qi * sm[SM::V + e];
      }
      part += (-0.5 * ((eta[d] - sm[SM::GX + d]) * a)) - (-0.5 * (sm[SM::V + d] * b));
    }
    for (int k = t; k < NZ; k += 64) {
      double a = 0.0;
      for (int l = 0; l < NZ; ++l) a += Pm[L::RI + k * NZ + l] * (p.z[l] - sm[SM::HV + l]);
      part += -0.5 * ((p.z[k] - sm[SM::HV + k]) * a);
    }
    const double tot = wave_sum64(part);
    if (t == 0) p.lw[i] = (log(p.w_in[i] + 1e-300) + theta) + tot;
    for (int d = t; d < NX; d += 64) p.x_out[(int64_t)d * p.Npad + i] = eta[d];
    __syncthreads();
    LR_MARK(8);
  }
}

// ---------------------------------------------------------------------------
// weight pipeline
// ---------------------------------------------------------------------------
__device__ __forceinline__ double block_reduce_sum(double v, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum64(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += red[k];
  __syncthreads();
  return s;
}
__device__ __forceinline__ double block_reduce_max(double v, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
  for (int k = 1; k < (int)(blockDim.x >> 6); ++k) s = fmax(s, red[k]);
  __syncthreads();
  return s;
}

struct WParams {
  double* x_in;        // [NX][Npad] current particles
  double* x_out;       // [NX][Npad] resample target
  const double* lw;    // [N]
  double* w;           // [N] weights (normalised in place)
  double* w_out;       // [N] resample target weights
  double* tmax;        // [G]
  double* tsum;        // [G]
  double* trec;        // [G][2 + NX]  sum w, sum w^2, sum w x (per tile)
  double* cdf;         // [N]
  double* stat;        // [8]: ess, flag, sw, ...
  double* mean;        // [NX] the new posterior mean
  const double* shift; // [NX] the previous mean (shift of the one-pass moments)
  double* cpart;       // [Gc][1 + NX + NX(NX+1)/2]
  double* o_mean;      // output mean [NX] (nullable)
  double* o_cov;       // output cov [NX][NX] (nullable)
  double* o_ess;       // output ess (nullable)
  int32_t* o_flag;     // output flag (nullable)
  const double* unif;  // host U [1] or null
  int64_t N, Npad;
  int G, Gc;
  double ratio;
  uint64_t seed;
  uint32_t epoch;
  int uniform;         // weights are exactly 1/N (after init / resample)
};

// tile max of the log weights
__global__ void __launch_bounds__(TB) k_tile_max(WParams p) {
  __shared__ double red[TB / 64];
  const int b = blockIdx.x, t = threadIdx.x;
  const int64_t o0 = (int64_t)b * LT, o1 = min(o0 + LT, p.N);
  double m = -INFINITY;
  for (int64_t i = o0 + t; i < o1; i += TB) m = fmax(m, p.lw[i]);
  m = block_reduce_max(m, red);
  if (t == 0) p.tmax[b] = m;
}

// global max (every workgroup, same order), e_i = exp(l_i - max), tile sums
__global__ void __launch_bounds__(TB) k_exp_sum(WParams p) {
  __shared__ double red[TB / 64];
  const int b = blockIdx.x, t = threadIdx.x;
  double m = -INFINITY;
  for (int k = t; k < p.G; k += TB) m = fmax(m, p.tmax[k]);
  m = block_reduce_max(m, red);
  const int64_t o0 = (int64_t)b * LT, o1 = min(o0 + LT, p.N);
  double s = 0.0;
  for (int64_t i = o0 + t; i < o1; i += TB) {
    const double e = exp(p.lw[i] - m);
    p.w[i] = e;
    s += e;
  }
  s = block_reduce_sum(s, red);
  if (t == 0) p.tsum[b] = s;
}

// w /= sum(w) (ledh.py:195); per tile: sum w, sum w^2  (trec width 2)
__global__ void __launch_bounds__(TB) k_normalise(WParams p) {
  __shared__ double red[TB / 64];
  const int b = blockIdx.x, t = threadIdx.x;
  double S = 0.0;
  for (int k = t; k < p.G; k += TB) S += p.tsum[k];
  S = block_reduce_sum(S, red);
  const int64_t o0 = (int64_t)b * LT, o1 = min(o0 + LT, p.N);
  double a0 = 0.0, a1 = 0.0;
  for (int64_t i = o0 + t; i < o1; i += TB) {
    const double wi = p.w[i] / S;
    p.w[i] = wi;
    a0 += wi;
    a1 += wi * wi;
  }
  a0 = block_reduce_sum(a0, red);
  a1 = block_reduce_sum(a1, red);
  if (t == 0) {
    p.trec[(int64_t)b * 2] = a0;
    p.trec[(int64_t)b * 2 + 1] = a1;
  }
}

// ESS of the normalised weights (ledh.py:39-41, 202) and the resample decision (:201-203)
__global__ void __launch_bounds__(TB) k_decide(WParams p, int rec_w) {
  __shared__ double red[TB / 64];
  const int t = threadIdx.x;
  double sw = 0.0, sw2 = 0.0;
  for (int k = t; k < p.G; k += TB) {
    sw += p.trec[(int64_t)k * rec_w];
    sw2 += p.trec[(int64_t)k * rec_w + 1];
  }
  sw = block_reduce_sum(sw, red);
  sw2 = block_reduce_sum(sw2, red);
  if (t == 0) {
    const double ess = 1.0 / (sw2 / (sw * sw));
    const int flag = (p.ratio > 0.0) && (ess < p.ratio * (double)p.N);
    p.stat[0] = ess;
    p.stat[1] = flag;
    p.stat[2] = sw;
    if (p.o_ess) *p.o_ess = ess;
    if (p.o_flag) *p.o_flag = flag;
  }
}

// systematic resampling CDF: cdf_i = (prefix of tile sums + in-tile inclusive scan) / sum(w)
__global__ void __launch_bounds__(TB) k_cdf(WParams p, int rec_w) {
  __shared__ double red[TB / 64];
  __shared__ double sc[TB];
  if (p.stat[1] == 0.0) return;
  const int b = blockIdx.x, t = threadIdx.x;
  double pre = 0.0;
  for (int k = t; k < b; k += TB) pre += p.trec[(int64_t)k * rec_w];
  pre = block_reduce_sum(pre, red);
  const double sw = p.stat[2];
  const int64_t o0 = (int64_t)b * LT, o1 = min(o0 + LT, p.N);
  constexpr int PER = LT / TB;
  const int64_t s0 = o0 + (int64_t)t * PER;
  double loc[PER];
  double run = 0.0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int64_t i = s0 + q;
    run += (i < o1) ? p.w[i] : 0.0;
    loc[q] = run;
  }
  sc[t] = run;
  __syncthreads();
  double off = 0.0;
  for (int k = 0; k < t; ++k) off += sc[k];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int64_t i = s0 + q;
    if (i < o1) p.cdf[i] = (pre + (off + loc[q])) / sw;
  }
}

// ancestors: idx_i = first j with (U + i)/N < cdf_j (ledh.py:28-37), clamped; gather x, w = 1/N.
// Without a resample decision the kernel copies x, w through, so the caller can swap
// the ping-pong buffers unconditionally (device-decided resampling in pf_ledh_run).
constexpr int64_t GCAP = 16384;  // CDF entries staged in LDS by k_gather (128 KiB)
template <int NX>
__global__ void __launch_bounds__(TB) k_gather(WParams p) {
  extern __shared__ double cs[];
  const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
  const bool res = p.stat[1] != 0.0;
  const bool staged = res && p.N <= GCAP;
  if (staged) {
    // batches of 8 independent loads, then the LDS stores (one memory round trip per batch)
    for (int64_t k0 = threadIdx.x; k0 < p.N; k0 += 8 * TB) {
      double v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = k0 + r * TB < p.N ? p.cdf[k0 + r * TB] : 0.0;
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (k0 + r * TB < p.N) cs[k0 + r * TB] = v[r];
    }
    __syncthreads();
  }
  if (i >= p.N) return;
  int64_t a = i;
  double wi;
  if (res) {
    const double U = p.unif ? p.unif[0] : uniform53(p.seed, 0u, 0u, p.epoch);
    const double pos = (U + (double)i) / (double)p.N;
    const double* C = staged ? cs : p.cdf;
    int64_t lo = 0, hi = p.N;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (pos < C[mid]) hi = mid; else lo = mid + 1;
    }
    a = lo < p.N ? lo : p.N - 1;
    wi = 1.0 / (double)p.N;
  } else {
    wi = p.w[i];
  }
#pragma unroll
  for (int d = 0; d < NX; ++d) p.x_out[(int64_t)d * p.Npad + i] = p.x_in[(int64_t)d * p.Npad + a];
  p.w_out[i] = wi;
}

// the whole weight step in one workgroup for N <= SMALL_N: max, exp, normalise (ledh.py:191-195),
// ESS and decision (ledh.py:39-41, 201-203), and the systematic-resampling CDF.
constexpr int WB = 1024;
constexpr int64_t SMALL_N = 16384;  // LDS-staged weights (128 KiB) and 16 weights per thread in registers
__device__ __forceinline__ double wave_incl_scan64(double v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}
constexpr int WPT = (int)(SMALL_N / WB);  // weights per thread kept in registers (N <= SMALL_N)
__global__ void __launch_bounds__(WB) k_weights_small(WParams p) {
  __shared__ double red[WB / 64];
  extern __shared__ double wl[];  // [N] normalised weights staged for the CDF scan
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double v[WPT];  // this thread's log weights, then weights: loaded once (coalesced i = t + r WB)
#pragma unroll
  for (int r = 0; r < WPT; ++r) {
    const int64_t i = t + (int64_t)r * WB;
    v[r] = i < p.N ? p.lw[i] : -INFINITY;
  }
  double m = -INFINITY;
#pragma unroll
  for (int r = 0; r < WPT; ++r) m = fmax(m, v[r]);
  const double M = block_reduce_max(m, red);
  double s = 0.0;
#pragma unroll
  for (int r = 0; r < WPT; ++r) {
    v[r] = (t + (int64_t)r * WB < p.N) ? exp(v[r] - M) : 0.0;
    s += v[r];
  }
  const double S = block_reduce_sum(s, red);
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int r = 0; r < WPT; ++r) {
    const int64_t i = t + (int64_t)r * WB;
    v[r] = v[r] / S;  // w /= sum(w) (ledh.py:195)
    if (i < p.N) {
      p.w[i] = v[r];
      wl[i] = v[r];
    }
    a0 += v[r];
    a1 += v[r] * v[r];
  }
  const double sw = block_reduce_sum(a0, red);
  const double sw2 = block_reduce_sum(a1, red);
  const double ess = 1.0 / (sw2 / (sw * sw));
  const int flag = (p.ratio > 0.0) && (ess < p.ratio * (double)p.N);
  if (flag) {  // cdf = cumsum(w / sum w): contiguous chunks per thread from LDS, one block scan
    const int64_t per = (p.N + WB - 1) / WB;
    const int64_t i0 = (int64_t)t * per, i1 = min(i0 + per, p.N);
    double c = 0.0;
    for (int64_t i = i0; i < i1; ++i) c += wl[i];
    const double inc = wave_incl_scan64(c, lane);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    double off = 0.0;
    for (int k = 0; k < wv; ++k) off += red[k];
    double run = off + inc - c;
    for (int64_t i = i0; i < i1; ++i) {
      run += wl[i];
      p.cdf[i] = run / sw;
    }
  }
  if (t == 0) {
    p.stat[0] = ess;
    p.stat[1] = flag;
    p.stat[2] = sw;
    if (p.o_ess) *p.o_ess = ess;
    if (p.o_flag) *p.o_flag = flag;
  }
}

// K simultaneous block sums (one pass): result valid in every thread
template <int K>
__device__ __forceinline__ void block_sum_multi(double (&v)[K], double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = (int)(blockDim.x >> 6);
#pragma unroll
  for (int f = 0; f < K; ++f) v[f] = wave_sum64(v[f]);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int f = 0; f < K; ++f) red[w * K + f] = v[f];
  __syncthreads();
#pragma unroll
  for (int f = 0; f < K; ++f) {
    double s = 0.0;
    for (int k = 0; k < nw; ++k) s += red[k * K + f];
    v[f] = s;
  }
  __syncthreads();
}

// Posterior moments (ledh.py:217-224) in one pass over the particles, shifted by the
// previous mean c (so sum w (x-c)(x-c)^T / sw - (m-c)(m-c)^T loses nothing to cancellation):
// per tile of CT particles the partial sums  sum w | sum w (x-c) | sum w (x-c)(x-c)^T (upper).
template <int NX>
struct Mom {
  static constexpr int NP = NX * (NX + 1) / 2;
  static constexpr int E = 1 + NX + NP;
};
__device__ __forceinline__ void pair_of(int q, int NX, int* d, int* e) {
  int dd = 0, rem = q;
  while (rem >= NX - dd) { rem -= NX - dd; ++dd; }
  *d = dd;
  *e = dd + rem;
}
// Register-blocked: thread = (4x4 block of the upper triangle, particle slice); the slices are
// combined in LDS.  s0 and s1 by the first 1 + NX threads.
template <int NX>
struct MomBlk {
  static constexpr int NB = (NX + 3) / 4;            // 4-wide blocks per dimension
  static constexpr int NPAIR = NB * (NB + 1) / 2;     // upper-triangular block pairs
  static constexpr int SL = NPAIR * 4 <= TB ? 4 : (NPAIR * 2 <= TB ? 2 : 1);  // particle slices
  static constexpr int XW = NB * 4;                   // padded row width of the staged tile
};
template <int NX>
__global__ void __launch_bounds__(TB) k_mom_part(WParams p) {
  using MM = Mom<NX>;
  using MB = MomBlk<NX>;
  static_assert(MB::NPAIR * MB::SL <= TB, "block pairs x slices fit the workgroup");
  __shared__ double xs[CT * MB::XW];
  __shared__ double ws[CT];
  __shared__ double red[MB::SL][MB::NPAIR][16];
  const int b = blockIdx.x, t = threadIdx.x;
  const int64_t o0 = (int64_t)b * CT;
  const int n = (int)max((int64_t)0, min((int64_t)CT, p.N - o0));
#pragma unroll 8
  for (int q = t; q < CT * MB::XW; q += TB) {
    const int j = q / MB::XW, d = q - j * MB::XW;
    xs[q] = (j < n && d < NX) ? p.x_in[(int64_t)d * p.Npad + o0 + j] - p.shift[d] : 0.0;
  }
  for (int j = t; j < CT; j += TB) ws[j] = j < n ? (p.uniform ? 1.0 / (double)p.N : p.w[o0 + j]) : 0.0;
  __syncthreads();
  double* out = p.cpart + (int64_t)b * MM::E;
  if (t <= NX) {  // s0 = sum w, s1_d = sum w (x_d - c_d)
    double a = 0.0;
    if (t == 0)
      for (int j = 0; j < n; ++j) a += ws[j];
    else
      for (int j = 0; j < n; ++j) a += ws[j] * xs[j * MB::XW + t - 1];
    out[t] = a;
  }
  const int pair = t % MB::NPAIR, sl = t / MB::NPAIR;
  if (sl < MB::SL) {
    int bi = 0, rem = pair;
    while (rem >= MB::NB - bi) { rem -= MB::NB - bi; ++bi; }
    const int bj = bi + rem;
    double acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = 0.0;
    for (int j = sl; j < n; j += MB::SL) {
      const double* r = xs + j * MB::XW;
      const double wj = ws[j];
      double u[4], v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        u[k] = r[4 * bi + k] * wj;
        v[k] = r[4 * bj + k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int l = 0; l < 4; ++l) acc[k * 4 + l] += u[k] * v[l];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) red[sl][pair][k] = acc[k];
  }
  __syncthreads();
  if (t < MB::NPAIR) {  // combine slices, scatter the block's upper-triangle entries
    int bi = 0, rem = t;
    while (rem >= MB::NB - bi) { rem -= MB::NB - bi; ++bi; }
    const int bj = bi + rem;
    for (int k = 0; k < 4; ++k)
      for (int l = 0; l < 4; ++l) {
        const int d = 4 * bi + k, e = 4 * bj + l;
        if (d >= NX || e >= NX || e < d) continue;
        double a = 0.0;
        for (int s2 = 0; s2 < MB::SL; ++s2) a += red[s2][t][k * 4 + l];
        // upper-triangle index of (d, e): rows 0..d-1 hold NX - r entries each
        const int q = d * NX - d * (d - 1) / 2 + (e - d);
        out[1 + NX + q] = a;
      }
  }
}

// sum of entry q over the Gc tile partials, fixed order
__device__ __forceinline__ double part_sum(const double* cpart, int Gc, int E, int q) {
  double acc[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) acc[r] = 0.0;
  int k = 0;
  for (; k + 8 <= Gc; k += 8) {
    double v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = cpart[(int64_t)(k + r) * E + q];  // 8 loads in flight
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] += v[r];
  }
  for (; k < Gc; ++k) acc[0] += cpart[(int64_t)k * E + q];
  return ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

// mean = c + s1/sw, cov = s2/sw - (s1/sw)(s1/sw)^T.  Workgroup = 16 output entries x 16 partial
// lanes: lane p sums partials p, p+16, ... (independent loads), then an LDS tree per entry.
constexpr int MF_E = 16, MF_P = 16;
template <int NX>
__global__ void __launch_bounds__(MF_E * MF_P) k_mom_final(WParams p) {
  using MM = Mom<NX>;
  __shared__ double part[4][MF_E][MF_P + 1];
  const int t = threadIdx.x, el = t / MF_P, pl = t % MF_P;
  const int q = blockIdx.x * MF_E + el;  // output entry: q < NX mean, else cov pair
  const bool live = q < NX + MM::NP;
  int d = 0, e = 0;
  if (live && q >= NX) pair_of(q - NX, NX, &d, &e);
  const int src[4] = {0, 1 + (q < NX ? q : d), 1 + e, q >= NX ? 1 + NX + (q - NX) : 0};
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  if (live)
    for (int k = pl; k < p.Gc; k += MF_P) {
      double v[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) v[f] = p.cpart[(int64_t)k * MM::E + src[f]];
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[f] += v[f];
    }
#pragma unroll
  for (int f = 0; f < 4; ++f) part[f][el][pl] = acc[f];
  __syncthreads();
  if (pl != 0 || !live) return;
  double tot[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    double sum = 0.0;
    for (int k = 0; k < MF_P; ++k) sum += part[f][el][k];
    tot[f] = sum;
  }
  const double sw = tot[0];
  if (q < NX) {
    const double m = p.shift[q] + tot[1] / sw;
    p.mean[q] = m;
    if (p.o_mean) p.o_mean[q] = m;
    if (q == 0) p.stat[3] = sw;
    return;
  }
  const double c = tot[3] / sw - (tot[1] / sw) * (tot[2] / sw);
  if (p.o_cov) {
    p.o_cov[d * NX + e] = c;
    p.o_cov[e * NX + d] = c;
  }
}

// initial particles: x = mean0 + eps, eps = host draw [N][NX] or chol(cov0) n (Philox)
template <int NX>
__global__ void __launch_bounds__(TB) k_init(double* x, double* w, const double* mean0, const double* Lc,
                                              const double* eps, int64_t N, int64_t Npad, uint64_t seed,
                                              uint32_t epoch) {
  const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
  if (i >= N) return;
  double n[NX];
  if (!eps) normals_range<NX>(seed, i * NX, epoch, STREAM_INIT, n);
#pragma unroll
  for (int d = 0; d < NX; ++d) {
    double e;
    if (eps) {
      e = eps[i * NX + d];
    } else {
      e = 0.0;
#pragma unroll
      for (int c = 0; c <= d; ++c) e += Lc[d * NX + c] * n[c];
    }
    x[(int64_t)d * Npad + i] = mean0[d] + e;
  }
  w[i] = 1.0 / (double)N;
}

}  // namespace ledh
}  // namespace pf
