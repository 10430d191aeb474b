// Device EKF tracker for the LEDH run loop (fp64, one workgroup).
//
// The LEDH flow needs the Gaussian tracker's predicted covariance P_k every step
// (LEDH_particle_filter.py:105-106).  The tracker never sees the particles, so the
// whole sequence P_1..P_T can be produced before the particle loop: k_ekf_seq runs
// the additive-noise EKF of extended_kalman_filter.py:164-241 (predict: x = g(x),
// P = G P G^T + Q; update: S = H P H^T + R, K = P H^T S^{-1}, x += K (z - h(x)),
// P = (I - K H) P) for T steps in one workgroup, with the models' analytic Jacobians
// (LINEAR: A; L96: the tangent-linear RK4 step, as models.L96Transition.jacobian;
// h: H, the acoustic / exp-half derivatives of pf_ledh_kernels.h obs_jac_block), and
// writes the symmetrised 0.5 (P + P^T) of every predicted covariance for the flow.
#pragma once
#include "pf_ledh_kernels.h"

namespace pf {
namespace ledh {

// EKF workgroup: 16 waves; 8 (256 VGPRs a lane) where the update's Gauss-Jordan holds 25 rows
template <int NZ>
constexpr int ekf_block() { return NZ > 16 ? 512 : 1024; }

template <int NX, int NZ>
struct EkfSmem {
  static constexpr int X = 0;                   // NX   state mean (x_{k-1|k-1}, then x_{k|k})
  static constexpr int XP = X + NX;             // NX   predicted mean g(x)
  static constexpr int S2 = XP + NX;            // NX   RK4 stage points y2, y3, y4
  static constexpr int S3 = S2 + NX;
  static constexpr int S4 = S3 + NX;
  static constexpr int HV = S4 + NX;            // NZ   h(x_pred)
  static constexpr int P = HV + NZ;             // NX*NX  covariance
  static constexpr int G = P + NX * NX;         // NX*NX  Jacobian of g
  static constexpr int W1 = G + NX * NX;        // NX*NX  tangent stages / G P
  static constexpr int W2 = W1 + NX * NX;       // NX*NX  tangent stages
  static constexpr int QS = W2 + NX * NX;       // NX*NX  Q
  static constexpr int H = QS + NX * NX;        // NZ*NX  Jacobian of h
  static constexpr int PHT = H + NZ * NX;       // NX*NZ  P H^T
  static constexpr int SA = PHT + NX * NZ;      // NZ*NZ  S = H P H^T + R
  static constexpr int RS = SA + NZ * NZ;       // NZ*NZ  R
  static constexpr int KG = RS + NZ * NZ;       // NX*NZ  gain
  static constexpr int SIZE = KG + NX * NZ;
};

// C = A op(B) for small row-major LDS matrices on the fp64 matrix cores (v_mfma_f64_16x16x4):
// A(r, k) = A[r lda + k] (M x K), op(B)(k, c) = TB ? B[c ldb + k] : B[k ldb + c] (K x N).  Waves
// w0, w0 + nw, ... of the workgroup take the 16 x 16 output tiles in turn; out-of-range operands are
// zeros (selects, no divergent branches around the MFMA); epi(r, c, v) receives every entry.
template <int M, int N, int K, bool TB, class Epi>
__device__ __forceinline__ void mfma_mm(const double* A, int lda, const double* B, int ldb, int w0, int nw,
                                        Epi epi) {
  typedef double dbl4 __attribute__((ext_vector_type(4)));
  constexpr int TM = (M + 15) / 16, TN = (N + 15) / 16, KS = (K + 3) / 4;
  const int lane = threadIdx.x & 63, r16 = lane & 15, kq = lane >> 4;
  for (int tile = (int)(threadIdx.x >> 6) - w0; tile < TM * TN; tile += nw) {
    if (tile < 0) break;
    const int I = tile / TN, J = tile - I * TN;
    const int ra = 16 * I + r16, cb = 16 * J + r16;
    const bool va = ra < M, vb = cb < N;
    const int rac = va ? ra : 0, cbc = vb ? cb : 0;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 4 * ks + kq;
      const bool vk = k < K;
      const int kc = vk ? k : 0;
      const double a = A[rac * lda + kc];
      const double b = TB ? B[cbc * ldb + kc] : B[kc * ldb + cbc];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64((va && vk) ? a : 0.0, (vb && vk) ? b : 0.0, acc, 0, 0, 0);
    }
    // D layout: col = lane & 15, row = (lane >> 4) + 4 reg
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * I + kq + 4 * r, col = 16 * J + r16;
      if (row < M && col < N) epi(row, col, acc[r]);
    }
  }
}

// LDS writes of this wave complete before its next LDS reads (one wave, no workgroup barrier)
__device__ __forceinline__ void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// V = I + cf W, (J(y) V)[a][c] for the L96 right-hand side (y[a+1] - y[a-2]) y[a-1] - y[a] + F
template <int NX>
__device__ __forceinline__ double l96_jv(const double* y, const double* W, double cf, int a, int c) {
  const int ap1 = (a + 1) % NX, am1 = (a + NX - 1) % NX, am2 = (a + NX - 2) % NX;
  auto V = [&](int r) { return ((r == c) ? 1.0 : 0.0) + cf * W[r * NX + c]; };
  return V(ap1) * y[am1] - V(am2) * y[am1] + V(am1) * (y[ap1] - y[am2]) - V(a);
}

// One workgroup, 9 workgroup barriers per step (L96; 6 for a linear transition):
//   A   wave 0: the RK4 step x -> x_pred (stage points kept for the tangent), wave-synchronous;
//       the other waves: D1 = J(x) (L96) - or wave 0: x_pred = A x (linear)
//   T1..T3  the tangent stages D_s = J(y_s)(I + c D_{s-1}), G += w D_s (L96), with H, h(x_pred)
//   M1, M2  P = G P G^T + Q on the matrix cores
//   M3  P H^T on the matrix cores; the symmetrised predicted covariance written out
//   U   wave 0: S = H P H^T + R (matrix cores), Gauss-Jordan with partial pivoting on [S | (P H^T)^T]
//       held column per lane -> K^T = S^{-1} (P H^T)^T (S symmetric), x += K (z - h)
//   M4  P -= K (P H^T)^T on the matrix cores (= (I - K H) P for symmetric P)
// The algebra is the reference's up to the order of fp64 rounding (the host EKF agrees to ~1e-13,
// tests/test_gpu_ledh.py::test_device_tracker_covariances_equal_host_ekf).
template <int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(ekf_block<NZ>()) k_ekf_seq(const double* __restrict__ Pm, const double* x0, const double* P0,
                                               const double* __restrict__ Qt, const double* __restrict__ Rt,
                                               const double* Z, int64_t T, double* Ps, double* x_out, double* P_out,
                                               double* Xp) {
  static_assert(NX + NZ <= 64, "the update's Gauss-Jordan holds [S | (P H^T)^T] column per lane of one wave");
  using L = Lay<NX, NZ>;
  using SM = EkfSmem<NX, NZ>;
  constexpr int EB = ekf_block<NZ>();
  __shared__ double sm[SM::SIZE];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  constexpr int NW = EB / 64;
  double* x = sm + SM::X;
  double* xp = sm + SM::XP;
  double* P = sm + SM::P;
  double* G = sm + SM::G;
  double* W1 = sm + SM::W1;
  double* W2 = sm + SM::W2;
  double* H = sm + SM::H;
  double* PHT = sm + SM::PHT;
  double* KG = sm + SM::KG;
  const double* QS = sm + SM::QS;
  const double* RS = sm + SM::RS;
  for (int d = t; d < NX; d += EB) x[d] = x0[d];
  for (int q = t; q < NX * NX; q += EB) {
    P[q] = P0[q];
    sm[SM::QS + q] = Qt[q];
    if constexpr (TK == PF_TRANS_LINEAR) G[q] = Pm[L::A + q];
  }
  for (int q = t; q < NZ * NZ; q += EB) sm[SM::RS + q] = Rt[q];
  __syncthreads();
  for (int64_t k = 0; k < T; ++k) {
    if (Xp)  // the tracker's past mean x_{k-1|k-1} (EDH linearisation start, edh.py:200)
      for (int d = t; d < NX; d += EB) Xp[k * NX + d] = x[d];
    // ---- predict: x = g(x), G = dg/dx at x (extended_kalman_filter.py:178-192) -------
    if constexpr (TK == PF_TRANS_LINEAR) {
      if (wv == 0 && lane < NX) {
        double acc = 0.0;
        for (int e = 0; e < NX; ++e) acc += G[lane * NX + e] * x[e];
        xp[lane] = acc;
      }
      __syncthreads();
      obs_jac_block<NX, NZ, OK>(xp, H, sm + SM::HV, Pm);  // (ends on a barrier)
    } else {  // L96 RK4 and its tangent (models.L96Transition.jacobian)
      const double F = Pm[L::EX], dt = Pm[L::EX + 1];
      double* s2 = sm + SM::S2;
      double* s3 = sm + SM::S3;
      double* s4 = sm + SM::S4;
      if (wv == 0) {
        const int a = lane < NX ? lane : 0;
        const bool on = lane < NX;
        double k1 = l96_rhs_at<NX>(x, a, F);
        double acc = k1;
        if (on) s2[a] = x[a] + 0.5 * dt * k1;
        wave_lds_fence();
        k1 = l96_rhs_at<NX>(s2, a, F);
        acc += 2.0 * k1;
        if (on) s3[a] = x[a] + 0.5 * dt * k1;
        wave_lds_fence();
        k1 = l96_rhs_at<NX>(s3, a, F);
        acc += 2.0 * k1;
        if (on) s4[a] = x[a] + dt * k1;
        wave_lds_fence();
        k1 = l96_rhs_at<NX>(s4, a, F);  // k4
        if (on) xp[a] = x[a] + (dt / 6.0) * (acc + k1);
      } else {
        // D1 = J(x): row a has entries at a+1, a-2, a-1, a;  W1 = D1, G accumulates
        for (int q = t - 64; q < NX * NX; q += EB - 64) {
          const int a = q / NX, c = q - a * NX;
          const int ap1 = (a + 1) % NX, am1 = (a + NX - 1) % NX, am2 = (a + NX - 2) % NX;
          const double v = (c == ap1 ? x[am1] : 0.0) - (c == am2 ? x[am1] : 0.0) +
                           (c == am1 ? x[ap1] - x[am2] : 0.0) - (c == a ? 1.0 : 0.0);
          W1[q] = v;
          G[q] = v;
        }
      }
      __syncthreads();
      // D2 = J(y2)(I + dt/2 D1), D3 = J(y3)(I + dt/2 D2), D4 = J(y4)(I + dt D3);
      // G = I + dt/6 (D1 + 2 D2 + 2 D3 + D4)
      for (int q = t; q < NX * NX; q += EB) {
        const int a = q / NX, c = q - a * NX;
        const double v = l96_jv<NX>(s2, W1, 0.5 * dt, a, c);
        W2[q] = v;
        G[q] += 2.0 * v;
      }
      obs_jac_block<NX, NZ, OK>(xp, H, sm + SM::HV, Pm);  // (ends on a barrier)
      for (int q = t; q < NX * NX; q += EB) {
        const int a = q / NX, c = q - a * NX;
        const double v = l96_jv<NX>(s3, W2, 0.5 * dt, a, c);
        W1[q] = v;
        G[q] += 2.0 * v;
      }
      __syncthreads();
      for (int q = t; q < NX * NX; q += EB) {
        const int a = q / NX, c = q - a * NX;
        const double v = l96_jv<NX>(s4, W1, dt, a, c);
        G[q] = ((a == c) ? 1.0 : 0.0) + (dt / 6.0) * (G[q] + 1.0 * v);
      }
      __syncthreads();
    }
    // P = G P G^T + Q
    mfma_mm<NX, NX, NX, false>(G, NX, P, NX, 0, NW, [&](int r, int c, double v) { W1[r * NX + c] = v; });
    __syncthreads();
    mfma_mm<NX, NX, NX, true>(W1, NX, G, NX, 0, NW,
                              [&](int r, int c, double v) { P[r * NX + c] = v + QS[r * NX + c]; });
    __syncthreads();
    // ---- update (extended_kalman_filter.py:208-239) ---------------------------------
    mfma_mm<NX, NZ, NX, true>(P, NX, H, NX, 0, NW, [&](int r, int c, double v) { PHT[r * NZ + c] = v; });
    for (int q = t; q < NX * NX; q += EB) {
      const int a = q / NX, c = q - a * NX;
      Ps[k * NX * NX + q] = 0.5 * (P[a * NX + c] + P[c * NX + a]);  // ledh.py:106
    }
    __syncthreads();
    if (wv == 0) {
      double* SA = sm + SM::SA;
      mfma_mm<NZ, NZ, NX, false>(H, NX, PHT, NZ, 0, 1,
                                 [&](int r, int c, double v) { SA[r * NZ + c] = v + RS[r * NZ + c]; });
      wave_lds_fence();
      // [S | (P H^T)^T]: lane c < NZ column c of S, lane NZ + d column d of (P H^T)^T = row d of P H^T
      double col[NZ];
#pragma unroll
      for (int r = 0; r < NZ; ++r)
        col[r] = lane < NZ ? SA[r * NZ + lane] : (lane < NZ + NX ? PHT[(lane - NZ) * NZ + r] : 0.0);
      DetAcc det;
      int sg;
      lr_gauss_jordan<NZ>(col, &det, &sg);
      (void)det;
      (void)sg;
      if (lane >= NZ && lane < NZ + NX) {  // row d of K = P H^T S^{-1}; x += K (z - h(x))
        const int d = lane - NZ;
        double acc = 0.0;
#pragma unroll
        for (int r = 0; r < NZ; ++r) {
          KG[d * NZ + r] = col[r];
          acc += col[r] * (Z[k * NZ + r] - sm[SM::HV + r]);
        }
        x[d] = xp[d] + acc;
      }
    }
    __syncthreads();
    // P = (I - K H) P, as P - K (P H^T)^T
    mfma_mm<NX, NX, NZ, true>(KG, NZ, PHT, NZ, 0, NW, [&](int r, int c, double v) { P[r * NX + c] -= v; });
    __syncthreads();
  }
  if (x_out)
    for (int d = t; d < NX; d += EB) x_out[d] = x[d];
  if (P_out)
    for (int q = t; q < NX * NX; q += EB) P_out[q] = P[q];
}

}  // namespace ledh
}  // namespace pf
