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

constexpr int EB = 1024;  // EKF workgroup

template <int NX, int NZ>
struct EkfSmem {
  static constexpr int X = 0;                   // NX   state mean
  static constexpr int Y = X + NX;              // NX   stage point / scratch
  static constexpr int K1 = Y + NX;             // NX   RK4 slopes
  static constexpr int ACC = K1 + NX;           // NX
  static constexpr int S2 = ACC + NX;           // NX   stage points y2, y3, y4
  static constexpr int S3 = S2 + NX;
  static constexpr int S4 = S3 + NX;
  static constexpr int P = S4 + NX;             // NX*NX  covariance
  static constexpr int G = P + NX * NX;         // NX*NX  Jacobian of g
  static constexpr int W1 = G + NX * NX;        // NX*NX  scratch (tangent stage / G P)
  static constexpr int W2 = W1 + NX * NX;       // NX*NX  scratch
  static constexpr int H = W2 + NX * NX;        // NZ*NX  Jacobian of h
  static constexpr int HV = H + NZ * NX;        // NZ     h(x_pred)
  static constexpr int PHT = HV + NZ;           // NX*NZ  P H^T
  static constexpr int AUG = PHT + NX * NZ;     // NZ*2NZ [S | I] -> [I | S^{-1}]
  static constexpr int KG = AUG + 2 * NZ * NZ;  // NX*NZ  gain
  static constexpr int FAC = KG + NX * NZ;      // NZ
  static constexpr int SIZE = FAC + NZ;
};

// C = A B (+ D) for row-major NX x NX LDS matrices; `transB` uses B^T
template <int NX>
__device__ __forceinline__ void lds_mm(const double* A, const double* B, double* C, const double* D, bool transB) {
  for (int q = threadIdx.x; q < NX * NX; q += blockDim.x) {
    const int a = q / NX, c = q - a * NX;
    double acc = 0.0;
    for (int k = 0; k < NX; ++k) acc += A[a * NX + k] * (transB ? B[c * NX + k] : B[k * NX + c]);
    C[q] = D ? acc + D[q] : acc;
  }
  __syncthreads();
}

// (J(y) V)[a][c] for the L96 right-hand side (y[a+1] - y[a-2]) y[a-1] - y[a] + F
template <int NX>
__device__ __forceinline__ double l96_jv(const double* y, const double* V, int a, int c) {
  const int ap1 = (a + 1) % NX, am1 = (a + NX - 1) % NX, am2 = (a + NX - 2) % NX;
  return V[ap1 * NX + c] * y[am1] - V[am2 * NX + c] * y[am1] + V[am1 * NX + c] * (y[ap1] - y[am2]) - V[a * NX + c];
}

template <int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(EB) k_ekf_seq(const double* __restrict__ Pm, const double* x0, const double* P0,
                                               const double* __restrict__ Qt, const double* __restrict__ Rt,
                                               const double* Z, int64_t T, double* Ps, double* x_out, double* P_out,
                                               double* Xp) {
  using L = Lay<NX, NZ>;
  using SM = EkfSmem<NX, NZ>;
  __shared__ double sm[SM::SIZE];
  const int t = threadIdx.x;
  double* x = sm + SM::X;
  double* P = sm + SM::P;
  double* G = sm + SM::G;
  double* W1 = sm + SM::W1;
  double* W2 = sm + SM::W2;
  double* H = sm + SM::H;
  double* aug = sm + SM::AUG;
  for (int d = t; d < NX; d += EB) x[d] = x0[d];
  for (int q = t; q < NX * NX; q += EB) {
    P[q] = P0[q];
    if constexpr (TK == PF_TRANS_LINEAR) G[q] = Pm[L::A + q];
  }
  __syncthreads();
  for (int64_t k = 0; k < T; ++k) {
    if (Xp)  // the tracker's past mean x_{k-1|k-1} (EDH linearisation start, edh.py:200)
      for (int d = t; d < NX; d += EB) Xp[k * NX + d] = x[d];
    // ---- predict: x = g(x), G = dg/dx at x (extended_kalman_filter.py:178-192) -------
    if constexpr (TK == PF_TRANS_LINEAR) {
      for (int d = t; d < NX; d += EB) {
        double acc = 0.0;
        for (int e = 0; e < NX; ++e) acc += Pm[L::A + d * NX + e] * x[e];
        sm[SM::Y + d] = acc;
      }
      __syncthreads();
      for (int d = t; d < NX; d += EB) x[d] = sm[SM::Y + d];
      __syncthreads();
    } else {  // L96 RK4 and its tangent (models.L96Transition.jacobian)
      const double F = Pm[L::EX], dt = Pm[L::EX + 1];
      double* k1 = sm + SM::K1;
      double* acc = sm + SM::ACC;
      double* s2 = sm + SM::S2;
      double* s3 = sm + SM::S3;
      double* s4 = sm + SM::S4;
      for (int a = t; a < NX; a += EB) { k1[a] = l96_rhs_at<NX>(x, a, F); acc[a] = k1[a]; s2[a] = x[a] + 0.5 * dt * k1[a]; }
      __syncthreads();
      for (int a = t; a < NX; a += EB) k1[a] = l96_rhs_at<NX>(s2, a, F);
      __syncthreads();
      for (int a = t; a < NX; a += EB) { acc[a] += 2.0 * k1[a]; s3[a] = x[a] + 0.5 * dt * k1[a]; }
      __syncthreads();
      for (int a = t; a < NX; a += EB) k1[a] = l96_rhs_at<NX>(s3, a, F);
      __syncthreads();
      for (int a = t; a < NX; a += EB) { acc[a] += 2.0 * k1[a]; s4[a] = x[a] + dt * k1[a]; }
      __syncthreads();
      // tangent: D1 = J(x); D2 = J(s2)(I + dt/2 D1); D3 = J(s3)(I + dt/2 D2); D4 = J(s4)(I + dt D3)
      //          G = I + dt/6 (D1 + 2 D2 + 2 D3 + D4);  W1 = current D, W2 = I + c D, G accumulates
      for (int q = t; q < NX * NX; q += EB) {
        const int a = q / NX, c = q - a * NX;
        // J(x) I: row a has entries at a+1, a-2, a-1, a
        const int ap1 = (a + 1) % NX, am1 = (a + NX - 1) % NX, am2 = (a + NX - 2) % NX;
        double v = (c == ap1 ? x[am1] : 0.0) - (c == am2 ? x[am1] : 0.0) + (c == am1 ? x[ap1] - x[am2] : 0.0) -
                   (c == a ? 1.0 : 0.0);
        W1[q] = v;
        G[q] = v;
      }
      __syncthreads();
      const double* stage[3] = {s2, s3, s4};
      const double cf[3] = {0.5 * dt, 0.5 * dt, dt};
      const double wt[3] = {2.0, 2.0, 1.0};
      for (int st = 0; st < 3; ++st) {
        for (int q = t; q < NX * NX; q += EB) W2[q] = ((q / NX == q % NX) ? 1.0 : 0.0) + cf[st] * W1[q];
        __syncthreads();
        for (int q = t; q < NX * NX; q += EB) {
          const int a = q / NX, c = q - a * NX;
          const double v = l96_jv<NX>(stage[st], W2, a, c);
          W1[q] = v;
        }
        __syncthreads();
        for (int q = t; q < NX * NX; q += EB) G[q] += wt[st] * W1[q];
        __syncthreads();
      }
      for (int q = t; q < NX * NX; q += EB) G[q] = ((q / NX == q % NX) ? 1.0 : 0.0) + (dt / 6.0) * G[q];
      for (int a = t; a < NX; a += EB) k1[a] = l96_rhs_at<NX>(s4, a, F);  // k4
      __syncthreads();
      const double h6 = dt / 6.0;
      for (int a = t; a < NX; a += EB) x[a] = x[a] + h6 * (acc[a] + k1[a]);
      __syncthreads();
    }
    // P = G P G^T + Q
    lds_mm<NX>(G, P, W1, nullptr, false);
    lds_mm<NX>(W1, G, P, Qt, true);
    for (int q = t; q < NX * NX; q += EB) {
      const int a = q / NX, c = q - a * NX;
      Ps[k * NX * NX + q] = 0.5 * (P[a * NX + c] + P[c * NX + a]);  // ledh.py:106
    }
    // ---- update (extended_kalman_filter.py:208-239) ---------------------------------
    obs_jac_block<NX, NZ, OK>(x, H, sm + SM::HV, Pm);
    for (int q = t; q < NX * NZ; q += EB) {  // P H^T
      const int d = q / NZ, kz = q - d * NZ;
      double acc = 0.0;
      for (int e = 0; e < NX; ++e) acc += P[d * NX + e] * H[kz * NX + e];
      sm[SM::PHT + q] = acc;
    }
    __syncthreads();
    for (int q = t; q < NZ * NZ; q += EB) {  // S = H P H^T + R -> [S | I]
      const int r = q / NZ, c = q - r * NZ;
      double acc = 0.0;
      for (int d = 0; d < NX; ++d) acc += H[r * NX + d] * sm[SM::PHT + d * NZ + c];
      aug[r * 2 * NZ + c] = acc + Rt[q];
      aug[r * 2 * NZ + NZ + c] = (r == c) ? 1.0 : 0.0;
    }
    __syncthreads();
    double ld;
    int sg;
    block_gauss_jordan<NZ>(aug, sm + SM::FAC, &ld, &sg);
    for (int q = t; q < NX * NZ; q += EB) {  // K = (P H^T) S^{-1}
      const int d = q / NZ, c = q - d * NZ;
      double acc = 0.0;
      for (int kz = 0; kz < NZ; ++kz) acc += sm[SM::PHT + d * NZ + kz] * aug[kz * 2 * NZ + NZ + c];
      sm[SM::KG + q] = acc;
    }
    __syncthreads();
    for (int d = t; d < NX; d += EB) {  // x += K (z - h(x))
      double acc = 0.0;
      for (int kz = 0; kz < NZ; ++kz) acc += sm[SM::KG + d * NZ + kz] * (Z[k * NZ + kz] - sm[SM::HV + kz]);
      sm[SM::Y + d] = x[d] + acc;
    }
    for (int q = t; q < NX * NX; q += EB) {  // W2 = I - K H
      const int a = q / NX, c = q - a * NX;
      double acc = 0.0;
      for (int kz = 0; kz < NZ; ++kz) acc += sm[SM::KG + a * NZ + kz] * H[kz * NX + c];
      W2[q] = ((a == c) ? 1.0 : 0.0) - acc;
    }
    __syncthreads();
    for (int d = t; d < NX; d += EB) x[d] = sm[SM::Y + d];
    lds_mm<NX>(W2, P, W1, nullptr, false);  // P = (I - K H) P
    for (int q = t; q < NX * NX; q += EB) P[q] = W1[q];
    __syncthreads();
  }
  if (x_out)
    for (int d = t; d < NX; d += EB) x_out[d] = x[d];
  if (P_out)
    for (int q = t; q < NX * NX; q += EB) P_out[q] = P[q];
}

}  // namespace ledh
}  // namespace pf
