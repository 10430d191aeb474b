// EDH (exact Daum-Huang) particle-flow kernels for gfx950 (fp64, wave64).
//
// The reference's EDHFlowPF.step (/root/reference/models/EDH_particle_filter.py, "edh.py:LINE")
// linearises h once per pseudo-time step lambda_j at the tracker-driven mean trajectory etabar
// (edh.py:213, 229-264), never at a particle, so A_j and b_j are shared by every particle:
//   S = lam H P H^T + R,  A = -1/2 P H^T S^{-1} H,  b = (I + 2 lam A)[(I + lam A) P H^T R^{-1}(z - e) + A etabar]
//   eta_i <- rk4 / euler step of d eta / d lambda = A eta + b            (edh.py:266-280)
// One integrator step of an affine field is itself an affine map eta -> Phi eta + psi.  With
// A = Gm H (Gm = -1/2 K S^{-1}, K = P H^T, W = H Gm):
//   rk4:   Phi - I = U H,  U = Gm h (I + h/2 W (I + h/3 W (I + h/4 W))),
//          psi = h b + Gm (h^2/2) (I + h/3 W (I + h/4 W)) H b
//   euler: U = h Gm, psi = h b
// so the whole lambda integration of every particle is ONE affine map of eta0, composed by a
// single workgroup per time step (k_edh_setup, O(L (nx^2 nz + nz^3)) flops):
//   h linear:  eta_L = eta0 + d0 + D (H eta0)   -> the LEDH shared-path table (TLay aff block, theta = 0),
//              consumed unchanged by k_flow_affine (lane groups, L96 d = 40)
//   otherwise: eta_L = M eta0 + d               -> k_flow_edh (one thread per particle, small nx)
// A particle then costs g, its noise, one small mat-vec and the weight of edh.py:287-297
//   l_i = log(w_i + 1e-300) + log N(x_i; g(x_{k-1}), Q) + log N(z; h(x_i), R) - log N(eta0_i; g(x_{k-1}), Q)
// (no Jacobian-determinant term: the global flow's determinant is common to all particles).
// The weight / resample / moment pipeline is LEDH's (identical code in both reference modules).
#pragma once

#include "../../include/pf_edh.h"
#include "pf_ledh_kernels.h"

namespace pf {
namespace ledh {

// general (nonlinear-h) composed map at TLay::aff(L)
template <int NX>
struct ELay {
  static constexpr int EM = 0;           // NX*NX  M
  static constexpr int ED = EM + NX * NX; // NX     d
  static constexpr int SIZE = ED + NX;
};

template <int NX, int NZ, bool LIN>
struct EdhSmem {
  static constexpr int CW = LIN ? NZ : NX;  // columns of the composed matrix (D: NX x NZ, M: NX x NX)
  static constexpr int P = 0;                   // NX*NX  tracker covariance
  static constexpr int R = P + NX * NX;         // NZ*NZ
  static constexpr int H = R + NZ * NZ;         // NZ*NX  Jacobian at etabar
  static constexpr int K = H + NZ * NX;         // NX*NZ  P H^T
  static constexpr int AUG = K + NX * NZ;       // NZ*2NZ [S | I] -> [I | S^{-1}]
  static constexpr int GM = AUG + 2 * NZ * NZ;  // NX*NZ  Gm
  static constexpr int W = GM + NX * NZ;        // NZ*NZ  H Gm
  static constexpr int X3 = W + NZ * NZ;        // NZ*NZ  polynomial scratch
  static constexpr int X2 = X3 + NZ * NZ;       // NZ*NZ
  static constexpr int PW = X2 + NZ * NZ;       // NZ*NZ
  static constexpr int U = PW + NZ * NZ;        // NX*NZ
  static constexpr int CM = U + NX * NZ;        // NX*CW  composed D or M
  static constexpr int HC = CM + NX * CW;       // NZ*CW  H (D or M)
  static constexpr int EB = HC + NZ * CW;       // NX  etabar
  static constexpr int DV = EB + NX;            // NX  d
  static constexpr int CV = DV + NX;            // NX  c = K R^{-1}(z - e)
  static constexpr int T1 = CV + NX;            // NX
  static constexpr int T2 = T1 + NX;            // NX
  static constexpr int BV = T2 + NX;            // NX  b
  static constexpr int PS = BV + NX;            // NX  psi
  static constexpr int HV = PS + NX;            // NZ  h(etabar)
  static constexpr int ZE = HV + NZ;            // NZ  e
  static constexpr int RV = ZE + NZ;            // NZ  R^{-1}(z - e)
  static constexpr int ZT = RV + NZ;            // NZ
  static constexpr int ZB = ZT + NZ;            // NZ  H etabar
  static constexpr int ZD = ZB + NZ;            // NZ  H d
  static constexpr int ZY = ZD + NZ;            // NZ  H b, then the psi polynomial
  static constexpr int FAC = ZY + NZ;           // NZ
  static constexpr int SIZE = FAC + NZ;
};

// C = A B for LDS row-major A [n][m], B [m][k] (block-strided)
__device__ __forceinline__ void lds_gemm(const double* A, const double* B, double* C, int n, int m, int k) {
  for (int q = threadIdx.x; q < n * k; q += blockDim.x) {
    const int r = q / k, c = q - r * k;
    double acc = 0.0;
    for (int e = 0; e < m; ++e) acc += A[r * m + e] * B[e * k + c];
    C[q] = acc;
  }
}

// One workgroup per time step (blockIdx.x): the composed EDH flow map of that step.
// p.Pk / p.z / p.xbar / p.u strided by pk_stride / z_stride / xbar_stride / u_stride (batched over a run).
template <int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(SB) k_edh_setup(FlowParams p, double* table) {
  constexpr bool LIN = (OK == PF_OBS_LINEAR);
  using L = Lay<NX, NZ>;
  using T = TLay<NX, NZ>;
  using SM = EdhSmem<NX, NZ, LIN>;
  constexpr int CW = SM::CW;
  static_assert(SM::SIZE * 8 <= 64 * 1024, "EDH setup LDS");
  __shared__ double sm[SM::SIZE];
  const int t = threadIdx.x;
  const int64_t step = blockIdx.x;
  const double* Pk = p.Pk + step * p.pk_stride;
  const double* zk = p.z + step * p.z_stride;
  const double* xb = p.xbar + step * p.xbar_stride;
  const double* uk = p.u ? p.u + step * p.u_stride : nullptr;
  table += step * p.table_stride;
  double* af = table + T::aff(p.L);
  double* diagS = gridDim.x == 1 ? p.diagS : nullptr;
  const double* __restrict__ Pm = p.Pm;
  double* H = sm + SM::H;
  double* K = sm + SM::K;
  double* aug = sm + SM::AUG;
  double* Gm = sm + SM::GM;
  double* eb = sm + SM::EB;
  for (int q = t; q < NX * NX; q += SB) sm[SM::P + q] = Pk[q];
  for (int q = t; q < NZ * NZ; q += SB) sm[SM::R + q] = Pm[L::R + q];
  for (int d = t; d < NX; d += SB) sm[SM::T1 + d] = xb[d];
  for (int d = t; d < NX; d += SB) sm[SM::DV + d] = 0.0;
  for (int q = t; q < NX * CW; q += SB) sm[SM::CM + q] = LIN ? 0.0 : ((q / NX == q % NX) ? 1.0 : 0.0);
  __syncthreads();
  // etabar = g(x_{k-1|k-1}, u, 0)  (edh.py:213)
  g_block<NX, NZ, TK>(sm + SM::T1, eb, sm + SM::T2, sm + SM::PS, Pm, uk);
  const double h = p.dlam;
  for (int j = 0; j < p.L; ++j) {
    const double lam = p.lams[j];
    // H, h(etabar), e = h(etabar) - H etabar  (edh.py:229-231)
    obs_jac_block<NX, NZ, OK>(eb, H, sm + SM::HV, Pm);
    for (int k = t; k < NZ; k += SB) {
      double acc = 0.0;
      for (int e = 0; e < NX; ++e) acc += H[k * NX + e] * eb[e];
      sm[SM::ZE + k] = sm[SM::HV + k] - acc;
    }
    for (int q = t; q < NX * NZ; q += SB) {  // K = P H^T
      const int d = q / NZ, k = q - d * NZ;
      double acc = 0.0;
      for (int e = 0; e < NX; ++e) acc += sm[SM::P + d * NX + e] * H[k * NX + e];
      K[q] = acc;
    }
    __syncthreads();
    // S = lam H K + R -> [S | I]  (edh.py:236);  r = R^{-1}(z - e)  (edh.py:258)
    for (int q = t; q < NZ * NZ; q += SB) {
      const int k = q / NZ, l = q - k * NZ;
      double acc = 0.0;
      for (int d = 0; d < NX; ++d) acc += H[k * NX + d] * K[d * NZ + l];
      aug[k * 2 * NZ + l] = lam * acc + sm[SM::R + q];
      aug[k * 2 * NZ + NZ + l] = (k == l) ? 1.0 : 0.0;
    }
    for (int k = t; k < NZ; k += SB) {
      double acc = 0.0;
      for (int l = 0; l < NZ; ++l) acc += Pm[L::RI + k * NZ + l] * (zk[l] - sm[SM::ZE + l]);
      sm[SM::RV + k] = acc;
    }
    __syncthreads();
    if (diagS)
      for (int q = t; q < NZ * NZ; q += SB) diagS[(int64_t)j * NZ * NZ + q] = aug[(q / NZ) * 2 * NZ + q % NZ];
    for (int d = t; d < NX; d += SB) {  // c = K r  (edh.py:263)
      double acc = 0.0;
      for (int k = 0; k < NZ; ++k) acc += K[d * NZ + k] * sm[SM::RV + k];
      sm[SM::CV + d] = acc;
    }
    __syncthreads();
    double S_ld;
    int S_sg;
    block_gauss_jordan<NZ>(aug, sm + SM::FAC, &S_ld, &S_sg);
    for (int q = t; q < NX * NZ; q += SB) {  // Gm = -1/2 K S^{-1}  (A = Gm H, edh.py:254)
      const int d = q / NZ, l = q - d * NZ;
      double acc = 0.0;
      for (int k = 0; k < NZ; ++k) acc += K[d * NZ + k] * aug[k * 2 * NZ + NZ + l];
      Gm[q] = -0.5 * acc;
    }
    __syncthreads();
    lds_gemm(H, Gm, sm + SM::W, NZ, NX, NZ);  // W = H Gm
    // b = (I + 2 lam A)[(I + lam A) c + A etabar]  (edh.py:264)
    apply_A<NX, NZ>(H, Gm, eb, sm + SM::ZT, sm + SM::T1);           // A etabar
    apply_A<NX, NZ>(H, Gm, sm + SM::CV, sm + SM::ZT, sm + SM::T2);  // A c
    for (int d = t; d < NX; d += SB) sm[SM::T1 + d] = (sm[SM::CV + d] + lam * sm[SM::T2 + d]) + sm[SM::T1 + d];
    __syncthreads();
    apply_A<NX, NZ>(H, Gm, sm + SM::T1, sm + SM::ZT, sm + SM::T2);
    for (int d = t; d < NX; d += SB) sm[SM::BV + d] = sm[SM::T1 + d] + 2.0 * lam * sm[SM::T2 + d];
    __syncthreads();
    // the integrator step as x -> x + U (H x) + psi
    if (p.integ == PF_EDH_EULER) {
      for (int q = t; q < NX * NZ; q += SB) sm[SM::U + q] = h * Gm[q];
      for (int d = t; d < NX; d += SB) sm[SM::PS + d] = h * sm[SM::BV + d];
      __syncthreads();
    } else {
      // X3 = I + h/4 W ; X2 = I + h/3 W X3 ; PW = h (I + h/2 W X2)
      for (int q = t; q < NZ * NZ; q += SB) sm[SM::X3 + q] = ((q / NZ == q % NZ) ? 1.0 : 0.0) + (0.25 * h) * sm[SM::W + q];
      for (int k = t; k < NZ; k += SB) {  // H b
        double acc = 0.0;
        for (int e = 0; e < NX; ++e) acc += H[k * NX + e] * sm[SM::BV + e];
        sm[SM::ZY + k] = acc;
      }
      __syncthreads();
      lds_gemm(sm + SM::W, sm + SM::X3, sm + SM::PW, NZ, NZ, NZ);
      __syncthreads();
      for (int q = t; q < NZ * NZ; q += SB)
        sm[SM::X2 + q] = ((q / NZ == q % NZ) ? 1.0 : 0.0) + (h / 3.0) * sm[SM::PW + q];
      __syncthreads();
      lds_gemm(sm + SM::W, sm + SM::X2, sm + SM::X3, NZ, NZ, NZ);  // X3 <- W X2
      for (int k = t; k < NZ; k += SB) {  // ZT = (h^2/2) X2 (H b)
        double acc = 0.0;
        for (int l = 0; l < NZ; ++l) acc += sm[SM::X2 + k * NZ + l] * sm[SM::ZY + l];
        sm[SM::ZT + k] = (0.5 * h * h) * acc;
      }
      __syncthreads();
      for (int q = t; q < NZ * NZ; q += SB)
        sm[SM::PW + q] = h * (((q / NZ == q % NZ) ? 1.0 : 0.0) + (0.5 * h) * sm[SM::X3 + q]);
      for (int d = t; d < NX; d += SB) {  // psi = h b + Gm ZT
        double acc = 0.0;
        for (int l = 0; l < NZ; ++l) acc += Gm[d * NZ + l] * sm[SM::ZT + l];
        sm[SM::PS + d] = h * sm[SM::BV + d] + acc;
      }
      __syncthreads();
      lds_gemm(Gm, sm + SM::PW, sm + SM::U, NX, NZ, NZ);  // U = Gm PW
      __syncthreads();
    }
    // compose: etabar, d, D / M   (H of the OLD values first)
    for (int k = t; k < NZ; k += SB) {
      double ab = 0.0, ad = 0.0;
      for (int e = 0; e < NX; ++e) {
        ab += H[k * NX + e] * eb[e];
        ad += H[k * NX + e] * sm[SM::DV + e];
      }
      sm[SM::ZB + k] = ab;
      sm[SM::ZD + k] = ad;
    }
    lds_gemm(H, sm + SM::CM, sm + SM::HC, NZ, NX, CW);
    __syncthreads();
    if constexpr (LIN)  // I + H D
      for (int k = t; k < NZ; k += SB) sm[SM::HC + k * NZ + k] += 1.0;
    __syncthreads();
    for (int d = t; d < NX; d += SB) {
      double ab = 0.0, ad = 0.0;
      for (int l = 0; l < NZ; ++l) {
        const double u = sm[SM::U + d * NZ + l];
        ab += u * sm[SM::ZB + l];
        ad += u * sm[SM::ZD + l];
      }
      eb[d] = (eb[d] + ab) + sm[SM::PS + d];
      sm[SM::DV + d] = (sm[SM::DV + d] + ad) + sm[SM::PS + d];
    }
    for (int q = t; q < NX * CW; q += SB) {
      const int d = q / CW, c = q - d * CW;
      double acc = 0.0;
      for (int l = 0; l < NZ; ++l) acc += sm[SM::U + d * NZ + l] * sm[SM::HC + l * CW + c];
      sm[SM::CM + q] += acc;
    }
    __syncthreads();
  }
  if constexpr (LIN) {
    // eta_L = eta0 + d0 + D y0 ; H eta_L = H d0 + (I + H D) y0 ; theta = 0
    for (int d = t; d < NX; d += SB) af[T::D0 + d] = sm[SM::DV + d];
    for (int q = t; q < NX * NZ; q += SB) af[T::DM + q] = sm[SM::CM + q];
    for (int k = t; k < NZ; k += SB) {
      double acc = 0.0;
      for (int e = 0; e < NX; ++e) acc += Pm[L::H + k * NX + e] * sm[SM::DV + e];
      af[T::PL + k] = acc;
    }
    for (int q = t; q < NZ * NZ; q += SB) {
      const int k = q / NZ, l = q - k * NZ;
      double acc = (k == l) ? 1.0 : 0.0;
      for (int e = 0; e < NX; ++e) acc += Pm[L::H + k * NX + e] * sm[SM::CM + e * NZ + l];
      af[T::QL + q] = acc;
    }
    if (t == 0) af[T::TH] = 0.0;
  } else {
    using E = ELay<NX>;
    for (int q = t; q < NX * NX; q += SB) af[E::EM + q] = sm[SM::CM + q];
    for (int d = t; d < NX; d += SB) af[E::ED + d] = sm[SM::DV + d];
  }
}

// h(x) of one particle in registers
template <int NX, int NZ, int OK>
__device__ __forceinline__ void h_thread(const double* x, const double* __restrict__ Pm, double* hv) {
  using L = Lay<NX, NZ>;
  if constexpr (OK == PF_OBS_LINEAR) {
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
      double acc = 0.0;
#pragma unroll
      for (int e = 0; e < NX; ++e) acc += Pm[L::H + k * NX + e] * x[e];
      hv[k] = acc + Pm[L::C + k];
    }
  } else if constexpr (OK == PF_OBS_EXP_HALF) {
#pragma unroll
    for (int k = 0; k < NZ; ++k) hv[k] = Pm[L::C + k] * exp(0.5 * x[k]);
  } else {
    const double psi = Pm[L::AC], d0 = Pm[L::AC + 1];
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
      const double sx = Pm[L::AC + 2 + k], sy = Pm[L::AC + 2 + NZ + k];
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < NX / 4; ++c) {
        const double dx = x[4 * c] - sx, dy = x[4 * c + 1] - sy;
        acc += psi / ((dx * dx + dy * dy) + d0);
      }
      hv[k] = acc;
    }
  }
}

// One thread per particle: eta0 = g(x) + v, x_k = M eta0 + d, weight (edh.py:287-297).
template <int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(TB) k_flow_edh(FlowParams p) {
  using L = Lay<NX, NZ>;
  using T = TLay<NX, NZ>;
  using E = ELay<NX>;
  const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
  if (i >= p.N) return;
  const double* __restrict__ Pm = p.Pm;
  const double* __restrict__ af = p.table + T::aff(p.L);
  double gx[NX], v[NX];
#pragma unroll
  for (int d = 0; d < NX; ++d) gx[d] = p.x_in[(int64_t)d * p.Npad + i];
  g_thread<NX, NZ, TK>(gx, Pm, p.u);
  noise_thread<NX, NZ>(p, i, v);
  double e0[NX], dd[NX];
#pragma unroll
  for (int d = 0; d < NX; ++d) e0[d] = gx[d] + v[d];
  double xk[NX];
#pragma unroll
  for (int d = 0; d < NX; ++d) {
    double acc = af[E::ED + d];
#pragma unroll
    for (int e = 0; e < NX; ++e) acc += af[E::EM + d * NX + e] * e0[e];
    xk[d] = acc;
    dd[d] = acc - gx[d];
    p.x_out[(int64_t)d * p.Npad + i] = acc;
  }
  const bool qd = p.q_diag != 0;
  const double num_t = -0.5 * quad_form<NX>(dd, Pm + L::QI, qd);
  const double den_t = -0.5 * quad_form<NX>(v, Pm + L::QI, qd);
  double hv[NZ];
  h_thread<NX, NZ, OK>(xk, Pm, hv);
#pragma unroll
  for (int k = 0; k < NZ; ++k) hv[k] = p.z[k] - hv[k];
  const double like = -0.5 * quad_form<NZ>(hv, Pm + L::RI, p.r_diag != 0);
  p.lw[i] = log(p.w_in[i] + 1e-300) + ((num_t + like) - den_t);
}

}  // namespace ledh
}  // namespace pf
