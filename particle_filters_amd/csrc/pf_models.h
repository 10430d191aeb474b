// Device-side state-space models (the g / h plugin surface of the reference,
// particle_filter.py:20-22, made compile-time so a particle's state lives in
// registers for the whole step).
//
//   transition kinds (g):  PF_TRANS_LINEAR  x' = A x (+ u)         SV alpha*x, CV blocks, test systems
//                          PF_TRANS_L96     one RK4 step of Lorenz-96 (simulator_Lorenz_96.py:35-84)
//   observation kinds (h): PF_OBS_LINEAR    z = H x + c            SV log-squared, L96 x[::k], linear tests
//                          PF_OBS_EXP_HALF  z_k = beta_k exp(x_k/2) SV standard / test-harness wiring
//                          PF_OBS_ACOUSTIC  z_s = sum_c psi/(|p_c - s|^2 + d0)  (simulator_Multi_acoustic_tracking.py:273-309)
//                          PF_OBS_SV_EXACT  the exact SV likelihood y_k ~ N(0, beta_k^2 e^{x_k}):
//                                           log p = -x/2 - y^2 e^{-x} / (2 beta^2) (+ const)
//                                           (tests/integration_tests/test_dpf_vs_sv_simulator.py:60-97)
//
// Parameters live in one read-only array (uniform across the grid -> scalar
// loads) laid out by ParamLayout<NX, NZ>, in the engine's compute precision.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/pf_engine.h"

namespace pf {

template <int NX, int NZ>
struct ParamLayout {
  static constexpr int A = 0;                // NX*NX  transition matrix (row-major)
  static constexpr int LQ = A + NX * NX;     // NX*NX  chol(Q) (predict, +1e-10 I fallback)
  static constexpr int LJ = LQ + NX * NX;     // NX*NX  0.001*chol(Q) (jitter, +1e-12 I fallback)
  static constexpr int H = LJ + NX * NX;     // NZ*NX  observation matrix
  static constexpr int C = H + NZ * NX;      // NZ     observation offset (LINEAR) / beta (EXP_HALF)
  static constexpr int LR = C + NZ;          // NZ*NZ  chol(R + 1e-12 I)
  static constexpr int EX = LR + NZ * NZ;    // model extras: L96 {F, dt}; ACOUSTIC {psi, d0, sx[NZ], sy[NZ]}
  static constexpr int ILR = EX + 2 + 2 * NZ; // NZ     1 / diag(LR) (fp32 engine multiplies)
  static constexpr int SIZE = ILR + NZ;
};

template <typename Real, int NX, int NZ, int TK, int OK>
struct Model {
  using L = ParamLayout<NX, NZ>;
  static constexpr int nx = NX;
  static constexpr int nz = NZ;

  // ---- g ------------------------------------------------------------------
  __device__ static __forceinline__ void l96_rhs(const Real* x, Real* out, Real F) {
#pragma unroll
    for (int a = 0; a < NX; ++a) {
      const Real xp1 = x[(a + 1) % NX];
      const Real xm1 = x[(a + NX - 1) % NX];
      const Real xm2 = x[(a + NX - 2) % NX];
      out[a] = (xp1 - xm2) * xm1 - x[a] + F;
    }
  }

  __device__ static __forceinline__ void transition(Real* x, const Real* __restrict__ P,
                                                    const Real* u) {
    if constexpr (TK == PF_TRANS_LINEAR) {
      Real y[NX];
#pragma unroll
      for (int d = 0; d < NX; ++d) {
        Real acc = Real(0);
#pragma unroll
        for (int e = 0; e < NX; ++e) acc += P[L::A + d * NX + e] * x[e];
        y[d] = acc;
      }
#pragma unroll
      for (int d = 0; d < NX; ++d) x[d] = u ? y[d] + u[d] : y[d];
    } else {  // PF_TRANS_L96: x + dt/6 (k1 + 2k2 + 2k3 + k4)
      const Real F = P[L::EX + 0], dt = P[L::EX + 1];
      Real k[NX], acc[NX], tmp[NX];
      l96_rhs(x, k, F);
#pragma unroll
      for (int a = 0; a < NX; ++a) { acc[a] = k[a]; tmp[a] = x[a] + Real(0.5) * dt * k[a]; }
      l96_rhs(tmp, k, F);
#pragma unroll
      for (int a = 0; a < NX; ++a) { acc[a] += Real(2) * k[a]; tmp[a] = x[a] + Real(0.5) * dt * k[a]; }
      l96_rhs(tmp, k, F);
#pragma unroll
      for (int a = 0; a < NX; ++a) { acc[a] += Real(2) * k[a]; tmp[a] = x[a] + dt * k[a]; }
      l96_rhs(tmp, k, F);
      const Real h6 = dt / Real(6);
#pragma unroll
      for (int a = 0; a < NX; ++a) x[a] = x[a] + h6 * (acc[a] + k[a]);
    }
  }

  // ---- h ------------------------------------------------------------------
  __device__ static __forceinline__ void observe(const Real* x, Real* zp, const Real* __restrict__ P) {
    if constexpr (OK == PF_OBS_SV_EXACT) {  // the observation scale beta e^{x/2} (no Gaussian h)
#pragma unroll
      for (int k = 0; k < NZ; ++k) zp[k] = P[L::C + k] * exp(Real(0.5) * x[k]);
    } else if constexpr (OK == PF_OBS_LINEAR) {
#pragma unroll
      for (int k = 0; k < NZ; ++k) {
        Real acc = Real(0);
#pragma unroll
        for (int d = 0; d < NX; ++d) acc += P[L::H + k * NX + d] * x[d];
        zp[k] = acc + P[L::C + k];
      }
    } else if constexpr (OK == PF_OBS_EXP_HALF) {
      static_assert(NX == NZ, "EXP_HALF observes every state component");
#pragma unroll
      for (int k = 0; k < NZ; ++k) zp[k] = P[L::C + k] * exp(Real(0.5) * x[k]);
    } else {  // PF_OBS_ACOUSTIC, targets are consecutive [x, y, vx, vy] blocks
      static_assert(NX % 4 == 0, "acoustic state is 4 per target");
      const Real psi = P[L::EX + 0], d0 = P[L::EX + 1];
#pragma unroll
      for (int s = 0; s < NZ; ++s) {
        const Real sx = P[L::EX + 2 + s], sy = P[L::EX + 2 + NZ + s];
        Real acc = Real(0);
#pragma unroll
        for (int c = 0; c < NX / 4; ++c) {
          const Real dx = x[4 * c] - sx, dy = x[4 * c + 1] - sy;
          acc += psi / ((dx * dx + dy * dy) + d0);
        }
        zp[s] = acc;
      }
    }
  }

  // ---- Gaussian log-likelihood: -0.5 |LR^{-1} (z - h(x))|^2 (particle_filter.py:257-261)
  __device__ static __forceinline__ Real loglik(const Real* x, const Real* z, const Real* __restrict__ P,
                                                bool r_diag) {
    if constexpr (OK == PF_OBS_SV_EXACT) {
      // -0.5 sum_k (x_k + y_k^2 e^{-x_k} / beta_k^2): the reference test's log N(y; 0, (beta e^{x/2})^2)
      // without its constants (pf.py drops the Gaussian constants the same way).  fp32: the product
      // is one exp of (log(y^2/beta^2) - x), so a far-negative x gives -inf (weight 0) rather than
      // inf * 0; an all -inf step is caught by the all-dead guard (PF_E_NAN).
      static_assert(NX == NZ, "SV_EXACT observes every state component");
      Real quad = Real(0);
#pragma unroll
      for (int k = 0; k < NZ; ++k) {
        const Real b = P[L::C + k];
        if constexpr (sizeof(Real) == 4) {
          const Real c = __logf((z[k] * z[k]) / (b * b));  // per step, hoisted out of the particle loop
          quad += x[k] + __expf(c - x[k]);
        } else {
          quad += x[k] + z[k] * z[k] * exp(-x[k]) / (b * b);
        }
      }
      return Real(-0.5) * quad;
    }
    Real zp[NZ];
    observe(x, zp, P);
    Real y[NZ];
    Real quad = Real(0);
    if (NZ == 1 || r_diag) {
#pragma unroll
      for (int k = 0; k < NZ; ++k) {
        if constexpr (sizeof(Real) == 4)
          y[k] = (z[k] - zp[k]) * P[L::ILR + k];  // fp32: reciprocal multiply
        else
          y[k] = (z[k] - zp[k]) / P[L::LR + k * NZ + k];  // fp64: the reference's division
        quad += y[k] * y[k];
      }
    } else {  // forward substitution with the lower-triangular LR
#pragma unroll
      for (int k = 0; k < NZ; ++k) {
        Real acc = z[k] - zp[k];
#pragma unroll
        for (int m = 0; m < k; ++m) acc -= P[L::LR + k * NZ + m] * y[m];
        y[k] = acc / P[L::LR + k * NZ + k];
        quad += y[k] * y[k];
      }
    }
    return Real(-0.5) * quad;
  }

  // noise = L n  with L lower triangular (reference: n @ L.T)
  __device__ static __forceinline__ void add_lower(Real* x, const Real* n, const Real* __restrict__ P,
                                                   int off) {
#pragma unroll
    for (int d = 0; d < NX; ++d) {
      Real acc = Real(0);
#pragma unroll
      for (int e = 0; e <= d; ++e) acc += n[e] * P[off + d * NX + e];
      x[d] = x[d] + acc;
    }
  }
};

}  // namespace pf
