// k_step for large states (L96 nx = 40, joint acoustic nx = 16): one particle per
// GROUP of GL = 4 lanes, each lane owning PER = nx / 4 contiguous state components.
//
// Why: with one particle per thread an nx = 40 RK4 step keeps ~160 live values per
// lane; the compiler spilled (256 VGPR + 223 AGPR + scratch, occupancy 1).  Spread
// over 4 lanes a particle costs ~40 live values per lane, so several waves per SIMD
// hide the Philox -> g -> h -> weight latency chain and the 4x more lanes fill the chip.
// Cross-lane work is small and stays in registers:
//   * L96 RK4 stages need x[a+1], x[a-1], x[a-2] across a lane boundary: 3 shuffles;
//   * dense A x, chol(Q) n (when chol(Q) is not block-diagonal in the lanes' blocks):
//     the components are streamed through shuffles (group_rows);
//   * h(x) partial sums over a lane's components + a 2-step xor all-reduce; the
//     Gaussian quadratic form is then evaluated redundantly in the 4 lanes.
// Everything else — prologue, outputs, systematic/multinomial ancestors, the tile
// records — is k_step's (pf_kernels.h), with the weighted sums reduced per lane
// class (q = lane % GL) so that each component lands in its record field.
#pragma once
#include "pf_kernels.h"

namespace pf {

#ifndef PF_GRP_WPE
#define PF_GRP_WPE 4
#endif
#ifndef PF_GRP_WPE_SMALL
#define PF_GRP_WPE_SMALL 4
#endif
#ifndef PF_GRP_RCP
#define PF_GRP_RCP 1
#endif
constexpr int SYS_STAGE = 4;  // source tiles of a block's systematic positions staged in LDS (sys_cdf)

template <int NX>
struct SGrp {
  // lanes per particle: 8 for nx >= 32 (L96: 5 components per lane), else 4 (MAT: one target per lane)
  static constexpr int GL = (NX >= 32 && NX % 8 == 0) ? 8 : 4;
  static constexpr bool ON = NX >= 16 && NX % GL == 0;
  static constexpr int PER = NX / GL;
};

// normals of the flat indices f0 .. f0+PER-1 (f = particle * NX + component): the same
// Philox counters as fill_normals of the one-thread-per-particle kernels
template <typename Real, int PER>
__device__ __forceinline__ void grp_normals(uint64_t seed, int64_t f0, uint32_t rep, uint32_t ep, uint32_t stream,
                                            Real* n) {
  constexpr int GMAX = PER / 4 + 2;
  const int64_t g0 = f0 >> 2, g1 = (f0 + PER - 1) >> 2;
  const int sh = (int)(f0 & 3);
#pragma unroll
  for (int gg = 0; gg < GMAX; ++gg) {
    if (g0 + gg <= g1) {
      const Normal4<Real> q4 = normal4<Real>(seed, (uint32_t)(g0 + gg), rep, ep, stream);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < PER; ++j)
          if (4 * gg + e - sh == j) n[j] = q4.v[e];
    }
  }
}

template <int GL, typename Real>
__device__ __forceinline__ Real gsum(Real v) {
#pragma unroll
  for (int o = 1; o < GL; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// acc[j] += sum_e C[a_j][e] vec_e (e <= a_j if lower), vec distributed over the group
template <typename Real, int NX>
__device__ __forceinline__ void grp_rows(const Real* loc, const Real* __restrict__ C, int q, int base, Real* acc,
                                         bool lower) {
  constexpr int PER = SGrp<NX>::PER, SGL = SGrp<NX>::GL;
#pragma unroll
  for (int r = 0; r < SGL; ++r) {
#pragma unroll
    for (int jj = 0; jj < PER; ++jj) {
      const Real val = __shfl(loc[jj], base + r);
      const int e = r * PER + jj;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int a = q * PER + j;
        if (!lower || e <= a) acc[j] += C[a * NX + e] * val;
      }
    }
  }
}

// x += L n for lower-triangular L at P[off]; `local`: L is block-diagonal in the lanes' blocks
template <typename Real, int NX, bool LOCAL>
__device__ __forceinline__ void grp_add_lower(Real* x, const Real* n, const Real* __restrict__ P, int off, int q,
                                              int base) {
  constexpr int PER = SGrp<NX>::PER;
  Real acc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) acc[j] = Real(0);
  if constexpr (LOCAL) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int a = q * PER + j;
#pragma unroll
      for (int jj = 0; jj <= j; ++jj) acc[j] += P[off + a * NX + q * PER + jj] * n[jj];
    }
  } else {
    grp_rows<Real, NX>(n, P + off, q, base, acc, true);
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) x[j] = x[j] + acc[j];
}

// LOCAL: A is block-diagonal in the lanes' blocks (the joint MAT model's per-target constant-
// velocity blocks): each lane applies its own PER x PER block, no shuffles
template <typename Real, int NX, int NZ, int TK, bool LOCAL>
__device__ __forceinline__ void grp_transition(Real* x, const Real* __restrict__ P, const Real* u, int q, int base) {
  using L = ParamLayout<NX, NZ>;
  constexpr int PER = SGrp<NX>::PER, SGL = SGrp<NX>::GL;
  if constexpr (TK == PF_TRANS_LINEAR) {
    Real y[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) y[j] = Real(0);
    if constexpr (LOCAL) {
#pragma unroll
      for (int j = 0; j < PER; ++j)
#pragma unroll
        for (int jj = 0; jj < PER; ++jj) y[j] += P[L::A + (q * PER + j) * NX + q * PER + jj] * x[jj];
    } else {
      grp_rows<Real, NX>(x, P + L::A, q, base, y, false);
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) x[j] = u ? y[j] + u[q * PER + j] : y[j];
  } else {  // L96 RK4 (simulator_Lorenz_96.py:62-84), neighbours across lanes by shuffles
    static_assert(PER >= 2, "L96 lanes hold >= 2 components");
    const Real F = P[L::EX + 0], dt = P[L::EX + 1];
    const int nxt = base + (q + 1) % SGL, prv = base + (q + SGL - 1) % SGL;
    auto rhs = [&](const Real* y, Real* k) {
      const Real n0 = __shfl(y[0], nxt);
      const Real p1 = __shfl(y[PER - 1], prv);
      const Real p2 = __shfl(y[PER - 2], prv);
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const Real yp1 = j + 1 < PER ? y[j + 1] : n0;
        const Real ym1 = j >= 1 ? y[j - 1] : p1;
        const Real ym2 = j >= 2 ? y[j - 2] : (j == 1 ? p1 : p2);
        k[j] = (yp1 - ym2) * ym1 - y[j] + F;
      }
    };
    Real k[PER], acc[PER], tmp[PER];
    rhs(x, k);
#pragma unroll
    for (int j = 0; j < PER; ++j) { acc[j] = k[j]; tmp[j] = x[j] + Real(0.5) * dt * k[j]; }
    rhs(tmp, k);
#pragma unroll
    for (int j = 0; j < PER; ++j) { acc[j] += Real(2) * k[j]; tmp[j] = x[j] + Real(0.5) * dt * k[j]; }
    rhs(tmp, k);
#pragma unroll
    for (int j = 0; j < PER; ++j) { acc[j] += Real(2) * k[j]; tmp[j] = x[j] + dt * k[j]; }
    rhs(tmp, k);
    const Real h6 = dt / Real(6);
#pragma unroll
    for (int j = 0; j < PER; ++j) x[j] = x[j] + h6 * (acc[j] + k[j]);
    if (u) {
#pragma unroll
      for (int j = 0; j < PER; ++j) x[j] += u[q * PER + j];
    }
  }
}

// -1/2 |LR^{-1}(z - h(x))|^2 (particle_filter.py:257-261), same value in the 4 lanes; z in LDS.
//   LINEAR:   partial H x over the lane's components for every k at once, all-reduced with
//             independent (pipelined) shuffles.
//   ACOUSTIC: the targets' positions are all-gathered (2 shuffles per other lane) and each
//             lane evaluates the full h for the sensors s = q (mod 4), so no per-sensor
//             reduction; the partial quadratic form is all-reduced once.
//   EXP_HALF: each lane owns its components' observations.
// RD (diagonal R): the quadratic form is a sum over k; otherwise forward substitution
// with LR over the all-reduced residual.
template <typename Real, int NX, int NZ, int OK, bool RD>
__device__ __forceinline__ Real grp_loglik(const Real* x, const Real* z, const Real* __restrict__ P, int q, int base) {
  using L = ParamLayout<NX, NZ>;
  constexpr int PER = SGrp<NX>::PER, SGL = SGrp<NX>::GL;
  auto ylin = [&](int k, Real zp) -> Real {  // diagonal-R residual scaled by 1/LR_kk
    if constexpr (sizeof(Real) == 4)
      return (z[k] - zp) * P[L::ILR + k];
    else
      return (z[k] - zp) / P[L::LR + k * NZ + k];
  };
  if constexpr (OK == PF_OBS_ACOUSTIC && (NZ == 1 || RD)) {
    static_assert(PER % 4 == 0, "acoustic lanes own whole targets");
    constexpr int TPL = PER / 4;  // targets per lane
    Real px[SGL * TPL], py[SGL * TPL];
#pragma unroll
    for (int r = 0; r < SGL; ++r)
#pragma unroll
      for (int c = 0; c < TPL; ++c) {
        px[r * TPL + c] = __shfl(x[4 * c], base + r);
        py[r * TPL + c] = __shfl(x[4 * c + 1], base + r);
      }
    const Real psi = P[L::EX + 0], d0 = P[L::EX + 1];
    Real quad = Real(0);
    for (int k = q; k < NZ; k += SGL) {
      const Real sx = P[L::EX + 2 + k], sy = P[L::EX + 2 + NZ + k];
      Real zp = Real(0);
#pragma unroll
      for (int c = 0; c < SGL * TPL; ++c) {
        const Real dx = px[c] - sx, dy = py[c] - sy;
#if PF_GRP_RCP
        if constexpr (sizeof(Real) == 4)  // fp32 engine: v_rcp_f32 (1 ulp) instead of the IEEE division sequence
          zp += psi * __builtin_amdgcn_rcpf((dx * dx + dy * dy) + d0);
        else
#endif
          zp += psi / ((dx * dx + dy * dy) + d0);
      }
      const Real y = ylin(k, zp);
      quad += y * y;
    }
    return Real(-0.5) * gsum<SGL>(quad);
  } else {
    Real zp[NZ];
    if constexpr (OK == PF_OBS_LINEAR) {
#pragma unroll 2
      for (int k = 0; k < NZ; ++k) {  // (a rolled loop keeps only one H row of loads in flight)
        Real acc = Real(0);
#pragma unroll
        for (int j = 0; j < PER; ++j) acc += P[L::H + k * NX + q * PER + j] * x[j];
        zp[k] = acc;
      }
#pragma unroll
      for (int o = 1; o < SGL; o <<= 1)
#pragma unroll
        for (int k = 0; k < NZ; ++k) zp[k] += __shfl_xor(zp[k], o);
#pragma unroll
      for (int k = 0; k < NZ; ++k) zp[k] += P[L::C + k];
    } else if constexpr (OK == PF_OBS_ACOUSTIC) {
      const Real psi = P[L::EX + 0], d0 = P[L::EX + 1];
#pragma unroll
      for (int k = 0; k < NZ; ++k) {
        const Real sx = P[L::EX + 2 + k], sy = P[L::EX + 2 + NZ + k];
        Real acc = Real(0);
#pragma unroll
        for (int c = 0; c < PER / 4; ++c) {
          const Real dx = x[4 * c] - sx, dy = x[4 * c + 1] - sy;
          acc += psi / ((dx * dx + dy * dy) + d0);
        }
        zp[k] = gsum<SGL>(acc);
      }
    } else {  // EXP_HALF (nz == nx)
      static_assert(NX == NZ, "EXP_HALF observes every component");
#pragma unroll
      for (int k = 0; k < NZ; ++k) {
        Real acc = Real(0);
#pragma unroll
        for (int j = 0; j < PER; ++j)
          if (q * PER + j == k) acc = P[L::C + k] * exp(Real(0.5) * x[j]);
        zp[k] = gsum<SGL>(acc);
      }
    }
    Real quad = Real(0);
    if constexpr (NZ == 1 || RD) {
#pragma unroll
      for (int k = 0; k < NZ; ++k) {
        const Real y = ylin(k, zp[k]);
        quad += y * y;
      }
    } else {
      Real y[NZ];
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
}

// selection h with diagonal R: each observation is ONE component owned by one lane, so a lane
// adds the residuals of its own observed components and the group sums the partial quadratic
// form (3 shuffles instead of the H-row partials + an NZ-wide all-reduce)
template <typename Real, int NX, int NZ>
__device__ __forceinline__ Real grp_loglik_sel(const Real* x, const Real* z, const Real* __restrict__ P, int q,
                                               const int32_t* hcol2k) {
  using L = ParamLayout<NX, NZ>;
  constexpr int PER = SGrp<NX>::PER, SGL = SGrp<NX>::GL;
  Real quad = Real(0);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int k = hcol2k[q * PER + j];
    if (k >= 0) {
      const Real zp = x[j] + P[L::C + k];
      Real y;
      if constexpr (sizeof(Real) == 4) y = (z[k] - zp) * P[L::ILR + k];
      else y = (z[k] - zp) / P[L::LR + k * NZ + k];
      quad += y * y;
    }
  }
  return Real(-0.5) * gsum<SGL>(quad);
}

// weighted accumulator of one lane: online max, s0, s00 and its PER components' s1
template <typename Real, int NX>
struct GAcc {
  static constexpr int PER = SGrp<NX>::PER, SGL = SGrp<NX>::GL;
  static constexpr int NS = 2 + NX;  // record fields S0, S00, S1[NX]
  Real m, s0, s00, s1[PER];
  __device__ __forceinline__ void init() {
    m = -INFINITY;
    s0 = s00 = Real(0);
#pragma unroll
    for (int j = 0; j < PER; ++j) s1[j] = Real(0);
  }
  __device__ __forceinline__ void add(Real l, const Real* x) {
    if (!(l > -INFINITY)) return;
    if (l > m) {
      if (m > -INFINITY) {
        const Real f = exp_r<Real>(m - l);
        s0 *= f;
        s00 *= f * f;
#pragma unroll
        for (int j = 0; j < PER; ++j) s1[j] *= f;
      }
      m = l;
    }
    const Real e = exp_r<Real>(l - m);
    s0 += e;
    s00 += e * e;
#pragma unroll
    for (int j = 0; j < PER; ++j) s1[j] += e * x[j];
  }
  // block merge, max first, straight into the staged tile record `fin` (LDS, by thread 0)
  template <int BS>
  __device__ __forceinline__ void block_merge(double* red, double* fin) {
    using RC = Rec<NX>;
    constexpr int NW = BS / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane % SGL;
    const double md = (double)m;
    // the lane maxima are Real values: for fp32 the DPP max of the floats (the same value as the
    // shuffle butterfly over their doubles, without the LDS-crossbar round trips)
    const double Mw = sizeof(Real) == 4 ? (double)wave_max_u((float)m) : wave_max(md);
    const double f = (md > -INFINITY) ? exp(md - Mw) : 0.0;
    double v0 = (double)s0 * f, v1 = (double)s00 * f * f, vj[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) vj[j] = (double)s1[j] * f;
    // sum over the lanes of one class q (one lane per group): xor offsets SGL .. 32
#pragma unroll
    for (int o = 32; o >= SGL; o >>= 1) {
      v0 += __shfl_xor(v0, o);
      v1 += __shfl_xor(v1, o);
#pragma unroll
      for (int j = 0; j < PER; ++j) vj[j] += __shfl_xor(vj[j], o);
    }
    __syncthreads();
    if (lane < SGL) {
      double* rw = red + w * (NS + 1);
      if (q == 0) {
        rw[0] = Mw;
        rw[1] = v0;
        rw[2] = v1;
      }
#pragma unroll
      for (int j = 0; j < PER; ++j) rw[3 + q * PER + j] = vj[j];
    }
    __syncthreads();
    if (w != 0) return;
    // wave 0: the global max, then lane i sums field i over the NW wave partials (fixed order)
    double M = -INFINITY;
#pragma unroll
    for (int j = 0; j < NW; ++j) M = fmax(M, red[j * (NS + 1)]);
    for (int i = lane; i < NS; i += 64) {
      double sv = 0.0;
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        const double mj = red[j * (NS + 1)];
        const double fj = (mj > -INFINITY) ? exp(mj - M) : 0.0;
        sv += red[j * (NS + 1) + 1 + i] * (i == 1 ? fj * fj : fj);
      }
      fin[i == 0 ? RC::S0 : (i == 1 ? RC::S00 : RC::S1 + i - 2)] = sv;
    }
    if (lane == 0) {
      fin[RC::M] = M;
      fin[RC::UNI] = 0.0;
    }
  }
};

// RD: R diagonal (the likelihood streams over k); QL: chol(Q), the jitter factor and (linear g)
// A are block-diagonal in the lanes' blocks (noise and transition are lane-local).  Variants picked on the host.
// The fp32 L96-size variant with diagonal R and lane-local noise fits 128 VGPRs: keep
// it at 4 waves per SIMD (the others need more registers than that).
template <typename Real, int NX, int NZ, int TK, int OK, bool RD, bool QL>
constexpr int grp_waves_per_eu = (sizeof(Real) == 4 && RD && QL) ? (NX >= 32 ? PF_GRP_WPE : PF_GRP_WPE_SMALL) : 1;

template <typename Real, int NX, int NZ, int TK, int OK, bool RD, bool QL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(grp_waves_per_eu<Real, NX, NZ, TK, OK, RD, QL>)))
k_step_grp(StepParams p) {
  using M = Model<Real, NX, NZ, TK, OK>;
  using RC = Rec<NX>;
  using GA = GAcc<Real, NX>;
  constexpr int SGL = SGrp<NX>::GL, BS = 256, VB = BS / SGL, PER = SGrp<NX>::PER;
  static_assert(SGrp<NX>::ON && !RC::COV, "group step is for large states");
  static_assert((BS / 64) * (GA::NS + 1) <= LDS_RED, "scratch too small");
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  double* Pl = smem + LDS_PL;
  double* cdf = smem + lds_tile(p.G);
  int* anc_l = (int*)(cdf + p.tile);

  const int b = blockIdx.x, r = blockIdx.y, R = gridDim.y;
  const int t = threadIdx.x, q = t % SGL, vt = t / SGL;
  const int lane = t & 63, base = lane - q;
  const Real* __restrict__ P = (const Real*)p.P;
  const Real* x_in = (const Real*)p.x_in + (int64_t)r * NX * p.Npad;
  Real* x_out = (Real*)p.x_out + (int64_t)r * NX * p.Npad;
  const Real* lw_in = (const Real*)p.lw_in + (int64_t)r * p.Npad;
  Real* lw_out = (Real*)p.lw_out + (int64_t)r * p.Npad;
  const double* rec_in = p.rec_in + (int64_t)r * RC::SIZE * p.G;
  const int64_t o0 = (int64_t)b * p.tile;
  const int64_t o1 = min(o0 + (int64_t)p.tile, p.N);
  const int nchunks = (int)(o1 - o0);
  const uint32_t rep = (uint32_t)(r + p.rep_base);
  const Real* u = p.u ? (const Real*)p.u + (int64_t)r * p.u_rs : nullptr;
  __shared__ Real z[NZ];  // the observation, read per particle from LDS (not held in registers)
  if (p.do_update)
    for (int k = t; k < NZ; k += BS) z[k] = ((const Real*)p.z)[(int64_t)r * p.z_rs + k];

  // ---- (0) prologue / outputs (k_step's) ----------------------------------------
  const bool stamp_on = p.do_predict && p.do_update;
  (void)stamp_on;
  PF_STAMP(0);
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

  // ---- (1) ancestors of the tile's slots (lane 0 of each group) ---------------
  if (gather) {
    if (p.method == 0 && p.sys_cdf) {
      // the tile of pos from the prefix Pl, then the slot inside that tile's span of the CDF that
      // k_cdf materialised (tile_cdf arithmetic: the same ancestors as the per-tile path below).
      // The source tiles of this block's (monotone) positions are staged in LDS when they are few.
      const double U = p.rp_unif ? p.rp_unif[r] : uniform53(p.seed, 0, rep, p.ep_resample);
      // the CDF: materialised by k_cdf (C), or built on the fly from the in-tile prefix the
      // previous launch left (L): cdf[j] = P_k + c_k L[j], c_k = e^(m_k - M) / S (tile_cdf's
      // arithmetic, so both give the same doubles)
      const double* C = p.lcum_in ? nullptr : p.cdf + (int64_t)r * p.N;
      const double* Lc = p.lcum_in ? p.lcum_in + (int64_t)r * p.N : nullptr;
      auto ck = [&](int k) {
        const double mk = rec_in[RC::M * p.G + k];
        return (mk > -INFINITY) ? exp(mk - h.M) / h.Sscan : 0.0;
      };
      __shared__ int krange[2];
      __shared__ double cks[SYS_STAGE];  // c_k of the staged source tiles (one fp64 exp per tile)
      if (t < 64) {  // wave 0: the first and last source tile by two lanes at once, then their c_k
        int kk = 0;
        if (lane < 2) kk = prefix_tile(Pl, p.G, (U + (double)(lane == 0 ? o0 : o1 - 1)) / (double)p.N);
        const int klo_ = __shfl(kk, 0), khi_ = __shfl(kk, 1);
        if (lane == 0) {
          krange[0] = klo_;
          krange[1] = khi_;
        }
        if (Lc && lane < SYS_STAGE && klo_ + lane <= khi_) cks[lane] = ck(klo_ + lane);
      }
      __syncthreads();
      const int klo = krange[0], nk = krange[1] - krange[0] + 1;
      const bool staged = nk <= SYS_STAGE;
      double* stg = (double*)(anc_l + ((p.tile + 1) & ~1));  // SYS_STAGE * tile doubles (step_lds)
      if (staged)
        for (int e = t; e < nk * p.tile; e += BS) {
          const int64_t g = (int64_t)klo * p.tile + e;
          if (Lc) {
            const int kq = e / p.tile;
            stg[e] = g < p.N ? Pl[klo + kq] + cks[kq] * Lc[g] : INFINITY;
          } else {
            stg[e] = g < p.N ? C[g] : INFINITY;
          }
        }
      __syncthreads();
      for (int c = t; c < nchunks; c += BS) {  // every lane takes a slot (independent searches)
          const double pos = (U + (double)(o0 + c)) / (double)p.N;
          const int k = prefix_tile(Pl, p.G, pos);
          const int64_t s0 = (int64_t)k * p.tile;
          const int len = (int)min((int64_t)p.tile, p.N - s0);
          int lo = 0, hi = len;
          if (staged && k >= klo && k < klo + nk) {
            const double* cs = stg + (int64_t)(k - klo) * p.tile;
            while (lo < hi) {
              const int mid = (lo + hi) >> 1;
              if (pos < cs[mid]) hi = mid; else lo = mid + 1;
            }
          } else if (Lc) {
            const double bk = Pl[k], cc = ck(k);
            while (lo < hi) {
              const int mid = (lo + hi) >> 1;
              if (pos < bk + cc * Lc[s0 + mid]) hi = mid; else lo = mid + 1;
            }
          } else {
            while (lo < hi) {
              const int mid = (lo + hi) >> 1;
              if (pos < C[s0 + mid]) hi = mid; else lo = mid + 1;
            }
          }
          anc_l[c] = (int)(s0 + (lo < len ? lo : len - 1));
        }
    } else if (p.method == 0) {
      const double U = p.rp_unif ? p.rp_unif[r] : uniform53(p.seed, 0, rep, p.ep_resample);
      int nextk = p.G;
      if (q == 0)
        for (int c = vt; c < nchunks; c += VB) {
          const int64_t i = o0 + c;
          const int k = prefix_tile(Pl, p.G, (U + (double)i) / (double)p.N);
          anc_l[c] = -1 - k;
          nextk = min(nextk, k);
        }
      int k = block_min_i<BS>(nextk, red);
      while (k < p.G) {
        const int len = tile_cdf<Real, NX, BS>(lw_in, rec_in, p.G, p.N, p.tile, k, h, Pl, cdf, red);
        nextk = p.G;
        if (q == 0)
          for (int c = vt; c < nchunks; c += VB) {
            const int64_t i = o0 + c;
            const int a = anc_l[c];
            if (a == -1 - k) {
              anc_l[c] = (int)((int64_t)k * p.tile + lds_upper(cdf, len, (U + (double)i) / (double)p.N));
            } else if (a < 0) {
              nextk = min(nextk, -1 - a);
            }
          }
        __syncthreads();
        k = block_min_i<BS>(nextk, red);
      }
    } else {
      const double* C = p.cdf + (int64_t)r * p.N;
      const double last = C[p.N - 1];
      if (q == 0)
        for (int c = vt; c < nchunks; c += VB) {
          const int64_t i = o0 + c;
          const double uu = p.rp_unif ? p.rp_unif[(int64_t)r * p.N + i] : uniform53(p.seed, (uint32_t)i, rep, p.ep_resample);
          int64_t lo = 0, hi = p.N;
          while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (uu < C[mid] / last) hi = mid; else lo = mid + 1;
          }
          anc_l[c] = (int)(lo < p.N ? lo : p.N - 1);
        }
    }
    __syncthreads();
  }

  PF_STAMP(3);
  // ---- (2)+(3) per particle: [gather + jitter] -> [predict] -> [weight] -> store ---
  GA acc;
  acc.init();
  double aux0 = 0.0, auxj[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) auxj[j] = 0.0;
  const double lse_prev = h.uniform ? 0.0 : (p.use_lse_ext ? p.lse_ext : h.lse);  // shards: the global lse
  const Real lse_r = (Real)lse_prev;
  const bool write_x = p.do_predict || p.allow_gather;
  for (int c = vt; c < nchunks; c += VB) {
    // keep the per-lane model parameters (H rows, chol(Q) blocks, A rows) in L1 rather than
    // hoisted into ~100 VGPRs across the loop: that hoisting cost 3 of 4 waves per SIMD
    asm volatile("" ::: "memory");
    const int64_t i = o0 + c;
    Real x[PER];
    Real lp = Real(0);
    if (gather) {
      const int a = anc_l[c];
#pragma unroll
      for (int j = 0; j < PER; ++j) x[j] = x_in[(int64_t)(q * PER + j) * p.Npad + a];
      lp = (Real)lprev_uniform;
      if (p.regularize) {
        Real n[PER];
        if (p.rp_jit) {
#pragma unroll
          for (int j = 0; j < PER; ++j) n[j] = (Real)p.rp_jit[((int64_t)r * p.N + i) * NX + q * PER + j];
        } else {
          grp_normals<Real, PER>(p.seed, (i + p.pbase) * NX + q * PER, rep, p.ep_resample, STREAM_JITTER, n);
        }
        grp_add_lower<Real, NX, QL>(x, n, P, M::L::LJ, q, base);
      }
      aux0 += 1.0;
#pragma unroll
      for (int j = 0; j < PER; ++j) auxj[j] += (double)x[j];
      if (p.anc_out) {  // the post-resample rows for the device loop's covariance (pf_cov.h): by index
        if (q == 0) p.anc_out[(int64_t)r * p.N + i] = a;
      } else if (p.xr_out) {  // ... or (jittered) by value
        Real* xr = (Real*)p.xr_out + (int64_t)r * NX * p.Npad;
#pragma unroll
        for (int j = 0; j < PER; ++j) xr[(int64_t)(q * PER + j) * p.Npad + i] = x[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < PER; ++j) x[j] = x_in[(int64_t)(q * PER + j) * p.Npad + i];
      if (p.do_update) lp = h.uniform ? (Real)lprev_uniform : lw_in[i] - lse_r;
    }
    if (p.do_predict) {
      Real n[PER];
      if (p.rp_noise) {
#pragma unroll
        for (int j = 0; j < PER; ++j) n[j] = (Real)p.rp_noise[((int64_t)r * p.N + i) * NX + q * PER + j];
      } else {
        grp_normals<Real, PER>(p.seed, (i + p.pbase) * NX + q * PER, rep, p.ep_predict, STREAM_PROCESS, n);
      }
      grp_transition<Real, NX, NZ, TK, QL>(x, P, u, q, base);
      grp_add_lower<Real, NX, QL>(x, n, P, M::L::LQ, q, base);
    }
    if (p.do_update) {
      Real ll = Real(0);
      if (p.do_update == 1) {
        if constexpr (OK == PF_OBS_LINEAR && RD && NX <= 64) {
          if (p.h_sel) ll = grp_loglik_sel<Real, NX, NZ>(x, z, P, q, p.hcol2k);
          else ll = grp_loglik<Real, NX, NZ, OK, RD>(x, z, P, q, base);
        } else {
          ll = grp_loglik<Real, NX, NZ, OK, RD>(x, z, P, q, base);
        }
      }
      lp = lp + ll;
      acc.add(lp, x);
    }
    if (write_x)
#pragma unroll
      for (int j = 0; j < PER; ++j) x_out[(int64_t)(q * PER + j) * p.Npad + i] = x[j];
    if (p.do_update && q == 0) lw_out[i] = lp;
  }

  PF_STAMP(4);
  // ---- (4) this tile's partial record (field-major) -----------------------------
  if (!(p.do_update || p.allow_gather)) return;
  double* rec_out = p.rec_out + (int64_t)r * RC::SIZE * p.G;
  double* fin = cdf;  // staged record
  __syncthreads();
  if (p.do_update) {
    acc.template block_merge<BS>(red, fin);
  } else if (t == 0) {
    if (gather) {
      fin[RC::M] = 0.0; fin[RC::S0] = 0.0; fin[RC::S00] = 0.0; fin[RC::UNI] = 1.0;
      for (int k = RC::S1; k < RC::A1; ++k) fin[k] = 0.0;
    } else {
      for (int k = 0; k < RC::A1; ++k) fin[k] = rec_in[k * p.G + b];
    }
  }
  if (gather) {  // aux: count and unweighted sums of the resampled particles, per lane class
#pragma unroll
    for (int o = 32; o >= SGL; o >>= 1) {
      aux0 += __shfl_xor(aux0, o);
#pragma unroll
      for (int j = 0; j < PER; ++j) auxj[j] += __shfl_xor(auxj[j], o);
    }
    __syncthreads();
    const int w = t >> 6;
    if (lane < SGL) {
      double* rw = red + w * (1 + NX);
      if (q == 0) rw[0] = aux0;
#pragma unroll
      for (int j = 0; j < PER; ++j) rw[1 + q * PER + j] = auxj[j];
    }
    __syncthreads();
    for (int k = t; k < 1 + NX; k += BS) {
      double s = 0.0;
      for (int ww = 0; ww < BS / 64; ++ww) s += red[ww * (1 + NX) + k];
      if (k == 0) fin[RC::CNT] = s;
      else fin[RC::A1 + k - 1] = s;
    }
  } else if (t == 0) {
    fin[RC::CNT] = 0.0;
    for (int k = RC::A1; k < RC::SIZE; ++k) fin[k] = 0.0;
  }
  __syncthreads();
  PF_STAMP(5);
  for (int k = t; k < RC::SIZE; k += BS) rec_out[k * p.G + b] = fin[k];
  if (p.lcum_out && p.do_update) {
    // the in-tile prefix of the new weights, exactly as tile_cdf (k_cdf) sums them: thread t owns
    // the contiguous elements [t per, t per + per), block exclusive scan, then the running sum.
    // lw_out of this tile was written above by this workgroup (visible after the barrier).
    const int64_t s0 = o0;
    const int len = nchunks;
    const int per = (len + BS - 1) / BS;
    const int j0 = t * per;
    const double mk = fin[RC::M];
    const Real m = (Real)mk;
    double accs = 0.0;
    for (int j = j0; j < j0 + per && j < len; ++j) {
      const Real l = lw_out[s0 + j];
      accs += (l > -INFINITY) ? (double)exp_r<Real>(l - m) : 0.0;
    }
    double tot;
    double off = block_excl_scan<BS>(accs, red, &tot);
    double* Lo = p.lcum_out + (int64_t)r * p.N + s0;
    for (int j = j0; j < j0 + per && j < len; ++j) {
      const Real l = lw_out[s0 + j];
      off += (l > -INFINITY) ? (double)exp_r<Real>(l - m) : 0.0;
      Lo[j] = off;
    }
  }
}

}  // namespace pf
