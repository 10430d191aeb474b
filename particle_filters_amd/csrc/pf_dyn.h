// Runtime-shape SIR kernels: any (nx, nz) for every g / h kind, for the models outside the
// compiled (nx, nz, g, h) list of pf_inst_*.hip — the reference's ParticleFilter takes
// arbitrary shapes (particle_filter.py:79-107; simulate_lorenz96 defaults to nx = 1000,
// simulator_Lorenz_96.py:299-300; the 9-D bearings-only SIR of SPF_results_reproduction_
// example2.ipynb cell 7).
//
// Same step protocol, records, heads, Philox counters and CDF search as k_step
// (pf_kernels.h), so every host path of pf_engine.hip (predict / update / resample / run /
// replay / shards / moments) drives these kernels unchanged.  What differs is where a
// particle lives during the step: k_step keeps its NX components in registers (NX is a
// template argument), here nx is a kernel argument, so a thread walks its particle's column
// of the structure-of-arrays state in HBM (x[d][i], coalesced across the wave for every d)
// and keeps the RK4 stages / normals / whitened residuals in a per-replicate scratch
// `wbuf` [rows][Npad] of the same layout.  The tile record's moment fields are reduced
// after the particle loop, one field per wave (lanes stride the tile's particles, one
// wave_sum), from the tile's freshly written rows (L2-hot).
//
// Layout (runtime DynLay / DynRec = ParamLayout<nx, nz> / Rec<nx> with the same offsets).
#pragma once
#include "pf_dyn_layout.h"
#include "pf_kernels.h"

namespace pf {

// pair index c of the upper triangle (d <= e), the order of Rec's S2 / A2 fields
__device__ __forceinline__ void tri_pair(int c, int nx, int& d, int& e) {
  d = 0;
  while (c >= nx - d) {
    c -= nx - d;
    ++d;
  }
  e = d + c;
}

// Normals of one particle in flat order f = (i + pbase) * nx + d (fill_normals' numbering:
// Philox group f >> 2, element f & 3), or the replayed host draws [lrep][N][nx].
template <typename Real>
struct NStream {
  uint64_t seed;
  int64_t f;
  uint32_t rep, ep, stream, g;
  const double* rp;
  int64_t ri;
  bool have;
  Normal4<Real> q;
  __device__ __forceinline__ NStream(uint64_t seed_, int64_t i, int nx, uint32_t lrep, uint32_t rep_, uint32_t ep_,
                                     uint32_t stream_, const double* replay, int64_t N, int64_t pbase)
      : seed(seed_), f((i + pbase) * nx), rep(rep_), ep(ep_), stream(stream_), g(0), rp(replay),
        ri(((int64_t)lrep * N + i) * nx), have(false) {}
  __device__ __forceinline__ Real next() {
    if (rp) return (Real)rp[ri++];
    const uint32_t gg = (uint32_t)(f >> 2);
    if (!have || gg != g) {
      q = normal4<Real>(seed, gg, rep, ep, stream);
      g = gg;
      have = true;
    }
    const int j = (int)(f++ & 3);
    return j == 0 ? q.v[0] : j == 1 ? q.v[1] : j == 2 ? q.v[2] : q.v[3];
  }
};

// x[d] += sum_{e <= d} Lf[d][e] n_e on the column x (stride S); the normals go through the
// scratch column w unless Lf is diagonal.  Model::add_lower's summation order.
template <typename Real>
__device__ __forceinline__ void dyn_add_lower(Real* x, Real* w, int64_t S, int nx, const Real* __restrict__ Lf,
                                              bool diag, NStream<Real>& ns) {
  if (diag) {
    for (int d = 0; d < nx; ++d) {
      const Real n = ns.next();
      Real acc = Real(0);
      acc += n * Lf[d * nx + d];
      x[d * S] = x[d * S] + acc;
    }
    return;
  }
  for (int e = 0; e < nx; ++e) w[e * S] = ns.next();
  for (int d = 0; d < nx; ++d) {
    Real acc = Real(0);
    for (int e = 0; e <= d; ++e) acc += w[e * S] * Lf[d * nx + e];
    x[d * S] = x[d * S] + acc;
  }
}

template <typename Real>
__device__ __forceinline__ Real l96_rhs_at(const Real* v, int64_t S, int nx, int a, Real F) {
  const int ap1 = a + 1 < nx ? a + 1 : a + 1 - nx;
  const int am1 = a >= 1 ? a - 1 : a - 1 + nx;
  const int am2 = a >= 2 ? a - 2 : a - 2 + nx;
  return (v[ap1 * S] - v[am2 * S]) * v[am1 * S] - v[a * S] + F;
}

// g: src -> dst (columns of stride S; dst may be src).  Model::transition's arithmetic.
template <typename Real, int TK>
__device__ __forceinline__ void dyn_transition(const Real* src, Real* dst, Real* w, int64_t S, int nx,
                                               const Real* __restrict__ P, const DynLay& L, const Real* u,
                                               bool a_diag) {
  if constexpr (TK == PF_TRANS_LINEAR) {
    if (a_diag) {
      for (int d = 0; d < nx; ++d) {
        Real acc = Real(0);
        acc += P[L.A + d * nx + d] * src[d * S];
        dst[d * S] = u ? acc + u[d] : acc;
      }
      return;
    }
    Real* y = (src == dst) ? w : dst;
    for (int d = 0; d < nx; ++d) {
      Real acc = Real(0);
      for (int e = 0; e < nx; ++e) acc += P[L.A + d * nx + e] * src[e * S];
      y[d * S] = u ? acc + u[d] : acc;
    }
    if (y != dst)
      for (int d = 0; d < nx; ++d) dst[d * S] = y[d * S];
  } else {  // PF_TRANS_L96: x + dt/6 (k1 + 2k2 + 2k3 + k4); scratch rows T1 | K | ACC
    const Real F = P[L.EX + 0], dt = P[L.EX + 1];
    Real* T1 = w;
    Real* K = w + (int64_t)nx * S;
    Real* AC = w + 2 * (int64_t)nx * S;
    for (int a = 0; a < nx; ++a) {
      const Real k = l96_rhs_at(src, S, nx, a, F);
      AC[a * S] = k;
      T1[a * S] = src[a * S] + Real(0.5) * dt * k;
    }
    for (int stage = 0; stage < 2; ++stage) {  // k2 then k3; T1 <- x + 0.5 dt k2, then x + dt k3
      for (int a = 0; a < nx; ++a) {
        const Real k = l96_rhs_at(T1, S, nx, a, F);
        AC[a * S] = AC[a * S] + Real(2) * k;
        K[a * S] = k;
      }
      if (stage == 0)
        for (int a = 0; a < nx; ++a) T1[a * S] = src[a * S] + Real(0.5) * dt * K[a * S];
      else
        for (int a = 0; a < nx; ++a) T1[a * S] = src[a * S] + dt * K[a * S];
    }
    const Real h6 = dt / Real(6);
    for (int a = 0; a < nx; ++a) {
      const Real k = l96_rhs_at(T1, S, nx, a, F);
      dst[a * S] = src[a * S] + h6 * (AC[a * S] + k);
    }
  }
}

// h_k(x) (Model::observe), k < nz
template <typename Real, int OK>
__device__ __forceinline__ Real dyn_observe(const Real* x, int64_t S, int nx, int k, const Real* __restrict__ P,
                                            const DynLay& L, bool h_sel) {
  if constexpr (OK == PF_OBS_LINEAR) {
    if (h_sel) {  // H row k selects component col_k (P[EX + 2 + k]): H x = x[col_k] exactly
      const int col = (int)P[L.EX + 2 + k];
      return x[col * S] + P[L.C + k];
    }
    Real acc = Real(0);
    for (int d = 0; d < nx; ++d) acc += P[L.H + k * nx + d] * x[d * S];
    return acc + P[L.C + k];
  } else if constexpr (OK == PF_OBS_EXP_HALF) {
    return P[L.C + k] * exp(Real(0.5) * x[k * S]);
  } else if constexpr (OK == PF_OBS_ACOUSTIC) {
    const Real psi = P[L.EX + 0], d0 = P[L.EX + 1];
    const int nzz = (L.ILR - L.EX - 2) / 2;
    const Real sx = P[L.EX + 2 + k], sy = P[L.EX + 2 + nzz + k];
    Real acc = Real(0);
    for (int c = 0; c < nx / 4; ++c) {
      const Real dx = x[(4 * c) * S] - sx, dy = x[(4 * c + 1) * S] - sy;
      acc += psi / ((dx * dx + dy * dy) + d0);
    }
    return acc;
  } else {  // PF_OBS_BEARINGS: azimuth atan2(x - sx, y - sy), elevation atan2(z - sz, |(x, y) - s|)
    const Real dx = x[0] - P[L.EX + 2], dy = x[S] - P[L.EX + 3];
    if (k == 0) return atan2(dx, dy);
    const Real dz = x[2 * S] - P[L.EX + 4];
    return atan2(dz, sqrt(dx * dx + dy * dy));
  }
}

// -0.5 |LR^{-1} (z - h(x))|^2 (Model::loglik; SV_EXACT: -0.5 sum x + y^2 e^{-x} / beta^2)
template <typename Real, int OK>
__device__ __forceinline__ Real dyn_loglik(const Real* x, Real* w, int64_t S, int nx, int nz, const Real* z,
                                           const Real* __restrict__ P, const DynLay& L, bool r_diag, bool h_sel) {
  Real quad = Real(0);
  if constexpr (OK == PF_OBS_SV_EXACT) {
    for (int k = 0; k < nz; ++k) {
      const Real b = P[L.C + k];
      const Real xk = x[k * S];
      if constexpr (sizeof(Real) == 4) {
        const Real c = __logf((z[k] * z[k]) / (b * b));
        quad += xk + __expf(c - xk);
      } else {
        quad += xk + z[k] * z[k] * exp(-xk) / (b * b);
      }
    }
    return Real(-0.5) * quad;
  }
  if (nz == 1 || r_diag) {
    for (int k = 0; k < nz; ++k) {
      const Real zp = dyn_observe<Real, OK>(x, S, nx, k, P, L, h_sel);
      Real y;
      if constexpr (sizeof(Real) == 4)
        y = (z[k] - zp) * P[L.ILR + k];
      else
        y = (z[k] - zp) / P[L.LR + k * nz + k];
      quad += y * y;
    }
  } else {  // forward substitution with the lower-triangular LR, residuals in the scratch column
    for (int k = 0; k < nz; ++k) {
      Real acc = z[k] - dyn_observe<Real, OK>(x, S, nx, k, P, L, h_sel);
      for (int m = 0; m < k; ++m) acc -= P[L.LR + k * nz + m] * w[m * S];
      const Real y = acc / P[L.LR + k * nz + k];
      w[k * S] = y;
      quad += y * y;
    }
  }
  return Real(-0.5) * quad;
}

// Sum over the tile's particles c in [0, n) of val(c), one value per lane stride, wave-reduced:
// every lane of the wave gets the total.
template <typename F>
__device__ __forceinline__ double wave_tile_sum(int n, int lane, F val) {
  double s = 0.0;
  for (int c = lane; c < n; c += 64) s += val(c);
  return wave_sum(s);
}

// write_outputs (pf_kernels.h) for a runtime nx: the same outputs from the same record fields.
template <int BS>
__device__ __forceinline__ void write_outputs_dyn(const StepParams& p, const double* rec, const DynRec& RC, const Head& h, int r, int R,
                                  int blk, int nblk, double* red) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  constexpr int NW = BS / 64;
  const int G = p.G, nx = RC.nx;
  const bool pre = p.out_step >= 0 && !h.uniform;
  const bool want_post = p.out_post_step >= 0;
  if (!pre && !want_post) return;
  if (pre && blk == 0 && t == 0) {
    const int64_t o = p.out_step * R + r;
    p.o_neff[o] = h.neff;
    p.o_lse[o] = h.lse;
    p.o_flag[o] = h.resample;
  }
  if (RC.cov) {
    if (blk != 0) return;
    const int NF = nx + RC.nc;
    double v[2 * DYN_NFM + 1];
#pragma unroll
    for (int f = 0; f < 2 * DYN_NFM + 1; ++f) v[f] = 0.0;
    for (int k = t; k < G; k += BS) {
      if (pre) {
        const double s0 = rec[1 * G + k];
        if (s0 > 0.0) {
          const double fk = exp(rec[k] - h.M);
#pragma unroll
          for (int f = 0; f < DYN_NFM; ++f)
            if (f < NF) v[f] += rec[(RC.S1 + f) * G + k] * fk;
        }
      }
      if (want_post) {
        v[2 * DYN_NFM] += rec[4 * G + k];
#pragma unroll
        for (int f = 0; f < DYN_NFM; ++f)
          if (f < NF) v[DYN_NFM + f] += rec[(RC.A1 + f) * G + k];
      }
    }
    block_sum_k<2 * DYN_NFM + 1, BS>(v, red);
    if (t != 0) return;
    // runtime-indexed below: staged in LDS past the reduction scratch (keeps v in registers)
    double* vs = red + 256;
#pragma unroll
    for (int f = 0; f < 2 * DYN_NFM + 1; ++f) vs[f] = v[f];
    const double cnt = v[2 * DYN_NFM];
    for (int pass = 0; pass < 2; ++pass) {
      if (pass == 0 ? !pre : !(want_post && cnt > 0.0)) continue;
      const int64_t o = (pass == 0 ? p.out_step : p.out_post_step) * R + r;
      const double* m = vs + pass * DYN_NFM;
      const double den = pass == 0 ? h.S : cnt;
      for (int d = 0; d < nx; ++d) p.o_mean[o * nx + d] = m[d] / den;
      if (p.o_cov) {
        int c = 0;
        for (int d = 0; d < nx; ++d)
          for (int e = d; e < nx; ++e, ++c) {
            const double val = m[nx + c] / den - (m[d] / den) * (m[e] / den);
            p.o_cov[o * nx * nx + d * nx + e] = val;
            p.o_cov[o * nx * nx + e * nx + d] = val;
          }
      }
    }
    return;
  }
  if (blk >= 2 * nx) return;  // no field of this workgroup
  // fields f = blk + nblk * j of this workgroup, field j on wave j % NW; every wave that has one
  // counts the freshly resampled particles itself (no block barrier)
  double cnt = 0.0;
  if (want_post) cnt = wave_tile_sum(G, lane, [&](int k) { return rec[4 * G + k]; });
  const bool post = want_post && cnt > 0.0;
  int j = w;
  for (int f = blk + nblk * w; f < 2 * nx; f += nblk * NW, j += NW) {
    const bool is_post = f >= nx;
    if (is_post ? !post : !pre) continue;
    const int d = is_post ? f - nx : f;
    const double acc = wave_tile_sum(G, lane, [&](int k) {
      if (is_post) return rec[(RC.A1 + d) * G + k];
      const double s0 = rec[1 * G + k];
      return s0 > 0.0 ? rec[(RC.S1 + d) * G + k] * exp(rec[k] - h.M) : 0.0;
    });
    if (lane == 0) {
      const int64_t o = (is_post ? p.out_post_step : p.out_step) * R + r;
      p.o_mean[o * nx + d] = acc / (is_post ? cnt : h.S);
    }
  }
}

// ---------------------------------------------------------------------------
// The step: [prologue] -> [ancestors] -> A: [gather + jitter, aux moments] -> B: [predict,
// weight] -> [tile record].  k_step's phases and StepParams semantics.
// ---------------------------------------------------------------------------
template <typename Real, int TK, int OK>
__global__ void __launch_bounds__(DBS) k_dyn_step(StepParams p) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  double* Pl = smem + LDS_PL;
  double* cdf = smem + lds_tile(p.G);
  int* anc_l = (int*)(cdf + p.tile);
  const int nx = p.dnx, nz = p.dnz;
  const DynRec RC(nx);
  const DynLay L(nx, nz);
  const int b = blockIdx.x, r = blockIdx.y, R = gridDim.y;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  constexpr int NW = DBS / 64;
  const int64_t S = p.Npad;
  const Real* __restrict__ P = (const Real*)p.P;
  const Real* x_in = (const Real*)p.x_in + (int64_t)r * nx * S;
  Real* x_out = (Real*)p.x_out + (int64_t)r * nx * S;
  const Real* lw_in = (const Real*)p.lw_in + (int64_t)r * S;
  Real* lw_out = (Real*)p.lw_out + (int64_t)r * S;
  const double* rec_in = p.rec_in + (int64_t)r * RC.SIZE * p.G;
  double* rec_out = p.rec_out + (int64_t)r * RC.SIZE * p.G;
  Real* W = (Real*)p.wbuf + (int64_t)r * p.wrows * S;
  const int64_t o0 = (int64_t)b * p.tile;
  const int64_t o1 = min(o0 + (int64_t)p.tile, p.N);
  const int n = (int)(o1 - o0);
  const uint32_t rep = (uint32_t)(r + p.rep_base);
  const Real* z = (const Real*)p.z + (int64_t)r * p.z_rs;
  const Real* u = p.u ? (const Real*)p.u + (int64_t)r * p.u_rs : nullptr;

  // ---- (0) prologue (the record heads, fields 0..3, do not depend on nx) --------
  Head h;
  if (p.head) {
    h = load_head<DBS>(p.head, r, p.G, p.allow_gather != 0 && p.method == 0, Pl);
  } else {
    h = prologue<1, DBS>(rec_in, p.G, p.N, p.thresh, p.allow_gather != 0, p.force_gather != 0,
                         p.allow_gather != 0 && p.method == 0, red, Pl);
    write_outputs_dyn<DBS>(p, rec_in, RC, h, r, R, b, p.G, red);
  }
  const bool gather = h.resample != 0;
  const double lprev_uniform = -log((double)p.N);

  // ---- (1) ancestors of the tile's slots (k_step's search) ------------------------
  if (gather) {
    if (p.method == 0) {
      const double U = p.rp_unif ? p.rp_unif[r] : uniform53(p.seed, 0, rep, p.ep_resample);
      int nextk = p.G;
      for (int c = t; c < n; c += DBS) {
        const int64_t i = o0 + c;
        const int k = prefix_tile(Pl, p.G, (U + (double)i) / (double)p.N);
        anc_l[c] = -1 - k;
        nextk = min(nextk, k);
      }
      int k = block_min_i<DBS>(nextk, red);
      while (k < p.G) {
        const int len = tile_cdf<Real, 1, DBS>(lw_in, rec_in, p.G, p.N, p.tile, k, h, Pl, cdf, red);
        nextk = p.G;
        for (int c = t; c < n; c += DBS) {
          const int a = anc_l[c];
          if (a == -1 - k) {
            anc_l[c] = (int)((int64_t)k * p.tile + lds_upper(cdf, len, (U + (double)(o0 + c)) / (double)p.N));
          } else if (a < 0) {
            nextk = min(nextk, -1 - a);
          }
        }
        __syncthreads();
        k = block_min_i<DBS>(nextk, red);
      }
    } else {
      const double* Cf = p.cdf + (int64_t)r * p.N;
      const double last = Cf[p.N - 1];
      for (int c = t; c < n; c += DBS) {
        const int64_t i = o0 + c;
        const double uu = p.rp_unif ? p.rp_unif[(int64_t)r * p.N + i] : uniform53(p.seed, (uint32_t)i, rep, p.ep_resample);
        int64_t lo = 0, hi = p.N;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (uu < Cf[mid] / last) hi = mid; else lo = mid + 1;
        }
        anc_l[c] = (int)(lo < p.N ? lo : p.N - 1);
      }
    }
  }

  // ---- A: gather + jitter into x_out, then the resampled particles' aux moments ----
  if (gather) {
    const bool ldiag = p.lj_diag != 0;
    for (int c = t; c < n; c += DBS) {
      const int64_t i = o0 + c;
      const int a = anc_l[c];
      Real* xo = x_out + i;
      for (int d = 0; d < nx; ++d) xo[d * S] = x_in[d * S + a];
      if (p.regularize) {
        NStream<Real> ns(p.seed, i, nx, (uint32_t)r, rep, p.ep_resample, STREAM_JITTER, p.rp_jit, p.N, p.pbase);
        dyn_add_lower<Real>(xo, W + i, S, nx, P + L.LJ, ldiag, ns);
      }
      if (p.anc_out) {  // the post-resample rows for the device loop's covariance (pf_cov.h): by index
        p.anc_out[(int64_t)r * p.N + i] = a;
      } else if (p.xr_out) {  // ... or (jittered) by value
        Real* xr = (Real*)p.xr_out + (int64_t)r * nx * S + i;
        for (int d = 0; d < nx; ++d) xr[d * S] = xo[d * S];
      }
    }
    __syncthreads();  // the tile's gathered rows are complete
    const int nfa = 1 + nx + RC.nc;
    for (int f = wv; f < nfa; f += NW) {
      double s;
      if (f == 0) {
        s = (double)n;
      } else if (f <= nx) {
        const Real* row = x_out + (int64_t)(f - 1) * S + o0;
        s = wave_tile_sum(n, lane, [&](int c) { return (double)row[c]; });
      } else {
        int d, e;
        tri_pair(f - 1 - nx, nx, d, e);
        const Real* rd = x_out + (int64_t)d * S + o0;
        const Real* re = x_out + (int64_t)e * S + o0;
        s = wave_tile_sum(n, lane, [&](int c) { return (double)rd[c] * (double)re[c]; });
      }
      if (lane == 0) rec_out[(f == 0 ? 4 : RC.A1 + f - 1) * p.G + b] = s;
    }
  }

  // ---- B: predict + weight ---------------------------------------------------------
  const double lse_prev = h.uniform ? 0.0 : (p.use_lse_ext ? p.lse_ext : h.lse);
  const Real lse_r = (Real)lse_prev;
  const bool write_x = p.do_predict || p.allow_gather;
  const bool adiag = p.a_diag != 0, qdiag = p.lq_diag != 0;
  // where the particle is after this phase: x_out when written, else still x_in
  const Real* cur = write_x ? x_out : x_in;
  for (int c = t; c < n; c += DBS) {
    const int64_t i = o0 + c;
    Real* xo = x_out + i;
    const Real* src = gather ? xo : x_in + i;
    if (p.do_predict) {
      dyn_transition<Real, TK>(src, xo, W + i, S, nx, P, L, u, adiag);
      NStream<Real> ns(p.seed, i, nx, (uint32_t)r, rep, p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, p.pbase);
      dyn_add_lower<Real>(xo, W + i, S, nx, P + L.LQ, qdiag, ns);
    } else if (write_x && !gather) {
      for (int d = 0; d < nx; ++d) xo[d * S] = src[d * S];
    }
    if (p.do_update) {
      Real lp;
      if (gather || h.uniform) lp = (Real)lprev_uniform;
      else lp = lw_in[i] - lse_r;
      const Real ll = (p.do_update == 1)
                          ? dyn_loglik<Real, OK>(cur + i, W + i, S, nx, nz, z, P, L, p.r_diag != 0, p.h_sel != 0)
                          : Real(0);
      lw_out[i] = lp + ll;
    }
  }

  // ---- (4) the tile record ---------------------------------------------------------
  if (!(p.do_update || p.allow_gather)) return;
  const int G = p.G;
  if (p.do_update) {
    __syncthreads();  // the tile's weights and rows are complete
    double* wl = cdf;  // e^(l - m) per particle of the tile (the tile area is free again)
    double lm = -INFINITY;
    for (int c = t; c < n; c += DBS) {
      const Real l = lw_out[o0 + c];
      if (l > -INFINITY) lm = fmax(lm, (double)l);
    }
    const double m = block_max<DBS>(lm, red);
    double s[2] = {0.0, 0.0};
    for (int c = t; c < n; c += DBS) {
      const Real l = lw_out[o0 + c];
      const double e = (l > -INFINITY) ? exp((double)l - m) : 0.0;
      wl[c] = e;
      s[0] += e;
      s[1] += e * e;
    }
    block_sum_k<2, DBS>(s, red);  // its barriers also publish wl
    if (t == 0) {
      rec_out[0 * G + b] = m;
      rec_out[1 * G + b] = s[0];
      rec_out[2 * G + b] = s[1];
      rec_out[3 * G + b] = 0.0;
    }
    const int nf = nx + RC.nc;
    for (int f = wv; f < nf; f += NW) {
      double v;
      if (f < nx) {
        const Real* row = cur + (int64_t)f * S + o0;
        v = wave_tile_sum(n, lane, [&](int c) { return wl[c] * (double)row[c]; });
      } else {
        int d, e;
        tri_pair(f - nx, nx, d, e);
        const Real* rd = cur + (int64_t)d * S + o0;
        const Real* re = cur + (int64_t)e * S + o0;
        v = wave_tile_sum(n, lane, [&](int c) { return wl[c] * (double)rd[c] * (double)re[c]; });
      }
      if (lane == 0) rec_out[(RC.S1 + f) * G + b] = v;
    }
  } else if (gather) {  // gather-only launch: weights become uniform
    for (int q = t; q < RC.A1; q += DBS)
      if (q != 4) rec_out[q * G + b] = (q == 3) ? 1.0 : 0.0;
  } else {  // gather-only launch that did not resample: carry the update's record over
    for (int q = t; q < RC.A1; q += DBS)
      if (q != 4) rec_out[q * G + b] = rec_in[q * G + b];
  }
  if (!gather) {
    if (t == 0) rec_out[4 * G + b] = 0.0;
    for (int q = RC.A1 + t; q < RC.SIZE; q += DBS) rec_out[q * G + b] = 0.0;
  }
}

// posterior outputs of the records in rec_in (one workgroup per replicate; k_finalize)
__global__ void __launch_bounds__(DBS) k_dyn_finalize(StepParams p) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int r = blockIdx.x, R = gridDim.x;
  const DynRec RC(p.dnx);
  const double* rec = p.rec_in + (int64_t)r * RC.SIZE * p.G;
  const Head h = prologue<1, DBS>(rec, p.G, p.N, p.thresh, p.allow_gather != 0, false, false, smem, nullptr);
  write_outputs_dyn<DBS>(p, rec, RC, h, r, R, 0, 1, smem);
}

// the fp64 CDF of the update in rec_in (k_cdf)
template <typename Real>
__global__ void __launch_bounds__(DBS) k_dyn_cdf(StepParams p, double* cdf_out) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  double* Pl = smem + LDS_PL;
  double* cdf = smem + lds_tile(p.G);
  const int b = blockIdx.x, r = blockIdx.y;
  const double* rec = p.rec_in + (int64_t)r * DynRec(p.dnx).SIZE * p.G;
  const Head h = p.head ? load_head<DBS>(p.head, r, p.G, true, Pl)
                        : prologue<1, DBS>(rec, p.G, p.N, p.thresh, true, p.force_gather != 0, true, red, Pl);
  if (!h.resample) return;
  const Real* lw = (const Real*)p.lw_in + (int64_t)r * p.Npad;
  const int len = tile_cdf<Real, 1, DBS>(lw, rec, p.G, p.N, p.tile, b, h, Pl, cdf, red);
  for (int j = threadIdx.x; j < len; j += DBS) cdf_out[(int64_t)r * p.N + (int64_t)b * p.tile + j] = cdf[j];
}

// per-replicate heads (k_head)
__global__ void __launch_bounds__(DBS) k_dyn_head(StepParams p, double* head) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  double* Pl = smem + LDS_PL;
  const int b = blockIdx.x, r = blockIdx.y, R = gridDim.y;
  const DynRec RC(p.dnx);
  const double* rec = p.rec_in + (int64_t)r * RC.SIZE * p.G;
  const bool allow = p.allow_gather != 0;
  const Head h = prologue<1, DBS>(rec, p.G, p.N, p.thresh, allow, p.force_gather != 0, allow, red, Pl);
  write_outputs_dyn<DBS>(p, rec, RC, h, r, R, b, gridDim.x, red);
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
    for (int k = threadIdx.x; k <= p.G; k += DBS) o[HEAD_F + k] = Pl[k];
}

// initialize(): x = mean + chol(cov) n (k_init).  The normals are written into the particle's
// column first; row d is then finished from the last row up, so the normals of rows e <= d
// are still in place when row d reads them.
template <typename Real>
__global__ void __launch_bounds__(DBS) k_dyn_init(Real* x, double* rec, const Real* mean, const Real* Lc,
                                                  const double* replay, int64_t N, int64_t Npad, int G, uint64_t seed,
                                                  uint32_t epoch, int rep_base, int64_t pbase, int nx,
                                                  int lc_diag) {
  const DynRec RC(nx);
  const int r = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * DBS + threadIdx.x;
  if (i < N) {
    Real* xc = x + (int64_t)r * nx * Npad + i;
    NStream<Real> ns(seed, i, nx, (uint32_t)r, (uint32_t)(r + rep_base), epoch, STREAM_INIT, replay, N, pbase);
    for (int d = 0; d < nx; ++d) xc[d * Npad] = ns.next();
    const Real* L = Lc + (int64_t)r * nx * nx;
    for (int d = nx - 1; d >= 0; --d) {
      Real acc = Real(0);
      for (int e = lc_diag ? d : 0; e <= d; ++e) acc += xc[e * Npad] * L[d * nx + e];  // (zeros add exactly)
      xc[d * Npad] = acc + mean[r * nx + d];
    }
  }
  if (i < G) {
    double* o = rec + (int64_t)r * RC.SIZE * G;
    for (int q = 0; q < RC.SIZE; ++q) o[(int64_t)q * G + i] = 0.0;
    o[(int64_t)3 * G + i] = 1.0;
  }
}

// exact two-pass weighted moments (k_mom_mean / k_mom_cov)
template <typename Real>
__global__ void __launch_bounds__(BLOCK) k_dyn_mom_mean(const Real* x, const Real* lw, const double* rec, int RS, int G,
                                                        const double* lse, int64_t N, int64_t Npad, double* mean,
                                                        int nx) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int d = blockIdx.x, r = blockIdx.y;
  const bool uni = rec[(int64_t)r * G * RS + 3 * (int64_t)G] != 0.0;
  const Real* xr = x + ((int64_t)r * nx + d) * Npad;
  const Real* lr = lw + (int64_t)r * Npad;
  double v[2] = {0.0, 0.0};
  for (int64_t i = threadIdx.x; i < N; i += BLOCK) {
    const double w = mom_weight<Real>(lr, i, uni, lse[r]);
    v[0] += w;
    v[1] += w * (double)xr[i];
  }
  block_sum_k<2>(v, smem);
  if (threadIdx.x == 0) mean[(int64_t)r * nx + d] = v[1] / v[0];
}

template <typename Real>
__global__ void __launch_bounds__(BLOCK) k_dyn_mom_cov(const Real* x, const Real* lw, const double* rec, int RS, int G,
                                                       const double* lse, int64_t N, int64_t Npad, const double* mean,
                                                       double* cov, int nx) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int d = blockIdx.x / nx, e = blockIdx.x % nx, r = blockIdx.y;
  if (e < d) return;
  const bool uni = rec[(int64_t)r * G * RS + 3 * (int64_t)G] != 0.0;
  const Real* xd = x + ((int64_t)r * nx + d) * Npad;
  const Real* xe = x + ((int64_t)r * nx + e) * Npad;
  const Real* lr = lw + (int64_t)r * Npad;
  const double md = mean[(int64_t)r * nx + d], me = mean[(int64_t)r * nx + e];
  double v[2] = {0.0, 0.0};
  for (int64_t i = threadIdx.x; i < N; i += BLOCK) {
    const double w = mom_weight<Real>(lr, i, uni, lse[r]);
    v[0] += w;
    v[1] += w * ((double)xd[i] - md) * ((double)xe[i] - me);
  }
  block_sum_k<2>(v, smem);
  if (threadIdx.x == 0) {
    cov[(int64_t)r * nx * nx + d * nx + e] = v[1] / v[0];
    cov[(int64_t)r * nx * nx + e * nx + d] = v[1] / v[0];
  }
}

// within-filter sharding (pf_shard_kernels.h) for a runtime nx
template <typename Real>
__global__ void __launch_bounds__(BLOCK) k_dyn_shard_offspring(const Real* __restrict__ x, int64_t N, int64_t Npad,
                                                               const double* __restrict__ cdf, double U, double lo,
                                                               double mass, int64_t Ntot, int64_t a, int64_t n,
                                                               Real* __restrict__ out, int nx) {
  const int64_t s = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (s >= n) return;
  const double pos = ((U + (double)(a + s)) / (double)Ntot - lo) / mass;
  int64_t l = 0, hi = N;
  while (l < hi) {
    const int64_t mid = (l + hi) >> 1;
    if (pos < cdf[mid]) hi = mid; else l = mid + 1;
  }
  const int64_t j = l < N ? l : N - 1;
  for (int d = 0; d < nx; ++d) out[s * nx + d] = x[(int64_t)d * Npad + j];
}

template <typename Real>
__global__ void __launch_bounds__(BLOCK) k_dyn_shard_adopt(const Real* __restrict__ rows, Real* __restrict__ x,
                                                           int64_t N, int64_t Npad, double* rec, int G,
                                                           const Real* __restrict__ P, int jitter,
                                                           const double* __restrict__ rp_jit, uint64_t seed,
                                                           uint32_t rep, uint32_t ep, int64_t pbase, int nx, int nz) {
  const DynRec RC(nx);
  const DynLay L(nx, nz);
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i < N) {
    Real* xc = x + i;
    if (jitter) {  // normals in the column, rows finished from the last one up (k_dyn_init)
      NStream<Real> ns(seed, i, nx, 0u, rep, ep, STREAM_JITTER, rp_jit, N, pbase);
      for (int d = 0; d < nx; ++d) xc[d * Npad] = ns.next();
      for (int d = nx - 1; d >= 0; --d) {
        Real acc = Real(0);
        for (int e = 0; e <= d; ++e) acc += xc[e * Npad] * P[L.LJ + d * nx + e];
        xc[d * Npad] = rows[i * nx + d] + acc;
      }
    } else {
      for (int d = 0; d < nx; ++d) xc[d * Npad] = rows[i * nx + d];
    }
  }
  if (i < G) {
    for (int q = 0; q < RC.SIZE; ++q) rec[(int64_t)q * G + i] = 0.0;
    rec[(int64_t)3 * G + i] = 1.0;
  }
}

}  // namespace pf
