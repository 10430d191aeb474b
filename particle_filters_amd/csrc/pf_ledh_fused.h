// One LEDH / EDH step of the shared-Jacobian (linear h) path in ONE launch: the affine flow,
// the weights (ledh.py:186-195 / edh.py:287-297), ESS and decision (ledh.py:39-41, 201-203),
// systematic resampling (ledh.py:25-37, 204-206) and the posterior moments (ledh.py:209,
// 217-224) — the work of k_flow_affine, k_weights_small, k_gather, k_mom_part and k_mom_final,
// whose floors (10-17 us each on 1e4 particles, fewer waves than SIMDs) dominated config 5.
//
// NBK co-resident workgroups (<= one per CU), each owning PPB consecutive particles (and the
// same PPB destination slots), meet at grid barriers (per-workgroup phase words; data handed
// between workgroups goes through write-through stores / loads, as in k_resident):
//   P1  flow of its particles -> x_out (SoA, write-through), log weights in LDS; max     | B1
//   P2  global max M; e = exp(l - M); workgroup sum e, sum e^2, inclusive scan in LDS   | B2
//   P3  S = sum e, ESS = S^2 / sum e^2, decision; on a resample its slice of the global
//       CDF c_j = (offset + scan_j) / S (c = 1 for the last particle, the reference's
//       clamp) and its last value are published                                       | B3
//   P4  its slots: ancestors by a two-level search (source workgroup over the published
//       last values, then inside the source slice staged in LDS) = searchsorted(cdf,
//       (U + i)/N, 'right'); rows copied into x_res (or copied through with w = e/S), and
//       the one-pass shifted moment partials of the rows (4x4 register blocks)          | B4
//   P5  the NOUT = NX + NX(NX+1)/2 output entries, 16 per round, over the NBK partials;
//       workgroup 0 also writes ESS / decision.
// The new state always lands in x_res (the previous state's buffer, dead after P1) and w_out.
#pragma once
#include "pf_ledh_kernels.h"

namespace pf {
namespace ledh {

// workgroup: 64 particles per flow round at GL lanes each (512 lanes for L96's 8-lane groups)
template <int NX>
struct FusedBlk {
  static constexpr int FB = Grp<NX>::GL >= 8 ? 512 : 256;
};
constexpr int FMAX = 256;                      // max workgroups (one per CU, co-resident)
constexpr int FPPB = 256;                      // max particles per workgroup (N <= FMAX * FPPB)
constexpr int FMC = 64;                        // particles per moment chunk (staged in LDS)
constexpr unsigned FSPIN = 1u << 24;           // barrier spin limit (then the launch fails)
constexpr int FNST = 4;                        // source CDF slices staged in LDS per moment chunk
#ifndef PF_LEDH_LDS
#define PF_LEDH_LDS 1                          // parameters and composed flow staged in LDS (P1)
#endif

// diagnostic phase stamps (PF_STAMPS builds only): s_memrealtime (100 MHz) per workgroup
#ifdef PF_STAMPS
constexpr int FST = 12;
__device__ unsigned long long g_ledh_stamps[FMAX * FST];
#define LF_STAMP(k)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0) g_ledh_stamps[blockIdx.x * FST + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LF_STAMP(k) \
  do {              \
  } while (0)
#endif

struct FusedParams {
  FlowParams f;                  // x_in (previous state), x_out (flow scratch), w_in, table, ...
  double* x_res;                 // [NX][Npad] the new state (== f.x_in)
  double* w_out;                 // [N] the new weights
  const double* shift;           // [NX] previous posterior mean (moment shift)
  double* mean;                  // [NX] new posterior mean (next shift)
  double* o_mean;                // [NX] or null
  double* o_cov;                 // [NX][NX] or null
  double* o_ess;                 // or null
  int32_t* o_flag;               // or null
  double* stat;                  // [4] ess, flag, sw
  double* cdf;                   // [N] the global CDF (resample steps)
  unsigned long long* words;     // [NBK] barrier phase words (monotonic across launches)
  unsigned long long* part;      // [4][FMAX] workgroup max / sum e / sum e^2 / last CDF value (bits)
  unsigned long long* cpart;     // [NBK][E] moment partials (double bits)
  unsigned int* err;             // barrier timeout flag
  unsigned long long phase0;     // phase word base of this launch
  double ratio;
  uint32_t ep_res;               // Philox epoch of the resampling offset U
  const double* rp_unif;         // replayed U of this step (host draw stream) or null (Philox)
  int nbk, ppb;
};

__device__ __forceinline__ void f_st(unsigned long long* p, double v) {
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double f_ld(const unsigned long long* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void f_std(double* p, double v) { f_st((unsigned long long*)p, v); }
__device__ __forceinline__ double f_ldd(const double* p) { return f_ld((const unsigned long long*)p); }

// grid barrier: every workgroup publishes `phase` in its word, then waits for all words >= phase.
// False on timeout (the launch is abandoned and *err set; the host reports it).
__device__ __forceinline__ bool f_barrier(const FusedParams& p, unsigned long long phase) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(p.words + blockIdx.x, phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (unsigned spins = 0;; ++spins) {
    int good = 1;
    if ((int)threadIdx.x < p.nbk)
      good = __hip_atomic_load(p.words + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= phase;
    if (__syncthreads_and(good)) return true;
    if (spins >= FSPIN || __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
      if (threadIdx.x == 0) atomicOr(p.err, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

template <int NX, int NZ, int TK>
__global__ void __launch_bounds__(FusedBlk<NX>::FB) k_ledh_fused(FusedParams p) {
  constexpr int FB = FusedBlk<NX>::FB;
  using MM = Mom<NX>;
  using MB = MomBlk<NX>;
  constexpr int GL = Grp<NX>::GL;
  constexpr int FCH = FB / GL;  // particles per flow round
  __shared__ double lws[FPPB];   // log weights, then e, of this workgroup's particles
  __shared__ double scan[FPPB];  // inclusive scan of e
  __shared__ double red[64];
  __shared__ double boff[FMAX + 1];
  __shared__ double xs[FMC * MB::XW];
  __shared__ double ws[FMC];
  __shared__ double mred[MB::SL][MB::NPAIR][16];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t N = p.f.N, Npad = p.f.Npad;
  const int64_t i0 = (int64_t)b * p.ppb;
  const int n = (int)max((int64_t)0, min((int64_t)p.ppb, N - i0));  // this workgroup's particles
  const unsigned long long ph = p.phase0;
  LF_STAMP(0);

  // ---- P1: flow --------------------------------------------------------------------
  // The parameter block and the composed flow are read by every lane group many times over
  // (H, D, QL, ... at lane-dependent offsets): staged once per workgroup in LDS, so the
  // per-particle chain waits on LDS instead of L2 round trips at one wave per SIMD.
#if PF_LEDH_LDS
  using L = Lay<NX, NZ>;
  using TL = TLay<NX, NZ>;
  __shared__ double pms[L::SIZE];
  __shared__ double afs[TL::AFF_SIZE];
  {
    const bool qd = p.f.q_diag != 0;
    auto need = [&](int k) {
      if (k < L::EX) return TK != PF_TRANS_L96;             // A (linear g)
      if (k < L::AC) return true;                           // F, dt, H, c
      if (k < L::LQ) return false;                          // acoustic geometry (not a linear h)
      if (k < L::R) {                                       // chol(Q), Q^{-1}: the diagonal when diagonal
        const int e = (k - L::LQ) % (NX * NX);
        return !qd || (e / NX == e % NX);
      }
      return k >= L::RI;                                    // R^{-1}
    };
    for (int k = t; k < L::SIZE; k += FB)
      if (need(k)) pms[k] = p.f.Pm[k];
    const double* __restrict__ afg = p.f.table + TL::aff(p.f.L);
    for (int k = t; k < TL::AFF_SIZE; k += FB) afs[k] = afg[k];
    __syncthreads();
  }
  const double* Pm_f = pms;
  const double* af_f = afs;
#else
  const double* Pm_f = p.f.Pm;
  const double* af_f = p.f.table + TLay<NX, NZ>::aff(p.f.L);
#endif
  double m = -INFINITY;
  {
    const int q = t % GL, slot = t / GL, base = lane - q;
    for (int c0 = 0; c0 < n; c0 += FCH) {
      const int j = c0 + slot;
      const bool live = j < n;
      // whole lane groups stay together; dead groups run particle i0 (results discarded)
      const double l = flow_affine_particle<NX, NZ, TK, true>(p.f, Pm_f, af_f, live ? i0 + j : i0, q, base);
      if (live && q == 0) lws[j] = l;
      if (live) m = fmax(m, l);
    }
  }
  m = block_reduce_max(m, red);

  // ---- P2: exponentials relative to the WORKGROUP max, sums and scan (no grid max needed:
  //      the workgroups' (max, sum, sum of squares) combine exactly after one barrier) ----------
  // thread t owns the contiguous run [t*per, t*per + per) of this workgroup's particles
  const int per = (n + FB - 1) / FB;
  double s1 = 0.0, s2 = 0.0;
  for (int j = t * per; j < min(n, t * per + per); ++j) {
    const double l = lws[j];
    const double e = (l > -INFINITY) ? exp(l - m) : 0.0;
    lws[j] = e;
    s1 += e;
    s2 += e * e;
  }
  {
    const double inc = wave_incl_scan64(s1, lane);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    double off = 0.0;
    for (int k = 0; k < wv; ++k) off += red[k];
    double run = off + inc - s1;
    for (int j = t * per; j < min(n, t * per + per); ++j) {
      run += lws[j];
      scan[j] = run;
    }
    __syncthreads();
  }
  const double S_b = block_reduce_sum(s1, red);
  const double S2_b = block_reduce_sum(s2, red);
  if (t == 0) {
    f_st(p.part + 0 * FMAX + b, m);
    f_st(p.part + 1 * FMAX + b, S_b);
    f_st(p.part + 2 * FMAX + b, S2_b);
  }
  LF_STAMP(1);
  if (!f_barrier(p, ph + 1)) return;
  LF_STAMP(2);

  // ---- P3: global normaliser, ESS, decision; the CDF slice on a resample -----------------
  double mk = -INFINITY, sk = 0.0, s2k = 0.0;
  if (t < p.nbk) {
    mk = f_ld(p.part + 0 * FMAX + t);
    sk = f_ld(p.part + 1 * FMAX + t);
    s2k = f_ld(p.part + 2 * FMAX + t);
  }
  const double M = block_reduce_max(sk > 0.0 ? mk : -INFINITY, red);
  const double fk = (sk > 0.0) ? exp(mk - M) : 0.0;
  {
    const double v = sk * fk;
    const double inc = wave_incl_scan64(v, lane);
    if (lane == 63) red[wv] = inc;
    __syncthreads();
    double off = 0.0;
    for (int k = 0; k < wv; ++k) off += red[k];
    if (t < p.nbk) boff[t] = off + inc - v;  // exclusive prefix of the scaled workgroup sums
    if (t == b) red[8] = fk;  // this workgroup's scale e^(m_b - M)
    if (t == FB - 1) boff[FMAX] = off + inc;  // total
    __syncthreads();
  }
  const double S = boff[FMAX];
  const double fb = red[8];
  const double E2 = block_reduce_sum(s2k * fk * fk, red);
  const double ess = 1.0 / (E2 / (S * S));
  const bool flag = (p.ratio > 0.0) && (ess < p.ratio * (double)N);
  if (flag) {
    const double Ob = boff[b];
    for (int j = t; j < n; j += FB) wt_store(p.cdf + i0 + j, (i0 + j == N - 1) ? 1.0 : (Ob + fb * scan[j]) / S);
    if (t == 0) f_st(p.part + 3 * FMAX + b, (b == p.nbk - 1) ? 1.0 : (Ob + fb * scan[n - 1]) / S);
    LF_STAMP(5);
    if (!f_barrier(p, ph + 3)) return;
    LF_STAMP(6);
    if (t < p.nbk) boff[t] = f_ld(p.part + 3 * FMAX + t);  // last CDF value of every workgroup
    __syncthreads();
  }

  // ---- P4: this workgroup's slots -> x_res, staged rows, moment partials ------------------
  __shared__ double slice[FNST * FPPB];
  __shared__ int anc[FMC];
  __shared__ int krange[2];
  // ledh.py:28: the step's U (Philox, as k_gather; or the replayed host draw)
  const double U = flag ? (p.rp_unif ? *p.rp_unif : uniform53(p.f.seed, 0u, 0u, p.ep_res)) : 0.0;
  const double dN = (double)N;
  // first workgroup whose last CDF value exceeds pos (the last one if none)
  auto src_block = [&](double pos) {
    int lo = 0, hi = p.nbk;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (pos < boff[mid]) hi = mid; else lo = mid + 1;
    }
    return lo < p.nbk ? lo : p.nbk - 1;
  };
  double a0acc = 0.0, a1acc = 0.0;
  const int pair = t % MB::NPAIR, sl = t / MB::NPAIR;
  int bi = 0, bj = 0;
  {
    int rem = pair;
    while (rem >= MB::NB - bi) { rem -= MB::NB - bi; ++bi; }
    bj = bi + rem;
  }
  double acc[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.0;
  for (int c0 = 0; c0 < n; c0 += FMC) {
    const int cn = min(FMC, n - c0);
    if (flag) {
      if (t == 0) {
        krange[0] = src_block((U + (double)(i0 + c0)) / dN);
        krange[1] = src_block((U + (double)(i0 + c0 + cn - 1)) / dN);
      }
      __syncthreads();
      const int klo = krange[0], nk = krange[1] - krange[0] + 1;
      const bool staged = nk <= FNST;
      if (staged)
        for (int q2 = t; q2 < nk * FPPB; q2 += FB) {
          const int kk = klo + q2 / FPPB, jj = q2 % FPPB;
          const int64_t g = (int64_t)kk * p.ppb + jj;
          slice[q2] = (jj < p.ppb && g < N) ? wt_load(p.cdf + g) : INFINITY;
        }
      __syncthreads();
      if (t < cn) {
        const double pos = (U + (double)(i0 + c0 + t)) / dN;
        const int k = src_block(pos);
        const int64_t g0 = (int64_t)k * p.ppb;
        const int len = (int)min((int64_t)p.ppb, N - g0);
        int lo = 0, hi = len;
        if (staged && k >= klo && k < klo + nk) {
          const double* cs = slice + (k - klo) * FPPB;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (pos < cs[mid]) hi = mid; else lo = mid + 1;
          }
        } else {
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (pos < wt_load(p.cdf + g0 + mid)) hi = mid; else lo = mid + 1;
          }
        }
        anc[t] = (int)(g0 + (lo < len ? lo : len - 1));
      }
      __syncthreads();
    }
    // rows: particle-fastest mapping (coalesced copy-through; gathered rows on a resample);
    // all of a thread's loads are issued before any store so their latencies overlap
    constexpr int RPT = (FMC * MB::XW + FB - 1) / FB;
    double rv[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int q2 = t + r * FB;
      const int j = q2 % FMC, d = q2 / FMC;
      rv[r] = 0.0;
      if (q2 < FMC * MB::XW && j < cn && d < NX)
        rv[r] = wt_load(p.f.x_out + (int64_t)d * Npad + (flag ? (int64_t)anc[j] : i0 + c0 + j));
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int q2 = t + r * FB;
      const int j = q2 % FMC, d = q2 / FMC;
      if (q2 < FMC * MB::XW) {
        double v = 0.0;
        if (j < cn && d < NX) {
          wt_store(p.x_res + (int64_t)d * Npad + i0 + c0 + j, rv[r]);
          v = rv[r] - p.shift[d];
        }
        xs[j * MB::XW + d] = v;
      }
    }
    for (int j = t; j < FMC; j += FB) {
      const double wj = j < cn ? (flag ? 1.0 / dN : (fb * lws[c0 + j]) / S) : 0.0;
      ws[j] = wj;
      if (j < cn) p.w_out[i0 + c0 + j] = wj;
    }
    __syncthreads();
    if (t <= NX) {
      if (t == 0)
        for (int j = 0; j < cn; ++j) a0acc += ws[j];
      else
        for (int j = 0; j < cn; ++j) a1acc += ws[j] * xs[j * MB::XW + t - 1];
    }
    if (sl < MB::SL) {
      for (int j = sl; j < cn; j += MB::SL) {
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
    }
    __syncthreads();
  }
  unsigned long long* cp = p.cpart + (int64_t)b * MM::E;
  if (t <= NX) f_st(cp + t, t == 0 ? a0acc : a1acc);
  if (sl < MB::SL)
#pragma unroll
    for (int k = 0; k < 16; ++k) mred[sl][pair][k] = acc[k];
  __syncthreads();
  if (t < MB::NPAIR) {
    int ci = 0, rem = t;
    while (rem >= MB::NB - ci) { rem -= MB::NB - ci; ++ci; }
    const int cj = ci + rem;
    for (int k = 0; k < 4; ++k)
      for (int l = 0; l < 4; ++l) {
        const int d = 4 * ci + k, e = 4 * cj + l;
        if (d >= NX || e >= NX || e < d) continue;
        double a = 0.0;
        for (int s2 = 0; s2 < MB::SL; ++s2) a += mred[s2][t][k * 4 + l];
        f_st(cp + 1 + NX + (d * NX - d * (d - 1) / 2 + (e - d)), a);
      }
  }
  LF_STAMP(7);
  if (!f_barrier(p, ph + 4)) return;
  LF_STAMP(8);

  // ---- P5: final reduction, 16 output entries per round, rounds strided over workgroups ----
  constexpr int NOUT = NX + MM::NP;
  __shared__ double fpart[4][FB / 16][17];
  if (b == 0 && t == 0) {
    p.stat[0] = ess;
    p.stat[1] = flag ? 1.0 : 0.0;
    p.stat[2] = S;
    if (p.o_ess) *p.o_ess = ess;
    if (p.o_flag) *p.o_flag = flag ? 1 : 0;
  }
  const int el = t / 16, pl = t % 16;
  for (int g0 = b * (FB / 16); g0 < NOUT; g0 += p.nbk * (FB / 16)) {
    const int qo = g0 + el;
    const bool live = qo < NOUT;
    int d = 0, e = 0;
    if (live && qo >= NX) pair_of(qo - NX, NX, &d, &e);
    const int src[4] = {0, 1 + (qo < NX ? qo : d), 1 + e, qo >= NX ? 1 + NX + (qo - NX) : 0};
    double tot4[4] = {0.0, 0.0, 0.0, 0.0};
    if (live)
      for (int k = pl; k < p.nbk; k += 16) {
#pragma unroll
        for (int f = 0; f < 4; ++f) tot4[f] += f_ld(p.cpart + (int64_t)k * MM::E + src[f]);
      }
#pragma unroll
    for (int f = 0; f < 4; ++f) fpart[f][el][pl] = tot4[f];
    __syncthreads();
    if (pl == 0 && live) {
      double tot[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        double sum = 0.0;
        for (int k = 0; k < 16; ++k) sum += fpart[f][el][k];
        tot[f] = sum;
      }
      const double sw = tot[0];
      if (qo < NX) {
        const double mv = p.shift[qo] + tot[1] / sw;
        p.mean[qo] = mv;
        if (p.o_mean) p.o_mean[qo] = mv;
      } else {
        const double c = tot[3] / sw - (tot[1] / sw) * (tot[2] / sw);
        if (p.o_cov) {
          p.o_cov[d * NX + e] = c;
          p.o_cov[e * NX + d] = c;
        }
      }
    }
    __syncthreads();
  }
  LF_STAMP(9);
}

}  // namespace ledh
}  // namespace pf
