// One LEDH / EDH step of the shared-Jacobian (linear h) path in ONE launch with ONE grid barrier:
// the affine flow, the weights (ledh.py:186-195 / edh.py:287-297), ESS and decision (ledh.py:39-41,
// 201-203), systematic resampling (ledh.py:25-37, 204-206) and the posterior moments (ledh.py:209,
// 217-224) - the work of k_flow_affine, k_weights_small, k_gather, k_mom_part and k_mom_final,
// whose floors (10-17 us each on 1e4 particles, fewer waves than SIMDs) dominated config 5.
//
// NBK co-resident workgroups (<= one per CU), each owning PPB consecutive particles (slots):
//   P1  flow of its slots.  The state enters as (rows, ancestors): slot i starts from row anc[i]
//       of the previous step's flow output - the previous resample is applied by this gather, no
//       separate copy.  Flow rows -> x_out (write-through; the first FCH also stay in LDS), log
//       weights in LDS; the workgroup max
//   P2  e = exp(l - m) relative to the WORKGROUP max, sum e, sum e^2 and the inclusive scan in LDS;
//       published: (m, sum e, sum e^2, last scan value)                                   | B1
//   P5' (waves 1.. while wave 0 runs P3's combine) the PREVIOUS step's output entries (NX +
//       NX(NX+1)/2) over the NBK moment partials it left, spread over every workgroup; its mean is
//       the moment shift of the NEXT step (a shift only conditions the one-pass sums: the posterior
//       mean of two steps back serves as well as the last one, and is already in HBM at launch)
//   P3  every workgroup combines the NBK partials in one fixed order: normaliser S, ESS,
//       decision, the exclusive prefix O_k of the scaled workgroup sums and every workgroup's
//       scale, hence its own CDF slice c_j = (O_b + f_b scan_j) / S (c = 1 for the last particle,
//       the reference's clamp) and its predecessor's last value.  Resampling is SOURCE-driven:
//       particle j is the ancestor of the slots {i : max(last_{b-1}, c_{j-1}) <= (U + i)/N < c_j}
//       (the last particle of the last workgroup also takes positions past the end, as the
//       destination search's clamp did) - exactly the ancestors of the two-level
//       searchsorted(cdf, (U+i)/N, 'right') over the slices; the workgroup counts them (positions
//       below a CDF value, with the reference's comparison where it is close) and writes its index
//       into those slots of anc_out (4 bytes a slot: the imbalance of a degenerate resample is
//       cheap).  No resample: identity ancestors, w = e / S.
//   P4  moment partials of the reported set from the workgroup's OWN rows: weights n_j / N (n_j
//       = offspring count) after a resample - the sums over the post-resample slots - or e_j / S;
//       one-pass, shifted by the previous mean, 4x4 register blocks; left for the next launch.
// A run ends with a tail launch (step = 0): the last P5' and the materialised state
// x_res[i] = rows[anc[i]].
#pragma once
#include "pf_ledh_kernels.h"

namespace pf {
namespace ledh {

// workgroup: FCH = 64 particles per flow round at GL lanes each (512 lanes for 8-lane groups)
template <int NX>
struct FusedBlk {
  static constexpr int FB = Grp<NX>::GL >= 8 ? 512 : 256;
  static constexpr int FCH = FB / Grp<NX>::GL;
};
constexpr int FMAX = 256;                      // max workgroups (one per CU, co-resident)
constexpr int FPPB = 256;                      // max particles per workgroup (N <= FMAX * FPPB)
constexpr unsigned FSPIN = 1u << 24;           // barrier spin limit (then the launch fails)

struct FusedParams {
  FlowParams f;                  // x_in: the rows slots start from (previous flow output, or the state),
                                 // x_out: this step's flow rows, w_in, table, ...
  const int32_t* anc_in;         // [N] slot i starts from row anc_in[i] of f.x_in; null: row i
  int32_t* anc_out;              // [N] this step's ancestors (identity without a resample)
  double* x_res;                 // tail launch: [NX][Npad] the materialised state rows[anc[i]]
  double* w_out;                 // [N] the new weights
  const double* shift;           // [NX] this step's moment shift: the posterior mean of two steps back
  int step;                      // 1: run a filter step; 0: a run's tail (P5' and the materialised state)
  int p5;                        // 1: reduce the previous step's moment partials (cpart) first
  const double* shift5;          // [NX] the previous step's shift
  double* mean5;                 // [NX] the previous step's posterior mean (the shift of the next step)
  double* o_mean5;               // [NX] or null: the previous step's outputs
  double* o_cov5;                // [NX][NX] or null
  double* o_ess;                 // or null: this step's
  int32_t* o_flag;               // or null
  double* stat;                  // [4] ess, flag, sw
  unsigned long long* part;      // [8][FMAX] granules {32-bit tag, 32-bit half} of the workgroup max /
                                 // sum e / sum e^2 / last scan value (hi, lo halves of each double)
  unsigned long long* cpart;     // [NBK][E] this step's moment partials (double bits), written by P4
  const unsigned long long* cpart5;  // [NBK][E] the previous step's, read by P5' (the other buffer of a pair:
                                     // P5' may still read while faster workgroups are past B1 in P4)
  unsigned int* err;             // barrier timeout flag
  unsigned long long phase0;     // tag base of this launch (monotonic across launches)
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

// Block reductions with the wave step on the DPP network (a fixed tree: the same result in every
// workgroup); an LDS-only barrier variant (s_waitcnt lgkmcnt(0) + s_barrier instead of
// __syncthreads' vmcnt(0) wait for the write-through stores) was measured: no change.
__device__ __forceinline__ double dpp_reduce_sum(double v, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum_ud(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += red[k];
  __syncthreads();
  return s;
}
__device__ __forceinline__ double dpp_reduce_max(double v, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max_ud(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
  for (int k = 1; k < (int)(blockDim.x >> 6); ++k) s = fmax(s, red[k]);
  __syncthreads();
  return s;
}

// workgroup barrier for LDS hand-offs only: unlike __syncthreads it does not wait for this wave's
// outstanding global stores (P3's ancestors and weights keep draining under P4)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The grid hand-off (B1) is the partials themselves: each double is published as two 64-bit granules
// {tag, 32-bit half} (one atomic store each, no fence and no separate phase word), and a reader takes a
// workgroup's partials once all 8 of its granules carry this launch's tag - one round trip instead of
// store completion + phase word + poll + reload.  Tags are the launch's phase base + 1 (the host
// advances it per launch), so the buffer never needs clearing.
__device__ __forceinline__ void g_pub(unsigned long long* p, unsigned tag, unsigned pay) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | pay, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long g_ld(const unsigned long long* p) {
  return __hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double g_double(unsigned long long hi, unsigned long long lo) {
  return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
}

// #{ i in [0, N) : (U + i) / N < x } with the destination search's comparison (pos = (U + i) / N
// in fp64; x = -inf / +inf give 0 / N).  Exactly, (U + i) / N < x <=> i < y = x N - U; the fp64
// division can only disagree when y is within ~1e-11 of an integer, so only there are the
// candidate positions evaluated the reference's way.
__device__ __forceinline__ int64_t fcount_exact(double x, double U, int64_t N, int64_t c) {
  const double Nd = (double)N;
  while (c > 0 && (U + (double)(c - 1)) / Nd >= x) --c;
  while (c < N && (U + (double)c) / Nd < x) ++c;
  return c;
}
__device__ __forceinline__ int64_t fcount_below(double x, double U, int64_t N) {
  if (!(x > -INFINITY)) return 0;
  if (x == INFINITY) return N;
  const double y = fma(x, (double)N, -U);
  const double fl = floor(y), d = y - fl;
  const int64_t c = min(max((int64_t)fl + 1, (int64_t)0), N);
  if (d > 1e-7 && d < 1.0 - 1e-7) return c;
  return fcount_exact(x, U, N, c);
}

// P5': the NOUT = NX + NX(NX+1)/2 output entries of the previous step over the NBK partials it left
// (ledh.py:209, 217-224).  Entry q is reduced by a group of LPE lanes (64, or 32 / 16 so that every
// entry gets a group in one round), lane l summing partials l, l + LPE, ... (loaded in one batch:
// p5_load issues them, p5_finish consumes them, so their latency can overlap other loads), then a
// fixed xor tree: the same order in every run.  The partials were written by the previous launch
// (visible after the kernel boundary): plain loads.
constexpr int P5K = 8;  // partials per lane in one batch
template <int NX>
struct P5 {
  static constexpr int NOUT = NX + Mom<NX>::NP;
  int lpe, groups, gl, qo, d, e, src[4];
  bool live;
  // threads [base, base + nthr) of the workgroup (a whole number of waves) do the reduction; tid =
  // threadIdx.x - base
  static __device__ int lpe_of(const FusedParams& p, int nthr) {
    return (p.nbk * (nthr / 64) >= NOUT) ? 64 : (p.nbk * (nthr / 32) >= NOUT ? 32 : 16);
  }
  __device__ P5(const FusedParams& p, int round, int tid, int nthr) {
    lpe = lpe_of(p, nthr);
    groups = nthr / lpe;
    gl = tid % lpe;
    qo = (blockIdx.x + round * p.nbk) * groups + tid / lpe;
    live = qo < NOUT;
    d = 0;
    e = 0;
    if (live && qo >= NX) pair_of(qo - NX, NX, &d, &e);
    src[0] = 0;
    src[1] = 1 + (qo < NX ? qo : d);
    src[2] = 1 + e;
    src[3] = qo >= NX ? 1 + NX + (qo - NX) : 0;
  }
  static __device__ int rounds(const FusedParams& p, int nthr) {
    const int per = p.nbk * (nthr / lpe_of(p, nthr));
    return (NOUT + per - 1) / per;
  }
  // all rounds of the threads [base, base + nthr)
  static __device__ void run(const FusedParams& p, int tid, int nthr) {
    double v[P5K][4];
    for (int r = 0; r < rounds(p, nthr); ++r) {
      const P5 q5(p, r, tid, nthr);
      q5.load(p, 0, v);
      q5.finish(p, v);
    }
  }
  __device__ void load(const FusedParams& p, int k0, double (&v)[P5K][4]) const {
    const double* cp5 = (const double*)p.cpart5;
#pragma unroll
    for (int r = 0; r < P5K; ++r) {
      const int k = k0 + gl + r * lpe;
      const bool ok = live && k < p.nbk;
#pragma unroll
      for (int f = 0; f < 4; ++f) v[r][f] = ok ? cp5[(int64_t)k * Mom<NX>::E + src[f]] : 0.0;
    }
  }
  __device__ void finish(const FusedParams& p, double (&v)[P5K][4]) const {
    double tot[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0;; k0 += P5K * lpe) {
#pragma unroll
      for (int r = 0; r < P5K; ++r)
#pragma unroll
        for (int f = 0; f < 4; ++f) tot[f] += v[r][f];
      if (k0 + P5K * lpe >= p.nbk) break;
      load(p, k0 + P5K * lpe, v);
    }
    // the group sum on the DPP network: 16-lane rows, then rows 0+1 / 2+3 into lanes 31 / 63, then
    // the whole wave into lane 63 (a fixed tree; the group's last lane holds its sum)
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      tot[f] = row_sum_d(tot[f]);
      if (lpe >= 32) tot[f] += dpp_d<DPP_ROW_BCAST15, 0xa>(0.0, tot[f]);
      if (lpe == 64) tot[f] += dpp_d<DPP_ROW_BCAST31, 0xc>(0.0, tot[f]);
    }
    if (live && gl == lpe - 1) {
      const double sw = tot[0];
      if (qo < NX) {
        const double mv = p.shift5[qo] + tot[1] / sw;
        f_std(p.mean5 + qo, mv);
        if (p.o_mean5) p.o_mean5[qo] = mv;
      } else {
        const double c = tot[3] / sw - (tot[1] / sw) * (tot[2] / sw);
        if (p.o_cov5) {
          p.o_cov5[d * NX + e] = c;
          p.o_cov5[e * NX + d] = c;
        }
      }
    }
  }
};

template <int NX, int NZ, int TK>
__global__ void __launch_bounds__(FusedBlk<NX>::FB) k_ledh_fused(FusedParams p) {
  constexpr int FB = FusedBlk<NX>::FB;
  constexpr int FCH = FusedBlk<NX>::FCH;  // particles per flow round = rows per moment chunk
  using MM = Mom<NX>;
  using MB = MomBlk<NX>;
  using L = Lay<NX, NZ>;
  using TL = TLay<NX, NZ>;
  constexpr int GL = Grp<NX>::GL, PER = Grp<NX>::PER;
  constexpr int XW = MB::XW;
  static_assert(MB::NPAIR * MB::SL <= FB, "block pairs x slices fit the workgroup");
  __shared__ double lws[FPPB];   // log weights, then e, of this workgroup's particles
  __shared__ double scan[FPPB];  // inclusive scan of e
  __shared__ double red[64];
  __shared__ double boff[FMAX + 1];   // exclusive prefix of the scaled workgroup sums (+ total)
  __shared__ double xs[FCH * XW];     // raw rows of a chunk (the first flow round's stay from P1)
  __shared__ double ws[FCH];
  __shared__ double shs[NX];            // P4's moment shift (the previous posterior mean)
  __shared__ int64_t shi[FPPB];       // resample: end of each particle's slot range
  __shared__ double pms[L::SIZE];     // the parameter block (the parts the flow reads)
  __shared__ double afs[TL::AFF_SIZE];  // the composed flow
  __shared__ double zs[NZ];             // the step's observation
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t N = p.f.N, Npad = p.f.Npad;
  const int64_t i0 = (int64_t)b * p.ppb;
  const int n = (int)max((int64_t)0, min((int64_t)p.ppb, N - i0));  // this workgroup's particles
  // the first flow round's slot, source row and weight: loaded first, their latency under the staging
  const int slot1 = t / GL;
  const int64_t i1 = slot1 < n ? i0 + slot1 : i0;
  const int64_t src1 = (p.step && p.anc_in) ? (int64_t)p.anc_in[i1] : i1;
  const double w1 = p.step ? p.f.w_in[i1] : 0.0;
  double x1[PER];  // and its row's components of this lane
#pragma unroll
  for (int jj = 0; jj < PER; ++jj) {
    const int a = (t % GL) * PER + jj;
    x1[jj] = (p.step && a < NX) ? p.f.x_in[(int64_t)a * Npad + src1] : 0.0;
  }
  if (!p.step) {  // a run's tail: the last step's outputs and the materialised state rows[anc[i]]
    if (p.p5) P5<NX>::run(p, t, FB);
    if (p.anc_in)
      for (int e = t; e < n * NX; e += FB) {
        const int j = e % n, d = e / n;
        p.x_res[(int64_t)d * Npad + i0 + j] = p.f.x_in[(int64_t)d * Npad + p.anc_in[i0 + j]];
      }
    return;
  }
  const unsigned long long ph = p.phase0;
  LF_STAMP(0);

  // ---- staging: the parameter block and the composed flow are read by every lane group many times
  // over (H, D, QL, ... at lane-dependent offsets): copied once per workgroup into LDS, so the
  // per-particle chain waits on LDS instead of L2 round trips at one wave per SIMD.  Only the parts
  // the flow reads (the diagonals of chol(Q) and Q^{-1} when Q is diagonal), in batches of loads.
  // (Tried: the first flow round's prior under the staging loads - slower, 25.7 -> 27.1 us: its
  // chol(Q) loads queue behind the staging loads in vmcnt order.)
  const int q = t % GL, slot = t / GL, base = lane - q;
  {
    const bool qd = p.f.q_diag != 0;
    constexpr int nA = TK != PF_TRANS_L96 ? NX * NX : 0;
    constexpr int n0 = L::AC - L::EX;  // F, dt, H, c
    const int nq = qd ? NX : NX * NX;  // per chol(Q) and Q^{-1}
    constexpr int nR = NZ * NZ;        // R^{-1}
    const int tot = nA + n0 + 2 * nq + nR + TL::AFF_SIZE;
    const double* __restrict__ afg = p.f.table + TL::aff(p.f.L);
    auto src_of = [&](int f, bool& to_af) -> int {  // flat staging index -> source offset
      to_af = false;
      if (f < nA) return L::A + f;
      f -= nA;
      if (f < n0) return L::EX + f;
      f -= n0;
      if (f < 2 * nq) {
        const int m = f / nq, r = f % nq;
        return (m == 0 ? L::LQ : L::QI) + (qd ? r * NX + r : r);
      }
      f -= 2 * nq;
      if (f < nR) return L::RI + f;
      to_af = true;
      return f - nR;
    };
    constexpr int SB = 8;
    for (int f0 = 0; f0 < tot; f0 += SB * FB) {
      double sv[SB];
#pragma unroll
      for (int r = 0; r < SB; ++r) {
        const int f = f0 + t + r * FB;
        bool af = false;
        const int k = f < tot ? src_of(f, af) : 0;
        sv[r] = f < tot ? (af ? afg[k] : p.f.Pm[k]) : 0.0;
      }
#pragma unroll
      for (int r = 0; r < SB; ++r) {
        const int f = f0 + t + r * FB;
        bool af = false;
        const int k = f < tot ? src_of(f, af) : 0;
        if (f < tot) {
          if (af) afs[k] = sv[r];
          else pms[k] = sv[r];
        }
      }
    }
  }
  if (t < NZ) zs[t] = p.f.z[t];
  // P4's moment shift: the posterior mean of two steps back (written by the previous launch)
  if (t < NX) shs[t] = p.shift[t];
  lds_barrier();
  LF_STAMP(1);

  // ---- P1: flow --------------------------------------------------------------------
  double m = -INFINITY;
  {
    for (int c0 = 0; c0 < n; c0 += FCH) {
      const int j = c0 + slot;
      const bool live = j < n;
      // whole lane groups stay together; dead groups run particle i0 (results discarded)
      const int64_t i = live ? i0 + j : i0;
      // the previous step's resample: the slot starts from its ancestor's row (the first round's row
      // and weight were loaded at entry)
      const int64_t src = c0 == 0 ? src1 : (p.anc_in ? (int64_t)p.anc_in[i] : i);
      const double wi = c0 == 0 ? w1 : p.f.w_in[i];
      double eta[PER], gx[PER], v[PER];
      group_prior<NX, NZ, TK>(p.f, pms, i, src, q, base, gx, v, x1, c0 == 0);
      const double l = flow_affine_post<NX, NZ, TK>(p.f, pms, afs, q, base, gx, v, eta, wi, zs);
#ifdef PF_STAMPS
      asm volatile("" ::"v"(l));
      if (c0 == 0) LF_STAMP(11);
#endif
      if (live) {
#pragma unroll
        for (int jj = 0; jj < PER; ++jj) {
          const int a = q * PER + jj;
          if (a < NX) wt_store(p.f.x_out + (int64_t)a * Npad + i, eta[jj]);  // the next step's gather
          if (c0 == 0 && a < XW) xs[j * XW + a] = a < NX ? eta[jj] : 0.0;
        }
        if (q == 0) lws[j] = l;
        m = fmax(m, l);
      } else if (c0 == 0) {  // a slot past the workgroup's particles: a zero row for P4's products
#pragma unroll
        for (int jj = 0; jj < PER; ++jj) {
          const int a = q * PER + jj;
          if (a < XW) xs[j * XW + a] = 0.0;
        }
      }
    }
    if constexpr (GL * PER < XW) {  // pad columns past the lane groups' components
      for (int e = t; e < FCH * (XW - GL * PER); e += FB) {
        const int j = e / (XW - GL * PER), a = GL * PER + e % (XW - GL * PER);
        xs[j * XW + a] = 0.0;
      }
    }
  }
  (void)m;
  lds_barrier();  // every slot's log weight is in lws
  LF_STAMP(12);

  // ---- P2: exponentials relative to the WORKGROUP max, sums and scan (no grid max needed:
  //      the workgroups' (max, sum, sum of squares) combine exactly after one barrier) ----------
  // One wave does it (lane l: particles PL l .. PL l + PL - 1, at most FPPB of them), so that the
  // workgroup's max, sums and scan cost no barrier beyond the grid barrier's own; the other waves
  // go straight on to it.
  if (wv == 0) {
    constexpr int PL = FPPB / 64;
    double e[PL], s1 = 0.0, s2 = 0.0, ml = -INFINITY;
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const int j = PL * lane + k;
      e[k] = j < n ? lws[j] : -INFINITY;
      ml = fmax(ml, e[k]);
    }
    const double mw = wave_max_ud(ml);
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      e[k] = (e[k] > -INFINITY) ? exp(e[k] - mw) : 0.0;
      s1 += e[k];
      s2 += e[k] * e[k];
    }
    const double inc = wave_incl_scan_dpp(s1);
    double run = inc - s1, last = 0.0;
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const int j = PL * lane + k;
      run += e[k];
      if (j < n) {
        lws[j] = e[k];
        scan[j] = run;
      }
      if (j == n - 1) last = run;
    }
    const double S_b = lane63_d(inc);
    const double S2_b = wave_sum_ud(s2);
    last = readlane_d(last, (n - 1) / PL);  // scan[n - 1], the value this workgroup's slice ends on
    if (lane < 8) {  // granule g = lane: value g / 2, high half for even g
      const double val = lane < 2 ? mw : (lane < 4 ? S_b : (lane < 6 ? S2_b : last));
      const unsigned long long bits = (unsigned long long)__double_as_longlong(val);
      g_pub(p.part + lane * FMAX + b, (unsigned)(p.phase0 + 1), (lane & 1) ? (unsigned)bits : (unsigned)(bits >> 32));
    }
  }
  LF_STAMP(13);
  LF_STAMP(2);
  // P5' (waves 1..): the previous step's moment partials (written by the previous launch) are loaded
  // before the grid barrier, so their latency hides under the wait
  const P5<NX> q5(p, 0, t - 64, FB - 64);
  double v5[P5K][4];
  if (wv != 0 && p.p5) q5.load(p, 0, v5);

  // ---- P3: global normaliser, ESS, decision; this slice of the CDF; the ancestors -----------
  // the NBK partials combined by one wave (lane l: workgroups KL l .. KL l + KL - 1) in one fixed
  // order, so every workgroup derives the same normaliser, ESS, decision and CDF slices; one
  // barrier hands the results to the other waves.  Meanwhile the other waves reduce the previous
  // step's moment partials (P5').
  LF_STAMP(14);
  if (wv != 0) {
    if (p.p5) {
      q5.finish(p, v5);
      for (int r = 1; r < P5<NX>::rounds(p, FB - 64); ++r) {
        const P5<NX> r5(p, r, t - 64, FB - 64);
        r5.load(p, 0, v5);
        r5.finish(p, v5);
      }
    }
  } else {
    constexpr int KL = FMAX / 64;
    // B1: poll the granules of workgroups KL lane .. KL lane + KL - 1 until all carry this launch's tag
    const unsigned tag = (unsigned)(ph + 1);
    unsigned long long gv[KL][8];
    bool ok_b1 = true;
    for (unsigned spins = 0;; ++spins) {
      bool good = true;
#pragma unroll
      for (int k = 0; k < KL; ++k) {
        const int kk = KL * lane + k;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          gv[k][g] = kk < p.nbk ? g_ld(p.part + g * FMAX + kk) : ((unsigned long long)tag << 32);
          good &= (unsigned)(gv[k][g] >> 32) == tag;
        }
      }
      if (__all(good)) break;
      if (spins >= FSPIN || __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        if (lane == 0) atomicOr(p.err, 1u);
        ok_b1 = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) red[11] = ok_b1 ? 1.0 : 0.0;
    LF_STAMP(3);
    double mk[KL], sk[KL], s2k[KL], slk[KL];
#pragma unroll
    for (int k = 0; k < KL; ++k) {
      const bool ok = KL * lane + k < p.nbk;
      mk[k] = ok ? g_double(gv[k][0], gv[k][1]) : -INFINITY;
      sk[k] = ok ? g_double(gv[k][2], gv[k][3]) : 0.0;
      s2k[k] = ok ? g_double(gv[k][4], gv[k][5]) : 0.0;
      slk[k] = ok ? g_double(gv[k][6], gv[k][7]) : 0.0;
    }
    double ml = -INFINITY;
#pragma unroll
    for (int k = 0; k < KL; ++k) ml = fmax(ml, sk[k] > 0.0 ? mk[k] : -INFINITY);
    const double M = wave_max_ud(ml);
    double fk[KL], v[KL], sl = 0.0, e2 = 0.0;
#pragma unroll
    for (int k = 0; k < KL; ++k) {
      fk[k] = (sk[k] > 0.0) ? exp(mk[k] - M) : 0.0;
      v[k] = sk[k] * fk[k];
      sl += v[k];
      e2 += s2k[k] * fk[k] * fk[k];
    }
    const double inc = wave_incl_scan_dpp(sl);
    const double S = lane63_d(inc);
    const double E2 = wave_sum_ud(e2);
    double run = inc - sl;  // exclusive prefix of the scaled workgroup sums
#pragma unroll
    for (int k = 0; k < KL; ++k) {
      const int kk = KL * lane + k;
      if (kk < p.nbk) boff[kk] = run;
      if (kk == b) red[8] = fk[k];  // this workgroup's scale e^(m_b - M)
      // the predecessor's last CDF value, as that workgroup evaluates its own slice
      if (kk + 1 == b) red[9] = (run + fk[k] * slk[k]) / S;
      run += v[k];
    }
    if (lane == 0) {
      boff[FMAX] = S;  // total
      red[10] = E2;
    }
  }
  lds_barrier();
  if (red[11] == 0.0) return;  // B1 timed out (the host reports it)
  const double S = boff[FMAX];
  const double fb = red[8];
  const double lastprev = b > 0 ? red[9] : -INFINITY;
  const double E2 = red[10];
  const double ess = 1.0 / (E2 / (S * S));
  const bool flag = (p.ratio > 0.0) && (ess < p.ratio * (double)N);
  if (b == 0 && t == 0) {
    p.stat[0] = ess;
    p.stat[1] = flag ? 1.0 : 0.0;
    p.stat[2] = S;
    if (p.o_ess) *p.o_ess = ess;
    if (p.o_flag) *p.o_flag = flag ? 1 : 0;
  }
  LF_STAMP(15);
  const double dN = (double)N;
  const double Ob = boff[b];
  int64_t slo0 = 0;
  if (flag) {
    // ledh.py:28: the step's U (Philox, as k_gather; or the replayed host draw)
    const double U = p.rp_unif ? *p.rp_unif : uniform53(p.f.seed, 0u, 0u, p.ep_res);
    for (int j = t; j < n; j += FB) {
      const double c = (i0 + j == N - 1) ? 1.0 : (Ob + fb * scan[j]) / S;
      shi[j] = (b == p.nbk - 1 && j == n - 1) ? N : fcount_below(c, U, N);
    }
    slo0 = fcount_below(lastprev, U, N);
    lds_barrier();
    // slots [slo0, shi[n-1]): slot s takes the first own particle j with s < shi[j] - a binary
    // search for the thread's first slot, then a cursor (slots rise by FB per iteration: a
    // degenerate resample, one particle over most slots, costs O(1) per slot)
    const int64_t s_end = shi[n - 1];
    int jc = 0;
    if (slo0 + t < s_end) {
      int hi = n - 1;
      while (jc < hi) {
        const int mid = (jc + hi) >> 1;
        if (slo0 + t < shi[mid]) hi = mid; else jc = mid + 1;
      }
    }
    for (int64_t s = slo0 + t; s < s_end; s += FB) {
      while (shi[jc] <= s) ++jc;
      p.anc_out[s] = (int32_t)(i0 + jc);
    }
  } else {
    for (int j = t; j < n; j += FB) p.anc_out[i0 + j] = (int32_t)(i0 + j);
  }
  for (int j = t; j < n; j += FB) p.w_out[i0 + j] = flag ? 1.0 / dN : (fb * lws[j]) / S;
  LF_STAMP(4);

  // ---- P4: moment partials of the reported set from the own rows --------------------------
  // after a resample particle j stands for its n_j slots (weight n_j / N): the same sums as over
  // the post-resample slots; otherwise its normalised weight.  All of them - W = sum w_j, S1 =
  // sum w_j u_j and the upper triangle of S2 = sum w_j u_j u_j^T (u_j = row_j - shift) - are the
  // augmented Gram matrix G = sum_j w_j [u_j; 1][u_j; 1]^T, accumulated on the fp64 matrix cores
  // (v_mfma_f64_16x16x4: A[d][j] = w_j [u_j; 1]_d, B[j][e] = [u_j; 1]_e, 4 rows per instruction):
  // 16 x 16 tiles (I, J), I <= J, wave w owning tiles w, w + NW, ...; each lane then stores the
  // entries of the tiles it holds.  No cross-thread reduction, no LDS staging of partial sums.
  constexpr int NT = (NX + 1 + 15) / 16;      // tiles per dimension of the augmented Gram matrix
  constexpr int NPT = NT * (NT + 1) / 2;      // upper-triangular tile pairs
  constexpr int NW = FB / 64;
  constexpr int TPW = (NPT + NW - 1) / NW;    // tile pairs per wave (at most)
  typedef double dbl4 __attribute__((ext_vector_type(4)));
  dbl4 gacc[TPW];
  int ti[TPW], tj[TPW];
#pragma unroll
  for (int q = 0; q < TPW; ++q) {
    gacc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
    int rem = wv + q * NW, I = 0;  // pair index -> (I, J), row-major over the upper triangle
    if (rem >= NPT) rem = 0;       // a wave with fewer pairs repeats pair 0 (its result is not stored)
    while (rem >= NT - I && I < NT) { rem -= NT - I; ++I; }
    ti[q] = I;
    tj[q] = I + rem;
  }
  const int r16 = lane & 15, kq = lane >> 4;  // A row / B column in the tile; k within the 4-row step
  // per pair: the lane's A row / B column, clamped into the staged row (x - shift where it is a state
  // component, the augmented 1 at NX, 0 past it) - operands by selects, no divergent branches
  // as multiply-adds: u = fma(x - shift, m, c) with (m, c) = (1, 0) for a state component, (0, 1) for
  // the augmented 1, (0, 0) past it - the same value as the selects for finite rows, and the LDS
  // reads stay unconditional (a select let the compiler sink each read into a branch of its own,
  // serialising four LDS round trips per k-step)
  int xa_[TPW], xb_[TPW];
  double sa_[TPW], sb_[TPW], ma_[TPW], mb_[TPW], ca_[TPW], cb_[TPW];
#pragma unroll
  for (int q = 0; q < TPW; ++q) {
    const int da = 16 * ti[q] + r16, db = 16 * tj[q] + r16;
    ma_[q] = da < NX ? 1.0 : 0.0;
    mb_[q] = db < NX ? 1.0 : 0.0;
    ca_[q] = da == NX ? 1.0 : 0.0;
    cb_[q] = db == NX ? 1.0 : 0.0;
    xa_[q] = min(da, NX - 1);
    xb_[q] = min(db, NX - 1);
    sa_[q] = shs[xa_[q]];
    sb_[q] = shs[xb_[q]];
  }
  if (n > FCH) {  // rows past the first flow round are read back from x_out: every wave's stores done
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
  }
  for (int c0 = 0; c0 < n; c0 += FCH) {
    const int cn = min(FCH, n - c0);
    lds_barrier();  // the previous chunk has consumed xs (and shi / lws are complete)
    if (c0 == 0) LF_STAMP(18);
    if (c0 > 0)  // own rows past the first flow round, from x_out
      for (int e = t; e < FCH * XW; e += FB) {
        const int j = e % FCH, d = e / FCH;
        xs[j * XW + d] = (j < cn && d < NX) ? wt_load(p.f.x_out + (int64_t)d * Npad + i0 + c0 + j) : 0.0;
      }
    for (int j = t; j < FCH; j += FB) {
      double wj = 0.0;
      if (j < cn) {
        const int jg = c0 + j;
        if (flag) {
          const int64_t lo = jg == 0 ? slo0 : max(slo0, shi[jg - 1]);
          wj = shi[jg] > lo ? (double)(shi[jg] - lo) / dN : 0.0;
        } else {
          wj = (fb * lws[jg]) / S;
        }
      }
      ws[j] = wj;  // 0 past the chunk
    }
    lds_barrier();
    if (c0 == 0) LF_STAMP(19);
    // all FCH rows (rows past the chunk have weight 0 and operands 0), 4 per instruction, the wave's
    // tile pairs interleaved (independent accumulators)
#pragma unroll
    for (int j0 = 0; j0 < FCH; j0 += 4) {
      const int j = j0 + kq;
      const bool live = j < cn;
      const double wl = ws[j], ll = live ? 1.0 : 0.0;  // ws is 0 past the chunk
#pragma unroll
      for (int q = 0; q < TPW; ++q) {
        const double ua = fma(xs[j * XW + xa_[q]] - sa_[q], ma_[q], ca_[q]) * wl;
        const double ub = fma(xs[j * XW + xb_[q]] - sb_[q], mb_[q], cb_[q]) * ll;
        gacc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(ua, ub, gacc[q], 0, 0, 0);
      }
    }
  }
  LF_STAMP(16);
  unsigned long long* cp = p.cpart + (int64_t)b * MM::E;
  // D layout of v_mfma_f64_16x16x4: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int q = 0; q < TPW; ++q) {
    if (wv + q * NW >= NPT) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = 16 * ti[q] + kq + 4 * r, e = 16 * tj[q] + r16;
      const double v = gacc[q][r];
      if (d < NX && e < NX && d <= e) f_st(cp + 1 + NX + (d * NX - d * (d - 1) / 2 + (e - d)), v);
      else if (d < NX && e == NX) f_st(cp + 1 + d, v);   // S1
      else if (d == NX && e == NX) f_st(cp, v);          // W
    }
  }
  LF_STAMP(17);
  LF_STAMP(5);
}

}  // namespace ledh
}  // namespace pf
