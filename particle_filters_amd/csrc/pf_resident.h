// Register-resident multi-step SIR kernel (gfx950): the whole T-step filter of
// a scalar-state model in ONE launch, particles held in VGPRs from the first
// step to the last.
//
// Why: at N = 1e6 a step moves 16 MB — too little for a launch to reach HBM
// streaming rate, and every step of the launch-per-step path (k_step) pays the
// grid fill/drain plus a serial global reduction.  Here each workgroup (1024
// threads, 4 particles per thread, one workgroup per CU, all co-resident)
// keeps its 4096-particle tile in registers and runs the steps back to back.
//
// The only global dependency of a step is the resample decision of the
// previous step (Neff needs the sum over all tiles).  Steps are therefore run
// SPECULATIVELY, assuming "no resample", LAG steps ahead of their
// verification:
//   * after computing a step, a workgroup publishes its tile record
//     (max l, sum e^(l-m), sum e^2(l-m), sum e^(l-m) x, sum e^(l-m) x^2, and
//     the unweighted sums of freshly resampled particles) as 8-byte
//     {tag, float} granules stored write-through (sc1): the data is its own
//     flag, no fences (MI355X_MICROARCH.md, inter-workgroup visibility, R2);
//   * LAG steps later every workgroup loads all records of that step (sc1
//     loads, one round trip that the intervening steps have hidden), reduces
//     them in one fixed order — so all workgroups agree bit for bit — and
//     gets the step's Neff, log normaliser, decision and posterior moments;
//   * no resample (the ~95% case): renormalise the live log-weights by the
//     verified log mass (a uniform shift) and go on;
//   * resample: every workgroup rolls back to its register snapshot of that
//     step, hands the snapshot to the others through HBM (sc1 stores + one
//     flag per workgroup), builds the needed input tiles' fp64 CDF in LDS,
//     gathers the systematic-resampling ancestors, adds the jitter and
//     recomputes the discarded steps.  Noise is counter-based (Philox keyed
//     by particle group / replicate / step epoch), so recomputed steps draw
//     exactly the numbers the speculative ones did.
//
// Random draws, epochs, the systematic position rule and the tile CDF are the
// ones of k_step (pf_kernels.h): the same filter as the launch-per-step path,
// up to fp32 rounding of the reductions' grouping.
#pragma once
#include "pf_kernels.h"

namespace pf {

constexpr int RBS = 512;           // threads per resident workgroup (8 waves, 2 per SIMD)
constexpr int RNW = RBS / 64;      // waves per workgroup
constexpr int RPPT = 8;            // particles per thread = two Philox groups
constexpr int RPV = RPPT / 4;      // float4 vectors per thread
constexpr int RTILE = RBS * RPPT;  // 4096 particles per workgroup
constexpr int RMAXG = 256;         // workgroups per replicate (<= CUs: all co-resident)
constexpr int RCW = RMAXG / 64;    // waves that hold one record each per lane when verifying
constexpr int RRING = 8;           // record ring slots (>= 2*LAG + 2)
constexpr int RF = 7;              // record granules: M, S0, S00, S1, S2, A1, A2
constexpr int RLAG = 2;            // verification lag (steps)
constexpr unsigned RSPIN_LIMIT = 1u << 24;

// Diagnostic phase accounting (PF_STAMPS builds only): workgroup 0, thread 0
// accumulates s_memrealtime ticks (100 MHz) per phase into g_pf_stamps[0..15].
#ifdef PF_STAMPS
#define PF_RMARK(k)                                                      \
  do {                                                                   \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {        \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();  \
      g_pf_stamps[(k)] += now_ - rstamp_last;                            \
      rstamp_last = now_;                                                \
    }                                                                    \
  } while (0)
#define PF_RCOUNT(k)                                                                    \
  do {                                                                                  \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) g_pf_stamps[(k)] += 1; \
  } while (0)
#else
#define PF_RMARK(k) \
  do {              \
  } while (0)
#define PF_RCOUNT(k) \
  do {               \
  } while (0)
#endif

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

struct ResParams {
  const float* x_in;    // [R][Npad] state at entry
  const float* lw_in;   // [R][Npad]
  const double* rec_in; // [R][RS][Gk] k_step records of the entry state
  float* x_fin;         // [R][Npad] state at exit (may alias x_in: each thread reads/writes only its slots)
  float* lw_fin;
  double* rec_fin;      // [R][RS][Gk] k_step records of the exit state
  float* xg;            // [R][Npad] rollback hand-off buffers
  float* lg;
  unsigned long long* gran;   // [R][RRING][RF][RMAXG] record granules (zeroed per launch)
  unsigned long long* sflag;  // [R][RMAXG] hand-off flags (zeroed per launch)
  double* tsum;               // [R][RMAXG] exact tile weight sums published with a hand-off
  unsigned int* err;          // spin timeout word (zeroed per launch)
  const void* P;
  const float* z;  // [T][R][NZ]
  const float* u;  // [T][R][NX] or null
  double* o_mean;
  double* o_cov;   // or null
  double* o_neff;
  double* o_lse;
  int32_t* o_flag;
  int64_t N, Npad, T;
  int G;    // resident workgroups per replicate
  int Gk;   // k_step tiles per replicate (record layout of rec_in / rec_fin)
  int tile_k;
  uint64_t seed;
  uint32_t ep0;
  int first_update_only;
  double thresh;
  int regularize, r_diag, rep_base;
};

__device__ __forceinline__ unsigned long long granule(unsigned tag, float v) {
  return ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v);
}
__device__ __forceinline__ void st_sc1(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_f(float* p, float v) {
  __hip_atomic_store((gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1_f(const float* p) {
  return __uint_as_float(__hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// A value every lane of the workgroup holds identically: move it to scalar registers.
__device__ __forceinline__ double uni(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ long long uni_i64(long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)v >> 32));
  return (long long)(((unsigned long long)hi << 32) | lo);
}

__device__ __noinline__ double pf_dlog(double v) { return log(v); }

// log of a positive double: exact binary exponent + fp32 log of the mantissa
// (|error| ~1e-7 absolute; used for the uniform log-mass shift and lse output).
__device__ __forceinline__ double log_pos(double w) {
  int e;
  const double m = frexp(w, &e);  // w = m 2^e, m in [0.5, 1)
  return (double)e * 0.69314718055994530942 + (double)__logf((float)m);
}

// ---------------------------------------------------------------------------
// Wave reductions on the DPP network (GFX9 DPP: quad_perm, row mirrors,
// row_bcast) instead of LDS-crossbar shuffles.  Fixed combination tree ->
// deterministic, identical in every workgroup.
// ---------------------------------------------------------------------------
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ int dpp_i(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ float dpp_f(float old, float v) {
  return __int_as_float(dpp_i<CTRL, RM>(__float_as_int(old), __float_as_int(v)));
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ double dpp_d(double old, double v) {
  const long long o = __double_as_longlong(old), x = __double_as_longlong(v);
  const int lo = dpp_i<CTRL, RM>((int)o, (int)x);
  const int hi = dpp_i<CTRL, RM>((int)(o >> 32), (int)(x >> 32));
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
enum : int {
  DPP_QP_1032 = 0xB1,
  DPP_QP_2301 = 0x4E,
  DPP_ROW_MIRROR = 0x140,
  DPP_ROW_HMIRROR = 0x141,
  DPP_ROW_BCAST15 = 0x142,
  DPP_ROW_BCAST31 = 0x143
};

// every lane of each 16-lane row gets its row's result
__device__ __forceinline__ float row_max_f(float v) {
  v = fmaxf(v, dpp_f<DPP_QP_1032>(-INFINITY, v));
  v = fmaxf(v, dpp_f<DPP_QP_2301>(-INFINITY, v));
  v = fmaxf(v, dpp_f<DPP_ROW_HMIRROR>(-INFINITY, v));
  v = fmaxf(v, dpp_f<DPP_ROW_MIRROR>(-INFINITY, v));
  return v;
}
__device__ __forceinline__ float row_sum_f(float v) {
  v += dpp_f<DPP_QP_1032>(0.0f, v);
  v += dpp_f<DPP_QP_2301>(0.0f, v);
  v += dpp_f<DPP_ROW_HMIRROR>(0.0f, v);
  v += dpp_f<DPP_ROW_MIRROR>(0.0f, v);
  return v;
}
__device__ __forceinline__ double row_sum_d(double v) {
  v += dpp_d<DPP_QP_1032>(0.0, v);
  v += dpp_d<DPP_QP_2301>(0.0, v);
  v += dpp_d<DPP_ROW_HMIRROR>(0.0, v);
  v += dpp_d<DPP_ROW_MIRROR>(0.0, v);
  return v;
}
__device__ __forceinline__ float lane63_f(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ double lane63_d(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, 63), hi = __builtin_amdgcn_readlane((int)(x >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// whole-wave results (uniform: scalar registers)
__device__ __forceinline__ float wave_max_u(float v) {
  v = row_max_f(v);
  v = fmaxf(v, dpp_f<DPP_ROW_BCAST15, 0xa>(-INFINITY, v));
  v = fmaxf(v, dpp_f<DPP_ROW_BCAST31, 0xc>(-INFINITY, v));
  return lane63_f(v);
}
__device__ __forceinline__ float wave_sum_u(float v) {
  v = row_sum_f(v);
  v += dpp_f<DPP_ROW_BCAST15, 0xa>(0.0f, v);
  v += dpp_f<DPP_ROW_BCAST31, 0xc>(0.0f, v);
  return lane63_f(v);
}
__device__ __forceinline__ double wave_sum_ud(double v) {
  v = row_sum_d(v);
  v += dpp_d<DPP_ROW_BCAST15, 0xa>(0.0, v);
  v += dpp_d<DPP_ROW_BCAST31, 0xc>(0.0, v);
  return lane63_d(v);
}

// Rollback hand-off + systematic resampling of one step (pf.py:146-171, 188-218)
// for the tile of workgroup b.  The step's pre-resample state is this thread's
// snapshot slot (sx_slot / sl_slot); the resampled (and jittered) particles are
// written back into sx_slot.  Out of line: it runs on ~5% of steps and its fp64
// position arithmetic must not occupy registers in the step loop.
// Returns false if the hand-off timed out.
template <typename Real, int NX, int NZ, int TK, int OK>
__device__ __noinline__ bool rb_gather(float* xg, float* lg, unsigned long long* sflag, double* tsum,
                                       unsigned* err, unsigned* err_sh, float4* sx_slot, const float4* sl_slot,
                                       double* red, double* Pl, double* Ck, float* Mk, double* cdf, int G, int b,
                                       int64_t N, unsigned nres, float m_g, float s0_g, double Mx, uint64_t seed,
                                       uint32_t rep, uint32_t ep_res, int regularize, const Real* P) {
  using Mo = Model<Real, NX, NZ, TK, OK>;
  const int t = threadIdx.x;
  const int64_t o0 = (int64_t)b * RTILE;
  const int64_t i0 = o0 + RPPT * (int64_t)t;
  float xv[RPPT], lv[RPPT];
#pragma unroll
  for (int q = 0; q < RPV; ++q) {
    const float4 xs = sx_slot[q * RBS + t], ls = sl_slot[q * RBS + t];
    xv[4 * q] = xs.x; xv[4 * q + 1] = xs.y; xv[4 * q + 2] = xs.z; xv[4 * q + 3] = xs.w;
    lv[4 * q] = ls.x; lv[4 * q + 1] = ls.y; lv[4 * q + 2] = ls.z; lv[4 * q + 3] = ls.w;
  }
  // this tile's exact weight sum, by the very procedure every reader uses to
  // build its CDF below (so the tile's last CDF value meets the next prefix)
  float mown = -INFINITY;
#pragma unroll
  for (int e = 0; e < RPPT; ++e) mown = fmaxf(mown, lv[e]);  // slots past N hold -inf
  {
    const float mw = wave_max_u(mown);
    if ((t & 63) == 0) red[64 + (t >> 6)] = mw;
    __syncthreads();
    mown = -INFINITY;
#pragma unroll
    for (int j = 0; j < RNW; ++j) mown = fmaxf(mown, (float)red[64 + j]);
  }
  double own = 0.0;
#pragma unroll
  for (int e = 0; e < RPPT; ++e) own += (lv[e] > -INFINITY) ? (double)exp_r<float>(lv[e] - mown) : 0.0;
  double Town;
  (void)block_excl_scan<RBS>(own, red, &Town);
  // hand the snapshot to every workgroup: sc1 stores, drain, barrier, one flag
#pragma unroll
  for (int e = 0; e < RPPT; ++e)
    if (i0 + e < N) {
      st_sc1_f(xg + i0 + e, xv[e]);
      st_sc1_f(lg + i0 + e, lv[e]);
    }
  if (t == 0) __hip_atomic_store((gu64*)(tsum + b), (unsigned long long)__double_as_longlong(Town), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) st_sc1(sflag + b, (unsigned long long)nres);
  // wait for every snapshot
  for (unsigned spins = 0;; ++spins) {
    int good = 1;
    if (t < G) good = ld_sc1(sflag + t) == (unsigned long long)nres;
    if (__syncthreads_and(good)) break;
    if (spins >= RSPIN_LIMIT) {
      if (t == 0) {
        *err_sh = 1;
        atomicOr(err, 2u);
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  // global tile prefix in fp64 from the exact tile sums (fixed order)
  double fg = 0.0, wg = 0.0;
  if (t < G && s0_g > 0.0f) {
    fg = exp((double)m_g - Mx);
    wg = __longlong_as_double((long long)ld_sc1((const unsigned long long*)(tsum + t))) * fg;
  }
  double Stot;
  const double run = block_excl_scan<RBS>(wg, red, &Stot);
  if (t < G) {
    Pl[t] = run / Stot;
    Ck[t] = fg / Stot;
    Mk[t] = m_g;
  }
  if (t == 0) Pl[G] = 1.0;
  __syncthreads();
  // systematic positions (U + i) / N of this tile's slots, ancestors by tile CDF
  const double U = uniform53(seed, 0, rep, ep_res);
  const int64_t last = min(o0 + (int64_t)RTILE, N) - 1;
  const int k_lo = prefix_tile(Pl, G, (U + (double)o0) / (double)N);
  const int k_hi = prefix_tile(Pl, G, (U + (double)last) / (double)N);
  int anc[RPPT];
#pragma unroll
  for (int e = 0; e < RPPT; ++e) anc[e] = -1;
  for (int k = k_lo; k <= k_hi; ++k) {
    if (!(Pl[k + 1] > Pl[k])) continue;  // no mass: no position lands here
    const int64_t sk = (int64_t)k * RTILE;
    const int len = (int)min((int64_t)RTILE, N - sk);
    const float mk = Mk[k];
    float lt[RPPT];
    double part = 0.0;
#pragma unroll
    for (int e = 0; e < RPPT; ++e) {
      const int j = RPPT * t + e;
      lt[e] = j < len ? ld_sc1_f(lg + sk + j) : -INFINITY;
      part += (lt[e] > -INFINITY) ? (double)exp_r<float>(lt[e] - mk) : 0.0;
    }
    double tot;
    double off = block_excl_scan<RBS>(part, red, &tot);
    const double c = Ck[k], base = Pl[k];
#pragma unroll
    for (int e = 0; e < RPPT; ++e) {
      const int j = RPPT * t + e;
      off += (lt[e] > -INFINITY) ? (double)exp_r<float>(lt[e] - mk) : 0.0;
      if (j < len) cdf[j] = base + c * off;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < RPPT; ++e) {
      const int64_t i = i0 + e;
      if (i < N && anc[e] < 0) {
        const double pos = (U + (double)i) / (double)N;
        if (prefix_tile(Pl, G, pos) == k) anc[e] = (int)(sk + lds_upper(cdf, len, pos));
      }
    }
    __syncthreads();  // the CDF is rebuilt for the next tile
  }
  Real nj[RPPT];
#pragma unroll
  for (int e = 0; e < RPPT; ++e) nj[e] = Real(0);
  if (regularize) {
#pragma unroll
    for (int q = 0; q < RPV; ++q) {
      const Normal4<Real> nq = normal4<Real>(seed, (uint32_t)((i0 >> 2) + q), rep, ep_res, STREAM_JITTER);
#pragma unroll
      for (int e = 0; e < 4; ++e) nj[4 * q + e] = nq.v[e];
    }
  }
  float xn[RPPT];
#pragma unroll
  for (int e = 0; e < RPPT; ++e) {
    xn[e] = 0.0f;
    if (i0 + e < N) {
      const int a = anc[e] < 0 ? (int)(N - 1) : anc[e];
      Real xe[1] = {ld_sc1_f(xg + a)};
      if (regularize) {
        Real n[1] = {nj[e]};
        Mo::add_lower(xe, n, P, Mo::L::LJ);
      }
      xn[e] = xe[0];
    }
  }
#pragma unroll
  for (int q = 0; q < RPV; ++q) sx_slot[q * RBS + t] = make_float4(xn[4 * q], xn[4 * q + 1], xn[4 * q + 2], xn[4 * q + 3]);
  return true;
}

template <typename Real, int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(RBS) k_resident(ResParams p) {
  static_assert(NX == 1 && sizeof(Real) == 4, "resident path: scalar fp32 state");
  using Mo = Model<Real, NX, NZ, TK, OK>;
  using WA = WAcc<Real, NX>;
  using RC = Rec<NX>;
  constexpr int LAG = RLAG;
  constexpr int NSNAP = LAG + 1;
  __shared__ __attribute__((aligned(16))) double red[LDS_RED];
  __shared__ double mslot[RNW][8];  // per-wave partials of this workgroup's step record
  __shared__ double cslot[RCW][8];  // per-wave partials of a verified step's summary
  __shared__ int okw[RNW];
  __shared__ double sF[NSNAP];  // frame of each snapshot slot
  __shared__ long long sT[NSNAP];  // filter step of each snapshot slot
  __shared__ double Pl[RMAXG + 1];
  __shared__ double Ck[RMAXG];
  __shared__ float Mk[RMAXG];
  __shared__ __attribute__((aligned(16))) double cdf[RTILE];
  __shared__ unsigned err_sh;
  // snapshot ring, thread-private slots: state after each of the last LAG+1 steps
  __shared__ float4 snx[NSNAP][RPV * RBS];
  __shared__ float4 snl[NSNAP][RPV * RBS];

  const int b = blockIdx.x, r = blockIdx.y, R = gridDim.y;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t rep = (uint32_t)(r + p.rep_base);
  // model parameters, loaded once into registers (uniform; a few floats)
  Real P[ParamLayout<NX, NZ>::SIZE];
#pragma unroll
  for (int k = 0; k < ParamLayout<NX, NZ>::SIZE; ++k) P[k] = ((const Real*)p.P)[k];
  const int64_t N = p.N;
  const int G = p.G;
  const int64_t o0 = (int64_t)b * RTILE;
  const int64_t i0 = o0 + RPPT * (int64_t)t;
  const int64_t rN = (int64_t)r * p.Npad;
  const float lunif = (float)(-pf_dlog((double)N));
  const unsigned long long* gbase = p.gran + (size_t)r * RRING * RF * RMAXG;
  if (t == 0) err_sh = 0;
  unsigned long long rstamp_last = 0;
  (void)rstamp_last;
#ifdef PF_STAMPS
  if (b == 0 && r == 0 && t == 0) rstamp_last = __builtin_amdgcn_s_memrealtime();
#endif

  // ---- entry state (k_step layout) and its normaliser ------------------------
  float x[RPPT], l[RPPT];
  {
    const Head h0 = prologue<NX, RBS>(p.rec_in + (int64_t)r * RC::SIZE * p.Gk, p.Gk, N, p.thresh, false, false,
                                      false, red, Pl);
    const float lse0 = (float)uni(h0.lse);
#pragma unroll
    for (int e = 0; e < RPPT; ++e) {
      const bool v = i0 + e < N;
      x[e] = v ? p.x_in[rN + i0 + e] : 0.0f;
      const float lr = v ? p.lw_in[rN + i0 + e] : -INFINITY;
      l[e] = !v ? -INFINITY : (h0.uniform ? lunif : lr - lse0);
    }
  }


  const int fo = p.first_update_only ? 1 : 0;
  int64_t tstep = 0;       // next filter step to compute
  unsigned s_next = 0;     // next sequence number (executed steps, incl. discarded ones)
  unsigned vnext = 0;      // next sequence number to verify
  unsigned nres = 0;       // hand-offs so far (flag tags)
  double F = 0.0;          // frame of the live log-weights
  double Tprev = 0.0;      // absolute log mass of the last verified step
  bool prev_res = false;   // last verified step resampled: next record carries its aux sums
  bool have_aux = false;   // the live state was just gathered
  double aux1 = 0.0, aux2 = 0.0;
  bool last_uniform = false;
  bool alive = true;

  while (alive) {
    const bool computing = tstep < p.T;
    const unsigned s_after = s_next + (computing ? 1u : 0u);
    const bool verify =
        vnext < s_after && (s_after - vnext > (unsigned)LAG || tstep + (computing ? 1 : 0) >= p.T);
    if (!computing && !verify) break;

    // ---------------- prefetch the records to verify (overlaps the step) -----
    unsigned long long pg[RF];
    const unsigned vtag = vnext + 1;
    const unsigned long long* vbase = gbase + (size_t)(vnext % RRING) * RF * RMAXG + t;
    if (verify && t < G) {
#pragma unroll
      for (int f = 0; f < RF; ++f) pg[f] = ld_sc1(vbase + f * RMAXG);
    }
    PF_RMARK(0);

    // ---------------- compute filter step tstep (speculative) ----------------
    if (computing) {
      const bool pred = !(fo && tstep == 0);
      const uint32_t ep_pred = p.ep0 + (uint32_t)(2 * tstep) - fo;
      const float* zt = p.z + ((size_t)tstep * R + r) * NZ;
      Real z[NZ];
#pragma unroll
      for (int k = 0; k < NZ; ++k) z[k] = zt[k];
      const Real* u = p.u ? (const Real*)(p.u + ((size_t)tstep * R + r) * NX) : nullptr;
      Real n4[RPPT];
#pragma unroll
      for (int e = 0; e < RPPT; ++e) n4[e] = Real(0);
      if (pred) {
        // keys made opaque per step: the compiler would otherwise hoist the whole
        // Philox key schedule into (spilled) scalar registers for the entire loop
        uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
        asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
        for (int q = 0; q < RPV; ++q) {
          const Normal4<Real> nq =
              box_muller4(philox4x32_10(u32x4{(uint32_t)((i0 >> 2) + q), rep, ep_pred, STREAM_PROCESS}, k0, k1));
#pragma unroll
          for (int e = 0; e < 4; ++e) n4[4 * q + e] = nq.v[e];
        }
      }
      // branch-free over the thread's slots: slots past N keep l = -inf
#pragma unroll
      for (int e = 0; e < RPPT; ++e) {
        Real xe[1] = {x[e]};
        if (pred) {
          Mo::transition(xe, P, u);
          Real n[1] = {n4[e]};
          Mo::add_lower(xe, n, P, Mo::L::LQ);
        }
        x[e] = xe[0];
        l[e] = l[e] + Mo::loglik(xe, z, P, p.r_diag != 0);
      }
      // this thread's max-first partial sums (invalid slots hold l = -inf)
      float m = l[0];
#pragma unroll
      for (int e = 1; e < RPPT; ++e) m = fmaxf(m, l[e]);
      float s0 = 0.0f, s00 = 0.0f, s1 = 0.0f, s2 = 0.0f;
      if (m > -INFINITY) {
#pragma unroll
        for (int e = 0; e < RPPT; ++e) {
          const float we = (l[e] > -INFINITY) ? __expf(l[e] - m) : 0.0f;
          s0 += we;
          s00 += we * we;
          s1 += we * x[e];
          s2 += we * x[e] * x[e];
        }
      }
      PF_RMARK(1);
      // wave partials (DPP), one LDS slot per wave
      const float Mw = wave_max_u(m);
      const float fw = (m > -INFINITY) ? __expf(m - Mw) : 0.0f;
      const float w0 = wave_sum_u(s0 * fw), w00 = wave_sum_u(s00 * fw * fw);
      const float w1 = wave_sum_u(s1 * fw), w2 = wave_sum_u(s2 * fw);
      double a1 = 0.0, a2 = 0.0;
      if (have_aux) {
        a1 = wave_sum_ud(aux1);
        a2 = wave_sum_ud(aux2);
      }
      if (lane == 0) {
        mslot[w][0] = Mw;
        mslot[w][1] = w0;
        mslot[w][2] = w00;
        mslot[w][3] = w1;
        mslot[w][4] = w2;
        mslot[w][5] = a1;
        mslot[w][6] = a2;
      }
      {  // snapshot of this step in slot s_next % NSNAP
        const int slot = (int)(s_next % NSNAP);
#pragma unroll
        for (int q = 0; q < RPV; ++q) {
          snx[slot][q * RBS + t] = make_float4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
          snl[slot][q * RBS + t] = make_float4(l[4 * q], l[4 * q + 1], l[4 * q + 2], l[4 * q + 3]);
        }
        if (t == 0) {
          sF[slot] = F;
          sT[slot] = tstep;
        }
      }
      __syncthreads();
      if (w == 0) {  // combine the 16 wave partials (row 0 of wave 0) and publish
        const bool in = lane < RNW;
        const float mj = in ? (float)mslot[lane][0] : -INFINITY;
        const float Mt = row_max_f(mj);
        const float fj = (mj > -INFINITY) ? __expf(mj - Mt) : 0.0f;
        const float t0 = row_sum_f(in ? (float)mslot[lane][1] * fj : 0.0f);
        const float t00 = row_sum_f(in ? (float)mslot[lane][2] * fj * fj : 0.0f);
        const float t1 = row_sum_f(in ? (float)mslot[lane][3] * fj : 0.0f);
        const float t2 = row_sum_f(in ? (float)mslot[lane][4] * fj : 0.0f);
        const double ta1 = row_sum_d(in ? mslot[lane][5] : 0.0);
        const double ta2 = row_sum_d(in ? mslot[lane][6] : 0.0);
        if (lane == 0) {  // 7 granules, each one sc1 store (the data is its own flag)
          const unsigned tag = s_next + 1;
          unsigned long long* g = p.gran + ((size_t)r * RRING + s_next % RRING) * RF * RMAXG + b;
          st_sc1(g + 0 * RMAXG, granule(tag, Mt));
          st_sc1(g + 1 * RMAXG, granule(tag, t0));
          st_sc1(g + 2 * RMAXG, granule(tag, t00));
          st_sc1(g + 3 * RMAXG, granule(tag, t1));
          st_sc1(g + 4 * RMAXG, granule(tag, t2));
          st_sc1(g + 5 * RMAXG, granule(tag, (float)ta1));
          st_sc1(g + 6 * RMAXG, granule(tag, (float)ta2));
        }
      }
      PF_RMARK(2);
      PF_RCOUNT(14);
      have_aux = false;
      ++s_next;
      ++tstep;
    }

    // ---------------- verify the oldest unverified step ----------------------
    if (verify) {
      const unsigned v = vnext;
      const int idx = (int)(v % NSNAP);  // snapshot slot of step v
      const double Fv = uni(sF[idx]);  // written before the step's barrier
      const int64_t tv = uni_i64(sT[idx]);
      // all tags in? (the prefetched loads usually are)
      int good = 1;
      if (t < G) {
#pragma unroll
        for (int f = 0; f < RF; ++f) good &= (unsigned)(pg[f] >> 32) == vtag;
      }
      for (unsigned spins = 0;; ++spins) {
        const int wg = __all(good);
        if (lane == 0) okw[w] = wg;
        __syncthreads();
        int all = 1;
#pragma unroll
        for (int j = 0; j < RCW; ++j) all &= okw[j];
        all = __builtin_amdgcn_readfirstlane(all);
        if (all) break;
        __syncthreads();  // okw is rewritten below
        PF_RCOUNT(15);
        if (spins >= RSPIN_LIMIT) {
          if (t == 0) {
            err_sh = 1;
            atomicOr(p.err, 1u);
          }
          alive = false;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        good = 1;
        if (t < G) {
#pragma unroll
          for (int f = 0; f < RF; ++f) {
            pg[f] = ld_sc1(vbase + f * RMAXG);
            good &= (unsigned)(pg[f] >> 32) == vtag;
          }
        }
      }
      if (!alive) break;
      PF_RMARK(3);
      // summary of the step: waves 0..RCW-1 hold one record per lane
      const bool in = t < G;
      const float m_g = in ? __uint_as_float((unsigned)pg[0]) : -INFINITY;
      const float s0_g = in ? __uint_as_float((unsigned)pg[1]) : 0.0f;
      float fl_g = 0.0f;  // e^(m_g - wave max)
      if (w < RCW) {
        const float mg = (s0_g > 0.0f) ? m_g : -INFINITY;
        const float Mw = wave_max_u(mg);
        fl_g = (mg > -INFINITY) ? __expf(mg - Mw) : 0.0f;
        const double f = (double)fl_g;
        const double d0 = wave_sum_ud((double)s0_g * f);
        const double d1 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[2]) * f * f : 0.0);
        const double d2 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[3]) * f : 0.0);
        const double d3 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[4]) * f : 0.0);
        const double d4 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[5]) : 0.0);
        const double d5 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[6]) : 0.0);
        if (lane == 0) {
          cslot[w][0] = Mw;
          cslot[w][1] = d0;
          cslot[w][2] = d1;
          cslot[w][3] = d2;
          cslot[w][4] = d3;
          cslot[w][5] = d4;
          cslot[w][6] = d5;
        }
      }
      __syncthreads();
      double Mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < RCW; ++j) Mx = fmax(Mx, cslot[j][0]);
      Mx = uni(Mx);
      double W = 0.0, W2 = 0.0, S1 = 0.0, S2 = 0.0, A1 = 0.0, A2 = 0.0;
#pragma unroll
      for (int j = 0; j < RCW; ++j) {
        const double mj = cslot[j][0];
        const double Fj = (mj > -INFINITY) ? (double)__expf((float)(mj - Mx)) : 0.0;
        W += cslot[j][1] * Fj;
        W2 += cslot[j][2] * Fj * Fj;
        S1 += cslot[j][3] * Fj;
        S2 += cslot[j][4] * Fj;
        A1 += cslot[j][5];
        A2 += cslot[j][6];
      }
      W = uni(W);
      W2 = uni(W2);
      S1 = uni(S1);
      S2 = uni(S2);
      A1 = uni(A1);
      A2 = uni(A2);
      PF_RMARK(4);
      const double lse_rel = Mx + log_pos(W);
      const double neff = (W * W) / W2;
      const bool dec = neff < p.thresh * (double)N;
      const double Tv = lse_rel + Fv;
      if (b == 0 && t == 0) {
        const int64_t o = tv * R + r;
        p.o_neff[o] = neff;
        p.o_lse[o] = Tv - Tprev;
        p.o_flag[o] = dec ? 1 : 0;
        const double mean = S1 / W;
        p.o_mean[o] = mean;
        if (p.o_cov) p.o_cov[o] = S2 / W - mean * mean;
        if (prev_res) {  // post-resample moments of step tv - 1 (uniform weights)
          const int64_t o2 = (tv - 1) * R + r;
          const double mp = A1 / (double)N;
          p.o_mean[o2] = mp;
          if (p.o_cov) p.o_cov[o2] = A2 / (double)N - mp * mp;
        }
      }
      prev_res = false;
      if (!dec) {
        Tprev = Tv;
        const float delta = (float)(Tv - F);
#pragma unroll
        for (int e = 0; e < RPPT; ++e) l[e] = l[e] - delta;  // -inf stays -inf
        F += (double)delta;
        vnext = v + 1;
        last_uniform = false;
      } else {
        // ---- rollback to step tv and resample it (out of line: rare) ----------
        PF_RCOUNT(13);
        ++nres;
        const uint32_t ep_res = p.ep0 + (uint32_t)(2 * tv + 1) - fo;
        if (!rb_gather<Real, NX, NZ, TK, OK>(p.xg + rN, p.lg + rN, p.sflag + (size_t)r * RMAXG,
                                              p.tsum + (size_t)r * RMAXG, p.err, &err_sh, snx[idx], snl[idx], red,
                                              Pl, Ck, Mk, cdf, G, b, N, nres, m_g, s0_g, Mx, p.seed, rep, ep_res,
                                              p.regularize, (const Real*)p.P)) {
          alive = false;
          break;
        }
#pragma unroll
        for (int q = 0; q < RPV; ++q) {
          const float4 xs = snx[idx][q * RBS + t];
          x[4 * q] = xs.x;
          x[4 * q + 1] = xs.y;
          x[4 * q + 2] = xs.z;
          x[4 * q + 3] = xs.w;
        }
        aux1 = 0.0;
        aux2 = 0.0;
#pragma unroll
        for (int e = 0; e < RPPT; ++e) {
          if (i0 + e < N) {
            l[e] = lunif;
            aux1 += (double)x[e];
            aux2 += (double)x[e] * (double)x[e];
          } else {
            x[e] = 0.0f;
            l[e] = -INFINITY;
          }
        }
        PF_RMARK(5);
        have_aux = true;
        prev_res = true;
        last_uniform = true;
        F = 0.0;
        Tprev = 0.0;
        tstep = tv + 1;
        vnext = s_next;  // the speculative steps after tv are discarded
      }
    }
  }

  // ---- the last step resampled: its post-resample moments -------------------
  if (alive && prev_res) {
    const double a1 = wave_sum_ud(aux1), a2 = wave_sum_ud(aux2);
    if (lane == 0) {
      mslot[w][5] = a1;
      mslot[w][6] = a2;
    }
    __syncthreads();
    if (t == 0) {
      double A1 = 0.0, A2 = 0.0;
      for (int j = 0; j < RNW; ++j) {
        A1 += mslot[j][5];
        A2 += mslot[j][6];
      }
      const unsigned tag = s_next + 1;
      unsigned long long* g = p.gran + ((size_t)r * RRING + s_next % RRING) * RF * RMAXG + b;
      st_sc1(g + 5 * RMAXG, granule(tag, (float)A1));
      st_sc1(g + 6 * RMAXG, granule(tag, (float)A2));
    }
    // every workgroup's aux granules (fixed-order sum in each workgroup)
    const unsigned tag = s_next + 1;
    const unsigned long long* base = gbase + (size_t)(s_next % RRING) * RF * RMAXG + t;
    for (unsigned spins = 0;; ++spins) {
      int good = 1;
      unsigned long long g5 = 0, g6 = 0;
      if (t < G) {
        g5 = ld_sc1(base + 5 * RMAXG);
        g6 = ld_sc1(base + 6 * RMAXG);
        good = ((unsigned)(g5 >> 32) == tag) && ((unsigned)(g6 >> 32) == tag);
      }
      const int wg = __all(good);
      if (lane == 0) okw[w] = wg;
      __syncthreads();
      int all = 1;
#pragma unroll
      for (int j = 0; j < RCW; ++j) all &= okw[j];
      all = __builtin_amdgcn_readfirstlane(all);
      if (all) {
        if (w < RCW) {
          const double d4 = wave_sum_ud(t < G ? (double)__uint_as_float((unsigned)g5) : 0.0);
          const double d5 = wave_sum_ud(t < G ? (double)__uint_as_float((unsigned)g6) : 0.0);
          if (lane == 0) {
            cslot[w][5] = d4;
            cslot[w][6] = d5;
          }
        }
        __syncthreads();
        if (b == 0 && t == 0) {
          double S5 = 0.0, S6 = 0.0;
          for (int j = 0; j < RCW; ++j) {
            S5 += cslot[j][5];
            S6 += cslot[j][6];
          }
          const int64_t o2 = (p.T - 1) * R + r;
          const double mp = S5 / (double)N;
          p.o_mean[o2] = mp;
          if (p.o_cov) p.o_cov[o2] = S6 / (double)N - mp * mp;
        }
        break;
      }
      __syncthreads();
      if (spins >= RSPIN_LIMIT) {
        if (t == 0) atomicOr(p.err, 4u);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }

  // ---- exit state in the k_step layout ---------------------------------------
#pragma unroll
  for (int e = 0; e < RPPT; ++e)
    if (i0 + e < N) {
      p.x_fin[rN + i0 + e] = x[e];
      p.lw_fin[rN + i0 + e] = l[e];
    }
  // one k_step record per group of KQ threads (k_step tile = 1024 particles)
  {
    constexpr int KQ = 1024 / RPPT, KW = KQ / 64;
    const int q = t / KQ;
    const int kt = b * (RTILE / 1024) + q;
    WA acc;
    acc.init();
#pragma unroll
    for (int e = 0; e < RPPT; ++e)
      if (i0 + e < N) {
        Real xe[1] = {x[e]};
        acc.add(l[e], xe);
      }
    const float Mw = wave_max_u(acc.m);
    const float f = (acc.m > -INFINITY) ? __expf(acc.m - Mw) : 0.0f;
    double vs[WA::NS];
#pragma unroll
    for (int i = 0; i < WA::NS; ++i) vs[i] = wave_sum_ud((double)acc.s[i] * (double)(i == 1 ? f * f : f));
    __syncthreads();
    if (lane == 0) {
      red[w * (WA::NS + 1)] = Mw;
#pragma unroll
      for (int i = 0; i < WA::NS; ++i) red[w * (WA::NS + 1) + 1 + i] = vs[i];
    }
    __syncthreads();
    if ((t % KQ) == 0 && kt < p.Gk) {
      double Mq = -INFINITY;
      for (int j = 0; j < KW; ++j) Mq = fmax(Mq, red[(KW * q + j) * (WA::NS + 1)]);
      double sum[WA::NS];
#pragma unroll
      for (int i = 0; i < WA::NS; ++i) sum[i] = 0.0;
      for (int j = 0; j < KW; ++j) {
        const double mj = red[(KW * q + j) * (WA::NS + 1)];
        const double fj = (mj > -INFINITY) ? (double)__expf((float)(mj - Mq)) : 0.0;
#pragma unroll
        for (int i = 0; i < WA::NS; ++i) sum[i] += red[(KW * q + j) * (WA::NS + 1) + 1 + i] * (i == 1 ? fj * fj : fj);
      }
      double* o = p.rec_fin + (int64_t)r * RC::SIZE * p.Gk;
      for (int f2 = 0; f2 < RC::SIZE; ++f2) o[(int64_t)f2 * p.Gk + kt] = 0.0;
      if (last_uniform) {
        o[(int64_t)RC::UNI * p.Gk + kt] = 1.0;
      } else {
        o[(int64_t)RC::M * p.Gk + kt] = Mq;
        o[(int64_t)RC::S0 * p.Gk + kt] = sum[0];
        o[(int64_t)RC::S00 * p.Gk + kt] = sum[1];
        for (int i = 0; i < NX + RC::NC; ++i) o[(int64_t)(RC::S1 + i) * p.Gk + kt] = sum[2 + i];
      }
    }
  }
}

}  // namespace pf
