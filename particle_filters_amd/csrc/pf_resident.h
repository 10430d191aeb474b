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
#include <type_traits>

#include "pf_kernels.h"

namespace pf {

#ifndef PF_RBS
#define PF_RBS 512
#endif
constexpr int RBS = PF_RBS;        // threads per resident workgroup (8 waves, 2 per SIMD)
constexpr int RNW = RBS / 64;      // waves per workgroup
constexpr int RPPT = 4096 / RBS;   // particles per thread (8 = two Philox groups); tile fixed at 4096
constexpr int RPV = RPPT / 4;      // float4 vectors per thread
constexpr int RTILE = RBS * RPPT;  // 4096 particles per workgroup
constexpr int RMAXG = 256;         // workgroups per replicate (<= CUs: all co-resident)
constexpr int RCW = RMAXG / 64;    // waves that hold one record each per lane when verifying
constexpr int RRING = 8;           // record ring slots (>= 2*LAG + 2)
constexpr int RF = 8;              // record granules: M, S0 (high word), S00, S1, S2, A1, A2, S0 (low word)
#ifndef PF_RSHARDS
#define PF_RSHARDS 8
#endif
constexpr int RSHARDS = PF_RSHARDS;  // arrival count shards (res_arrive_sharded)
constexpr int RSHARD_WORDS = 512;  // 4 KiB between shards (different lines and channels)
#ifndef PF_RLAG
#define PF_RLAG 2
#endif
constexpr int RLAG = PF_RLAG;      // verification lag (steps)
#ifndef PF_PUB_PRIO
#define PF_PUB_PRIO 1
#endif
#ifndef PF_PUBW
#define PF_PUBW (RNW - 1)  // the wave that combines and publishes the workgroup's record
#endif
#ifndef PF_RCOPIES
#define PF_RCOPIES 8
#endif
// Replicas of the record ring.  Every workgroup reads every record of every step: with one
// copy, ~1000 sc1 loads per step hit the same few lines, i.e. the same memory channels.
// Writers store all replicas in one instruction (lane = field + RF * replica); reader b uses
// replica b % RCOPIES.
constexpr int RCOPIES = PF_RCOPIES;
static_assert(RF * RCOPIES <= 64, "one publishing wave stores every granule of every replica");
// elements between replicas: one replica ([R][RRING][RF][RMAXG]) rounded up to 4 KiB, plus
// 36 KiB, so that the replicas start on different memory channels
__host__ __device__ inline size_t gran_copy_stride(int R) {
  const size_t n = (size_t)R * RRING * RF * RMAXG;
  return (n + 511) / 512 * 512 + 4608;
}
constexpr unsigned RSPIN_LIMIT = 1u << 24;
#ifndef PF_CB_FLOOR
#define PF_CB_FLOOR 1
#endif
#ifndef PF_RSTAGE
#define PF_RSTAGE 8192
#endif
constexpr int RSTAGE = PF_RSTAGE;  // rollback scatter staging chunk (floats of LDS)

// Diagnostic phase accounting (PF_STAMPS builds only): one thread (PF_STAMP_T of workgroup
// PF_STAMP_B) accumulates s_memrealtime ticks (100 MHz) per phase into g_pf_stamps[0..15, 22, 23].
#ifdef PF_STAMPS
// accumulated in registers (thread 0 of workgroup 0), written once at the end
#define PF_RMARK(k)                                                     \
  do {                                                                  \
    if (stamp_me) {                                                     \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime(); \
      racc[(k)] += now_ - rstamp_last;                                  \
      rstamp_last = now_;                                               \
    }                                                                   \
  } while (0)
#define PF_RCOUNT(k)            \
  do {                          \
    if (stamp_me) racc[(k)] += 1; \
  } while (0)
// rare-path phases (rollback): register accumulators of thread 0 of workgroup 0, added to the
// global slots once at the end of the rollback (a global read-modify-write at every mark would
// put its load latency into the next phase)
#define PF_GMARK(k)                                                                   \
  do {                                                                                \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {                     \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();               \
      gacc[(k) - 6] += now_ - gstamp_last;                                            \
      gstamp_last = now_;                                                             \
    }                                                                                 \
  } while (0)
#define PF_GFLUSH()                                                                    \
  do {                                                                                \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)                       \
      for (int k_ = 0; k_ < 6; ++k_) g_pf_stamps[6 + k_] += gacc[k_];                 \
  } while (0)
#else
#define PF_GMARK(k) \
  do {              \
  } while (0)
#define PF_GFLUSH() \
  do {              \
  } while (0)
#define PF_RMARK(k) \
  do {              \
  } while (0)
#define PF_RCOUNT(k) \
  do {               \
  } while (0)
#endif

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int PF_AUX_SC1 = 16;  // buffer instruction cache-policy bits: sc1 (write-through / L1 bypass)

typedef const __attribute__((address_space(4))) float CReal;  // uniform read-only inputs: scalar loads
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
  unsigned long long* gran;   // [R][RRING][RF][RMAXG] record granules, tag = tag0 + sequence + 1
  unsigned long long* sflag;  // [R][RMAXG] hand-off flags, value = flag0 + rollback count
  unsigned int* err;          // spin timeout / all-dead word (zeroed at allocation and after a report)
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
  // Launch-unique bases of the granule tags and hand-off flag values: the handle
  // advances them past everything a launch can publish (tags <= 3T + 2 per launch,
  // flags <= T), so words left by earlier launches never match and the sync words
  // need no zeroing launch per launch (no memset in front of the kernel).
  uint32_t tag0;
  unsigned long long flag0;
  int r0, Rtot;  // first replicate of this launch's group; the handle's replicate count (strides)
  // Co-residency check (res_arrive / res_try_abort).  arrive[0]: workgroups arrived over all
  // launches, plus RABORT per aborted launch (arrive0: its value before this launch); arrive[1]:
  // the first aborted launch's sequence number (atomicMin; all-ones when none).
  unsigned long long* arrive;
  unsigned long long arrive0, seq;
  // Arrival shards (res_arrive_sharded): workgroup w counts itself into shard w % nshard (RSHARD_WORDS
  // apart, values grow by the shard's workgroup count per launch from shard_base, +RABORT per abort
  // mark); arrive[0] is the launch's abort decision word (res_try_abort_sharded), arrive[1] the first
  // aborted launch's sequence number.
  unsigned long long* arrive_sh;
  unsigned long long shard_base[RSHARDS];
  int nshard;
  int test_abort;  // test hook: the last workgroup arrives only after the others gave up
  // Entry header [R][4] {run id, lse of the exit log-weights (double bits), uniform, -}: written
  // at exit by workgroup 0 of each replicate (id hdr_out); a launch whose hdr_in matches the
  // stored id skips the records' prologue (the host invalidates it on any other state write).
  unsigned long long* hdr;
  unsigned long long hdr_in, hdr_out;
  // Verification trace (k_resident<..., TR = true> only; tests): for every VERIFIED step tv < tr_T
  // of the launch - the version that was kept, after any rollback and recomputation - its
  // predicted particles and pre-resample log-weights (any frame: the snapshot the verification
  // read) into tr_x / tr_l [tr_T][Rtot][Npad], and on a resample step the ancestor of every
  // output slot into tr_anc [tr_T][Rtot][Npad].
  float* tr_x;
  float* tr_l;
  int32_t* tr_anc;
  int64_t tr_T;
};


// Granules a verifying workgroup reads: every workgroup needs M, S0 (both words), S00
// (log mass, Neff, decision, rollback prefix); only the output workgroup needs the
// moment and aux granules (S1, S2, A1, A2).  The tile mass S0 travels as an fp64 value
// split over two granules: it places the tile's slice of the systematic-resampling CDF
// (rb_gather), where an fp32 tile mass (~1e-7 relative) would move ~0.1 N slot
// boundaries per resample against the fp64 reference.
__device__ __forceinline__ bool vg_need(int f, bool outwg) {
#ifdef PF_VG_ALL
  return true;
#else
  return f < 3 || f == 7 || outwg;
#endif
}

__device__ __forceinline__ unsigned long long granule(unsigned tag, float v) {
  return ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v);
}
// an fp64 value carried by two granules (payload = high / low 32 bits)
__device__ __forceinline__ double granule_f64(unsigned long long hi, unsigned long long lo) {
  return __longlong_as_double((long long)(((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull)));
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

constexpr unsigned long long RARRIVE_TICKS = 100000;  // 1 ms of s_memrealtime (100 MHz) for the grid to arrive
constexpr unsigned long long RABORT = 1ull << 40;      // added to the arrival count by an abort

// Co-residency.  The workgroups wait for each other's records, so the whole grid must be
// resident at once; a plain launch does not promise that (other work may hold CUs), so the
// kernel checks it.  Each workgroup counts itself in (res_arrive) before it touches any state.
// Verifying a step needs every workgroup's record, so once any step is verified every
// workgroup has arrived: nothing else is needed on the normal path.  A workgroup that waits
// for records for more than 1 ms tries to abort (res_try_abort): a compare-and-swap that adds
// RABORT to the count, possible only while the count is incomplete - so "abort" and "all
// arrived" exclude each other.  Workgroups arriving after an abort see it in their count and
// leave at once; nobody writes state, the host reports PF_E_RETRY.  Thread 0; vector atomics.
__device__ __forceinline__ unsigned long long res_arrive(unsigned long long* arrive) { return atomicAdd(arrive, 1ull); }

// true: the launch is aborted (leave); false: every workgroup has arrived (keep waiting)
__device__ __forceinline__ bool res_try_abort(unsigned long long* arrive, unsigned* err, unsigned long long arrive0,
                                              unsigned long long total, unsigned long long seq) {
  for (;;) {
    const unsigned long long w = ld_sc1(arrive), rel = w - arrive0;
    if (rel >= RABORT) return true;
    if (rel >= total) return false;
    if (atomicCAS(arrive, w, w + RABORT) == w) {
      atomicOr(err, 16u);
      atomicMin(arrive + 1, seq);
      return true;
    }
  }
}

// Arrival (co-residency) in one uncontended round trip (rounds 1-5: one counter, res_arrive).  The
// single counter serialised the launch's entry: ~245 device-scope adds on one word, the last workgroup's
// return ~3 us after the first - on the critical path of every launch (84.0-84.5 vs 87.1-87.8 us per
// 20-step window without it, profiles/r06/arrive).  Now workgroup w adds 1 to shard w % nshard
// (RSHARD_WORDS apart; the host advances shard k's base by its workgroup count ck per launch) and
// goes on unless that add finds an abort mark (+RABORT) on its shard.  An abort is decided once per
// launch by the first workgroup that waits 1 ms for the first verification (res_try_abort_sharded):
// it takes the decision word arrive[0] for this launch (CAS to seq << 2 | LOCK), adds RABORT to every
// shard, and the abort stands iff some shard had not all its ck arrivals when marked; it stores the
// decision (ABORT, or COMPLETE after taking its marks back).  Exclusion: a workgroup passes the first
// verification only when every workgroup has published, i.e. every add returned no mark - all before
// the marks, so the decision was COMPLETE; after ABORT the missing workgroup's add finds the mark and it
// leaves unpublished, so nobody passes, and the waiting ones leave on reading ABORT (state untouched).
// The host re-reads the shards after an abort (check_resident).  Returns 1: go on, 0: leave.  Thread 0.
// (p: the kernel arguments in the kernarg segment - read where used, not carried in registers)
constexpr unsigned long long RDEC_LOCK = 1, RDEC_ABORT = 2, RDEC_COMPLETE = 3;
template <class CResP>
__device__ __forceinline__ int res_arrive_sharded(CResP p, unsigned long long sh_old) {
  const unsigned nsh = (unsigned)p->nshard;
  const unsigned k = (blockIdx.y * gridDim.x + blockIdx.x) % nsh;
  return sh_old - p->shard_base[k] < RABORT ? 1 : 0;
}
template <class CResP>
__device__ __forceinline__ bool res_try_abort_sharded(CResP p) {
  unsigned long long* dec = p->arrive;
  const unsigned long long mine = (unsigned long long)p->seq << 2;
  for (;;) {
    const unsigned long long d = ld_sc1(dec);
    if ((d >> 2) == p->seq) {  // decided or being decided for this launch
      if ((d & 3) == RDEC_ABORT) return true;
      if ((d & 3) == RDEC_COMPLETE) return false;
      __builtin_amdgcn_s_sleep(8);
      continue;
    }
    if (atomicCAS(dec, d, mine | RDEC_LOCK) != d) continue;
    const unsigned nsh = (unsigned)p->nshard, nwg = gridDim.x * gridDim.y;
    bool open = false;
    for (unsigned k = 0; k < nsh; ++k) {
      const unsigned long long ck = (nwg - k + nsh - 1) / nsh;
      const unsigned long long old = atomicAdd(p->arrive_sh + (size_t)k * RSHARD_WORDS, RABORT) - p->shard_base[k];
      open |= old < ck;  // (no earlier mark in this launch: only the lock holder marks)
    }
    if (!open) {  // every workgroup had arrived: take the marks back, nobody arrives any more
      for (unsigned k = 0; k < nsh; ++k) atomicAdd(p->arrive_sh + (size_t)k * RSHARD_WORDS, 0ull - RABORT);
      __hip_atomic_exchange((gu64*)dec, mine | RDEC_COMPLETE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    atomicOr(p->err, 16u);
    atomicMin(p->arrive + 1, p->seq);
    __hip_atomic_exchange((gu64*)dec, mine | RDEC_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
}
// every shard has all its arrivals and no mark (the whole grid is in); thread 0
template <class CResP>
__device__ __forceinline__ bool res_all_arrived(CResP p) {
  const unsigned nsh = (unsigned)p->nshard, nwg = gridDim.x * gridDim.y;
  bool all = true;
  for (unsigned k = 0; k < nsh; ++k)
    all &= ld_sc1(p->arrive_sh + (size_t)k * RSHARD_WORDS) - p->shard_base[k] == (unsigned long long)((nwg - k + nsh - 1) / nsh);
  return all;
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

// Number of systematic positions below x: #{ i in [0, N) : (U + i) / N < x },
// evaluated with the very comparison the reference makes (pf.py:146-171: pos =
// (U + arange(N)) / N in fp64, ancestor = first j with pos < cdf[j]).
__device__ __noinline__ int count_below_exact(double x, double U, int N, int c) {
  const double Nd = (double)N;
  while (c > 0 && (U + (double)(c - 1)) / Nd >= x) --c;
  while (c < N && (U + (double)c) / Nd < x) ++c;
  return c;
}
__device__ __forceinline__ int count_below(double x, double U, int N) {
  // exactly, (U + i) / N < x  <=>  i < y = x N - U; the fp64 division can only
  // disagree when (U + i) / N lies within an ulp of x, i.e. when y is within
  // ~1e-10 of an integer: only then are the candidate positions evaluated the
  // reference's way (out of line: it is rare).  32-bit slot indices (N < 2^31).
  const double y = fma(x, (double)N, -U);
#if PF_CB_FLOOR
  // floor + fraction: the same test in fewer fp64 instructions (the clamp in integers)
  const double fl = floor(y), d = y - fl;
  const int c = min(max((int)fl + 1, 0), N);
  if (d > 1e-7 && d < 1.0 - 1e-7) return c;
#else
  const double c0 = ceil(y);
  const int c = (int)fmin(fmax(c0, 0.0), (double)N);
  if (c0 - y > 1e-7 && y - (c0 - 1.0) > 1e-7) return c;
#endif
  return count_below_exact(x, U, N, c);
}

// Two exclusive block scans in one pass (one pair of barriers): returns a's exclusive prefix,
// *tot_a / *tot_b the totals, *excl_b b's exclusive prefix.  red >= 2 * BS / 64 doubles.
template <int BS>
__device__ __forceinline__ double block_excl_scan2(double a, double b, double* red, double* tot_a, double* excl_b,
                                                   double* tot_b) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double ia = wave_incl_scan_dpp(a), ib = wave_incl_scan_dpp(b);
  __syncthreads();
  if (lane == 63) {
    red[w] = ia;
    red[NW + w] = ib;
  }
  __syncthreads();
  double oa = 0.0, ta = 0.0, ob = 0.0, tb = 0.0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    if (i < w) {
      oa += red[i];
      ob += red[NW + i];
    }
    ta += red[i];
    tb += red[NW + i];
  }
  *tot_a = ta;
  *tot_b = tb;
  *excl_b = ob + ib - b;
  return oa + ia - a;
}

// Rollback + systematic resampling of one step (pf.py:146-171, 188-218), source-
// driven: workgroup b owns input tile b (its snapshot in LDS), builds that tile's
// fp64 CDF segment, and writes each particle into its offspring slots
// [C(cdf_{j-1}), C(cdf_j)) of the gathered array — no remote tile reads, work per
// workgroup proportional to its tile's offspring.  One grid hand-off (the
// gathered array): the global tile prefix comes from the verified records.  The resampled
// (and jittered) particles of this workgroup's output slots land in sx_slot.
// Out of line: it runs on ~5% of steps and its fp64 position arithmetic must not
// occupy registers in the step loop.  Returns false if a hand-off timed out.
template <typename Real, int NX, int NZ, int TK, int OK>
__device__ __forceinline__ bool rb_gather(float* xn, unsigned long long* sflag, unsigned long long flag0, unsigned* err,
                                       unsigned* err_sh, float4* sx_slot, const float4* sl_slot, double* red,
                                       double* Pl, double* Ck, double* offs, float* stage, int G, int b, int64_t N,
                                       unsigned nres,
                                       float m_g, double s0_g, double Mx, uint64_t seed, uint32_t rep,
                                       uint32_t ep_res, int regularize, const Real* P, int32_t* tanc) {
  using Mo = Model<Real, NX, NZ, TK, OK>;
  const int t = threadIdx.x;
  const int N32 = (int)N;  // resident grids: N <= RMAXG * RTILE < 2^31
  const int o0 = b * RTILE;
  const int i0 = o0 + RPPT * t;
#ifdef PF_STAMPS
  unsigned long long gstamp_last = __builtin_amdgcn_s_memrealtime();
  unsigned long long gacc[6] = {0, 0, 0, 0, 0, 0};
#endif
  float xv[RPPT], lv[RPPT];
#pragma unroll
  for (int q = 0; q < RPV; ++q) {
    const float4 xs = sx_slot[q * RBS + t], ls = sl_slot[q * RBS + t];
    xv[4 * q] = xs.x; xv[4 * q + 1] = xs.y; xv[4 * q + 2] = xs.z; xv[4 * q + 3] = xs.w;
    lv[4 * q] = ls.x; lv[4 * q + 1] = ls.y; lv[4 * q + 2] = ls.z; lv[4 * q + 3] = ls.w;
  }
  // ---- this tile's weights relative to its max, exclusive prefix, exact sum --
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
  double wv[RPPT];
  double part = 0.0;
#pragma unroll
  for (int e = 0; e < RPPT; ++e) {
    wv[e] = (lv[e] > -INFINITY) ? (double)exp_r<float>(lv[e] - mown) : 0.0;
    part += wv[e];
  }
  // No hand-off for the tile masses: every workgroup already holds all tiles'
  // verified records {m_g, s0_g} (thread t: tile t), so the global tile prefix is
  // computed from those; each tile then maps its own fp64 CDF exactly onto its
  // prefix interval [Pl[b], Pl[b+1]) (the offspring ranges still partition [0, N)).
  // The xn write-after-read hazard across rollbacks is ordered by the granule
  // protocol: a rollback is decided only after every workgroup has published a
  // step computed from its previous gathered read.
  // One pair of scans: this tile's exclusive prefix and the global tile prefix (fp64, fixed
  // order: identical in every workgroup).
  double fg = 0.0, wg = 0.0;
  if (t < G && s0_g > 0.0) {
    fg = exp((double)m_g - Mx);
    wg = s0_g * fg;
  }
  double Town, Stot, run;
  const double off = block_excl_scan2<RBS>(part, wg, red, &Town, &run, &Stot);
  offs[t] = off;
  PF_GMARK(6);
  if (t < G) {
    Pl[t] = run / Stot;
    Ck[t] = fg / Stot;
  }
  if (t == 0) Pl[G] = 1.0;  // the reference's cdf[-1] = 1.0
  __syncthreads();
  PF_GMARK(8);
  // ---- offspring ranges of this tile's particles ------------------------------
  // particle j of the tile takes output slots [C(cdf_{j-1}), C(cdf_j)); the whole
  // tile takes the contiguous range [C(Pl[b]), C(Pl[b+1])), staged through LDS
  // in chunks and written with coalesced 16-byte sc1 stores.
  const double U = uniform53(seed, 0, rep, ep_res);
  const double base = Pl[b], hi = Pl[b + 1], c = (Town > 0.0) ? (hi - base) / Town : 0.0;
  const int tile_last = min(o0 + RTILE, N32) - 1;
  int cb[RPPT + 1];  // cb[e] .. cb[e+1]: slots of particle i0 + e (empty past the tile)
  {
    const double xb = (i0 + RPPT - 1 >= tile_last) ? hi : base + c * offs[t + 1];
    cb[0] = (i0 <= tile_last) ? count_below(base + c * off, U, N32) : 0;
    double cum = off;
#pragma unroll
    for (int e = 0; e < RPPT; ++e) {
      const int j = i0 + e;
      if (j > tile_last) {
        cb[e + 1] = cb[e];
        continue;
      }
      cum += wv[e];
      const double xe = (e == RPPT - 1 || j == tile_last) ? xb : fmin(base + c * cum, xb);
      cb[e + 1] = max(count_below(xe, U, N32), cb[e]);
    }
  }
  const int R0 = count_below(base, U, N32), R1 = count_below(hi, U, N32);
  // the hand-off below waits only for the tiles whose offspring land in this workgroup's
  // output slots [o0, o0 + RTILE) (thread t: tile t; typically this tile and a neighbour)
  bool is_src = false;
  if (t < G) {
    const int c0 = count_below(Pl[t], U, N32), c1 = count_below(Pl[t + 1], U, N32);
    is_src = c0 < o0 + RTILE && c1 > o0 && c1 > c0;
  }
  PF_GMARK(7);
  if (tanc) {  // trace build: the ancestor of every offspring slot (tanc is a null constant otherwise)
#pragma unroll
    for (int e = 0; e < RPPT; ++e)
      for (int i = cb[e]; i < cb[e + 1]; ++i) tanc[i] = i0 + e;
  }
  for (int cs = R0; cs < R1; cs += RSTAGE) {
    const int ce = min(cs + RSTAGE, R1);
#pragma unroll
    for (int e = 0; e < RPPT; ++e) {
      const int a0 = max(cb[e], cs), a1 = min(cb[e + 1], ce);
      for (int i = a0; i < a1; ++i) stage[i - cs] = xv[e];
    }
    __syncthreads();
    // coalesced write of stage[0, ce - cs) to xn[cs, ce): unaligned head/tail scalar
    const int body0 = (cs + 3) & ~3, body1 = ce & ~3;
    if (body0 >= body1) {
      for (int i = cs + t; i < ce; i += RBS) st_sc1_f(xn + i, stage[i - cs]);
    } else {
      if (t < body0 - cs) st_sc1_f(xn + cs + t, stage[t]);
      if (t < ce - body1) st_sc1_f(xn + body1 + t, stage[body1 - cs + t]);
      const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(xn, 0, (int)(N * 4), 0x00020000);
      for (int i = body0 + 4 * t; i < body1; i += 4 * RBS) {
        const int k = i - cs;
        const v4f v = {stage[k], stage[k + 1], stage[k + 2], stage[k + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(v, rw, (int)(i * 4), 0, PF_AUX_SC1);
      }
    }
    __syncthreads();  // stage is refilled by the next chunk
  }
  PF_GMARK(9);
  // ---- hand-off: the gathered array (from the source tiles of this workgroup's slots) ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long f2 = flag0 + nres;  // one hand-off per rollback: flags count rollbacks
  if (t == 0) st_sc1(sflag + b, f2);
  for (unsigned spins = 0;; ++spins) {
    int good = 1;
    if (is_src) good = ld_sc1(sflag + t) >= f2;
    if (__syncthreads_and(good)) break;
    if (spins >= RSPIN_LIMIT) {
      if (t == 0) {
        *err_sh = 1;
        atomicOr(err, 2u);
      }
      PF_GFLUSH();
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  PF_GMARK(10);
  // ---- this workgroup's output slots: gathered ancestors + jitter -------------
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(xn, 0, (int)(N * 4), 0x00020000);
  float xg8[RPPT];
#pragma unroll
  for (int q = 0; q < RPV; ++q) {
    const v4f v = __builtin_amdgcn_raw_buffer_load_b128(rx, (int)((i0 + 4 * q) * 4), 0, PF_AUX_SC1);
    xg8[4 * q] = v.x;
    xg8[4 * q + 1] = v.y;
    xg8[4 * q + 2] = v.z;
    xg8[4 * q + 3] = v.w;
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
  float xo[RPPT];
#pragma unroll
  for (int e = 0; e < RPPT; ++e) {
    Real xe[1] = {xg8[e]};
    if (regularize) {
      Real n[1] = {nj[e]};
      Mo::add_lower(xe, n, P, Mo::L::LJ);
    }
    xo[e] = (i0 + e < N) ? xe[0] : 0.0f;
  }
#pragma unroll
  for (int q = 0; q < RPV; ++q) sx_slot[q * RBS + t] = make_float4(xo[4 * q], xo[4 * q + 1], xo[4 * q + 2], xo[4 * q + 3]);
  PF_GMARK(11);
  PF_GFLUSH();
  return true;
}

template <typename Real, int NX, int NZ, int TK, int OK, bool TR = false>
__global__ void __launch_bounds__(RBS) k_resident(ResParams p) {
  static_assert(NX == 1 && sizeof(Real) == 4, "resident path: scalar fp32 state");
  using Mo = Model<Real, NX, NZ, TK, OK>;
  using RC = Rec<NX>;
  constexpr int LAG = RLAG;
  constexpr int NSNAP = LAG + 1;
  __shared__ __attribute__((aligned(16))) double red[LDS_RED];
  // per-wave partials, double-buffered by iteration parity: with ONE barrier per
  // iteration a wave is at most one iteration ahead of any other
  __shared__ double mslot[2][RNW][8];  // this workgroup's step record
  __shared__ __attribute__((aligned(16))) float mmax[2][RNW];  // the wave maxima again, for one vector read
  __shared__ double cslot[2][RCW][8];  // the verified step's summary (+ tags-complete flag)
  __shared__ int okw[RNW];
  __shared__ double auxw[RNW][2];  // wave sums of the freshly resampled state (x, x^2): the next record's aux
  __shared__ double sF[NSNAP];     // frame of each snapshot slot
  __shared__ int sT[NSNAP];  // filter step of each snapshot slot
  __shared__ double Pl[RMAXG + 1];
  __shared__ double Ck[RMAXG];
  __shared__ double offs[RBS];
  __shared__ float stage[RSTAGE];
  __shared__ unsigned err_sh;
  // snapshot ring, thread-private slots: state after each of the last LAG+1 steps
  __shared__ float4 snx[NSNAP][RPV * RBS];
  __shared__ float4 snl[NSNAP][RPV * RBS];

  // replicate r of the handle's R: a launch covers replicates [r0, r0 + gridDim.y) (a group
  // that fits co-resident; groups run one after another, each replicate is independent)
  const int b = blockIdx.x, r = p.r0 + (int)blockIdx.y, R = p.Rtot;
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
  const size_t cstride = gran_copy_stride(R);
  // this workgroup's replica of its replicate's record ring (reads), and replica 0
  const unsigned long long* gbase = p.gran + (size_t)(b % RCOPIES) * cstride + (size_t)r * RRING * RF * RMAXG;
  if (t == 0) err_sh = 0;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  __shared__ unsigned long long t_start_sh;  // for the slow polls' 1 ms check (not held in registers)
  if (t == 0) t_start_sh = t_start;
  __shared__ int arr_sh;
  if (p.test_abort && b == p.G - 1 && blockIdx.y == 0) {  // test hook: arrive after the others gave up
    if (t == 0)
      while (ld_sc1(p.arrive) != (((unsigned long long)p.seq << 2) | RDEC_ABORT) &&
             __builtin_amdgcn_s_memrealtime() - t_start < 5 * RARRIVE_TICKS)
        __builtin_amdgcn_s_sleep(8);
    __syncthreads();
  }
  unsigned long long arr_old = 0;  // this workgroup's shard count before its arrival
  if (t == 0)  // its return is checked after the entry loads
    arr_old = atomicAdd(p.arrive_sh + (size_t)((blockIdx.y * gridDim.x + blockIdx.x) % (unsigned)p.nshard) * RSHARD_WORDS, 1ull);
#ifdef PF_STAMPS
#ifndef PF_STAMP_T
#define PF_STAMP_T 0
#endif
#ifndef PF_STAMP_B
#define PF_STAMP_B 0
#endif
  // PF_STAMP_T: the stamped thread (wave); PF_STAMP_B: the stamped workgroup (-1: the output one)
  const bool stamp_me = (PF_STAMP_B < 0 ? b == p.G - 1 : b == PF_STAMP_B) && r == 0 && t == PF_STAMP_T;
  unsigned long long racc[24];
#pragma unroll
  for (int k = 0; k < 24; ++k) racc[k] = 0;
  unsigned long long rstamp_last = __builtin_amdgcn_s_memrealtime();
#endif

  // The body is instantiated twice: for the workgroup that writes the step outputs (it also
  // loads and reduces the moment / aux granules) and for all others.  A compile-time flag
  // keeps the granule loads unconditional inside one uniform branch, so their registers need
  // no merge copies (a copy right after the loads would wait for them at the loop top).
  // Kernel arguments that only cold paths use (rollback, outputs, slow polls, trace, exit) are
  // re-read from the kernarg segment where they are used, through a pointer the compiler cannot
  // hoist: carried around the loop they cost ~100 scalar registers, spilled and reloaded in the
  // step loop.
  auto KA = []() {
    typedef const __attribute__((address_space(4))) ResParams CRes;
    CRes* q = (CRes*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(q));
    return q;
  };
  auto body = [&, p](auto out_tag) {  // p by value: its fields stay in registers, not kernarg reloads
  constexpr bool outwg = decltype(out_tag)::value;  // b == G - 1
  // ---- entry state (k_step layout) and its normaliser ------------------------
  float x[RPPT], l[RPPT];
  double F0 = 0.0, T0 = 0.0;  // entry frame and absolute log mass (from the entry header)
  {
    // the particles' loads first: their latency overlaps the records' reduction below
    float lr[RPPT];
    if (i0 + RPPT <= N) {
#pragma unroll
      for (int q4 = 0; q4 < RPV; ++q4) {
        const float4 xv = *(const float4*)(p.x_in + rN + i0 + 4 * q4), lv = *(const float4*)(p.lw_in + rN + i0 + 4 * q4);
        x[4 * q4] = xv.x; x[4 * q4 + 1] = xv.y; x[4 * q4 + 2] = xv.z; x[4 * q4 + 3] = xv.w;
        lr[4 * q4] = lv.x; lr[4 * q4 + 1] = lv.y; lr[4 * q4 + 2] = lv.z; lr[4 * q4 + 3] = lv.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < RPPT; ++e) {
        const bool v = i0 + e < N;
        x[e] = v ? p.x_in[rN + i0 + e] : 0.0f;
        lr[e] = v ? p.lw_in[rN + i0 + e] : -INFINITY;
      }
    }
    // the previous resident run's exit header when it still describes the state (scalar loads:
    // uniform), else the records' prologue
    double lse0d = 0.0;
    bool uniform0 = false;
    bool have_hdr = false;
    if (p.hdr_in) {
      typedef const __attribute__((address_space(4))) unsigned long long cu64;
      const cu64* hp = (const cu64*)(p.hdr + (size_t)r * 4);
      if (hp[0] == p.hdr_in) {  // the exit frame continues: raw log-weights, its F and absolute mass
        T0 = __longlong_as_double((long long)hp[1]);
        F0 = __longlong_as_double((long long)hp[3]);
        uniform0 = hp[2] != 0ull;
        have_hdr = true;
      }
    }
    if (!have_hdr) {
      const Head h0 = prologue<NX, RBS>(p.rec_in + (int64_t)r * RC::SIZE * KA()->Gk, KA()->Gk, N, p.thresh, false, false,
                                        false, red, Pl);
      lse0d = uni(h0.lse);
      uniform0 = h0.uniform != 0;
    }
    const float lse0 = (float)lse0d;
#ifdef PF_STAMPS
    if (b == 0 && r == 0 && t == 0) g_pf_stamps[20] = __builtin_amdgcn_s_memrealtime();
#endif
#pragma unroll
    for (int e = 0; e < RPPT; ++e)
      l[e] = (i0 + e >= N) ? -INFINITY : (uniform0 ? lunif : (have_hdr ? lr[e] : lr[e] - lse0));
    if (uniform0) F0 = T0 = 0.0;
  }
  if (t == 0) arr_sh = res_arrive_sharded(KA(), arr_old);  // arrived after an abort: leave
  __syncthreads();
  if (!arr_sh) return;
#ifdef PF_STAMPS
  if (b == 0 && r == 0 && t == 0) {  // whole-launch phases: start, loop entry (+ loop exit, end below)
    g_pf_stamps[16] = t_start;
    g_pf_stamps[17] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  bool verified_any = false;  // a verified step proves the whole grid has arrived

  const int fo = p.first_update_only ? 1 : 0;
  const int T32 = (int)p.T;  // the host keeps T < 2^30
  int tstep = 0;           // next filter step to compute
  unsigned s_next = 0;     // next sequence number (executed steps, incl. discarded ones)
  unsigned vnext = 0;      // next sequence number to verify
  unsigned nres = 0;       // hand-offs so far (flag tags)
  unsigned it = 0;         // iteration parity (LDS double buffers)
  // frame of the live log-weights (the log-weights are l + F); absolute log mass of the last
  // verified step.  A run that follows a resident run continues that run's frame (entry header):
  // the raw exit log-weights with its F and mass, so a run cut into pieces is bitwise the
  // uninterrupted run
  double F = F0;
  double Tprev = T0;
  bool prev_res = false;   // last verified step resampled: next record carries its aux sums
  bool have_aux = false;   // the live state was just gathered
  bool rec_aux = false;    // the record being published carries the aux sums
  bool last_uniform = false;
  bool alive = true;
  bool aborted = false;
  double Tlast = T0;    // absolute log mass of the last verified (not resampled) step
  int last_cur = 0;     // mslot buffer of the last computed step (its frame: sF of its snapshot slot)
  float zwin = 0.0f;    // observation window (NZ == 1): lane k holds z of step zbase + k
  int zbase = -64;
  while (alive) {
    // granules of the step this iteration verifies (waves 0..RCW-1: one record per lane); per
    // iteration, so they are not carried around the loop (and through the rollback) in VGPRs.
    // Left undefined where not loaded: a zero default would merge with the loaded values.
    unsigned long long pg[RF];
    const bool computing = tstep < T32;
    const unsigned s_after = s_next + (computing ? 1u : 0u);
#if defined(PF_ABLATE) && PF_ABLATE == 1
    const bool verify = false;  // ablation: no verification at all (timing floor of the step)
    if (!computing) break;
#else
    const bool verify =
        vnext < s_after && (s_after - vnext > (unsigned)LAG || tstep + (computing ? 1 : 0) >= T32);
#endif
    if (!computing && !verify) break;
    // observations: a window of 64 steps in one VGPR (lane k: step zbase + k), read per step
    // with v_readlane; refilled when tstep leaves it (every 64 steps, or after a rollback
    // across its start) - no memory wait in the step
    if (NZ == 1 && computing && (tstep < zbase || tstep >= zbase + 64)) {
      zbase = tstep;
      const int tl = tstep + lane;
      zwin = tl < T32 ? KA()->z[(size_t)tl * R + r] : 0.0f;
      // wait for it here, in the rare branch: otherwise the wait lands before every step's
      // readlane and (vmcnt counts in order) takes the granule loads issued below with it
      asm volatile("; z window %0" ::"v"(zwin));
    }
    const int cur = (int)(it & 1u);
    ++it;
    const unsigned v = vnext;
    const unsigned vtag = p.tag0 + v + 1;
    const unsigned long long* vbase = gbase + (size_t)(v % RRING) * RF * RMAXG + t;
    const int idx = (int)(v % NSNAP);  // snapshot slot of step v
    double Fv = 0.0;
    int tv = 0;
    if (verify) {
      // granule loads for v (their latency overlaps the step below); slot info
      // read before this iteration's barrier (written iterations ago)
      // every lane of the wave loads (t < RMAXG: in bounds); lanes t >= G are masked later
      if (w < RCW) {
#pragma unroll
        for (int f = 0; f < RF; ++f)
          if (vg_need(f, outwg)) pg[f] = ld_sc1(vbase + f * RMAXG);
      }
      if (computing && v == s_next) {  // verifying the step computed right now (T=1 / drain)
        Fv = F;
        tv = tstep;
      } else {
        Fv = uni(sF[idx]);
        tv = __builtin_amdgcn_readfirstlane(sT[idx]);
      }
    }
    // the step's observation (and control) are uniform: scalar loads through the constant
    // address space (lgkmcnt), so waiting for them never waits for the granule loads (vmcnt).
    // Issued after the LDS reads above: an LDS wait with a scalar load in flight is a full wait.
    Real z[NZ], uc[NX];
    if (computing) {
      if constexpr (NZ == 1) {
        z[0] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(zwin), (int)(tstep - zbase)));
      } else {
        const CReal* zt = (const CReal*)(p.z + ((size_t)tstep * R + r) * NZ);
#pragma unroll
        for (int k = 0; k < NZ; ++k) z[k] = zt[k];
      }
#pragma unroll
      for (int k = 0; k < NX; ++k) uc[k] = Real(0);  // no control input: u = 0 (g(x) + 0 == g(x))
      if (p.u) {
        const CReal* ut = (const CReal*)(p.u + ((size_t)tstep * R + r) * NX);
#pragma unroll
        for (int k = 0; k < NX; ++k) uc[k] = ut[k];
      }
    }
    PF_RMARK(0);

    // ---------------- compute filter step tstep (speculative) ----------------
    if (computing) {
      const bool pred = !(fo && tstep == 0);
      const uint32_t ep_pred = p.ep0 + (uint32_t)(2 * tstep) - fo;
      const Real* u = uc;
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
      // this thread's max-first partial sums
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
#ifdef PF_YOUNG_PRIO
      if (w >= RCW) __builtin_amdgcn_s_setprio(2);
#endif
      // wave partials (DPP), one LDS slot per wave
      const float Mw = wave_max_u(m);
      const float fw = (m > -INFINITY) ? __expf(m - Mw) : 0.0f;
      const double w0 = wave_sum_ud((double)s0 * (double)fw);  // fp64 tile mass (see vg_need)
      const float w00 = wave_sum_u(s00 * fw * fw);
      const float w1 = wave_sum_u(s1 * fw), w2 = wave_sum_u(s2 * fw);
      double a1 = 0.0, a2 = 0.0;
      if (have_aux) {
        a1 = auxw[w][0];
        a2 = auxw[w][1];
      }
      PF_RMARK(22);  // the wave's own partials (DPP)
      if (lane == 0) {
        mmax[cur][w] = Mw;
        mslot[cur][w][0] = Mw;
        mslot[cur][w][1] = w0;
        mslot[cur][w][2] = w00;
        mslot[cur][w][3] = w1;
        mslot[cur][w][4] = w2;
        mslot[cur][w][5] = a1;
        mslot[cur][w][6] = a2;
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
      rec_aux = have_aux;
      have_aux = false;
      last_cur = cur;  // exit records: this step's wave partials
    }

    // ---------------- wave-level summary of the step being verified ----------
    const bool in = t < G;
    float m_g = -INFINITY;
    double s0_g = 0.0;
    if (verify && w < RCW) {
      int good = 1;
      if (in) {
#pragma unroll
        for (int f = 0; f < RF; ++f)
          if (vg_need(f, outwg)) good &= (unsigned)(pg[f] >> 32) == vtag;
      }
      m_g = in ? __uint_as_float((unsigned)pg[0]) : -INFINITY;
      s0_g = in ? granule_f64(pg[1], pg[7]) : 0.0;
      const float mg = (s0_g > 0.0) ? m_g : -INFINITY;
      const float Mw = wave_max_u(mg);
      const double f = (mg > -INFINITY) ? (double)__expf(mg - Mw) : 0.0;
      const double d0 = wave_sum_ud(s0_g * f);
      const double d1 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[2]) * f * f : 0.0);
      // moments only where the outputs are written; aux sums only after a resample
      double d2 = 0.0, d3 = 0.0, d4 = 0.0, d5 = 0.0;
      if (outwg) {
        d2 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[3]) * f : 0.0);
        d3 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[4]) * f : 0.0);
        if (prev_res) {
          d4 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[5]) : 0.0);
          d5 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[6]) : 0.0);
        }
      }
      const int wgood = __all(good);
      if (lane == 0) {
        cslot[cur][w][0] = Mw;
        cslot[cur][w][1] = d0;
        cslot[cur][w][2] = d1;
        cslot[cur][w][3] = d2;
        cslot[cur][w][4] = d3;
        cslot[cur][w][5] = d4;
        cslot[cur][w][6] = d5;
        cslot[cur][w][7] = wgood ? 1.0 : 0.0;
      }
    }
    PF_RMARK(23);  // the verification summary (waits for the granule loads)
    __syncthreads();  // the iteration's one barrier
#ifdef PF_YOUNG_PRIO
    if (w >= RCW && w != PF_PUBW) __builtin_amdgcn_s_setprio(0);
#endif
    PF_RMARK(2);

    // ---------------- publish this workgroup's record ------------------------
    if (computing) {
      // combine the wave partials and publish.  The last wave does it (waves 0..RCW-1 carry the
      // verification summaries).  Transposed: lane = granule field + RF * replica, every lane
      // sums its field over the RNW wave partials itself (a short, independent chain per lane)
      // instead of a chain of row reductions that the wave would run one after the other.
#if PF_PUB_PRIO
      // the publishing wave is the younger of its SIMD's two: without priority it issues only when
      // the older wave stalls, and the record is on every workgroup's critical path (-4%/step)
      if (w == PF_PUBW) __builtin_amdgcn_s_setprio(3);
#endif
      if (w == PF_PUBW && lane < RF * RCOPIES) {
        const int f = lane % RF, c = lane / RF;
        const int src = (f == 7) ? 1 : f;  // the S0 low word is the same fp64 sum as the high word
        // all LDS reads first, then branch-free arithmetic (per-lane selects, no divergence)
        static_assert(RNW % 4 == 0, "16-byte reads of the wave maxima");
        float mjv[RNW];
#pragma unroll
        for (int j = 0; j < RNW; j += 4) {
          const float4 m4 = *(const float4*)&mmax[cur][j];
          mjv[j] = m4.x;
          mjv[j + 1] = m4.y;
          mjv[j + 2] = m4.z;
          mjv[j + 3] = m4.w;
        }
        double vv[RNW];
#pragma unroll
        for (int j = 0; j < RNW; ++j) vv[j] = mslot[cur][j][src];
        float Mt = mjv[0];
#pragma unroll
        for (int j = 1; j < RNW; ++j) Mt = fmaxf(Mt, mjv[j]);
        const bool sq = src == 2, plain = src >= 5;
        double sum = 0.0;
#pragma unroll
        for (int j = 0; j < RNW; ++j) {
          const float fj = (mjv[j] > -INFINITY) ? __expf(mjv[j] - Mt) : 0.0f;
          const float wf = sq ? fj * fj : fj;
          sum = fma(vv[j], plain ? 1.0 : (double)wf, sum);
        }
        sum = (src == 0 || (plain && !rec_aux)) ? 0.0 : sum;
        const unsigned long long sb = (unsigned long long)__double_as_longlong(sum);
        const unsigned pay = f == 0 ? __float_as_uint(Mt) : f == 1 ? (unsigned)(sb >> 32)
                           : f == 7 ? (unsigned)sb : __float_as_uint((float)sum);
        unsigned long long* g = p.gran + (size_t)c * cstride + ((size_t)r * RRING + s_next % RRING) * RF * RMAXG + b;
        st_sc1(g + f * RMAXG, ((unsigned long long)(p.tag0 + s_next + 1) << 32) | pay);
      }
#if PF_PUB_PRIO && !defined(PF_PRIO_STICKY)
      if (w == PF_PUBW) __builtin_amdgcn_s_setprio(0);
#endif
      PF_RCOUNT(14);
      ++s_next;
      ++tstep;
    }
    PF_RMARK(3);
    if (!verify) continue;

    // ---------------- verify step v -------------------------------------------
    // the RCW (= 4) wave summaries in cslot combine across each quad of lanes (lane & 3 reads
    // summary lane & 3; quad_perm DPP): independent short chains, the same order everywhere
    static_assert(RCW == 4, "quad combine of the verification summaries");
    auto quad_sum = [](double v) {
      v += dpp_d<DPP_QP_1032>(0.0, v);
      return v + dpp_d<DPP_QP_2301>(0.0, v);
    };
    auto quad_all = [&](int cur_) {
      int g = cslot[cur_][lane & 3][7] != 0.0;
      g &= dpp_i<DPP_QP_1032>(0, g);
      g &= dpp_i<DPP_QP_2301>(0, g);
      return __builtin_amdgcn_readfirstlane(g);
    };
    int all = quad_all(cur);
    PF_RMARK(4);
    for (unsigned spins = 0; !all; ++spins) {  // slow path: not every record was in yet
      PF_RCOUNT(15);
      __syncthreads();  // every wave has read cslot[cur]
      if (!verified_any && (spins & 63u) == 63u && __builtin_amdgcn_s_memrealtime() - t_start_sh > RARRIVE_TICKS) {
        // still no step verified after 1 ms: is the grid resident at all?
        if (t == 0) arr_sh = res_try_abort_sharded(KA()) ? 2 : 1;
        __syncthreads();
        if (arr_sh == 2) {
          aborted = true;
          alive = false;
          break;
        }
        verified_any = true;  // every workgroup has arrived: wait on as usual
      }
      if (spins >= RSPIN_LIMIT) {
        if (t == 0) {
          err_sh = 1;
          atomicOr(KA()->err, 1u);
        }
        alive = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      if (w < RCW) {
        int good = 1;
        unsigned long long pg[RF];  // the slow path's own reload
#pragma unroll
        for (int f = 0; f < RF; ++f) {
          if (!vg_need(f, outwg)) continue;
          pg[f] = ld_sc1(vbase + f * RMAXG);
          if (in) good &= (unsigned)(pg[f] >> 32) == vtag;
        }
        m_g = in ? __uint_as_float((unsigned)pg[0]) : -INFINITY;
        s0_g = in ? granule_f64(pg[1], pg[7]) : 0.0;
        const float mg = (s0_g > 0.0) ? m_g : -INFINITY;
        const float Mw = wave_max_u(mg);
        const double f = (mg > -INFINITY) ? (double)__expf(mg - Mw) : 0.0;
        const double d0 = wave_sum_ud(s0_g * f);
        const double d1 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[2]) * f * f : 0.0);
        // moments only where the outputs are written; aux sums only after a resample
        double d2 = 0.0, d3 = 0.0, d4 = 0.0, d5 = 0.0;
        if (outwg) {
          d2 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[3]) * f : 0.0);
          d3 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[4]) * f : 0.0);
          if (prev_res) {
            d4 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[5]) : 0.0);
            d5 = wave_sum_ud(in ? (double)__uint_as_float((unsigned)pg[6]) : 0.0);
          }
        }
        const int wgood = __all(good);
        if (lane == 0) {
          cslot[cur][w][0] = Mw;
          cslot[cur][w][1] = d0;
          cslot[cur][w][2] = d1;
          cslot[cur][w][3] = d2;
          cslot[cur][w][4] = d3;
          cslot[cur][w][5] = d4;
          cslot[cur][w][6] = d5;
          cslot[cur][w][7] = wgood ? 1.0 : 0.0;
        }
      }
      __syncthreads();
      all = quad_all(cur);
    }
    if (alive && !verified_any && gridDim.y > 1) {
      // A verified step proves only that THIS replicate's workgroups arrived.  Several replicates
      // in one plain launch: before anything is written in place, wait until the whole grid has
      // counted in - or the launch aborts (another replicate's workgroup found it incomplete):
      // then every replicate leaves with its state untouched.
      if (t == 0) {
        int res = 0;
        while (res == 0) {
          const unsigned long long d = ld_sc1(KA()->arrive);
          if ((d >> 2) == KA()->seq && (d & 3) == RDEC_ABORT) res = 2;
          else if (res_all_arrived(KA())) res = 1;  // every shard complete, unmarked
          else if (__builtin_amdgcn_s_memrealtime() - t_start_sh > RARRIVE_TICKS)
            res = res_try_abort_sharded(KA()) ? 2 : 1;
          else
            __builtin_amdgcn_s_sleep(2);
        }
        arr_sh = res;
      }
      __syncthreads();
      if (arr_sh == 2) {
        aborted = true;
        alive = false;
      }
    }
    if (!alive) break;
    verified_any = true;
    PF_RMARK(12);  // slow polls
    double Mx, W, W2, S1, S2, A1, A2;
    {
      const double* cs = cslot[cur][lane & 3];
      const double mj = cs[0];
      double mq = fmax(mj, dpp_d<DPP_QP_1032>(-INFINITY, mj));
      mq = fmax(mq, dpp_d<DPP_QP_2301>(-INFINITY, mq));
      const double Fj = (mj > -INFINITY) ? (double)__expf((float)(mj - mq)) : 0.0;
      const double w1 = quad_sum(cs[1] * Fj), w2 = quad_sum(cs[2] * Fj * Fj);
      const double s1 = outwg ? quad_sum(cs[3] * Fj) : 0.0, s2 = outwg ? quad_sum(cs[4] * Fj) : 0.0;
      const double a1 = (outwg && prev_res) ? quad_sum(cs[5]) : 0.0, a2 = (outwg && prev_res) ? quad_sum(cs[6]) : 0.0;
      Mx = uni(mq);
      W = uni(w1);
      W2 = uni(w2);
      S1 = uni(s1);
      S2 = uni(s2);
      A1 = uni(a1);
      A2 = uni(a2);
    }
    PF_RMARK(4);
    if (!(W > 0.0)) {
      // every particle's weight is zero or NaN (e.g. an all -inf log-likelihood,
      // SURVEY 8c(vi)): the filter is dead.  Every workgroup reduces the same records
      // to the same W, so all of them stop here; the host reports PF_E_NAN.
      if (outwg && t == 0) {
        const int64_t o = (int64_t)tv * R + r;
        KA()->o_neff[o] = __builtin_nan("");
        KA()->o_lse[o] = __builtin_nan("");
        KA()->o_mean[o] = __builtin_nan("");
        if (KA()->o_cov) KA()->o_cov[o] = __builtin_nan("");
        KA()->o_flag[o] = 0;
        atomicOr(KA()->err, 8u);
      }
      alive = false;
      break;
    }
    const double lse_rel = Mx + log_pos(W);
#if defined(PF_ABLATE) && PF_ABLATE == 2
    const bool dec = false;  // ablation: never resample (cost of verification without rollbacks)
#else
    const bool dec = W * W < p.thresh * (double)N * W2;  // Neff = W^2 / W2 < thresh * N
#endif
    const double Tv = lse_rel + Fv;
    if constexpr (TR) {  // trace build: the verified step's predicted state, from its snapshot
      if (tv < KA()->tr_T) {
        const size_t to = ((size_t)tv * R + r) * (size_t)KA()->Npad;
#pragma unroll
        for (int q = 0; q < RPV; ++q) {
          const float4 xs = snx[idx][q * RBS + t], ls = snl[idx][q * RBS + t];
          const float xa[4] = {xs.x, xs.y, xs.z, xs.w}, la[4] = {ls.x, ls.y, ls.z, ls.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (i0 + 4 * q + e < KA()->Npad) {
              KA()->tr_x[to + i0 + 4 * q + e] = xa[e];
              KA()->tr_l[to + i0 + 4 * q + e] = la[e];
            }
        }
      }
    }
    if (outwg && t == 0) {  // outputs: the last workgroup (the partial tile, least work)
      const int64_t o = (int64_t)tv * R + r;
      KA()->o_neff[o] = (W * W) / W2;
      KA()->o_lse[o] = Tv - Tprev;
      KA()->o_flag[o] = dec ? 1 : 0;
      const double mean = S1 / W;
      KA()->o_mean[o] = mean;
      if (KA()->o_cov) KA()->o_cov[o] = S2 / W - mean * mean;
      if (prev_res) {  // post-resample moments of step tv - 1 (uniform weights)
        const int64_t o2 = (int64_t)(tv - 1) * R + r;
        const double mp = A1 / (double)N;
        KA()->o_mean[o2] = mp;
        if (KA()->o_cov) KA()->o_cov[o2] = A2 / (double)N - mp * mp;
      }
    }
    prev_res = false;
    if (!dec) {
      Tprev = Tv;
      Tlast = Tv;
      const float delta = (float)(Tv - F);
#pragma unroll
      for (int e = 0; e < RPPT; ++e) l[e] = l[e] - delta;  // -inf stays -inf
      F += (double)delta;
      vnext = v + 1;
      last_uniform = false;
      continue;
    }
    // ---- rollback to step tv and resample it (out of line: rare) --------------
    PF_RCOUNT(13);
    ++nres;
    const uint32_t ep_res = p.ep0 + (uint32_t)(2 * tv + 1) - fo;
    if (!rb_gather<Real, NX, NZ, TK, OK>(KA()->xg + rN, KA()->sflag + (size_t)r * RMAXG, KA()->flag0,
                                          KA()->err, &err_sh, snx[idx], snl[idx], red, Pl, Ck, offs, stage, G, b, N, nres, m_g,
                                          s0_g, Mx, p.seed, rep, ep_res, KA()->regularize, (const Real*)KA()->P,
                                          (TR && tv < KA()->tr_T) ? KA()->tr_anc + ((size_t)tv * R + r) * (size_t)KA()->Npad
                                                              : (int32_t*)nullptr)) {
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
    {
      double aux1 = 0.0, aux2 = 0.0;
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
      // their wave sums now, kept in LDS until the next record (not in registers around the loop)
      aux1 = wave_sum_ud(aux1);
      aux2 = wave_sum_ud(aux2);
      if (lane == 0) {
        auxw[w][0] = aux1;
        auxw[w][1] = aux2;
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

  if (aborted) return;  // nothing was written: the entry state stays as it was
#ifdef PF_STAMPS
  if (b == 0 && r == 0 && t == 0) g_pf_stamps[18] = __builtin_amdgcn_s_memrealtime();
#endif
  // ---- the last step resampled: its post-resample moments -------------------
  if (alive && prev_res) {
    __syncthreads();
    if (t == 0) {
      double A1 = 0.0, A2 = 0.0;
      for (int j = 0; j < RNW; ++j) {
        A1 += auxw[j][0];
        A2 += auxw[j][1];
      }
      const unsigned tag = p.tag0 + s_next + 1;
      unsigned long long* g = KA()->gran + ((size_t)r * RRING + s_next % RRING) * RF * RMAXG + b;
      st_sc1(g + 5 * RMAXG, granule(tag, (float)A1));
      st_sc1(g + 6 * RMAXG, granule(tag, (float)A2));
    }
    // every workgroup's aux granules (fixed-order sum in each workgroup)
    const unsigned tag = p.tag0 + s_next + 1;
    const unsigned long long* base = KA()->gran + ((size_t)r * RRING + s_next % RRING) * RF * RMAXG + t;  // replica 0
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
      int allg = 1;
#pragma unroll
      for (int j = 0; j < RCW; ++j) allg &= okw[j];
      allg = __builtin_amdgcn_readfirstlane(allg);
      if (allg) {
        if (w < RCW) {
          const double d4 = wave_sum_ud(t < G ? (double)__uint_as_float((unsigned)g5) : 0.0);
          const double d5 = wave_sum_ud(t < G ? (double)__uint_as_float((unsigned)g6) : 0.0);
          if (lane == 0) {
            cslot[0][w][5] = d4;
            cslot[0][w][6] = d5;
          }
        }
        __syncthreads();
        if (outwg && t == 0) {
          double S5 = 0.0, S6 = 0.0;
          for (int j = 0; j < RCW; ++j) {
            S5 += cslot[0][j][5];
            S6 += cslot[0][j][6];
          }
          const int64_t o2 = (KA()->T - 1) * R + r;
          const double mp = S5 / (double)N;
          KA()->o_mean[o2] = mp;
          if (KA()->o_cov) KA()->o_cov[o2] = S6 / (double)N - mp * mp;
        }
        break;
      }
      __syncthreads();
      if (spins >= RSPIN_LIMIT) {
        if (t == 0) atomicOr(KA()->err, 4u);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }

  // ---- exit state in the k_step layout ---------------------------------------
  if (i0 + RPPT <= N) {
#pragma unroll
    for (int q4 = 0; q4 < RPV; ++q4) {
      *(float4*)(KA()->x_fin + rN + i0 + 4 * q4) = make_float4(x[4 * q4], x[4 * q4 + 1], x[4 * q4 + 2], x[4 * q4 + 3]);
      *(float4*)(KA()->lw_fin + rN + i0 + 4 * q4) = make_float4(l[4 * q4], l[4 * q4 + 1], l[4 * q4 + 2], l[4 * q4 + 3]);
    }
  } else {
#pragma unroll
    for (int e = 0; e < RPPT; ++e)
      if (i0 + e < N) {
        KA()->x_fin[rN + i0 + e] = x[e];
        KA()->lw_fin[rN + i0 + e] = l[e];
      }
  }
#ifdef PF_STAMPS
  if (b == 0 && r == 0 && t == 0) g_pf_stamps[21] = __builtin_amdgcn_s_memrealtime();
#endif
  // One k_step record per 1024-particle tile (KW waves).  They are the wave partials of the
  // last computed step (mslot, written before that iteration's barrier), moved to the exit
  // frame: the live log-weights have only been shifted uniformly since (by F - F_last).
  {
    constexpr int KQ = 1024 / RPPT, KW = KQ / 64;
    static_assert(KW >= 1 && KQ % 64 == 0, "k_step tiles of whole waves");
    const int q = t / KQ;
    const int kt = b * (RTILE / 1024) + q;
    if ((t % KQ) == 0 && kt < KA()->Gk) {
      double* o = KA()->rec_fin + (int64_t)r * RC::SIZE * KA()->Gk;
      for (int f2 = 0; f2 < RC::SIZE; ++f2) o[(int64_t)f2 * KA()->Gk + kt] = 0.0;
      if (last_uniform) {
        o[(int64_t)RC::UNI * KA()->Gk + kt] = 1.0;
      } else {
        const double(*ms)[8] = mslot[last_cur];
        double Mq = -INFINITY;
        for (int j = 0; j < KW; ++j) Mq = fmax(Mq, ms[KW * q + j][0]);
        double s0 = 0.0, s00 = 0.0, s1 = 0.0, s2 = 0.0;
        for (int j = 0; j < KW; ++j) {
          const double mj = ms[KW * q + j][0];
          const double fj = (mj > -INFINITY) ? (double)__expf((float)(mj - Mq)) : 0.0;
          s0 += ms[KW * q + j][1] * fj;
          s00 += ms[KW * q + j][2] * fj * fj;
          s1 += ms[KW * q + j][3] * fj;
          s2 += ms[KW * q + j][4] * fj;
        }
        const double F_last = sF[(s_next - 1) % NSNAP];  // the last computed step's frame
        o[(int64_t)RC::M * KA()->Gk + kt] = Mq - (F - F_last);
        o[(int64_t)RC::S0 * KA()->Gk + kt] = s0;
        o[(int64_t)RC::S00 * KA()->Gk + kt] = s00;
        o[(int64_t)RC::S1 * KA()->Gk + kt] = s1;
        if constexpr (RC::COV) o[(int64_t)RC::S2 * KA()->Gk + kt] = s2;
      }
    }
  }
  // entry header of the next launch: the exit frame F and the last verified step's absolute log
  // mass Tlast (the exit log-weights sum to e^(Tlast - F): the fp32 residual of the final shift),
  // or uniform
  if (b == 0 && t == 0 && alive) {
    unsigned long long* hp = KA()->hdr + (size_t)r * 4;
    hp[1] = (unsigned long long)__double_as_longlong(last_uniform ? 0.0 : Tlast);
    hp[2] = last_uniform ? 1ull : 0ull;
    hp[3] = (unsigned long long)__double_as_longlong(last_uniform ? 0.0 : F);
    hp[0] = KA()->hdr_out;
  }
#ifdef PF_STAMPS
  if (stamp_me)
    for (int k = 0; k < 24; ++k)
      if (k < 6 || (k > 11 && k < 16) || k > 21) g_pf_stamps[k] = racc[k];
  if (b == 0 && r == 0 && t == 0) g_pf_stamps[19] = __builtin_amdgcn_s_memrealtime();
#endif
  };
  if (b == G - 1)
    body(std::true_type{});
  else
    body(std::false_type{});
}

}  // namespace pf
