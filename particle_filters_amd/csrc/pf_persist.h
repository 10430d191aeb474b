// k_persist: the fp64 scalar-state SIR filter (BASELINE config 2 at the reference's own precision,
// pf.py:223-269 + 146-171) for a whole pf_run_device call in ONE launch, the launch-per-step
// k_step<double> arithmetic bit for bit.
//
// Why: k_step<double> is ~23 us per step at N = 1e6, of which ~5 us is the launch boundary and the
// grid fill / drain, and its prologue's record loads wait for the previous launch to finish.  Here the
// k_step geometry (2048-particle tiles, 256 threads, two 4-particle chunks per thread) stays resident
// for all T steps plus the tail (the last update's resample and the final statistics):
//   * the state the thread owns (its 8 slots' x and log-weight) stays in registers from step to step,
//     and is also stored to the ping-pong buffers (16-byte sc1 stores: write-through, so a gathering
//     workgroup on another XCD reads it from memory) - the HBM state k_step would leave, step by step;
//   * the tile record (k_step's 9 fp64 fields) is published as 18 data-tagged granules {tag, 32-bit
//     half} (one sc1 store per granule, one instruction for all of them: the data is its own flag,
//     MI355X_MICROARCH.md R2) into a ring of PRING steps; the next step's prologue polls the granules
//     of all G tiles instead of a kernel boundary - no counter, no fence on the step's critical path;
//   * right after publishing, every workgroup computes the next step's predict + likelihood of its
//     8 slots (Philox normals, transition, log-likelihood: the step's fp64 bulk) while the other
//     tiles' records arrive; the prologue then decides, and on the no-resample path (~95 % of steps)
//     only the weight shift, the record merge and the stores remain;
//   * a resample (the decision of the previous step) waits for every tile's data flag (set after the
//     tile's x / lw stores drained), acquires (L1 invalidate) and runs k_step's source-driven
//     systematic ancestors and gather over the previous step's buffers.
// Records, ancestors, decisions and outputs are computed by the same functions in the same order as
// k_step / k_finalize (prologue_reduce, sys_ancestors, WAcc::add / block_merge, write_outputs_f), so
// the run is bitwise the launch-per-step run (tests/test_gpu_persist.py, PF_PERSIST=0 for the other).
//
// Co-residency: every workgroup counts itself in before it writes anything (res_arrive); a workgroup
// that waits more than 1 ms for step 0's records tries to abort (res_try_abort, pf_resident.h) and the
// host reports PF_E_RETRY with the state untouched (step 0 writes only the other ping-pong buffers).
#pragma once
#include "pf_kernels.h"
#include "pf_resident.h"

namespace pf {

constexpr int PRING = 4;                     // granule ring slots (steps)
constexpr int PGF = 2 * Rec<1>::SIZE;        // granules per record: hi / lo word of each fp64 field
constexpr int PBS = 256;                     // k_step's workgroup size for the scalar state
constexpr int PMAXG = 2 * PBS;               // tiles per replicate (workgroup 0 holds two records per thread)
constexpr unsigned long long PSPIN_TICKS = 20000000ull;  // 200 ms of s_memrealtime: a hand-off timed out

// persistent-run sync words of one handle: granules [R][PRING][PGF][G], data flags [R][G]
__host__ __device__ inline size_t persist_gran_words(int R, int G) { return (size_t)R * PRING * PGF * G; }
__host__ __device__ inline size_t persist_sync_words(int R, int G) {
  return persist_gran_words(R, G) + (size_t)R * G;
}
// LDS (doubles): scratch | Pl[G + 1] | area | the polled record heads M_k[G], S0_k[G], S00_k[G].
// The area holds the threads' slot state between steps ([3][8][PBS]: x (predicted once speculated),
// log-weight, log-likelihood) and, on a resample step, the tile's fp64 CDF + int ancestors instead
// (the state is dead then: the gather recomputes it).
constexpr int PST = 3 * 8 * PBS;  // slot-state doubles
__host__ __device__ inline int persist_mk_off(int G, int tile) {
  const int area = (tile * 12 + 15) / 16 * 2;  // tile doubles + tile ints, 16-byte aligned
  return lds_tile(G) + (area > PST ? area : PST);
}
__host__ __device__ inline size_t persist_lds_bytes(int G, int tile) {
  return (size_t)(persist_mk_off(G, tile) + 3 * ((G + 8) & ~7)) * sizeof(double);
}

struct PersistParams {
  StepParams p;      // launch-invariant fields (P, N, Npad, G, tile, seed, thresh, regularize, r_diag,
                     // rep_base, pbase, outputs o_*); the per-step fields are set in the kernel
  void* X[2];        // [R][Npad] state ping-pong (k_step's x_in / x_out)
  void* L[2];        // [R][Npad] log-weights
  double* RB[2];     // [R][RS][G] records
  int cx, cl, cr;    // entry buffers
  const void* z;     // [T][R][NZ]
  const void* u;     // [T][R][NX] or null
  int64_t T;
  int fo;            // step 0 is update-only (no predict)
  int pending;       // step 0 applies the decision of the last update before the run
  uint32_t ep0;      // Philox epoch of step 0's predict
  uint32_t ep_res0;  // epoch of a pending resample
  unsigned long long* gran;
  unsigned long long* dflag;
  uint32_t tag0;     // granule tag of step s: tag0 + s + 1 (the host advances tag0 past every launch)
  unsigned long long* arrive;
  unsigned long long arrive0, seq;
  unsigned int* err;
};

__device__ __forceinline__ unsigned long long pgran(unsigned tag, unsigned half) {
  return ((unsigned long long)tag << 32) | (unsigned long long)half;
}
__device__ __forceinline__ bool pgran_pair(const unsigned long long* hi_p, const unsigned long long* lo_p, unsigned tag,
                                           double& v) {
  const unsigned long long hi = ld_sc1(hi_p), lo = ld_sc1(lo_p);
  v = __longlong_as_double((long long)(((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull)));
  return (unsigned)(hi >> 32) == tag && (unsigned)(lo >> 32) == tag;
}

// field f of tile k from a ring slot's granules, waiting for the tag (bounded: a timeout sets err 2)
__device__ __forceinline__ double pgran_wait(const unsigned long long* gs, int f, int k, int G, unsigned tag,
                                             unsigned int* err) {
  double v;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (!pgran_pair(gs + (2 * f) * G + k, gs + (2 * f + 1) * G + k, tag, v)) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > PSPIN_TICKS) {
      atomicOr(err, 2u);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return v;
}

typedef unsigned int pv4u __attribute__((ext_vector_type(4)));
// 4 consecutive doubles (16-byte aligned) as two 16-byte sc1 stores
__device__ __forceinline__ void st4_sc1(__amdgpu_buffer_rsrc_t rs, int64_t i, const double* v) {
  const pv4u a = __builtin_bit_cast(pv4u, make_double2(v[0], v[1]));
  const pv4u b = __builtin_bit_cast(pv4u, make_double2(v[2], v[3]));
  __builtin_amdgcn_raw_buffer_store_b128(a, rs, (int)(i * 8), 0, PF_AUX_SC1);
  __builtin_amdgcn_raw_buffer_store_b128(b, rs, (int)(i * 8 + 16), 0, PF_AUX_SC1);
}
__device__ __forceinline__ void st1_sc1(double* p, double v) {
  st_sc1((unsigned long long*)p, (unsigned long long)__double_as_longlong(v));
}

// Every thread calls it with a uniform `res`: 0 go on, 2 leave (aborted or timed out).
template <int BS>
__device__ __forceinline__ int persist_slow_poll(const PersistParams& q, bool first_wait, unsigned long long t0,
                                                 int* res_sh) {
  if (threadIdx.x == 0) {
    const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
    int res = 0;
    if (first_wait && dt > RARRIVE_TICKS) {
      // the grid may not be co-resident: abort while not every workgroup has arrived
      res = res_try_abort(q.arrive, q.err, q.arrive0, (unsigned long long)gridDim.x * gridDim.y, q.seq) ? 2 : 0;
    }
    if (res == 0 && dt > PSPIN_TICKS) {
      atomicOr(q.err, 2u);
      res = 2;
    }
    *res_sh = res;
  }
  __syncthreads();
  const int res = *res_sh;
  __syncthreads();
  return res;
}

// Diagnostic phase accounting (PF_STAMPS builds only): thread 0 of workgroup PF_PSTAMP_B accumulates
// s_memrealtime ticks (100 MHz) per phase of the step loop into g_pf_stamps[0..7] (7: steps).
#ifndef PF_PSTAMP_B
#define PF_PSTAMP_B 100
#endif
#ifdef PF_STAMPS
#define PX_MARK(k)                                                      \
  do {                                                                  \
    if (px_me) {                                                        \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime(); \
      px_acc[(k)] += now_ - px_last;                                    \
      px_last = now_;                                                   \
    }                                                                   \
  } while (0)
#else
#define PX_MARK(k) \
  do {             \
  } while (0)
#endif

template <typename Real, int NX, int NZ, int TK, int OK>
__global__ void __launch_bounds__(PBS) __attribute__((amdgpu_waves_per_eu(2))) k_persist(PersistParams q) {
  static_assert(NX == 1 && sizeof(Real) == 8, "persistent path: scalar fp64 state");
  using M = Model<Real, NX, NZ, TK, OK>;
  using RC = Rec<NX>;
  using WA = WAcc<Real, NX>;
  constexpr int BS = PBS, CH = 4, RPT = MAXG / BS;
  constexpr int NA = 1 + NX + RC::NC;  // aux: cnt, sum x, sum x^2
  static_assert(PGF <= 64, "one wave publishes a record");
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ double fin[RC::SIZE];   // the staged record
  __shared__ double finp[RC::SIZE];  // this tile's last record (the tail carries it over)
  __shared__ int res_sh;
  const StepParams& p = q.p;
  const int G = p.G;
  double* red = smem;
  double* Pl = smem + LDS_PL;
  double* cdf = smem + lds_tile(G);
  int* anc_l = (int*)(cdf + p.tile);
  double* st = cdf;  // slot state [3][8][BS] (aliases the gather's CDF / ancestors)
  const int G8 = (G + 8) & ~7;
  double* Mk = smem + persist_mk_off(G, p.tile);  // [3][G8]: M_k, S0_k, S00_k of the polled records
  const int b = blockIdx.x, r = blockIdx.y, R = gridDim.y, t = threadIdx.x;
  const Real* __restrict__ P = (const Real*)p.P;
  const int64_t o0 = (int64_t)b * p.tile, o1 = min(o0 + (int64_t)p.tile, p.N);
  const int nchunks = (int)((o1 - o0 + CH - 1) / CH);  // <= 2 BS (host: tile <= 2 BS CH)
  const int rep_i = r + p.rep_base;
  const uint32_t rep = (uint32_t)rep_i;
  const int64_t roff = (int64_t)r * p.Npad;
  unsigned long long* gr = q.gran + (size_t)r * PRING * PGF * G;
  unsigned long long* dfl = q.dflag + (size_t)r * G;
  const double lprev_uniform = -log((double)p.N);
  const int kfo = q.fo ? 1 : 0;
  // The thread index as the step loop sees it: laundered at the top of every step (an opaque copy),
  // so that the slot addresses and masks derived from it are recomputed per step (a few integer
  // instructions) instead of being hoisted out of the loop and held in registers for all T steps.
  int tix = t;
  auto SX = [&](int c, int e) -> double& { return st[(0 * 8 + 4 * c + e) * BS + tix]; };
  auto SL = [&](int c, int e) -> double& { return st[(1 * 8 + 4 * c + e) * BS + tix]; };
  auto SLL = [&](int c, int e) -> double& { return st[(2 * 8 + 4 * c + e) * BS + tix]; };
  // chunk c of the thread: slots [i0(c), i0(c) + nv(c)) of the tile
  auto i0_of = [&](int c) { return o0 + (int64_t)(tix + c * BS) * CH; };
  auto nv_of = [&](int c) { return tix + c * BS < nchunks ? (int)min((int64_t)CH, o1 - i0_of(c)) : 0; };

#ifdef PF_STAMPS
  const bool px_me = t == 0 && blockIdx.y == 0 && b == (PF_PSTAMP_B < G ? PF_PSTAMP_B : 0);
  unsigned long long px_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, px_last = __builtin_amdgcn_s_memrealtime();
#endif
  // ---- entry: count in (nothing is written before) ---------------------------------------
  if (t == 0) res_sh = (res_arrive(q.arrive) - q.arrive0) >= RABORT ? 2 : 0;  // arrived after an abort
  __syncthreads();
  if (res_sh == 2) return;
  __syncthreads();

  // the state of the thread's slots into LDS (k_step reloads it every step; slots past the tile: 0, -inf)
  int cx = q.cx, cl = q.cl, cr = q.cr;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int nv = nv_of(c);
    Real xv[4] = {0, 0, 0, 0}, lv[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    if (nv > 0) {
      load4<Real>((const Real*)q.X[cx] + roff + i0_of(c), xv);
      load4<Real>((const Real*)q.L[cl] + roff + i0_of(c), lv);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      SX(c, e) = xv[e];
      SL(c, e) = lv[e];
    }
  }
  Head h;  // the decision of the step before (kept for the outputs written after the publish)

  for (int64_t s = 0; s <= q.T; ++s) {
    tix = t;
    asm volatile("" : "+v"(tix));
    const bool tail = s == q.T;  // the last update's resample + statistics (k_step's tail launch)
    const int pred = tail ? 0 : !(q.fo && s == 0);
    const int upd = tail ? 0 : 1;
    const int allow = tail ? 1 : (s > 0 || q.pending);
    const uint32_t ep_p = pred ? q.ep0 + (uint32_t)(2 * s) - kfo : 0;
    const uint32_t ep_r = s == 0 ? q.ep_res0 : q.ep0 + (uint32_t)(2 * s) - 1 - kfo;
    const unsigned tag_prev = q.tag0 + (unsigned)s, tag = tag_prev + 1;  // steps s - 1, s
    const Real* x_in = (const Real*)q.X[cx] + roff;
    Real* x_out = (Real*)q.X[cx ^ 1] + roff;
    const Real* lw_in = (const Real*)q.L[cl] + roff;
    Real* lw_out = (Real*)q.L[cl ^ 1] + roff;
    double* rec_out = q.RB[cr ^ 1] + (int64_t)r * RC::SIZE * G;
    const Real* u = (q.u && pred) ? (const Real*)q.u + ((int64_t)s * R + r) * NX : nullptr;
    Real z[NZ];
    if (upd) {
#pragma unroll
      for (int k = 0; k < NZ; ++k) z[k] = ((const Real*)q.z)[((int64_t)s * R + r) * NZ + k];
    }

    // ---- (S) predict + likelihood of the thread's slots, before the decision ----------------
    // (k_step: the first chunk speculated under the prologue's loads, the second in its chunk loop;
    // the same calls on the same values).  One chunk at a time, through LDS.
#pragma unroll 1
    for (int c = 0; c < 2; ++c) {
      if (nv_of(c) == 0) continue;
      Real n4[4];
      if (pred) chunk_normals4<Real>(p.seed, i0_of(c), (uint32_t)r, rep, ep_p, STREAM_PROCESS, nullptr, p.N, n4, p.pbase);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        Real xe[1] = {SX(c, e)};
        if (pred) {
          Real ne[1] = {n4[e]};
          M::transition(xe, P, u);
          M::add_lower(xe, ne, P, M::L::LQ);
        }
        SX(c, e) = xe[0];
        SLL(c, e) = upd ? M::loglik(xe, z, P, p.r_diag != 0) : Real(0);
      }
    }

    PX_MARK(0);
    // ---- (D) this tile's step s - 1 state is in memory: its data flag --------------------------
    if (s > 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's x / lw stores of step s - 1
      __syncthreads();
      if (t == 0) st_sc1(dfl + b, (unsigned long long)tag_prev);
    }

    PX_MARK(1);
    // ---- (P) the records of step s - 1 -> decision (prologue_reduce: k_step's arithmetic) -----
    double mk[RPT], s0k[RPT], s00k[RPT], uni = 0.0;
    const int k0 = t * RPT;
    if (s == 0) {  // the entry records (written before this launch)
      const double* rec_in = q.RB[cr] + (int64_t)r * RC::SIZE * G;
      uni = rec_in[RC::UNI * G];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int k = k0 + j;
        const bool in = k < G;
        mk[j] = in ? rec_in[RC::M * G + k] : -INFINITY;
        s0k[j] = in ? rec_in[RC::S0 * G + k] : 0.0;
        s00k[j] = in ? rec_in[RC::S00 * G + k] : 0.0;
        if (in) Mk[k] = mk[j];  // sys_ancestors reads the tile maxima as rec_in[M G + k]
      }
    } else {
      // every thread polls some of the 3 G heads (M, S0, S00 of each tile: two granules each) into
      // LDS, then takes its own RPT records from there
      const unsigned long long* gs = gr + (size_t)(((s - 1) % PRING) * PGF) * G;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        int good = 1;
        if (t == 0) {
          double v;
          good &= pgran_pair(gs + (2 * RC::UNI) * G, gs + (2 * RC::UNI + 1) * G, tag_prev, v);
          red[LDS_RED - 1] = v;
        }
#pragma unroll 1
        for (int j = t; j < 3 * G; j += BS) {
          const int f = j / G, k = j - f * G;  // f: 0 M, 1 S0, 2 S00 (fields 0, 1, 2 of the record)
          double v;
          good &= pgran_pair(gs + (2 * f) * G + k, gs + (2 * f + 1) * G + k, tag_prev, v);
          Mk[f * G8 + k] = v;
        }
        if (__syncthreads_and(good)) break;
        if (persist_slow_poll<BS>(q, s == 1, t0, &res_sh) == 2) return;
        __builtin_amdgcn_s_sleep(1);
      }
      uni = red[LDS_RED - 1];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int k = k0 + j;
        const bool in = k < G;
        mk[j] = in ? Mk[k] : -INFINITY;
        s0k[j] = in ? Mk[G8 + k] : 0.0;
        s00k[j] = in ? Mk[2 * G8 + k] : 0.0;
      }
      __syncthreads();  // prologue_reduce reuses red
    }
    PX_MARK(2);
    h = prologue_reduce<NX, BS>(mk, s0k, s00k, uni, G, p.N, p.thresh, allow != 0, false, allow != 0, red, Pl);
    PX_MARK(3);
    const bool gather = h.resample != 0;
    const double lse_prev = h.uniform ? 0.0 : h.lse;
    const Real lse_r = (Real)lse_prev;
    const Real lu = (Real)lprev_uniform;
    const bool write_x = pred || allow;  // k_step: gather launches always produce x_out

    WA acc;
    acc.init();
    double aux[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) aux[i] = 0.0;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(x_out, 0, (int)(p.Npad * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(lw_out, 0, (int)(p.Npad * 8), 0x00020000);
    // the chunk's new slots: written through to HBM now, into the LDS state after the record merge
    Real xv[8], lp[8];
    auto store_chunk = [&](int c) {
      const int64_t i0 = i0_of(c);
      const int nv = nv_of(c);
      if (nv == 4) {
        if (write_x) st4_sc1(rx, i0, xv + 4 * c);
        if (upd) st4_sc1(rl, i0, lp + 4 * c);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (e >= nv) break;
          if (write_x) st1_sc1(x_out + i0 + e, xv[4 * c + e]);
          if (upd) st1_sc1(lw_out + i0 + e, lp[4 * c + e]);
        }
      }
    };
    // k_step's fast finishes (FASTD): one reference maximum for the workgroup, one exponential per slot
    const bool ref_merge = upd && (!gather || pred);
    if (!gather) {
      // ---- (N) no resample: the weight shift of the speculated slots (k_step's fast finish) -----
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int nv = nv_of(c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const Real v = (h.uniform ? lu : SL(c, e) - lse_r) + SLL(c, e);
          xv[4 * c + e] = e < nv ? SX(c, e) : Real(0);  // slots past the tile: zero weight, finite value
          lp[4 * c + e] = (upd && e < nv) ? v : -INFINITY;
        }
        store_chunk(c);
      }
    } else {
      // ---- (G) resample: every tile's step s - 1 state, then k_step's ancestors and gather --------
      if (s > 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
          int good = 1;
          for (int k = t; k < G; k += BS) good &= ld_sc1(dfl + k) >= (unsigned long long)tag_prev;
          if (__syncthreads_and(good)) break;
          if (persist_slow_poll<BS>(q, false, t0, &res_sh) == 2) return;
          __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();  // Mk staged; the slot state (dead now) becomes the CDF / ancestor area
      const double U = uniform53(p.seed, 0, rep, ep_r);
      sys_ancestors<Real, NX, BS, 1>(lw_in, Mk, G, p.N, p.tile, o0, o1, U, h, Pl, anc_l, red, false);
#pragma unroll 1
      for (int c = 0; c < 2; ++c) {
        const int64_t i0 = i0_of(c);
        const int nv = nv_of(c);
        const int cc = t + c * BS;  // chunk index in the tile
        Real x[4], lq[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int a = e < nv ? anc_l[cc * CH + e] : 0;
          x[e] = x_in[a];
          lq[e] = lu;
        }
        Real nj4[4], np4[4];  // (the process normals: the speculation's values, drawn again)
        if (p.regularize && nv > 0)
          chunk_normals4<Real>(p.seed, i0, (uint32_t)r, rep, ep_r, STREAM_JITTER, nullptr, p.N, nj4, p.pbase);
        if (pred && nv > 0)
          chunk_normals4<Real>(p.seed, i0, (uint32_t)r, rep, ep_p, STREAM_PROCESS, nullptr, p.N, np4, p.pbase);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (e >= nv) break;
          Real xe[1] = {x[e]};
          if (p.regularize) {
            Real n1[1] = {nj4[e]};
            M::add_lower(xe, n1, P, M::L::LJ);
          }
          aux[0] += 1.0;
          aux[1] += (double)xe[0];
          if constexpr (RC::COV) aux[2] += (double)xe[0] * (double)xe[0];
          if (pred) {
            Real n1[1] = {np4[e]};
            M::transition(xe, P, u);
            M::add_lower(xe, n1, P, M::L::LQ);
          }
          const Real ll = upd ? M::loglik(xe, z, P, p.r_diag != 0) : Real(0);
          if (upd) {
            lq[e] = lq[e] + ll;
            if (!ref_merge) acc.add(lq[e], xe);  // (k_step's generic gather loop)
          }
          x[e] = xe[0];
        }
        // chunk c's slots (dynamic c: through the scratch-free selects below)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const Real xo = e < nv ? x[e] : Real(0);
          const Real lo = e < nv ? lq[e] : -INFINITY;
          if (c == 0) {
            xv[e] = xo;
            lp[e] = lo;
          } else {
            xv[4 + e] = xo;
            lp[4 + e] = lo;
          }
        }
        if (c == 0) store_chunk(0);
        else store_chunk(1);
      }
    }

    PX_MARK(4);
    if (ref_merge) {  // the workgroup maximum, then every thread's sums against it (add_ref8)
      Real mt = -INFINITY;
#pragma unroll
      for (int e = 0; e < 8; ++e) mt = rmax<Real>(mt, lp[e]);
      const Real Mb = block_max<BS>(mt, red);
      if (tix < nchunks) acc.add_ref8(lp, xv, Mb);
    }
    // ---- (R) the tile record (k_step's merge), stored and published ---------------------------
    __syncthreads();  // all tile-CDF / ancestor / Mk reads are done
    if (upd) {
      double w[1 + WA::NS];
      if (ref_merge) acc.template block_sum_ref<BS>(red, w);
      else acc.template block_merge<BS>(red, w);
      if (t == 0) {
        fin[RC::M] = w[0];
        fin[RC::S0] = w[1];
        fin[RC::S00] = w[2];
        fin[RC::UNI] = 0.0;
        for (int i = 0; i < NX + RC::NC; ++i) fin[RC::S1 + i] = w[3 + i];
      }
    } else if (t == 0) {
      if (gather) {  // gather-only step: weights become uniform
        fin[RC::M] = 0.0; fin[RC::S0] = 0.0; fin[RC::S00] = 0.0; fin[RC::UNI] = 1.0;
        for (int f = RC::S1; f < RC::A1; ++f) fin[f] = 0.0;
      } else {  // carry the update's record over
        for (int f = 0; f < RC::A1; ++f) fin[f] = finp[f];
      }
    }
    if (gather) {
      block_sum_k<NA, BS>(aux, red);
      if (t == 0) {
        fin[RC::CNT] = aux[0];
        for (int i = 0; i < NX + RC::NC; ++i) fin[RC::A1 + i] = aux[1 + i];
      }
    } else if (t == 0) {
      fin[RC::CNT] = 0.0;
      for (int f = RC::A1; f < RC::SIZE; ++f) fin[f] = 0.0;
    }
    __syncthreads();
    if (t < PGF) {  // wave 0: one granule per lane, all in one store instruction
      const unsigned long long bits = (unsigned long long)__double_as_longlong(fin[t >> 1]);
      const unsigned half = (t & 1) ? (unsigned)bits : (unsigned)(bits >> 32);
      st_sc1(gr + (size_t)((s % PRING) * PGF + t) * G + b, pgran(tag, half));
    }
    if (t < RC::SIZE) {
      rec_out[t * G + b] = fin[t];
      finp[t] = fin[t];
    }
    // the new slot state (own slots only: no barrier between this thread's writes and reads)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        SX(c, e) = xv[4 * c + e];
        if (upd) SL(c, e) = lp[4 * c + e];
      }
    if (write_x) cx ^= 1;
    if (upd) cl ^= 1;
    cr ^= 1;

    PX_MARK(5);
    // ---- outputs of step s - 1 (k_step's write_outputs in workgroup 0), off the critical path ----
#ifndef PX_NOOUT  // (A/B only: -DPX_NOOUT drops the outputs, profiles/r06/persist)
    if (b == 0 && s > 0)
#else
    if (false)
#endif
    {
      // the step s - 1 records' other fields (CNT, S1, S2, A1, A2) of this thread's tiles t, t + BS:
      // one batch of granule loads, repeated until every tag matches; M and S0 are the polled heads
      const unsigned long long* gs = gr + (size_t)(((s - 1) % PRING) * PGF) * G;
      constexpr int NF = RC::SIZE - RC::CNT;
      double rv[2][NF];
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        int good = 1;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int f = 0; f < NF; ++f) {
            const int k = t + j * BS;
            rv[j][f] = 0.0;
            if (k < G)
              good &= pgran_pair(gs + (2 * (RC::CNT + f)) * G + k, gs + (2 * (RC::CNT + f) + 1) * G + k, tag_prev,
                                 rv[j][f]);
          }
        if (good) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > PSPIN_TICKS) {
          atomicOr(q.err, 2u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      auto rec_at = [&](int f, int k) -> double {  // k is t or t + BS (G <= 2 BS)
        if (f == RC::M) return Mk[k];
        if (f == RC::S0) return Mk[G8 + k];
        return k < t + BS ? rv[0][f - RC::CNT] : rv[1][f - RC::CNT];
      };
      write_outputs_f<NX, BS>(p, s - 1, s >= 2 ? s - 2 : -1, rec_at, h, r, R, 0, G, red);
    }
    PX_MARK(6);
#ifdef PF_STAMPS
    if (px_me) px_acc[7] += 1;
#endif
  }
#ifdef PF_STAMPS
  if (px_me)
    for (int k = 0; k < 8; ++k) g_pf_stamps[k] = px_acc[k];
#endif

  // ---- finalize (k_finalize): the tail's records -> the post-resample statistics of step T - 1 ----
  if (b != 0) return;
  __syncthreads();
  const unsigned tag_fin = q.tag0 + (unsigned)q.T + 1;
  const unsigned long long* gs = gr + (size_t)((q.T % PRING) * PGF) * G;
  auto rec_at = [&](int f, int k) { return pgran_wait(gs, f, k, G, tag_fin, q.err); };
  double mk[RPT], s0k[RPT], s00k[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int k = t * RPT + j;
    mk[j] = k < G ? rec_at(RC::M, k) : -INFINITY;
    s0k[j] = k < G ? rec_at(RC::S0, k) : 0.0;
    s00k[j] = k < G ? rec_at(RC::S00, k) : 0.0;
  }
  if (t == 0) red[LDS_RED - 1] = rec_at(RC::UNI, 0);
  __syncthreads();
  const double uni = red[LDS_RED - 1];
  __syncthreads();
  const Head hf = prologue_reduce<NX, BS>(mk, s0k, s00k, uni, G, p.N, p.thresh, true, false, false, red, nullptr);
  write_outputs_f<NX, BS>(p, -1, q.T - 1, rec_at, hf, r, R, 0, 1, red);
}

}  // namespace pf
