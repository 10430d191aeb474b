// k_step_stream: the fp32 scalar-state fused SIR step (predict + update; the resample decided by
// k_head and fused into the next step, pf.py:223-269 + 146-171) as a persistent, software-pipelined
// grid - the many-replicate launches (SURVEY 8(d) roofline run: 64 x 1e6 SV filters per GPU).
//
// k_step gives each 2048-particle tile its own workgroup: a workgroup loads its tile, waits for the
// loads, computes and exits, and the four workgroups a CU holds (VGPR-limited) hide each other's
// load latency only partly (sv64: ~9 us workgroup lifetimes, ~5.7 of them before the head decision).
// Here a grid of a few workgroups per CU walks the tiles (tile id = blockIdx.x + k gridDim.x,
// replicate-major), and the x / lw of tile k + 1 (and its replicate's head and observation) are in
// flight while tile k is computed: HBM latency overlaps the Philox / transition / weight arithmetic
// inside every wave instead of across workgroups.
//
// Per tile the arithmetic is k_step's fast path (no resample: the thread's 8 slots straight from the
// prefetched registers) or its gather-fast path (the replicate resampled: sys_ancestors over the
// k_head prefix, gathered slots, jitter, predict, weigh), weighed against the workgroup maximum
// (add_ref8) and merged by block_sum_lds: the same records and outputs k_step writes for these
// launches, with the same Philox counters.  Every step of a run with this kernel is computed by it
// (segmented runs: a gather-only k_step launch + a stream launch equal one fused stream launch).
#pragma once
#include "pf_kernels.h"

namespace pf {

#ifndef PF_STREAM
#define PF_STREAM 1
#endif

template <int NZ>
struct StreamPre {  // one tile's operands, loaded one tile ahead
  float xa[4], la[4], xb[4], lb[4];  // slots [4t, 4t + 4) and [4(t + BS), ...) of the tile
  double hd;                          // lane q < HEAD_F: head field q of the tile's replicate
  float z[NZ];                        // the replicate's observation
};

template <int BS, int NZ>
__device__ __forceinline__ void stream_fetch(const StepParams& p, int id, StreamPre<NZ>& f) {
  const int t = threadIdx.x;
  const int r = id / p.G, b = id - r * p.G;
  const int64_t o0 = (int64_t)b * p.tile, o1 = min(o0 + (int64_t)p.tile, p.N);
  const int nch = (int)((o1 - o0 + 3) / 4);
  const float* x = (const float*)p.x_in + (int64_t)r * p.Npad + o0;
  const float* lw = (const float*)p.lw_in + (int64_t)r * p.Npad + o0;
  if (t < nch) {
    load4<float>(x + 4 * t, f.xa);
    load4<float>(lw + 4 * t, f.la);
  }
  if (t + BS < nch) {
    load4<float>(x + 4 * (t + BS), f.xb);
    load4<float>(lw + 4 * (t + BS), f.lb);
  }
  const int lane = t & 63;
  f.hd = lane < HEAD_F ? p.head[(int64_t)r * HEAD_STRIDE + lane] : 0.0;
#pragma unroll
  for (int k = 0; k < NZ; ++k) f.z[k] = ((const float*)p.z)[(int64_t)r * p.z_rs + k];
}


// this tile's slots stored, weighed against the workgroup maximum and merged into its record
// (k_step's record layout and arithmetic for these launches); aux: the post-resample sums (gather)
template <int BS, int NA>
__device__ __forceinline__ void stream_finish(const StepParams& p, int r, int b, int64_t ia, int64_t ib, int na, int nb,
                                              int nchunks, float (&xv)[8], float (&lp)[8], double (&aux)[NA],
                                              bool gather, float* stage, double* fin, double* red) {
  using RC = Rec<1>;
  using WA = WAcc<float, 1>;
  const int t = threadIdx.x;
  float* x_out = (float*)p.x_out + (int64_t)r * p.Npad;
  float* lw_out = (float*)p.lw_out + (int64_t)r * p.Npad;
  float mt = -INFINITY;
#pragma unroll
  for (int e = 0; e < 8; ++e) mt = fmaxf(mt, lp[e]);
  if (na == 4) {
    store4<float>(x_out + ia, xv);
    store4<float>(lw_out + ia, lp);
  } else {
    for (int e = 0; e < na; ++e) {
      x_out[ia + e] = xv[e];
      lw_out[ia + e] = lp[e];
    }
  }
  if (nb == 4) {
    store4<float>(x_out + ib, xv + 4);
    store4<float>(lw_out + ib, lp + 4);
  } else {
    for (int e = 0; e < nb; ++e) {
      x_out[ib + e] = xv[4 + e];
      lw_out[ib + e] = lp[4 + e];
    }
  }
  WA acc;
  acc.init();
  const float Mb = block_max_f<BS>(mt, stage);
  if (t < nchunks) acc.add_ref8(lp, xv, Mb);
  double* rec_out = p.rec_out + (int64_t)r * RC::SIZE * p.G;
  __syncthreads();  // the block maximum's slots are read before the staging reuses them
  double w[1 + WA::NS];
  acc.template block_sum_lds<BS>(stage, w);
  if (t == 0) {
    fin[RC::M] = w[0];
    fin[RC::S0] = w[1];
    fin[RC::S00] = w[2];
    fin[RC::UNI] = 0.0;
    for (int i = 0; i < 1 + RC::NC; ++i) fin[RC::S1 + i] = w[3 + i];
  }
  if (gather) {
    block_sum_k<NA, BS>(aux, red);
    if (t == 0) {
      fin[RC::CNT] = aux[0];
      for (int i = 0; i < 1 + RC::NC; ++i) fin[RC::A1 + i] = aux[1 + i];
    }
  } else if (t == 0) {
    fin[RC::CNT] = 0.0;
    for (int q = RC::A1; q < RC::SIZE; ++q) fin[q] = 0.0;
  }
  __syncthreads();
  for (int q = t; q < RC::SIZE; q += BS) rec_out[q * p.G + b] = fin[q];
  __syncthreads();  // fin / staging / red are reused by the next tile
}

// Two passes over the workgroup's tiles (tile id = blockIdx.x + k gridDim.x): first the tiles of
// replicates that did not resample, software-pipelined; then those of replicates that did (the gather
// path, no pipelining).  The passes have disjoint live ranges, so the streaming pass keeps its
// registers (the gather path's fp64 search state would otherwise be co-allocated with the prefetched
// operands).  The replicates' decisions are staged in LDS once (flags: R ints after the ancestors).
// The smallest tile the host launches k_step_stream with (pf_engine.hip launch_step).  The decisions
// flags[R] start 12 tile bytes past cdf (the fp64 CDF and the int ancestors of one tile), and the
// record merge's staging occupies cdf bytes [256, MERGE_LDS_BYTES): the two are disjoint only for
// tiles of at least MERGE_LDS_BYTES / 12 particles.
constexpr int STREAM_MIN_TILE = 512;
static_assert(12 * STREAM_MIN_TILE >= MERGE_LDS_BYTES, "k_step_stream: flags would overlap the merge staging");

#ifndef PF_STREAM_WPE
#define PF_STREAM_WPE 4
#endif
template <int NZ, int TK, int OK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PF_STREAM_WPE)))
k_step_stream(StepParams p, int R) {
  using M = Model<float, 1, NZ, TK, OK>;
  using RC = Rec<1>;
  constexpr int BS = 256, CH = 4;
  constexpr int NA = 1 + 1 + RC::NC;  // aux: cnt, sum x, sum x^2
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* red = smem;
  double* Pl = smem + LDS_PL;
  double* cdf = smem + lds_tile(p.G);
  int* anc_l = (int*)(cdf + p.tile);
  int* flags = anc_l + p.tile;         // [R] the replicates' resample decisions (k_head)
  float* stage = (float*)(cdf + 32);   // the record merge's staging (MERGE_LDS_BYTES)
  double* fin = cdf;                   // the staged record
  const int t = threadIdx.x;
  const int G = p.G, ntiles = G * R;
  const float* __restrict__ P = (const float*)p.P;
  const double lprev_uniform = -log((double)p.N);
  const float lu = (float)lprev_uniform;
  for (int q = t; q < R; q += BS) flags[q] = p.head[(int64_t)q * HEAD_STRIDE + 7] != 0.0 ? 1 : 0;

  // ---- pass 1: replicates that did not resample, the next tile's operands in flight --------
  StreamPre<NZ> cur;
  int id = blockIdx.x;
  __syncthreads();  // flags
  if (id < ntiles && !flags[id / G]) stream_fetch<BS, NZ>(p, id, cur);
  int ngather = 0;
  for (; id < ntiles; id += gridDim.x) {  // uniform per workgroup
    const StepParams& q = p;
    const int r = id / G, b = id - r * G;
    StreamPre<NZ> nxt;
    const int nid = id + gridDim.x;
    if (nid < ntiles && !flags[nid / G]) stream_fetch<BS, NZ>(q, nid, nxt);  // (a gathering tile reads its own)
    if (flags[r]) {  // pass 2
      ++ngather;
      cur = nxt;
      continue;
    }
    const int64_t o0 = (int64_t)b * q.tile, o1 = min(o0 + (int64_t)q.tile, q.N);
    const int nchunks = (int)((o1 - o0 + CH - 1) / CH);
    const uint32_t rep = (uint32_t)(r + q.rep_base);
    const bool uniform = readlane_d(cur.hd, 6) != 0.0;
    const double lse = readlane_d(cur.hd, 4);
    const float* u = q.u ? (const float*)q.u + (int64_t)r * q.u_rs : nullptr;
    const int64_t ia = o0 + (int64_t)t * CH, ib = o0 + (int64_t)(t + BS) * CH;
    const int na = t < nchunks ? (int)min((int64_t)4, o1 - ia) : 0;
    const int nb = t + BS < nchunks ? (int)min((int64_t)4, o1 - ib) : 0;
    float pa[4], pb[4];  // the process noise of the thread's two chunks
    const uint64_t seed = q.seed;
    if (na > 0)
      chunk_normals4<float>(seed, ia, (uint32_t)r, rep, q.ep_predict, STREAM_PROCESS, q.rp_noise, q.N, pa, q.pbase);
    if (nb > 0)
      chunk_normals4<float>(seed, ib, (uint32_t)r, rep, q.ep_predict, STREAM_PROCESS, q.rp_noise, q.N, pb, q.pbase);
    // predicted slots and their log-weights l_prev - lse + loglik (pf.py:254-256)
    const float lse_r = (float)(uniform ? 0.0 : (q.use_lse_ext ? q.lse_ext : lse));
    float xv[8], lp[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool in = e < 4 ? e < na : e - 4 < nb;
      float xe[1] = {e < 4 ? cur.xa[e] : cur.xb[e - 4]};
      float ne[1] = {e < 4 ? pa[e] : pb[e - 4]};
      M::transition(xe, P, u);
      M::add_lower(xe, ne, P, M::L::LQ);
      const float ll = M::loglik(xe, cur.z, P, q.r_diag != 0);
      const float lraw = e < 4 ? cur.la[e] : cur.lb[e - 4];
      const float v = (uniform ? lu : lraw - lse_r) + ll;
      xv[e] = in ? xe[0] : 0.0f;  // slots past the tile: zero weight, finite value
      lp[e] = in ? v : -INFINITY;
    }
    double aux[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) aux[i] = 0.0;
    stream_finish<BS, NA>(q, r, b, ia, ib, na, nb, nchunks, xv, lp, aux, false, stage, fin, red);
    cur = nxt;
  }
  if (ngather == 0) return;  // uniform

  // ---- pass 2: replicates that resampled at the previous step ------------------------------
  // their tile prefix (k_head) -> ancestors -> gathered slots (+ jitter) -> predict -> weigh,
  // uniform previous weights (pf.py:188-218), as k_step's gather-fast block
  for (id = blockIdx.x; id < ntiles; id += gridDim.x) {
    const int r = id / G, b = id - r * G;
    if (!flags[r]) continue;
    const int64_t o0 = (int64_t)b * p.tile, o1 = min(o0 + (int64_t)p.tile, p.N);
    const int nchunks = (int)((o1 - o0 + CH - 1) / CH);
    const uint32_t rep = (uint32_t)(r + p.rep_base);
    const double* o = p.head + (int64_t)r * HEAD_STRIDE;
    Head h;
    h.M = o[0];
    h.S = o[1];
    h.S2 = o[2];
    h.Sscan = o[3];
    h.lse = o[4];
    h.neff = o[5];
    h.uniform = o[6] != 0.0;
    h.resample = 1;
    for (int k = t; k <= G; k += BS) Pl[k] = o[HEAD_F + k];
    __syncthreads();
    const float* x_in = (const float*)p.x_in + (int64_t)r * p.Npad;
    const float* lw_in = (const float*)p.lw_in + (int64_t)r * p.Npad;
    const double* rec_in = p.rec_in + (int64_t)r * RC::SIZE * G;
    const float* u = p.u ? (const float*)p.u + (int64_t)r * p.u_rs : nullptr;
    float z[NZ];
#pragma unroll
    for (int k = 0; k < NZ; ++k) z[k] = ((const float*)p.z)[(int64_t)r * p.z_rs + k];
    const double U = p.rp_unif ? p.rp_unif[r] : uniform53(p.seed, 0, rep, p.ep_resample);
    sys_ancestors<float, 1, BS, 8>(lw_in, rec_in, G, p.N, p.tile, o0, o1, U, h, Pl, anc_l, red, false);
    const int64_t ia = o0 + (int64_t)t * CH, ib = o0 + (int64_t)(t + BS) * CH;
    const int na = t < nchunks ? (int)min((int64_t)4, o1 - ia) : 0;
    const int nb = t + BS < nchunks ? (int)min((int64_t)4, o1 - ib) : 0;
    float xv[8], lp[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xv[e] = e < na ? x_in[anc_l[t * CH + e]] : 0.0f;
      xv[4 + e] = e < nb ? x_in[anc_l[(t + BS) * CH + e]] : 0.0f;
    }
    if (p.regularize) {
      float ja[4], jb[4];
      if (na > 0)
        chunk_normals4<float>(p.seed, ia, (uint32_t)r, rep, p.ep_resample, STREAM_JITTER, p.rp_jit, p.N, ja, p.pbase);
      if (nb > 0)
        chunk_normals4<float>(p.seed, ib, (uint32_t)r, rep, p.ep_resample, STREAM_JITTER, p.rp_jit, p.N, jb, p.pbase);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float xe[1] = {xv[e]}, ne[1] = {e < 4 ? ja[e] : jb[e - 4]};
        M::add_lower(xe, ne, P, M::L::LJ);
        if (e < 4 ? e < na : e - 4 < nb) xv[e] = xe[0];
      }
    }
    double aux[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) aux[i] = 0.0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // k_step's order: chunk t's slots, then chunk t + BS's
      if (e < 4 ? e < na : e - 4 < nb) {
        aux[0] += 1.0;
        aux[1] += (double)xv[e];
        if constexpr (RC::COV) aux[2] += (double)xv[e] * (double)xv[e];
      }
    }
    float pa[4], pb[4];
    if (na > 0)
      chunk_normals4<float>(p.seed, ia, (uint32_t)r, rep, p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, pa, p.pbase);
    if (nb > 0)
      chunk_normals4<float>(p.seed, ib, (uint32_t)r, rep, p.ep_predict, STREAM_PROCESS, p.rp_noise, p.N, pb, p.pbase);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool in = e < 4 ? e < na : e - 4 < nb;
      float xe[1] = {xv[e]};
      float ne[1] = {e < 4 ? pa[e] : pb[e - 4]};
      M::transition(xe, P, u);
      M::add_lower(xe, ne, P, M::L::LQ);
      xv[e] = in ? xe[0] : 0.0f;
      lp[e] = in ? lu + M::loglik(xe, z, P, p.r_diag != 0) : -INFINITY;
    }
    stream_finish<BS, NA>(p, r, b, ia, ib, na, nb, nchunks, xv, lp, aux, true, stage, fin, red);
  }
}

}  // namespace pf
