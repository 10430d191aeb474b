// Host side of the MI355X SIR engine: the C ABI of include/pf_engine.h.
//
// Owns one device, one HIP stream and the device-resident filter state of R
// replicates; turns the reference's call sequence (initialize / predict /
// update / _resample, /root/reference/models/particle_filter.py:110-287) into
// launches of the fused kernels in pf_kernels.h, and runs the whole T loop on
// device (pf_run_device) with no host synchronisation inside T.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pf_engine.h"
#include "pf_cov.h"
#include "pf_hooks.h"
#include "pf_order.h"
#include "../../include/pf_shard.h"
#include "pf_diag.h"
#include "pf_dyn_layout.h"
#include "pf_ops.h"
#include "pf_resample_w.h"

namespace pf {

static thread_local std::string g_err;
void set_last_error(const std::string& msg) { g_err = msg; }  // shared with pf_ledh.hip

static pf_status fail(pf_status code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return fail(PF_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));             \
  } while (0)

static std::vector<Ops>& registry() {
  static std::vector<Ops> r;
  return r;
}
void register_ops(const Ops& o) { registry().push_back(o); }
static void ensure_registered() {
  static std::once_flag once;
  std::call_once(once, [] {
    register_sv_models();
    register_linear_models();
    register_l96_models();
    register_mat_models();
    register_dyn_models();
  });
}
// compiled-shape kernels of exactly (nx, nz, tk, ok, prec), or null
const Ops* find_ops(int nx, int nz, int tk, int ok, int prec) {
  ensure_registered();
  for (const Ops& o : registry())
    if (!o.dyn && o.nx == nx && o.nz == nz && o.tk == tk && o.ok == ok && o.prec == prec) return &o;
  return nullptr;
}
// do the kinds fit the shape (pf_model_supported's rules)?
static bool kinds_fit(int nx, int nz, int tk, int ok) {
  if (nx <= 0 || nz <= 0) return false;
  if (tk != PF_TRANS_LINEAR && tk != PF_TRANS_L96) return false;
  switch (ok) {
    case PF_OBS_LINEAR: return true;
    case PF_OBS_EXP_HALF:
    case PF_OBS_SV_EXACT: return nz == nx;
    case PF_OBS_ACOUSTIC: return nx % 4 == 0;
    case PF_OBS_BEARINGS: return nz == 2 && nx >= 3;
    default: return false;
  }
}
// runtime-shape kernels (pf_dyn.h) for (nx, nz, tk, ok, prec): the registered shape template,
// materialised once per concrete shape (stable addresses: handles keep the pointer)
const Ops* find_ops_dyn(int nx, int nz, int tk, int ok, int prec) {
  ensure_registered();
  if (!kinds_fit(nx, nz, tk, ok)) return nullptr;
  static std::mutex mu;
  static std::deque<Ops> shapes;
  std::lock_guard<std::mutex> lock(mu);
  for (const Ops& o : shapes)
    if (o.nx == nx && o.nz == nz && o.tk == tk && o.ok == ok && o.prec == prec) return &o;
  for (const Ops& t : registry())
    if (t.dyn && t.tk == tk && t.ok == ok && t.prec == prec) {
      Ops o = t;
      o.nx = nx;
      o.nz = nz;
      o.rec_size = DynRec(nx).SIZE;
      o.psize = DynLay(nx, nz).SIZE;
      shapes.push_back(o);
      return &shapes.back();
    }
  return nullptr;
}

// Lower Cholesky factor of an n x n row-major SPD matrix (+ jitter * I); false if not PD.
static bool cholesky(const double* A, int n, double jitter, std::vector<double>& L) {
  L.assign((size_t)n * n, 0.0);
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j] + jitter;
    for (int k = 0; k < j; ++k) d -= L[j * n + k] * L[j * n + k];
    if (!(d > 0.0) || !std::isfinite(d)) return false;
    const double ljj = std::sqrt(d);
    L[j * n + j] = ljj;
    for (int i = j + 1; i < n; ++i) {
      double s = A[i * n + j] + (i == j ? jitter : 0.0);
      for (int k = 0; k < j; ++k) s -= L[i * n + k] * L[j * n + k];
      L[i * n + j] = s / ljj;
    }
  }
  return true;
}

}  // namespace pf

using namespace pf;

// What a k_head launch depends on: a later launch with an equal key reads the same heads.
struct HeadKey {
  const double* rec_in;
  int allow_gather, force_gather;
  int64_t out_step, out_post_step;
  const void *o_mean, *o_cov, *o_neff, *o_lse, *o_flag;
  bool operator==(const HeadKey& o) const {
    return rec_in == o.rec_in && allow_gather == o.allow_gather && force_gather == o.force_gather &&
           out_step == o.out_step && out_post_step == o.out_post_step && o_mean == o.o_mean && o_cov == o.o_cov &&
           o_neff == o.o_neff && o_lse == o.o_lse && o_flag == o.o_flag;
  }
};
HeadKey head_key(const StepParams& p) {
  return HeadKey{p.rec_in, p.allow_gather, p.force_gather, p.out_step, p.out_post_step,
                 p.o_mean, p.o_cov, p.o_neff, p.o_lse, p.o_flag};
}

struct pf_handle {
  const Ops* ops = nullptr;
  int nx = 0, nz = 0, tk = 0, ok = 0, prec = 0;
  int64_t N = 0, Npad = 0;
  int R = 1, G = 1, tile = 0, method = 0, regularize = 0, r_diag = 1;
  double thresh = 0.5;
  uint64_t seed = 0;
  int device = 0;
  int rep_base = 0;
  size_t esz = 4;  // sizeof(Real)
  hipStream_t stream = nullptr;
  // device state
  void* x[2] = {nullptr, nullptr};
  void* lw[2] = {nullptr, nullptr};
  double* rec[2] = {nullptr, nullptr};
  int cx = 0, clw = 0, crec = 0;
  void* P = nullptr;   // model params (Real)
  double* cdf = nullptr;
  // small device staging
  void* d_z = nullptr;       // Real [R][nz]
  void* d_u = nullptr;       // Real [R][nx]
  double* d_out = nullptr;   // API outputs: mean[R*nx] cov[R*nx*nx] neff[R] lse[R] flags(int)[R] + post
  double* d_replay_a = nullptr;  // [R][N][nx] normals
  double* d_replay_b = nullptr;  // [R][N][nx] jitter normals
  double* d_unif = nullptr;      // [R][N] uniforms
  // host-side bookkeeping
  bool initialized = false;
  bool pending = false;       // last update decided to resample some replicate (not yet applied)
  uint32_t epoch = 1;         // Philox epoch counter (one per predict, one per update)
  uint32_t ep_res = 0;        // epoch reserved by the last update for its resample
  bool chol_q_ok = true;
  int lq_local = 0, lj_local = 0;  // chol(Q) / 0.001 chol(Q) block-diagonal in nx/4 blocks (k_step_grp)
  int sys_cdf = 0;  // systematic ancestors from the materialised CDF (k_cdf) instead of per-tile scans
  int h_sel = 0;    // LINEAR h is a component selection (StepParams.hcol2k; runtime-shape kernels: P[EX+2+k])
  // runtime-shape kernels (pf_dyn.h): per-replicate scratch [R][wrows][Npad], diagonal factors
  void* wbuf = nullptr;
  int64_t wrows = 0;
  int a_diag = 0, lq_diag = 0, lj_diag = 0;
  int32_t hcol2k[64];
  // within-filter sharding (pf_shard.h): global index of particle 0, filter size, CDF epoch
  bool sharded = false;
  int64_t pbase = 0, n_total = 0;
  uint32_t shard_cdf_ep = 0;
  bool needs_cdf() const { return method == 1 || sys_cdf || sharded; }
  // large-state systematic path: the update launch leaves the in-tile CDF prefix (StepParams::
  // lcum_out) and the next gather reads it, so no k_cdf launch (lcum_valid: the current
  // weights' prefix exists; set_state / gather-only launches invalidate it)
  bool lcum_mode = false;
  double* lcum[2] = {nullptr, nullptr};
  int clcum = 0;
  bool lcum_valid = false;
  bool cdf_needed() const { return needs_cdf() && !(lcum_mode && lcum_valid && method == 0 && !sharded); }
  // per-step replicate heads (k_head, StepParams::head): -1 auto, 0 off, 1 on (PF_HEAD)
  int head_mode = -1;
  // persistent fused step for head launches of the fp32 scalar models (k_step_stream): 1 on, 0 off (PF_STREAM)
  int stream_mode = 1;
  bool last_stream = false;  // the last fused step launch ran k_step_stream
  double* head = nullptr;  // [R][HEAD_STRIDE]
  // the launch that produced the current heads (reused by the next launch when equal)
  bool head_valid = false;
  HeadKey head_key;
  std::vector<double> Pd;     // params (double)
  // register-resident whole-run path (k_resident): hand-off words, zeroed per launch
  unsigned long long* rsync = nullptr;
  size_t rsync_bytes = 0;
  uint32_t res_tag = 0;           // granule tag base of the next resident launch (ResParams::tag0)
  unsigned long long res_flag = 0; // hand-off flag base of the next resident launch
  bool res_unchecked = false;  // a resident launch whose timeout word is not yet read
  // plain-launch co-residency check (ResParams::arrive): workgroups counted so far, launch
  // sequence; after an abort the handle launches cooperatively from then on
  unsigned long long res_arrive = 0, res_seq = 0;
  unsigned long long res_shard[RSHARDS] = {};  // k_resident's arrival shards: counts before the next launch
  bool res_force_coop = false;
  // entry header (ResParams::hdr): id of the last resident run whose exit header still
  // describes the state (0: none; any other write of the state clears it), run counter
  unsigned long long res_hdr = 0, res_run = 0;
  // entry header restored by pf_restore ([R][4] words, id filled in at the next resident run)
  std::vector<unsigned long long> hdr_restore;
  // bookkeeping before each resident run not yet checked (check_resident), by launch sequence
  // number: an aborted launch (and every later one, which aborts too) is undone to its entry
  struct ResUndo {
    unsigned long long seq;
    uint32_t epoch, ep_res;
    int crec, cx, clw;
    unsigned long long hdr;
  };
  std::vector<ResUndo> res_undo;
  int resident_runs = 0;       // diagnostics: pf_run_device calls served by k_resident
  bool last_resident = false;  // the last pf_run_device ran k_resident
  // persistent fp64 whole-run path (pf_persist.h): granule ring + data flags, tag base, diagnostics
  unsigned long long* psync = nullptr;
  size_t psync_words = 0;
  uint32_t pers_tag = 0;
  int persist_runs = 0;
  bool last_persist = false;
  // device-loop covariance for nx > 4 (pf_cov.h): post-resample rows, block partials, sums,
  // per-replicate arrival counters, and the launch geometry
  void* xr = nullptr;        // post-resample rows (with jitter) ...
  int32_t* anc = nullptr;    // ... or the ancestors of the post-resample slots (without)
  void* cov_part = nullptr;  // [tc][R][nblk][P] block partials (doubles)
  double* cov_tot = nullptr;
  int cov_tc = 0;       // ring slots (steps) of partials
  int64_t cov_s0 = 0;   // first step of the pending chunk
  int cov_pending = 0;  // steps in the ring
  bool cov_ready = false;  // every buffer above allocated and the geometry checked (ensure_cov)
  CovParams covp{};
  // verification trace of resident runs (pf_set_trace; tests): [tr_T][R][Npad] each
  float* tr_x = nullptr;
  float* tr_l = nullptr;
  int32_t* tr_anc = nullptr;
  int64_t tr_T = 0;
  // live kernel timing (pf_set_timing): events recorded on the handle's stream right
  // before the first and after the last filter kernel of each pf_run_device
  bool timing = false;
  hipEvent_t tev[2] = {nullptr, nullptr};
};

namespace {

// Any write of the state other than a resident run: the last resident exit header (or one a
// checkpoint restored) no longer describes it.
void state_written(pf_handle* h) {
  h->res_hdr = 0;
  h->hdr_restore.clear();
}

size_t rec_bytes(const pf_handle* h) { return (size_t)h->R * h->G * h->ops->rec_size * sizeof(double); }

// Tiles of one chunk per thread (BLOCK*CH particles) so that a large filter runs
// several workgroups per CU; past MAXG tiles the tile grows (chunks per thread).
// PF_CHUNKS_PER_THREAD overrides the chunks per thread (tuning experiments).
bool choose_geometry(pf_handle* h) {
  const int64_t tile_min = h->ops->tile_min;
  const char* env = std::getenv("PF_CHUNKS_PER_THREAD");
  int64_t tile = tile_min * (env ? std::max(1, std::atoi(env)) : 1);
  if ((h->N + tile - 1) / tile > MAXG) tile = (h->N + MAXG - 1) / MAXG;
  // many replicates: a whole number of chunk-loop passes per tile.  A partial last pass
  // costs a whole pass of latency for a few particles, and the R x G grid runs in several
  // rounds, so fuller tiles cut rounds (MAT 8 x 1e5: tile 196 = 3 passes + 4 particles ->
  // 256, 216 -> 199 us/step).  One replicate fits one round either way (L96 N = 1e5 measured
  // 56.3 us at tile 98 vs 57.8 at 128), so it keeps the smaller tiles.
  const char* rnd = std::getenv("PF_TILE_ROUND");
  if (!(rnd && std::atoi(rnd) == 0) && h->R >= 2 && tile > tile_min && tile_min * ((tile + tile_min - 1) / tile_min) <= h->ops->tile_max)
    tile = tile_min * ((tile + tile_min - 1) / tile_min);
  tile = (tile + h->ops->ch - 1) / h->ops->ch * h->ops->ch;
  if (tile > h->N) tile = (h->N + h->ops->ch - 1) / h->ops->ch * h->ops->ch;
  // many replicates: grow small tiles while the grid exceeds ~4096 workgroups (every workgroup
  // reduces all G records of its replicate in the prologue: O(G^2 R) record reads)
  while (!env && (int64_t)h->R * ((h->N + tile - 1) / tile) > 4096 && tile < 256 && tile * 2 <= h->ops->tile_max)
    tile *= 2;
  // large-state lane-group step (fp32, diagonal R, lane-local noise: 4 workgroups per CU, 1024
  // resident on the 256 CUs) over many replicates: the R x G grid runs in rounds of 1024 and a
  // workgroup's time is its chunk passes plus a fixed part (prologue / head, ancestors, record:
  // ~1.5 passes), so take the passes per tile (<= 8) that minimise rounds x (passes + 1.5).
  // MAT 8 x 1e5: 256 -> 448 (3.05 -> 1.75 rounds), 93.6 -> 87.1 us/step; 64 x 1e5 on one GPU:
  // 651 -> 561 us/step (profiles/r02/mattile).
  if (!env && h->ops->grp && h->esz == 4 && h->R >= 2 && h->r_diag && h->lq_local && h->lj_local &&
      tile % tile_min == 0) {
    auto cost = [&](int64_t t) {
      const int64_t rounds = ((int64_t)h->R * ((h->N + t - 1) / t) + 1023) / 1024;
      return (double)rounds * ((double)(t / tile_min) + 1.5);
    };
    int64_t best = tile;
    for (int64_t t = tile + tile_min; t <= 8 * tile_min && t <= h->ops->tile_max && t <= h->N; t += tile_min)
      if (cost(t) < cost(best)) best = t;
    tile = best;
  }
  // scalar-state kernels (4-particle chunks, 1024-particle minimum tile) with many
  // replicates: two chunk-loop passes per thread halve the grid and amortise the per-
  // workgroup head load and record reduction (sv64, 64 x 1e6: 463 -> 442 us/step); more
  // passes lose occupancy to the gather LDS (3: 492 us, 4: 618 us)
  if (!env && h->ops->ch > 1 && tile == tile_min && (int64_t)h->R * ((h->N + tile - 1) / tile) > 4096 &&
      tile * 2 <= h->ops->tile_max && tile * 2 <= h->N)
    tile *= 2;
  // fp64 scalar state, one replicate: k_step<double> holds 167 VGPRs (3 workgroups per CU, 768
  // on the 256 CUs), so 1024-particle tiles of N = 1e6 (977 workgroups) run in two rounds; two
  // chunk passes per thread keep the grid in one (fp64 SV N = 1e6: 32.0 -> 30.4 us/step)
  if (!env && h->esz == 8 && h->ops->ch > 1 && h->R == 1 && tile == tile_min && (h->N + tile - 1) / tile > 768 &&
      tile * 2 <= h->ops->tile_max)
    tile *= 2;
  if (tile > h->ops->tile_max) return false;
  h->tile = (int)tile;
  h->G = (int)((h->N + tile - 1) / tile);
  return h->G <= MAXG;
}

// k_step LDS: base | tile CDF (doubles) + ancestor slots (ints) when gathering | epilogue record staging
size_t step_lds(const pf_handle* h, bool gather) {
  if (h->ops->dyn)  // tile CDF / per-particle weights (doubles) + ancestor slots (ints)
    return base_lds_bytes(h->G) + (size_t)h->tile * (sizeof(double) + sizeof(int));
  size_t epi = (size_t)h->ops->rec_size * sizeof(double);
  if (h->nx == 1 && h->ops->prec == PF_PRECISION_FP32) epi = std::max(epi, (size_t)MERGE_LDS_BYTES);
  size_t gat = gather ? (size_t)h->tile * (sizeof(double) + sizeof(int)) : 0;
  if (gather && h->sys_cdf) gat += (size_t)SYS_STAGE * h->tile * sizeof(double) + 16;  // staged source tiles
  return base_lds_bytes(h->G) + std::max(epi, gat);
}

template <typename T>
void to_real(const double* src, size_t n, std::vector<char>& dst, size_t esz) {
  dst.resize(n * esz);
  if (esz == 8) {
    std::memcpy(dst.data(), src, n * 8);
  } else {
    float* f = (float*)dst.data();
    for (size_t i = 0; i < n; ++i) f[i] = (float)src[i];
  }
}

StepParams base_params(pf_handle* h) {
  StepParams p;
  std::memset(&p, 0, sizeof(p));
  p.P = h->P;
  p.N = h->N;
  p.Npad = h->Npad;
  p.G = h->G;
  p.tile = h->tile;
  p.seed = h->seed;
  p.thresh = h->thresh;
  p.method = h->method;
  p.regularize = h->regularize;
  p.r_diag = h->r_diag;
  p.rep_base = h->rep_base;
  p.lq_local = h->lq_local;
  p.lj_local = h->lj_local;
  p.sys_cdf = h->sys_cdf;
  p.h_sel = h->h_sel;
  std::memcpy(p.hcol2k, h->hcol2k, sizeof(p.hcol2k));
  p.pbase = h->pbase;
  p.out_step = -1;
  p.out_post_step = -1;
  p.z_rs = h->nz;
  p.u_rs = h->nx;
  p.dnx = h->nx;
  p.dnz = h->nz;
  p.wbuf = h->wbuf;
  p.wrows = h->wrows;
  p.a_diag = h->a_diag;
  p.lq_diag = h->lq_diag;
  p.lj_diag = h->lj_diag;
  return p;
}

// API output slots inside d_out
struct OutSlots {
  double *mean, *cov, *neff, *lse;
  int32_t* flag;
};
OutSlots out_slots(pf_handle* h) {
  OutSlots s;
  s.mean = h->d_out;
  s.cov = s.mean + (size_t)h->R * h->nx;
  s.neff = s.cov + (size_t)h->R * h->nx * h->nx;
  s.lse = s.neff + h->R;
  s.flag = (int32_t*)(s.lse + h->R);
  return s;
}
size_t out_doubles(const pf_handle* h) {
  return (size_t)h->R * h->nx + (size_t)h->R * h->nx * h->nx + 2 * (size_t)h->R + (size_t)h->R;
}

void set_outputs(StepParams& p, const OutSlots& s, bool cov_ok) {
  p.o_mean = s.mean;
  p.o_cov = cov_ok ? s.cov : nullptr;
  p.o_neff = s.neff;
  p.o_lse = s.lse;
  p.o_flag = s.flag;
}

// Many replicates: every k_step / k_cdf workgroup re-reducing all G records of its
// replicate costs O(R G^2) record reads per step; past ~2048 workgroups one k_head
// launch per step reduces them once per replicate (bitwise the same summary).
bool use_head(const pf_handle* h) {
  if (h->sharded || h->G > MAXG) return false;
  if (h->head_mode >= 0) return h->head_mode != 0;
  return h->R >= 2 && (int64_t)h->R * h->G >= 2048;
}

// k_head over the records in p.rec_in; its H workgroups also write p's outputs.
pf_status launch_head(pf_handle* h, const StepParams& p) {
  // one-shot reuse: k_cdf's heads serve the step launch that follows it when the keys match
  const bool reuse = h->head_valid && h->head_key == head_key(p);
  h->head_valid = false;
  if (reuse) return PF_OK;
  const int H = h->nx <= 4 ? 1 : std::max(1, std::min(h->G, 2 * h->nx));  // output fields per workgroup
  HIPCHK(h->ops->head(p, h->head, dim3((unsigned)H, (unsigned)h->R), base_lds_bytes(h->G), h->stream));
  return PF_OK;
}

pf_status launch_step(pf_handle* h, StepParams& p, bool writes_x, bool writes_lw, bool writes_rec) {
  p.head = nullptr;
  if (use_head(h)) {
    p.rec_in = h->rec[h->crec];
    pf_status st = launch_head(h, p);
    if (st) return st;
    p.head = h->head;
  }
  if (writes_x || writes_lw || writes_rec) state_written(h);  // the resident exit header no longer applies
  p.x_in = h->x[h->cx];
  p.x_out = h->x[h->cx ^ 1];
  p.lw_in = h->lw[h->clw];
  p.lw_out = h->lw[h->clw ^ 1];
  p.rec_in = h->rec[h->crec];
  p.rec_out = h->rec[h->crec ^ 1];
  const bool use_lcum = h->lcum_mode && !h->sharded && h->method == 0;
  p.lcum_in = (use_lcum && h->lcum_valid && p.allow_gather) ? h->lcum[h->clcum] : nullptr;
  p.lcum_out = (use_lcum && p.do_update) ? h->lcum[h->clcum ^ 1] : nullptr;
  // the fused many-replicate fp32 scalar step: the persistent kernel (its paths need the heads, the
  // systematic method, <= 2 chunks of 4 per thread and the state in the record)
  const bool stream = h->stream_mode && h->ops->stream && p.head && p.do_predict && p.do_update == 1 &&
                      p.method == 0 && h->tile <= 2048 && h->tile >= STREAM_MIN_TILE && h->R <= 1024 && !p.use_lse_ext &&
                      !p.xr_out && !p.anc_out;
  if (p.do_predict && p.do_update == 1) h->last_stream = stream;
  if (stream) {  // LDS: k_step's gather layout + the replicates' decisions (R ints after the ancestors)
    const size_t smem = base_lds_bytes(h->G) + (size_t)h->tile * (sizeof(double) + sizeof(int)) +
                        (((size_t)h->R * sizeof(int) + 15) & ~(size_t)15);
    HIPCHK(h->ops->stream(p, h->R, std::max(smem, step_lds(h, true)), h->stream));
  } else {
    dim3 grid((unsigned)h->G, (unsigned)h->R);
    HIPCHK(h->ops->step(p, grid, step_lds(h, p.allow_gather != 0), h->stream));
  }
  if (p.lcum_out) h->clcum ^= 1;
  // the prefix describes exactly the weights an update launch wrote
  if (writes_lw || p.allow_gather) h->lcum_valid = p.lcum_out != nullptr;
  h->head_valid = false;  // the heads describe records this launch may have replaced
  if (writes_x) h->cx ^= 1;
  if (writes_lw) h->clw ^= 1;
  if (writes_rec) h->crec ^= 1;
  return PF_OK;
}

pf_status launch_cdf(pf_handle* h, StepParams p) {
  p.rec_in = h->rec[h->crec];
  p.lw_in = h->lw[h->clw];
  p.head = nullptr;
  if (use_head(h)) {
    // k_cdf's own view is "resampling allowed": a step launch that allows it too reads the
    // same heads (launch_head reuses them when its key is equal); otherwise no outputs here
    StepParams q = p;
    if (!q.allow_gather) {
      q.allow_gather = 1;
      q.out_step = -1;
      q.out_post_step = -1;
    }
    pf_status st = launch_head(h, q);
    if (st) return st;
    p.head = h->head;
  }
  dim3 grid((unsigned)h->G, (unsigned)h->R);
  HIPCHK(h->ops->cdf(p, h->cdf, grid, base_lds_bytes(h->G) + (size_t)h->tile * sizeof(double), h->stream));
  if (p.head) {  // the next launch_step may read these heads (launch_head checks the key)
    StepParams q = p;
    if (!q.allow_gather) {
      q.allow_gather = 1;
      q.out_step = -1;
      q.out_post_step = -1;
    }
    h->head_valid = true;
    h->head_key = head_key(q);
  }
  return PF_OK;
}

pf_status launch_finalize(pf_handle* h, StepParams p) {
  p.rec_in = h->rec[h->crec];
  HIPCHK(h->ops->finalize(p, h->R, h->stream));
  return PF_OK;
}

pf_status upload_real(pf_handle* h, void* dst, const double* src, size_t n) {
  std::vector<char> buf;
  to_real<double>(src, n, buf, h->esz);
  HIPCHK(hipMemcpyAsync(dst, buf.data(), n * h->esz, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));  // buf is pageable & local
  return PF_OK;
}

pf_status ensure_replay(pf_handle* h, double** buf, size_t n) {
  if (!*buf) HIPCHK(hipMalloc((void**)buf, n * sizeof(double)));
  return PF_OK;
}

// Apply a resample decided by the last update (gather-only launch) + finalize aux stats.
pf_status apply_pending(pf_handle* h, const double* uniforms, const double* jitter, bool want_stats,
                        bool force = false) {
  StepParams p = base_params(h);
  p.force_gather = force;
  const size_t nrep = (size_t)h->R * h->N;
  if (uniforms) {
    const size_t n = h->method == 0 ? (size_t)h->R : nrep;
    pf_status st = ensure_replay(h, &h->d_unif, nrep > (size_t)h->R ? nrep : (size_t)h->R);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(h->d_unif, uniforms, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
    p.rp_unif = h->d_unif;
  }
  if (jitter && h->regularize) {
    pf_status st = ensure_replay(h, &h->d_replay_b, nrep * h->nx);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(h->d_replay_b, jitter, nrep * h->nx * sizeof(double), hipMemcpyHostToDevice,
                          h->stream));
    p.rp_jit = h->d_replay_b;
  }
  p.cdf = h->cdf;
  p.allow_gather = 1;
  p.ep_resample = h->ep_res;
  if (h->cdf_needed()) {
    pf_status st = launch_cdf(h, p);
    if (st) return st;
  }
  pf_status st = launch_step(h, p, true, false, true);
  if (st) return st;
  h->pending = false;
  if (want_stats) {
    StepParams f = base_params(h);
    set_outputs(f, out_slots(h), h->nx <= 4);
    f.out_post_step = 0;
    st = launch_finalize(h, f);
    if (st) return st;
  }
  if (uniforms || jitter) HIPCHK(hipStreamSynchronize(h->stream));
  return PF_OK;
}

// ---------------------------------------------------------------------------
// Device-loop covariance for nx > 4 (pf_cov.h).  Buffers and geometry once per handle: blocks of
// 4 waves over ~2048 waves per launch (or one block per replicate and block pair for nx > 48).
// ---------------------------------------------------------------------------
pf_status ensure_cov(pf_handle* h) {
  if (h->cov_ready) return PF_OK;
  // The compiled register-state kernels write post-resample ancestors / rows only in k_step_grp;
  // a compiled nx > 4 shape on plain k_step would leave anc / xr unwritten.
  if (!h->ops->grp && !h->ops->dyn)
    return fail(PF_E_UNSUPPORTED, "device-loop covariance: the step kernel writes no post-resample rows");
  CovParams c = h->covp;
  c.N = h->N;
  c.Npad = h->Npad;
  c.nx = h->nx;
  c.nb = (h->nx + 15) / 16;
  c.npairs = c.nb * (c.nb + 1) / 2;
  if (c.nb > 3 && c.npairs > 65535) return fail(PF_E_UNSUPPORTED, "device-loop covariance: nx too large");
  c.P = c.npairs * 256 + c.nb * 16 + 1;
  c.cpb = cov_chunks_per_block(h->N, h->R);
  if (const char* e = std::getenv("PF_COV_CPB")) c.cpb = std::max(1, std::min(COV_CPB_MAX, std::atoi(e)));  // experiments
  c.nblk = (int)((h->N + (int64_t)COV_BLK * c.cpb - 1) / ((int64_t)COV_BLK * c.cpb));
  c.diag = std::getenv("PF_COV_DIAG") ? std::atoi(std::getenv("PF_COV_DIAG")) : 0;
  const size_t slot = (size_t)h->R * c.nblk * c.P * sizeof(double);
  const int tc = (int)std::max<size_t>(1, std::min<size_t>(32, ((size_t)256 << 20) / slot));  // <= 256 MiB of ring
  // allocate into locals; the handle takes them only when every allocation succeeded
  void* xr = nullptr;
  int32_t* anc = nullptr;
  void* part = nullptr;
  double* tot = nullptr;
  hipError_t e = h->regularize ? hipMalloc(&xr, (size_t)h->R * h->nx * h->Npad * h->esz)
                               : hipMalloc((void**)&anc, (size_t)h->R * h->N * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&part, (size_t)tc * slot);
  if (e == hipSuccess) e = hipMalloc((void**)&tot, (size_t)tc * h->R * c.P * sizeof(double));
  if (e != hipSuccess) {
    (void)hipGetLastError();
    for (void* q : {xr, (void*)anc, part, (void*)tot})
      if (q) (void)hipFree(q);
    return fail(PF_E_HIP, std::string("device-loop covariance buffers: ") + hipGetErrorString(e));
  }
  // dynamic LDS above 64 KiB (fp64 rows, nb = 3): a per-device attribute, set on this handle's device
  for (auto [fn, lds] : {std::pair<const void*, size_t>{(const void*)k_cov_part<double, 3>, cov_part_lds<double, 3>()},
                         {(const void*)k_cov_part<double, 2>, cov_part_lds<double, 2>()},
                         {(const void*)k_cov_part<double, 0>, cov_part_lds<double, 0>()}})
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  h->covp = c;
  h->xr = xr;
  h->anc = anc;
  h->cov_part = part;
  h->cov_tot = tot;
  h->cov_tc = tc;
  h->cov_pending = 0;
  h->cov_ready = true;
  return PF_OK;
}

template <typename Real, int NB>
void launch_cov_part(dim3 grid, const CovParams& c, hipStream_t s) {
  const size_t lds = cov_part_lds<Real, NB>();
  lds_poison_hook(s);  // tests only (pf_hooks.h)
  hipLaunchKernelGGL((k_cov_part<Real, NB>), grid, dim3(256), lds, s, c);
}

// The pending chunk of the ring -> d_covs[s0 .. s0 + pending)
pf_status flush_cov(pf_handle* h, double* d_covs) {
  if (h->cov_pending == 0) return PF_OK;
  const CovParams& c = h->covp;
  CovFin f;
  f.part = h->cov_part;
  f.part_f32 = 0;
  f.tot = h->cov_tot;
  f.cov = d_covs + h->cov_s0 * h->R * h->nx * h->nx;
  f.R = h->R;
  f.nblk = c.nblk;
  f.P = c.P;
  f.nx = h->nx;
  f.nb = c.nb;
  f.npairs = c.npairs;
  const unsigned nr = (unsigned)(h->cov_pending * h->R);
  if (f.part_f32) hipLaunchKernelGGL(k_cov_fin_sum<float>, dim3((unsigned)((c.P + 255) / 256), nr), dim3(256), 0, h->stream, f);
  else hipLaunchKernelGGL(k_cov_fin_sum<double>, dim3((unsigned)((c.P + 255) / 256), nr), dim3(256), 0, h->stream, f);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_cov_fin_out, dim3((unsigned)((h->nx * h->nx + 255) / 256), nr), dim3(256), 0, h->stream, f);
  HIPCHK(hipGetLastError());
  h->cov_pending = 0;
  return PF_OK;
}

// Covariance of step s (its predicted rows xs / log-weights lw; the post-resample rows in h->xr,
// written by the gather that followed) from the step's outputs (flag, lse, mean): its block
// partials into the ring; d_covs[s] when the chunk is flushed (full, or the end of the run).
pf_status launch_cov(pf_handle* h, const void* xs, const void* lw, int64_t s, const double* d_means,
                     const int32_t* d_flags, const double* d_lse, double* d_covs) {
  CovParams c = h->covp;
  const int R = h->R;
  if (h->cov_pending == 0) h->cov_s0 = s;
  if (s != h->cov_s0 + h->cov_pending) return fail(PF_E_ARG, "device-loop covariance: steps out of order");
  c.part = (double*)h->cov_part + (size_t)h->cov_pending * R * c.nblk * c.P;
  c.xs = xs;
  c.xr = h->xr;
  c.anc = h->anc;
  c.lw = lw;
  c.flag = d_flags + s * R;
  c.lse = d_lse + s * R;
  c.mean = d_means + s * R * h->nx;
  const bool f32 = h->esz == 4;
  if (c.nb <= 3) {
    const dim3 grid((unsigned)c.nblk, (unsigned)R);
    if (f32) {
      if (c.nb == 1) launch_cov_part<float, 1>(grid, c, h->stream);
      else if (c.nb == 2) launch_cov_part<float, 2>(grid, c, h->stream);
      else launch_cov_part<float, 3>(grid, c, h->stream);
    } else {
      if (c.nb == 1) launch_cov_part<double, 1>(grid, c, h->stream);
      else if (c.nb == 2) launch_cov_part<double, 2>(grid, c, h->stream);
      else launch_cov_part<double, 3>(grid, c, h->stream);
    }
  } else {
    const dim3 grid((unsigned)c.nblk, (unsigned)R, (unsigned)c.npairs);
    if (f32) launch_cov_part<float, 0>(grid, c, h->stream);
    else launch_cov_part<double, 0>(grid, c, h->stream);
  }
  HIPCHK(hipGetLastError());
  if (++h->cov_pending == h->cov_tc) return flush_cov(h, d_covs);
  return PF_OK;
}

// ---------------------------------------------------------------------------
// Sync words of the resident and persistent launches (h->rsync): the resident granule ring and
// hand-off flags, the timeout word, the arrival count (ResParams::arrive / PersistParams::arrive) and
// the resident entry headers.  Allocated on first use; tags and flag values grow from launch to
// launch (ResParams::tag0 / flag0), so the words are zeroed only when allocated or when the 32-bit
// tag space would wrap (rsync_fits false -> rsync_reset).
// k_resident's arrival shards: after the entry headers, 4 KiB aligned, RSHARD_WORDS apart
size_t rsync_shard_offset(const pf_handle* h) {
  const size_t gran_n = RCOPIES * gran_copy_stride(h->R), flag_n = (size_t)h->R * RMAXG;
  return (gran_n + 2 * flag_n + 4 + 4 * (size_t)h->R + RSHARD_WORDS - 1) / RSHARD_WORDS * RSHARD_WORDS;
}
size_t rsync_bytes_needed(const pf_handle* h) {
  return (rsync_shard_offset(h) + (size_t)RSHARDS * RSHARD_WORDS) * sizeof(unsigned long long);
}
bool rsync_fits(const pf_handle* h, int64_t T) {
  const uint64_t tag_span = 4 * (uint64_t)T + 16;
  return h->rsync && h->rsync_bytes >= rsync_bytes_needed(h) && (uint64_t)h->res_tag + tag_span < 0xFFFFFFFFull;
}
pf_status rsync_reset(pf_handle* h) {
  const size_t bytes = rsync_bytes_needed(h);
  if (h->rsync_bytes < bytes) {
    if (h->rsync) HIPCHK(hipFree(h->rsync));
    h->rsync = nullptr;
    h->rsync_bytes = 0;
    HIPCHK(hipMalloc((void**)&h->rsync, bytes));
    h->rsync_bytes = bytes;
  }
  const size_t gran_n = RCOPIES * gran_copy_stride(h->R), flag_n = (size_t)h->R * RMAXG;
  const size_t arr_off = gran_n + 2 * flag_n + 2;
  HIPCHK(hipMemsetAsync(h->rsync, 0, h->rsync_bytes, h->stream));
  HIPCHK(hipMemsetAsync(h->rsync + arr_off + 1, 0xff, sizeof(unsigned long long), h->stream));
  h->res_tag = 0;
  h->res_flag = 0;
  h->res_arrive = 0;
  for (unsigned long long& c : h->res_shard) c = 0;
  h->res_seq = 0;
  h->res_hdr = 0;
  return PF_OK;
}

// ---------------------------------------------------------------------------
// Register-resident whole-run path (pf_resident.h).  Used by pf_run_device when
// the model has a resident kernel (scalar fp32), systematic resampling, the
// default k_step geometry and a grid that fits co-resident on the device;
// otherwise *used stays false and the caller runs the launch-per-step loop.
// PF_RESIDENT=0 disables it (A/B comparisons).
// ---------------------------------------------------------------------------
pf_status run_resident(pf_handle* h, const void* dZ, const void* dU, int64_t T, int32_t fo, double* dm,
                       double* dc, double* dn, int32_t* df, double* dl, bool* used) {
  *used = false;
  const char* env = std::getenv("PF_RESIDENT");
  if (env && std::atoi(env) == 0) return PF_OK;
  if (!h->ops->resident || h->method != 0 || h->sharded || !(h->tile == 1024 || h->N <= 1024) || T <= 0) return PF_OK;
  const int G = (int)((h->N + RTILE - 1) / RTILE);
  if (G > RMAXG || T > (int64_t)0x3fffffff) return PF_OK;
  const size_t gran_n = RCOPIES * gran_copy_stride(h->R), flag_n = (size_t)h->R * RMAXG;
  const size_t hdr_off = gran_n + 2 * flag_n + 4;  // entry headers [R][4]
  const size_t arr_off = gran_n + 2 * flag_n + 2;  // arrival count, first aborted launch
  const bool zero = !rsync_fits(h, T);
  if (h->pending) {  // a decision taken before this run is applied first (gather-only launch)
    pf_status st = apply_pending(h, nullptr, nullptr, false);
    if (st) return st;
  }
  if (zero) {
    pf_status st = rsync_reset(h);
    if (st) return st;
  }
  if (!h->hdr_restore.empty()) {  // a restored checkpoint's entry header, under a fresh id
    const unsigned long long id = ++h->res_run;
    for (int r = 0; r < h->R; ++r) h->hdr_restore[4 * (size_t)r] = id;
    HIPCHK(hipMemcpyAsync(h->rsync + hdr_off, h->hdr_restore.data(), h->hdr_restore.size() * sizeof(unsigned long long),
                          hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));  // pageable source
    h->res_hdr = id;
    h->hdr_restore.clear();
  }
  if (!h->res_unchecked) h->res_undo.clear();
  h->res_undo.push_back({h->res_seq + 1, h->epoch, h->ep_res, h->crec, h->cx, h->clw, h->res_hdr});
  ResParams q;
  std::memset(&q, 0, sizeof(q));
  q.x_in = (const float*)h->x[h->cx];
  q.lw_in = (const float*)h->lw[h->clw];
  q.rec_in = h->rec[h->crec];
  q.x_fin = (float*)h->x[h->cx];    // in place: every thread rewrites only its own slots
  q.lw_fin = (float*)h->lw[h->clw];
  q.rec_fin = h->rec[h->crec ^ 1];
  q.xg = (float*)h->x[h->cx ^ 1];
  q.lg = (float*)h->lw[h->clw ^ 1];
  q.gran = h->rsync;
  q.sflag = h->rsync + gran_n;
  q.err = (unsigned int*)(h->rsync + gran_n + 2 * flag_n);
  q.tag0 = h->res_tag;
  q.flag0 = h->res_flag;
  q.P = h->P;
  q.z = (const float*)dZ;
  q.u = (const float*)dU;
  q.o_mean = dm;
  q.o_cov = dc;
  q.o_neff = dn;
  q.o_lse = dl;
  q.o_flag = df;
  q.N = h->N;
  q.Npad = h->Npad;
  q.T = T;
  q.G = G;
  q.Gk = h->G;
  q.tile_k = h->tile;
  q.seed = h->seed;
  q.ep0 = h->epoch;
  q.first_update_only = fo ? 1 : 0;
  q.thresh = h->thresh;
  q.regularize = h->regularize;
  q.r_diag = h->r_diag;
  q.rep_base = h->rep_base;
  q.Rtot = h->R;
  q.hdr = h->rsync + hdr_off;
  const char* hdr_env = std::getenv("PF_RES_HDR");  // PF_RES_HDR=0: always the records' prologue (tests)
  q.hdr_in = (hdr_env && std::atoi(hdr_env) == 0) ? 0ull : h->res_hdr;
  q.hdr_out = ++h->res_run;
  q.tr_x = h->tr_x;
  q.tr_l = h->tr_l;
  q.tr_anc = h->tr_anc;
  q.tr_T = h->tr_T;
  // Replicates are independent filters: when all R do not fit co-resident, groups of as many
  // as fit run one after another (each replicate computes exactly what it computes alone, so
  // the path - and every replicate's result - does not depend on R or on the sharding).
  // with a verification trace set, the trace instance's occupancy sizes the groups (it may fit fewer
  // workgroups than the plain instance; a group sized for the plain one would not launch resident)
  const int cap = h->ops->resident_cap ? h->ops->resident_cap(h->tr_x != nullptr) : 0;
  const int Rg = cap >= G ? std::max(1, std::min(h->R, cap / G)) : h->R;
  // Launch mode: one plain launch that checks its own co-residency (ResParams::arrive; ~17 us
  // cheaper than a cooperative launch), or cooperative launches when the run needs several
  // replicate groups (an abort must leave every replicate's state untouched), after an abort
  // on this handle, or with PF_COOP=1.
  const char* coop_env = std::getenv("PF_COOP");
  const bool coop = (coop_env && std::atoi(coop_env) == 1) || h->res_force_coop || Rg < h->R;
  q.test_abort = (test_hook("PF_TEST_ABORT") && !coop) ? 1 : 0;  // test hook (pf_hooks.h)
  // Resident launches of different handles (streams) on one device never overlap: two grids that
  // each hold part of the CUs would wait for each other's missing workgroups.
  GridOrderScope order(h->device, h->stream);
  // timing: the start event is a marker queued right before the launch, the stop event is stamped
  // by the plain launch's own dispatch (hipExtLaunchKernel): the interval covers the kernel and
  // nothing queued after it, and the run's wall time stays that of two markers (a dispatch-stamped
  // start costs ~3 us of host time before the launch; profiles/r04/ab/README.md).  Cooperative
  // launches keep both markers.  PF_EXT_EVENTS (A/B): 0 markers, 1 both stamped by the dispatch,
  // 2 start only, 3 stop only (default)
  const char* xe_env = std::getenv("PF_EXT_EVENTS");
  const int xe = xe_env ? std::atoi(xe_env) : 3;
  const bool ext0 = h->timing && !coop && (xe == 1 || xe == 2), ext1 = h->timing && !coop && (xe == 1 || xe == 3);
  if (h->timing && !ext0) HIPCHK(hipEventRecord(h->tev[0], h->stream));
  for (int r0 = 0; r0 < h->R; r0 += Rg) {
    q.r0 = r0;
    q.arrive = h->rsync + arr_off;
    q.arrive0 = h->res_arrive;
    q.seq = ++h->res_seq;
    const unsigned nwg = (unsigned)G * (unsigned)std::min(Rg, h->R - r0);
    q.nshard = (int)std::min<unsigned>(RSHARDS, nwg);
    q.arrive_sh = h->rsync + rsync_shard_offset(h);
    for (int k = 0; k < RSHARDS; ++k) q.shard_base[k] = h->res_shard[k];
    const hipError_t e = h->ops->resident(q, G, std::min(Rg, h->R - r0), h->stream, coop,
                                          (ext0 && r0 == 0) ? h->tev[0] : nullptr,
                                          (ext1 && r0 + Rg >= h->R) ? h->tev[1] : nullptr);
    if (e == hipSuccess) {  // the shards count every workgroup, arrive[0] every shard (an aborted launch too)
      h->res_arrive += (unsigned long long)q.nshard;
      for (int k = 0; k < q.nshard; ++k) h->res_shard[k] += (nwg - (unsigned)k + (unsigned)q.nshard - 1) / (unsigned)q.nshard;
    }
    if (e == hipErrorCooperativeLaunchTooLarge && r0 == 0) {
      (void)hipGetLastError();
      return PF_OK;  // not co-resident here: launch-per-step path
    }
    if (e != hipSuccess) return fail(PF_E_HIP, std::string("k_resident launch: ") + hipGetErrorString(e));
  }
  if (h->timing && !ext1) HIPCHK(hipEventRecord(h->tev[1], h->stream));
  order.end();
  h->res_hdr = q.hdr_out;  // the state is now what this run's exit header describes
  h->res_tag += (uint32_t)(4 * (uint64_t)T + 16);  // the tag span rsync_fits reserves
  h->res_flag += (unsigned long long)T + 1;
  const int k = fo ? 1 : 0;
  h->epoch = q.ep0 + (uint32_t)(2 * T) - k;
  h->ep_res = h->epoch - 1;
  h->pending = false;
  h->crec ^= 1;
  h->res_unchecked = true;
  h->resident_runs++;
  h->last_resident = true;
  *used = true;
  return PF_OK;
}

// ---------------------------------------------------------------------------
// Persistent fp64 whole-run path (pf_persist.h): the launch-per-step loop below, bit for bit, in
// one launch (its T fused steps, the tail and the finalize), for the scalar fp64 models with
// systematic resampling, per-workgroup prologues (no k_head), unsharded state and a grid that fits
// co-resident.  Opt-in (PF_PERSIST=1): at N = 1e6 it measured 25.0 us per step against 23.1 for the
// launch-per-step loop (same box, profiles/r06/persist): the step is bound by the fp64 Box-Muller /
// weight chains at 2 waves per SIMD, not by the launch boundary it removes.
// ---------------------------------------------------------------------------
pf_status run_persist(pf_handle* h, const void* dZ, const void* dU, int64_t T, int32_t fo, double* dm, double* dc,
                      double* dn, int32_t* df, double* dl, bool* used) {
  *used = false;
  const char* env = std::getenv("PF_PERSIST");
  if (!(env && std::atoi(env) == 1)) return PF_OK;
  if (!h->ops->persist || h->res_force_coop || h->method != 0 || h->sharded || use_head(h) || h->lcum_mode || T <= 0 ||
      T > (int64_t)0x3fffffff || h->tile > 2 * PBS * 4 || h->G > PMAXG)
    return PF_OK;
  const int G = h->G, R = h->R;
  const size_t smem = persist_lds_bytes(G, h->tile);
  if (smem > 160 * 1024) return PF_OK;
  const int cap = h->ops->persist_cap ? h->ops->persist_cap(smem) : 0;
  if ((long long)G * R > (long long)cap) return PF_OK;
  // the arrival count and timeout word (shared with the resident path), the granule ring and flags
  if (!rsync_fits(h, T)) {
    pf_status st = rsync_reset(h);
    if (st) return st;
  }
  const size_t pw = persist_sync_words(R, G);
  bool zero = (uint64_t)h->pers_tag + (uint64_t)T + 2 >= 0xFFFFFFFFull;
  if (h->psync_words < pw) {
    if (h->psync) HIPCHK(hipFree(h->psync));
    h->psync = nullptr;
    h->psync_words = 0;
    HIPCHK(hipMalloc((void**)&h->psync, pw * sizeof(unsigned long long)));
    h->psync_words = pw;
    zero = true;
  }
  if (zero) {
    HIPCHK(hipMemsetAsync(h->psync, 0, h->psync_words * sizeof(unsigned long long), h->stream));
    h->pers_tag = 0;
  }
  const size_t gran_n = RCOPIES * gran_copy_stride(R), flag_n = (size_t)R * RMAXG;
  const size_t arr_off = gran_n + 2 * flag_n + 2;
  if (!h->res_unchecked) h->res_undo.clear();
  h->res_undo.push_back({h->res_seq + 1, h->epoch, h->ep_res, h->crec, h->cx, h->clw, h->res_hdr});
  state_written(h);
  PersistParams q;
  std::memset(&q, 0, sizeof(q));
  q.p = base_params(h);
  q.p.o_mean = dm;
  q.p.o_cov = dc;
  q.p.o_neff = dn;
  q.p.o_lse = dl;
  q.p.o_flag = df;
  for (int k = 0; k < 2; ++k) {
    q.X[k] = h->x[k];
    q.L[k] = h->lw[k];
    q.RB[k] = h->rec[k];
  }
  q.cx = h->cx;
  q.cl = h->clw;
  q.cr = h->crec;
  q.z = dZ;
  q.u = dU;
  q.T = T;
  q.fo = fo ? 1 : 0;
  q.pending = h->pending ? 1 : 0;
  q.ep0 = h->epoch;
  q.ep_res0 = h->ep_res;
  q.gran = h->psync;
  q.dflag = h->psync + persist_gran_words(R, G);
  q.tag0 = h->pers_tag;
  q.arrive = h->rsync + arr_off;
  q.arrive0 = h->res_arrive;
  q.seq = ++h->res_seq;
  q.err = (unsigned int*)(h->rsync + gran_n + 2 * flag_n);
  GridOrderScope order(h->device, h->stream);
  if (h->timing) HIPCHK(hipEventRecord(h->tev[0], h->stream));  // stop: stamped by the launch's dispatch
  const hipError_t e = h->ops->persist(q, G, R, smem, h->stream, h->timing ? h->tev[1] : nullptr);
  if (e == hipErrorCooperativeLaunchTooLarge) {
    (void)hipGetLastError();
    h->res_undo.pop_back();
    --h->res_seq;
    return PF_OK;  // launch-per-step path
  }
  if (e != hipSuccess) return fail(PF_E_HIP, std::string("k_persist launch: ") + hipGetErrorString(e));
  order.end();
  h->res_arrive += (unsigned long long)G * R;
  h->pers_tag += (uint32_t)T + 2;
  // the buffers the launch-per-step loop would leave current: x flips on every step that predicts or
  // may gather (and in the tail), the log-weights on every update, the records on every launch
  const int xflips = (int)((T - ((fo && !h->pending) ? 1 : 0) + 1) & 1);
  h->cx ^= xflips;
  h->clw ^= (int)(T & 1);
  h->crec ^= (int)((T + 1) & 1);
  const int k = fo ? 1 : 0;
  h->epoch = q.ep0 + (uint32_t)(2 * T) - k;
  h->ep_res = h->epoch - 1;
  h->pending = false;
  h->lcum_valid = false;
  h->head_valid = false;
  h->res_unchecked = true;
  h->persist_runs++;
  h->last_persist = true;
  *used = true;
  return PF_OK;
}

// After a stream sync: a resident launch that timed out in a hand-off is an error.
pf_status check_resident(pf_handle* h) {
  if (!h->res_unchecked) return PF_OK;
  h->res_unchecked = false;
  const size_t gran_n = RCOPIES * gran_copy_stride(h->R), flag_n = (size_t)h->R * RMAXG;
  unsigned int err = 0;
  HIPCHK(hipMemcpy(&err, (const void*)(h->rsync + gran_n + 2 * flag_n), sizeof(err), hipMemcpyDeviceToHost));
  if (!err) return PF_OK;
  HIPCHK(hipMemset((void*)(h->rsync + gran_n + 2 * flag_n), 0, sizeof(err)));
  if (err == 16u) {
    // A plain launch did not get its whole grid resident (other work held CUs): every
    // workgroup left before touching any state, and so did every launch after it.  Undo the
    // bookkeeping to that launch's entry, launch cooperatively from now on, and report it
    // (pf_run repeats the run itself).
    const size_t arr_off = gran_n + 2 * flag_n + 2;
    unsigned long long aw[2] = {0, 0};
    HIPCHK(hipMemcpy(aw, (const void*)(h->rsync + arr_off), sizeof(aw), hipMemcpyDeviceToHost));
    HIPCHK(hipMemset((void*)(h->rsync + arr_off + 1), 0xff, sizeof(unsigned long long)));
    h->res_arrive = aw[0];
    // k_resident's arrival shards carry the abort's marks and every arrival of the aborted launches:
    // the next launch's bases are their values now
    for (int k = 0; k < RSHARDS; ++k)
      HIPCHK(hipMemcpy(&h->res_shard[k], (const void*)(h->rsync + rsync_shard_offset(h) + (size_t)k * RSHARD_WORDS),
                       sizeof(unsigned long long), hipMemcpyDeviceToHost));
    const auto u = std::find_if(h->res_undo.begin(), h->res_undo.end(),
                                [&](const pf_handle::ResUndo& x) { return x.seq == aw[1]; });
    if (u == h->res_undo.end()) {
      h->initialized = false;
      return fail(PF_E_HIP, "k_resident: aborted launch not found; call initialize() again");
    }
    h->epoch = u->epoch;
    h->ep_res = u->ep_res;
    h->crec = u->crec;
    h->cx = u->cx;
    h->clw = u->clw;
    h->res_hdr = u->hdr;
    h->res_undo.clear();
    h->res_force_coop = true;  // resident runs launch cooperatively, persistent ones not at all
    h->last_resident = false;
    h->last_persist = false;
    return fail(PF_E_RETRY, "k_resident / k_persist: the grid was not co-resident (other work on the GPU); nothing was "
                            "computed, the state is unchanged and the next run launches cooperatively");
  }
  // The launch wrote its particles and records in place: the state is unusable.  Poison
  // the handle (the next call reports "not initialized").
  h->initialized = false;
  if (err & 8u)
    return fail(PF_E_NAN, "every particle weight is zero or NaN (all-dead filter); call initialize() again");
  return fail(PF_E_HIP, "k_resident: inter-workgroup hand-off timed out (code " + std::to_string(err) +
                            "); call initialize() again");
}

// Entry of every host API that reads or writes the state: an asynchronous resident run
// (pf_run_device) not yet checked is waited for and checked first, so nothing acts on a
// state an aborted launch never produced (PF_E_RETRY then reaches this caller).
pf_status settle(pf_handle* h) {
  if (!h->res_unchecked) return PF_OK;
  HIPCHK(hipStreamSynchronize(h->stream));
  return check_resident(h);
}

// Every particle weight of some replicate is zero or NaN.  The update that found it has already
// advanced the state and the Philox epochs, so the handle is poisoned: the next call reports
// "not initialized" instead of continuing silently from a half-applied step.
pf_status dead_filter(pf_handle* h, const std::string& where) {
  h->initialized = false;
  h->pending = false;
  return fail(PF_E_NAN, "every particle weight is zero or NaN " + where +
                            ": the filter is dead; call initialize() again");
}

}  // namespace

namespace pf {

// ---------------------------------------------------------------------------
// Uninitialised-LDS test hook (pf_hooks.h): k_lds_poison fills a workgroup's whole LDS allocation
// (160 KB: one workgroup per CU at a time) with 0xFFFFFFFF; 4 workgroups per CU visit every CU.
// k_lds_probe (test of the mechanism) counts, per workgroup, the words of its uninitialised LDS
// that do not hold the pattern.
// ---------------------------------------------------------------------------
constexpr int PF_LDS_CU_BYTES = 160 * 1024;
constexpr unsigned PF_LDS_POISON = 0xFFFFFFFFu;

__global__ void __launch_bounds__(1024) k_lds_poison(unsigned pattern) {
  extern __shared__ unsigned lds_all[];
  volatile unsigned* v = lds_all;  // volatile: the stores are the kernel's only effect
  for (int i = threadIdx.x; i < PF_LDS_CU_BYTES / 4; i += blockDim.x) v[i] = pattern;
}

__global__ void __launch_bounds__(1024) k_lds_probe(unsigned pattern, int32_t* out) {
  extern __shared__ unsigned lds_all[];
  __shared__ int bad;
  volatile unsigned* v = lds_all;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  int mine = 0;
  for (int i = threadIdx.x; i < PF_LDS_CU_BYTES / 4 - 64; i += blockDim.x) mine += v[i] != pattern;
  atomicAdd(&bad, mine);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = bad;
}

static int lds_poison_blocks() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return 4 * (cus > 0 ? cus : 256);
}

static long long g_lds_poison_count = 0;
void lds_poison_count_add() { ++g_lds_poison_count; }

void lds_poison(hipStream_t s) {
  (void)hipFuncSetAttribute((const void*)k_lds_poison, hipFuncAttributeMaxDynamicSharedMemorySize, PF_LDS_CU_BYTES);
  hipLaunchKernelGGL(k_lds_poison, dim3(lds_poison_blocks()), dim3(1024), PF_LDS_CU_BYTES, s, PF_LDS_POISON);
}

}  // namespace pf

extern "C" {

const char* pf_last_error(void) { return g_err.c_str(); }
const char* pf_version(void) { return "particle_filters_amd 0.1 (gfx950)"; }

int32_t pf_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int32_t pf_model_supported(int32_t nx, int32_t nz, int32_t tk, int32_t ok) {
  return find_ops(nx, nz, tk, ok, PF_PRECISION_FP32) != nullptr || find_ops_dyn(nx, nz, tk, ok, PF_PRECISION_FP32) != nullptr;
}

int32_t pf_model_compiled(int32_t nx, int32_t nz, int32_t tk, int32_t ok) {
  return find_ops(nx, nz, tk, ok, PF_PRECISION_FP32) != nullptr;
}

int32_t pf_kernel_path(pf_handle* h) { return (h && h->ops && h->ops->dyn) ? PF_PATH_RUNTIME : PF_PATH_AUTO; }
int32_t pf_last_step_streamed(pf_handle* h) { return (h && h->last_stream) ? 1 : 0; }

pf_status pf_create(const pf_model_desc* m, const pf_opts* o, pf_handle** out) {
  if (!m || !o || !out) return fail(PF_E_ARG, "null argument");
  *out = nullptr;
  if (m->nx <= 0 || m->nz <= 0) return fail(PF_E_ARG, "nx and nz must be positive");
  if (o->n_particles <= 0) return fail(PF_E_ARG, "n_particles must be positive");
  if (o->n_replicates <= 0) return fail(PF_E_ARG, "n_replicates must be positive");
  if (o->precision != PF_PRECISION_FP32 && o->precision != PF_PRECISION_FP64)
    return fail(PF_E_ARG, "precision must be PF_PRECISION_FP32 or PF_PRECISION_FP64");
  if (o->kernel_path != PF_PATH_AUTO && o->kernel_path != PF_PATH_RUNTIME)
    return fail(PF_E_ARG, "kernel_path must be PF_PATH_AUTO or PF_PATH_RUNTIME");
  // the compiled shape's register-state kernels when there are some, else the runtime-shape ones
  const Ops* ops = o->kernel_path == PF_PATH_RUNTIME ? nullptr
                                                     : find_ops(m->nx, m->nz, m->trans_kind, m->obs_kind, o->precision);
  if (!ops) ops = find_ops_dyn(m->nx, m->nz, m->trans_kind, m->obs_kind, o->precision);
  if (!ops)
    return fail(PF_E_UNSUPPORTED, "model (nx=" + std::to_string(m->nx) + ", nz=" + std::to_string(m->nz) +
                                      ", g=" + std::to_string(m->trans_kind) + ", h=" +
                                      std::to_string(m->obs_kind) + ") does not fit its g / h kinds");
  const int nx = m->nx, nz = m->nz;
  // ---- parameters (double, host) -------------------------------------------
  std::vector<double> P((size_t)ops->psize, 0.0);
  auto lay_A = 0, lay_LQ = nx * nx, lay_LJ = 2 * nx * nx, lay_H = 3 * nx * nx, lay_C = lay_H + nz * nx,
       lay_LR = lay_C + nz, lay_EX = lay_LR + nz * nz;
  if (m->trans_kind == PF_TRANS_LINEAR) {
    if (m->n_trans_params < (int64_t)nx * nx || !m->trans_params) return fail(PF_E_ARG, "LINEAR g needs A[nx*nx]");
    for (int i = 0; i < nx * nx; ++i) P[lay_A + i] = m->trans_params[i];
  } else if (m->trans_kind == PF_TRANS_L96) {
    if (m->n_trans_params < 2 || !m->trans_params) return fail(PF_E_ARG, "L96 g needs {F, dt}");
    P[lay_EX + 0] = m->trans_params[0];
    P[lay_EX + 1] = m->trans_params[1];
  }
  if (m->obs_kind == PF_OBS_LINEAR) {
    if (m->n_obs_params < (int64_t)nz * nx + nz || !m->obs_params) return fail(PF_E_ARG, "LINEAR h needs H[nz*nx], c[nz]");
    for (int i = 0; i < nz * nx; ++i) P[lay_H + i] = m->obs_params[i];
    for (int i = 0; i < nz; ++i) P[lay_C + i] = m->obs_params[nz * nx + i];
  } else if (m->obs_kind == PF_OBS_EXP_HALF || m->obs_kind == PF_OBS_SV_EXACT) {
    if (m->n_obs_params < nz || !m->obs_params) return fail(PF_E_ARG, "EXP_HALF / SV_EXACT h needs beta[nz]");
    if (nz != nx) return fail(PF_E_ARG, "EXP_HALF / SV_EXACT h observes every state component (nz == nx)");
    for (int i = 0; i < nz; ++i) P[lay_C + i] = m->obs_params[i];
  } else if (m->obs_kind == PF_OBS_ACOUSTIC) {
    if (m->n_obs_params < 2 + 2 * nz || !m->obs_params) return fail(PF_E_ARG, "ACOUSTIC h needs psi, d0, sx[nz], sy[nz]");
    for (int i = 0; i < 2 + 2 * nz; ++i) P[lay_EX + i] = m->obs_params[i];
  } else if (m->obs_kind == PF_OBS_BEARINGS) {
    if (m->n_obs_params < 3 || !m->obs_params) return fail(PF_E_ARG, "BEARINGS h needs the sensor position s[3]");
    for (int i = 0; i < 3; ++i) P[lay_EX + 2 + i] = m->obs_params[i];
  }
  if (!m->Q || !m->R) return fail(PF_E_ARG, "Q and R are required");
  std::vector<double> L;
  // LR = chol(R + 1e-12 I)  (particle_filter.py:107)
  if (!cholesky(m->R, nz, 1e-12, L)) return fail(PF_E_NOT_PD, "Matrix is not positive definite (R)");
  int r_diag = 1;
  for (int i = 0; i < nz; ++i)
    for (int j = 0; j < nz; ++j) {
      P[lay_LR + i * nz + j] = L[i * nz + j];
      if (i != j && L[i * nz + j] != 0.0) r_diag = 0;
    }
  const int lay_ILR = lay_EX + 2 + 2 * nz;
  for (int i = 0; i < nz; ++i) P[lay_ILR + i] = 1.0 / L[i * nz + i];
  // predict: chol(Q), fallback chol(Q + 1e-10 I)  (particle_filter.py:232-235)
  bool qok = cholesky(m->Q, nx, 0.0, L) || cholesky(m->Q, nx, 1e-10, L);
  if (qok)
    for (int i = 0; i < nx * nx; ++i) P[lay_LQ + i] = L[i];
  // jitter: 0.001 * (chol(Q), fallback chol(Q + 1e-12 I))  (particle_filter.py:213-217)
  if (cholesky(m->Q, nx, 0.0, L) || cholesky(m->Q, nx, 1e-12, L))
    for (int i = 0; i < nx * nx; ++i) P[lay_LJ + i] = 0.001 * L[i];

  HIPCHK(hipSetDevice(o->device));
  pf_handle* h = new pf_handle();
  h->ops = ops;
  h->nx = nx; h->nz = nz; h->tk = m->trans_kind; h->ok = m->obs_kind; h->prec = o->precision;
  h->N = o->n_particles;
  h->Npad = (o->n_particles + 3) / 4 * 4;
  h->R = o->n_replicates;
  h->method = o->resample_method == PF_RESAMPLE_SYSTEMATIC ? 0 : 1;
  {  // large-state kernels: systematic ancestors by one binary search in the k_cdf-materialised CDF
    const char* env = std::getenv("PF_SYS_CDF");
    h->sys_cdf = (h->method == 0 && ops->grp && !(env && env[0] == '0')) ? 1 : 0;
  }
  h->thresh = o->resample_thresh;
  h->regularize = o->regularize != 0;
  h->seed = o->seed;
  h->device = o->device;
  h->rep_base = o->replicate_base;
  h->esz = o->precision == PF_PRECISION_FP64 ? 8 : 4;
  h->r_diag = r_diag;
  h->chol_q_ok = qok;
  if (nx >= 16 && nx % 4 == 0) {  // block-diagonality in the lane blocks of k_step_grp (SGrp<NX>)
    const int per = nx / ((nx >= 32 && nx % 8 == 0) ? 8 : 4);
    auto local = [&](int off) {
      for (int i = 0; i < nx; ++i)
        for (int j = 0; j < nx; ++j)
          if (i / per != j / per && P[off + i * nx + j] != 0.0) return 0;
      return 1;
    };
    // a linear g's A joins the chol(Q) test: the lane-local variant also applies A within the blocks
    h->lq_local = local(lay_LQ) && (m->trans_kind != PF_TRANS_LINEAR || local(lay_A));
    h->lj_local = local(lay_LJ);
  }
  for (int c = 0; c < 64; ++c) h->hcol2k[c] = -1;
  if (m->obs_kind == PF_OBS_LINEAR && nx <= 64 && ops->grp) {  // selection H (every row one 1.0)
    bool sel = true;
    for (int k = 0; k < nz && sel; ++k) {
      int ones = 0, col = -1;
      for (int c = 0; c < nx; ++c) {
        const double v = P[lay_H + k * nx + c];
        if (v == 1.0) { ++ones; col = c; }
        else if (v != 0.0) sel = false;
      }
      if (ones != 1 || h->hcol2k[col] != -1) sel = false;
      else h->hcol2k[col] = k;
    }
    h->h_sel = (sel && r_diag) ? 1 : 0;
    if (!h->h_sel)
      for (int c = 0; c < 64; ++c) h->hcol2k[c] = -1;
  }
  if (ops->dyn) {  // runtime-shape kernels: diagonal factors, selection H, scratch rows
    auto diag = [&](int off) {
      for (int i = 0; i < nx; ++i)
        for (int j = 0; j < nx; ++j)
          if (i != j && P[off + i * nx + j] != 0.0) return 0;
      return 1;
    };
    h->a_diag = m->trans_kind == PF_TRANS_LINEAR ? diag(lay_A) : 0;
    h->lq_diag = diag(lay_LQ);
    h->lj_diag = diag(lay_LJ);
    h->h_sel = 0;
    if (m->obs_kind == PF_OBS_LINEAR) {
      bool sel = true;
      std::vector<double> cols(nz, 0.0);
      for (int k = 0; k < nz && sel; ++k) {
        int ones = 0;
        for (int c = 0; c < nx; ++c) {
          const double v = P[lay_H + k * nx + c];
          if (v == 1.0) { ++ones; cols[k] = c; }
          else if (v != 0.0) sel = false;
        }
        if (ones != 1) sel = false;
      }
      if (sel) {
        for (int k = 0; k < nz; ++k) P[lay_EX + 2 + k] = cols[k];
        h->h_sel = 1;
      }
    }
    h->wrows = dyn_wrows(m->trans_kind, nx, nz);
  }
  h->Pd = P;
  if (!choose_geometry(h)) {
    delete h;
    return fail(PF_E_ARG, "n_particles too large for this model (max " +
                              std::to_string((long long)MAXG * ops->tile_max) + ")");
  }
  ops->prepare();
  auto cleanup = [&](pf_status st) {
    pf_destroy(h);
    return st;
  };
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(PF_E_HIP, "hipStreamCreate failed"));
  const size_t xbytes = (size_t)h->R * nx * h->Npad * h->esz;
  const size_t lwbytes = (size_t)h->R * h->Npad * h->esz;
  for (int k = 0; k < 2; ++k) {
    if (hipMalloc(&h->x[k], xbytes) != hipSuccess || hipMalloc(&h->lw[k], lwbytes) != hipSuccess ||
        hipMalloc((void**)&h->rec[k], rec_bytes(h)) != hipSuccess)
      return cleanup(fail(PF_E_HIP, "hipMalloc of particle state failed"));
    (void)hipMemset(h->x[k], 0, xbytes);
    (void)hipMemset(h->lw[k], 0, lwbytes);
  }
  if (h->needs_cdf() && hipMalloc((void**)&h->cdf, (size_t)h->R * h->N * sizeof(double)) != hipSuccess)
    return cleanup(fail(PF_E_HIP, "hipMalloc of cdf failed"));
  {
    const char* le = std::getenv("PF_LCUM");  // PF_LCUM=0: materialise the CDF with k_cdf (A/B)
    h->lcum_mode = h->sys_cdf && !(le && le[0] == '0');
  }
  if (h->lcum_mode)
    for (int k = 0; k < 2; ++k)
      if (hipMalloc((void**)&h->lcum[k], (size_t)h->R * h->N * sizeof(double)) != hipSuccess)
        return cleanup(fail(PF_E_HIP, "hipMalloc of the CDF prefix failed"));
  if (const char* he = std::getenv("PF_HEAD")) h->head_mode = std::atoi(he) != 0 ? 1 : 0;
  if (const char* se = std::getenv("PF_STREAM")) h->stream_mode = std::atoi(se) != 0 ? 1 : 0;
  if (hipMalloc((void**)&h->head, (size_t)h->R * HEAD_STRIDE * sizeof(double)) != hipSuccess)
    return cleanup(fail(PF_E_HIP, "hipMalloc of replicate heads failed"));
  if (h->wrows > 0 && hipMalloc(&h->wbuf, (size_t)h->R * h->wrows * h->Npad * h->esz) != hipSuccess)
    return cleanup(fail(PF_E_HIP, "hipMalloc of the runtime-shape scratch failed"));
  if (hipMalloc(&h->P, P.size() * h->esz) != hipSuccess || hipMalloc(&h->d_z, (size_t)h->R * nz * h->esz) != hipSuccess ||
      hipMalloc(&h->d_u, (size_t)h->R * nx * h->esz) != hipSuccess ||
      hipMalloc((void**)&h->d_out, out_doubles(h) * sizeof(double)) != hipSuccess)
    return cleanup(fail(PF_E_HIP, "hipMalloc of parameters failed"));
  if (upload_real(h, h->P, P.data(), P.size()) != PF_OK) return cleanup(PF_E_HIP);
  *out = h;
  return PF_OK;
}

void pf_destroy(pf_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->stream) grid_order_forget(h->device, h->stream);
  for (int k = 0; k < 2; ++k) {
    if (h->x[k]) (void)hipFree(h->x[k]);
    if (h->lw[k]) (void)hipFree(h->lw[k]);
    if (h->rec[k]) (void)hipFree(h->rec[k]);
  }
  if (h->rsync) (void)hipFree(h->rsync);
  if (h->psync) (void)hipFree(h->psync);
  for (hipEvent_t e : h->tev)
    if (e) (void)hipEventDestroy(e);
  if (h->head) (void)hipFree(h->head);
  for (double* q : h->lcum)
    if (q) (void)hipFree(q);
  for (void* p : {h->wbuf, (void*)h->cdf, h->P, h->d_z, h->d_u, (void*)h->d_out, (void*)h->d_replay_a,
                  (void*)h->d_replay_b, (void*)h->d_unif, h->xr, (void*)h->anc, (void*)h->cov_part, (void*)h->cov_tot,
                  (void*)h->tr_x, (void*)h->tr_l, (void*)h->tr_anc})
    if (p) (void)hipFree(p);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

pf_status pf_initialize(pf_handle* h, const double* mean, const double* cov, const double* replay) {
  if (!h || !mean || !cov) return fail(PF_E_ARG, "null argument");
  HIPCHK(hipSetDevice(h->device));
  const int nx = h->nx, R = h->R;
  // Lc = chol(cov + 1e-10 I)  (particle_filter.py:127)
  std::vector<double> Lc((size_t)R * nx * nx), L;
  for (int r = 0; r < R; ++r) {
    if (!cholesky(cov + (size_t)r * nx * nx, nx, 1e-10, L))
      return fail(PF_E_NOT_PD, "Matrix is not positive definite (initial covariance)");
    std::copy(L.begin(), L.end(), Lc.begin() + (size_t)r * nx * nx);
  }
  void *dmean = nullptr, *dL = nullptr;
  HIPCHK(hipMalloc(&dmean, (size_t)R * nx * h->esz));
  HIPCHK(hipMalloc(&dL, (size_t)R * nx * nx * h->esz));
  pf_status st = upload_real(h, dmean, mean, (size_t)R * nx);
  if (!st) st = upload_real(h, dL, Lc.data(), Lc.size());
  const double* drep = nullptr;
  if (!st && replay) {
    st = ensure_replay(h, &h->d_replay_a, (size_t)R * h->N * nx);
    if (!st && hipMemcpy(h->d_replay_a, replay, (size_t)R * h->N * nx * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
      st = fail(PF_E_HIP, "replay upload failed");
    drep = h->d_replay_a;
  }
  if (!st) {
    const uint32_t ep = h->epoch++;
    int lc_diag = 1;  // every replicate's factor diagonal: the runtime-shape init skips the zeros
    for (int r = 0; r < R && lc_diag; ++r)
      for (int i = 0; i < nx && lc_diag; ++i)
        for (int j = 0; j < i; ++j)
          if (Lc[(size_t)r * nx * nx + i * nx + j] != 0.0) { lc_diag = 0; break; }
    hipError_t e = h->ops->init(h->x[h->cx ^ 1], h->rec[h->crec ^ 1], dmean, dL, drep, h->N, h->Npad, h->G, R,
                                h->seed, ep, h->rep_base, h->pbase, h->stream, nx, lc_diag);
    if (e != hipSuccess) st = fail(PF_E_HIP, std::string("init launch: ") + hipGetErrorString(e));
    h->cx ^= 1;
    h->crec ^= 1;
  }
  (void)hipStreamSynchronize(h->stream);
  (void)hipFree(dmean);
  (void)hipFree(dL);
  if (st) return st;
  h->initialized = true;
  h->pending = false;
  h->lcum_valid = false;
  state_written(h);
  return PF_OK;
}

pf_status pf_predict(pf_handle* h, const double* u, const double* replay) {
  if (!h) return fail(PF_E_ARG, "null handle");
  {
    const pf_status s0 = settle(h);
    if (s0) return s0;
  }
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  if (!h->chol_q_ok) return fail(PF_E_NOT_PD, "Matrix is not positive definite (Q)");
  if (h->sharded && !replay && h->ops->ch > 1 && h->pbase % 4)
    return fail(PF_E_ARG, "device-RNG predict of a scalar-state shard needs N_loc % 4 == 0 (or host replay)");
  HIPCHK(hipSetDevice(h->device));
  StepParams p = base_params(h);
  if (u) {
    pf_status st = upload_real(h, h->d_u, u, (size_t)h->R * h->nx);
    if (st) return st;
    p.u = h->d_u;
  }
  if (replay) {
    pf_status st = ensure_replay(h, &h->d_replay_a, (size_t)h->R * h->N * h->nx);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(h->d_replay_a, replay, (size_t)h->R * h->N * h->nx * sizeof(double),
                          hipMemcpyHostToDevice, h->stream));
    p.rp_noise = h->d_replay_a;
  }
  // a resample decided but not yet applied is fused into this launch
  const bool gather = h->pending;
  if (gather && h->cdf_needed()) {
    pf_status st = launch_cdf(h, p);
    if (st) return st;
  }
  p.allow_gather = gather;
  p.ep_resample = h->ep_res;
  p.cdf = h->cdf;
  p.do_predict = 1;
  p.ep_predict = h->epoch++;
  pf_status st = launch_step(h, p, true, false, gather);
  h->pending = false;
  if (replay || u) HIPCHK(hipStreamSynchronize(h->stream));
  return st;
}

pf_status pf_update(pf_handle* h, const double* z, pf_update_info* info, double* mean, double* cov) {
  if (!h || !z) return fail(PF_E_ARG, "null argument");
  {
    const pf_status s0 = settle(h);
    if (s0) return s0;
  }
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  if (h->pending) {  // an earlier decision nobody applied: apply it before re-weighting
    pf_status st = apply_pending(h, nullptr, nullptr, false);
    if (st) return st;
  }
  pf_status st = upload_real(h, h->d_z, z, (size_t)h->R * h->nz);
  if (st) return st;
  StepParams p = base_params(h);
  p.z = h->d_z;
  p.do_update = 1;
  st = launch_step(h, p, false, true, true);
  if (st) return st;
  h->ep_res = h->epoch++;
  StepParams f = base_params(h);
  set_outputs(f, out_slots(h), h->nx <= 4);
  f.out_step = 0;
  f.allow_gather = 1;
  st = launch_finalize(h, f);
  if (st) return st;
  std::vector<double> buf(out_doubles(h));
  HIPCHK(hipMemcpyAsync(buf.data(), h->d_out, buf.size() * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  const int R = h->R, nx = h->nx;
  const double* bm = buf.data();
  const double* bc = bm + (size_t)R * nx;
  const double* bn = bc + (size_t)R * nx * nx;
  const double* bl = bn + R;
  const int32_t* bf = (const int32_t*)(bl + R);
  for (int r = 0; r < R; ++r)
    if (!(bn[r] > 0.0))  // S == 0 or NaN: no particle has a finite weight
      return dead_filter(h, "(replicate " + std::to_string(r) + ")");
  bool any = false;
  for (int r = 0; r < R; ++r) {
    if (info) {
      info[r].neff = bn[r];
      info[r].log_norm = bl[r];
      info[r].resample = bf[r];
      info[r]._pad = 0;
    }
    any = any || bf[r];
  }
  if (mean) std::memcpy(mean, bm, (size_t)R * nx * sizeof(double));
  if (cov) {
    if (nx <= 4) {
      std::memcpy(cov, bc, (size_t)R * nx * nx * sizeof(double));
    } else {
      st = pf_moments(h, nullptr, cov);
      if (st) return st;
    }
  }
  h->pending = any;
  return PF_OK;
}

pf_status pf_resample(pf_handle* h, const double* uniforms, const double* jitter, double* mean, double* cov) {
  if (!h) return fail(PF_E_ARG, "null handle");
  {
    const pf_status s0 = settle(h);
    if (s0) return s0;
  }
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  if (!h->pending) return PF_OK;
  HIPCHK(hipSetDevice(h->device));
  pf_status st = apply_pending(h, uniforms, jitter, true);
  if (st) return st;
  if (mean || cov) {
    std::vector<double> buf(out_doubles(h));
    HIPCHK(hipMemcpyAsync(buf.data(), h->d_out, buf.size() * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    const size_t nm = (size_t)h->R * h->nx;
    if (mean) std::memcpy(mean, buf.data(), nm * sizeof(double));
    if (cov) {
      if (h->nx <= 4) {
        std::memcpy(cov, buf.data() + nm, nm * h->nx * sizeof(double));
      } else {
        st = pf_moments(h, nullptr, cov);
        if (st) return st;
      }
    }
  }
  return PF_OK;
}

pf_status pf_resample_state(pf_handle* h, const double* uniforms, const double* jitter) {
  if (!h) return fail(PF_E_ARG, "null handle");
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  h->ep_res = h->epoch++;
  pf_status st = apply_pending(h, uniforms, jitter, false, true);
  if (st) return st;
  HIPCHK(hipStreamSynchronize(h->stream));
  return PF_OK;
}

pf_status pf_run_device(pf_handle* h, const void* dZ, const void* dU, int64_t T, int32_t first_update_only,
                        double* d_means, double* d_covs, double* d_neff, int32_t* d_flags, double* d_lse) {
  if (!h || !dZ || T <= 0) return fail(PF_E_ARG, "bad argument");
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  if (!d_means || !d_neff || !d_flags || !d_lse) return fail(PF_E_ARG, "device outputs are required");
  if (!h->chol_q_ok) return fail(PF_E_NOT_PD, "Matrix is not positive definite (Q)");
  HIPCHK(hipSetDevice(h->device));
  {
    bool used = false;
    h->last_resident = false;
    pf_status st = run_resident(h, dZ, dU, T, first_update_only, d_means, (h->nx <= 4) ? d_covs : nullptr, d_neff,
                                d_flags, d_lse, &used);
    if (st || used) return st;
  }
  {
    bool used = false;
    h->last_persist = false;
    pf_status st = run_persist(h, dZ, dU, T, first_update_only, d_means, (h->nx <= 4) ? d_covs : nullptr, d_neff,
                               d_flags, d_lse, &used);
    if (st || used) return st;
  }
  const int R = h->R;
  StepParams p = base_params(h);
  p.o_mean = d_means;
  p.o_cov = (h->nx <= 4) ? d_covs : nullptr;
  // nx > 4: the step's covariance by pf_cov.h after the launch whose gather wrote its post-resample rows
  const bool cov_loop = d_covs && h->nx > 4;
  if (cov_loop) {
    pf_status st = ensure_cov(h);
    if (st) return st;
    h->cov_pending = 0;
    p.xr_out = h->xr;  // one of the two: rows with jitter, ancestors without
    p.anc_out = h->anc;
  }
  p.o_neff = d_neff;
  p.o_lse = d_lse;
  p.o_flag = d_flags;
  p.cdf = h->cdf;
  p.do_update = 1;
  bool gather_possible = h->pending;  // a pre-run decision is applied by kernel 0
  uint32_t prev_res = h->ep_res;
  if (h->timing) HIPCHK(hipEventRecord(h->tev[0], h->stream));
  for (int64_t s = 0; s < T; ++s) {
    const bool predict = !(first_update_only && s == 0);
    p.z = (const char*)dZ + (size_t)s * R * h->nz * h->esz;
    p.u = dU ? (const char*)dU + (size_t)s * R * h->nx * h->esz : nullptr;
    p.do_predict = predict;
    p.ep_predict = predict ? h->epoch++ : 0;
    p.allow_gather = gather_possible;
    p.ep_resample = prev_res;
    p.out_step = s >= 1 ? s - 1 : -1;
    p.out_post_step = s >= 2 ? s - 2 : -1;
    if (gather_possible && h->cdf_needed()) {
      pf_status st = launch_cdf(h, p);
      if (st) return st;
    }
    const void *xs_prev = h->x[h->cx], *lw_prev = h->lw[h->clw];  // step s - 1's predicted state
    pf_status st = launch_step(h, p, predict || gather_possible, true, true);
    if (st) return st;
    if (cov_loop && s >= 1) {
      st = launch_cov(h, xs_prev, lw_prev, s - 1, d_means, d_flags, d_lse, d_covs);
      if (st) return st;
    }
    prev_res = h->epoch++;
    gather_possible = true;
  }
  h->ep_res = prev_res;
  // tail: outputs of the last update, its resample (if any) and that resample's stats
  p.z = nullptr;
  p.u = nullptr;
  p.do_predict = 0;
  p.do_update = 0;
  p.allow_gather = 1;
  p.ep_resample = prev_res;
  p.out_step = T - 1;
  p.out_post_step = T >= 2 ? T - 2 : -1;
  if (h->cdf_needed()) {
    pf_status st = launch_cdf(h, p);
    if (st) return st;
  }
  const void *xs_last = h->x[h->cx], *lw_last = h->lw[h->clw];
  pf_status st = launch_step(h, p, true, false, true);
  if (st) return st;
  if (cov_loop) {
    st = launch_cov(h, xs_last, lw_last, T - 1, d_means, d_flags, d_lse, d_covs);
    if (st) return st;
    st = flush_cov(h, d_covs);
    if (st) return st;
  }
  p.out_step = -1;
  p.out_post_step = T - 1;
  st = launch_finalize(h, p);
  if (st) return st;
  if (h->timing) HIPCHK(hipEventRecord(h->tev[1], h->stream));
  h->pending = false;
  return PF_OK;
}

pf_status pf_set_timing(pf_handle* h, int32_t on) {
  if (!h) return fail(PF_E_ARG, "null handle");
  HIPCHK(hipSetDevice(h->device));
  if (on && !h->tev[0]) {
    HIPCHK(hipEventCreate(&h->tev[0]));
    HIPCHK(hipEventCreate(&h->tev[1]));
  }
  h->timing = on != 0;
  return PF_OK;
}

pf_status pf_set_trace(pf_handle* h, int64_t T_cap) {
  if (!h || T_cap < 0) return fail(PF_E_ARG, "bad argument");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (void* q : {(void*)h->tr_x, (void*)h->tr_l, (void*)h->tr_anc})
    if (q) HIPCHK(hipFree(q));
  h->tr_x = h->tr_l = nullptr;
  h->tr_anc = nullptr;
  h->tr_T = 0;
  if (T_cap == 0) return PF_OK;
  const size_t n = (size_t)T_cap * h->R * h->Npad;
  float *x = nullptr, *l = nullptr;
  int32_t* a = nullptr;
  hipError_t e = hipMalloc((void**)&x, n * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&l, n * 4);
  if (e == hipSuccess) e = hipMalloc((void**)&a, n * 4);
  if (e == hipSuccess) e = hipMemsetAsync(a, 0xff, n * 4, h->stream);  // -1: slot not written
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    for (void* q : {(void*)x, (void*)l, (void*)a})
      if (q) (void)hipFree(q);
    return fail(PF_E_HIP, std::string("trace buffers: ") + hipGetErrorString(e));
  }
  h->tr_x = x;
  h->tr_l = l;
  h->tr_anc = a;
  h->tr_T = T_cap;
  return PF_OK;
}

pf_status pf_get_trace(pf_handle* h, int64_t t, int32_t r, float* x, float* l, int32_t* anc) {
  if (!h || t < 0 || r < 0 || r >= h->R) return fail(PF_E_ARG, "bad argument");
  if (t >= h->tr_T) return fail(PF_E_ARG, "step outside the trace (pf_set_trace)");
  HIPCHK(hipSetDevice(h->device));
  {
    const pf_status s0 = settle(h);
    if (s0) return s0;
  }
  // only the resident kernel records the trace: after a launch-per-step run it would be stale
  if (!h->last_resident) return fail(PF_E_ARG, "the last run was not a resident launch: no trace recorded");
  HIPCHK(hipStreamSynchronize(h->stream));
  const size_t o = ((size_t)t * h->R + r) * h->Npad, n = (size_t)h->N * 4;
  if (x) HIPCHK(hipMemcpy(x, h->tr_x + o, n, hipMemcpyDeviceToHost));
  if (l) HIPCHK(hipMemcpy(l, h->tr_l + o, n, hipMemcpyDeviceToHost));
  if (anc) {
    HIPCHK(hipMemcpy(anc, h->tr_anc + o, n, hipMemcpyDeviceToHost));
    HIPCHK(hipMemsetAsync(h->tr_anc + o, 0xff, n, h->stream));  // ready for the next run
  }
  return PF_OK;
}

pf_status pf_last_run_ms(pf_handle* h, float* ms) {
  if (!h || !ms) return fail(PF_E_ARG, "null argument");
  if (!h->tev[0]) return fail(PF_E_ARG, "timing was not enabled (pf_set_timing)");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipEventSynchronize(h->tev[1]));
  HIPCHK(hipEventElapsedTime(ms, h->tev[0], h->tev[1]));
  return PF_OK;
}

pf_status pf_run(pf_handle* h, const double* Z, const double* U, int64_t T, int32_t first_update_only,
                 double* means, double* covs, double* neff, uint8_t* flags, double* lse) {
  if (!h || !Z || T <= 0) return fail(PF_E_ARG, "bad argument");
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  const int R = h->R, nx = h->nx, nz = h->nz;
  void *dZ = nullptr, *dU = nullptr;
  double *dm = nullptr, *dc = nullptr, *dn = nullptr, *dl = nullptr;
  int32_t* df = nullptr;
  pf_status st = PF_OK;
  auto bail = [&](pf_status s) {
    (void)hipStreamSynchronize(h->stream);
    for (void* q : {dZ, dU, (void*)dm, (void*)dc, (void*)dn, (void*)dl, (void*)df})
      if (q) (void)hipFree(q);
    return s;
  };
  if (hipMalloc(&dZ, (size_t)T * R * nz * h->esz) != hipSuccess ||
      (U && hipMalloc(&dU, (size_t)T * R * nx * h->esz) != hipSuccess) ||
      hipMalloc((void**)&dm, (size_t)T * R * nx * sizeof(double)) != hipSuccess ||
      (covs && hipMalloc((void**)&dc, (size_t)T * R * nx * nx * sizeof(double)) != hipSuccess) ||
      hipMalloc((void**)&dn, (size_t)T * R * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&dl, (size_t)T * R * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&df, (size_t)T * R * sizeof(int32_t)) != hipSuccess)
    return bail(fail(PF_E_HIP, "hipMalloc for pf_run buffers failed"));
  st = upload_real(h, dZ, Z, (size_t)T * R * nz);
  if (!st && U) st = upload_real(h, dU, U, (size_t)T * R * nx);
  if (st) return bail(st);
  for (int attempt = 0;; ++attempt) {
    st = pf_run_device(h, dZ, dU, T, first_update_only, dm, dc, dn, df, dl);
    if (st) return bail(st);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return bail(fail(PF_E_HIP, "pf_run: stream sync failed"));
    st = check_resident(h);
    if (st == PF_E_RETRY && attempt == 0) continue;  // aborted before computing: run again, cooperatively
    if (st) return bail(st);
    break;
  }
  std::vector<int32_t> fl((size_t)T * R);
  std::vector<double> nf((size_t)T * R);
  if ((means && hipMemcpy(means, dm, (size_t)T * R * nx * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) ||
      (covs && dc && hipMemcpy(covs, dc, (size_t)T * R * nx * nx * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) ||
      hipMemcpy(nf.data(), dn, nf.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
      (lse && hipMemcpy(lse, dl, (size_t)T * R * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) ||
      hipMemcpy(fl.data(), df, fl.size() * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
    return bail(fail(PF_E_HIP, "pf_run: output copy failed"));
  if (flags)
    for (size_t i = 0; i < fl.size(); ++i) flags[i] = (uint8_t)(fl[i] != 0);
  if (neff) std::memcpy(neff, nf.data(), nf.size() * sizeof(double));
  for (size_t i = 0; i < nf.size(); ++i)
    if (!(nf[i] > 0.0))
      return bail(dead_filter(h, "at step " + std::to_string(i / R) + " (replicate " + std::to_string(i % R) + ")"));
  return bail(PF_OK);
}

static pf_status download_real(pf_handle* h, const void* src, size_t n, std::vector<double>& out) {
  out.resize(n);
  if (h->esz == 8) {
    HIPCHK(hipMemcpyAsync(out.data(), src, n * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  } else {
    std::vector<float> f(n);
    HIPCHK(hipMemcpyAsync(f.data(), src, n * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    for (size_t i = 0; i < n; ++i) out[i] = (double)f[i];
  }
  return PF_OK;
}

pf_status pf_get_particles(pf_handle* h, double* particles) {
  if (!h || !particles) return fail(PF_E_ARG, "null argument");
  {
    const pf_status s0 = settle(h);
    if (s0) return s0;
  }
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  if (h->pending) {
    pf_status st = apply_pending(h, nullptr, nullptr, false);
    if (st) return st;
  }
  std::vector<double> soa;
  pf_status st = download_real(h, h->x[h->cx], (size_t)h->R * h->nx * h->Npad, soa);
  if (st) return st;
  const int nx = h->nx;
  for (int r = 0; r < h->R; ++r)
    for (int d = 0; d < nx; ++d) {
      const double* src = soa.data() + ((size_t)r * nx + d) * h->Npad;
      double* dst = particles + (size_t)r * h->N * nx + d;
      for (int64_t i = 0; i < h->N; ++i) dst[i * nx] = src[i];
    }
  return PF_OK;
}

int32_t pf_weights_uniform(pf_handle* h) {
  if (!h || !h->initialized) return 0;
  if (h->pending) {
    if (apply_pending(h, nullptr, nullptr, false) != PF_OK) return 0;
  }
  int32_t all = 1;
  for (int r = 0; r < h->R; ++r) {
    double u = 0.0;
    if (hipMemcpy(&u, h->rec[h->crec] + (size_t)r * h->G * h->ops->rec_size + 3 * (size_t)h->G, sizeof(double),
                  hipMemcpyDeviceToHost) != hipSuccess)
      return 0;
    all = all && (u != 0.0);
  }
  return all;
}

pf_status pf_get_weights(pf_handle* h, double* weights, double* log_weights) {
  if (!h) return fail(PF_E_ARG, "null argument");
  {
    const pf_status s0 = settle(h);
    if (s0) return s0;
  }
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  if (h->pending) {
    pf_status st = apply_pending(h, nullptr, nullptr, false);
    if (st) return st;
  }
  // per-replicate normaliser from the current records (k_finalize into scratch)
  StepParams f = base_params(h);
  set_outputs(f, out_slots(h), false);
  f.out_step = 0;
  pf_status st = launch_finalize(h, f);
  if (st) return st;
  std::vector<double> buf(out_doubles(h));
  HIPCHK(hipMemcpyAsync(buf.data(), h->d_out, buf.size() * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  std::vector<double> uni(h->R);
  for (int r = 0; r < h->R; ++r)
    HIPCHK(hipMemcpyAsync(&uni[r], h->rec[h->crec] + (size_t)r * h->G * h->ops->rec_size + 3 * (size_t)h->G, sizeof(double),
                          hipMemcpyDeviceToHost, h->stream));
  std::vector<double> lw;
  st = download_real(h, h->lw[h->clw], (size_t)h->R * h->Npad, lw);
  if (st) return st;
  const double* lse = buf.data() + (size_t)h->R * h->nx + (size_t)h->R * h->nx * h->nx + h->R;
  for (int r = 0; r < h->R; ++r) {
    for (int64_t i = 0; i < h->N; ++i) {
      const size_t o = (size_t)r * h->N + i;
      double l;
      if (uni[r] != 0.0) {
        if (weights) weights[o] = 1.0 / (double)h->N;
        l = -std::log((double)h->N);
      } else {
        l = lw[(size_t)r * h->Npad + i] - lse[r];
        if (weights) weights[o] = std::exp(l);
      }
      if (log_weights) log_weights[o] = l;
    }
  }
  return PF_OK;
}

// ---------------------------------------------------------------------------
// Within-filter sharding (include/pf_shard.h)
// ---------------------------------------------------------------------------
pf_status pf_shard_configure(pf_handle* h, int64_t n_total, int32_t rank) {
  if (!h) return fail(PF_E_ARG, "null handle");
  if (h->R != 1 || h->method != 0) return fail(PF_E_ARG, "sharding needs R = 1 and systematic resampling");
  if (n_total <= 0 || n_total % h->N != 0 || rank < 0 || (int64_t)rank >= n_total / h->N)
    return fail(PF_E_ARG, "sharding needs n_total = W * N_loc and 0 <= rank < W");
  if (n_total / 4 > (int64_t)UINT32_MAX / (h->nx > 0 ? h->nx : 1))
    return fail(PF_E_ARG, "n_total too large for 32-bit Philox counters");
  HIPCHK(hipSetDevice(h->device));
  h->sharded = true;
  h->n_total = n_total;
  h->pbase = (int64_t)rank * h->N;
  if (!h->cdf && hipMalloc((void**)&h->cdf, (size_t)h->R * h->N * sizeof(double)) != hipSuccess)
    return fail(PF_E_HIP, "hipMalloc of cdf failed");
  return PF_OK;
}

pf_status pf_shard_update(pf_handle* h, const double* z, double lse_prev, pf_shard_stats* st, double* mean,
                          double* cov) {
  if (!h || !z || !st) return fail(PF_E_ARG, "null argument");
  if (!h->sharded) return fail(PF_E_ARG, "pf_shard_update needs pf_shard_configure");
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  pf_status s = upload_real(h, h->d_z, z, (size_t)h->nz);
  if (s) return s;
  StepParams p = base_params(h);
  p.z = h->d_z;
  p.do_update = 1;
  p.use_lse_ext = 1;  // l = (l_prev - lse_global) + loglik (pf.py:254-256 over ALL shards' weights)
  p.lse_ext = lse_prev;
  s = launch_step(h, p, false, true, true);
  if (s) return s;
  h->ep_res = h->epoch++;  // the resample of this update (U, jitter) uses this epoch on every rank
  StepParams f = base_params(h);
  set_outputs(f, out_slots(h), h->nx <= 4);
  f.out_step = 0;
  s = launch_finalize(h, f);
  if (s) return s;
  std::vector<double> buf(out_doubles(h));
  HIPCHK(hipMemcpyAsync(buf.data(), h->d_out, buf.size() * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  const int nx = h->nx;
  const double* bm = buf.data();
  const double* bc = bm + nx;
  const double* bn = bc + (size_t)nx * nx;
  const double* bl = bn + 1;
  st->lse = bl[0];
  st->neff = bn[0];
  st->U = uniform53(h->seed, 0, (uint32_t)h->rep_base, h->ep_res);
  if (mean) std::memcpy(mean, bm, (size_t)nx * sizeof(double));
  if (cov) {
    if (nx <= 4) std::memcpy(cov, bc, (size_t)nx * nx * sizeof(double));
    else return pf_moments(h, nullptr, cov);
  }
  return PF_OK;
}

pf_status pf_shard_offspring(pf_handle* h, double U, double lo, double mass, int64_t a, int64_t n, void* out) {
  if (!h || (n > 0 && !out)) return fail(PF_E_ARG, "null argument");
  if (!h->sharded) return fail(PF_E_ARG, "pf_shard_offspring needs pf_shard_configure");
  if (n < 0 || a < 0 || a + n > h->n_total || !(mass > 0.0)) {
    if (n == 0) return PF_OK;
    return fail(PF_E_ARG, "pf_shard_offspring: slot range outside the filter or empty segment");
  }
  HIPCHK(hipSetDevice(h->device));
  if (h->shard_cdf_ep != h->ep_res) {  // this update's normalised CDF, once per resample
    StepParams p = base_params(h);
    p.allow_gather = 1;
    p.force_gather = 1;
    pf_status s = launch_cdf(h, p);
    if (s) return s;
    h->shard_cdf_ep = h->ep_res;
  }
  HIPCHK(h->ops->shard_offspring(h->x[h->cx], h->N, h->Npad, h->cdf, U, lo, mass, h->n_total, a, n, out, h->stream,
                                 h->nx));
  HIPCHK(hipStreamSynchronize(h->stream));
  return PF_OK;
}

pf_status pf_shard_adopt(pf_handle* h, const void* rows, const double* jitter, double* mean, double* cov) {
  if (!h || !rows) return fail(PF_E_ARG, "null argument");
  if (!h->sharded) return fail(PF_E_ARG, "pf_shard_adopt needs pf_shard_configure");
  HIPCHK(hipSetDevice(h->device));
  const double* rj = nullptr;
  if (jitter && h->regularize) {  // host replay: this shard's slots' jitter normals [N_loc][nx]
    pf_status st = ensure_replay(h, &h->d_replay_b, (size_t)h->N * h->nx);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(h->d_replay_b, jitter, (size_t)h->N * h->nx * sizeof(double), hipMemcpyHostToDevice,
                          h->stream));
    rj = h->d_replay_b;
  } else if (h->regularize && h->ops->ch > 1 && h->pbase % 4) {
    return fail(PF_E_ARG, "device-RNG jitter of a scalar-state shard needs N_loc % 4 == 0 (or host replay)");
  }
  state_written(h);
  HIPCHK(h->ops->shard_adopt(rows, h->x[h->cx], h->N, h->Npad, h->rec[h->crec], h->G, h->P, h->regularize, rj,
                             h->seed, (uint32_t)h->rep_base, h->ep_res, h->pbase, h->stream, h->nx, h->nz));
  h->pending = false;
  h->shard_cdf_ep = 0;
  if (mean || cov) return pf_moments(h, mean, cov);
  HIPCHK(hipStreamSynchronize(h->stream));
  return PF_OK;
}

// diag:61-91 on the device-resident state of every replicate (include/pf_diag.h)
pf_status pf_state_diagnostics(pf_handle* h, double tol, pf_diagnostics* out) {
  if (!h || !out) return fail(PF_E_ARG, "null argument");
  {
    const pf_status s0 = settle(h);
    if (s0) return s0;
  }
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  if (h->pending) {
    pf_status st = apply_pending(h, nullptr, nullptr, false);
    if (st) return st;
  }
  StepParams f = base_params(h);
  const OutSlots o = out_slots(h);
  set_outputs(f, o, false);
  f.out_step = 0;
  pf_status st = launch_finalize(h, f);
  if (st) return st;
  std::vector<double> lse(h->R), uni(h->R);
  HIPCHK(hipMemcpyAsync(lse.data(), o.lse, h->R * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  for (int r = 0; r < h->R; ++r)
    HIPCHK(hipMemcpyAsync(&uni[r], h->rec[h->crec] + (size_t)r * h->G * h->ops->rec_size + 3 * (size_t)h->G,
                          sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (int r = 0; r < h->R; ++r) {
    diag::DiagSrc s{};
    s.N = h->N;
    s.Npad = h->Npad;
    s.nx = h->nx;
    s.w = nullptr;
    s.lw = (const char*)h->lw[h->clw] + (size_t)r * h->Npad * h->esz;
    s.lse = lse[r];
    s.uniform = uni[r] != 0.0;
    s.x = (const char*)h->x[h->cx] + (size_t)r * h->nx * h->Npad * h->esz;
    s.real_is_double = h->esz == 8;
    s.tol = tol;
    s.spread = NAN;
    st = diag::compute(s, h->stream, out + r);
    if (st) return st;
  }
  return PF_OK;
}

pf_status pf_set_state(pf_handle* h, const double* particles, const double* weights) {
  if (!h || !particles) return fail(PF_E_ARG, "null argument");
  {
    const pf_status s0 = settle(h);
    if (s0) return s0;
  }
  HIPCHK(hipSetDevice(h->device));
  const int nx = h->nx, R = h->R;
  std::vector<double> soa((size_t)R * nx * h->Npad, 0.0);
  for (int r = 0; r < R; ++r)
    for (int d = 0; d < nx; ++d)
      for (int64_t i = 0; i < h->N; ++i)
        soa[((size_t)r * nx + d) * h->Npad + i] = particles[((size_t)r * h->N + i) * nx + d];
  pf_status st = upload_real(h, h->x[h->cx], soa.data(), soa.size());
  if (st) return st;
  state_written(h);
  h->lcum_valid = false;  // uploaded weights: k_cdf materialises their CDF when a resample needs it
  // records: one tile carrying S0 = 1 at m = 0 (so lse = 0), the rest empty; or uniform
  std::vector<double> rec((size_t)R * h->G * h->ops->rec_size, 0.0);
  const size_t G = (size_t)h->G;
  for (int r = 0; r < R; ++r)
    for (size_t k = 0; k < G; ++k) {
      double* o = rec.data() + (size_t)r * G * h->ops->rec_size + k;  // SoA: field q at o[q*G]
      if (!weights) {
        o[3 * G] = 1.0;
      } else {
        o[0] = k == 0 ? 0.0 : -INFINITY;
        o[1 * G] = k == 0 ? 1.0 : 0.0;
        o[2 * G] = k == 0 ? 1.0 : 0.0;
      }
    }
  HIPCHK(hipMemcpy(h->rec[h->crec], rec.data(), rec.size() * sizeof(double), hipMemcpyHostToDevice));
  if (weights) {
    std::vector<double> lw((size_t)R * h->Npad, -INFINITY);
    for (int r = 0; r < R; ++r)
      for (int64_t i = 0; i < h->N; ++i) lw[(size_t)r * h->Npad + i] = std::log(weights[(size_t)r * h->N + i]);
    st = upload_real(h, h->lw[h->clw], lw.data(), lw.size());
    if (st) return st;
    // re-derive proper per-tile records: an update launch with no likelihood term
    StepParams p = base_params(h);
    p.do_update = 2;  // 2 = reweigh only (log-likelihood skipped)
    p.z = h->d_z;
    st = launch_step(h, p, false, true, true);
    if (st) return st;
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  h->initialized = true;
  h->pending = false;
  return PF_OK;
}

// ---------------------------------------------------------------------------
// Philox position and bit-exact checkpoint / resume
// ---------------------------------------------------------------------------
pf_status pf_get_rng_state(pf_handle* h, pf_rng_state* out) {
  if (!h || !out) return fail(PF_E_ARG, "null argument");
  HIPCHK(hipSetDevice(h->device));
  const pf_status s0 = settle(h);
  if (s0) return s0;
  out->seed = h->seed;
  out->epoch = h->epoch;
  out->ep_res = h->ep_res;
  out->replicate_base = h->rep_base;
  out->pending = h->pending ? 1 : 0;
  return PF_OK;
}

pf_status pf_set_rng_state(pf_handle* h, const pf_rng_state* in) {
  if (!h || !in) return fail(PF_E_ARG, "null argument");
  if (in->epoch == 0) return fail(PF_E_ARG, "epoch 0 is never a handle's position (initialize draws at >= 1)");
  HIPCHK(hipSetDevice(h->device));
  const pf_status s0 = settle(h);
  if (s0) return s0;
  h->seed = in->seed;
  h->epoch = in->epoch;
  h->ep_res = in->ep_res;
  h->rep_base = in->replicate_base;
  return PF_OK;
}

namespace {
constexpr uint64_t CKPT_MAGIC = 0x3130544b43504650ull;  // "PFPCKT01"
struct CkptHead {
  uint64_t magic;
  int32_t nx, nz, R, G;
  int64_t N, Npad;
  int32_t rec_size, esz, method, rep_base;
  uint64_t seed;
  uint32_t epoch, ep_res;
  int32_t lcum_valid, hdr_valid;
  uint64_t x_bytes, lw_bytes, rec_bytes, lcum_bytes, hdr_bytes;
};
CkptHead ckpt_layout(const pf_handle* h) {
  CkptHead c;
  std::memset(&c, 0, sizeof(c));
  c.magic = CKPT_MAGIC;
  c.nx = h->nx;
  c.nz = h->nz;
  c.R = h->R;
  c.G = h->G;
  c.N = h->N;
  c.Npad = h->Npad;
  c.rec_size = h->ops->rec_size;
  c.esz = (int32_t)h->esz;
  c.method = h->method;
  c.x_bytes = (uint64_t)h->R * h->nx * h->Npad * h->esz;
  c.lw_bytes = (uint64_t)h->R * h->Npad * h->esz;
  c.rec_bytes = rec_bytes(h);
  c.lcum_bytes = h->lcum[0] ? (uint64_t)h->R * h->N * sizeof(double) : 0;
  c.hdr_bytes = 4 * (uint64_t)h->R * sizeof(unsigned long long);
  return c;
}
uint64_t ckpt_total(const CkptHead& c) {
  return sizeof(CkptHead) + c.x_bytes + c.lw_bytes + c.rec_bytes + c.lcum_bytes + c.hdr_bytes;
}
size_t res_hdr_offset(const pf_handle* h) {  // entry headers inside rsync (run_resident's layout)
  return RCOPIES * gran_copy_stride(h->R) + 2 * (size_t)h->R * RMAXG + 4;
}
}  // namespace

int64_t pf_checkpoint_bytes(pf_handle* h) {
  if (!h) return -1;
  return (int64_t)ckpt_total(ckpt_layout(h));
}

pf_status pf_checkpoint(pf_handle* h, void* buf, int64_t nbytes) {
  if (!h || !buf) return fail(PF_E_ARG, "null argument");
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  pf_status st = settle(h);
  if (st) return st;
  if (h->pending) {  // the checkpoint is a step boundary: a decided resample is applied first
    st = apply_pending(h, nullptr, nullptr, false);
    if (st) return st;
  }
  CkptHead c = ckpt_layout(h);
  if (nbytes < (int64_t)ckpt_total(c)) return fail(PF_E_ARG, "checkpoint buffer too small (pf_checkpoint_bytes)");
  c.seed = h->seed;
  c.epoch = h->epoch;
  c.ep_res = h->ep_res;
  c.rep_base = h->rep_base;
  c.lcum_valid = (c.lcum_bytes && h->lcum_valid) ? 1 : 0;
  char* o = (char*)buf + sizeof(CkptHead);
  HIPCHK(hipMemcpyAsync(o, h->x[h->cx], c.x_bytes, hipMemcpyDeviceToHost, h->stream));
  o += c.x_bytes;
  HIPCHK(hipMemcpyAsync(o, h->lw[h->clw], c.lw_bytes, hipMemcpyDeviceToHost, h->stream));
  o += c.lw_bytes;
  HIPCHK(hipMemcpyAsync(o, h->rec[h->crec], c.rec_bytes, hipMemcpyDeviceToHost, h->stream));
  o += c.rec_bytes;
  if (c.lcum_bytes) {
    if (c.lcum_valid) HIPCHK(hipMemcpyAsync(o, h->lcum[h->clcum], c.lcum_bytes, hipMemcpyDeviceToHost, h->stream));
    else std::memset(o, 0, c.lcum_bytes);
    o += c.lcum_bytes;
  }
  // the resident exit header that describes this state (a run that follows takes it instead of
  // reducing the records: part of the state for a bit-exact continuation)
  std::memset(o, 0, c.hdr_bytes);
  if (!h->hdr_restore.empty()) {
    std::memcpy(o, h->hdr_restore.data(), c.hdr_bytes);
    c.hdr_valid = 1;
  } else if (h->res_hdr && h->rsync) {
    HIPCHK(hipMemcpyAsync(o, h->rsync + res_hdr_offset(h), c.hdr_bytes, hipMemcpyDeviceToHost, h->stream));
    c.hdr_valid = 1;
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  std::memcpy(buf, &c, sizeof(c));
  return PF_OK;
}

pf_status pf_restore(pf_handle* h, const void* buf, int64_t nbytes) {
  if (!h || !buf) return fail(PF_E_ARG, "null argument");
  if (nbytes < (int64_t)sizeof(CkptHead)) return fail(PF_E_ARG, "checkpoint too short");
  CkptHead c;
  std::memcpy(&c, buf, sizeof(c));
  const CkptHead want = ckpt_layout(h);
  if (c.magic != CKPT_MAGIC) return fail(PF_E_ARG, "not a pf_checkpoint blob");
  if (c.nx != want.nx || c.nz != want.nz || c.R != want.R || c.G != want.G || c.N != want.N || c.Npad != want.Npad ||
      c.rec_size != want.rec_size || c.esz != want.esz || c.method != want.method || c.x_bytes != want.x_bytes ||
      c.lw_bytes != want.lw_bytes || c.rec_bytes != want.rec_bytes || c.lcum_bytes != want.lcum_bytes ||
      c.hdr_bytes != want.hdr_bytes)
    return fail(PF_E_ARG, "checkpoint of a different filter configuration (shape, N, replicates, precision or method)");
  if (nbytes < (int64_t)ckpt_total(c)) return fail(PF_E_ARG, "checkpoint truncated");
  HIPCHK(hipSetDevice(h->device));
  pf_status st = settle(h);
  if (st && st != PF_E_NAN) return st;  // a dead state is being replaced: fine
  const char* o = (const char*)buf + sizeof(CkptHead);
  HIPCHK(hipMemcpyAsync(h->x[h->cx], o, c.x_bytes, hipMemcpyHostToDevice, h->stream));
  o += c.x_bytes;
  HIPCHK(hipMemcpyAsync(h->lw[h->clw], o, c.lw_bytes, hipMemcpyHostToDevice, h->stream));
  o += c.lw_bytes;
  HIPCHK(hipMemcpyAsync(h->rec[h->crec], o, c.rec_bytes, hipMemcpyHostToDevice, h->stream));
  o += c.rec_bytes;
  if (c.lcum_bytes) {
    if (c.lcum_valid) HIPCHK(hipMemcpyAsync(h->lcum[h->clcum], o, c.lcum_bytes, hipMemcpyHostToDevice, h->stream));
    o += c.lcum_bytes;
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  state_written(h);
  if (c.hdr_valid) {
    h->hdr_restore.assign((const unsigned long long*)o, (const unsigned long long*)o + 4 * (size_t)h->R);
  }
  h->lcum_valid = c.lcum_valid != 0;
  h->seed = c.seed;
  h->epoch = c.epoch;
  h->ep_res = c.ep_res;
  h->rep_base = c.rep_base;
  h->pending = false;
  h->head_valid = false;
  h->shard_cdf_ep = 0;
  h->initialized = true;
  return PF_OK;
}

pf_status pf_moments(pf_handle* h, double* mean, double* cov) {
  if (!h) return fail(PF_E_ARG, "null handle");
  {
    const pf_status s0 = settle(h);
    if (s0) return s0;
  }
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  if (h->pending) {
    pf_status st = apply_pending(h, nullptr, nullptr, false);
    if (st) return st;
  }
  // lse of the current records -> scratch, then two-pass moments on device
  StepParams f = base_params(h);
  OutSlots o = out_slots(h);
  set_outputs(f, o, false);
  f.out_step = 0;
  pf_status st = launch_finalize(h, f);
  if (st) return st;
  const int nx = h->nx, R = h->R;
  double *dmean = nullptr, *dcov = nullptr;
  HIPCHK(hipMalloc((void**)&dmean, (size_t)R * nx * sizeof(double)));
  if (cov && hipMalloc((void**)&dcov, (size_t)R * nx * nx * sizeof(double)) != hipSuccess) {
    (void)hipFree(dmean);
    return fail(PF_E_HIP, "hipMalloc failed");
  }
  hipError_t e = h->ops->moments(h->x[h->cx], h->lw[h->clw], h->rec[h->crec], h->G, o.lse, h->N, h->Npad, R, dmean,
                                 dcov, h->stream, nx);
  if (e == hipSuccess && mean)
    e = hipMemcpyAsync(mean, dmean, (size_t)R * nx * sizeof(double), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess && cov)
    e = hipMemcpyAsync(cov, dcov, (size_t)R * nx * nx * sizeof(double), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(dmean);
  if (dcov) (void)hipFree(dcov);
  if (e != hipSuccess) return fail(PF_E_HIP, std::string("pf_moments: ") + hipGetErrorString(e));
  return PF_OK;
}

pf_status pf_resample_indices(int32_t device, int32_t method, const double* w, int64_t N, double U,
                              const double* uniforms, int64_t* idx) {
  if (!w || !idx || N <= 0) return fail(PF_E_ARG, "bad argument");
  if (method == 1 && !uniforms) return fail(PF_E_ARG, "multinomial needs uniforms");
  HIPCHK(hipSetDevice(device));
  const int tile = 4096;
  const int G = (int)((N + tile - 1) / tile);
  if (G > 4 * BLOCK) return fail(PF_E_ARG, "N too large for pf_resample_indices");
  double *dw = nullptr, *dsum = nullptr, *dcdf = nullptr, *du = nullptr;
  int64_t* didx = nullptr;
  auto done = [&](pf_status s) {
    for (void* q : {(void*)dw, (void*)dsum, (void*)dcdf, (void*)du, (void*)didx})
      if (q) (void)hipFree(q);
    return s;
  };
  if (hipMalloc((void**)&dw, N * 8) != hipSuccess || hipMalloc((void**)&dsum, G * 8) != hipSuccess ||
      hipMalloc((void**)&dcdf, N * 8) != hipSuccess || hipMalloc((void**)&didx, N * 8) != hipSuccess ||
      (method == 1 && hipMalloc((void**)&du, N * 8) != hipSuccess))
    return done(fail(PF_E_HIP, "hipMalloc failed"));
  if (hipMemcpy(dw, w, N * 8, hipMemcpyHostToDevice) != hipSuccess ||
      (du && hipMemcpy(du, uniforms, N * 8, hipMemcpyHostToDevice) != hipSuccess))
    return done(fail(PF_E_HIP, "upload failed"));
  hipLaunchKernelGGL(k_w_tile_sums, dim3(G), dim3(BLOCK), 64 * 8, 0, dw, N, tile, dsum);
  hipLaunchKernelGGL(k_w_cdf, dim3(G), dim3(BLOCK), 64 * 8, 0, dw, N, tile, G, dsum, dcdf, method == 0);
  hipLaunchKernelGGL(k_w_search, dim3((unsigned)((N + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, 0, dcdf, N, method, U,
                     du, didx);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return done(fail(PF_E_HIP, "resample kernels failed"));
  if (hipMemcpy(idx, didx, N * 8, hipMemcpyDeviceToHost) != hipSuccess) return done(fail(PF_E_HIP, "download failed"));
  return done(PF_OK);
}

void* pf_stream(pf_handle* h) { return h ? (void*)h->stream : nullptr; }

#ifdef PF_STAMPS
// diagnostic build only: copy out the per-workgroup phase stamps of the last k_step
pf_status pf_debug_stamps(unsigned long long* out, int n) {
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pf_stamps), (size_t)n * sizeof(unsigned long long)));
  return PF_OK;
}
#endif

pf_status pf_synchronize(pf_handle* h) {
  if (!h) return fail(PF_E_ARG, "null handle");
  HIPCHK(hipStreamSynchronize(h->stream));
  return check_resident(h);
}

int32_t pf_last_run_resident(pf_handle* h) { return (h && h->last_resident) ? 1 : 0; }
int32_t pf_last_run_persistent(pf_handle* h) { return (h && h->last_persist) ? 1 : 0; }

pf_status pf_test_lds_poison(void* stream) {
  pf::lds_poison((hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? PF_OK : fail(PF_E_HIP, "k_lds_poison launch failed");
}

int32_t pf_test_lds_probe_blocks(void) { return pf::lds_poison_blocks(); }

int64_t pf_test_lds_poison_count(void) { return pf::g_lds_poison_count; }

pf_status pf_test_lds_probe(void* stream, int32_t* out) {
  if (!out) return fail(PF_E_ARG, "pf_test_lds_probe: out is null");
  const int nb = pf::lds_poison_blocks();
  int32_t* d = nullptr;
  if (hipMalloc((void**)&d, nb * sizeof(int32_t)) != hipSuccess) return fail(PF_E_HIP, "pf_test_lds_probe: hipMalloc");
  (void)hipFuncSetAttribute((const void*)pf::k_lds_probe, hipFuncAttributeMaxDynamicSharedMemorySize,
                            pf::PF_LDS_CU_BYTES - 1024);
  hipLaunchKernelGGL(pf::k_lds_probe, dim3(nb), dim3(1024), pf::PF_LDS_CU_BYTES - 1024, (hipStream_t)stream,
                     pf::PF_LDS_POISON, d);
  hipError_t e = hipMemcpyAsync(out, d, nb * sizeof(int32_t), hipMemcpyDeviceToHost, (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  (void)hipFree(d);
  return e == hipSuccess ? PF_OK : fail(PF_E_HIP, std::string("pf_test_lds_probe: ") + hipGetErrorString(e));
}

pf_status pf_geometry(pf_handle* h, int32_t* G, int32_t* tile, int32_t* lds) {
  if (!h) return fail(PF_E_ARG, "null handle");
  if (G) *G = h->G;
  if (tile) *tile = h->tile;
  if (lds) *lds = (int32_t)step_lds(h, true);
  return PF_OK;
}

pf_status pf_profile_steps(pf_handle* h, const void* dZ, int64_t steps, float* ms_out) {
  if (!h || !dZ || steps <= 0 || !ms_out) return fail(PF_E_ARG, "bad argument");
  if (!h->initialized) return fail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  HIPCHK(hipSetDevice(h->device));
  const int R = h->R;
  double *dm = nullptr, *dn = nullptr, *dl = nullptr;
  int32_t* df = nullptr;
  HIPCHK(hipMalloc((void**)&dm, (size_t)steps * R * h->nx * sizeof(double)));
  HIPCHK(hipMalloc((void**)&dn, (size_t)steps * R * sizeof(double)));
  HIPCHK(hipMalloc((void**)&dl, (size_t)steps * R * sizeof(double)));
  HIPCHK(hipMalloc((void**)&df, (size_t)steps * R * sizeof(int32_t)));
  std::vector<hipEvent_t> ev((size_t)steps + 1);
  for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  StepParams p = base_params(h);
  p.o_mean = dm;
  p.o_neff = dn;
  p.o_lse = dl;
  p.o_flag = df;
  p.cdf = h->cdf;
  p.do_update = 1;
  p.do_predict = 1;
  bool gather_possible = h->pending;
  uint32_t prev_res = h->ep_res;
  pf_status st = PF_OK;
  for (int64_t s = 0; s < steps && !st; ++s) {
    p.z = (const char*)dZ + (size_t)s * R * h->nz * h->esz;
    p.ep_predict = h->epoch++;
    p.allow_gather = gather_possible;
    p.ep_resample = prev_res;
    p.out_step = s >= 1 ? s - 1 : -1;
    p.out_post_step = s >= 2 ? s - 2 : -1;
    if (gather_possible && h->cdf_needed()) st = launch_cdf(h, p);
    if (!st) {
      (void)hipEventRecord(ev[s], h->stream);
      st = launch_step(h, p, true, true, true);
    }
    prev_res = h->epoch++;
    gather_possible = true;
  }
  (void)hipEventRecord(ev[steps], h->stream);
  (void)hipStreamSynchronize(h->stream);
  h->ep_res = prev_res;
  h->pending = false;
  // leave a consistent state: apply the last decision
  if (!st) {
    StepParams q = base_params(h);
    q.allow_gather = 1;
    q.ep_resample = prev_res;
    q.cdf = h->cdf;
    if (h->cdf_needed()) st = launch_cdf(h, q);
    if (!st) st = launch_step(h, q, true, false, true);
  }
  (void)hipStreamSynchronize(h->stream);
  for (int64_t s = 0; s < steps; ++s) (void)hipEventElapsedTime(&ms_out[s], ev[s], ev[s + 1]);
  for (auto& e : ev) (void)hipEventDestroy(e);
  for (void* q : {(void*)dm, (void*)dn, (void*)dl, (void*)df}) (void)hipFree(q);
  return st;
}

}  // extern "C"
