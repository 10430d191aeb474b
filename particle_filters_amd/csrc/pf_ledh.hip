// Host side of the MI355X LEDH particle-flow filter: the C ABI of include/pf_ledh.h.
//
// Turns LEDHFlowPF's call sequence (/root/reference/models/LEDH_particle_filter.py:
// init_from_gaussian 84-91, step 93-214) into launches of pf_ledh_kernels.h, and runs
// the whole T loop on the device (pf_ledh_run) with no host synchronisation inside T.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <optional>
#include <vector>

#include "../../include/pf_ledh.h"
#include "pf_hooks.h"
#include "pf_ledh_ekf.h"
#include "pf_ledh_kernels.h"
#include "pf_diag.h"
#include "pf_edh_kernels.h"
#include "pf_ledh_fused.h"
#include "pf_order.h"

namespace pf {
// the engine's thread-local error message (pf_last_error, pf_engine.hip)
void set_last_error(const std::string& msg);
namespace ledh {
static pf_status lfail(pf_status code, const std::string& msg) {
  set_last_error(msg);
  return code;
}

// size (doubles) of the shared-path flow table, TLay<nx, nz>::size(L); its aff block also holds
// the EDH general map (ELay: nx*nx + nx)
static size_t TLayHost(int nx, int nz, int L) {
  return (size_t)(nx + nz) + (size_t)L * (size_t)(nx * nz + nz * nz + nx + nz + 1) +
         std::max((size_t)(nx + nx * nz + nz + nz * nz + 1), (size_t)(nx * nx + nx));
}
#define LCHK(expr)                                                                          \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return lfail(PF_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct LOps {
  int nx, nz, tk, ok, psize;
  hipError_t (*setup)(const FlowParams&, double*, int, int, hipStream_t);  // (.., L, n_steps, ..)
  hipError_t (*flow_shared)(const FlowParams&, hipStream_t);
  hipError_t (*flow_wave)(const FlowParams&, int, hipStream_t);
  hipError_t (*normalise_chain)(const WParams&, hipStream_t);  // tile_max, exp_sum, normalise, decide
  hipError_t (*resample)(const WParams&, hipStream_t);
  hipError_t (*stats)(const WParams&, bool cov, hipStream_t);
  hipError_t (*init)(double*, double*, const double*, const double*, const double*, int64_t, int64_t, uint64_t,
                     uint32_t, hipStream_t);
  void (*prepare)();
  hipError_t (*ekf)(const double* Pm, const double* x0, const double* P0, const double* Qt, const double* Rt,
                    const double* Z, int64_t T, double* Ps, double* x_out, double* P_out, double* Xp, hipStream_t);
  // EDH (pf_edh_kernels.h): composed flow maps of n_steps time steps; the particle kernel (nonlinear h)
  hipError_t (*edh_setup)(const FlowParams&, double*, int, hipStream_t);
  hipError_t (*flow_edh)(const FlowParams&, hipStream_t);
  // the whole shared-path step in one cooperative launch (pf_ledh_fused.h); null for nonlinear h
  hipError_t (*fused)(const FusedParams&, hipStream_t);
  int (*fused_blocks_per_cu)();
  int fused_E;  // moment partial entries per workgroup
};

template <int NX, int NZ, int TK, int OK>
struct LL {
  // flow tables of n_steps time steps at once (P_k, z_k, table_k strided by the FlowParams strides)
  static hipError_t setup(const FlowParams& p, double* table, int L, int n_steps, hipStream_t s) {
    hipLaunchKernelGGL((k_setup<NX, NZ>), dim3(L, n_steps), dim3(SB), 0, s, p, table);
    const size_t lds = (size_t)L * (TLay<NX, NZ>::PJ) * sizeof(double);
    hipLaunchKernelGGL((k_compose<NX, NZ>), dim3(n_steps), dim3(SB), lds, s, table, p.lams, L, p.dlam,
                       p.table_stride);
    return hipGetLastError();
  }
  static hipError_t flow_shared(const FlowParams& p, hipStream_t s) {
    if constexpr (OK == PF_OBS_LINEAR) {
      const int64_t threads = p.N * Grp<NX>::GL;
      hipLaunchKernelGGL((k_flow_affine<NX, NZ, TK>), dim3((unsigned)((threads + TB - 1) / TB)), dim3(TB), 0, s, p);
      return hipGetLastError();
    } else {
      return hipErrorInvalidValue;
    }
  }
  static hipError_t flow_wave(const FlowParams& p, int grid, hipStream_t s) {
    if constexpr (OK == PF_OBS_ACOUSTIC) {
      // the acoustic h reads the positions only: the flow's algebra in their NX / 2 dimensions
      // (k_flow_wave_lr); PF_FLOW_LR=0 runs the observation-space kernel (A/B and the test that
      // compares the two), read per launch
      const char* lr_env = std::getenv("PF_FLOW_LR");
      const bool lr = !(lr_env && std::atoi(lr_env) == 0);
      if (lr && p.r_diag) {  // U = R^{-1/2} H8 by a diagonal scaling
        pf::lds_poison_hook(s);  // tests only (pf_hooks.h)
        FlowParams q = p;
        q.lr_force = pf::test_hook_int("PF_TEST_FLOW_LR_FORCE");  // tests only (pf_hooks.h)
        hipLaunchKernelGGL((k_flow_wave_lr<NX, NZ, TK>), dim3(grid), dim3(64), 0, s, q);
        return hipGetLastError();
      }
    }
    pf::lds_poison_hook(s);  // tests only (pf_hooks.h)
    hipLaunchKernelGGL((k_flow_wave<NX, NZ, TK, OK>), dim3(grid), dim3(64), 0, s, p);
    return hipGetLastError();
  }
  static hipError_t normalise_chain(const WParams& p, hipStream_t s) {
    if (p.N <= SMALL_N) {
      hipLaunchKernelGGL(k_weights_small, dim3(1), dim3(WB), (size_t)p.N * sizeof(double), s, p);
      return hipGetLastError();
    }
    hipLaunchKernelGGL(k_tile_max, dim3(p.G), dim3(TB), 0, s, p);
    hipLaunchKernelGGL(k_exp_sum, dim3(p.G), dim3(TB), 0, s, p);
    hipLaunchKernelGGL(k_normalise, dim3(p.G), dim3(TB), 0, s, p);
    hipLaunchKernelGGL(k_decide, dim3(1), dim3(TB), 0, s, p, 2);
    hipLaunchKernelGGL(k_cdf, dim3(p.G), dim3(TB), 0, s, p, 2);
    return hipGetLastError();
  }
  // ancestors + gather into x_out / w_out, or copy-through when the decision was "no resample"
  static hipError_t resample(const WParams& p, hipStream_t s) {
    const size_t lds = p.N <= GCAP ? (size_t)p.N * sizeof(double) : 0;
    hipLaunchKernelGGL((k_gather<NX>), dim3((unsigned)((p.N + TB - 1) / TB)), dim3(TB), lds, s, p);
    return hipGetLastError();
  }
  // posterior mean / cov (ledh.py:209, 217-224): one-pass shifted partials + final
  static hipError_t stats(const WParams& p, bool cov, hipStream_t s) {
    (void)cov;
    hipLaunchKernelGGL((k_mom_part<NX>), dim3(p.Gc), dim3(TB), 0, s, p);
    constexpr int NOUT = NX + NX * (NX + 1) / 2;
    hipLaunchKernelGGL((k_mom_final<NX>), dim3((NOUT + MF_E - 1) / MF_E), dim3(MF_E * MF_P), 0, s, p);
    return hipGetLastError();
  }
  static void prepare() {
    (void)hipFuncSetAttribute((const void*)k_gather<NX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(GCAP * sizeof(double)));
    (void)hipFuncSetAttribute((const void*)k_compose<NX, NZ>, hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024);
    (void)hipFuncSetAttribute((const void*)k_weights_small, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(SMALL_N * sizeof(double)));
  }
  static hipError_t init(double* x, double* w, const double* mean0, const double* Lc, const double* eps, int64_t N,
                         int64_t Npad, uint64_t seed, uint32_t epoch, hipStream_t s) {
    hipLaunchKernelGGL((k_init<NX>), dim3((unsigned)((N + TB - 1) / TB)), dim3(TB), 0, s, x, w, mean0, Lc, eps, N,
                       Npad, seed, epoch);
    return hipGetLastError();
  }
  static hipError_t ekf(const double* Pm, const double* x0, const double* P0, const double* Qt, const double* Rt,
                        const double* Z, int64_t T, double* Ps, double* x_out, double* P_out, double* Xp,
                        hipStream_t s) {
    pf::lds_poison_hook(s);  // tests only (pf_hooks.h)
    hipLaunchKernelGGL((k_ekf_seq<NX, NZ, TK, OK>), dim3(1), dim3(ekf_block<NZ>()), 0, s, Pm, x0, P0, Qt, Rt, Z, T, Ps, x_out, P_out,
                       Xp);
    return hipGetLastError();
  }
  static hipError_t fused(const FusedParams& p, hipStream_t s) {
    if constexpr (OK == PF_OBS_LINEAR) {
      pf::lds_poison_hook(s);  // tests only (pf_hooks.h)
      hipLaunchKernelGGL((k_ledh_fused<NX, NZ, TK>), dim3(p.nbk), dim3(FusedBlk<NX>::FB), 0, s, p);
      return hipGetLastError();
    } else {
      return hipErrorInvalidValue;
    }
  }
  static int fused_blocks_per_cu() {
    if constexpr (OK == PF_OBS_LINEAR) {
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k_ledh_fused<NX, NZ, TK>, FusedBlk<NX>::FB,
                                                       0) !=
          hipSuccess)
        return 0;
      return nb;
    } else {
      return 0;
    }
  }
  static hipError_t edh_setup(const FlowParams& p, double* table, int n_steps, hipStream_t s) {
    hipLaunchKernelGGL((k_edh_setup<NX, NZ, TK, OK>), dim3(n_steps), dim3(SB), 0, s, p, table);
    return hipGetLastError();
  }
  static hipError_t flow_edh(const FlowParams& p, hipStream_t s) {
    if constexpr (OK == PF_OBS_LINEAR) {
      return flow_shared(p, s);  // eta_L = eta0 + d0 + D (H eta0): the LEDH affine kernel, theta = 0
    } else {
      hipLaunchKernelGGL((k_flow_edh<NX, NZ, TK, OK>), dim3((unsigned)((p.N + TB - 1) / TB)), dim3(TB), 0, s, p);
      return hipGetLastError();
    }
  }
  static LOps make() {
    LOps o;
    o.ekf = &ekf;
    o.edh_setup = &edh_setup;
    o.fused = (OK == PF_OBS_LINEAR) ? &fused : nullptr;
    o.fused_blocks_per_cu = &fused_blocks_per_cu;
    o.fused_E = Mom<NX>::E;
    o.flow_edh = &flow_edh;
    o.nx = NX; o.nz = NZ; o.tk = TK; o.ok = OK;
    o.psize = Lay<NX, NZ>::SIZE;
    o.setup = &setup;
    o.flow_shared = (OK == PF_OBS_LINEAR) ? &flow_shared : nullptr;
    o.flow_wave = &flow_wave;
    o.normalise_chain = &normalise_chain;
    o.resample = &resample;
    o.stats = &stats;
    o.init = &init;
    o.prepare = &prepare;
    return o;
  }
};

// compiled LEDH model shapes
static const std::vector<LOps>& lregistry() {
  static const std::vector<LOps> r = {
      LL<1, 1, PF_TRANS_LINEAR, PF_OBS_LINEAR>::make(),      // linear 1-D (test_ledh_flow_pf.py fixtures)
      LL<1, 1, PF_TRANS_LINEAR, PF_OBS_EXP_HALF>::make(),    // SV, h = beta exp(x/2)
      LL<2, 1, PF_TRANS_LINEAR, PF_OBS_LINEAR>::make(),      // 2-D linear test system
      LL<4, 9, PF_TRANS_LINEAR, PF_OBS_ACOUSTIC>::make(),    // one acoustic target, 3x3 sensors
      LL<4, 12, PF_TRANS_LINEAR, PF_OBS_ACOUSTIC>::make(),   // one acoustic target, 3x4 sensors
      LL<4, 25, PF_TRANS_LINEAR, PF_OBS_ACOUSTIC>::make(),   // one acoustic target, 5x5 sensors
      LL<16, 25, PF_TRANS_LINEAR, PF_OBS_ACOUSTIC>::make(),  // joint 4-target acoustic tracking
      LL<40, 10, PF_TRANS_L96, PF_OBS_LINEAR>::make(),       // Lorenz-96 d = 40 (BASELINE config 5)
  };
  return r;
}
static const LOps* find_lops(int nx, int nz, int tk, int ok) {
  for (const LOps& o : lregistry())
    if (o.nx == nx && o.nz == nz && o.tk == tk && o.ok == ok) return &o;
  return nullptr;
}

static bool chol_lower(const double* A, int n, double jitter, std::vector<double>& L) {
  L.assign((size_t)n * n, 0.0);
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j] + jitter;
    for (int k = 0; k < j; ++k) d -= L[j * n + k] * L[j * n + k];
    if (!(d > 0.0) || !std::isfinite(d)) return false;
    const double ljj = std::sqrt(d);
    L[j * n + j] = ljj;
    for (int i = j + 1; i < n; ++i) {
      double s = A[i * n + j];
      for (int k = 0; k < j; ++k) s -= L[i * n + k] * L[j * n + k];
      L[i * n + j] = s / ljj;
    }
  }
  return true;
}

// inverse of an SPD matrix via its Cholesky factor
static bool spd_inverse(const double* A, int n, std::vector<double>& Ainv) {
  std::vector<double> L;
  if (!chol_lower(A, n, 0.0, L)) return false;
  Ainv.assign((size_t)n * n, 0.0);
  std::vector<double> col(n), y(n);
  for (int c = 0; c < n; ++c) {
    for (int i = 0; i < n; ++i) {
      double s = (i == c) ? 1.0 : 0.0;
      for (int k = 0; k < i; ++k) s -= L[i * n + k] * y[k];
      y[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
      double s = y[i];
      for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * col[k];
      col[i] = s / L[i * n + i];
    }
    for (int i = 0; i < n; ++i) Ainv[i * n + c] = col[i];
  }
  return true;
}

static bool is_diag(const double* A, int n) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      if (i != j && A[i * n + j] != 0.0) return false;
  return true;
}

}  // namespace ledh
}  // namespace pf

using namespace pf::ledh;
using pf::GridOrderScope;
using pf::grid_order_forget;

struct pf_ledh_handle {
  const LOps* ops = nullptr;
  int nx = 0, nz = 0, tk = 0, ok = 0;
  int64_t N = 0, Npad = 0;
  int L = 1, G = 1, Gc = 1;
  double dlam = 1.0, ratio = 0.0;
  uint64_t seed = 0;
  int device = 0;
  bool shared = false;
  int algo = 0;   // 0 LEDH, 1 EDH (pf_edh_create)
  int integ = 0;  // EDH integrator (PF_EDH_RK4 / PF_EDH_EULER)
  int q_diag = 0, r_diag = 0;
  uint32_t epoch = 1;
  bool initialized = false;
  bool pending = false;  // the last step decided to resample
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;  // tracker + flow tables, run ahead of the particle loop (pf_ledh_run_ekf)
  std::vector<double> lams;
  // device buffers
  double *x = nullptr, *x_alt = nullptr, *w = nullptr, *w_alt = nullptr, *lw = nullptr;
  double *tmax = nullptr, *tsum = nullptr, *trec = nullptr, *cdf = nullptr, *stat = nullptr, *mean = nullptr;
  double* mean_prev = nullptr;  // shift of the one-pass moments (ping-pong with mean)
  double* mean3 = nullptr;      // third mean buffer of the fused run (shift of two steps back)
  double *cpart = nullptr, *Pm = nullptr, *Pk = nullptr, *z = nullptr, *u = nullptr, *vbuf = nullptr;
  double* xbar = nullptr;  // EDH: tracker past mean of the current step
  // fused shared-path step (pf_ledh_fused.h): grid geometry, barrier words, partials
  int fused_nbk = 0, fused_ppb = 0;
  unsigned long long fphase = 0;
  unsigned long long *fpart = nullptr, *fcpart = nullptr;
  int fcp = 0;  // which half of fcpart the last fused step's P4 wrote
  int32_t* fanc = nullptr;  // [N] ancestors of the slots between fused steps
  // run_impl's device buffers (tracker covariances, observations, outputs, flow tables), one
  // allocation kept across runs: a run allocates only when it needs more than the last one
  char* arena = nullptr;
  size_t arena_bytes = 0;
  unsigned int* ferr = nullptr;
  double *table = nullptr, *d_lams = nullptr, *diagS = nullptr, *out = nullptr, *unif = nullptr, *Lc = nullptr;
  // replayed draws for the next run (pf_ledh_set_run_replay): noise [T][N][nx], U [T]
  double *rp_noise = nullptr, *rp_unif = nullptr;
  int64_t rp_T = 0;
};

namespace {

FlowParams flow_params(pf_ledh_handle* h, const double* Pk, const double* z, const double* u, int noise,
                       const double* v, double* diagS) {
  FlowParams p;
  p.x_in = h->x;
  p.x_out = h->x_alt;
  p.w_in = h->w;
  p.lw = h->lw;
  p.Pm = h->Pm;
  p.Pk = Pk;
  p.z = z;
  p.u = u;
  p.v_host = v;
  p.table = h->table;
  p.pk_stride = p.z_stride = p.table_stride = 0;
  p.lams = h->d_lams;
  p.diagS = diagS;
  p.N = h->N;
  p.Npad = h->Npad;
  p.L = h->L;
  p.dlam = h->dlam;
  p.noise = noise;
  p.seed = h->seed;
  p.epoch = h->epoch;
  p.q_diag = h->q_diag;
  p.r_diag = h->r_diag;
  p.xbar = nullptr;
  p.xbar_stride = p.u_stride = 0;
  p.integ = h->integ;
  return p;
}

WParams w_params(pf_ledh_handle* h) {
  WParams p;
  p.x_in = h->x;
  p.x_out = h->x_alt;
  p.lw = h->lw;
  p.w = h->w;
  p.w_out = h->w_alt;
  p.tmax = h->tmax;
  p.tsum = h->tsum;
  p.trec = h->trec;
  p.cdf = h->cdf;
  p.stat = h->stat;
  p.mean = h->mean;
  p.shift = h->mean_prev;
  p.cpart = h->cpart;
  p.o_mean = p.o_cov = p.o_ess = nullptr;
  p.o_flag = nullptr;
  p.unif = nullptr;
  p.N = h->N;
  p.Npad = h->Npad;
  p.G = h->G;
  p.Gc = h->Gc;
  p.ratio = h->ratio;
  p.seed = h->seed;
  p.epoch = 0;
  p.uniform = 0;
  return p;
}

// flow + weights + decision of one step (ledh.py:104-203), all enqueued on h->stream
pf_status enqueue_flow(pf_ledh_handle* h, const double* Pk, const double* z, const double* u, int noise,
                       const double* v, double* diagS, double* o_ess, int32_t* o_flag,
                       const double* pre_table = nullptr, const double* xbar = nullptr) {
  const uint32_t ep_noise = ++h->epoch;
  FlowParams fp = flow_params(h, Pk, z, u, noise, v, diagS);
  fp.epoch = ep_noise;
  if (h->algo == 1) {  // EDH: one composed affine map per step (pf_edh_kernels.h)
    if (pre_table) {
      fp.table = pre_table;
    } else {
      fp.xbar = xbar;
      LCHK(h->ops->edh_setup(fp, h->table, 1, h->stream));
    }
    LCHK(h->ops->flow_edh(fp, h->stream));
  } else if (h->shared) {
    if (pre_table) fp.table = pre_table;  // built for the whole run up front (pf_ledh_run)
    else LCHK(h->ops->setup(fp, h->table, h->L, 1, h->stream));
    LCHK(h->ops->flow_shared(fp, h->stream));
  } else {
    int grid = (int)std::min<int64_t>(h->N, 256 * 16);
    LCHK(h->ops->flow_wave(fp, grid, h->stream));
  }
  std::swap(h->x, h->x_alt);  // the flowed particles are current
  WParams wp = w_params(h);
  wp.o_ess = o_ess;
  wp.o_flag = o_flag;
  LCHK(h->ops->normalise_chain(wp, h->stream));
  return PF_OK;
}

// resample (flag on the device) + posterior moments of the current state
pf_status enqueue_finish(pf_ledh_handle* h, const double* U, double* o_mean, double* o_cov) {
  const uint32_t ep_res = ++h->epoch;
  WParams wp = w_params(h);
  wp.unif = U;
  wp.epoch = ep_res;
  LCHK(h->ops->resample(wp, h->stream));
  std::swap(h->x, h->x_alt);
  std::swap(h->w, h->w_alt);
  WParams sp = w_params(h);
  sp.o_mean = o_mean;
  sp.o_cov = o_cov;
  LCHK(h->ops->stats(sp, true, h->stream));
  std::swap(h->mean, h->mean_prev);  // the new mean is the next moments' shift
  return PF_OK;
}

pf_status sym_upload(pf_ledh_handle* h, const double* P, double* dst) {
  const int n = h->nx;
  std::vector<double> S((size_t)n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) S[i * n + j] = 0.5 * (P[i * n + j] + P[j * n + i]);  // ledh.py:106
  LCHK(hipMemcpyAsync(dst, S.data(), S.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
  LCHK(hipStreamSynchronize(h->stream));
  return PF_OK;
}

}  // namespace

extern "C" {

int32_t pf_ledh_model_supported(int32_t nx, int32_t nz, int32_t tk, int32_t ok) {
  return find_lops(nx, nz, tk, ok) != nullptr;
}

}  // extern "C"

// LEDHFlowPF.__init__ (ledh.py:63-81) / EDHFlowPF.__init__ (edh.py:138-171): algo 0 LEDH, 1 EDH
static pf_status create_impl(const pf_model_desc* m, const pf_ledh_opts* o, int algo, int integ,
                             pf_ledh_handle** out) {
  if (!m || !o || !out) return lfail(PF_E_ARG, "null argument");
  *out = nullptr;
  if (o->n_particles <= 0) return lfail(PF_E_ARG, "n_particles must be positive");
  if (o->n_particles > (int64_t)LT * MAXT) return lfail(PF_E_ARG, "n_particles too large (max 1048576)");
  const LOps* ops = find_lops(m->nx, m->nz, m->trans_kind, m->obs_kind);
  if (!ops)
    return lfail(PF_E_UNSUPPORTED, "LEDH model (nx=" + std::to_string(m->nx) + ", nz=" + std::to_string(m->nz) +
                                       ", g=" + std::to_string(m->trans_kind) + ", h=" + std::to_string(m->obs_kind) +
                                       ") is not compiled into libpf_hip");
  const int nx = m->nx, nz = m->nz;
  std::vector<double> P((size_t)ops->psize, 0.0);
  // Lay offsets (mirrors pf_ledh_kernels.h Lay<NX, NZ>)
  const int oA = 0, oEX = nx * nx, oH = oEX + 2, oC = oH + nz * nx, oAC = oC + nz, oLQ = oAC + 2 + 2 * nz,
            oQI = oLQ + nx * nx, oR = oQI + nx * nx, oRI = oR + nz * nz;
  if (m->trans_kind == PF_TRANS_LINEAR) {
    if (m->n_trans_params < (int64_t)nx * nx || !m->trans_params) return lfail(PF_E_ARG, "LINEAR g needs A[nx*nx]");
    for (int i = 0; i < nx * nx; ++i) P[oA + i] = m->trans_params[i];
  } else if (m->trans_kind == PF_TRANS_L96) {
    if (m->n_trans_params < 2 || !m->trans_params) return lfail(PF_E_ARG, "L96 g needs {F, dt}");
    P[oEX] = m->trans_params[0];
    P[oEX + 1] = m->trans_params[1];
  }
  if (m->obs_kind == PF_OBS_LINEAR) {
    if (m->n_obs_params < (int64_t)nz * nx + nz || !m->obs_params) return lfail(PF_E_ARG, "LINEAR h needs H, c");
    for (int i = 0; i < nz * nx; ++i) P[oH + i] = m->obs_params[i];
    for (int i = 0; i < nz; ++i) P[oC + i] = m->obs_params[nz * nx + i];
  } else if (m->obs_kind == PF_OBS_EXP_HALF) {
    if (m->n_obs_params < nz || !m->obs_params) return lfail(PF_E_ARG, "EXP_HALF h needs beta[nz]");
    for (int i = 0; i < nz; ++i) P[oC + i] = m->obs_params[i];
  } else if (m->obs_kind == PF_OBS_ACOUSTIC) {
    if (m->n_obs_params < 2 + 2 * nz || !m->obs_params) return lfail(PF_E_ARG, "ACOUSTIC h needs psi, d0, sx, sy");
    for (int i = 0; i < 2 + 2 * nz; ++i) P[oAC + i] = m->obs_params[i];
  }
  if (!m->Q || !m->R) return lfail(PF_E_ARG, "Q and R are required");
  std::vector<double> Lq, Qi, Ri;
  if (!chol_lower(m->Q, nx, 0.0, Lq) && !chol_lower(m->Q, nx, 1e-10, Lq))
    return lfail(PF_E_NOT_PD, "Matrix is not positive definite (Q)");
  if (!spd_inverse(m->Q, nx, Qi)) return lfail(PF_E_NOT_PD, "Matrix is not positive definite (Q)");
  if (!spd_inverse(m->R, nz, Ri)) return lfail(PF_E_NOT_PD, "Matrix is not positive definite (R)");
  for (int i = 0; i < nx * nx; ++i) {
    P[oLQ + i] = Lq[i];
    P[oQI + i] = Qi[i];
  }
  for (int i = 0; i < nz * nz; ++i) {
    P[oR + i] = m->R[i];
    P[oRI + i] = Ri[i];
  }
  LCHK(hipSetDevice(o->device));
  pf_ledh_handle* h = new pf_ledh_handle();
  h->ops = ops;
  h->nx = nx; h->nz = nz; h->tk = m->trans_kind; h->ok = m->obs_kind;
  h->N = o->n_particles;
  h->Npad = (h->N + 3) / 4 * 4;
  h->L = std::max(1, (int)o->n_lambda);                   // ledh.py:132
  h->algo = algo;
  h->integ = integ;
  // the shared-Jacobian path stages its whole flow table in LDS; past that size (many lambda
  // steps) a linear h takes the per-particle flow instead (the same flow, particle by particle)
  const bool table_fits = (size_t)h->L * (size_t)(nx * nz + nz * nz + nx + nz + 1) * 8 <= 120 * 1024;
  h->dlam = 1.0 / (double)h->L;                           // ledh.py:133
  double lam = 0.0;
  for (int j = 0; j < h->L; ++j) {                        // ledh.py:134-137
    lam = std::min(1.0, lam + h->dlam);
    h->lams.push_back(lam);
  }
  h->ratio = o->resample_ess_ratio;
  h->seed = o->seed;
  h->device = o->device;
  h->shared = ops->flow_shared && o->flow_mode == PF_LEDH_FLOW_AUTO && (algo != 0 || table_fits);
  h->q_diag = is_diag(Qi.data(), nx);
  h->r_diag = is_diag(Ri.data(), nz);
  h->G = (int)((h->N + LT - 1) / LT);
  h->Gc = (int)((h->N + CT * CTS - 1) / (CT * CTS));
  auto bail = [&](const char* what) {
    pf_ledh_destroy(h);
    return lfail(PF_E_HIP, std::string("hipMalloc failed: ") + what);
  };
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) return bail("stream");
  if (hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking) != hipSuccess) return bail("stream");
  const size_t xb = (size_t)nx * h->Npad * sizeof(double), nb = (size_t)h->N * sizeof(double);
  const int NP = nx * (nx + 1) / 2;
  struct A { double** p; size_t b; };
  A allocs[] = {{&h->x, xb}, {&h->x_alt, xb}, {&h->w, nb}, {&h->w_alt, nb}, {&h->lw, nb}, {&h->cdf, nb},
                {&h->tmax, (size_t)h->G * 8}, {&h->tsum, (size_t)h->G * 8}, {&h->trec, (size_t)h->G * (2 + nx) * 8},
                {&h->stat, 8 * 8}, {&h->mean, (size_t)nx * 8}, {&h->mean_prev, (size_t)nx * 8}, {&h->mean3, (size_t)nx * 8},
                {&h->cpart, (size_t)h->Gc * (1 + nx + NP) * 8},
                {&h->Pm, P.size() * 8}, {&h->Pk, (size_t)nx * nx * 8}, {&h->z, (size_t)nz * 8},
                {&h->u, (size_t)nx * 8}, {&h->table, (size_t)TLayHost(nx, nz, h->L) * 8}, {&h->d_lams, (size_t)h->L * 8},
                {&h->diagS, (size_t)h->L * nz * nz * 8}, {&h->out, (size_t)(nx + nx * nx + 2) * 8},
                {&h->unif, 8}, {&h->Lc, (size_t)nx * nx * 8}};
  for (auto& a : allocs)
    if (hipMalloc((void**)a.p, a.b) != hipSuccess) return bail("state");
  (void)hipMemset(h->x, 0, xb);
  (void)hipMemset(h->x_alt, 0, xb);
  (void)hipMemset(h->mean, 0, (size_t)nx * 8);
  (void)hipMemset(h->mean_prev, 0, (size_t)nx * 8);
  ops->prepare();
  if (hipMemcpy(h->Pm, P.data(), P.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->d_lams, h->lams.data(), h->lams.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
    return bail("upload");
  if (algo == 1 && hipMalloc((void**)&h->xbar, (size_t)nx * 8) != hipSuccess) return bail("xbar");
  // fused step geometry: <= one workgroup per CU, all co-resident (PF_LEDH_FUSED=0 disables)
  {
    const char* env = std::getenv("PF_LEDH_FUSED");
    const bool want = ops->fused && (h->shared || algo == 1) && !(env && env[0] == '0');
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device);
    const int per_cu = want ? ops->fused_blocks_per_cu() : 0;
    int64_t ppb = 64;
    while ((h->N + ppb - 1) / ppb > FMAX && ppb < FPPB) ppb += 64;
    const int64_t nbk = (h->N + ppb - 1) / ppb;
    if (want && nbk <= FMAX && nbk <= (int64_t)per_cu * cus) {
      h->fused_nbk = (int)nbk;
      h->fused_ppb = (int)ppb;
      if (hipMalloc((void**)&h->fpart, 8 * FMAX * 8) != hipSuccess ||
          hipMalloc((void**)&h->fcpart, 2 * (size_t)FMAX * ops->fused_E * 8) != hipSuccess ||
          hipMalloc((void**)&h->fanc, (size_t)h->N * sizeof(int32_t)) != hipSuccess ||
          hipMalloc((void**)&h->ferr, 8) != hipSuccess)
        return bail("fused step buffers");
      (void)hipMemset(h->fpart, 0, 8 * FMAX * 8);  // tag 0: never a launch's (tags start at 1)
      (void)hipMemset(h->ferr, 0, 8);
    }
  }
  *out = h;
  return PF_OK;
}

extern "C" {

pf_status pf_ledh_create(const pf_model_desc* m, const pf_ledh_opts* o, pf_ledh_handle** out) {
  return create_impl(m, o, 0, 0, out);
}

pf_status pf_edh_create(const pf_model_desc* m, const pf_edh_opts* o, pf_ledh_handle** out) {
  if (!o) return lfail(PF_E_ARG, "null argument");
  if (o->integrator != PF_EDH_RK4 && o->integrator != PF_EDH_EULER) return lfail(PF_E_ARG, "bad EDH integrator");
  pf_ledh_opts lo;
  lo.n_particles = o->n_particles;
  lo.n_lambda = o->n_lambda;
  lo.resample_ess_ratio = o->resample_ess_ratio;
  lo.seed = o->seed;
  lo.device = o->device;
  lo.flow_mode = PF_LEDH_FLOW_AUTO;
  return create_impl(m, &lo, 1, o->integrator, out);
}

int32_t pf_edh_is_edh(pf_ledh_handle* h) { return (h && h->algo == 1) ? 1 : 0; }

void pf_ledh_destroy(pf_ledh_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (double* p : {h->x, h->x_alt, h->w, h->w_alt, h->lw, h->tmax, h->tsum, h->trec, h->cdf, h->stat, h->mean, h->mean_prev, h->mean3,
                    h->cpart, h->Pm, h->Pk, h->z, h->u, h->vbuf, h->table, h->d_lams, h->diagS, h->out, h->unif, h->Lc,
                    h->xbar, h->rp_noise, h->rp_unif})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)h->fpart, (void*)h->fcpart, (void*)h->fanc, (void*)h->ferr, (void*)h->arena})
    if (p) (void)hipFree(p);
  if (h->side) (void)hipStreamSynchronize(h->side);
  if (h->side) (void)hipStreamDestroy(h->side);
  if (h->stream) grid_order_forget(h->device, h->stream);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

pf_status pf_ledh_init(pf_ledh_handle* h, const double* mean0, const double* cov0, const double* eps,
                       double* mean_out, double* cov_out) {
  if (!h || !mean0 || !cov0) return lfail(PF_E_ARG, "null argument");
  LCHK(hipSetDevice(h->device));
  const int nx = h->nx;
  std::vector<double> L;
  if (!eps && !chol_lower(cov0, nx, 0.0, L) && !chol_lower(cov0, nx, 1e-10, L))
    return lfail(PF_E_NOT_PD, "Matrix is not positive definite (cov0)");
  if (eps) L.assign((size_t)nx * nx, 0.0);
  double* dm = h->out;  // staging: mean0 in out[0..nx)
  double* deps = nullptr;
  LCHK(hipMemcpyAsync(dm, mean0, nx * 8, hipMemcpyHostToDevice, h->stream));
  LCHK(hipMemcpyAsync(h->Lc, L.data(), L.size() * 8, hipMemcpyHostToDevice, h->stream));
  if (eps) {
    if (!h->vbuf) LCHK(hipMalloc((void**)&h->vbuf, (size_t)h->N * nx * 8));
    LCHK(hipMemcpyAsync(h->vbuf, eps, (size_t)h->N * nx * 8, hipMemcpyHostToDevice, h->stream));
    deps = h->vbuf;
  }
  h->epoch = 1;
  LCHK(h->ops->init(h->x, h->w, dm, h->Lc, deps, h->N, h->Npad, h->seed, h->epoch, h->stream));
  // _weighted_stats of the initial set (ledh.py:90): mean -> h->mean, cov -> out[nx : nx + nx*nx)
  WParams sp = w_params(h);
  sp.uniform = 1;
  sp.o_cov = h->out + nx;
  LCHK(h->ops->stats(sp, true, h->stream));
  std::swap(h->mean, h->mean_prev);  // the new mean is the next moments' shift
  LCHK(hipStreamSynchronize(h->stream));
  if (mean_out) LCHK(hipMemcpy(mean_out, h->mean_prev, nx * 8, hipMemcpyDeviceToHost));
  if (cov_out) LCHK(hipMemcpy(cov_out, h->out + nx, (size_t)nx * nx * 8, hipMemcpyDeviceToHost));
  h->initialized = true;
  h->pending = false;
  return PF_OK;
}

static pf_status step_impl(pf_ledh_handle* h, const double* P, const double* xbar, const double* z, const double* u,
                           int32_t noise, const double* v, pf_ledh_info* info, double* cond_S);

pf_status pf_ledh_step(pf_ledh_handle* h, const double* P, const double* z, const double* u, int32_t noise,
                       const double* v, pf_ledh_info* info, double* cond_S) {
  if (h && h->algo == 1) return lfail(PF_E_ARG, "EDH handle: use pf_edh_step (it needs the tracker's past mean)");
  return step_impl(h, P, nullptr, z, u, noise, v, info, cond_S);
}

pf_status pf_edh_step(pf_ledh_handle* h, const double* P, const double* xbar, const double* z, const double* u,
                      int32_t noise, const double* v, pf_ledh_info* info, double* cond_S) {
  if (h && h->algo != 1) return lfail(PF_E_ARG, "pf_edh_step needs a handle from pf_edh_create");
  if (!xbar) return lfail(PF_E_ARG, "null argument");
  return step_impl(h, P, xbar, z, u, noise, v, info, cond_S);
}

}  // extern "C"

static pf_status step_impl(pf_ledh_handle* h, const double* P, const double* xbar, const double* z, const double* u,
                           int32_t noise, const double* v, pf_ledh_info* info, double* cond_S) {
  if (!h || !P || !z) return lfail(PF_E_ARG, "null argument");
  if (!h->initialized) return lfail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  if (noise == PF_NOISE_HOST && !v) return lfail(PF_E_ARG, "PF_NOISE_HOST needs v");
  if (noise < PF_NOISE_NONE || noise > PF_NOISE_DEVICE) return lfail(PF_E_ARG, "bad noise mode");
  LCHK(hipSetDevice(h->device));
  if (sym_upload(h, P, h->Pk) != PF_OK) return PF_E_HIP;
  LCHK(hipMemcpyAsync(h->z, z, h->nz * 8, hipMemcpyHostToDevice, h->stream));
  if (u) LCHK(hipMemcpyAsync(h->u, u, h->nx * 8, hipMemcpyHostToDevice, h->stream));
  if (xbar) LCHK(hipMemcpyAsync(h->xbar, xbar, h->nx * 8, hipMemcpyHostToDevice, h->stream));
  if (noise == PF_NOISE_HOST) {
    if (!h->vbuf) LCHK(hipMalloc((void**)&h->vbuf, (size_t)h->N * h->nx * 8));
    LCHK(hipMemcpyAsync(h->vbuf, v, (size_t)h->N * h->nx * 8, hipMemcpyHostToDevice, h->stream));
  }
  pf_status st = enqueue_flow(h, h->Pk, h->z, u ? h->u : nullptr, noise, noise == PF_NOISE_HOST ? h->vbuf : nullptr,
                              cond_S ? h->diagS : nullptr, nullptr, nullptr, nullptr, xbar ? h->xbar : nullptr);
  if (st != PF_OK) return st;
  double stat[3];
  LCHK(hipMemcpyAsync(stat, h->stat, 3 * 8, hipMemcpyDeviceToHost, h->stream));
  LCHK(hipStreamSynchronize(h->stream));
  if (cond_S) LCHK(hipMemcpy(cond_S, h->diagS, (size_t)h->L * h->nz * h->nz * 8, hipMemcpyDeviceToHost));
  h->pending = stat[1] != 0.0;
  if (info) {
    info->ess = stat[0];
    info->resample = h->pending ? 1 : 0;
    info->_pad = 0;
  }
  return PF_OK;
}

extern "C" {

pf_status pf_ledh_finish(pf_ledh_handle* h, const double* U, double* mean, double* cov) {
  if (!h) return lfail(PF_E_ARG, "null argument");
  if (!h->initialized) return lfail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  LCHK(hipSetDevice(h->device));
  const int nx = h->nx;
  if (h->pending && U) LCHK(hipMemcpyAsync(h->unif, U, 8, hipMemcpyHostToDevice, h->stream));
  if (h->pending) {
    const uint32_t ep_res = ++h->epoch;
    WParams wp = w_params(h);
    wp.unif = U ? h->unif : nullptr;
    wp.epoch = ep_res;
    LCHK(h->ops->resample(wp, h->stream));
    std::swap(h->x, h->x_alt);
    std::swap(h->w, h->w_alt);
    h->pending = false;
  }
  WParams sp = w_params(h);
  sp.o_cov = h->out + nx;
  LCHK(h->ops->stats(sp, true, h->stream));
  std::swap(h->mean, h->mean_prev);  // the new mean is the next moments' shift
  LCHK(hipStreamSynchronize(h->stream));
  if (mean) LCHK(hipMemcpy(mean, h->mean_prev, nx * 8, hipMemcpyDeviceToHost));
  if (cov) LCHK(hipMemcpy(cov, h->out + nx, (size_t)nx * nx * 8, hipMemcpyDeviceToHost));
  return PF_OK;
}

pf_status pf_ledh_get_particles(pf_ledh_handle* h, double* particles) {
  if (!h || !particles) return lfail(PF_E_ARG, "null argument");
  if (!h->initialized) return lfail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  LCHK(hipSetDevice(h->device));
  std::vector<double> soa((size_t)h->nx * h->Npad);
  LCHK(hipStreamSynchronize(h->stream));
  LCHK(hipMemcpy(soa.data(), h->x, soa.size() * 8, hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < h->N; ++i)
    for (int d = 0; d < h->nx; ++d) particles[i * h->nx + d] = soa[(size_t)d * h->Npad + i];
  return PF_OK;
}

pf_status pf_ledh_get_weights(pf_ledh_handle* h, double* weights) {
  if (!h || !weights) return lfail(PF_E_ARG, "null argument");
  if (!h->initialized) return lfail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  LCHK(hipSetDevice(h->device));
  LCHK(hipStreamSynchronize(h->stream));
  LCHK(hipMemcpy(weights, h->w, (size_t)h->N * 8, hipMemcpyDeviceToHost));
  return PF_OK;
}

// diag:61-91 on the device-resident state (include/pf_diag.h)
pf_status pf_ledh_diagnostics(pf_ledh_handle* h, double tol, pf_diagnostics* out) {
  if (!h || !out) return lfail(PF_E_ARG, "null argument");
  if (!h->initialized) return lfail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  LCHK(hipSetDevice(h->device));
  pf::diag::DiagSrc s{};
  s.N = h->N;
  s.Npad = h->Npad;
  s.nx = h->nx;
  s.w = h->w;
  s.x = h->x;
  s.real_is_double = 1;
  s.tol = tol;
  s.spread = NAN;
  return pf::diag::compute(s, h->stream, out);
}

pf_status pf_ledh_set_state(pf_ledh_handle* h, const double* particles, const double* weights) {
  if (!h || !particles || !weights) return lfail(PF_E_ARG, "null argument");
  LCHK(hipSetDevice(h->device));
  std::vector<double> soa((size_t)h->nx * h->Npad, 0.0);
  for (int64_t i = 0; i < h->N; ++i)
    for (int d = 0; d < h->nx; ++d) soa[(size_t)d * h->Npad + i] = particles[i * h->nx + d];
  LCHK(hipStreamSynchronize(h->stream));
  LCHK(hipMemcpy(h->x, soa.data(), soa.size() * 8, hipMemcpyHostToDevice));
  LCHK(hipMemcpy(h->w, weights, (size_t)h->N * 8, hipMemcpyHostToDevice));
  h->initialized = true;
  h->pending = false;
  return PF_OK;
}

}  // extern "C"

namespace {

// Device EKF spec: host arrays (x0, P0, Qt, Rt) or all null.
struct EkfSpec {
  const double *x0, *P0, *Qt, *Rt;
  double *x_final, *P_final;
};

// The T loop (pf_ledh_run / pf_ledh_run_ekf): tracker covariances from the host (Ps) or from the
// device EKF, all flow tables built up front, then flow -> weights -> resample -> moments per step.
// EDH handles also take the tracker's past means Xb [T][nx] (host) or get them from the device EKF.
// test hook (pf_hooks.h): PF_TEST_LEDH_FAIL=1 reports the fused grid barrier as timed out after a
// completed run
bool test_barrier_fail() { return pf::test_hook("PF_TEST_LEDH_FAIL"); }

pf_status run_impl(pf_ledh_handle* h, const double* Ps, const double* Xb, const EkfSpec* ekf, const double* Z,
                   const double* U, int64_t T, int32_t noise, double* means, double* covs, double* ess,
                   uint8_t* flags) {
  if (!h || !Z || (!Ps && !ekf)) return lfail(PF_E_ARG, "null argument");
  const bool edh = h->algo == 1;
  if (edh && !ekf && !Xb) return lfail(PF_E_ARG, "EDH run needs the tracker's past means");
  if (!h->initialized) return lfail(PF_E_NOT_INITIALIZED, "Filter not initialized.");
  if (noise == PF_NOISE_HOST && h->rp_T != T)
    return lfail(PF_E_ARG, "run: PF_NOISE_HOST needs pf_ledh_set_run_replay with the run's T");
  if (noise < PF_NOISE_NONE || noise > PF_NOISE_DEVICE) return lfail(PF_E_ARG, "run: bad noise mode");
  const bool replay = noise == PF_NOISE_HOST;
  if (T <= 0) return PF_OK;
  LCHK(hipSetDevice(h->device));
  const int nx = h->nx, nz = h->nz;
  std::vector<double> S;
  if (Ps) {
    S.resize((size_t)T * nx * nx);
    for (int64_t t = 0; t < T; ++t)
      for (int i = 0; i < nx; ++i)
        for (int j = 0; j < nx; ++j)
          S[(t * nx + i) * nx + j] = 0.5 * (Ps[(t * nx + i) * nx + j] + Ps[(t * nx + j) * nx + i]);  // ledh.py:106
  }
  double *dP = nullptr, *dZ = nullptr, *dU = nullptr, *dm = nullptr, *dc = nullptr, *de = nullptr, *dTab = nullptr;
  double* dE = nullptr;  // EKF inputs / outputs: x0 | P0 | Qt | Rt | x_final | P_final
  double* dX = nullptr;  // EDH: past means [T][nx]
  int32_t* df = nullptr;
  auto cleanup = [&]() {};  // the buffers live in the handle's arena
  const size_t ne = 2 * (size_t)nx + 3 * (size_t)nx * nx + (size_t)nz * nz;
  const size_t tsz = TLayHost(nx, nz, h->L);
  const bool tabled = h->shared || edh;
  {
    struct Piece { void** p; size_t b; };
    const Piece pieces[] = {{(void**)&dP, (size_t)T * nx * nx * 8}, {(void**)&dZ, (size_t)T * nz * 8},
                            {(void**)&dU, U ? (size_t)T * nx * 8 : 0}, {(void**)&dm, (size_t)T * nx * 8},
                            {(void**)&dc, (size_t)T * nx * nx * 8}, {(void**)&de, (size_t)T * 8},
                            {(void**)&df, (size_t)T * 4}, {(void**)&dE, ekf ? ne * 8 : 0},
                            {(void**)&dX, edh ? (size_t)T * nx * 8 : 0}, {(void**)&dTab, tabled ? (size_t)T * tsz * 8 : 0}};
    size_t need = 0;
    for (const Piece& q : pieces) need += (q.b + 255) / 256 * 256;
    if (need > h->arena_bytes) {
      if (h->arena) {
        (void)hipStreamSynchronize(h->stream);
        (void)hipStreamSynchronize(h->side);
        (void)hipFree(h->arena);
        h->arena = nullptr;
        h->arena_bytes = 0;
      }
      if (hipMalloc((void**)&h->arena, need) != hipSuccess) return lfail(PF_E_HIP, "hipMalloc of run buffers failed");
      h->arena_bytes = need;
    }
    size_t off = 0;
    for (const Piece& q : pieces) {
      *q.p = q.b ? (void*)(h->arena + off) : nullptr;
      off += (q.b + 255) / 256 * 256;
    }
  }
  pf_status st = PF_OK;
  bool touched = false;
  do {
    if ((Ps && hipMemcpyAsync(dP, S.data(), S.size() * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess) ||
        hipMemcpyAsync(dZ, Z, (size_t)T * nz * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
        (U && hipMemcpyAsync(dU, U, (size_t)T * nx * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess) ||
        (edh && !ekf && hipMemcpyAsync(dX, Xb, (size_t)T * nx * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess)) {
      st = lfail(PF_E_HIP, "upload of run inputs failed");
      break;
    }
    double *ex0 = dE, *eP0 = dE + nx, *eQ = eP0 + nx * nx, *eR = eQ + nx * nx, *exf = eR + nz * nz, *ePf = exf + nx;
    // flow tables of steps [c0, c0 + n) (they depend on (P_k, z_k) only, not on the particles)
    auto tables = [&](int64_t c0, int64_t n, hipStream_t s) -> bool {
      if (!tabled) return true;
      FlowParams fp = flow_params(h, dP + c0 * nx * nx, dZ + c0 * nz, nullptr, noise, nullptr, nullptr);
      fp.pk_stride = (int64_t)nx * nx;
      fp.z_stride = nz;
      fp.table_stride = (int64_t)tsz;
      if (edh) {
        fp.xbar = dX + c0 * nx;
        fp.xbar_stride = nx;
        fp.u = dU ? dU + c0 * nx : nullptr;
        fp.u_stride = nx;
        return h->ops->edh_setup(fp, dTab + c0 * tsz, (int)n, s) == hipSuccess;
      }
      return h->ops->setup(fp, dTab + c0 * tsz, h->L, (int)n, s) == hipSuccess;
    };
    // Device tracker: the EKF and the tables run on the side stream in chunks of steps, ahead of the
    // particle loop, which waits for each chunk's event (the tracker never needs the particles).  The
    // chunks grow 2, 4, 8, 16, 16, ...: the loop starts after two EKF steps, not sixteen.
    const int64_t CH = 16;
    std::vector<int64_t> cbeg;  // first step of each chunk
    for (int64_t c0 = 0, n = 2; c0 < T; c0 += n, n = std::min(CH, 2 * n)) cbeg.push_back(c0);
    std::vector<hipEvent_t> evs;
    if (ekf) {
      if (hipMemcpyAsync(ex0, ekf->x0, nx * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
          hipMemcpyAsync(eP0, ekf->P0, (size_t)nx * nx * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
          hipMemcpyAsync(eQ, ekf->Qt, (size_t)nx * nx * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
          hipMemcpyAsync(eR, ekf->Rt, (size_t)nz * nz * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
          hipMemcpyAsync(exf, ex0, nx * 8, hipMemcpyDeviceToDevice, h->stream) != hipSuccess ||
          hipMemcpyAsync(ePf, eP0, (size_t)nx * nx * 8, hipMemcpyDeviceToDevice, h->stream) != hipSuccess) {
        st = lfail(PF_E_HIP, "run: EKF input upload failed");
        break;
      }
      hipEvent_t up;
      if (hipEventCreateWithFlags(&up, hipEventDisableTiming) != hipSuccess || hipEventRecord(up, h->stream) != hipSuccess ||
          hipStreamWaitEvent(h->side, up, 0) != hipSuccess) {
        st = lfail(PF_E_HIP, "run: event setup failed");
        break;
      }
      evs.push_back(up);
      for (size_t k = 0; k < cbeg.size() && st == PF_OK; ++k) {
        const int64_t c0 = cbeg[k], n = (k + 1 < cbeg.size() ? cbeg[k + 1] : T) - c0;
        hipEvent_t ev;
        if (h->ops->ekf(h->Pm, exf, ePf, eQ, eR, dZ + c0 * nz, n, dP + c0 * nx * nx, exf, ePf,
                        edh ? dX + c0 * nx : nullptr, h->side) != hipSuccess ||
            !tables(c0, n, h->side) || hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(ev, h->side) != hipSuccess) {
          st = lfail(PF_E_HIP, "run: device EKF / flow-table launch failed");
          break;
        }
        evs.push_back(ev);
      }
    } else {
      for (int64_t c0 = 0; c0 < T && st == PF_OK; c0 += 65535)  // grid.y <= 65535 steps per launch
        if (!tables(c0, std::min<int64_t>(65535, T - c0), h->stream))
          st = lfail(PF_E_HIP, "run: batched flow-table launch failed");
    }
    const bool fused_run = h->fused_nbk > 0 && dTab;
    std::optional<GridOrderScope> order;  // no overlap with another handle's grid
    if (fused_run) order.emplace(h->device, h->stream);
    // fused path: launch t also reduces step t - 1's moments (its P5'); step t's moment shift is the
    // mean of step t - 2 (the latest mean before the run for t < 2); a P5-only launch ends the run.
    // shp: the shift step t - 1 used, shc: step t's, mw: where launch t puts the mean of step t - 1
    double* const mbuf[3] = {h->mean_prev, h->mean, h->mean3};
    double* shp = h->mean_prev;
    double* shc = h->mean_prev;
    double* mw = h->mean;
    double* spare = h->mean3;
    // and the state between its steps is (the last step's flow rows, ancestors): xa holds the rows
    // the next step starts from, xb takes its flow rows
    double* xa = h->x;
    double* xb = h->x_alt;
    auto fused_common = [&](FusedParams& fp) {
      fp.stat = h->stat;
      fp.part = h->fpart;
      // moment partials: P5' reads the pair's buffer the previous step's P4 wrote, P4 the other
      const size_t cps = (size_t)FMAX * h->ops->fused_E;
      fp.cpart5 = h->fcpart + h->fcp * cps;
      fp.cpart = h->fcpart + (h->fcp ^ 1) * cps;
      if (fp.step) h->fcp ^= 1;
      fp.err = h->ferr;
      fp.phase0 = h->fphase;
      h->fphase += 4;
      fp.ratio = h->ratio;
      fp.nbk = h->fused_nbk;
      fp.ppb = h->fused_ppb;
    };
    size_t next_chunk = 0;
    touched = true;  // from here on a failure leaves the particle state part-advanced
    for (int64_t t = 0; t < T && st == PF_OK; ++t) {
      if (ekf && next_chunk < cbeg.size() && t == cbeg[next_chunk] &&
          hipStreamWaitEvent(h->stream, evs[1 + next_chunk++], 0) != hipSuccess) {
        st = lfail(PF_E_HIP, "run: stream wait failed");
        break;
      }
      if (fused_run) {  // the whole step in one launch (pf_ledh_fused.h)
        FusedParams fp{};
        fp.f = flow_params(h, dP + t * nx * nx, dZ + t * nz, dU ? dU + t * nx : nullptr, noise,
                           replay ? h->rp_noise + t * h->N * nx : nullptr, nullptr);
        fp.f.table = dTab + t * tsz;
        fp.f.x_in = xa;
        fp.f.x_out = xb;
        fp.anc_in = t > 0 ? h->fanc : nullptr;
        fp.anc_out = h->fanc;
        fp.rp_unif = replay ? h->rp_unif + t : nullptr;
        fp.f.epoch = ++h->epoch;
        fp.ep_res = ++h->epoch;
        fp.w_out = h->w_alt;
        fp.step = 1;
        fp.p5 = t > 0;
        if (t > 0) {
          fp.shift5 = shp;
          fp.mean5 = mw;
          fp.o_mean5 = dm + (t - 1) * nx;
          fp.o_cov5 = dc + (t - 1) * nx * nx;
        }
        fp.shift = shc;
        fp.o_ess = de + t;
        fp.o_flag = df + t;
        fused_common(fp);
        if (h->ops->fused(fp, h->stream) != hipSuccess) {
          st = lfail(PF_E_HIP, "run: fused step launch failed");
          break;
        }
        std::swap(h->w, h->w_alt);
        std::swap(xa, xb);
        if (t > 0) {  // step t + 1: shifts (mean of t - 1 now in mw); the free buffer takes the next mean
          double* freed = shp != shc ? shp : spare;
          shp = shc;
          shc = mw;
          mw = freed;
        }  // (t = 0: steps 0 and 1 both shift by the latest mean before the run)
        continue;
      }
      st = enqueue_flow(h, dP + t * nx * nx, dZ + t * nz, dU ? dU + t * nx : nullptr, noise,
                        replay ? h->rp_noise + t * h->N * nx : nullptr, nullptr, de + t, df + t,
                        dTab ? dTab + t * tsz : nullptr);
      if (st == PF_OK) st = enqueue_finish(h, replay ? h->rp_unif + t : nullptr, dm + t * nx, dc + t * nx * nx);
    }
    if (fused_run && st == PF_OK) {  // the last step's outputs and the materialised state
      FusedParams fp{};
      fp.f.N = h->N;
      fp.f.Npad = h->Npad;
      fp.f.x_in = xa;
      fp.anc_in = h->fanc;
      fp.x_res = xb;
      h->x = xb;
      h->x_alt = xa;
      fp.step = 0;
      fp.p5 = 1;
      fp.shift5 = shp;
      fp.mean5 = mw;
      fp.o_mean5 = dm + (T - 1) * nx;
      fp.o_cov5 = dc + (T - 1) * nx * nx;
      fused_common(fp);
      if (h->ops->fused(fp, h->stream) != hipSuccess) st = lfail(PF_E_HIP, "run: fused tail launch failed");
      h->mean_prev = mw;  // the latest mean: the next moments' shift
      int k = 0;
      for (double* m : mbuf)
        if (m != mw) (k++ == 0 ? h->mean : h->mean3) = m;
    }
    if (order) order->end();
    if (ekf) (void)hipStreamSynchronize(h->side);
    for (hipEvent_t ev : evs) (void)hipEventDestroy(ev);
    if (st != PF_OK) break;
    if (hipStreamSynchronize(h->stream) != hipSuccess) {
      st = lfail(PF_E_HIP, "run: stream synchronisation failed");
      break;
    }
    if (h->ferr) {
      unsigned int fe = 0;
      if (hipMemcpy(&fe, h->ferr, 4, hipMemcpyDeviceToHost) != hipSuccess || fe != 0u || test_barrier_fail()) {
        (void)hipMemset(h->ferr, 0, 8);
        st = lfail(PF_E_HIP, "run: fused step grid barrier timed out (workgroups not co-resident)");
        break;
      }
    }
    std::vector<int32_t> fl((size_t)T);
    if ((means && hipMemcpy(means, dm, (size_t)T * nx * 8, hipMemcpyDeviceToHost) != hipSuccess) ||
        (covs && hipMemcpy(covs, dc, (size_t)T * nx * nx * 8, hipMemcpyDeviceToHost) != hipSuccess) ||
        (ess && hipMemcpy(ess, de, (size_t)T * 8, hipMemcpyDeviceToHost) != hipSuccess) ||
        hipMemcpy(fl.data(), df, (size_t)T * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        (ekf && ekf->x_final && hipMemcpy(ekf->x_final, exf, nx * 8, hipMemcpyDeviceToHost) != hipSuccess) ||
        (ekf && ekf->P_final && hipMemcpy(ekf->P_final, ePf, (size_t)nx * nx * 8, hipMemcpyDeviceToHost) != hipSuccess)) {
      st = lfail(PF_E_HIP, "download of run outputs failed");
      break;
    }
    if (flags)
      for (int64_t t = 0; t < T; ++t) flags[t] = fl[t] ? 1 : 0;
  } while (false);
  cleanup();
  h->pending = false;
  h->rp_T = 0;  // a replay source serves one run
  // A failed launch or a timed-out grid barrier leaves x / anc / w / the moment shifts part-advanced:
  // the handle then reports 'not initialized' instead of continuing from a corrupt state.
  if (st != PF_OK && touched) h->initialized = false;
  return st;
}

}  // namespace

extern "C" {

pf_status pf_ledh_run(pf_ledh_handle* h, const double* Ps, const double* Z, const double* U, int64_t T, int32_t noise,
                      double* means, double* covs, double* ess, uint8_t* flags) {
  if (!Ps) return lfail(PF_E_ARG, "null argument");
  if (h && h->algo == 1) return lfail(PF_E_ARG, "EDH handle: use pf_edh_run (it needs the tracker's past means)");
  return run_impl(h, Ps, nullptr, nullptr, Z, U, T, noise, means, covs, ess, flags);
}

pf_status pf_edh_run(pf_ledh_handle* h, const double* Ps, const double* Xbars, const double* Z, const double* U,
                     int64_t T, int32_t noise, double* means, double* covs, double* ess, uint8_t* flags) {
  if (!Ps || !Xbars) return lfail(PF_E_ARG, "null argument");
  if (h && h->algo != 1) return lfail(PF_E_ARG, "pf_edh_run needs a handle from pf_edh_create");
  return run_impl(h, Ps, Xbars, nullptr, Z, U, T, noise, means, covs, ess, flags);
}

pf_status pf_ledh_run_ekf(pf_ledh_handle* h, const double* x0, const double* P0, const double* Qt, const double* Rt,
                          const double* Z, const double* U, int64_t T, int32_t noise, double* means, double* covs,
                          double* ess, uint8_t* flags, double* x_final, double* P_final) {
  if (!x0 || !P0 || !Qt || !Rt) return lfail(PF_E_ARG, "null argument");
  EkfSpec e{x0, P0, Qt, Rt, x_final, P_final};
  return run_impl(h, nullptr, nullptr, &e, Z, U, T, noise, means, covs, ess, flags);
}

pf_status pf_ledh_ekf_sequence(pf_ledh_handle* h, const double* x0, const double* P0, const double* Qt,
                               const double* Rt, const double* Z, int64_t T, double* Ps, double* x_final,
                               double* P_final) {
  if (!h || !x0 || !P0 || !Qt || !Rt || !Z) return lfail(PF_E_ARG, "null argument");
  if (T <= 0) return PF_OK;
  LCHK(hipSetDevice(h->device));
  const int nx = h->nx, nz = h->nz;
  const size_t ne = 2 * (size_t)nx + 3 * (size_t)nx * nx + (size_t)nz * nz;
  double *dE = nullptr, *dZ = nullptr, *dP = nullptr;
  pf_status st = PF_OK;
  if (hipMalloc((void**)&dE, ne * 8) != hipSuccess || hipMalloc((void**)&dZ, (size_t)T * nz * 8) != hipSuccess ||
      hipMalloc((void**)&dP, (size_t)T * nx * nx * 8) != hipSuccess) {
    st = lfail(PF_E_HIP, "hipMalloc of EKF buffers failed");
  } else {
    double *ex0 = dE, *eP0 = dE + nx, *eQ = eP0 + nx * nx, *eR = eQ + nx * nx, *exf = eR + nz * nz, *ePf = exf + nx;
    if (hipMemcpy(ex0, x0, nx * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(eP0, P0, (size_t)nx * nx * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(eQ, Qt, (size_t)nx * nx * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(eR, Rt, (size_t)nz * nz * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dZ, Z, (size_t)T * nz * 8, hipMemcpyHostToDevice) != hipSuccess ||
        h->ops->ekf(h->Pm, ex0, eP0, eQ, eR, dZ, T, dP, exf, ePf, nullptr, h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess ||
        (Ps && hipMemcpy(Ps, dP, (size_t)T * nx * nx * 8, hipMemcpyDeviceToHost) != hipSuccess) ||
        (x_final && hipMemcpy(x_final, exf, nx * 8, hipMemcpyDeviceToHost) != hipSuccess) ||
        (P_final && hipMemcpy(P_final, ePf, (size_t)nx * nx * 8, hipMemcpyDeviceToHost) != hipSuccess))
      st = lfail(PF_E_HIP, "device EKF failed");
  }
  for (double* p : {dE, dZ, dP})
    if (p) (void)hipFree(p);
  return st;
}

pf_status pf_ledh_set_run_replay(pf_ledh_handle* h, const double* noise, const double* uniforms, int64_t T) {
  if (!h || !noise || !uniforms || T <= 0) return lfail(PF_E_ARG, "null argument");
  LCHK(hipSetDevice(h->device));
  LCHK(hipStreamSynchronize(h->stream));
  for (double* p : {h->rp_noise, h->rp_unif})
    if (p) LCHK(hipFree(p));
  h->rp_noise = h->rp_unif = nullptr;
  h->rp_T = 0;
  LCHK(hipMalloc((void**)&h->rp_noise, (size_t)T * h->N * h->nx * 8));
  LCHK(hipMalloc((void**)&h->rp_unif, (size_t)T * 8));
  LCHK(hipMemcpy(h->rp_noise, noise, (size_t)T * h->N * h->nx * 8, hipMemcpyHostToDevice));
  LCHK(hipMemcpy(h->rp_unif, uniforms, (size_t)T * 8, hipMemcpyHostToDevice));
  h->rp_T = T;
  return PF_OK;
}

void* pf_ledh_stream(pf_ledh_handle* h) { return h ? (void*)h->stream : nullptr; }
pf_status pf_ledh_synchronize(pf_ledh_handle* h) {
  if (!h) return lfail(PF_E_ARG, "null argument");
  LCHK(hipStreamSynchronize(h->stream));
  return PF_OK;
}
int32_t pf_ledh_shared_path(pf_ledh_handle* h) { return (h && h->shared) ? 1 : 0; }

}  // extern "C"

#ifdef PF_STAMPS
// diagnostic build only: per-workgroup phase stamps of the last fused LEDH step
extern "C" int pf_debug_stamps_ledh(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pf::ledh::g_ledh_stamps), (size_t)n * sizeof(unsigned long long));
}
// k_flow_wave_lr phase accumulators (workgroup 0): read (n <= 16) and clear
extern "C" int pf_debug_lr_acc(unsigned long long* out, int n, int clear) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pf::ledh::g_lr_acc), (size_t)n * sizeof(unsigned long long)) != hipSuccess)
    return 1;
  if (clear) {
    static const unsigned long long zeros[16] = {};
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(pf::ledh::g_lr_acc), zeros, sizeof(zeros));
  }
  return 0;
}
#endif
