// Runtime-shape kernels (pf_dyn.h) for every (g kind, h kind, precision): the engine's path for
// models outside the compiled (nx, nz) list, or any model under PF_PATH_RUNTIME.  Registered as
// shape templates (nx = nz = 0); find_ops_dyn materialises one Ops per concrete shape.
#include "pf_dyn.h"
#include "pf_ops.h"

namespace pf {

template <typename Real, int TK, int OK>
struct DynLaunch {
  static hipError_t step(const StepParams& p, dim3 grid, size_t smem, hipStream_t s) {
    hipLaunchKernelGGL((k_dyn_step<Real, TK, OK>), grid, dim3(DBS), smem, s, p);
    return hipGetLastError();
  }
  static hipError_t finalize(const StepParams& p, int R, hipStream_t s) {
    hipLaunchKernelGGL(k_dyn_finalize, dim3(R), dim3(DBS), LDS_RED * sizeof(double), s, p);
    return hipGetLastError();
  }
  static hipError_t head(const StepParams& p, double* out, dim3 grid, size_t smem, hipStream_t s) {
    hipLaunchKernelGGL(k_dyn_head, grid, dim3(DBS), smem, s, p, out);
    return hipGetLastError();
  }
  static hipError_t cdf(const StepParams& p, double* out, dim3 grid, size_t smem, hipStream_t s) {
    hipLaunchKernelGGL((k_dyn_cdf<Real>), grid, dim3(DBS), smem, s, p, out);
    return hipGetLastError();
  }
  static hipError_t init(void* x, double* rec, const void* mean, const void* Lc, const double* replay, int64_t N,
                         int64_t Npad, int G, int R, uint64_t seed, uint32_t epoch, int rep_base, int64_t pbase,
                         hipStream_t s, int nx, int lc_diag) {
    const int64_t n = N > G ? N : G;
    dim3 grid((unsigned)((n + DBS - 1) / DBS), (unsigned)R);
    hipLaunchKernelGGL((k_dyn_init<Real>), grid, dim3(DBS), 0, s, (Real*)x, rec, (const Real*)mean, (const Real*)Lc,
                       replay, N, Npad, G, seed, epoch, rep_base, pbase, nx, lc_diag);
    return hipGetLastError();
  }
  static hipError_t moments(const void* x, const void* lw, const double* rec, int G, const double* lse, int64_t N,
                            int64_t Npad, int R, double* mean, double* cov, hipStream_t s, int nx) {
    const int RS = DynRec(nx).SIZE;
    hipLaunchKernelGGL((k_dyn_mom_mean<Real>), dim3(nx, R), dim3(BLOCK), 64 * sizeof(double), s, (const Real*)x,
                       (const Real*)lw, rec, RS, G, lse, N, Npad, mean, nx);
    if (cov)
      hipLaunchKernelGGL((k_dyn_mom_cov<Real>), dim3(nx * nx, R), dim3(BLOCK), 64 * sizeof(double), s, (const Real*)x,
                         (const Real*)lw, rec, RS, G, lse, N, Npad, mean, cov, nx);
    return hipGetLastError();
  }
  static hipError_t shard_offspring(const void* x, int64_t N, int64_t Npad, const double* cdf, double U, double lo,
                                    double mass, int64_t Ntot, int64_t a, int64_t n, void* out, hipStream_t s, int nx) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_dyn_shard_offspring<Real>), dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                       (const Real*)x, N, Npad, cdf, U, lo, mass, Ntot, a, n, (Real*)out, nx);
    return hipGetLastError();
  }
  static hipError_t shard_adopt(const void* rows, void* x, int64_t N, int64_t Npad, double* rec, int G, const void* P,
                                int jitter, const double* rp_jit, uint64_t seed, uint32_t rep, uint32_t ep, int64_t pbase,
                                hipStream_t s, int nx, int nz) {
    const int64_t n = N > G ? N : G;
    hipLaunchKernelGGL((k_dyn_shard_adopt<Real>), dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                       (const Real*)rows, (Real*)x, N, Npad, rec, G, (const Real*)P, jitter, rp_jit, seed, rep, ep,
                       pbase, nx, nz);
    return hipGetLastError();
  }
  static void prepare() {
    (void)hipFuncSetAttribute((const void*)k_dyn_step<Real, TK, OK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_dyn_cdf<Real>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  }
  static Ops make(int prec) {
    Ops o;
    o.nx = 0; o.nz = 0;  // shape template
    o.tk = TK; o.ok = OK; o.prec = prec;
    o.rec_size = 0;
    o.ch = 1;
    o.tile_max = DYN_TILE_MAX;
    o.tile_min = DBS;
    o.psize = 0;
    o.grp = 0;
    o.dyn = 1;
    o.step = &step;
    o.finalize = &finalize;
    o.cdf = &cdf;
    o.head = &head;
    o.init = &init;
    o.moments = &moments;
    o.prepare = &prepare;
    o.resident = nullptr;
    o.resident_cap = nullptr;
    o.persist = nullptr;
    o.persist_cap = nullptr;
    o.shard_offspring = &shard_offspring;
    o.shard_adopt = &shard_adopt;
    return o;
  }
};

template <int TK, int OK>
static void register_dyn_pair() {
  register_ops(DynLaunch<float, TK, OK>::make(PF_PRECISION_FP32));
  register_ops(DynLaunch<double, TK, OK>::make(PF_PRECISION_FP64));
}

void register_dyn_models() {
  register_dyn_pair<PF_TRANS_LINEAR, PF_OBS_LINEAR>();
  register_dyn_pair<PF_TRANS_LINEAR, PF_OBS_EXP_HALF>();
  register_dyn_pair<PF_TRANS_LINEAR, PF_OBS_ACOUSTIC>();
  register_dyn_pair<PF_TRANS_LINEAR, PF_OBS_SV_EXACT>();
  register_dyn_pair<PF_TRANS_LINEAR, PF_OBS_BEARINGS>();
  register_dyn_pair<PF_TRANS_L96, PF_OBS_LINEAR>();
  register_dyn_pair<PF_TRANS_L96, PF_OBS_EXP_HALF>();
  register_dyn_pair<PF_TRANS_L96, PF_OBS_ACOUSTIC>();
  register_dyn_pair<PF_TRANS_L96, PF_OBS_SV_EXACT>();
  register_dyn_pair<PF_TRANS_L96, PF_OBS_BEARINGS>();
}

}  // namespace pf
