// Type-erased launchers for one compiled model shape (nx, nz, g kind, h kind,
// precision).  Each pf_inst_*.hip translation unit instantiates the kernel
// templates for its model family and registers an Ops entry; pf_engine.hip
// looks the entry up at pf_create time.
#pragma once
#include "pf_hooks.h"
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstdlib>

#include "pf_kernels.h"
#include "pf_persist.h"
#include "pf_resident.h"
#include "pf_shard_kernels.h"
#include "pf_step_grp.h"
#include "pf_step_stream.h"

namespace pf {

struct Ops {
  int nx, nz, tk, ok, prec;
  int rec_size, ch, tile_max, tile_min, psize;
  int grp;  // the step kernel is k_step_grp (lane groups per particle)
  int dyn;  // runtime-shape kernels (pf_dyn.h): nx / nz come from StepParams::dnx / dnz and the
            // trailing nx / nz arguments below; the compiled-shape entries ignore those
  hipError_t (*step)(const StepParams&, dim3, size_t, hipStream_t);
  hipError_t (*finalize)(const StepParams&, int R, hipStream_t);
  hipError_t (*cdf)(const StepParams&, double* cdf_out, dim3, size_t, hipStream_t);
  hipError_t (*head)(const StepParams&, double* head_out, dim3, size_t, hipStream_t);
  hipError_t (*init)(void* x, double* rec, const void* mean, const void* Lc, const double* replay,
                     int64_t N, int64_t Npad, int G, int R, uint64_t seed, uint32_t epoch, int rep_base, int64_t pbase,
                     hipStream_t, int nx, int lc_diag);
  hipError_t (*moments)(const void* x, const void* lw, const double* rec, int G, const double* lse, int64_t N,
                        int64_t Npad, int R, double* mean, double* cov, hipStream_t, int nx);
  void (*prepare)();  // per-device kernel attributes, called once a device is current
  // register-resident whole-run kernel (scalar fp32 models only; null otherwise).
  // Cooperative launch: returns hipErrorCooperativeLaunchTooLarge when the grid
  // cannot be co-resident (the caller then runs the launch-per-step path).
  // ev0 / ev1 (plain launches; null: none): the launch's own start / stop timestamps
  hipError_t (*resident)(const ResParams&, int G, int R, hipStream_t, bool coop, hipEvent_t ev0, hipEvent_t ev1);
  // persistent fused step of the many-replicate fp32 scalar launches (pf_step_stream.h; null otherwise):
  // grid = min(G R, co-resident workgroups), tiles walked with the next tile's operands in flight
  hipError_t (*stream)(const StepParams&, int R, size_t smem, hipStream_t);
  int (*resident_cap)(bool trace);  // workgroups of k_resident (the trace instance when trace) co-resident
                                    // on the current device (0: unknown)
  // persistent whole-run kernel of the scalar fp64 models (pf_persist.h; null otherwise): a plain
  // launch of the G x R grid (hipErrorCooperativeLaunchTooLarge when it exceeds persist_cap); ev1: the
  // launch's own stop timestamp (null: none)
  hipError_t (*persist)(const PersistParams&, int G, int R, size_t smem, hipStream_t, hipEvent_t ev1);
  int (*persist_cap)(size_t smem);  // co-resident workgroups of k_persist with smem bytes of LDS
  // within-filter sharding (pf_shard_kernels.h)
  hipError_t (*shard_offspring)(const void* x, int64_t N, int64_t Npad, const double* cdf, double U, double lo,
                                double mass, int64_t Ntot, int64_t a, int64_t n, void* out, hipStream_t, int nx);
  hipError_t (*shard_adopt)(const void* rows, void* x, int64_t N, int64_t Npad, double* rec, int G, const void* P,
                            int jitter, const double* rp_jit, uint64_t seed, uint32_t rep, uint32_t ep, int64_t pbase,
                            hipStream_t, int nx, int nz);
};

void register_ops(const Ops& o);
const Ops* find_ops(int nx, int nz, int tk, int ok, int prec);

inline size_t base_lds_bytes(int G) { return (size_t)lds_tile(G) * sizeof(double); }

template <typename Real, int NX, int NZ, int TK, int OK>
struct Launch {
  static constexpr int BS = StepTraits<Real, NX, NZ, TK, OK>::BS;
  static hipError_t step(const StepParams& p, dim3 grid, size_t smem, hipStream_t s) {
    lds_poison_hook(s);  // tests only (pf_hooks.h)
    if constexpr (SGrp<NX>::ON) {  // large state: 4 lanes per particle (pf_step_grp.h)
      const bool rd = p.r_diag != 0, ql = p.lq_local != 0 && p.lj_local != 0;
      if (rd && ql) hipLaunchKernelGGL((k_step_grp<Real, NX, NZ, TK, OK, true, true>), grid, dim3(256), smem, s, p);
      else if (rd) hipLaunchKernelGGL((k_step_grp<Real, NX, NZ, TK, OK, true, false>), grid, dim3(256), smem, s, p);
      else if (ql) hipLaunchKernelGGL((k_step_grp<Real, NX, NZ, TK, OK, false, true>), grid, dim3(256), smem, s, p);
      else hipLaunchKernelGGL((k_step_grp<Real, NX, NZ, TK, OK, false, false>), grid, dim3(256), smem, s, p);
    } else {
      hipLaunchKernelGGL((k_step<Real, NX, NZ, TK, OK>), grid, dim3(BS), smem, s, p);
    }
    return hipGetLastError();
  }
  static hipError_t finalize(const StepParams& p, int R, hipStream_t s) {
    hipLaunchKernelGGL((k_finalize<NX, BS>), dim3(R), dim3(BS), LDS_RED * sizeof(double), s, p);
    return hipGetLastError();
  }
  static hipError_t head(const StepParams& p, double* out, dim3 grid, size_t smem, hipStream_t s) {
    hipLaunchKernelGGL((k_head<NX, BS>), grid, dim3(BS), smem, s, p, out);
    return hipGetLastError();
  }
  static hipError_t cdf(const StepParams& p, double* out, dim3 grid, size_t smem, hipStream_t s) {
    hipLaunchKernelGGL((k_cdf<Real, NX, BS>), grid, dim3(BS), smem, s, p, out);
    return hipGetLastError();
  }
  static hipError_t init(void* x, double* rec, const void* mean, const void* Lc, const double* replay,
                         int64_t N, int64_t Npad, int G, int R, uint64_t seed, uint32_t epoch,
                         int rep_base, int64_t pbase, hipStream_t s, int, int) {
    const int64_t n = N > G ? N : G;
    dim3 grid((unsigned)((n + BLOCK - 1) / BLOCK), (unsigned)R);
    hipLaunchKernelGGL((k_init<Real, NX>), grid, dim3(BLOCK), 0, s, (Real*)x, rec, (const Real*)mean,
                       (const Real*)Lc, replay, N, Npad, G, seed, epoch, rep_base, pbase);
    return hipGetLastError();
  }
  static hipError_t moments(const void* x, const void* lw, const double* rec, int G, const double* lse,
                            int64_t N, int64_t Npad, int R, double* mean, double* cov, hipStream_t s, int) {
    hipLaunchKernelGGL((k_mom_mean<Real, NX>), dim3(NX, R), dim3(BLOCK), 64 * sizeof(double), s, (const Real*)x,
                       (const Real*)lw, rec, Rec<NX>::SIZE, G, lse, N, Npad, mean);
    if (cov)
      hipLaunchKernelGGL((k_mom_cov<Real, NX>), dim3(NX * NX, R), dim3(BLOCK), 64 * sizeof(double), s,
                         (const Real*)x, (const Real*)lw, rec, Rec<NX>::SIZE, G, lse, N, Npad, mean, cov);
    return hipGetLastError();
  }
  static hipError_t shard_offspring(const void* x, int64_t N, int64_t Npad, const double* cdf, double U, double lo,
                                    double mass, int64_t Ntot, int64_t a, int64_t n, void* out, hipStream_t s, int) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_shard_offspring<Real, NX>), dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                       (const Real*)x, N, Npad, cdf, U, lo, mass, Ntot, a, n, (Real*)out);
    return hipGetLastError();
  }
  static hipError_t shard_adopt(const void* rows, void* x, int64_t N, int64_t Npad, double* rec, int G, const void* P,
                                int jitter, const double* rp_jit, uint64_t seed, uint32_t rep, uint32_t ep, int64_t pbase,
                                hipStream_t s, int, int) {
    const int64_t n = N > G ? N : G;
    hipLaunchKernelGGL((k_shard_adopt<Real, NX, NZ, TK, OK>), dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                       s, (const Real*)rows, (Real*)x, N, Npad, rec, G, (const Real*)P, jitter, rp_jit, seed, rep, ep,
                       pbase);
    return hipGetLastError();
  }
  static Ops make(int prec) {
    Ops o;
    o.nx = NX; o.nz = NZ; o.tk = TK; o.ok = OK; o.prec = prec;
    o.rec_size = Rec<NX>::SIZE;
    o.ch = StepTraits<Real, NX, NZ, TK, OK>::CH;
    o.tile_max = StepTraits<Real, NX, NZ, TK, OK>::TILE_MAX;
    // large states (k_step_grp): one particle per lane group per round -> 256 / GL particles
    o.tile_min = SGrp<NX>::ON ? 256 / SGrp<NX>::GL : BS * StepTraits<Real, NX, NZ, TK, OK>::CH;
    o.psize = ParamLayout<NX, NZ>::SIZE;
    o.grp = SGrp<NX>::ON ? 1 : 0;
    o.dyn = 0;
    o.step = &step;
    o.finalize = &finalize;
    o.cdf = &cdf;
    o.head = &head;
    o.init = &init;
    o.moments = &moments;
    o.prepare = &prepare;
    o.resident = nullptr;
    o.resident_cap = nullptr;
    o.stream = nullptr;
    o.persist = nullptr;
    o.persist_cap = nullptr;
    o.shard_offspring = &shard_offspring;
    o.shard_adopt = &shard_adopt;
    return o;
  }
  static void prepare() {
    // allow up to 160 KiB of dynamic LDS for the tile CDF
    if constexpr (SGrp<NX>::ON) {
      for (const void* fn : {(const void*)k_step_grp<Real, NX, NZ, TK, OK, true, true>,
                             (const void*)k_step_grp<Real, NX, NZ, TK, OK, true, false>,
                             (const void*)k_step_grp<Real, NX, NZ, TK, OK, false, true>,
                             (const void*)k_step_grp<Real, NX, NZ, TK, OK, false, false>})
        (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);  // + static z[NZ]
    } else
      (void)hipFuncSetAttribute((const void*)k_step<Real, NX, NZ, TK, OK>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_cdf<Real, NX, BS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
  }
};

// explicit registration (called once from pf_engine.hip; no static-init order games)
void register_sv_models();
void register_linear_models();
void register_l96_models();
void register_mat_models();
void register_dyn_models();

template <int NX, int NZ, int TK, int OK>
struct ResidentLaunch {
  // Every workgroup of the grid must be co-resident (they hand data to each other inside the
  // launch).  coop: cooperative launch (the runtime checks the grid against the device's
  // capacity and dispatches it so that all workgroups are resident together; ~10-17 us per
  // launch).  Otherwise a plain launch after the same check against the occupancy API; the
  // kernel verifies co-residency itself either way (res_arrive / res_try_abort).
  // hipErrorCooperativeLaunchTooLarge -> the caller runs the launch-per-step path.
  // p.tr_x set: the trace instance (the same kernel plus the verification-trace stores; tests)
  // ev0 / ev1 (plain launches): timing events stamped by the kernel's own dispatch
  // (hipExtLaunchKernel), instead of two marker packets queued around it
  static hipError_t launch(const ResParams& p, int G, int R, hipStream_t s, bool coop, hipEvent_t ev0, hipEvent_t ev1) {
    const bool tr = p.tr_x != nullptr;
    const void* fn = tr ? (const void*)k_resident<float, NX, NZ, TK, OK, true> : (const void*)k_resident<float, NX, NZ, TK, OK>;
    ResParams q = p;
    void* args[] = {&q};
    if (coop) return hipLaunchCooperativeKernel(fn, dim3(G, R), dim3(RBS), args, 0, s);
    if ((long long)G * R > (long long)cap(tr)) return hipErrorCooperativeLaunchTooLarge;
    return hipExtLaunchKernel(fn, dim3(G, R), dim3(RBS), args, 0, s, ev0, ev1, 0);
  }
  // CUs x workgroups per CU from the occupancy API, cached per device
  template <bool TR>
  static int cap_of() {
    static thread_local int cached_dev = -1, cached_cap = 0;  // per thread: no shared mutable state
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (dev != cached_dev) {
      int cus = 0, per_cu = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_resident<float, NX, NZ, TK, OK, TR>, RBS,
                                                       0) != hipSuccess)
        return 0;
      cached_dev = dev;
      cached_cap = cus * per_cu;
    }
    return cached_cap;
  }
  static int cap(bool trace) { return trace ? cap_of<true>() : cap_of<false>(); }
};

template <int NZ, int TK, int OK>
struct StreamLaunch {
  // one workgroup per co-resident slot (CUs x the occupancy API, cached per device and LDS size), at
  // most one per tile; no workgroup waits for another, so any grid is correct
  static hipError_t launch(const StepParams& p, int R, size_t smem, hipStream_t s) {
    static thread_local int cached_dev = -1, cached_cap = 0;  // per thread: no shared mutable state
    static thread_local size_t cached_smem = 0;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev != cached_dev || smem != cached_smem) {
      int cus = 0, per_cu = 0;
      (void)hipFuncSetAttribute((const void*)k_step_stream<NZ, TK, OK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
      if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_step_stream<NZ, TK, OK>, 256,
                                                            smem)) != hipSuccess)
        return e;
      cached_dev = dev;
      cached_smem = smem;
      cached_cap = cus * (per_cu > 0 ? per_cu : 1);
    }
    const long long ntiles = (long long)p.G * R;
    const unsigned grid = (unsigned)(ntiles < cached_cap ? ntiles : cached_cap);
    hipLaunchKernelGGL((k_step_stream<NZ, TK, OK>), dim3(grid), dim3(256), smem, s, p, R);
    return hipGetLastError();
  }
};

template <int NX, int NZ, int TK, int OK>
struct PersistLaunch {
  // Every workgroup waits for the others' records, so the grid must be co-resident: a plain launch
  // after the check against the occupancy API (the kernel checks it again itself: res_arrive)
  static hipError_t launch(const PersistParams& p, int G, int R, size_t smem, hipStream_t s, hipEvent_t ev1) {
    lds_poison_hook(s);  // tests only (pf_hooks.h)
    if ((long long)G * R > (long long)cap(smem)) return hipErrorCooperativeLaunchTooLarge;
    PersistParams q = p;
    void* args[] = {&q};
    return hipExtLaunchKernel((const void*)k_persist<double, NX, NZ, TK, OK>, dim3(G, R), dim3(PBS), args, smem, s,
                              nullptr, ev1, 0);
  }
  // CUs x workgroups per CU from the occupancy API, cached per device and LDS size
  static int cap(size_t smem) {
    static thread_local int cached_dev = -1, cached_cap = 0;  // per thread: no shared mutable state
    static thread_local size_t cached_smem = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (dev != cached_dev || smem != cached_smem) {
      const void* fn = (const void*)k_persist<double, NX, NZ, TK, OK>;
      int cus = 0, per_cu = 0;
      if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess) {
        (void)hipGetLastError();  // (not sticky for the launches that follow)
        return 0;
      }
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, PBS, smem) != hipSuccess)
        return 0;
      cached_dev = dev;
      cached_smem = smem;
      cached_cap = cus * per_cu;
    }
    return cached_cap;
  }
};

template <int NX, int NZ, int TK, int OK>
inline void register_both() {
  Ops f32 = Launch<float, NX, NZ, TK, OK>::make(PF_PRECISION_FP32);
  if constexpr (NX == 1) {
    f32.resident = &ResidentLaunch<NX, NZ, TK, OK>::launch;
    f32.resident_cap = &ResidentLaunch<NX, NZ, TK, OK>::cap;
    f32.stream = &StreamLaunch<NZ, TK, OK>::launch;
  }
  register_ops(f32);
  Ops f64 = Launch<double, NX, NZ, TK, OK>::make(PF_PRECISION_FP64);
  if constexpr (NX == 1) {
    f64.persist = &PersistLaunch<NX, NZ, TK, OK>::launch;
    f64.persist_cap = &PersistLaunch<NX, NZ, TK, OK>::cap;
  }
  register_ops(f64);
}

}  // namespace pf
