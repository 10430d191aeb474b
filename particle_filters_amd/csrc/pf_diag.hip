// Particle-degeneracy diagnostics on the GPU: the C ABI of include/pf_diag.h (host-array entry)
// and pf::diag::compute, which pf_engine.hip / pf_ledh.hip call on their device-resident state.
//
// Restates /root/reference/notebooks/particle_filter_NLNGSSM.ipynb cell 5 ("diag:LINE"):
//   entropy   -sum (w + 1e-300) log(w + 1e-300) [/ log N]                     diag:5-19
//   gini      (2 sum_i i w_(i)) / (N sum w) - (N + 1)/N over ascending w       diag:22-36
//   n_unique  distinct rows of round(x / tol) * tol                            diag:39-58
//   ess, max weight, trace(cov)                                                diag:61-91
// HBM-bound reductions over [N] weights and SoA [nx][Npad] particles (fixed-order block
// partials, one final workgroup), plus two device radix sorts (hipcub): the ascending
// weights for the Gini sum, and 64-bit row keys for the unique count.  Row keys: the bit
// pattern of the rounded value for nx = 1 (exact); a 64-bit mix of the rounded row for
// nx > 1 (distinct rows collide with probability ~N^2 / 2^65, 3e-8 at N = 1e6).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pf_diag.h"
#include "pf_diag.h"

namespace pf {
void set_last_error(const std::string& msg);
namespace diag {
namespace {

constexpr int DB = 256;    // workgroup
constexpr int DG = 1024;   // max partial blocks (grid-stride beyond)

__device__ __forceinline__ double wsum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wmax64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
// block sum / max (DB threads), result valid in every thread
__device__ __forceinline__ double bsum(double v, double* red) {
  v = wsum64(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < DB / 64; ++k) s += red[k];
  return s;
}
__device__ __forceinline__ double bmax(double v, double* red) {
  v = wmax64(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = -INFINITY;
#pragma unroll
  for (int k = 0; k < DB / 64; ++k) s = fmax(s, red[k]);
  return s;
}

template <typename Real>
__device__ __forceinline__ double weight_of(const DiagSrc& s, int64_t i) {
  if (s.w) return s.w[i];
  if (s.uniform) return 1.0 / (double)s.N;
  return exp((double)((const Real*)s.lw)[i] - s.lse);
}

// pass 1: w -> wbuf; partials [0][b] sum w, [1][b] sum w^2, [2][b] sum (w+1e-300) log(w+1e-300), [3][b] max w
template <typename Real>
__global__ void __launch_bounds__(DB) k_dg_weights(DiagSrc s, double* wbuf, double* part) {
  __shared__ double red[DB / 64];
  double a = 0.0, b = 0.0, c = 0.0, m = -INFINITY;
  for (int64_t i = (int64_t)blockIdx.x * DB + threadIdx.x; i < s.N; i += (int64_t)gridDim.x * DB) {
    const double w = weight_of<Real>(s, i);
    wbuf[i] = w;
    a += w;
    b += w * w;
    const double we = w + 1e-300;
    c += we * log(we);
    m = fmax(m, w);
  }
  const int G = gridDim.x;
  a = bsum(a, red);
  b = bsum(b, red);
  c = bsum(c, red);
  m = bmax(m, red);
  if (threadIdx.x == 0) {
    part[0 * G + blockIdx.x] = a;
    part[1 * G + blockIdx.x] = b;
    part[2 * G + blockIdx.x] = c;
    part[3 * G + blockIdx.x] = m;
  }
}

// per-dimension weighted sums: blockIdx.y = d; mean == null: sum w x_d, else sum w (x_d - mean_d)^2
template <typename Real>
__global__ void __launch_bounds__(DB) k_dg_moment(DiagSrc s, const double* wbuf, const double* mean, double* part) {
  __shared__ double red[DB / 64];
  const int d = blockIdx.y;
  const Real* x = (const Real*)s.x + (int64_t)d * s.Npad;
  const double mu = mean ? mean[d] : 0.0;
  double a = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * DB + threadIdx.x; i < s.N; i += (int64_t)gridDim.x * DB) {
    const double v = (double)x[i] - mu;
    a += wbuf[i] * (mean ? v * v : v);
  }
  a = bsum(a, red);
  if (threadIdx.x == 0) part[(int64_t)d * gridDim.x + blockIdx.x] = a;
}

// mean_d = (sum w x_d) / (sum w)  (np.average / np.cov aweights normalisation)
__global__ void __launch_bounds__(DB) k_dg_mean(const double* part_w, const double* part_x, int G, int nx, double* mean) {
  __shared__ double red[DB / 64];
  double sw = 0.0;
  for (int k = threadIdx.x; k < G; k += DB) sw += part_w[k];
  sw = bsum(sw, red);
  for (int d = 0; d < nx; ++d) {
    double a = 0.0;
    for (int k = threadIdx.x; k < G; k += DB) a += part_x[(int64_t)d * G + k];
    a = bsum(a, red);
    if (threadIdx.x == 0) mean[d] = a / sw;
  }
}

// sum_i (i + 1) ws[i] over the ascending weights
__global__ void __launch_bounds__(DB) k_dg_gini(const double* ws, int64_t N, double* part) {
  __shared__ double red[DB / 64];
  double a = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * DB + threadIdx.x; i < N; i += (int64_t)gridDim.x * DB)
    a += (double)(i + 1) * ws[i];
  a = bsum(a, red);
  if (threadIdx.x == 0) part[blockIdx.x] = a;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// row keys of round(x / tol) * tol (np.round = round-half-even = rint); -0.0 -> +0.0
template <typename Real>
__global__ void __launch_bounds__(DB) k_dg_keys(DiagSrc s, uint64_t* keys) {
  const int64_t i = (int64_t)blockIdx.x * DB + threadIdx.x;
  if (i >= s.N) return;
  const Real* x = (const Real*)s.x;
  uint64_t key = 0x9e3779b97f4a7c15ull;
  for (int d = 0; d < s.nx; ++d) {
    const double v = rint((double)x[(int64_t)d * s.Npad + i] / s.tol) * s.tol + 0.0;
    uint64_t bits;
    memcpy(&bits, &v, 8);
    key = s.nx == 1 ? bits : mix64(key ^ (bits + 0x632be59bd9b4e019ull * (uint64_t)(d + 1)));
  }
  keys[i] = key;
}

// boundaries of the sorted keys
__global__ void __launch_bounds__(DB) k_dg_count(const uint64_t* k, int64_t N, double* part) {
  __shared__ double red[DB / 64];
  double a = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * DB + threadIdx.x; i < N; i += (int64_t)gridDim.x * DB)
    a += (i == 0 || k[i] != k[i - 1]) ? 1.0 : 0.0;
  a = bsum(a, red);
  if (threadIdx.x == 0) part[blockIdx.x] = a;
}

// out: ess, entropy, entropy_raw, gini, max_weight, spread, n_unique
__global__ void __launch_bounds__(DB) k_dg_final(const double* pw, const double* pg, const double* pu,
                                                 const double* ps, int G, int nx, int64_t N, int has_x,
                                                 double spread_in, double* out) {
  __shared__ double red[DB / 64];
  double sw = 0.0, sw2 = 0.0, se = 0.0, mx = -INFINITY, sg = 0.0, su = 0.0, sp = 0.0;
  for (int k = threadIdx.x; k < G; k += DB) {
    sw += pw[k];
    sw2 += pw[G + k];
    se += pw[2 * G + k];
    mx = fmax(mx, pw[3 * G + k]);
    sg += pg[k];
    if (has_x) su += pu[k];
  }
  if (has_x && ps)
    for (int q = threadIdx.x; q < nx * G; q += DB) sp += ps[q];
  sw = bsum(sw, red);
  sw2 = bsum(sw2, red);
  se = bsum(se, red);
  mx = bmax(mx, red);
  sg = bsum(sg, red);
  su = bsum(su, red);
  sp = bsum(sp, red);
  if (threadIdx.x == 0) {
    const double n = (double)N;
    out[0] = 1.0 / sw2;
    out[2] = -se;
    out[1] = N > 1 ? -se / log(n) : -se;
    out[3] = (2.0 * sg) / (n * sw) - (n + 1.0) / n;
    out[4] = mx;
    out[5] = !isnan(spread_in) ? spread_in : (has_x && ps ? sp / sw : NAN);
    out[6] = has_x ? su : -1.0;
  }
}

template <typename Real>
pf_status compute_t(const DiagSrc& s, hipStream_t st, pf_diagnostics* out) {
  const int64_t N = s.N;
  const int G = (int)std::min<int64_t>(DG, (N + DB - 1) / DB);
  const bool has_x = s.x != nullptr && s.tol > 0.0;
  const bool need_spread = s.x != nullptr && std::isnan(s.spread);
  double *wbuf = nullptr, *ws = nullptr, *part = nullptr, *mean = nullptr, *res = nullptr;
  uint64_t *keys = nullptr, *ksort = nullptr;
  void* tmp = nullptr;
  size_t tb_w = 0, tb_k = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, tb_w, (const double*)nullptr, (double*)nullptr, (int)N, 0, 64, st);
  if (has_x)
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, tb_k, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)N, 0, 64,
                                            st);
  const size_t tb = std::max(tb_w, tb_k);
  const int nx = std::max(1, s.nx);
  const size_t np = (size_t)G * (4 + 1 + 1 + 2 * nx);
  auto cleanup = [&]() {
    for (void* p : {(void*)wbuf, (void*)ws, (void*)part, (void*)mean, (void*)res, (void*)keys, (void*)ksort, tmp})
      if (p) (void)hipFree(p);
  };
  bool ok = hipMalloc((void**)&wbuf, N * 8) == hipSuccess && hipMalloc((void**)&ws, N * 8) == hipSuccess &&
            hipMalloc((void**)&part, np * 8) == hipSuccess && hipMalloc((void**)&mean, nx * 8) == hipSuccess &&
            hipMalloc((void**)&res, 8 * 8) == hipSuccess && hipMalloc(&tmp, tb + 16) == hipSuccess &&
            (!has_x || (hipMalloc((void**)&keys, N * 8) == hipSuccess && hipMalloc((void**)&ksort, N * 8) == hipSuccess));
  if (!ok) {
    cleanup();
    set_last_error("diagnostics: hipMalloc failed");
    return PF_E_HIP;
  }
  double* pw = part;                  // [4][G]
  double* pg = pw + 4 * (size_t)G;    // [G]
  double* pu = pg + G;                // [G]
  double* px = pu + G;                // [nx][G]
  double* pv = px + (size_t)nx * G;   // [nx][G]
  hipLaunchKernelGGL(k_dg_weights<Real>, dim3(G), dim3(DB), 0, st, s, wbuf, pw);
  size_t t1 = tb;
  hipError_t e = hipcub::DeviceRadixSort::SortKeys(tmp, t1, wbuf, ws, (int)N, 0, 64, st);
  hipLaunchKernelGGL(k_dg_gini, dim3(G), dim3(DB), 0, st, ws, N, pg);
  if (need_spread) {
    hipLaunchKernelGGL(k_dg_moment<Real>, dim3(G, s.nx), dim3(DB), 0, st, s, wbuf, (const double*)nullptr, px);
    hipLaunchKernelGGL(k_dg_mean, dim3(1), dim3(DB), 0, st, pw, px, G, s.nx, mean);
    hipLaunchKernelGGL(k_dg_moment<Real>, dim3(G, s.nx), dim3(DB), 0, st, s, wbuf, (const double*)mean, pv);
  }
  if (has_x && e == hipSuccess) {
    hipLaunchKernelGGL(k_dg_keys<Real>, dim3((unsigned)((N + DB - 1) / DB)), dim3(DB), 0, st, s, keys);
    size_t t2 = tb;
    e = hipcub::DeviceRadixSort::SortKeys(tmp, t2, keys, ksort, (int)N, 0, 64, st);
    hipLaunchKernelGGL(k_dg_count, dim3(G), dim3(DB), 0, st, ksort, N, pu);
  }
  hipLaunchKernelGGL(k_dg_final, dim3(1), dim3(DB), 0, st, pw, pg, pu, need_spread ? pv : nullptr, G, s.nx, N,
                     has_x ? 1 : 0, s.spread, res);
  double h[8];
  if (e == hipSuccess) e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(h, res, 7 * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  cleanup();
  if (e != hipSuccess) {
    set_last_error(std::string("diagnostics: ") + hipGetErrorString(e));
    return PF_E_HIP;
  }
  out->ess = h[0];
  out->entropy = h[1];
  out->entropy_raw = h[2];
  out->gini = h[3];
  out->max_weight = h[4];
  out->posterior_spread = h[5];
  out->n_unique = (int64_t)h[6];
  return PF_OK;
}

}  // namespace

pf_status compute(const DiagSrc& s, hipStream_t st, pf_diagnostics* out) {
  if (s.N <= 0 || s.N > (int64_t)INT32_MAX) {
    set_last_error("diagnostics: N out of range");
    return PF_E_ARG;
  }
  return s.real_is_double ? compute_t<double>(s, st, out) : compute_t<float>(s, st, out);
}

}  // namespace diag
}  // namespace pf

extern "C" pf_status pf_diagnostics_host(int32_t device, const double* weights, const double* particles, int64_t N,
                                         int32_t nx, double tol, const double* cov, pf_diagnostics* out) {
  using namespace pf;
  if (!weights || !out || N <= 0 || (particles && nx <= 0)) {
    set_last_error("pf_diagnostics_host: bad argument");
    return PF_E_ARG;
  }
  if (hipSetDevice(device) != hipSuccess) {
    set_last_error("pf_diagnostics_host: hipSetDevice failed");
    return PF_E_HIP;
  }
  double *dw = nullptr, *dx = nullptr;
  auto done = [&](pf_status s) {
    if (dw) (void)hipFree(dw);
    if (dx) (void)hipFree(dx);
    return s;
  };
  if (hipMalloc((void**)&dw, N * 8) != hipSuccess || (particles && hipMalloc((void**)&dx, N * nx * 8) != hipSuccess)) {
    set_last_error("pf_diagnostics_host: hipMalloc failed");
    return done(PF_E_HIP);
  }
  std::vector<double> soa;
  if (particles) {  // [N][nx] -> SoA [nx][N]
    soa.resize((size_t)N * nx);
    for (int64_t i = 0; i < N; ++i)
      for (int d = 0; d < nx; ++d) soa[(size_t)d * N + i] = particles[i * nx + d];
  }
  if (hipMemcpy(dw, weights, N * 8, hipMemcpyHostToDevice) != hipSuccess ||
      (particles && hipMemcpy(dx, soa.data(), soa.size() * 8, hipMemcpyHostToDevice) != hipSuccess)) {
    set_last_error("pf_diagnostics_host: upload failed");
    return done(PF_E_HIP);
  }
  diag::DiagSrc s{};
  s.N = N;
  s.Npad = N;
  s.nx = particles ? nx : 0;
  s.w = dw;
  s.x = dx;
  s.real_is_double = 1;
  s.tol = tol;
  s.spread = NAN;
  if (cov) {
    double tr = 0.0;
    for (int d = 0; d < nx; ++d) tr += cov[d * nx + d];
    s.spread = tr;
  }
  return done(diag::compute(s, nullptr, out));
}
