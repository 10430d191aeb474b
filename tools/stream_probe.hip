// HBM ceiling of the many-replicate SV step's access pattern (diagnostic, not shipped).
// Each particle-step of k_step reads x, lw (4 B each) and writes x, lw: four streams of
// R x Npad floats.  This probe moves exactly those bytes with no filter arithmetic, in the
// step's geometry (256-thread workgroups, C float4 chunks per thread per array, one workgroup
// per tile) and as a grid-stride loop, to separate the access pattern from the step's own
// latency chain.  Build: hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o build/stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s\n", hipGetErrorString(e_)); std::exit(1); } } while (0)

// one workgroup per tile of 256*4*C particles of replicate blockIdx.y
template <int C>
__global__ void __launch_bounds__(256) tile_copy(const float* xi, const float* li, float* xo, float* lo, long npad, long n) {
  const long base = (long)blockIdx.y * npad;
  float4 a[C], b[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const long i = (long)blockIdx.x * 256 * 4 * C + (long)(threadIdx.x + 256 * c) * 4;
    if (i + 3 < n) {
      a[c] = *(const float4*)(xi + base + i);
      b[c] = *(const float4*)(li + base + i);
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const long i = (long)blockIdx.x * 256 * 4 * C + (long)(threadIdx.x + 256 * c) * 4;
    if (i + 3 < n) {
      float4 u = a[c], v = b[c];
      u.x += 1.0f; v.x += 1.0f;
      *(float4*)(xo + base + i) = u;
      *(float4*)(lo + base + i) = v;
    }
  }
}

// grid-stride over all float4 of all replicates (flat, replicate-major)
__global__ void __launch_bounds__(256) flat_copy(const float4* xi, const float4* li, float4* xo, float4* lo, long nv) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    float4 u = xi[i], v = li[i];
    u.x += 1.0f; v.x += 1.0f;
    xo[i] = u;
    lo[i] = v;
  }
}

int main(int argc, char** argv) {
  const long R = argc > 1 ? std::atol(argv[1]) : 64, n = argc > 2 ? std::atol(argv[2]) : 1000000;
  const long npad = (n + 3) / 4 * 4, tot = R * npad;
  float *xi, *li, *xo, *lo;
  CK(hipMalloc(&xi, tot * 4)); CK(hipMalloc(&li, tot * 4)); CK(hipMalloc(&xo, tot * 4)); CK(hipMalloc(&lo, tot * 4));
  CK(hipMemset(xi, 0, tot * 4)); CK(hipMemset(li, 0, tot * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 16.0 * R * n;
  auto timeit = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipEventRecord(e0));
    const int K = 20;
    for (int k = 0; k < K; ++k) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / K;
    std::printf("%-28s %8.1f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
  };
  timeit("tile C=1 (1024/tile)", [&] { hipLaunchKernelGGL(tile_copy<1>, dim3((n + 1023) / 1024, R), dim3(256), 0, 0, xi, li, xo, lo, npad, n); });
  timeit("tile C=2 (2048/tile)", [&] { hipLaunchKernelGGL(tile_copy<2>, dim3((n + 2047) / 2048, R), dim3(256), 0, 0, xi, li, xo, lo, npad, n); });
  timeit("tile C=4 (4096/tile)", [&] { hipLaunchKernelGGL(tile_copy<4>, dim3((n + 4095) / 4096, R), dim3(256), 0, 0, xi, li, xo, lo, npad, n); });
  for (int g : {1024, 2048, 4096, 8192}) {
    char name[64];
    std::snprintf(name, sizeof name, "grid-stride %d wg", g);
    timeit(name, [&] { hipLaunchKernelGGL(flat_copy, dim3(g), dim3(256), 0, 0, (const float4*)xi, (const float4*)li, (float4*)xo, (float4*)lo, tot / 4); });
  }
  return 0;
}
