// Minimal reproduction for the rocprofv3 exit crash seen with cooperative launches:
// no torch, no engine.  ./coop_min <coop 0|1> <destroy-stream 0|1> <launches>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_touch(int* p) {
  if (threadIdx.x == 0) atomicAdd(p, 1);
}

int main(int argc, char** argv) {
  const int coop = argc > 1 ? std::atoi(argv[1]) : 1;
  const int destroy = argc > 2 ? std::atoi(argv[2]) : 1;
  const int n = argc > 3 ? std::atoi(argv[3]) : 10;
  int* d = nullptr;
  hipStream_t s;
  if (hipMalloc(&d, sizeof(int)) != hipSuccess || hipMemset(d, 0, sizeof(int)) != hipSuccess ||
      hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    return 2;
  for (int i = 0; i < n; ++i) {
    hipError_t e;
    if (coop) {
      void* args[] = {&d};
      e = hipLaunchCooperativeKernel((const void*)k_touch, dim3(256), dim3(512), args, 0, s);
    } else {
      hipLaunchKernelGGL(k_touch, dim3(256), dim3(512), 0, s, d);
      e = hipGetLastError();
    }
    if (e != hipSuccess) {
      std::printf("launch %d: %s\n", i, hipGetErrorString(e));
      return 3;
    }
  }
  if (hipStreamSynchronize(s) != hipSuccess) return 4;
  int h = 0;
  if (hipMemcpy(&h, d, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 5;
  std::printf("coop=%d destroy=%d launches=%d count=%d (expect %d)\n", coop, destroy, n, h, 256 * n);
  if (destroy) (void)hipStreamDestroy(s);
  (void)hipFree(d);
  return h == 256 * n ? 0 : 1;
}
