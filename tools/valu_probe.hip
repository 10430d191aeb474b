// Issue cost of the VALU instructions the SIR / LEDH kernels are made of, on gfx950 (MI355X).
//   hipcc -O3 --offload-arch=gfx950 tools/valu_probe.hip -o build/valu_probe && build/valu_probe
// One workgroup per CU (256 workgroups of W waves: W = 4 is one wave per SIMD, W = 8 two), each
// wave runs ITERS x 8 independent instructions of one kind (8 accumulator chains, inline asm so
// nothing is folded) between two s_memtime reads.  Printed: shader cycles per wave-instruction,
// per wave and per SIMD (= per wave / waves per SIMD), median over the waves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int ITERS = 2048;

#define CHAINS8(ASM, T, INIT, CONS)                                          \
  T a0 = INIT + 1, a1 = INIT + 2, a2 = INIT + 3, a3 = INIT + 4, a4 = INIT + 5, \
    a5 = INIT + 6, a6 = INIT + 7, a7 = INIT + 8;                              \
  for (int it = 0; it < ITERS; ++it) {                                      \
    asm volatile(ASM : "+v"(a0) : CONS);                                    \
    asm volatile(ASM : "+v"(a1) : CONS);                                    \
    asm volatile(ASM : "+v"(a2) : CONS);                                    \
    asm volatile(ASM : "+v"(a3) : CONS);                                    \
    asm volatile(ASM : "+v"(a4) : CONS);                                    \
    asm volatile(ASM : "+v"(a5) : CONS);                                    \
    asm volatile(ASM : "+v"(a6) : CONS);                                    \
    asm volatile(ASM : "+v"(a7) : CONS);                                    \
  }                                                                         \
  sink = (double)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);

template <int OP>
__global__ void probe(unsigned long long* cyc, double* out) {
  const float fk = 1.0001f + threadIdx.x * 1e-7f;
  const double dk = 1.0000001 + threadIdx.x * 1e-12;
  const uint32_t uk = 0xD2511F53u + threadIdx.x;
  double sink = 0.0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (OP == 0) { CHAINS8("v_add_f32 %0, %0, %1", float, fk, "v"(fk)) }
  else if constexpr (OP == 1) { CHAINS8("v_fma_f32 %0, %0, %1, %1", float, fk, "v"(fk)) }
  else if constexpr (OP == 2) { CHAINS8("v_exp_f32 %0, %0", float, 0.01f * fk, "v"(fk)) }
  else if constexpr (OP == 3) { CHAINS8("v_sin_f32 %0, %0", float, 0.01f * fk, "v"(fk)) }
  else if constexpr (OP == 4) { CHAINS8("v_log_f32 %0, %0", float, fk, "v"(fk)) }
  else if constexpr (OP == 5) { CHAINS8("v_sqrt_f32 %0, %0", float, fk, "v"(fk)) }
  else if constexpr (OP == 6) { CHAINS8("v_add_f64 %0, %0, %1", double, dk, "v"(dk)) }
  else if constexpr (OP == 7) { CHAINS8("v_fma_f64 %0, %0, %1, %1", double, dk, "v"(dk)) }
  else if constexpr (OP == 8) { CHAINS8("v_mul_hi_u32 %0, %0, %1", uint32_t, uk, "v"(uk)) }
  else if constexpr (OP == 9) { CHAINS8("v_mul_lo_u32 %0, %0, %1", uint32_t, uk, "v"(uk)) }
  else if constexpr (OP == 10) {
    // v_mad_u64_u32 dst64, carry-out (vcc), src32, src32, src64: the Philox round's product
    uint64_t a0 = uk + 1, a1 = uk + 2, a2 = uk + 3, a3 = uk + 4, a4 = uk + 5, a5 = uk + 6, a6 = uk + 7, a7 = uk + 8;
    for (int it = 0; it < ITERS; ++it) {
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a0) : "v"((uint32_t)uk), "v"(uk) : "vcc");
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a1) : "v"((uint32_t)uk), "v"(uk) : "vcc");
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a2) : "v"((uint32_t)uk), "v"(uk) : "vcc");
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a3) : "v"((uint32_t)uk), "v"(uk) : "vcc");
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a4) : "v"((uint32_t)uk), "v"(uk) : "vcc");
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a5) : "v"((uint32_t)uk), "v"(uk) : "vcc");
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a6) : "v"((uint32_t)uk), "v"(uk) : "vcc");
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a7) : "v"((uint32_t)uk), "v"(uk) : "vcc");
    }
    sink = (double)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
  }
  else if constexpr (OP == 11) { CHAINS8("v_xor_b32 %0, %0, %1", uint32_t, uk, "v"(uk)) }
  else if constexpr (OP == 12) {
    CHAINS8("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf", float, fk, "v"(fk))
  }
  else if constexpr (OP == 13) { CHAINS8("v_mul_f64 %0, %0, %1", double, dk, "v"(dk)) }
  else if constexpr (OP == 14) { CHAINS8("v_cvt_f32_u32 %0, %0", uint32_t, uk, "v"(uk)) }
  else if constexpr (OP == 15) { CHAINS8("v_pk_fma_f32 %0, %0, %1, %1", double, dk, "v"(dk)) }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) cyc[wave] = t1 - t0;
  if (sink == 12345.678) out[0] = sink;  // keeps the chains alive
}

static const char* kName[] = {"v_add_f32", "v_fma_f32", "v_exp_f32", "v_sin_f32", "v_log_f32", "v_sqrt_f32",
                              "v_add_f64", "v_fma_f64", "v_mul_hi_u32", "v_mul_lo_u32", "v_mad_u64_u32",
                              "v_xor_b32", "v_mov_b32_dpp", "v_mul_f64", "v_cvt_f32_u32", "v_pk_fma_f32"};

template <int OP>
void run(int waves_per_wg, unsigned long long* dcyc, double* dout) {
  const int blocks = 256;
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(64 * waves_per_wg), 0, 0, dcyc, dout);  // warm
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(64 * waves_per_wg), 0, 0, dcyc, dout);
  (void)hipDeviceSynchronize();
  const int nw = blocks * waves_per_wg;
  std::vector<unsigned long long> c(nw);
  (void)hipMemcpy(c.data(), dcyc, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::sort(c.begin(), c.end());
  const double per_wave = (double)c[nw / 2] / (ITERS * 8.0);
  const int wps = waves_per_wg / 4;
  std::printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_wave_instr\": %.2f, \"cyc_per_simd_instr\": %.2f}\n",
              kName[OP], wps, per_wave, per_wave / wps);
}

template <int... OPS>
void all(int w, unsigned long long* c, double* o, std::integer_sequence<int, OPS...>) {
  (run<OPS>(w, c, o), ...);
}

int main() {
  unsigned long long* dcyc = nullptr;
  double* dout = nullptr;
  if (hipMalloc(&dcyc, 256 * 16 * sizeof(unsigned long long)) != hipSuccess || hipMalloc(&dout, 64) != hipSuccess) {
    std::printf("hipMalloc failed\n");
    return 1;
  }
  for (int w : {4, 8}) all(w, dcyc, dout, std::make_integer_sequence<int, 16>{});
  (void)hipFree(dcyc);
  (void)hipFree(dout);
  return 0;
}
