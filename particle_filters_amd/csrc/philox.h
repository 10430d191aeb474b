// Counter-based Philox4x32-10 (Salmon et al., SC'11) and Box-Muller normals.
//
// Every random number of the SIR step is a pure function of
//   key     = (seed_lo, seed_hi)
//   counter = (group index, replicate, epoch, stream)
// so any lane can draw its own numbers with no state and no ordering between
// workgroups: the same (seed, replicate) reproduces bit-identically whatever the
// grid, the replicate-to-GPU sharding or the call pattern (predict/update split
// vs the fused device-resident T loop).
//
// "group index" enumerates the normals of a draw in NumPy's row-major order
// (particle i, state dim d) -> flat f = i*nx + d: one Philox call yields the
// 4 normals f = 4g..4g+3 (two Box-Muller pairs).  fp32 and fp64 engines use the
// same 32-bit uniforms; only the Box-Muller arithmetic precision differs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pf {

enum : uint32_t {
  STREAM_INIT = 1,      // initialize(): particles ~ N(mean, cov)
  STREAM_PROCESS = 2,   // predict(): process noise
  STREAM_JITTER = 3,    // post-resample regularisation
  STREAM_RESAMPLE = 4,  // systematic U / multinomial uniforms
};

struct u32x4 {
  uint32_t x, y, z, w;
};

// PF_PHILOX_ROUNDS: experiment builds only (timing ablations, tools/build_sv_variants.sh); the
// shipped library and the oracle use the 10 rounds of Philox4x32-10.
#ifndef PF_PHILOX_ROUNDS
#define PF_PHILOX_ROUNDS 10
#endif
__host__ __device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < PF_PHILOX_ROUNDS; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c.x;
    const uint64_t p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// Uniform in (0, 1] from 32 random bits (never 0, so log() is finite).
__device__ __forceinline__ float u01_f32(uint32_t a) {
  return ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ double u01_f64(uint32_t a) {
  return ((double)a + 1.0) * (1.0 / 4294967296.0);
}
// Uniform in [0, 1) with 53 bits from two words (systematic U, multinomial u).
__host__ __device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  return (double)(((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6)) * (1.0 / 9007199254740992.0);
}

template <typename Real>
struct Normal4 {
  Real v[4];
};

// Box-Muller on the two pairs (x, y) and (z, w): r = sqrt(-2 ln u1), angle 2*pi*u2.
// fp32: the hardware v_sin/v_cos (argument in revolutions, so 2*pi*u2 needs no
// range reduction), v_log and v_sqrt — a handful of instructions per pair.  u1 is a
// normal float in [2^-24, 1], so the radius takes the raw v_log_f32 (log2, 1 ulp) times
// 2 ln 2 — no denormal rescaling and no compensated ln2 product (__logf's 10 instructions).
__device__ __forceinline__ float neg2_ln_u01(uint32_t a) {
  return -1.3862943611198906f * __builtin_amdgcn_logf(u01_f32(a));  // -2 ln u = -2 ln2 log2 u
}
__device__ __forceinline__ Normal4<float> box_muller4(u32x4 r) {
  Normal4<float> n;
  const float r0 = __builtin_amdgcn_sqrtf(neg2_ln_u01(r.x));
  const float r1 = __builtin_amdgcn_sqrtf(neg2_ln_u01(r.z));
  const float a0 = (float)(r.y >> 8) * (1.0f / 16777216.0f);
  const float a1 = (float)(r.w >> 8) * (1.0f / 16777216.0f);
  n.v[0] = r0 * __builtin_amdgcn_cosf(a0);
  n.v[1] = r0 * __builtin_amdgcn_sinf(a0);
  n.v[2] = r1 * __builtin_amdgcn_cosf(a1);
  n.v[3] = r1 * __builtin_amdgcn_sinf(a1);
  return n;
}
__device__ __forceinline__ Normal4<double> box_muller4_f64(u32x4 r) {
  Normal4<double> n;
  const double r0 = sqrt(-2.0 * log(u01_f64(r.x)));
  const double r1 = sqrt(-2.0 * log(u01_f64(r.z)));
  double s0, c0, s1, c1;
  sincospi((double)(r.y >> 8) * (2.0 / 16777216.0), &s0, &c0);
  sincospi((double)(r.w >> 8) * (2.0 / 16777216.0), &s1, &c1);
  n.v[0] = r0 * c0;
  n.v[1] = r0 * s0;
  n.v[2] = r1 * c1;
  n.v[3] = r1 * s1;
  return n;
}

template <typename Real>
__device__ __forceinline__ Normal4<Real> normal4(uint64_t seed, uint32_t group, uint32_t rep,
                                                 uint32_t epoch, uint32_t stream);
template <>
__device__ __forceinline__ Normal4<float> normal4<float>(uint64_t seed, uint32_t group, uint32_t rep,
                                                         uint32_t epoch, uint32_t stream) {
  return box_muller4(philox4x32_10(u32x4{group, rep, epoch, stream}, (uint32_t)seed,
                                   (uint32_t)(seed >> 32)));
}
template <>
__device__ __forceinline__ Normal4<double> normal4<double>(uint64_t seed, uint32_t group, uint32_t rep,
                                                           uint32_t epoch, uint32_t stream) {
  return box_muller4_f64(philox4x32_10(u32x4{group, rep, epoch, stream}, (uint32_t)seed,
                                       (uint32_t)(seed >> 32)));
}

// The flow filters' (LEDH / EDH, fp64 state) process-noise normals: the fp32 Box-Muller of the
// SIR engine's fp32 path (24-bit uniforms, hardware transcendentals) widened to double.  The
// fp64 Box-Muller (sincospi, log, sqrt in double) cost ~200 fp64 instructions per 4 normals and
// was the longest phase of the fused LEDH step's per-particle chain; a normal with 24-bit
// resolution is a draw of the same N(0, 1) (the reference's own draws come from NumPy's PCG64
// and are not reproduced bit for bit in device-RNG mode anyway), truncated where the 24-bit
// uniform bottoms out: |n| <= sqrt(-2 ln 2^-24) = 5.77 sigma (8e-9 of the N(0, 1) mass is never
// drawn).  tests/test_bm24_normals.py checks moments, tail masses to 5 sigma and the cut.
__device__ __forceinline__ Normal4<double> normal4_bm24d(uint64_t seed, uint32_t group, uint32_t rep,
                                                         uint32_t epoch, uint32_t stream) {
  const Normal4<float> f = normal4<float>(seed, group, rep, epoch, stream);
  return Normal4<double>{{(double)f.v[0], (double)f.v[1], (double)f.v[2], (double)f.v[3]}};
}

// element k (0..3, a run-time index) by selects: indexing the register array with k would put
// it in scratch memory
template <typename Real>
__device__ __forceinline__ Real pick4(const Normal4<Real>& q, int k) {
  const Real lo = (k & 1) ? q.v[1] : q.v[0], hi = (k & 1) ? q.v[3] : q.v[2];
  return (k & 2) ? hi : lo;
}

// One [0,1) double per (index, replicate, epoch) on the resample stream.
__host__ __device__ __forceinline__ double uniform53(uint64_t seed, uint32_t index, uint32_t rep,
                                                     uint32_t epoch) {
  u32x4 r = philox4x32_10(u32x4{index, rep, epoch, STREAM_RESAMPLE}, (uint32_t)seed,
                          (uint32_t)(seed >> 32));
  return u53(r.x, r.y);
}

}  // namespace pf
