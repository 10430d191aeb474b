// Wave-level exchanges and reductions on the DPP network (GFX9 DPP: quad_perm, row shifts,
// row mirrors, row_bcast) instead of LDS-crossbar shuffles (ds_bpermute): shared by the SIR step
// kernels (pf_kernels.h) and the LEDH / EDH flow kernels (pf_ledh_kernels.h).
#pragma once
#include <hip/hip_runtime.h>

namespace pf {

// ---------------------------------------------------------------------------
// Wave reductions on the DPP network (GFX9 DPP: quad_perm, row mirrors,
// row_bcast) instead of LDS-crossbar shuffles.  Fixed combination tree ->
// deterministic, identical in every workgroup.
// ---------------------------------------------------------------------------
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ int dpp_i(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ float dpp_f(float old, float v) {
  return __int_as_float(dpp_i<CTRL, RM>(__float_as_int(old), __float_as_int(v)));
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ double dpp_d(double old, double v) {
  const long long o = __double_as_longlong(old), x = __double_as_longlong(v);
  const int lo = dpp_i<CTRL, RM>((int)o, (int)x);
  const int hi = dpp_i<CTRL, RM>((int)(o >> 32), (int)(x >> 32));
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// the same move where every lane's source is valid (quad_perm, row mirrors, row_newbcast; or rows
// outside RM whose result is not read): no initialising move of the destination's old value
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ double dpp_mov_d(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)x, CTRL, RM, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(x >> 32), CTRL, RM, 0xf, true);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
enum : int {
  DPP_QP_1032 = 0xB1,
  DPP_QP_2301 = 0x4E,
  DPP_ROW_MIRROR = 0x140,
  DPP_ROW_HMIRROR = 0x141,
  DPP_ROW_BCAST15 = 0x142,
  DPP_ROW_BCAST31 = 0x143
};

// every lane of each 16-lane row gets its row's result
__device__ __forceinline__ float row_max_f(float v) {
  v = fmaxf(v, dpp_f<DPP_QP_1032>(-INFINITY, v));
  v = fmaxf(v, dpp_f<DPP_QP_2301>(-INFINITY, v));
  v = fmaxf(v, dpp_f<DPP_ROW_HMIRROR>(-INFINITY, v));
  v = fmaxf(v, dpp_f<DPP_ROW_MIRROR>(-INFINITY, v));
  return v;
}
__device__ __forceinline__ float row_sum_f(float v) {
  v += dpp_f<DPP_QP_1032>(0.0f, v);
  v += dpp_f<DPP_QP_2301>(0.0f, v);
  v += dpp_f<DPP_ROW_HMIRROR>(0.0f, v);
  v += dpp_f<DPP_ROW_MIRROR>(0.0f, v);
  return v;
}
__device__ __forceinline__ double row_sum_d(double v) {
  v += dpp_d<DPP_QP_1032>(0.0, v);
  v += dpp_d<DPP_QP_2301>(0.0, v);
  v += dpp_d<DPP_ROW_HMIRROR>(0.0, v);
  v += dpp_d<DPP_ROW_MIRROR>(0.0, v);
  return v;
}
__device__ __forceinline__ float lane63_f(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ double lane63_d(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, 63), hi = __builtin_amdgcn_readlane((int)(x >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// lane L's value (L uniform) in every lane
__device__ __forceinline__ double readlane_d(double v, int L) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, L), hi = __builtin_amdgcn_readlane((int)(x >> 32), L);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// whole-wave results (uniform: scalar registers)
__device__ __forceinline__ float wave_max_u(float v) {
  v = row_max_f(v);
  v = fmaxf(v, dpp_f<DPP_ROW_BCAST15, 0xa>(-INFINITY, v));
  v = fmaxf(v, dpp_f<DPP_ROW_BCAST31, 0xc>(-INFINITY, v));
  return lane63_f(v);
}
__device__ __forceinline__ float wave_sum_u(float v) {
  v = row_sum_f(v);
  v += dpp_f<DPP_ROW_BCAST15, 0xa>(0.0f, v);
  v += dpp_f<DPP_ROW_BCAST31, 0xc>(0.0f, v);
  return lane63_f(v);
}
__device__ __forceinline__ double wave_sum_ud(double v) {
  v = row_sum_d(v);
  v += dpp_d<DPP_ROW_BCAST15, 0xa>(0.0, v);
  v += dpp_d<DPP_ROW_BCAST31, 0xc>(0.0, v);
  return lane63_d(v);
}
__device__ __forceinline__ double wave_max_ud(double v) {
  v = fmax(v, dpp_d<DPP_QP_1032>(-INFINITY, v));
  v = fmax(v, dpp_d<DPP_QP_2301>(-INFINITY, v));
  v = fmax(v, dpp_d<DPP_ROW_HMIRROR>(-INFINITY, v));
  v = fmax(v, dpp_d<DPP_ROW_MIRROR>(-INFINITY, v));
  v = fmax(v, dpp_d<DPP_ROW_BCAST15, 0xa>(-INFINITY, v));
  v = fmax(v, dpp_d<DPP_ROW_BCAST31, 0xc>(-INFINITY, v));
  return lane63_d(v);
}

// Inclusive wave scan on the DPP network (row_shr 1/2/4/8 within 16-lane rows, then the row
// broadcasts): no LDS crossbar round trips.  A fixed order, identical in every workgroup.
__device__ __forceinline__ double wave_incl_scan_dpp(double v) {
  v += dpp_d<0x111>(0.0, v);  // row_shr:1
  v += dpp_d<0x112>(0.0, v);  // row_shr:2
  v += dpp_d<0x114>(0.0, v);  // row_shr:4
  v += dpp_d<0x118>(0.0, v);  // row_shr:8
  v += dpp_d<DPP_ROW_BCAST15, 0xa>(0.0, v);
  v += dpp_d<DPP_ROW_BCAST31, 0xc>(0.0, v);
  return v;
}

// Exchanges inside aligned 4-lane groups (quad_perm): the lane-group flow's neighbours and sums
enum : int {
  DPP_QP_ROT1 = 0x39,  // lane q reads lane (q + 1) & 3: quad_perm [1, 2, 3, 0]
  DPP_QP_ROT3 = 0x93   // lane q reads lane (q + 3) & 3: quad_perm [3, 0, 1, 2]
};
__device__ __forceinline__ double quad_sum_d(double v) {
  v += dpp_d<DPP_QP_1032>(0.0, v);
  return v + dpp_d<DPP_QP_2301>(0.0, v);
}

}  // namespace pf
