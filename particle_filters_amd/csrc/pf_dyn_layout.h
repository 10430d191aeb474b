// Runtime-shape layouts shared by the kernels of pf_dyn.h and the host (pf_engine.hip):
// ParamLayout<nx, nz> and Rec<nx> (pf_models.h, pf_kernels.h) with nx / nz as values.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/pf_engine.h"

namespace pf {

constexpr int DBS = 256;                 // workgroup size of every dyn kernel
constexpr int DYN_TILE_MAX = DBS * 16;   // at most 16 particles per thread per tile
constexpr int DYN_NFM = 4 + 10;          // output fields of a covariance-carrying record (nx <= 4)

struct DynLay {
  int A, LQ, LJ, H, C, LR, EX, ILR, SIZE;
  __host__ __device__ DynLay(int nx, int nz) {
    A = 0;
    LQ = nx * nx;
    LJ = 2 * nx * nx;
    H = 3 * nx * nx;
    C = H + nz * nx;
    LR = C + nz;
    EX = LR + nz * nz;
    ILR = EX + 2 + 2 * nz;
    SIZE = ILR + nz;
  }
};

struct DynRec {
  int nx, nc, S1, S2, A1, A2, SIZE;
  bool cov;
  __host__ __device__ explicit DynRec(int n) {
    nx = n;
    cov = n <= 4;
    nc = cov ? n * (n + 1) / 2 : 0;
    S1 = 5;
    S2 = S1 + n;
    A1 = S2 + nc;
    A2 = A1 + n;
    SIZE = A2 + nc;
  }
};

// scratch rows per replicate: L96 RK4 needs three nx-row stages; every kind needs nx rows for
// a dense noise factor's normals and nz rows for a non-diagonal R's whitened residuals
__host__ __device__ inline int dyn_wrows(int tk, int nx, int nz) {
  const int a = (tk == PF_TRANS_L96 ? 3 : 1) * nx;
  return a > nz ? a : nz;
}

}  // namespace pf
