// Internal interface of the diagnostics module (pf_diag.hip) for the engines' state entries.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/pf_diag.h"

namespace pf {
namespace diag {

// One filter state in HBM.  Weights: normalised fp64 w [N], or (w == null) log weights lw [Npad]
// of the storage type with the normaliser lse (w_i = exp(lw_i - lse)), or uniform (1/N).
// Particles: SoA x [nx][Npad] of the storage type, or null.
struct DiagSrc {
  int64_t N, Npad;
  int nx;
  const double* w;
  const void* lw;
  double lse;
  int uniform;
  const void* x;
  int real_is_double;
  double tol;     // unique-row rounding grid (diag:39-58)
  double spread;  // trace(cov) when known, NaN -> computed from the particles
};

pf_status compute(const DiagSrc& s, hipStream_t stream, pf_diagnostics* out);

}  // namespace diag
}  // namespace pf
