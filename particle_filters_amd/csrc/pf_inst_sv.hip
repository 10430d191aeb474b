// Scalar stochastic-volatility family: x' = alpha x + sigma n,
//   h = beta exp(x/2)            (test-harness / standard wiring, PF_OBS_EXP_HALF)
//   h = log beta^2 + x + E[..]   (log-squared wiring, PF_OBS_LINEAR)
//   y ~ N(0, beta^2 e^x)         (exact likelihood, PF_OBS_SV_EXACT)
// plus the 1-D linear test system (h = x) and the 3-D SV of the NLNGSSM notebook.
#include "pf_ops.h"
namespace pf {
void register_sv_models() {
  register_both<1, 1, PF_TRANS_LINEAR, PF_OBS_LINEAR>();
  register_both<1, 1, PF_TRANS_LINEAR, PF_OBS_EXP_HALF>();
  register_both<1, 1, PF_TRANS_LINEAR, PF_OBS_SV_EXACT>();
  register_both<3, 3, PF_TRANS_LINEAR, PF_OBS_EXP_HALF>();
}
}  // namespace pf

#ifdef PF_STAMPS
// diagnostic build only: this code object's copy of the stamp buffer
extern "C" int pf_debug_stamps_sv(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pf::g_pf_stamps), (size_t)n * sizeof(unsigned long long));
}
extern "C" int pf_debug_stamps_sv_zero(int n) {
  static unsigned long long zeros[4096];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pf::g_pf_stamps), zeros, (size_t)(n < 4096 ? n : 4096) * sizeof(unsigned long long));
}
#endif
