// Joint multi-target acoustic tracking: 4 CV targets (nx = 16), 5x5 sensor grid (BASELINE config 4).
#include "pf_ops.h"
namespace pf {
void register_mat_models() { register_both<16, 25, PF_TRANS_LINEAR, PF_OBS_ACOUSTIC>(); }
}  // namespace pf

#ifdef PF_STAMPS
// diagnostic build only: this code object's copy of the stamp buffer
extern "C" int pf_debug_stamps_mat(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pf::g_pf_stamps), (size_t)n * sizeof(unsigned long long));
}
#endif
