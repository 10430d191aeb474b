// Lorenz-96, d = 40, every 4th component observed (BASELINE configs 3 and 5).
#include "pf_ops.h"
namespace pf {
void register_l96_models() { register_both<40, 10, PF_TRANS_L96, PF_OBS_LINEAR>(); }
}  // namespace pf

#ifdef PF_STAMPS
// diagnostic build only: this code object's copy of the stamp buffer
extern "C" int pf_debug_stamps_l96(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pf::g_pf_stamps), (size_t)n * sizeof(unsigned long long));
}
#endif
