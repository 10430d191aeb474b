// Lorenz-96, d = 40, every 4th component observed (BASELINE configs 3 and 5).
#include "pf_ops.h"
namespace pf {
void register_l96_models() { register_both<40, 10, PF_TRANS_L96, PF_OBS_LINEAR>(); }
}  // namespace pf
