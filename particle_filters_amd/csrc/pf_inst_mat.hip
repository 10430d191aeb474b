// Joint multi-target acoustic tracking: 4 CV targets (nx = 16), 5x5 sensor grid (BASELINE config 4).
#include "pf_ops.h"
namespace pf {
void register_mat_models() { register_both<16, 25, PF_TRANS_LINEAR, PF_OBS_ACOUSTIC>(); }
}  // namespace pf
