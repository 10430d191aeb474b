// Small dense linear / elementwise-SV systems (tests/unit_tests/models/test_pf_*.py fixtures).
#include "pf_ops.h"
namespace pf {
void register_linear_models() {
  register_both<2, 1, PF_TRANS_LINEAR, PF_OBS_LINEAR>();
  register_both<2, 2, PF_TRANS_LINEAR, PF_OBS_LINEAR>();
  register_both<2, 2, PF_TRANS_LINEAR, PF_OBS_EXP_HALF>();
}
}  // namespace pf
