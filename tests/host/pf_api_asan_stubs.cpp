// Link stubs of the host-ASan driver (tests/host/pf_api_asan.cpp), test infrastructure only.
// The sanitizer build links the engine (pf_engine.hip) with the instantiation units of the models
// the driver runs - SV / linear scalar (pf_inst_sv), the 2-D linear systems (pf_inst_linear) and
// the runtime-shape kernels (pf_inst_dyn) - and not the L96 / acoustic / LEDH / diagnostics units,
// whose device code would triple the executable that every GPU push carries.  The engine's
// references into those units resolve here: their models stay unregistered (pf_create reports
// them unsupported) and the diagnostics entry reports an error; the driver calls neither.
#include "../../particle_filters_amd/csrc/pf_diag.h"

namespace pf {
void register_l96_models() {}
void register_mat_models() {}
namespace diag {
pf_status compute(const DiagSrc&, hipStream_t, pf_diagnostics*) { return PF_E_ARG; }
}  // namespace diag
}  // namespace pf
