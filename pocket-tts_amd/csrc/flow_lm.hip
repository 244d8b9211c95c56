// Product build of the persistent FlowLM transformer entry points (kernels.h: flow_lm*): no
// launch. The persistent kernel (probes/flow_lm.hip) was measured slower than the 48 launches it
// replaces, so only the -DPTTS_PROBES measurement build compiles it, in place of
// this file; Engine::use_flow_lm never selects it here.
#include <stdexcept>

#include "kernels.h"

namespace ptts {
bool flow_lm_fits(int) { return false; }
size_t flow_lm_set_floats() { return 0; }
int flow_lm_grid() { return 0; }
int flow_lm_max_resident(int) { return 0; }
void flow_lm(const FlowLmArgs&, hipStream_t) { throw std::runtime_error("flow_lm: probe builds only"); }
}  // namespace ptts
