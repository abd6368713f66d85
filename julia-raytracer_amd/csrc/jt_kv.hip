// jt_kv.hip — one kernel configuration of the megakernel (jt_kernels.h, LaunchConfig<JT_VARIANT>),
// instantiated for both samplers and both counter levels. The Makefile compiles this file once
// per configuration (-DJT_VARIANT=0..NUM_LAUNCH_CONFIGS-1), so the kernels build in parallel.
#include "jt_kernels.h"

#ifndef JT_VARIANT
#error "JT_VARIANT (the LaunchConfig index) must be defined"
#endif

namespace jtk {
static_assert(JT_VARIANT >= 0 && JT_VARIANT < NUM_LAUNCH_CONFIGS, "JT_VARIANT out of range");
JT_KV_FOR(JT_VARIANT, template)
}  // namespace jtk
