// Link stubs for host-only test binaries (tools/sanitize.sh): the CPU backend (device = -1) never
// launches a kernel, so the GPU launchers are replaced by functions that fail loudly if reached.
#include <stdexcept>

#include "mlapi/kernels.h"

namespace mlapi {
void launch_linear_small(int, const void*, int64_t, const void*, const void*, int64_t, int, int, int, int32_t*, void*,
                         hipStream_t) {
  throw std::logic_error("host-only test binary: launch_linear_small must not be reached");
}
void launch_serve_persistent(int, ServeMailSlot*, uint32_t*, const uint32_t*, int, uint64_t, uint64_t, hipStream_t) {
  throw std::logic_error("host-only test binary: launch_serve_persistent must not be reached");
}
}  // namespace mlapi
