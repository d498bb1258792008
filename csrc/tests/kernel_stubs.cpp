// Link stubs for host-only test binaries (tools/sanitize.sh): the CPU backend (device = -1) never
// launches a kernel, so the GPU launchers are replaced by functions that fail loudly if reached.
#include <stdexcept>

#include "mlapi/kernels.h"
#include "../runtime/direct_dispatch.h"
#include "../kernels/wide_plan.h"

namespace mlapi {
[[noreturn]] static void unreachable(const char* what) {
  throw std::logic_error(std::string("host-only test binary: ") + what + " must not be reached");
}
void launch_linear_small(int, const void*, int64_t, const void*, const void*, int64_t, int, int, int, int32_t*, void*,
                         hipStream_t, const ServeSignal&) {
  unreachable("launch_linear_small");
}
void launch_serve_signal(const ServeSignal&, hipStream_t) { unreachable("launch_serve_signal"); }
bool linear_inline_fits(int, int64_t, int, int) { return false; }
void launch_linear_inline(int, const InlineBatch&, hipStream_t) { unreachable("launch_linear_inline"); }
void launch_gemv_binary(int, const void*, const void*, float, int64_t, int, int, int32_t*, float*, hipStream_t, RecOut,
                        KernelLauncher*) {
  unreachable("launch_gemv_binary");
}
size_t gemm_softmax_workspace(int64_t, int, int) { return 0; }
void launch_gemm_softmax(const void*, const void*, const float*, int64_t, int, int, int, int32_t*, float*, void*, size_t,
                         hipStream_t, RecOut) {
  unreachable("launch_gemm_softmax");
}
bool linear_split_supported(int, int) { return false; }
size_t linear_split_workspace(int64_t, int) { return 0; }
int linear_split_nsplit(int K) { return (K + 63) / 64; }
void xcd_local_report_error(int) {}
void launch_linear_split(int, const void*, int64_t, const void*, const float*, int64_t, int, int, int, int32_t*, float*,
                         void*, size_t, hipStream_t, RecOut, SplitRecOut, KernelLauncher*) {
  unreachable("launch_linear_split");
}
WidePlan linear_wide_plan(int dt, int F, int K) { return wide_plan::plan(dt, F, K); }
void linear_wide_set_probe(int) {}
void linear_wide_set_trace(void*) {}
size_t linear_wide_workspace(int64_t B, int dt, int F, int K) { return wide_plan::workspace(B, dt, F, K); }
void launch_linear_wide(int, const void*, int64_t, const void*, const double*, int64_t, int, int, int, int32_t*, double*,
                        void*, size_t, hipStream_t, RecOut, WideRecOut, KernelLauncher*, bool) {
  unreachable("launch_linear_wide");
}
std::unique_ptr<InlineDispatcher> make_direct_dispatcher(int, const std::string&, int, std::string* why) {
  if (why) *why = "host-only build";
  return nullptr;
}
}  // namespace mlapi
