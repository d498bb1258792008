// Host launchers of the f64-accumulating wide-model predict (linear_wide.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

#include "linear_wide.h"
#include "wide_plan.h"
#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace {

template <typename T, int NB>
__global__ __launch_bounds__(256) void linear_wide_kernel(wide::WideArgs a) {
  wide::wide_predict<T, NB>(a);
}

static_assert(wide::CB == wide_plan::CB && wide::RG == wide_plan::RG && wide::WAVES == wide_plan::WAVES,
              "linear_wide.h and wide_plan.h disagree on the geometry");
using wide_plan::row_groups;

}  // namespace

int g_probe = 0;  // measurement hooks (linear_wide_set_probe / _set_trace)
uint64_t* g_trace = nullptr;

WidePlan linear_wide_plan(int dt, int F, int K) { return wide_plan::plan(dt, F, K); }

void linear_wide_set_probe(int probe) { g_probe = probe; }

void linear_wide_set_trace(void* trace) { g_trace = static_cast<uint64_t*>(trace); }

size_t linear_wide_workspace(int64_t B, int dt, int F, int K) { return wide_plan::workspace(B, dt, F, K); }

void launch_linear_wide(int dt, const void* X, int64_t ldx, const void* W, const double* b, int64_t B, int F, int K,
                        int kind, int32_t* out_idx, double* out_p, void* workspace, size_t ws_bytes, hipStream_t stream,
                        RecOut ro, WideRecOut hro, KernelLauncher* direct, bool ws_private) {
  if (B <= 0) return;
  const WidePlan p = linear_wide_plan(dt, F, K);
  const bool binary = kind == KIND_BINARY || kind == KIND_BINARY_SOFTMAX;
  if (binary ? K != 1 : (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR)))
    throw std::invalid_argument("linear_wide: binary kinds take K = 1, multiclass kinds K >= 2");
  if (ldx < p.ldx) throw std::invalid_argument("linear_wide: ldx below the plan's padded width");
  const size_t es = dt == DT_F64 ? 8 : 4;
  if ((ldx * es) % 16 != 0 || reinterpret_cast<uintptr_t>(X) % 16 != 0 || reinterpret_cast<uintptr_t>(W) % 16 != 0)
    throw std::invalid_argument("linear_wide: X and W rows must be 16-byte aligned");
  // host-merged launches (<= 32 rows) need ONE row group: 17-32 rows take the 2-tile group even
  // where the planner would spread a small batch over more blocks
  const int nb = hro.rec != nullptr && B > 16 ? 2 : wide_plan::tiles_per_group(B, p);
  const int rg = row_groups(B, nb);
  if (rg > 65535) throw std::invalid_argument("linear_wide: B too large for one launch");
  if (hro.rec != nullptr && (rg != 1 || binary)) throw std::invalid_argument("linear_wide: host merge needs one row group, multiclass");
  const bool needs_ws = p.nfs > 1 || (!binary && p.ncb > 1 && hro.rec == nullptr);
  if (needs_ws && ws_bytes < linear_wide_workspace(B, dt, F, K))
    throw std::invalid_argument("linear_wide: workspace too small (zero it once)");
  wide::WideArgs a{};
  a.X = X;
  a.ldx = ldx;
  a.W = W;
  a.bias = b;
  a.B = (int32_t)B;
  a.K = K;
  a.kind = kind;
  a.ncb = p.ncb;
  a.nfs = p.nfs;
  a.fsteps = p.fsteps;
  a.out_idx = out_idx;
  a.out_p = out_p;
  a.ro = ro;
  a.hrec = reinterpret_cast<uint4*>(hro.rec);
  a.hseq = hro.seq;
  a.row_groups = rg;
  a.probe = g_probe;
  a.trace = g_trace;
  a.clear_tags = 0;  // direct-dispatched launches are never captured (set below for the stream launch)
  static std::atomic<uint32_t> epochs{0};  // class-merge granule tags: distinct per launch, never 0
  a.epoch = epochs.fetch_add(1, std::memory_order_relaxed) + 1;
  if (a.epoch == 0) a.epoch = epochs.fetch_add(1, std::memory_order_relaxed) + 1;
  const wide_plan::Layout lay = wide_plan::layout(p);
  a.ws = static_cast<unsigned char*>(workspace);
  a.rg_bytes = (int64_t)lay.rg_bytes;
  a.cnt_bytes = (int64_t)lay.cnt_bytes;
  a.part_bytes = (int64_t)lay.part_bytes;
  const dim3 grid((unsigned)(p.ncb * p.nfs), (unsigned)rg);
  const bool nb2 = nb == 2;
  if (direct != nullptr) {
    char name[48];
    std::snprintf(name, sizeof name, "mlapi_wide_%s_nb%d", dt == DT_F64 ? "f64" : "f32", nb2 ? 2 : 1);
    // the workspace's tickets are re-armed by the kernel: launches that share them stay in order
    // (a workspace private to this launch lets it overlap the previous ones)
    if (direct->launch_kernel(name, &a, sizeof a, grid.x, grid.y, 256, needs_ws && !ws_private)) return;
  }
  {  // a launch being captured into a HIP graph replays its epoch: its merger clears the tags
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
    a.clear_tags = cs == hipStreamCaptureStatusActive ? 1 : 0;
  }
  if (dt == DT_F64) {
    if (nb2)
      hipLaunchKernelGGL((linear_wide_kernel<double, 2>), grid, dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((linear_wide_kernel<double, 1>), grid, dim3(256), 0, stream, a);
  } else {
    if (nb2)
      hipLaunchKernelGGL((linear_wide_kernel<float, 2>), grid, dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((linear_wide_kernel<float, 1>), grid, dim3(256), 0, stream, a);
  }
  MLAPI_HIP_CHECK(hipGetLastError());
}

}  // namespace mlapi
