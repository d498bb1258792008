// Host launchers of the class-split multiclass predict (linear_split.h).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

#include "linear_split.h"
#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace {

// workspace: [64 row-group counters (B <= 2048)] [xcd error word at byte 256] [pad] [partials]
constexpr size_t COUNTER_REGION = 512;
constexpr size_t MAX_ROW_GROUPS = 64;
static_assert(MAX_ROW_GROUPS * split::ROWS_PER_GROUP == (size_t)LINEAR_SPLIT_MAX_ROWS, "split row cap");
constexpr size_t XCD_ERR_OFFSET = 256;

template <typename T, int KS, int NB, bool OVR>
__global__ __launch_bounds__(256) void linear_split_kernel(split::SplitArgs a) {
  split::split_predict<T, KS, NB, OVR>(a);
}

int g_split_xcd = -1;  // test hook (linear_split_set_xcd): -1 = MLAPI_SPLIT_XCD / default, 0 off, 1 on

template <typename T, int KS>
void launch_ks(split::SplitArgs a, dim3 grid, bool nb2, bool ovr, hipStream_t stream, KernelLauncher* direct) {
  if (direct != nullptr) {
    // the same kernel, unmangled, in the serving code object (serve_direct.hip)
    char name[64];
    std::snprintf(name, sizeof name, "mlapi_split_%s_ks%d_nb%d_%s", sizeof(T) == 2 ? "bf16" : "f32", KS, nb2 ? 2 : 1,
                  ovr ? "ovr" : "mn");
    // host merge (hrec): write-through records and no workspace - unordered; the in-kernel merge
    // re-arms the workspace counters for the next launch - ordered
    if (direct->launch_kernel(name, &a, sizeof a, grid.x, grid.y, 256, a.hrec == nullptr)) return;
  }
  {  // a launch being captured into a HIP graph replays its epoch: its merger clears the tags
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
    a.clear_tags = cs == hipStreamCaptureStatusActive ? 1 : 0;
  }
  if (nb2) {
    if (ovr)
      hipLaunchKernelGGL((linear_split_kernel<T, KS, 2, true>), grid, dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((linear_split_kernel<T, KS, 2, false>), grid, dim3(256), 0, stream, a);
  } else {
    if (ovr)
      hipLaunchKernelGGL((linear_split_kernel<T, KS, 1, true>), grid, dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((linear_split_kernel<T, KS, 1, false>), grid, dim3(256), 0, stream, a);
  }
}

int row_groups(int64_t B) { return (int)((B + split::ROWS_PER_GROUP - 1) / split::ROWS_PER_GROUP); }
int nsplits(int K) { return (K + split::CLASSES_PER_BLOCK - 1) / split::CLASSES_PER_BLOCK; }

}  // namespace

bool linear_split_supported(int dt, int F) {
  const bool pow2 = F > 0 && (F & (F - 1)) == 0;
  if (dt == DT_BF16) return pow2 && F >= 32 && F <= 512;
  if (dt == DT_F32) return pow2 && F >= 16 && F <= 512;
  return false;
}

size_t linear_split_xcd_err_offset() { return XCD_ERR_OFFSET; }

void linear_split_set_xcd(int mode) { g_split_xcd = mode; }

size_t linear_split_workspace(int64_t B, int K) {
  const int rg = row_groups(B);
  return COUNTER_REGION + (size_t)rg * nsplits(K) * split::ROWS_PER_GROUP * sizeof(float4);
}

int linear_split_nsplit(int K) { return nsplits(K); }

void launch_linear_split(int dt, const void* X, int64_t ldx, const void* W, const float* b, int64_t B, int F, int K,
                         int kind, int32_t* out_idx, float* out_p, void* workspace, size_t ws_bytes,
                         hipStream_t stream, RecOut ro, SplitRecOut sro, KernelLauncher* direct) {
  if (B <= 0) return;
  if (!linear_split_supported(dt, F))
    throw std::invalid_argument("linear_split: bf16 F in 32..512 or f32 F in 16..512, a power of two");
  if (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("linear_split: multiclass kinds only");
  if (ldx < F || (ldx * (dt == DT_BF16 ? 2 : 4)) % 16 != 0)
    throw std::invalid_argument("linear_split: ldx must be >= F and rows 16-byte aligned");
  if (reinterpret_cast<uintptr_t>(X) % 16 != 0 || reinterpret_cast<uintptr_t>(W) % 16 != 0)
    throw std::invalid_argument("linear_split: X and W must be 16-byte aligned");
  const int rg = row_groups(B), ns = nsplits(K);
  if (rg > (int)MAX_ROW_GROUPS)
    throw std::invalid_argument("linear_split: B too large (<= LINEAR_SPLIT_MAX_ROWS rows per launch)");
  if (sro.rec != nullptr && rg != 1) throw std::invalid_argument("linear_split: host merge needs B <= 32");
  if (sro.rec == nullptr && ns > 1 && ws_bytes < linear_split_workspace(B, K))
    throw std::invalid_argument("linear_split: workspace too small (zero it once)");
  split::SplitArgs a{};
  a.X = X;
  a.ldx = ldx;
  a.W = W;
  a.bias = b;
  a.B = (int32_t)B;
  a.K = K;
  a.kind = kind;
  a.nsplit = ns;
  a.out_idx = out_idx;
  a.out_p = out_p;
  a.ro = ro;
  a.counters = static_cast<unsigned int*>(workspace);
  a.partials = reinterpret_cast<float4*>(static_cast<unsigned char*>(workspace) + COUNTER_REGION);
  static const int probe = [] {
    const char* e = getenv("MLAPI_SPLIT_PROBE");
    return e ? atoi(e) : 0;
  }();
  a.probe = probe;
  a.hrec = reinterpret_cast<uint4*>(sro.rec);
  a.rec_seq = sro.seq;
  // XCD-local merge (linear_split.h): default on; MLAPI_SPLIT_XCD=0 selects the agent-scope protocol
  static const int xcd_env = [] {
    const char* e = getenv("MLAPI_SPLIT_XCD");
    return e ? atoi(e) : 1;
  }();
  const int xcd_on = g_split_xcd >= 0 ? g_split_xcd : xcd_env;
  a.xcd_local = (xcd_on != 0 && ns > 1 && sro.rec == nullptr && xcd_local_allowed(stream)) ? 1 : 0;
  a.xcd_inject = a.xcd_local ? xcd_local_take_inject() : 0;
  // Split-merge granule tags: 28 bits, never 0, from one process-wide counter. Eager launches do
  // not clear the tags they consumed, so a granule keeps the epoch of the last launch that wrote
  // it; the counter wraps after 2^28 launches, and a granule left untouched for exactly that many
  // launches would match again. Bound: the engine's serving launches are one row group (B <= 32,
  // every split rewritten per launch, a workspace per model), so they never leave one behind;
  // library callers that alternate large and small batches on one workspace over 2^28 launches
  // should re-zero it (linear_split_workspace bytes) now and then. Graph captures clear their tags.
  static std::atomic<uint32_t> epochs{0};
  do a.epoch = (epochs.fetch_add(1, std::memory_order_relaxed) + 1) & 0x0fffffffu;
  while (a.epoch == 0);
  a.clear_tags = 0;  // direct-dispatched launches are never captured (launch_ks sets it for stream launches)
  a.row_groups = rg;
  a.xcd_err = reinterpret_cast<unsigned int*>(static_cast<unsigned char*>(workspace) + XCD_ERR_OFFSET);
  // XCD-ordered 1-D grid: 8 XCDs x ceil(rg / 8) row groups x ns splits (blocks past rg exit at once)
  const dim3 grid = a.xcd_local ? dim3((unsigned)(8 * ((rg + 7) / 8) * ns), 1u) : dim3((unsigned)ns, (unsigned)rg);
  const bool nb2 = B > 16;
  const bool ovr = kind == KIND_OVR;
  if (dt == DT_BF16) {
    switch (F) {
      case 32: launch_ks<uint16_t, 1>(a, grid, nb2, ovr, stream, direct); break;
      case 64: launch_ks<uint16_t, 2>(a, grid, nb2, ovr, stream, direct); break;
      case 128: launch_ks<uint16_t, 4>(a, grid, nb2, ovr, stream, direct); break;
      case 256: launch_ks<uint16_t, 8>(a, grid, nb2, ovr, stream, direct); break;
      default: launch_ks<uint16_t, 16>(a, grid, nb2, ovr, stream, direct); break;
    }
  } else {
    switch (F) {
      case 16: launch_ks<float, 1>(a, grid, nb2, ovr, stream, direct); break;
      case 32: launch_ks<float, 2>(a, grid, nb2, ovr, stream, direct); break;
      case 64: launch_ks<float, 4>(a, grid, nb2, ovr, stream, direct); break;
      case 128: launch_ks<float, 8>(a, grid, nb2, ovr, stream, direct); break;
      case 256: launch_ks<float, 16>(a, grid, nb2, ovr, stream, direct); break;
      default: launch_ks<float, 32>(a, grid, nb2, ovr, stream, direct); break;
    }
  }
  MLAPI_HIP_CHECK(hipGetLastError());
}

}  // namespace mlapi
