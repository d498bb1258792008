// Block -> XCD placement probe for the XCD-local split merges (gemm_softmax.hip put_partial,
// linear_split.h). Those protocols rely on blocks b and b + 8k running on one XCD (round-robin
// dispatch over the 8 XCDs of an SPX-mode MI355X; the rotation's start varies from launch to
// launch): every split of a row block then meets in one XCD's L2. Before the first XCD-local launch
// on a device, 1024 blocks record the XCD they run on (HW_REG_XCC_ID); any block whose XCD differs
// from that of block b % 8 (another partition mode, another dispatch order) switches the XCD-local
// protocol off for that device, and the agent-scope protocol is used.
#include <hip/hip_runtime.h>

#include <atomic>
#include <vector>

#include "mlapi/kernels.h"

namespace mlapi {
namespace {

constexpr int PROBE_BLOCKS = 1024;
constexpr int MAX_DEVICES = 64;

__global__ __launch_bounds__(64) void xcd_probe_kernel(unsigned* out) {
  unsigned hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(hw));
  if (threadIdx.x == 0) out[blockIdx.x] = hw & 15;
}

std::atomic<int> g_state[MAX_DEVICES];  // 0 unknown, 1 placement as planned, 2 off
std::atomic<int> g_mismatch[MAX_DEVICES];

int run_probe(int dev) {
  unsigned* d = nullptr;
  hipStream_t s = nullptr;
  std::vector<unsigned> h(PROBE_BLOCKS, 0xffffffffu);
  bool ok = hipMalloc(&d, PROBE_BLOCKS * sizeof(unsigned)) == hipSuccess &&
            hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
  if (ok) {
    hipLaunchKernelGGL(xcd_probe_kernel, dim3(PROBE_BLOCKS), dim3(64), 0, s, d);
    ok = hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(h.data(), d, PROBE_BLOCKS * sizeof(unsigned), hipMemcpyDeviceToHost, s) == hipSuccess &&
         hipStreamSynchronize(s) == hipSuccess;
  }
  if (s != nullptr) (void)hipStreamDestroy(s);
  if (d != nullptr) (void)hipFree(d);
  int bad = 0;
  // the merges need blocks b and b + 8k on one XCD; the first XCD of a launch follows the
  // dispatcher's rotation (block 0 need not run on XCD 0)
  for (int b = 0; b < PROBE_BLOCKS; ++b) bad += h[b] != h[b & 7] || h[b] > 15;
  g_mismatch[dev].store(ok ? bad : -1);
  return ok && bad == 0 ? 1 : 2;
}

}  // namespace

bool xcd_local_allowed(hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEVICES) return false;
  const int st = g_state[dev].load(std::memory_order_acquire);
  if (st != 0) return st == 1;
  // no allocation or synchronisation inside a stream capture: decide at the next eager launch
  // (the plan's default - round-robin placement - holds until the probe says otherwise)
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return true;
  const int r = run_probe(dev);
  int expected = 0;
  g_state[dev].compare_exchange_strong(expected, r);
  return g_state[dev].load() == 1;
}

std::atomic<uint64_t> g_errors[MAX_DEVICES];
std::atomic<int> g_inject{0};

void xcd_local_report_error(int device) {
  if (device < 0 || device >= MAX_DEVICES) return;
  g_state[device].store(2, std::memory_order_release);
  g_errors[device].fetch_add(1);
}

uint64_t xcd_local_errors(int device) {
  if (device < 0 || device >= MAX_DEVICES) return 0;
  return g_errors[device].load();
}

void xcd_local_inject(int launches) { g_inject.store(launches); }

void xcd_local_reset(int device) {
  if (device >= 0 && device < MAX_DEVICES) g_state[device].store(0);
}

int xcd_local_take_inject() {
  int v = g_inject.load(std::memory_order_relaxed);
  while (v > 0 && !g_inject.compare_exchange_weak(v, v - 1)) {
  }
  return v > 0 ? 1 : 0;
}

int xcd_placement_state(int device) {
  if (device < 0 || device >= MAX_DEVICES) return 0;
  return g_state[device].load();
}

int xcd_placement_mismatches(int device) {
  if (device < 0 || device >= MAX_DEVICES) return -1;
  return g_mismatch[device].load();
}

}  // namespace mlapi
