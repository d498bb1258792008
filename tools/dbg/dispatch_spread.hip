// Workgroup start spread of small grids: every block's first wave stamps the 100 MHz wall clock
// at entry (lane 0, vector store); the host prints quantiles of (entry - first entry) over many
// launches, for grids shaped like the serving WIDE kernel (63-126 blocks) at 64 / 256 / 512
// threads, with and without a large LDS / VGPR footprint.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/dispatch_spread tools/dbg/dispatch_spread.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                                \
    }                                                                          \
  } while (0)

template <int LDS_DOUBLES>
__global__ void stamp_kernel(uint64_t* out, int spin) {
  __shared__ double lds[LDS_DOUBLES > 0 ? LDS_DOUBLES : 1];
  const uint64_t t = wall_clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = t;
  // a little work so the block is resident for a while (not a store-only kernel)
  double acc = threadIdx.x;
  for (int i = 0; i < spin; ++i) acc = acc * 1.0000001 + 0.5;
  if (LDS_DOUBLES > 0) {
    lds[threadIdx.x % LDS_DOUBLES] = acc;
    __syncthreads();
    acc += lds[(threadIdx.x + 1) % LDS_DOUBLES];
  }
  if (acc == 12345.678) out[0] = 0;
}

template <int LDS_DOUBLES>
static int run(const char* name, int blocks, int threads, int iters) {
  uint64_t* d = nullptr;
  CK(hipMalloc(&d, blocks * sizeof(uint64_t)));
  std::vector<uint64_t> h(blocks);
  std::vector<double> last, med;
  for (int it = 0; it < iters + 10; ++it) {
    hipLaunchKernelGGL(stamp_kernel<LDS_DOUBLES>, dim3(blocks), dim3(threads), 0, 0, d, 200);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, blocks * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (it < 10) continue;
    std::vector<uint64_t> s = h;
    std::sort(s.begin(), s.end());
    last.push_back((s.back() - s.front()) / 100.0);
    med.push_back((s[blocks / 2] - s.front()) / 100.0);
  }
  std::sort(last.begin(), last.end());
  std::sort(med.begin(), med.end());
  std::printf("%-22s blocks %4d threads %4d: entry spread median-block %.2f us, last-block p50 %.2f p90 %.2f us\n", name,
              blocks, threads, med[med.size() / 2], last[last.size() / 2], last[last.size() * 9 / 10]);
  CK(hipFree(d));
  return 0;
}

int main() {
  const int iters = 200;
  for (int blocks : {63, 126, 252}) {
    for (int threads : {64, 256, 512}) {
      if (run<0>("plain", blocks, threads, iters)) return 1;
      if (run<1024>("lds 8KB", blocks, threads, iters)) return 1;
    }
  }
  return 0;
}
