// Kernel for tools/hsa_dispatch_probe.cpp, built as a standalone code object:
//   hipcc --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -O3 tools/hsa_probe_kernel.hip -o probe.hsaco
#include <hip/hip_runtime.h>

extern "C" __global__ __launch_bounds__(64) void probe_flag(int* idx, double* p, unsigned* done, unsigned seq) {
  idx[threadIdx.x] = (int)(threadIdx.x + seq);
  p[threadIdx.x] = 0.5 * threadIdx.x + seq;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
