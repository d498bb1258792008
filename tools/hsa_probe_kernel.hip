// Kernels for tools/hsa_dispatch_probe.cpp, built as a standalone code object:
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

// tools/dispatch_rate_probe.cpp: one write-through record store per launch (the serving kernels'
// completion shape), no fence, no done word
extern "C" __global__ __launch_bounds__(64) void probe_rec(unsigned* rec, unsigned seq) {
  if (threadIdx.x == 0) __hip_atomic_store(rec, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A serving-sized (3.5 KB) kernel argument: every lane sums its share of the payload, so a stale
// or partly written argument block shows up as a wrong checksum on the host.
struct BigArgs {
  unsigned long long* out;
  unsigned* done;
  unsigned seq;
  unsigned pad;
  unsigned long long payload[440];
};

extern "C" __global__ __launch_bounds__(64) void probe_big(const BigArgs) {
  const BigArgs* a = (const BigArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < 440; i += 64) s += a->payload[i];
  a->out[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(a->done, a->seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
