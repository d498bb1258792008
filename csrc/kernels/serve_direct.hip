// Serving kernels of the directly dispatched code object (mlapi_amd/serve_kernels.hsaco).
//
// The engine writes AQL packets for these kernels into its own HSA queue
// (csrc/runtime/direct_dispatch.cpp) instead of calling hipLaunchKernel: the submit costs ~0.03 us
// of batcher CPU instead of ~2.5 us, and launch -> done word is ~2 us shorter (5.3 vs 7.5 us,
// tools/hsa_dispatch_probe.cpp). Same row code as linear_small.hip (linear_rows.h); unmangled
// names so the loader finds them; one block, so the done word needs no counter and no implicit
// kernel argument (grid size) is read: the kernarg segment holds the InlineBatch only.
//   hipcc --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -O3 ... -o serve_kernels.hsaco
#include <hip/hip_runtime.h>

#include "linear_rows.h"

namespace {

template <typename T, int FMAX, int KMAX, bool EXACT = false>
__device__ __forceinline__ void direct_inline() {
  const mlapi::InlineBatch* a = (const mlapi::InlineBatch*)__builtin_amdgcn_kernarg_segment_ptr();
  if constexpr (EXACT)
    mlapi::rows::inline_batch_rows_exact<T, FMAX, KMAX>(a);
  else
    mlapi::rows::inline_batch_rows<T, FMAX, KMAX>(a);
  if (a->done == nullptr) return;  // uniform
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(a->done, a->seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

// (F <= 8, K <= 4) and (F <= 32, K <= 16) register shapes, f64 (sklearn parity) and f32
extern "C" __global__ __launch_bounds__(128) void mlapi_inline_f64_s(const mlapi::InlineBatch) {
  direct_inline<double, 8, 4>();
}
extern "C" __global__ __launch_bounds__(128) void mlapi_inline_f64_w(const mlapi::InlineBatch) {
  direct_inline<double, 32, 16>();
}
extern "C" __global__ __launch_bounds__(128) void mlapi_inline_f32_s(const mlapi::InlineBatch) {
  direct_inline<float, 8, 4>();
}
extern "C" __global__ __launch_bounds__(128) void mlapi_inline_f32_w(const mlapi::InlineBatch) {
  direct_inline<float, 32, 16>();
}
// exact F=4, K=3 (the headline Iris shape): all loads in one batch
extern "C" __global__ __launch_bounds__(128) void mlapi_inline_f64_4x3(const mlapi::InlineBatch) {
  direct_inline<double, 4, 3, true>();
}
extern "C" __global__ __launch_bounds__(128) void mlapi_inline_f32_4x3(const mlapi::InlineBatch) {
  direct_inline<float, 4, 3, true>();
}
