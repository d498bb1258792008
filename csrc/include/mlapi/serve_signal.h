// Device side of mlapi::ServeSignal (kernels.h): the end of a serving launch publishes the batch's
// sequence number in a host-coherent done word the engine's completer spins on. Included by the
// serving kernels (linear_small.hip, gemv_binary.hip, gemm_softmax.hip); HIP device code only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mlapi {

// Every wave makes its stores visible at system scope, the block meets, and the last of the
// gridDim.x calling blocks (one block: itself) publishes `seq`. `counter` is a device word that is
// zero between launches (the last block re-arms it). Every thread of a calling block must reach
// this call; done == nullptr (library callers) makes it a no-op.
__device__ __forceinline__ void serve_signal(uint32_t* done, uint32_t seq, uint32_t* counter) {
  if (done == nullptr) return;  // uniform
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    bool last = true;
    if (gridDim.x > 1) {
      last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM) == gridDim.x - 1;
      if (last) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    if (last) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace mlapi
