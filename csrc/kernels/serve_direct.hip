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
#include "gemv_binary.h"
#include "linear_split.h"
#include "linear_wide.h"
#include "serve_resident.h"

namespace {

template <typename T, int FMAX, int KMAX, bool EXACT = false>
__device__ __forceinline__ void direct_inline() {
  const mlapi::InlineBatch* a = (const mlapi::InlineBatch*)__builtin_amdgcn_kernarg_segment_ptr();
  if constexpr (EXACT)
    mlapi::rows::inline_batch_rows_exact<T, FMAX, KMAX>(a);
  else
    mlapi::rows::inline_batch_rows<T, FMAX, KMAX>(a);
  if (a->done == nullptr) return;  // uniform
  if (a->rec_scatter) {            // uniform: in-flight accounting only (records are already out)
    if (threadIdx.x == 0) {
      const uint32_t v = a->seq;
      asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(a->done), "v"(v) : "memory");
    }
    return;
  }
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

// The class-split multiclass predict (linear_split.h) for the engine's wide serving batches: the
// same device code as linear_split.hip's linear_split_kernel<T, KS, NB, OVR>, one unmangled entry
// per instantiation (launch_linear_split formats the name). It reads no implicit kernel argument
// (no gridDim / blockDim), so the kernarg block is the SplitArgs alone.
#define MLAPI_SPLIT_ENTRY(TN, T, KS, NB, OVR, SUF)                                                        \
  extern "C" __global__ __launch_bounds__(256) void mlapi_split_##TN##_ks##KS##_nb##NB##_##SUF(          \
      const mlapi::split::SplitArgs a) {                                                                \
    mlapi::split::split_predict<T, KS, NB, OVR>(a);                                                     \
  }
#define MLAPI_SPLIT_ENTRIES(TN, T, KS)           \
  MLAPI_SPLIT_ENTRY(TN, T, KS, 1, false, mn)     \
  MLAPI_SPLIT_ENTRY(TN, T, KS, 1, true, ovr)     \
  MLAPI_SPLIT_ENTRY(TN, T, KS, 2, false, mn)     \
  MLAPI_SPLIT_ENTRY(TN, T, KS, 2, true, ovr)
MLAPI_SPLIT_ENTRIES(bf16, uint16_t, 1)
MLAPI_SPLIT_ENTRIES(bf16, uint16_t, 2)
MLAPI_SPLIT_ENTRIES(bf16, uint16_t, 4)
MLAPI_SPLIT_ENTRIES(bf16, uint16_t, 8)
MLAPI_SPLIT_ENTRIES(bf16, uint16_t, 16)
MLAPI_SPLIT_ENTRIES(f32, float, 1)
MLAPI_SPLIT_ENTRIES(f32, float, 2)
MLAPI_SPLIT_ENTRIES(f32, float, 4)
MLAPI_SPLIT_ENTRIES(f32, float, 8)
MLAPI_SPLIT_ENTRIES(f32, float, 16)
MLAPI_SPLIT_ENTRIES(f32, float, 32)

// The binary GEMV (gemv_binary.h) for record-completing wide binary batches: the entries of
// gemv_binary.hip's dispatch table, named mlapi_gemv_<dtype>_l<LPR>_c<CPL>_u<U>.
#define MLAPI_GEMV_ENTRY(TN, T, LPR, CPL, U)                                                                    \
  extern "C" __global__ __launch_bounds__(256) void mlapi_gemv_##TN##_l##LPR##_c##CPL##_u##U(                   \
      const mlapi::gemv::GemvArgs a) {                                                                          \
    mlapi::gemv::gemv_rows<T, LPR, CPL, U>(a);                                                                  \
  }
#define MLAPI_GEMV_ENTRIES(TN, T) \
  MLAPI_GEMV_ENTRY(TN, T, 4, 1, 4)   \
  MLAPI_GEMV_ENTRY(TN, T, 8, 1, 8)   \
  MLAPI_GEMV_ENTRY(TN, T, 16, 1, 8)  \
  MLAPI_GEMV_ENTRY(TN, T, 32, 1, 8)  \
  MLAPI_GEMV_ENTRY(TN, T, 64, 1, 8)  \
  MLAPI_GEMV_ENTRY(TN, T, 64, 2, 4)  \
  MLAPI_GEMV_ENTRY(TN, T, 64, 4, 2)  \
  MLAPI_GEMV_ENTRY(TN, T, 64, 8, 1)
MLAPI_GEMV_ENTRIES(bf16, uint16_t)
MLAPI_GEMV_ENTRIES(f32, float)

// The f64-accumulating wide predict (linear_wide.h) for wide f64 / f32 models: the entries of
// linear_wide.hip's kernel, named mlapi_wide_<storage dtype>_nb<row tiles>.
#define MLAPI_WIDE_ENTRY(TN, T, NB)                                                                      \
  extern "C" __global__ __launch_bounds__(256) void mlapi_wide_##TN##_nb##NB(const mlapi::wide::WideArgs a) { \
    mlapi::wide::wide_predict<T, NB>(a);                                                                 \
  }
MLAPI_WIDE_ENTRY(f64, double, 1)
MLAPI_WIDE_ENTRY(f64, double, 2)
MLAPI_WIDE_ENTRY(f32, float, 1)
MLAPI_WIDE_ENTRY(f32, float, 2)

// The resident SMALL-path kernel (serve_resident.h): one wave per IO thread's submission ring,
// launched by the engine's supervisor onto a queue of its own. mlapi_resident_<dt>_r<LPE>_d<D>:
// LPE lanes per row (F <= LPE), D host-memory polls in flight.
#define MLAPI_RESIDENT_ENTRY(TN, T, LPE, D)                                                                      \
  extern "C" __global__ __launch_bounds__(64) void mlapi_resident_##TN##_r##LPE##_d##D(const mlapi::ResidentArgs a) { \
    mlapi::resident::resident_serve<T, LPE, D, 16>(a);                                                        \
  }
#define MLAPI_RESIDENT_ENTRIES(TN, T, LPE) \
  MLAPI_RESIDENT_ENTRY(TN, T, LPE, 1)      \
  MLAPI_RESIDENT_ENTRY(TN, T, LPE, 2)      \
  MLAPI_RESIDENT_ENTRY(TN, T, LPE, 4)
MLAPI_RESIDENT_ENTRIES(f64, double, 4)
MLAPI_RESIDENT_ENTRIES(f64, double, 8)
MLAPI_RESIDENT_ENTRIES(f64, double, 32)
MLAPI_RESIDENT_ENTRIES(f32, float, 4)
MLAPI_RESIDENT_ENTRIES(f32, float, 8)
MLAPI_RESIDENT_ENTRIES(f32, float, 32)
