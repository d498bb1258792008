// Device code shared by the row-per-lane serving kernels: the sklearn-exact epilogues
// (linear_small.hip) and the directly dispatched code object (serve_direct.hip, loaded by the
// engine through HSA: csrc/runtime/direct_dispatch.cpp). HIP device code only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace rows {

template <typename T>
__device__ __forceinline__ T dexp(T v);
template <>
__device__ __forceinline__ double dexp<double>(double v) { return exp(v); }
template <>
__device__ __forceinline__ float dexp<float>(float v) { return expf(v); }

// One row: z = x W^T + b and the sklearn epilogue of `kind`. FMAX/KMAX bound the register arrays;
// the runtime F <= FMAX, K <= KMAX. W/b indices are wave-uniform -> scalar loads.
template <typename T, int FMAX, int KMAX>
__device__ __forceinline__ void row_predict(const T* __restrict__ xr, const T* __restrict__ W,
                                            const T* __restrict__ b, int F, int K, int kind, int32_t& out_idx,
                                            T& out_p) {
  T x[FMAX];
#pragma unroll
  for (int f = 0; f < FMAX; ++f) x[f] = f < F ? xr[f] : T(0);

  T z[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k < K) {
      T acc = T(0);
#pragma unroll
      for (int f = 0; f < FMAX; ++f)
        if (f < F) acc = fma(x[f], W[k * F + f], acc);  // uniform W index -> scalar loads
      z[k] = acc + b[k];
    }
  }

  int32_t idx = 0;
  T p;
  if (kind == KIND_BINARY) {
    const T zz = z[0];
    const T p1 = T(1) / (T(1) + dexp<T>(-zz));  // scipy.special.expit
    const T p0 = T(1) - p1;                     // sklearn: vstack([1 - p, p])
    idx = zz > T(0);
    p = p0 > p1 ? p0 : p1;
    if (p1 != p1) p = p1;  // propagate NaN like ndarray.max()
  } else if (kind == KIND_BINARY_SOFTMAX) {
    const T zz = z[0];
    const T m = zz > -zz ? zz : -zz;
    const T e0 = dexp<T>(-zz - m), e1 = dexp<T>(zz - m);
    const T s = e0 + e1;
    const T q0 = e0 / s, q1 = e1 / s;
    idx = zz > T(0);
    p = q0 > q1 ? q0 : q1;
    if (s != s) p = s;
  } else if (kind == KIND_MULTINOMIAL) {
    T m = z[0];
#pragma unroll
    for (int k = 1; k < KMAX; ++k)
      if (k < K && z[k] > m) { m = z[k]; idx = k; }  // strict '>' : first max wins (np.argmax)
    T s = T(0);
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < K) s += dexp<T>(z[k] - m);  // sequential order == numpy's sum for K < 8
    p = T(1) / s;                         // max_k e_k / s with e_argmax = exp(0) = 1
    bool nan = m != m;
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < K) nan |= z[k] != z[k];
    if (nan) p = __builtin_nan("");
  } else {  // KIND_OVR: p_k = sigmoid(z_k) / sum_j sigmoid(z_j)
    T m = z[0];
#pragma unroll
    for (int k = 1; k < KMAX; ++k)
      if (k < K && z[k] > m) { m = z[k]; idx = k; }
    T s = T(0), smax = T(0);
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K) {
        const T sg = T(1) / (T(1) + dexp<T>(-z[k]));
        s += sg;
        smax = sg > smax ? sg : smax;
      }
    }
    p = smax / s;
  }
  out_idx = idx;
  out_p = p;
}


// End of a serving launch: every wave makes its stores visible at system scope, the block meets,
// and the last block to arrive (one block: itself) publishes the batch's sequence number.
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

// The rows of a kernel-argument batch (one lane per row, one block): z = x W^T + b and the epilogue,
// results straight to the (host-mapped) outputs.
template <typename T, int FMAX, int KMAX>
__device__ __forceinline__ void inline_batch_rows(const InlineBatch* a) {
  const int r = threadIdx.x;
  const int n = a->n, F = a->F, K = a->K, kind = a->kind;
  if (r < n) {
    const T* W = reinterpret_cast<const T*>(a->wb);
    const T* b = W + K * F;
    int32_t idx;
    T p;
    row_predict<T, FMAX, KMAX>(reinterpret_cast<const T*>(a->x) + r * F, W, b, F, K, kind, idx, p);
    if (a->rec != nullptr) {  // uniform: one 16-byte store carries the result and the batch's seq
      const uint64_t pb = __builtin_bit_cast(uint64_t, (double)p);
      typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
      const u32x4_t v = {a->seq, (uint32_t)idx, (uint32_t)pb, (uint32_t)(pb >> 32)};
      // System-scope (sc0 sc1) write-through vector store: the record reaches host memory without
      // a release fence or an end-of-kernel cache flush (a plain store sat in the GPU's caches
      // until something else flushed them: ~1 s with the fence-free direct-dispatch packet). The
      // compiler emits the same bits for a 4/8-byte system-scope atomic store; there is no 16-byte
      // atomic, hence the asm.
      ServeRecord* dst = static_cast<ServeRecord*>(a->rec) + (a->rec_scatter ? a->rec_idx[r] : (uint32_t)r);
      asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
    } else {
      a->out_idx[r] = idx;
      static_cast<T*>(a->out_p)[r] = p;
    }
  }
}

// Exact-shape variant (compile-time F, K: the headline Iris model is F=4, K=3). Every address is
// a constant offset from the kernarg base or the lane's row, so all loads issue at once: the
// runtime-shape kernel first waits for the header (n, F, K), then issues guarded loads, then walks
// W with a scalar load and a wait per element (5+ dependent round trips to the freshly written
// kernarg memory). Lanes past n read a clamped in-bounds row and do not store.
template <typename T, int F, int K>
__device__ __forceinline__ void inline_batch_rows_exact(const InlineBatch* a) {
  constexpr int XCAP = INLINE_X_BYTES / (F * (int)sizeof(T));
  const int r = threadIdx.x;
  const int rr = r < XCAP ? r : XCAP - 1;
  const T* W = reinterpret_cast<const T*>(a->wb);
  int32_t idx;
  T p;
  row_predict<T, F, K>(reinterpret_cast<const T*>(a->x) + rr * F, W, W + K * F, F, K, a->kind, idx, p);
  if (r >= a->n) return;
  if (a->rec != nullptr) {
    const uint64_t pb = __builtin_bit_cast(uint64_t, (double)p);
    typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
    const u32x4_t v = {a->seq, (uint32_t)idx, (uint32_t)pb, (uint32_t)(pb >> 32)};
    ServeRecord* dst = static_cast<ServeRecord*>(a->rec) + (a->rec_scatter ? a->rec_idx[r] : (uint32_t)r);
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
  } else {
    a->out_idx[r] = idx;
    static_cast<T*>(a->out_p)[r] = p;
  }
}

}  // namespace rows
}  // namespace mlapi
