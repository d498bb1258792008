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
    a->out_idx[r] = idx;
    static_cast<T*>(a->out_p)[r] = p;
  }
}

}  // namespace rows
}  // namespace mlapi
