// Fused small linear classifier: z = x W^T + b -> (label index, max class probability).
//
// Replaces the reference's per-request sklearn calls `loaded_model.predict(data_in)` and
// `loaded_model.predict_proba(data_in).max()` (main.py:21-22), which compute the decision
// function twice (K1 in SURVEY 2.3) and then argmax / softmax / max (K2-K5). Here the decision
// function is computed once per row and the epilogue produces only what /predict returns.
//
// Regime: Iris-scale models (F=4, K=3) at serving batch sizes (B = 1..a few thousand rows) are
// pure launch/latency-bound: 12 FMAs per row. One lane owns one row; W and b are wave-uniform
// and come in through the scalar cache (s_load) so every lane reads its x row from (host-mapped
// or device) memory exactly once. fp64 keeps bit-level parity with sklearn's float64 math
// (same epilogue formulas and summation order as numpy for K < 8); fp32 is the fast path.
#include <hip/hip_runtime.h>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace {

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


template <typename T, int FMAX, int KMAX>
__global__ __launch_bounds__(256) void linear_small_kernel(const T* __restrict__ X, int64_t ldx,
                                                           const T* __restrict__ W, const T* __restrict__ b,
                                                           int64_t B, int F, int K, int kind,
                                                           int32_t* __restrict__ out_idx, T* __restrict__ out_p) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  row_predict<T, FMAX, KMAX>(X + r * ldx, W, b, F, K, kind, out_idx[r], out_p[r]);
}

// Generic fallback for wider models (F > 32 or K > 16): one pass, online (max, sum-exp).
template <typename T>
__device__ __forceinline__ void row_predict_generic(const T* __restrict__ xr, const T* __restrict__ W,
                                                    const T* __restrict__ b, int F, int K, int kind,
                                                    int32_t& out_idx, T& out_p) {
  if (K == 1) {
    T acc = T(0);
    for (int f = 0; f < F; ++f) acc = fma(xr[f], W[f], acc);
    const T zz = acc + b[0];
    const T a = kind == KIND_BINARY ? (zz < 0 ? -zz : zz) : T(2) * (zz < 0 ? -zz : zz);
    out_idx = zz > T(0);
    out_p = T(1) / (T(1) + dexp<T>(-a));
    return;
  }
  T m = -__builtin_huge_val(), s = T(0);
  int32_t idx = 0;
  for (int k = 0; k < K; ++k) {
    T acc = T(0);
    for (int f = 0; f < F; ++f) acc = fma(xr[f], W[(int64_t)k * F + f], acc);
    const T zz = acc + b[k];
    if (kind == KIND_OVR) {
      s += T(1) / (T(1) + dexp<T>(-zz));
      if (zz > m || k == 0) { m = zz; idx = k; }
    } else if (zz > m) {
      s = s * dexp<T>(m - zz) + T(1);
      m = zz;
      idx = k;
    } else {
      s += dexp<T>(zz - m);
    }
  }
  out_idx = idx;
  out_p = kind == KIND_OVR ? (T(1) / (T(1) + dexp<T>(-m))) / s : T(1) / s;
}

template <typename T>
__global__ __launch_bounds__(256) void linear_generic_kernel(const T* __restrict__ X, int64_t ldx,
                                                             const T* __restrict__ W, const T* __restrict__ b,
                                                             int64_t B, int F, int K, int kind,
                                                             int32_t* __restrict__ out_idx, T* __restrict__ out_p) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  row_predict_generic<T>(X + r * ldx, W, b, F, K, kind, out_idx[r], out_p[r]);
}

// ---- persistent serving kernel --------------------------------------------------------------
// One resident workgroup that takes batches from a host-pinned mailbox instead of one kernel
// launch per batch: the host batcher writes the rows and the header, then publishes the slot's
// sequence number (release); thread 0 polls it (system-scope acquire over the host link, s_sleep
// between polls), the block computes the rows straight from / to host memory (zero-copy), and
// publishes `done` (system-scope release). Batches are consumed strictly in sequence order.
// The kernel leaves when told to stop or after `idle_ticks` of the constant-rate wall clock
// without work, so a device-wide synchronize in the process returns once traffic pauses; the
// engine relaunches it on demand (csrc/runtime/engine.cpp).
template <typename T>
__global__ __launch_bounds__(256) void serve_persistent_kernel(ServeMailSlot* mail, uint32_t* done,
                                                               const uint32_t* stop, int nslots,
                                                               uint64_t start_seq, uint64_t idle_ticks) {
  __shared__ ServeMailSlot hdr;
  __shared__ int go;
  uint64_t seq = start_seq;  // batch index; slot = seq % nslots, published value = seq + 1
  for (;;) {
    const int slot = (int)(seq % (uint64_t)nslots);
    if (threadIdx.x == 0) {
      const uint64_t t0 = wall_clock64();
      int g = 0;
      for (;;) {
        const uint32_t v = __hip_atomic_load(&mail[slot].seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v == (uint32_t)(seq + 1)) {
          g = 1;
          break;
        }
        if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
        if (wall_clock64() - t0 > idle_ticks) break;
        __builtin_amdgcn_s_sleep(8);
      }
      if (g) hdr = mail[slot];
      go = g;
    }
    __syncthreads();
    if (!go) return;  // every thread of the block leaves together
    const int n = (int)hdr.n, F = hdr.F, K = hdr.K, kind = hdr.kind;
    const T* X = reinterpret_cast<const T*>(hdr.x);
    const T* W = reinterpret_cast<const T*>(hdr.W);
    const T* b = reinterpret_cast<const T*>(hdr.b);
    int32_t* oi = reinterpret_cast<int32_t*>(hdr.idx);
    T* op = reinterpret_cast<T*>(hdr.p);
    for (int r = threadIdx.x; r < n; r += blockDim.x) {
      int32_t idx;
      T p;
      if (F <= 8 && K <= 4)
        row_predict<T, 8, 4>(X + (int64_t)r * F, W, b, F, K, kind, idx, p);
      else if (F <= 32 && K <= 16)
        row_predict<T, 32, 16>(X + (int64_t)r * F, W, b, F, K, kind, idx, p);
      else
        row_predict_generic<T>(X + (int64_t)r * F, W, b, F, K, kind, idx, p);
      oi[r] = idx;
      op[r] = p;
    }
    __threadfence_system();  // results reach host memory before `done`
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(&done[slot * SERVE_DONE_STRIDE], (uint32_t)(seq + 1), __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    ++seq;
  }
}

template <typename T>
void dispatch(const void* X, int64_t ldx, const void* W, const void* b, int64_t B, int F, int K, int kind,
              int32_t* out_idx, void* out_p, hipStream_t stream) {
  if (B <= 0) return;
  const int threads = B <= 64 ? 64 : 256;  // tiny serving batches: one wave, no idle waves
  const dim3 grid((unsigned)((B + threads - 1) / threads));
  auto x = static_cast<const T*>(X);
  auto w = static_cast<const T*>(W);
  auto bb = static_cast<const T*>(b);
  auto p = static_cast<T*>(out_p);
  if (F <= 8 && K <= 4)
    hipLaunchKernelGGL((linear_small_kernel<T, 8, 4>), grid, dim3(threads), 0, stream, x, ldx, w, bb, B, F, K, kind,
                       out_idx, p);
  else if (F <= 32 && K <= 16)
    hipLaunchKernelGGL((linear_small_kernel<T, 32, 16>), grid, dim3(threads), 0, stream, x, ldx, w, bb, B, F, K,
                       kind, out_idx, p);
  else
    hipLaunchKernelGGL((linear_generic_kernel<T>), grid, dim3(threads), 0, stream, x, ldx, w, bb, B, F, K, kind,
                       out_idx, p);
  MLAPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

void launch_serve_persistent(int dt, ServeMailSlot* mail, uint32_t* done, const uint32_t* stop, int nslots,
                             uint64_t start_seq, uint64_t idle_ticks, hipStream_t stream) {
  if (dt == DT_F64)
    hipLaunchKernelGGL((serve_persistent_kernel<double>), dim3(1), dim3(256), 0, stream, mail, done, stop, nslots,
                       start_seq, idle_ticks);
  else if (dt == DT_F32)
    hipLaunchKernelGGL((serve_persistent_kernel<float>), dim3(1), dim3(256), 0, stream, mail, done, stop, nslots,
                       start_seq, idle_ticks);
  else
    throw std::invalid_argument("serve_persistent: dtype must be f64 or f32");
  MLAPI_HIP_CHECK(hipGetLastError());
}

void launch_linear_small(int dt, const void* X, int64_t ldx, const void* W, const void* b, int64_t B, int F, int K,
                         int kind, int32_t* out_idx, void* out_p, hipStream_t stream) {
  if (dt == DT_F64)
    dispatch<double>(X, ldx, W, b, B, F, K, kind, out_idx, out_p, stream);
  else if (dt == DT_F32)
    dispatch<float>(X, ldx, W, b, B, F, K, kind, out_idx, out_p, stream);
  else
    throw std::invalid_argument("linear_small: dtype must be f64 or f32");
}

}  // namespace mlapi
