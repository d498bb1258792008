// Dtype packing (SURVEY 2.3 K0 / "pack_weights"): f64 / f32 / bf16 conversions for weights and
// staged inputs. f32 -> bf16 uses the compiler's round-to-nearest-even cast, which lowers to
// v_cvt_pk_bf16_f32 on gfx950 and keeps NaNs NaN (MI355X_MICROARCH.md "Correctness boundaries").
// 4 elements per thread, vectorized where the dtype allows.
#include <hip/hip_runtime.h>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace {

template <typename S>
__device__ __forceinline__ float to_f32(S v);
template <>
__device__ __forceinline__ float to_f32<double>(double v) { return (float)v; }
template <>
__device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f32<uint16_t>(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }

template <typename D>
__device__ __forceinline__ D from_f64(double v);
template <>
__device__ __forceinline__ double from_f64<double>(double v) { return v; }
template <>
__device__ __forceinline__ float from_f64<float>(double v) { return (float)v; }
template <>
__device__ __forceinline__ uint16_t from_f64<uint16_t>(double v) {
  return __builtin_bit_cast(uint16_t, (__bf16)(float)v);
}

template <typename S>
__device__ __forceinline__ double to_f64(S v) { return (double)to_f32<S>(v); }
template <>
__device__ __forceinline__ double to_f64<double>(double v) { return v; }

template <typename S, typename D>
__global__ __launch_bounds__(256) void cast_kernel(const S* __restrict__ src, D* __restrict__ dst, int64_t n) {
  const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = i0 + j;
    if (i < n) dst[i] = from_f64<D>(to_f64<S>(src[i]));
  }
}

template <typename S>
void dispatch_dst(const S* src, int dst_dt, void* dst, int64_t n, hipStream_t stream) {
  const dim3 grid((unsigned)((n + 1023) / 1024));
  if (dst_dt == DT_F64)
    hipLaunchKernelGGL((cast_kernel<S, double>), grid, dim3(256), 0, stream, src, static_cast<double*>(dst), n);
  else if (dst_dt == DT_F32)
    hipLaunchKernelGGL((cast_kernel<S, float>), grid, dim3(256), 0, stream, src, static_cast<float*>(dst), n);
  else
    hipLaunchKernelGGL((cast_kernel<S, uint16_t>), grid, dim3(256), 0, stream, src, static_cast<uint16_t*>(dst), n);
  MLAPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

void launch_cast(int src_dt, const void* src, int dst_dt, void* dst, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  if (src_dt == DT_F64)
    dispatch_dst(static_cast<const double*>(src), dst_dt, dst, n, stream);
  else if (src_dt == DT_F32)
    dispatch_dst(static_cast<const float*>(src), dst_dt, dst, n, stream);
  else
    dispatch_dst(static_cast<const uint16_t*>(src), dst_dt, dst, n, stream);
}

}  // namespace mlapi
