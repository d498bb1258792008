// Epilogues for sharded linear models (SURVEY 2.5 TP row, 5.7 "wide F" row): the GEMM runs on each
// rank's shard with the gemm_softmax tiles; these kernels finish the prediction after the
// collective.
//
//  * class-sharded (TP over K): every rank publishes the online softmax state {max logit, sum-exp
//    relative to that max (OvR: sum of sigmoids), argmax} of its class range per row
//    (gemm_softmax MODE 4); after an all-gather, merge_rowstates folds the N states in rank order
//    (= increasing class order, so the first maximum still wins) into (label, p_max). Only 16 B per
//    row cross xGMI instead of B x K logits.
//  * feature-sharded (split-F across GPUs): every rank computes partial logits X_r W_r^T of its
//    feature slice (gemm_softmax MODE 1), an all-reduce sums them, and logits_epilogue adds the
//    bias and applies the sklearn epilogue of `kind` row by row (one wave per row).
#include <hip/hip_runtime.h>

#include <cmath>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace {

struct State {
  float m, s;
  int bi;
};

// a precedes b in class order (a comes from the lower rank / lower class index): on an equal max
// the lower class index wins, which is also the earlier state.
__device__ __forceinline__ State merge(State a, State b, bool ovr) {
  const bool take_b = b.m > a.m || (b.m == a.m && b.bi < a.bi);
  State r;
  r.m = take_b ? b.m : a.m;
  r.bi = take_b ? b.bi : a.bi;
  if (ovr) {
    r.s = a.s + b.s;
  } else {
    const float sa = a.m == -INFINITY ? 0.f : a.s * __expf(a.m - r.m);
    const float sb = b.m == -INFINITY ? 0.f : b.s * __expf(b.m - r.m);
    r.s = sa + sb;
  }
  return r;
}

__device__ __forceinline__ float sigmoid(float z) { return 1.f / (1.f + __expf(-z)); }

__global__ __launch_bounds__(256) void merge_rowstates_kernel(const float4* __restrict__ parts, int nparts,
                                                              int64_t B, ShardOffsets offs, int ovr,
                                                              int32_t* __restrict__ out_idx,
                                                              float* __restrict__ out_p) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  State S{-INFINITY, 0.f, 0x7fffffff};
  for (int k = 0; k < nparts; ++k) {  // fixed rank order: deterministic
    const float4 p = parts[(int64_t)k * B + r];
    S = merge(S, State{p.x, p.y, __float_as_int(p.z) + offs.off[k]}, ovr != 0);
  }
  out_idx[r] = S.bi;
  out_p[r] = ovr ? sigmoid(S.m) / S.s : 1.f / S.s;
}

// One wave per row: lane l owns classes l, l + 64, ...; online state per lane, then a butterfly
// merge (the xor partner order does not change the result: ties resolve by class index).
__global__ __launch_bounds__(256) void logits_epilogue_kernel(const float* __restrict__ Z, const float* __restrict__ b,
                                                              int64_t B, int K, int kind,
                                                              int32_t* __restrict__ out_idx,
                                                              float* __restrict__ out_p) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;  // wave-uniform
  const float* z = Z + r * K;
  if (kind == KIND_BINARY || kind == KIND_BINARY_SOFTMAX) {  // K == 1
    if (lane == 0) {
      const float zz = z[0] + b[0];
      out_idx[r] = zz > 0.f;
      out_p[r] = sigmoid((kind == KIND_BINARY ? 1.f : 2.f) * fabsf(zz));
    }
    return;
  }
  const bool ovr = kind == KIND_OVR;
  State S{-INFINITY, 0.f, 0x7fffffff};
  for (int k = lane; k < K; k += 64) {
    const float v = z[k] + b[k];
    if (ovr) {
      S.s += sigmoid(v);
      if (v > S.m) {
        S.m = v;
        S.bi = k;
      }
    } else if (v > S.m) {  // strict: the first (lowest class) maximum of this lane wins
      S.s = (S.m == -INFINITY ? 0.f : S.s * __expf(S.m - v)) + 1.f;
      S.m = v;
      S.bi = k;
    } else {
      S.s += __expf(v - S.m);
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const State o{__shfl_xor(S.m, off, 64), __shfl_xor(S.s, off, 64), __shfl_xor(S.bi, off, 64)};
    S = (lane & off) ? merge(o, S, ovr) : merge(S, o, ovr);
  }
  if (lane == 0) {
    out_idx[r] = S.bi;
    out_p[r] = ovr ? sigmoid(S.m) / S.s : 1.f / S.s;
  }
}

}  // namespace

void launch_merge_rowstates(const void* parts, int nparts, int64_t B, const ShardOffsets& offs, int kind,
                            int32_t* out_idx, float* out_p, hipStream_t stream) {
  if (B <= 0) return;
  if (nparts < 1 || nparts > ShardOffsets::MAX)
    throw std::invalid_argument("merge_rowstates: 1..64 shards");
  if (kind != KIND_MULTINOMIAL && kind != KIND_OVR) throw std::invalid_argument("merge_rowstates: multiclass kinds");
  hipLaunchKernelGGL(merge_rowstates_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, stream,
                     static_cast<const float4*>(parts), nparts, B, offs, kind == KIND_OVR ? 1 : 0, out_idx, out_p);
  MLAPI_HIP_CHECK(hipGetLastError());
}

void launch_logits_epilogue(const float* Z, const float* b, int64_t B, int K, int kind, int32_t* out_idx, float* out_p,
                            hipStream_t stream) {
  if (B <= 0) return;
  if (K < 1 || ((kind == KIND_BINARY || kind == KIND_BINARY_SOFTMAX) && K != 1))
    throw std::invalid_argument("logits_epilogue: binary kinds need K == 1");
  hipLaunchKernelGGL(logits_epilogue_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, stream, Z, b, B, K, kind,
                     out_idx, out_p);
  MLAPI_HIP_CHECK(hipGetLastError());
}

}  // namespace mlapi
