// Binary logistic-regression predict over a large batch: z = X w + b, label = z > 0,
// p_max = sigmoid(|z|)  (BASELINE config 2: 1M x 256 bf16; reference op K1+K3+K5).
//
// Roofline: 1M x 256 bf16 = 512 MiB read once (> 256 MiB Infinity Cache) vs 8 B/row written,
// ~1 FLOP/byte -> HBM-bound; target ~6 TB/s => ~85 us. Design (cdna_hip_programming.md
// "GEMV / M <= 16" row: no LDS round trip):
//  * a row is split into 16-byte chunks; LPR lanes cover one row (F=256 bf16: 32 lanes, so one
//    global_load_dwordx4 wave-instruction reads 2 full rows = 1 KiB, perfectly coalesced);
//  * each lane keeps its weight chunk in registers for the whole kernel (w read once per wave);
//  * U rows per lane-group are loaded back-to-back (U x 16 B in flight per lane, non-temporal:
//    X is streamed exactly once) before any is consumed -> latency hidden by ILP + 8 waves/SIMD;
//  * bf16 products use v_dot2_f32_bf16 (2 MACs per instruction, f32 accumulate);
//  * the U partial dot products are reduced across the LPR lanes with a butterfly
//    reduce-scatter: log2(U) halving steps + the remaining xor steps (9 shuffles for U=8,
//    LPR=32 instead of 40), after which lane groups own whole rows and one lane per row writes.
// Shared by gemv_binary.hip (hipLaunchKernel) and serve_direct.hip (the engine's AQL queue).
#pragma once
#include <hip/hip_runtime.h>

#include "mlapi/common.h"
#include "mlapi/kernels.h"
#include "mlapi/device.h"
#include "mlapi/rowreduce.h"

namespace mlapi {
namespace gemv {

// the kernel's by-value argument block (its whole kernarg segment)
struct GemvArgs {
  const void* X;  // [B][F] row stride F, 16-byte aligned
  const void* w;  // [F]
  float bias;
  int32_t F;
  int64_t B;
  int32_t kind;
  int32_t blocks;  // grid size (256-thread blocks)
  int32_t* out_idx;
  float* out_p;
  RecOut ro;
};

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

template <typename T>
struct Chunk;  // 16 bytes of one row
template <>
struct Chunk<uint16_t> {
  static constexpr int N = 8;
  // Elements are copied out by value before the bit_cast: __builtin_bit_cast of an ext-vector
  // element lvalue (x.y) reads from the vector's base address in this clang (every component
  // came out as x.x and the loads shrank to dwords).
  __device__ static __forceinline__ bf16x2_t bf2(uint32_t u) { return __builtin_bit_cast(bf16x2_t, u); }
  __device__ static __forceinline__ float dot(const u32x4_t& x, const u32x4_t& w, float acc) {
    acc = __builtin_amdgcn_fdot2_f32_bf16(bf2(x.x), bf2(w.x), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(bf2(x.y), bf2(w.y), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(bf2(x.z), bf2(w.z), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(bf2(x.w), bf2(w.w), acc, false);
    return acc;
  }
};
template <>
struct Chunk<float> {
  static constexpr int N = 4;
  __device__ static __forceinline__ float dot(const u32x4_t& x, const u32x4_t& w, float acc) {
    acc = fmaf(__uint_as_float(x.x), __uint_as_float(w.x), acc);
    acc = fmaf(__uint_as_float(x.y), __uint_as_float(w.y), acc);
    acc = fmaf(__uint_as_float(x.z), __uint_as_float(w.z), acc);
    acc = fmaf(__uint_as_float(x.w), __uint_as_float(w.w), acc);
    return acc;
  }
};

template <typename T, int LPR, int CPL, int U>
__device__ __forceinline__ void gemv_rows(const GemvArgs& a) {
  const T* __restrict__ X = static_cast<const T*>(a.X);
  const T* __restrict__ w = static_cast<const T*>(a.w);
  const float bias = a.bias;
  const int64_t B = a.B;
  const int F = a.F, kind = a.kind;
  int32_t* __restrict__ out_idx = a.out_idx;
  float* __restrict__ out_p = a.out_p;
  const RecOut& ro = a.ro;
  constexpr int RPW = 64 / LPR;  // rows per wave-instruction
  constexpr int NE = Chunk<T>::N;
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR;       // row within the wave-instruction
  const int cl = lane % LPR;        // chunk lane
  const int chunks = F / NE;        // 16-byte chunks per row
  const int64_t ld16 = chunks;      // row stride in uint4

  u32x4_t wv[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = cl + c * LPR;
    wv[c] = ch < chunks ? reinterpret_cast<const u32x4_t*>(w)[ch] : u32x4_t{0u, 0u, 0u, 0u};
  }
  const float scale = kind == KIND_BINARY_SOFTMAX ? 2.f : 1.f;
  const int slot = slot_of<LPR, U>(lane % LPR);
  const bool writer = ((lane % LPR) & writer_mask<LPR, U>()) == 0;

  const int64_t rows_per_wave_iter = (int64_t)U * RPW;
  // 4 waves per block; the grid size comes in the arguments (no implicit kernel argument is read,
  // so the serving code object's entries take the GemvArgs block alone)
  const int64_t waves_total = (int64_t)a.blocks * 4;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR
  const u32x4_t* X16 = reinterpret_cast<const u32x4_t*>(X);
  // Chunk column per c, clamped into the row (lanes past the last chunk have zero weights).
  int coff[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) coff[c] = min(cl + c * LPR, chunks - 1);
  const int64_t stride_u = (int64_t)RPW * ld16;

  for (int64_t base = wave_id * rows_per_wave_iter; base < B; base += waves_total * rows_per_wave_iter) {
    // Unconditional loads: full iterations (wave-uniform test) use one base pointer + constant
    // strides, only the final partial one clamps its rows.
    u32x4_t xv[U][CPL];
    if (base + rows_per_wave_iter <= B) {
      const u32x4_t* p = X16 + (base + sub) * ld16;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < CPL; ++c) xv[u][c] = __builtin_nontemporal_load(p + u * stride_u + coff[c]);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = min(base + (int64_t)u * RPW + sub, B - 1);
#pragma unroll
        for (int c = 0; c < CPL; ++c) xv[u][c] = __builtin_nontemporal_load(X16 + row * ld16 + coff[c]);
      }
    }
    float part[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc = Chunk<T>::dot(xv[u][c], wv[c], acc);
      part[u] = acc;
    }
    const float z0 = reduce_scatter<LPR, U>(part, lane % LPR);
    const int64_t row = base + (int64_t)slot * RPW + sub;
    if (writer && row < B) {
      const float z = z0 + bias;
      const float a = scale * fabsf(z);
      put_result(out_idx, out_p, ro, row, z > 0.f, 1.f / (1.f + __expf(-a)));
    }
  }
}

}  // namespace gemv
}  // namespace mlapi
