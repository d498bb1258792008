// Row-group kernel pieces (gemm_softmax.hip): the per-row online softmax state (max, sum,
// first argmax), its merges, and the argument block of the row-group kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "mlapi/kernels.h"

namespace mlapi {
namespace rows {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

constexpr int CLASS_CHUNK = 64;
constexpr float LOG2E_F = 1.4426950408889634f;

struct RowState {
  float m;  // running max logit (-inf if nothing seen yet)
  float s;  // softmax: sum exp(z - m);  OvR: sum sigmoid(z)
  int bi;   // argmax class (first max wins)
};

__device__ __forceinline__ float sigmoidf_(float z) { return 1.f / (1.f + __expf(-z)); }

__device__ __forceinline__ RowState merge_state(RowState a, RowState b, bool ovr) {
  RowState r;
  const bool take_b = (b.m > a.m) || (b.m == a.m && b.bi < a.bi);
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

__device__ __forceinline__ RowState shfl_state(RowState a, int off) {
  return RowState{__shfl_xor(a.m, off, 64), __shfl_xor(a.s, off, 64), __shfl_xor(a.bi, off, 64)};
}

// Online (max, sum, first argmax) update of a row state with the 16 logits a lane holds for one
// chunk (class of v[i] = c0 + (i >> 2) * 16 + q * 4 + (i & 3), increasing with i), in three
// stages so the pipelined loop can spread them between MFMA groups. Tree-shaped for
// instruction-level parallelism (v3 issued one 16-step cmp -> s_nop -> cndmask chain): chunk max
// by max3, first index holding it by a min tree over (v == max ? i : 16).
struct OnlineTmp {
  float m_new, part;
  int bi;
};

template <bool OVR>
__device__ __forceinline__ void online_stage(int stage, const float (&v)[16], int c0, int q, const RowState& S,
                                             OnlineTmp& T) {
  if (stage == 0) {  // chunk max, its first index, the new running max / argmax
    float m4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) m4[j] = fmaxf(fmaxf(v[4 * j], v[4 * j + 1]), fmaxf(v[4 * j + 2], v[4 * j + 3]));
    const float cm = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
    unsigned id[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) id[i] = v[i] == cm ? (unsigned)i : 16u;
    unsigned i4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) i4[j] = min(min(id[4 * j], id[4 * j + 1]), min(id[4 * j + 2], id[4 * j + 3]));
    const unsigned ci = min(min(i4[0], i4[1]), min(i4[2], i4[3]));
    const bool take = cm > S.m;  // strict: an earlier class (chunk) keeps a tie
    T.m_new = take ? cm : S.m;
    // A bit blend through an opaque mask, not a select: as a select hipcc sank the whole index
    // computation under `take` (an exec branch splitting the pipelined MFMA / epilogue block)
    // and rebuilt the min tree as a serial compare/select chain.
    const int cls = c0 + (int)((ci >> 2) * 16 + q * 4 + (ci & 3));
    int mask = -(int)take;
    asm("" : "+v"(mask));
    T.bi = S.bi ^ ((S.bi ^ cls) & mask);
  } else {  // stage 1 / 2: exp (or sigmoid) terms of elements 0-7 / 8-15
    const int i0 = stage == 1 ? 0 : 8;
    float e[8];
    if constexpr (OVR) {
#pragma unroll
      for (int i = 0; i < 8; ++i) e[i] = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-v[i0 + i] * LOG2E_F));
    } else {
      const float m2 = T.m_new * LOG2E_F;
#pragma unroll
      for (int i = 0; i < 8; ++i) e[i] = __builtin_amdgcn_exp2f(fmaf(v[i0 + i], LOG2E_F, -m2));
    }
    const float sum = ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
    T.part = stage == 1 ? sum : T.part + sum;
  }
}

template <bool OVR>
__device__ __forceinline__ void online_finish(const OnlineTmp& T, RowState& S) {
  if constexpr (OVR) {
    S.s += T.part;
  } else {
    // rescale the running sum to the new max; S.m = -inf (nothing accumulated yet) gives
    // exp2(-inf) = 0. Unconditional: a select here became a branch around the exp2. (A lane that
    // has seen only padded classes carries m = -inf with a NaN sum; merge_state drops it.)
    const float scale = __builtin_amdgcn_exp2f(fmaf(S.m, LOG2E_F, -T.m_new * LOG2E_F));
    S.s = fmaf(S.s, scale, T.part);
  }
  S.bi = T.bi;
  S.m = T.m_new;
}

template <bool OVR>
__device__ __forceinline__ void online_update(const float (&v)[16], int c0, int q, RowState& S) {
  OnlineTmp T;
  online_stage<OVR>(0, v, c0, q, S, T);
  online_stage<OVR>(1, v, c0, q, S, T);
  online_stage<OVR>(2, v, c0, q, S, T);
  online_finish<OVR>(T, S);
}

constexpr int ROWS_MAX_WAVES = 8;

struct RowsArgs {
  const uint16_t* X;
  int64_t ldx;
  const uint16_t* W;  // [K, F] bf16, row stride F
  const float* bias;
  int64_t B;
  int K;
  int F;
  int32_t* out_idx;
  float* out_p;
  RecOut ro;  // serving: per-row completion records (MODE 0)
  float* Z;
  float2* rowstat;
  float4* rowstate;
  // MODE 5
  const int32_t* y;
  uint16_t* G;  // [B][Kp] bf16, columns K..Kp-1 written 0
  int Kp;
  float* Zs;  // [B][Kp] f32: the first pass's logits, read back by the second (null: recomputed)
  float* stat_slabs;  // [gridDim.x][2] {loss, correct}
  const uint16_t* Wp;  // W in MFMA-fragment order (softmax_rows_g2_kernel<., true>), null otherwise
};

__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

// XLDS (F in (512, XLDS_FMAX], large B): the block's X rows are staged in LDS ONCE (all F; 64 rows
// x (F + 8) bf16 <= 132 KB) and every wave reads its slices from there, instead of each of the 8
// waves re-loading each slice from L2 for each of its class chunks (16x the X traffic at F = 1024);
// the registers that held X then double-buffer the W slices (the next slice's W loads are in
// flight under this slice's MFMAs). The MODE 5 second pass reuses the staged X.
constexpr int XLDS_ROWS = 64;
constexpr int XLDS_FMAX = 1024;
constexpr int XLDS_PITCH = XLDS_FMAX + 8;

typedef __attribute__((address_space(3))) void lds_void_t;
constexpr int WAIT_VM0 = (7 << 4) | (15 << 8);  // s_waitcnt vmcnt(0) (expcnt / lgkmcnt left alone)

// Stage the block's XLDS_ROWS rows of X (all F features; rows past B clamped to the last one) into
// xs by LDS-DMA: one 1 KB wave-instruction per 512 features of a row, no registers, every one in
// flight at once. (The register copy it replaces issued a dependent load -> ds_write pair per 16
// bytes per thread: 16-32 serialised HBM round trips per block before the first MFMA.) The caller
// waits WAIT_VM0 and barriers before reading xs; lanes past F read zeros (inside the row pitch).
__device__ __forceinline__ void stage_rows_dma(uint16_t (*xs)[XLDS_PITCH], const uint16_t* X, int64_t ldx, int F,
                                               int64_t row0, int64_t B, int wave, int nw, int lane) {
  const int per_row = (F + 511) / 512;
  for (int i = wave; i < XLDS_ROWS * per_row; i += nw) {
    const int r = i / per_row, j = i - r * per_row;
    const int64_t row = min(row0 + r, B - 1);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + row * ldx), 0, F * 2, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)&xs[r][512 * j], 16, (uint32_t)(lane * 16 + j * 1024),
                                             0, 0, 0);
  }
}

}  // namespace rows
}  // namespace mlapi
