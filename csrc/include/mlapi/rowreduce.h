// Cross-lane row reductions shared by the row-streaming kernels (gemv_binary, train_binary).
//
// A wave holds U row-slots x (64/LPR) rows; each row is spread over LPR lanes, every lane has a
// partial dot product per slot. The butterfly reduce-scatter halves the number of live slots on
// each of the first log2(U) xor steps (lower half of the lane pair keeps slots [0, H), upper half
// keeps [H, 2H)) and finishes with plain xor-adds, so after log2(LPR) shuffles every lane holds the
// FULL sum of exactly one slot (slot_of) and each slot is held by LPR/U lanes (owner_of = lowest).
//
// Everything is resolved at compile time via recursion on (OFF, CNT): a runtime loop counter here
// made hipcc lower the slot selects into compare/select chains over the whole partial array
// (hundreds of v_cmp_eq + v_cndmask per iteration in the disassembly).
#pragma once
#include <hip/hip_runtime.h>

namespace mlapi {

template <int OFF, int CNT, int U>
__device__ __forceinline__ void reduce_scatter_step(float (&p)[U], int cl) {
  if constexpr (OFF >= 1) {
    if constexpr (CNT > 1) {
      constexpr int H = CNT / 2;
      const bool upper = (cl & OFF) != 0;
#pragma unroll
      for (int j = 0; j < H; ++j) {
        const float keep = upper ? p[j + H] : p[j];
        const float send = upper ? p[j] : p[j + H];
        p[j] = keep + __shfl_xor(send, OFF, 64);
      }
      reduce_scatter_step<OFF / 2, H, U>(p, cl);
    } else {
      p[0] += __shfl_xor(p[0], OFF, 64);
      reduce_scatter_step<OFF / 2, 1, U>(p, cl);
    }
  }
}

// Returns the full sum of slot slot_of<LPR, U>(cl) (cl = lane index within its LPR group).
template <int LPR, int U>
__device__ __forceinline__ float reduce_scatter(float (&p)[U], int cl) {
  static_assert(U <= LPR, "reduce-scatter needs U <= LPR");
  reduce_scatter_step<LPR / 2, U, U>(p, cl);
  return p[0];
}

template <int LPR, int U>
__host__ __device__ constexpr int slot_of(int cl) {
  int u = 0, cnt = U;
  for (int off = LPR / 2; off >= 1; off >>= 1) {
    if (cnt > 1) {
      const int half = cnt / 2;
      if (cl & off) u += half;
      cnt = half;
    }
  }
  return u;
}

// Lowest lane (within the LPR group) holding slot u.
template <int LPR, int U>
__host__ __device__ constexpr int owner_of(int u) {
  int lane = 0, cnt = U;
  for (int off = LPR / 2; off >= 1; off >>= 1) {
    if (cnt > 1) {
      const int half = cnt / 2;
      if (u >= half) {
        lane += off;
        u -= half;
      }
      cnt = half;
    }
  }
  return lane;
}

// Lanes whose bits under this mask are zero are the owners (one writer per slot).
template <int LPR, int U>
__host__ __device__ constexpr int writer_mask() {
  int cnt = U, last = LPR;
  for (int off = LPR / 2; off >= 1; off >>= 1) {
    if (cnt > 1) {
      cnt /= 2;
      last = off;
    }
  }
  return last - 1;
}

}  // namespace mlapi
