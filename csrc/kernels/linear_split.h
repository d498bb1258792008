// Class-split multiclass predict for small serving batches and for f32 models (VERDICT r2 next 3
// and 7): z = X W^T + b -> (first argmax, p_max) with the sklearn epilogue of `kind`.
//
// Why a separate kernel: served multiclass batches average a handful of rows, and the B = 1024
// tiles kernel (gemm_softmax.hip) spends ~9.6 us on them - its 64-class LDS-DMA chunks, double
// buffer and three dependent round trips of the split merge are built for throughput. Here:
//  * grid = (ceil(K / 64) class blocks, ceil(B / 32) row groups); a block = 4 waves, a wave owns
//    16 classes: its W fragments (16 classes x F) are loaded ONCE, straight to registers (no LDS
//    staging: at <= 32 rows every W element is used by at most 2 MFMAs), together with the X
//    fragments of its <= 32 rows - one round trip to L2 / MALL for everything;
//  * MFMA: bf16 -> v_mfma_f32_16x16x32_bf16 (A = 16 classes, B = 16 rows, 8 k per lane);
//    f32 -> v_mfma_f32_16x16x4_f32 with each lane's 16-byte load feeding 4 MFMAs (a consistent
//    permutation of k for A and B: k = 16 j + 4 g + e, g = lane >> 4), accumulators start at the
//    bias (-inf for padding classes, which every reduction maps to "absent");
//  * epilogue in registers: a lane holds 4 classes of one row; 2 xor-shuffles merge the 4 lane
//    groups, the 4 waves merge through 512 B of LDS in fixed order (first max wins: ties go to the
//    lower class index, like numpy's argmax);
//  * split merge with ONE cross-block round trip (round 4: tagged granules): wave 0 of every split
//    but the last stores the block's row states as 16-byte granules tagged with the launch's epoch
//    and exits; the row group's last split polls them, merges in fixed split order and writes
//    (label, p_max) - or the serving completion record. (Round 3: a drained store, a ticket and an
//    acquire in the last arriver.)
//  * XCD-local merge (xcd_local): the grid is 1-D and ordered so that every split of a row group
//    runs on ONE XCD (blocks are dealt round-robin over the 8 XCDs, starting wherever the
//    dispatcher's rotation stood: block b runs on XCD (c + b) % 8, and the splits of row group r
//    are the blocks with b % 8 == r % 8). The granules are then plain stores into that XCD's L2
//    (no write-through to HBM), polled with sc1 loads. Each granule carries the XCD that wrote it
//    (HW_REG_XCC_ID); the merging block checks them and flags a mismatch in the error word.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "mlapi/kernels.h"

namespace mlapi {
namespace split {

typedef __attribute__((ext_vector_type(8))) __bf16 sbf16x8_t;
typedef __attribute__((ext_vector_type(4))) float sf32x4_t;

constexpr int CLASSES_PER_BLOCK = 64;
constexpr int ROWS_PER_GROUP = 32;

struct SplitArgs {
  const void* X;
  int64_t ldx;          // X row stride (elements)
  const void* W;        // [K][F] row stride F, same dtype as X
  const float* bias;    // [K]
  int32_t B, K, kind, nsplit;
  int32_t* out_idx;
  float* out_p;
  RecOut ro;            // serving: per-row completion records instead of out_idx / out_p
  unsigned int* counters;  // start of the workspace (its error word: xcd_err)
  float4* partials;        // [row groups][nsplit][32] state granules {m, s, argmax bits, epoch << 4 | XCD}
  unsigned int* xcd_err;   // xcd_local: bit x set when a merging block on XCD x read a partial written elsewhere
  int32_t xcd_local;        // 1-D XCD-ordered grid + L2-local merge protocol (see the header)
  int32_t xcd_inject;       // test hook (xcd_local_inject): every merged row reports a misplaced partial
  int32_t row_groups;
  int32_t probe;           // measurement only (MLAPI_SPLIT_PROBE): 1 = stop after the block merge, 2 = after the partial stores
  // Host merge (serving, one row group): each block publishes its per-row states as 16-byte
  // completion records {seq, argmax, m, s} into host-mapped memory at hrec[block * 32 + row] and
  // is done - no ticket, no cross-block round trips; the engine's completer merges the splits in
  // split order (csrc/runtime/engine.cpp, collect()).
  uint4* hrec;
  uint32_t rec_seq;
  uint32_t epoch;  // split merge: this launch's granule tag (1 .. 2^28 - 1)
  int32_t clear_tags;  // the merger clears the tags it consumed (set for HIP-graph captures only)
};

struct SState {
  float m, s;
  int bi;
};

__device__ __forceinline__ SState smerge(SState a, SState b, bool ovr) {
  const bool take_b = (b.m > a.m) || (b.m == a.m && b.bi < a.bi);
  SState r;
  r.m = take_b ? b.m : a.m;
  r.bi = take_b ? b.bi : a.bi;
  if (ovr) {
    r.s = a.s + b.s;
  } else {
    const float sa = a.m == -INFINITY ? 0.f : a.s * expf(a.m - r.m);
    const float sb = b.m == -INFINITY ? 0.f : b.s * expf(b.m - r.m);
    r.s = sa + sb;
  }
  return r;
}

__device__ __forceinline__ SState sshfl(SState a, int off) {
  return SState{__shfl_xor(a.m, off, 64), __shfl_xor(a.s, off, 64), __shfl_xor(a.bi, off, 64)};
}

__device__ __forceinline__ float ssigmoid(float z) { return 1.f / (1.f + expf(-z)); }

// T = uint16_t (bf16 bits) or float. KS: 16-byte units per lane per row (bf16: F / 32, f32: F / 16).
// NB: 16-row tiles per wave (1 or 2).
template <typename T, int KS, int NB, bool OVR>
__device__ __forceinline__ void split_predict(const SplitArgs& a) {
  constexpr bool BF = sizeof(T) == 2;
  constexpr int F = BF ? KS * 32 : KS * 16;
  __shared__ float4 red[4][NB * 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  int split = blockIdx.x, rgi = blockIdx.y;
  if (a.xcd_local) {  // b -> XCD b & 7; its j-th block: row group xcd + 8 (j / nsplit), split j % nsplit
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    rgi = xcd + 8 * (j / a.nsplit);
    split = j % a.nsplit;
    if (rgi >= a.row_groups) return;  // uniform per block
  }
  const int c0 = split * CLASSES_PER_BLOCK + wave * 16;
  const int row0 = rgi * ROWS_PER_GROUP;
  // ---- every load of the block up front: W fragments, X fragments, bias
  const int ca = min(c0 + r16, a.K - 1);  // padding classes read a real row (masked by a -inf bias)
  const uint4* wp = reinterpret_cast<const uint4*>(static_cast<const T*>(a.W) + (int64_t)ca * F) + g;
  uint4 af[KS];
#pragma unroll
  for (int j = 0; j < KS; ++j) af[j] = wp[j * 4];
  uint4 xf[NB][KS];
#pragma unroll
  for (int t = 0; t < NB; ++t) {
    const int row = min(row0 + t * 16 + r16, a.B - 1);
    const uint4* xp = reinterpret_cast<const uint4*>(static_cast<const T*>(a.X) + (int64_t)row * a.ldx) + g;
#pragma unroll
    for (int j = 0; j < KS; ++j) xf[t][j] = xp[j * 4];
  }
  sf32x4_t bias;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = c0 + g * 4 + r;
    const float bv = a.bias[min(c, a.K - 1)];
    bias[r] = c < a.K ? bv : -INFINITY;
  }
  // keep every load above in flight together: without this fence the scheduler sinks half of them
  // below the first MFMAs to save registers (two dependent round trips instead of one)
  __builtin_amdgcn_sched_barrier(0);
  // ---- logits
  sf32x4_t acc[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) acc[t] = bias;
#pragma unroll
  for (int j = 0; j < KS; ++j) {
    if constexpr (BF) {
      const sbf16x8_t av = __builtin_bit_cast(sbf16x8_t, af[j]);
#pragma unroll
      for (int t = 0; t < NB; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(sbf16x8_t, xf[t][j]), acc[t], 0, 0, 0);
    } else {
      const uint32_t aw[4] = {af[j].x, af[j].y, af[j].z, af[j].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int t = 0; t < NB; ++t) {
          const uint32_t xw[4] = {xf[t][j].x, xf[t][j].y, xf[t][j].z, xf[t][j].w};
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(aw[e]), __uint_as_float(xw[e]), acc[t], 0, 0,
                                                        0);
        }
      }
    }
  }
  // ---- row states: 4 classes per lane -> 16 per wave (2 shuffles) -> 64 per block (LDS)
#pragma unroll
  for (int t = 0; t < NB; ++t) {
    float m = acc[t][0];
    int br = 0;
#pragma unroll
    for (int r = 1; r < 4; ++r) {
      if (acc[t][r] > m) {
        m = acc[t][r];
        br = r;
      }
    }
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) s += OVR ? ssigmoid(acc[t][r]) : (m == -INFINITY ? 0.f : expf(acc[t][r] - m));
    SState S{m, s, m == -INFINITY ? 0x7fffffff : c0 + g * 4 + br};
    S = smerge(S, sshfl(S, 16), OVR);
    S = smerge(S, sshfl(S, 32), OVR);
    if (g == 0) red[wave][t * 16 + r16] = make_float4(S.m, S.s, __int_as_float(S.bi), 0.f);
  }
  __syncthreads();
  if (wave != 0 || a.probe == 1) return;
  const int l = lane;  // row of the group this lane finishes
  const int64_t row = row0 + l;
  const bool live = l < NB * 16 && row < a.B;
  SState S{-INFINITY, 0.f, 0x7fffffff};
  if (l < NB * 16) {
    const float4 v0 = red[0][l];
    S = SState{v0.x, v0.y, __float_as_int(v0.z)};
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 v = red[w][l];
      S = smerge(S, SState{v.x, v.y, __float_as_int(v.z)}, OVR);
    }
  }
  if (a.hrec != nullptr) {
    if (live) {
      typedef __attribute__((ext_vector_type(4))) uint32_t su32x4_t;
      const su32x4_t r = {a.rec_seq, (uint32_t)S.bi, __float_as_uint(S.m), __float_as_uint(S.s)};
      uint4* dst = a.hrec + (int64_t)split * ROWS_PER_GROUP + l;
      // write-through (sc0 sc1): visible to the host poller without a fence, as one 16-byte unit
      asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(dst), "v"(r) : "memory");
    }
    return;
  }
  int fail = 0;  // 1: misplaced (XCD-local) partial, 2: the poll gave up
  if (a.nsplit > 1) {
    // Tagged granules (cdna_hip_programming.md Guideline 16 R2; the protocol of gemm_softmax.hip):
    // every split but the last stores its rows' states as ONE 16-byte granule {m, s, argmax,
    // epoch << 4 | XCD} and exits - no drain, ticket or fence; the row group's last split (its
    // highest block index in both grid orders: dispatched after its producers) polls them with sc1
    // loads, merges in split order and clears the tags it consumed (graph replays re-use one epoch).
    typedef __attribute__((ext_vector_type(4))) uint32_t su32x4_t;
    typedef __attribute__((address_space(1))) unsigned int gu32_t;
    float4* part = a.partials + ((int64_t)rgi * a.nsplit) * ROWS_PER_GROUP;
    unsigned me = 0;
    if (a.xcd_local) {
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(me));
      me &= 15;
    }
    if (split + 1 < a.nsplit) {
      if (live) {
        const su32x4_t v = {__float_as_uint(S.m), __float_as_uint(S.s), (uint32_t)S.bi, (a.epoch << 4) | me};
        float4* dst = part + (int64_t)split * ROWS_PER_GROUP + l;
        if (a.xcd_local)  // plain store: L1 is write-through, the row group's L2 is the meeting point
          *reinterpret_cast<su32x4_t*>(dst) = v;
        else  // write-through past this XCD's L2
          asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
      }
      return;
    }
    if (a.probe == 2) return;
    // sc1 loads (agent scope: past the CU's L1, which would keep serving a stale line to an sc0 poll)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)part, 0, a.nsplit * ROWS_PER_GROUP * 16, 0x00020000);
    const SState own = S;
    S = SState{-INFINITY, 0.f, 0x7fffffff};
    bool bad = a.xcd_inject != 0, timeout = false;
    const uint64_t t0 = wall_clock64();
    su32x4_t v[16];
    for (int sp0 = 0; sp0 < a.nsplit && !timeout; sp0 += 16) {
      for (;;) {  // 16 granules in flight per pass
        bool ok = true;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (live && sp0 + u + 1 < a.nsplit)
            v[u] = __builtin_bit_cast(su32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rs, (uint32_t)(((sp0 + u) * ROWS_PER_GROUP + l) * 16), 0, 16));
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (live && sp0 + u + 1 < a.nsplit) ok &= (v[u][3] >> 4) == a.epoch;
        if (__all(ok)) break;
        if (wall_clock64() - t0 > 100000000ull) {  // 1 s at 100 MHz: a split never published
          timeout = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");  // the next pass loads again
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {  // fixed split order (deterministic)
        const int sp = sp0 + u;
        if (sp + 1 == a.nsplit) {
          S = smerge(S, own, OVR);
        } else if (sp + 1 < a.nsplit) {
          bad |= a.xcd_local && (v[u][3] & 15u) != me;
          S = smerge(S, SState{__uint_as_float(v[u][0]), __uint_as_float(v[u][1]), (int)v[u][2]}, OVR);
        }
      }
    }
    // graph captures: clear the tags (write-through: no dirty line) - also after a timeout (the
    // rows already fail), so the next replay never reads this replay's granules as its own
    if (a.clear_tags && live)
      for (int sp = 0; sp + 1 < a.nsplit; ++sp)
        __hip_atomic_store((gu32_t*)(part + (int64_t)sp * ROWS_PER_GROUP + l) + 3, 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    bad = live && bad;
    fail = (bad || (timeout && a.xcd_local)) ? 1 : timeout ? 2 : 0;
    if (fail == 1) __hip_atomic_fetch_or(a.xcd_err, 1u << me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!live) return;
  const float p = OVR ? ssigmoid(S.m) / S.s : 1.f / S.s;
  // a misplaced merge never answers: the row comes back as XCD_BAD_IDX / NaN (the engine fails it
  // and switches the XCD-local protocol off); a poll that gave up, WIDE_TIMEOUT_IDX / NaN
  put_result(a.out_idx, a.out_p, a.ro, row, fail == 1 ? XCD_BAD_IDX : fail == 2 ? WIDE_TIMEOUT_IDX : S.bi,
             fail ? __builtin_nanf("") : p);
}

}  // namespace split
}  // namespace mlapi
