// Multiclass (softmax / OvR) logistic-regression predict:  Z = X W^T + b  ->  argmax, p_max
// (BASELINE config 3: B=1024, F=256, K=1000 bf16; reference ops K1+K2+K4+K5).
//
// MFMA layout (v_mfma_f32_16x16x32_bf16, cdna_hip_programming.md S3): the class dimension is the
// MFMA "M" (A operand = W rows) and the batch row is "N" (B operand = X rows), so the C/D tile
// puts ONE batch row on each lane (col = lane & 15) and 4 classes in its registers
// (row = (lane >> 4) * 4 + reg). The softmax reduction over classes is lane-local: each lane keeps
// an online (max, sum-exp, argmax) state over the classes it owns; the 4 lanes sharing a batch
// row merge once at the end (2 xor-shuffles). No LDS is needed for the epilogue.
//
// Data movement (v3):
//  * X: each wave loads its NT x 16 batch rows for the whole F once, straight to registers;
//  * W: 64-class chunks are DMA'd by all 4 waves (global_load_lds_dwordx4) into a double-buffered
//    LDS image [64 classes][F] whose 16-byte chunks are XOR-swizzled by class (chunk ^ (class & 15))
//    on the source side, so the ds_read_b128 fragment reads (16 classes x 16 B at one k-offset per
//    lane group) are conflict-free; chunk c+1 streams in while chunk c computes, one barrier per
//    chunk. Without staging registers a wave can hold 32 rows (NT = 2), halving the LDS fragment
//    reads per MFMA (B=262144: 230 -> 172 us);
//  * small batches (B=1024 -> 16 row blocks) split the class range over gridDim.y so the launch
//    fills the chip; the splits are merged IN THE SAME LAUNCH by the last split's block of each
//    row block, which polls the others' tagged 16-byte state granules (Guideline 16 R2; round 3
//    took a ticket, round 1 ran a separate merge kernel: 7.3 us of a 18.6 us total);
//  * the epilogue is branch-free per element (kind is a template parameter; a split's partial
//    last chunk is masked to -inf) and uses exp2/rcp; accumulators start at the bias.
//
// Training (multinomial / OvR mini-batch SGD, SURVEY 2.3 K6 at BASELINE config 5 scale) reuses the
// same tiles for its row-stats pass (MODE 2): the online (max, sum-exp, argmax) state, merged
// across class splits like MODE 0, is published as {lse = m + log s, argmax} per row; the fused
// gradient kernel (softmax_grad_dw.hip) consumes it. X_aug may carry extra columns (row stride
// ldx >= F; the forward reads only its first F columns).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "mlapi/common.h"
#include "mlapi/kernels.h"
#include "kernels/softmax_rows.h"

namespace mlapi {
namespace {
using namespace rows;

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
constexpr float LN2_F = 0.6931471805599453f;
// The workspace starts with a counter region (its last slot: the XCD-local merge's error bits) and
// the partial-state granules always start after it; granules carry a per-launch tag, so plans of
// different batch sizes can share one zero-initialised workspace.
constexpr int COUNTER_BYTES = 65536;
constexpr int MERGE_MAX = 16;        // split partials the merging block loads at once (automatic plans: <= 16)

// LDS image of a 64-class W chunk: [64 rows][KS * 64 B], filled by LDS-DMA, whose destination is
// lane-linear per wave-instruction: rows are unpadded and the fragment reads' conflict-free
// swizzle (16-B chunk ^ (row & 15); KS = 1: ^ ((row >> 1) & 3)) is applied on the SOURCE address.
// Every width is a power of two (the host pads F; the training X_aug is read with its own row
// stride), for which this layout is conflict-free on the ds_read_b128 lane groups.
template <int KS>
__host__ __device__ constexpr int lds_row_stride() {
  return KS * 64;
}
// Position of 16-byte chunk `ch` of row `r` inside its row (an involution: also maps a row
// position back to the chunk that belongs there).
template <int KS>
__device__ __forceinline__ int lds_pos(int r, int ch) {
  if constexpr (KS == 1) return ch ^ ((r >> 1) & 3);
  return ch ^ (r & (KS * 4 >= 16 ? 15 : KS * 4 - 1));
}
template <int KS>
__device__ __forceinline__ int lds_off(int r, int ch) {
  return r * lds_row_stride<KS>() + (lds_pos<KS>(r, ch) << 4);
}

typedef __attribute__((address_space(1))) const void glob_void_t;

struct GemmArgs {
  const uint16_t* X;
  const uint16_t* W;
  const float* bias;       // [K] f32 (every mode)
  int64_t ldx;             // X row stride in elements (F, or F + 8 for the training X_aug)
  int64_t B;
  int K;
  int kind;
  int classes_per_split;
  int32_t* out_idx;        // MODE 0
  float* out_p;            // MODE 0
  RecOut ro;               // MODE 0 serving: per-row completion records instead of out_idx / out_p
  unsigned int* counters;  // split merge (MODE 0/2)
  float4* partials;        // split merge (MODE 0/2)
  float* Z;                // MODE 1
  float2* rowstat;         // MODE 2 output: {lse, argmax bits}
  float4* rowstate;        // MODE 4 output: {max, sum, argmax bits, 0} (class-sharded TP)
  unsigned long long* stamps;  // profiling (tools/gemm_phase_probe.py): 8 s_memtime slots per wave
  int xcd_local;               // split merge meets in one XCD's L2 (grid.x % 8 == 0; see put_granule)
  int xcd_inject;              // test hook (xcd_local_inject): every merged row reports a misplaced partial
  unsigned epoch;              // split merge: this launch's granule tag (1 .. 2^28 - 1, see put_granule)
  int x_nt;                    // 16x16 kernel, NT = 2: X with the nontemporal hint (MLAPI_GEMM_XNT16=1, measurement)
};

// ---- split-merge protocol (tiles kernels): tagged granules (cdna_hip_programming.md Guideline 16
// R2, "the data is the flag", as in the WIDE kernel). Every class split but the last publishes each
// of its rows' states as ONE 16-byte granule {m, s, argmax, tag = epoch << 4 | XCD} and exits: no
// drain, ticket, barrier or fence on the producers. The last split's block of a row block (the
// highest block index of the row block: dispatched after its producers) polls those granules with
// sc1 loads until every tag carries this launch's epoch, merges them with its own state in
// a fixed order, and clears the tags it consumed, so a HIP-graph replay (same epoch in its baked
// arguments) never reads the previous replay's partials.
// XCD-local (a.xcd_local, chosen by the host when gridDim.x % 8 == 0): hardware blocks are dealt
// round-robin over the 8 XCDs, so block b = y * gridDim.x + x runs on XCD (c + b) % 8 = (c + x) % 8
// - c is wherever the dispatcher's rotation stood when the launch began - and every split of row
// block x runs on ONE XCD: the granules are plain stores into that XCD's L2 (no write-through).
// The poll must not use sc0 loads: those are workgroup scope, the first pass leaves the stale line
// in the CU's L1 and every later pass hits it (measured: every merge timed out, and buffer_inv sc0
// between passes did not help; sc1 loads, or sc0 loads after buffer_inv sc1, saw the plain stores,
// tools/dbg/gemm_merge_dbg.py). The tag's XCD field lets the merger check the placement; a
// misplaced partial (or a poll that never completes, which is what a misplaced plain store looks
// like) answers XCD_BAD_IDX and flags the last counter slot (bit = XCD), and the engine then turns
// the protocol off. Agent scope: sc1 write-through stores; a poll that does not complete within 1 s
// answers WIDE_TIMEOUT_IDX.
constexpr int XCD_ERR_SLOT = COUNTER_BYTES / 4 - 1;
constexpr int MERGE_OK = 0, MERGE_MISPLACED = 1, MERGE_TIMEOUT = 2;

__device__ __forceinline__ unsigned my_xcc() {
  unsigned hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(hw));
  return hw & 15;
}
__device__ __forceinline__ void put_granule(const GemmArgs& a, int64_t idx, const RowState& S) {
  const u32x4_t v{__float_as_uint(S.m), __float_as_uint(S.s), (unsigned)S.bi,
                  (a.epoch << 4) | (a.xcd_local ? my_xcc() : 0u)};
  if (a.xcd_local)
    *reinterpret_cast<u32x4_t*>(a.partials + idx) = v;
  else
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(a.partials + idx), "v"(v) : "memory");
}

// Merging block: called by every lane of a wave. LPR lanes (lane offsets 64 / LPR apart) hold the
// own state `own` of one row; lane qi of them takes splits qi, qi + LPR, ... (the first LPR * SL
// splits' granules loaded together, one poll round trip; forced plans with more splits poll the
// rest one by one). The merged state is the same on the row's LPR lanes; fail: MERGE_*.
template <int LPR, int SL>
__device__ __forceinline__ RowState granule_merge(const GemmArgs& a, int64_t row, int qi, const RowState& own,
                                                  bool live, bool ovr, int& fail) {
  const unsigned ns = gridDim.y;
  const int64_t B = a.B;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.partials, 0, 0x7fffffff, 0x00020000);
  auto ld = [&](unsigned sp) -> u32x4_t {
    return __builtin_bit_cast(u32x4_t,
                              __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(((int64_t)sp * B + row) * 16), 0, 16));
  };
  const uint64_t t0 = wall_clock64();
  bool timeout = false;
  u32x4_t g[SL];
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int u = 0; u < SL; ++u) {
      const unsigned sp = qi + LPR * u;
      if (live && sp + 1 < ns) g[u] = ld(sp);
    }
#pragma unroll
    for (int u = 0; u < SL; ++u) {
      const unsigned sp = qi + LPR * u;
      if (live && sp + 1 < ns) ok &= (g[u][3] >> 4) == a.epoch;
    }
    if (__all(ok)) break;
    if (wall_clock64() - t0 > 100000000ull) {  // 1 s at 100 MHz: a producer never published
      timeout = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");  // the next pass loads again
  }
  const unsigned me = a.xcd_local ? my_xcc() : 0u;
  bool bad = a.xcd_inject != 0;
  RowState S{-INFINITY, 0.f, 0x7fffffff};  // identity of merge_state (exact)
  auto take = [&](unsigned sp, const u32x4_t& v) {
    if (sp + 1 == ns) {
      S = merge_state(S, own, ovr);
      return;
    }
    bad |= a.xcd_local && (v[3] & 15u) != me;
    S = merge_state(S, RowState{__uint_as_float(v[0]), __uint_as_float(v[1]), (int)v[2]}, ovr);
  };
#pragma unroll
  for (int u = 0; u < SL; ++u) {
    const unsigned sp = qi + LPR * u;
    if (sp < ns) take(sp, g[u]);
  }
  for (unsigned sp = qi + LPR * SL; sp < ns; sp += LPR) {  // forced plans beyond MERGE_MAX splits
    u32x4_t v{0u, 0u, 0u, 0u};
    if (sp + 1 < ns && live && !timeout) {
      for (;;) {
        v = ld(sp);
        if ((v[3] >> 4) == a.epoch) break;
        if (wall_clock64() - t0 > 100000000ull) {
          timeout = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
      }
    }
    take(sp, v);
  }
  // consumed: clear the tags. Plain stores: this kernel is only launched on HIP streams, whose
  // system-scope release at kernel end writes dirty L2 lines back before the next launch (the
  // direct-dispatched serving kernels, which may run without that release, clear write-through).
  // Measured: B = 1024 5.72 vs 5.82 us, B = 8192 9.8 vs 10.0 us with write-through clears
  // (profiles/r4_gemm_merge/s34/).
  // also after a timeout (the row already fails): no granule of this launch outlives it
  if (live) {
    unsigned* const base = reinterpret_cast<unsigned*>(a.partials);
    for (unsigned sp = qi; sp + 1 < ns; sp += LPR) base[((int64_t)sp * B + row) * 4 + 3] = 0u;
  }
  int f = timeout ? 2 : bad ? 1 : 0;
#pragma unroll
  for (int off = 64 / LPR; off < 64; off <<= 1) {
    S = merge_state(S, shfl_state(S, off), ovr);  // commutative: every lane of the row ends identical
    f |= __shfl_xor(f, off, 64);
  }
  fail = f == 0 ? MERGE_OK : (a.xcd_local || (f & 1)) ? MERGE_MISPLACED : MERGE_TIMEOUT;
  if (fail == MERGE_MISPLACED && live && qi == 0)
    __hip_atomic_fetch_or(a.counters + XCD_ERR_SLOT, 1u << me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return S;
}

// a merged row's output; a failed merge answers XCD_BAD_IDX / WIDE_TIMEOUT_IDX with p NaN (MODE 0) or
// NaN statistics (MODE 2 / 4: the loss turns NaN instead of training on a stale state)
template <int MODE>
__device__ __forceinline__ void finish_merged(const GemmArgs& a, int64_t row, const RowState& S, int fail, bool ovr) {
  const float nan = __builtin_nanf("");
  if constexpr (MODE == 0) {
    if (fail != MERGE_OK)
      put_result(a.out_idx, a.out_p, a.ro, row, fail == MERGE_MISPLACED ? XCD_BAD_IDX : WIDE_TIMEOUT_IDX, nan);
    else
      put_result(a.out_idx, a.out_p, a.ro, row, S.bi, ovr ? sigmoidf_(S.m) / S.s : 1.f / S.s);
  } else if constexpr (MODE == 4) {
    a.rowstate[row] = fail != MERGE_OK ? make_float4(nan, nan, __int_as_float(S.bi), 0.f)
                                       : make_float4(S.m, S.s, __int_as_float(S.bi), 0.f);
  } else {
    a.rowstat[row] = make_float2(fail != MERGE_OK ? nan : S.m + __logf(S.s), __int_as_float(S.bi));
  }
}

// Phase stamps of one wave (profiled launches only: a.stamps is null otherwise): 0 entry, 1 first
// W chunk + X landed, 2 class loop done, 3 row state reduced; slot 4: cycles the class loop spent
// in its per-chunk wait + barrier (32x32 kernel).
__device__ __forceinline__ void phase_put(const GemmArgs& a, int waves_per_block, int wave, int lane, int j,
                                          unsigned long long v) {
  if (a.stamps != nullptr && lane == 0) {
    const unsigned long long gid =
        ((unsigned long long)blockIdx.y * gridDim.x + blockIdx.x) * (unsigned)waves_per_block + (unsigned)wave;
    a.stamps[gid * 8 + j] = v;
  }
}
__device__ __forceinline__ void phase_stamp(const GemmArgs& a, int waves_per_block, int wave, int lane, int j) {
  if (a.stamps != nullptr) phase_put(a, waves_per_block, wave, lane, j, __builtin_amdgcn_s_memtime());
}

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Lane state of the tiles kernel (v5): running max / sum and, instead of a running argmax, the 16
// logits of the chunk that last raised the max plus that chunk's first class. The first index
// holding the max is resolved ONCE, after the class loop (tile_result). Per chunk that costs 16
// bit-blends (one v_bitop3 each, no VCC) where v4's in-loop argmax paid 16 compare/select pairs,
// each pair separated by a VCC hazard pad (hipcc rebuilt the min tree as a serial chain).
struct TileState {
  float m, s;
  int bc;         // first class of the chunk held in bv (0x7fffffff: none yet)
  unsigned bv[16];  // that chunk's logits (float bits), element i = class bc + (i>>2)*16 + q*4 + (i&3)
};

__device__ __forceinline__ float vmax(float a, float b) { return __builtin_elementwise_maximum(a, b); }

struct TileTmp {
  float m_new, part;
};

__device__ __forceinline__ void tile_init(TileState& S) {
  S.m = -INFINITY;
  S.s = 0.f;
  S.bc = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < 16; ++i) S.bv[i] = __float_as_uint(-INFINITY);
}

template <bool OVR>
__device__ __forceinline__ void tile_stage(int stage, const float (&v)[16], int c0, TileState& S, TileTmp& T) {
  if (stage == 0) {  // chunk max, new running max, keep this chunk's logits if it raised the max
    // IEEE-2019 maximum (NaN-propagating) maps to v_maximum3_f32 with no operand quieting; fmaxf
    // (maxnum) made hipcc canonicalize every MFMA result first (one extra v_max per element).
    float cm = vmax(v[0], v[1]);
#pragma unroll
    for (int i = 2; i < 16; ++i) cm = vmax(cm, v[i]);
    // strict: an earlier chunk keeps a tie (first max wins). The blend goes through an opaque
    // mask: as selects, hipcc sank them under an exec branch splitting the pipelined block.
    unsigned mask = -(unsigned)(cm > S.m);
    asm("" : "+v"(mask));
    T.m_new = vmax(cm, S.m);
#pragma unroll
    for (int i = 0; i < 16; ++i) S.bv[i] = S.bv[i] ^ ((S.bv[i] ^ __float_as_uint(v[i])) & mask);
    S.bc = (int)((unsigned)S.bc ^ (((unsigned)S.bc ^ (unsigned)c0) & mask));
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
__device__ __forceinline__ void tile_finish(const TileTmp& T, TileState& S) {
  if constexpr (OVR) {
    S.s += T.part;
  } else {
    // rescale the running sum to the new max (S.m = -inf: exp2(-inf) = 0); unconditional, a
    // select here became a branch around the exp2
    const float scale = __builtin_amdgcn_exp2f(fmaf(S.m, LOG2E_F, -T.m_new * LOG2E_F));
    S.s = fmaf(S.s, scale, T.part);
  }
  S.m = T.m_new;
}

template <bool OVR>
__device__ __forceinline__ void tile_update(const float (&v)[16], int c0, TileState& S) {
  TileTmp T;
  tile_stage<OVR>(0, v, c0, S, T);
  tile_stage<OVR>(1, v, c0, S, T);
  tile_stage<OVR>(2, v, c0, S, T);
  tile_finish<OVR>(T, S);
}

// (max, sum, first argmax) of a lane: the first element of the kept chunk equal to the max
__device__ __forceinline__ RowState tile_result(const TileState& S, int q) {
  int ci = 16;
#pragma unroll
  for (int i = 15; i >= 0; --i) ci = __uint_as_float(S.bv[i]) == S.m ? i : ci;
  const int bi = (S.m == -INFINITY || ci == 16) ? 0x7fffffff : S.bc + (ci >> 2) * 16 + q * 4 + (ci & 3);
  return RowState{S.m, S.s, bi};
}

// Logits of one 64-class chunk against the LDS image `wb`: MFMAs into bias-initialised
// accumulators (the bias was DMA'd into LDS next to the W chunk, so no global load sits between
// the staging pipeline's counted waits). Classes >= c_end (only the very last chunk of the
// problem) get a -inf bias, which every reduction of the epilogue maps to "absent" (exp2 -> 0,
// sigmoid -> 0, never the max): the epilogue then needs no per-element class check.
template <int KS, int NT>
__device__ __forceinline__ void mfma_chunk(const unsigned char* wb, const bf16x8_t (&xf)[NT][KS], int c0, int c_end,
                                           int q, int col, const float* bias_lds, f32x4_t (&acc)[NT][4]) {
  f32x4_t b4[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) b4[mt] = *reinterpret_cast<const f32x4_t*>(bias_lds + mt * 16 + q * 4);
  if (c0 + CLASS_CHUNK > c_end) {  // wave-uniform: the last chunk only
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) b4[mt][r] = c0 + mt * 16 + q * 4 + r < c_end ? b4[mt][r] : -INFINITY;
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t][mt] = b4[mt];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8_t wf[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      wf[mt] = *reinterpret_cast<const bf16x8_t*>(wb + lds_off<KS>(mt * 16 + col, 4 * ks + q));
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[mt], xf[t][ks], acc[t][mt], 0, 0, 0);
  }
}

// One pipelined step (MODE 0 / 2 / 4): the MFMAs of the next chunk (nb -> nxt) with the epilogue
// of the current one (acc -> st) spread over its k-steps: after the MFMAs of k-step k come the
// epilogue stages scheduled there, and a sched_barrier that lets only LDS reads cross keeps the
// interleave (the scheduler otherwise hoists all 64 MFMAs and leaves the VALU work exposed).
template <int KS, int NT, bool OVR>
__device__ __forceinline__ void fused_step(const unsigned char* nb, const bf16x8_t (&xf)[NT][KS], int cn, int c_end,
                                           int q, int col, f32x4_t (&nxt)[NT][4], const f32x4_t (&acc)[NT][4], int c0,
                                           TileState (&st)[NT]) {
  const float* bias_lds = reinterpret_cast<const float*>(nb + CLASS_CHUNK * lds_row_stride<KS>());
  f32x4_t b4[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) b4[mt] = *reinterpret_cast<const f32x4_t*>(bias_lds + mt * 16 + q * 4);
  if (cn + CLASS_CHUNK > c_end) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) b4[mt][r] = cn + mt * 16 + q * 4 + r < c_end ? b4[mt][r] : -INFINITY;
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) nxt[t][mt] = b4[mt];
  float v[NT][16];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) v[t][i] = acc[t][i >> 2][i & 3];
  TileTmp T[NT];
  constexpr int NSTAGE = 3 * NT + NT;  // 3 stages + finish per row tile
  static_for<KS>([&](auto kc) {
    constexpr int ks = decltype(kc)::value;
    bf16x8_t wf[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
      wf[mt] = *reinterpret_cast<const bf16x8_t*>(nb + lds_off<KS>(mt * 16 + col, 4 * ks + q));
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        nxt[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[mt], xf[t][ks], nxt[t][mt], 0, 0, 0);
    // epilogue stages j with slot(j) == ks, slot(j) = j * KS / NSTAGE (every stage placed once)
    static_for<NSTAGE>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr ((j * KS) / NSTAGE == ks) {
        constexpr int t = j / 4, stg = j % 4;
        if constexpr (stg < 3)
          tile_stage<OVR>(stg, v[t], c0, st[t], T[t]);
        else
          tile_finish<OVR>(T[t], st[t]);
      }
    });
    if constexpr (KS >= 4) __builtin_amdgcn_sched_barrier(0x100);  // only LDS reads may cross
  });
}

// Epilogue of one chunk's logits: lane owns classes c0 + mt*16 + q*4 + r (i = mt*4 + r, increasing
// class order) of batch row (t, col). Branch-free per element (a runtime kind or bound check here
// made hipcc emit exec-mask branches around every element: SQ_INSTS_VALU 5.4k per wave).
template <int NT, int MODE, bool OVR>
__device__ __forceinline__ void epilogue_chunk(const f32x4_t (&acc)[NT][4], int c0, int c_end, int q, int col,
                                               int64_t row0, int64_t B, int K, const GemmArgs& a,
                                               TileState (&st)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = acc[t][i >> 2][i & 3];
    if constexpr (MODE == 1) {
      const int64_t row = row0 + t * 16 + col;
      if (row < B) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int cls = c0 + (i >> 2) * 16 + q * 4 + (i & 3);
          if (cls < c_end) a.Z[row * K + cls] = v[i];
        }
      }
    } else {  // MODE 0 / 2 / 4: online (max, sum, first argmax)
      tile_update<OVR>(v, c0, st[t]);
    }
  }
}

// KS = F/32 (exact), NT = 16-row N-tiles per wave, MODE: 0 = fused predict epilogue,
// 1 = write logits, 2 = training row stats (see header), 4 = raw online softmax state per row
// (class-sharded TP, merged across ranks by shard.hip).
// Two waves per SIMD (2 blocks of 4 waves per CU, LDS 2 x 66 KB): the register budget is 256.
// v5's kept-chunk logits (16 VGPRs per row tile) put NT = 2 at 261 without the cap; with it
// 4 VGPRs spill around (not inside) the class loop. F = 512 runs one block per CU anyway (its
// double-buffered W chunks take 2 x 66 KB of LDS), so it keeps the whole register file.
template <int KS, int MODE>
constexpr int tiles_waves_per_eu() {
  return KS == 16 ? 1 : 2;
}
// Waves per block: 4 (two blocks per CU). 8-wave blocks (256 rows, one block per CU, a third W
// buffer) halve W's L2 -> CU traffic but measured slower at B = 262144 (170 vs 145 us,
// profiles/r2_gemm/phase_probe.log): one barrier then stalls all 8 waves of the CU.
template <int KS, int NT>
constexpr int tiles_block_waves() {
  return 4;
}

template <int KS, int NT, int MODE, bool OVR>
__global__ __launch_bounds__((64 * tiles_block_waves<KS, NT>())) __attribute__((amdgpu_waves_per_eu(tiles_waves_per_eu<KS, MODE>(),
                                                                     tiles_waves_per_eu<KS, MODE>()))) void
gemm_softmax_kernel(GemmArgs a) {
  const uint16_t* __restrict__ X = a.X;
  const uint16_t* __restrict__ W = a.W;
  const float* __restrict__ bias = a.bias;
  const int64_t B = a.B;
  const int K = a.K;
  const int kind = a.kind;
  const int classes_per_split = a.classes_per_split;
  // Everything below is compile-time shaped: F == KS * 32 exactly (the wrapper pads other F).
  // No runtime guard may sit on a load: hipcc then branches around each load and waits vmcnt(0)
  // per element, serializing the W stream (seen in the v2 ISA; cdna_hip_programming.md S5 trap c).
  constexpr int ROWS_PER_WAVE = 16 * NT;
  constexpr int WV = tiles_block_waves<KS, NT>();
  constexpr int NTHR = 64 * WV;
  constexpr int ROWS_PER_BLOCK = WV * ROWS_PER_WAVE;
  if ((int64_t)blockIdx.x * ROWS_PER_BLOCK >= a.B) return;  // XCD-padded grid (uniform per block)
  constexpr int F_ = KS * 32;
  constexpr int NCH = F_ / 8;                          // 16-byte chunks per W row
  constexpr int W_BYTES = CLASS_CHUNK * lds_row_stride<KS>();
  constexpr int BUF_BYTES = W_BYTES + CLASS_CHUNK * 4;  // [W chunk][64 f32 bias]
  constexpr int PIECES = CLASS_CHUNK * NCH / NTHR;     // 16-byte pieces per thread per chunk
  // W chunk buffers: 8-wave blocks (one per CU) have the LDS for a third, which gives every DMA
  // two iterations to land instead of one; logits mode (stores in the loop) keeps two.
  constexpr int NBUF = (WV == 8 && MODE != 1) ? 3 : 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NBUF * BUF_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int q = lane >> 4;
  const int col = lane & 15;
  constexpr bool ovr = OVR;
  (void)kind;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS_PER_BLOCK + wave * ROWS_PER_WAVE;
  phase_stamp(a, WV, wave, lane, 0);
  const int c_begin = blockIdx.y * classes_per_split;
  const int c_end = min(K, c_begin + classes_per_split);
  const int c_last = c_begin + ((c_end - 1 - c_begin) / CLASS_CHUNK) * CLASS_CHUNK;  // last chunk start

  bf16x8_t xf[NT][KS];

  // ---- W chunk staging: global -> registers (issue early) -> LDS (write late). Plain unrolled
  // code with ext_vector registers: a lambda capture or HIP_vector_type array goes to scratch.
  // W staging: chunk c + 1 is DMA'd into the idle buffer while chunk c computes (no staging
  // VGPRs, no ds_write pass); the barrier's vmcnt(0) retires it. On the last chunk the (valid)
  // last chunk address is re-loaded instead of branching around the loads.
  // Lane-linear destination: 16-B position P = i*NTHR + wave*64 + lane holds row P / NCH, in-row
  // position P % NCH, i.e. source chunk lds_pos(row, P % NCH).
  // buffer_load ... lds through range-checked descriptors: the per-thread source offsets are
  // chunk-invariant (hoisted out of the loop by the compiler; a local offset array here made
  // hipcc's host pass drop every device stub of this kernel), the chunk base is a scalar offset, and classes past K read
  // as zeros (masked in the epilogue) instead of being clamped per piece - v3 recomputed a clamped
  // 64-bit address per piece and chunk (~90 VALU per chunk).
  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, K * F_ * 2, 0x00020000);
  const auto brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)bias, 0, K * 4, 0x00020000);
#define MLAPI_DMA_CHUNK(C0, BUF)                                                                          \
  {                                                                                                        \
  _Pragma("unroll") for (int i = 0; i < PIECES; ++i)                                                       \
    __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                              \
        wrsrc, (lds_void_t*)(smem + (BUF) * BUF_BYTES + (i * NTHR + wave * 64) * 16), 16, (uint32_t)((((tid + i * NTHR) / NCH) * F_ + lds_pos<KS>((tid + i * NTHR) / NCH, (tid + i * NTHR) % NCH) * 8) * 2),         \
        (C0) * F_ * 2, 0, 0);                                                                              \
  /* bias: 64 floats per chunk, every wave DMAs the same 256 B (one more VM op per wave: uniform count) */ \
  __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void_t*)(smem + (BUF) * BUF_BYTES + W_BYTES), 4,   \
                                           (uint32_t)lane * 4, (C0) * 4, 0, 0);                           \
  }

  TileState ts[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) tile_init(ts[t]);

  // Raw s_barrier, not __syncthreads(): the latter's fence waits vmcnt(0) and would drain the
  // in-flight DMA (cdna_hip_programming.md "Pipelining across barriers"); the empty asm statements
  // keep the compiler from moving LDS accesses across it.
#define MLAPI_RAW_BARRIER()          \
  asm volatile("" ::: "memory");     \
  __builtin_amdgcn_s_barrier();      \
  asm volatile("" ::: "memory");
  MLAPI_DMA_CHUNK(c_begin, 0)
  // X fragments for the whole feature range, straight to registers, in flight with chunk 0
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int64_t r = row0 + t * 16 + col;
    r = r < B ? r : B - 1;
    const uint16_t* xr = X + r * a.ldx + 8 * q;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      // Plain loads, as in the 32x32 kernel (where dropping the nontemporal hint took 147.7 ->
      // 137.3 us); here neutral: F = 512, B = 262,144 514-517 vs 514-523 us with the hint
      // (MLAPI_GEMM_XNT16=1, profiles/r6_gemm/xnt16/)
      if (NT == 2 && a.x_nt)
        xf[t][ks] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(xr + ks * 32));
      else
        xf[t][ks] = *reinterpret_cast<const bf16x8_t*>(xr + ks * 32);
    }
  }
  // (the builtin form of s_waitcnt is visible to the compiler's wait insertion; encoding:
  // vmcnt[3:0,15:14], expcnt[6:4], lgkmcnt[11:8] with the other two counters left at "no wait")
  constexpr int kWaitAll = (7 << 4) | (15 << 8);
  constexpr int kWaitChunk = kWaitAll | ((PIECES + 1) & 15) | (((PIECES + 1) >> 4) << 14);  // one chunk may fly
  // Software pipeline over class chunks (v4): iteration c issues the MFMAs of chunk c+1 and the
  // epilogue of chunk c in ONE basic block, so the epilogue's VALU work (max / exp2 / sums, ~250
  // instructions a chunk) issues in the MFMA shadow instead of after it, and no VALU reads an
  // accumulator right behind its MFMA (v3: 50 s_nop hazard pads per chunk). One barrier per chunk:
  // at the top of iteration c every wave has finished reading the buffer of chunk c (last
  // iteration's MFMAs), so the DMA of chunk c+2 goes there and has a whole iteration to land.
  if constexpr (NBUF == 3) {
    if (c_begin + CLASS_CHUNK < c_end) {  // chunk 1 flies on while chunk 0 computes
      MLAPI_DMA_CHUNK(c_begin + CLASS_CHUNK, 1)
      __builtin_amdgcn_s_waitcnt(kWaitChunk);  // chunk 0 + X
    } else {
      __builtin_amdgcn_s_waitcnt(kWaitAll);
    }
  } else {
    __builtin_amdgcn_s_waitcnt(kWaitAll);  // chunk 0 + X
  }
  MLAPI_RAW_BARRIER()
  phase_stamp(a, WV, wave, lane, 1);
  if (c_begin + (NBUF - 1) * CLASS_CHUNK < c_end) MLAPI_DMA_CHUNK(c_begin + (NBUF - 1) * CLASS_CHUNK, NBUF - 1)
  f32x4_t acc[NT][4];
  mfma_chunk<KS, NT>(smem, xf, c_begin, c_end, q, col, reinterpret_cast<const float*>(smem + W_BYTES), acc);
  int buf = 0;  // buffer of chunk c0
  for (int c0 = c_begin;; c0 += CLASS_CHUNK) {
    if (c0 + CLASS_CHUNK >= c_end) {
      epilogue_chunk<NT, MODE, OVR>(acc, c0, c_end, q, col, row0, B, K, a, ts);
      break;
    }
    // chunk c+1 landed: with 3 buffers chunk c+2 (if issued) may stay in flight
    if (NBUF == 3 && c0 + 2 * CLASS_CHUNK < c_end)
      __builtin_amdgcn_s_waitcnt(kWaitChunk);
    else
      __builtin_amdgcn_s_waitcnt(kWaitAll);
    MLAPI_RAW_BARRIER()  // ... for every wave; and everyone is done with chunk c's buffer
    if (c0 + NBUF * CLASS_CHUNK < c_end) MLAPI_DMA_CHUNK(c0 + NBUF * CLASS_CHUNK, buf)
    const int nbuf = buf + 1 == NBUF ? 0 : buf + 1;
    const unsigned char* nb = smem + nbuf * BUF_BYTES;
    f32x4_t nxt[NT][4];
    if constexpr (MODE == 1) {
      mfma_chunk<KS, NT>(nb, xf, c0 + CLASS_CHUNK, c_end, q, col, reinterpret_cast<const float*>(nb + W_BYTES), nxt);
      epilogue_chunk<NT, MODE, OVR>(acc, c0, c_end, q, col, row0, B, K, a, ts);
    } else {
      fused_step<KS, NT, OVR>(nb, xf, c0 + CLASS_CHUNK, c_end, q, col, nxt, acc, c0, ts);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[t][mt] = nxt[t][mt];
    buf = nbuf;
  }
#undef MLAPI_RAW_BARRIER
#undef MLAPI_DMA_CHUNK
  phase_stamp(a, WV, wave, lane, 2);
  if constexpr (MODE == 0 || MODE == 2 || MODE == 4) {
    RowState st[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      RowState S = tile_result(ts[t], q);
      S = merge_state(S, shfl_state(S, 16), ovr);
      S = merge_state(S, shfl_state(S, 32), ovr);
      st[t] = S;
    }
    phase_stamp(a, WV, wave, lane, 3);
    if (gridDim.y == 1) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int64_t row = row0 + t * 16 + col;
        if (q == 0 && row < B) {
          if constexpr (MODE == 0) {
            put_result(a.out_idx, a.out_p, a.ro, row, st[t].bi, ovr ? sigmoidf_(st[t].m) / st[t].s : 1.f / st[t].s);
          } else if constexpr (MODE == 4) {
            a.rowstate[row] = make_float4(st[t].m, st[t].s, __int_as_float(st[t].bi), 0.f);
          } else {
            a.rowstat[row] = make_float2(st[t].m + __logf(st[t].s), __int_as_float(st[t].bi));
          }
        }
      }
      return;
    }
    // ---- split classes: tagged-granule merge (put_granule / granule_merge)
    if (blockIdx.y + 1 < gridDim.y) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int64_t row = row0 + t * 16 + col;
        if (q == 0 && row < B) put_granule(a, (int64_t)blockIdx.y * B + row, st[t]);
      }
      return;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int64_t row = row0 + t * 16 + col;
      int fail;
      const RowState S = granule_merge<4, 4>(a, row, q, st[t], row < B, ovr, fail);
      if (q == 0 && row < B) finish_merged<MODE>(a, row, S, fail, ovr);
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Large-batch tiles kernel (v6): v_mfma_f32_32x32x16_bf16. One 32-row N tile per wave; a 64-class
// chunk is two 32-class M tiles x F/16 k-steps = 2F/16 MFMAs of 32 cycles (the 16x16x32 NT=2
// kernel issues twice as many of half the length for the same work). Each 32-cycle MFMA gap
// hides ~5 VALU fillers where a 16-cycle gap hides ~2 (MI355X_MICROARCH.md constants table), so
// the softmax epilogue of the previous chunk fits the MFMA shadow; a lane's 16 accumulators of a
// tile all belong to ONE batch row (col = lane & 31; class 8*(i>>2) + 4*(lane>>5) + (i&3)), so the
// row state is one TileState per lane (v5's NT = 2 kept two) and the 2 lanes of a row merge with
// one shuffle. Same LDS image, DMA and split merge as the 16x16 kernel; F in {64, 128, 256}.
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

__device__ __forceinline__ RowState tile_result32(const TileState& S, int h) {
  int ci = 16;
#pragma unroll
  for (int i = 15; i >= 0; --i) ci = __uint_as_float(S.bv[i]) == S.m ? i : ci;
  const int bi = (S.m == -INFINITY || ci == 16) ? 0x7fffffff : S.bc + (ci >> 2) * 8 + h * 4 + (ci & 3);
  return RowState{S.m, S.s, bi};
}

// Finer epilogue stages for the 32x32 kernel (7 per tile, ~10-16 VALU each) so the scheduler can
// spread a tile's update across the MFMA gaps of many k-steps:
//   0: chunk max + new running max + take mask   1/2: keep-chunk blends of elements 0-7 / 8-15
//   3..6: exp (sigmoid) terms of elements 4(s-3)..+3; stage 6 also rescales the sum and commits m
struct TileTmp7 {
  float m_new, m2, part;
  unsigned mask;
};

template <bool OVR>
__device__ __forceinline__ void tile_stage7(int stage, const float (&v)[16], int c0, TileState& S, TileTmp7& T) {
  if (stage == 0) {
    float cm = vmax(v[0], v[1]);
#pragma unroll
    for (int i = 2; i < 16; ++i) cm = vmax(cm, v[i]);
    unsigned mask = -(unsigned)(cm > S.m);  // strict: an earlier chunk keeps a tie
    asm("" : "+v"(mask));
    T.mask = mask;
    T.m_new = vmax(cm, S.m);
    T.m2 = T.m_new * LOG2E_F;
    T.part = 0.f;
  } else if (stage <= 2) {
    const int i0 = stage == 1 ? 0 : 8;
#pragma unroll
    for (int i = i0; i < i0 + 8; ++i) S.bv[i] = S.bv[i] ^ ((S.bv[i] ^ __float_as_uint(v[i])) & T.mask);
    if (stage == 2) S.bc = (int)((unsigned)S.bc ^ (((unsigned)S.bc ^ (unsigned)c0) & T.mask));
  } else {
    const int i0 = (stage - 3) * 4;
    float e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (OVR)
        e[i] = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-v[i0 + i] * LOG2E_F));
      else
        e[i] = __builtin_amdgcn_exp2f(fmaf(v[i0 + i], LOG2E_F, -T.m2));
    }
    T.part += (e[0] + e[1]) + (e[2] + e[3]);
    if (stage == 6) {
      if constexpr (OVR) {
        S.s += T.part;
      } else {
        const float scale = __builtin_amdgcn_exp2f(fmaf(S.m, LOG2E_F, -T.m2));
        S.s = fmaf(S.s, scale, T.part);
      }
      S.m = T.m_new;
    }
  }
}

// bias of the two 32-class tiles of chunk c0 in accumulator layout; classes >= c_end -> -inf
__device__ __forceinline__ void bias32(const float* bias_lds, int c0, int c_end, int h, f32x16_t (&bt)[2]) {
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(bias_lds + ct * 32 + 8 * j + 4 * h);
#pragma unroll
      for (int r = 0; r < 4; ++r) bt[ct][4 * j + r] = v[r];
    }
  if (c0 + CLASS_CHUNK > c_end) {  // wave-uniform: the last chunk only
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        bt[ct][i] = c0 + ct * 32 + 8 * (i >> 2) + 4 * h + (i & 3) < c_end ? bt[ct][i] : -INFINITY;
  }
}

template <int KS, int RT>
__device__ __forceinline__ void mfma32_chunk(const unsigned char* wb, const bf16x8_t (&xf)[RT][2 * KS], int c0,
                                             int c_end, int h, int col, f32x16_t (&acc)[RT][2]) {
  f32x16_t bt[2];
  bias32(reinterpret_cast<const float*>(wb + CLASS_CHUNK * lds_row_stride<KS>()), c0, c_end, h, bt);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    acc[rt][0] = bt[0];
    acc[rt][1] = bt[1];
  }
#pragma unroll
  for (int k = 0; k < 2 * KS; ++k) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const bf16x8_t wf = *reinterpret_cast<const bf16x8_t*>(wb + lds_off<KS>(ct * 32 + col, 2 * k + h));
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf[rt][k], acc[rt][ct], 0, 0, 0);
    }
  }
}

// Per-lane LDS byte offsets of the W fragments of one k-step period: the XOR swizzle repeats every
// P = (mask + 1) / 2 k-steps (8 at F >= 128), so fragment (ct, k) sits at off[k % P] + ct * 32 rows
// + (k / P) * 256 B, and with the buffer index a template constant every read is
// `ds_read_b128 v, off offset:IMM` (v5 recomputed ~30 address VALU per chunk).
template <int KS>
constexpr int t32_period() {
  return KS * 4 >= 16 ? 8 : KS * 2;
}
template <int KS>
struct FragOff {
  uint32_t o[t32_period<KS>()];
};
template <int KS>
__device__ __forceinline__ FragOff<KS> frag_offsets(int h, int col) {
  FragOff<KS> f;
#pragma unroll
  for (int j = 0; j < t32_period<KS>(); ++j) f.o[j] = (uint32_t)lds_off<KS>(col, 2 * j + h);
  return f;
}
template <int KS, int BUF, int BUF_BYTES>
__device__ __forceinline__ bf16x8_t frag32(const unsigned char* smem, const FragOff<KS>& f, int ct, int k) {
  constexpr int P = t32_period<KS>();
  return *reinterpret_cast<const bf16x8_t*>(smem + BUF * BUF_BYTES + f.o[k % P] + ct * 32 * lds_row_stride<KS>() +
                                            (k / P) * (P * 2 * 16));
}

// MFMAs of chunk cn (LDS buffer BUF -> nxt) with the epilogue of chunk c0 (acc -> S) spread over
// the k-steps
template <int KS, int RT, bool OVR, int BUF, int BUF_BYTES, bool EPI = true, int AHEAD = 2, bool PRIO = false>
__device__ __forceinline__ void fused32_step(const unsigned char* smem, const FragOff<KS>& fo,
                                             const bf16x8_t (&xf)[RT][2 * KS], int cn, int c_end, int h,
                                             f32x16_t (&nxt)[RT][2], const f32x16_t (&acc)[RT][2], int c0,
                                             TileState (&S)[RT]) {
  f32x16_t bt[2];
  bias32(reinterpret_cast<const float*>(smem + BUF * BUF_BYTES + CLASS_CHUNK * lds_row_stride<KS>()), cn, c_end, h,
         bt);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    nxt[rt][0] = bt[0];
    nxt[rt][1] = bt[1];
  }
  float v[RT][2][16];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int i = 0; i < 16; ++i) v[rt][ct][i] = acc[rt][ct][i];
  TileTmp7 T[RT][2];
  constexpr int K2 = 2 * KS;
  constexpr int NSTAGE = 14 * RT;  // 7 per class tile; class tile 1 follows tile 0 (same row state)
  // W fragments one k-step ahead in registers: the reads of step k+1 issue before the MFMAs of
  // step k (a 64-cycle MFMA pair of cover for the LDS latency); the scheduling barriers pin them
  // there (left free, hipcc sank every read next to its MFMA).
  // W fragments AHEAD k-steps in flight ahead of their MFMAs
  bf16x8_t wf[AHEAD + 1][2];
  static_for<AHEAD>([&](auto pc) {
    constexpr int k0 = decltype(pc)::value;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) wf[k0][ct] = frag32<KS, BUF, BUF_BYTES>(smem, fo, ct, k0);
  });
  static_for<K2>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if constexpr (k + AHEAD < K2) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
        wf[(k + AHEAD) % (AHEAD + 1)][ct] = frag32<KS, BUF, BUF_BYTES>(smem, fo, ct, k + AHEAD);
    }
    __builtin_amdgcn_sched_barrier(0);
    // PRIO (measurement variant): the wave issuing its MFMAs outranks the SIMD's other wave, whose
    // epilogue VALU then fills the gaps instead of delaying the next MFMA issue
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        nxt[rt][ct] =
            __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k % (AHEAD + 1)][ct], xf[rt][k], nxt[rt][ct], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    static_for<NSTAGE>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr ((j * K2) / NSTAGE == k) {
        constexpr int rt = j / 14, t = (j % 14) / 7, stg = j % 7;
        if constexpr (EPI) tile_stage7<OVR>(stg, v[rt][t], c0 + 32 * t, S[rt], T[rt][t]);
      }
    });
    __builtin_amdgcn_sched_barrier(0);
  });
}

template <bool OVR, int RT>
__device__ __forceinline__ void epilogue32(const f32x16_t (&acc)[RT][2], int c0, TileState (&ts)[RT]) {
  float v[16];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = acc[rt][ct][i];
      tile_update<OVR>(v, c0 + 32 * ct, ts[rt]);
    }
}

// RT = 32-row tiles per wave. RT = 1 (two waves per SIMD) is the one launched: RT = 2 (one wave per
// SIMD, 64 rows, each W fragment feeding 4 MFMAs) needs 412 registers, pays ~90 AGPR reads per
// chunk and measured 26% slower at B = 262144 (loop 69.5k cycles per 64 rows vs 52.7k for two
// 32-row waves; profiles/r2_gemm/phase_probe_rt2.log).
// EPI = false: the softmax epilogue compiled out (measurement only: forced kernel 5 in
// tools/gemm_phase_probe.py; its outputs are meaningless). It splits the class loop's time into the
// MFMA / LDS feed and the epilogue: 44.4k of 52.2k cycles per wave are the feed
// (profiles/r2_gemm/phase_probe_noepi.log).
template <int KS, int WV, int RT, int MODE, bool OVR, bool EPI = true, int AHEAD = 2, bool PRIO = false, bool XNT = false>
__global__ __launch_bounds__(64 * WV) __attribute__((amdgpu_waves_per_eu(RT == 2 ? 1 : 2, RT == 2 ? 1 : 2))) void
gemm_softmax32_kernel(GemmArgs a) {
  static_assert(MODE == 0 || MODE == 2 || MODE == 4, "logits mode runs the 16x16 kernel");
  const uint16_t* __restrict__ X = a.X;
  const uint16_t* __restrict__ W = a.W;
  const float* __restrict__ bias = a.bias;
  const int64_t B = a.B;
  const int K = a.K;
  const int classes_per_split = a.classes_per_split;
  constexpr int K2 = 2 * KS;
  constexpr int NTHR = 64 * WV;
  constexpr int ROWS_PER_BLOCK = 32 * RT * WV;
  if ((int64_t)blockIdx.x * ROWS_PER_BLOCK >= a.B) return;  // XCD-padded grid (uniform per block)
  constexpr int F_ = KS * 32;
  constexpr int NCH = F_ / 8;
  constexpr int W_BYTES = CLASS_CHUNK * lds_row_stride<KS>();
  constexpr int BUF_BYTES = W_BYTES + CLASS_CHUNK * 4;
  constexpr int PIECES = CLASS_CHUNK * NCH / NTHR;
  constexpr int NBUF = 2;
  static_assert(PIECES >= 1 && CLASS_CHUNK * NCH % NTHR == 0, "W chunk must split evenly over the block");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NBUF * BUF_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int h = lane >> 5;
  const int col = lane & 31;
  constexpr bool ovr = OVR;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS_PER_BLOCK + wave * 32 * RT;
  const int c_begin = blockIdx.y * classes_per_split;
  const int c_end = min(K, c_begin + classes_per_split);
  phase_stamp(a, WV, wave, lane, 0);

  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, K * F_ * 2, 0x00020000);
  const auto brsrc = __builtin_amdgcn_make_buffer_rsrc((void*)bias, 0, K * 4, 0x00020000);
#define MLAPI_DMA32(C0, BUF)                                                                                    \
  {                                                                                                              \
    _Pragma("unroll") for (int i = 0; i < PIECES; ++i) __builtin_amdgcn_raw_ptr_buffer_load_lds(                \
        wrsrc, (lds_void_t*)(smem + (BUF) * BUF_BYTES + (i * NTHR + wave * 64) * 16), 16,                        \
        (uint32_t)((((tid + i * NTHR) / NCH) * F_ + lds_pos<KS>((tid + i * NTHR) / NCH, (tid + i * NTHR) % NCH) * 8) * \
                   2),                                                                                           \
        (C0) * F_ * 2, 0, 0);                                                                                    \
    __builtin_amdgcn_raw_ptr_buffer_load_lds(brsrc, (lds_void_t*)(smem + (BUF) * BUF_BYTES + W_BYTES), 4,       \
                                             (uint32_t)lane * 4, (C0) * 4, 0, 0);                                \
  }
#define MLAPI_RAW_BARRIER32()    \
  asm volatile("" ::: "memory"); \
  __builtin_amdgcn_s_barrier();  \
  asm volatile("" ::: "memory");

  TileState ts[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) tile_init(ts[rt]);
  bf16x8_t xf[RT][K2];
  MLAPI_DMA32(c_begin, 0)
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    int64_t r = row0 + rt * 32 + col;
    r = r < B ? r : B - 1;
    const uint16_t* xr = X + r * a.ldx + 8 * h;
#pragma unroll
    for (int k = 0; k < K2; ++k)
      // Plain loads: an X row's 512 bytes reach a wave as 16 instructions of 32 bytes per lane, so
      // each 128-byte line is touched by 4 of them; with the nontemporal hint (XNT, measurement
      // variant) the line was not kept for the other 3 - prologue 10.9k -> 6.8k cycles per wave,
      // the B = 262,144 launch 166.9 -> 150.4 us under the phase stamps (profiles/r6_gemm/)
      xf[rt][k] = XNT ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(xr + k * 16))
                      : *reinterpret_cast<const bf16x8_t*>(xr + k * 16);
  }
  constexpr int kWaitAll = (7 << 4) | (15 << 8);
  __builtin_amdgcn_s_waitcnt(kWaitAll);  // chunk 0 + X
  MLAPI_RAW_BARRIER32()
  phase_stamp(a, WV, wave, lane, 1);
  if (c_begin + CLASS_CHUNK < c_end) MLAPI_DMA32(c_begin + CLASS_CHUNK, 1)
  const FragOff<KS> fo = frag_offsets<KS>(h, col);
  f32x16_t accA[RT][2], accB[RT][2];
  mfma32_chunk<KS, RT>(smem, xf, c_begin, c_end, h, col, accA);
  // Unrolled by the two LDS buffers: chunk c (in accA, buffer 0) / c+1 (accB, buffer 1) swap roles
  // each half, so the buffer offsets are immediates and no accumulator is copied.
  unsigned long long waited = 0;  // profiling only (a.stamps)
  const bool prof = a.stamps != nullptr;
#define MLAPI_WAIT_BARRIER32()                                    \
  {                                                               \
    const unsigned long long w0 = prof ? __builtin_amdgcn_s_memtime() : 0; \
    __builtin_amdgcn_s_waitcnt(kWaitAll);                         \
    MLAPI_RAW_BARRIER32()                                         \
    if (prof) waited += __builtin_amdgcn_s_memtime() - w0;        \
  }
  for (int c0 = c_begin;;) {
    if (c0 + CLASS_CHUNK >= c_end) {
      epilogue32<OVR, RT>(accA, c0, ts);
      break;
    }
    MLAPI_WAIT_BARRIER32()
    if (c0 + 2 * CLASS_CHUNK < c_end) MLAPI_DMA32(c0 + 2 * CLASS_CHUNK, 0)
    fused32_step<KS, RT, OVR, 1, BUF_BYTES, EPI, AHEAD, PRIO>(smem, fo, xf, c0 + CLASS_CHUNK, c_end, h, accB, accA, c0,
                                                        ts);
    c0 += CLASS_CHUNK;
    if (c0 + CLASS_CHUNK >= c_end) {
      epilogue32<OVR, RT>(accB, c0, ts);
      break;
    }
    MLAPI_WAIT_BARRIER32()
    if (c0 + 2 * CLASS_CHUNK < c_end) MLAPI_DMA32(c0 + 2 * CLASS_CHUNK, 1)
    fused32_step<KS, RT, OVR, 0, BUF_BYTES, EPI, AHEAD, PRIO>(smem, fo, xf, c0 + CLASS_CHUNK, c_end, h, accA, accB, c0,
                                                        ts);
    c0 += CLASS_CHUNK;
  }
#undef MLAPI_WAIT_BARRIER32
#undef MLAPI_RAW_BARRIER32
#undef MLAPI_DMA32
  phase_stamp(a, WV, wave, lane, 2);
  if (prof) phase_put(a, WV, wave, lane, 4, waited);
  RowState S[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    S[rt] = tile_result32(ts[rt], h);
    S[rt] = merge_state(S[rt], shfl_state(S[rt], 32), ovr);
  }
  phase_stamp(a, WV, wave, lane, 3);
  if (gridDim.y == 1) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int64_t row = row0 + rt * 32 + col;
      if (h == 0 && row < B) {
        if constexpr (MODE == 0) {
          put_result(a.out_idx, a.out_p, a.ro, row, S[rt].bi, ovr ? sigmoidf_(S[rt].m) / S[rt].s : 1.f / S[rt].s);
        } else if constexpr (MODE == 4) {
          a.rowstate[row] = make_float4(S[rt].m, S[rt].s, __int_as_float(S[rt].bi), 0.f);
        } else {
          a.rowstat[row] = make_float2(S[rt].m + __logf(S[rt].s), __int_as_float(S[rt].bi));
        }
      }
    }
    return;
  }
  // split classes: the 16x16 kernel's tagged-granule merge (see put_granule / granule_merge)
  if (blockIdx.y + 1 < gridDim.y) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int64_t row = row0 + rt * 32 + col;
      if (h == 0 && row < B) put_granule(a, (int64_t)blockIdx.y * B + row, S[rt]);
    }
    return;
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int64_t row = row0 + rt * 32 + col;
    int fail;
    const RowState R = granule_merge<2, 4>(a, row, h, S[rt], row < B, ovr, fail);
    if (h == 0 && row < B) finish_merged<MODE>(a, row, R, fail, ovr);
  }
}

// ---------------------------------------------------------------------------------------------
// Row-group kernel (small / medium batches, and any F): one block owns 16 * NT batch rows and
// ALL classes. Its nw waves split the 64-class chunks round-robin; every wave streams its W
// fragments straight from L2 into VGPRs (no LDS staging, no barrier per chunk: for a small batch
// the tiles kernel above spends its time in DMA latency and the cross-block split merge), keeps
// the online (max, sum, argmax) state per row in registers, and the waves merge through LDS once
// at the end, in wave order (deterministic). The feature dimension is looped in slices of KS * 32
// (F <= 256: one slice, X kept in registers; wider F: 256-feature slices with X reloaded per slice
// from L2), so any F that is a multiple of 256 (or a power of two <= 256) runs in ONE launch with
// no split-K partials and no extra merge pass. MODE: 0 predict, 1 logits, 2 row stats, 4 row state,
// 5 training G: the row stats, then (same block, LDS-held lse) a second pass over the class chunks
// that recomputes the logits and writes G = softmax(z) - onehot(y) (OvR: sigmoid(z) - onehot) as
// bf16 [B][Kp] plus the block's {loss, correct} - the wide-F training step's first launch, so the
// B x K logits never go through HBM (softmax_grad_wide.hip).
template <int KS, int NT, int MODE, bool OVR, bool XLDS = false>
__global__ __launch_bounds__(512) void softmax_rows_kernel(RowsArgs a) {
  constexpr int ROWS = 16 * NT;
  constexpr int SLICE = KS * 32;
  static_assert(!XLDS || ROWS == XLDS_ROWS, "XLDS stages 64 rows");
  __shared__ __attribute__((aligned(16))) uint16_t xs[XLDS ? XLDS_ROWS : 1][XLDS ? XLDS_PITCH : 8];
  __shared__ float4 part[ROWS_MAX_WAVES][ROWS];
  __shared__ float lse_s[MODE == 5 ? ROWS : 1], hit_s[MODE == 5 ? ROWS : 1], wsum_s[MODE == 5 ? ROWS_MAX_WAVES : 1];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int q = lane >> 4;
  const int col = lane & 15;
  const int64_t B = a.B;
  const int K = a.K;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;
  const int nslices = a.F / SLICE;
  const int nchunks = (K + CLASS_CHUNK - 1) / CLASS_CHUNK;

  bf16x8_t xf[NT][KS];
  auto load_x = [&](int slice) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr (XLDS) {
        const uint16_t* xr = &xs[t * 16 + col][slice * SLICE + 8 * q];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) xf[t][ks] = *reinterpret_cast<const bf16x8_t*>(xr + ks * 32);
      } else {
        const int64_t r = min(row0 + t * 16 + col, B - 1);
        const uint16_t* xr = a.X + r * a.ldx + slice * SLICE + 8 * q;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) xf[t][ks] = *reinterpret_cast<const bf16x8_t*>(xr + ks * 32);
      }
    }
  };
  if constexpr (XLDS) {  // stage the block's rows (clamped like load_x) by LDS-DMA
    stage_rows_dma(xs, a.X, a.ldx, a.F, row0, B, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), (int)blockDim.x >> 6,
                   (int)threadIdx.x & 63);
    __builtin_amdgcn_s_waitcnt(WAIT_VM0);
    __syncthreads();
  } else if (nslices == 1) {
    load_x(0);
  }

  RowState st[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) st[t] = RowState{-INFINITY, 0.f, 0x7fffffff};

  // logits of class chunk c0 (bias included) for the block's rows: acc[t][mt] = classes
  // c0 + mt*16 + q*4 + r of batch row (t, col)
  auto chunk_logits = [&](int c0, f32x4_t (&acc)[NT][4]) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int cb = c0 + mt * 16 + q * 4;
      const f32x4_t b0 = {a.bias[min(cb, K - 1)], a.bias[min(cb + 1, K - 1)], a.bias[min(cb + 2, K - 1)],
                          a.bias[min(cb + 3, K - 1)]};
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t][mt] = b0;
    }
    auto load_w = [&](int sl, bf16x8_t(&wf)[4][KS]) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int cls = min(c0 + mt * 16 + col, K - 1);  // classes past K: masked below
        const uint16_t* wr = a.W + (int64_t)cls * a.F + sl * SLICE + 8 * q;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wf[mt][ks] = *reinterpret_cast<const bf16x8_t*>(wr + ks * 32);
      }
    };
    auto mma = [&](const bf16x8_t(&wf)[4][KS]) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[mt][ks], xf[t][ks], acc[t][mt], 0, 0, 0);
    };
    if constexpr (XLDS) {  // nslices even (F a multiple of 256, SLICE 64): W double buffered
      bf16x8_t w0[4][KS], w1[4][KS];
      load_w(0, w0);
      for (int sl = 0; sl < nslices; sl += 2) {
        load_w(sl + 1, w1);
        load_x(sl);
        __builtin_amdgcn_sched_barrier(0);  // the next slice's W loads stay in flight over these MFMAs
        mma(w0);
        if (sl + 2 < nslices) load_w(sl + 2, w0);
        load_x(sl + 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(w1);
      }
    } else {
      for (int sl = 0; sl < nslices; ++sl) {
        if (nslices > 1) load_x(sl);
        bf16x8_t wf[4][KS];
        load_w(sl, wf);
        mma(wf);
      }
    }
  };
  for (int c = wave; c < nchunks; c += nw) {
    const int c0 = c * CLASS_CHUNK;
    f32x4_t acc[NT][4];
    chunk_logits(c0, acc);
    // epilogue: lane owns classes c0 + mt*16 + q*4 + r of batch row (t, col)
    const bool partial = c0 + CLASS_CHUNK > K;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = acc[t][i >> 2][i & 3];
      if (partial) {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = c0 + (i >> 2) * 16 + q * 4 + (i & 3) < K ? v[i] : -INFINITY;
      }
      if constexpr (MODE == 1) {
        const int64_t row = row0 + t * 16 + col;
        if (row < B) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int cls = c0 + (i >> 2) * 16 + q * 4 + (i & 3);
            if (cls < K) a.Z[row * K + cls] = v[i];
          }
        }
      } else {
        if constexpr (MODE == 5) {  // keep the logits for the second pass (each lane re-reads its own)
          const int64_t row = row0 + t * 16 + col;
          if (a.Zs != nullptr && row < B) {
            float* zr = a.Zs + row * (int64_t)a.Kp + c0 + q * 4;
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) *reinterpret_cast<f32x4_t*>(zr + mt * 16) = acc[t][mt];
          }
        }
        online_update<OVR>(v, c0, q, st[t]);
      }
    }
  }
  if constexpr (MODE != 1) {
    // the 4 lanes of a row (q = 0..3) hold disjoint class subsets: merge them, then the waves
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      RowState S = st[t];
      S = merge_state(S, shfl_state(S, 16), OVR);
      S = merge_state(S, shfl_state(S, 32), OVR);
      if (q == 0) part[wave][t * 16 + col] = make_float4(S.m, S.s, __int_as_float(S.bi), 0.f);
    }
    __syncthreads();
    if ((int)threadIdx.x < ROWS) {
      const int r = threadIdx.x;
      const float4 p0 = part[0][r];
      RowState S{p0.x, p0.y, __float_as_int(p0.z)};
      for (int w = 1; w < nw; ++w) {
        const float4 pw = part[w][r];
        S = merge_state(S, RowState{pw.x, pw.y, __float_as_int(pw.z)}, OVR);
      }
      const int64_t row = row0 + r;
      if constexpr (MODE == 5) {
        lse_s[r] = S.m + __logf(S.s);
        hit_s[r] = row < B && S.bi == a.y[row] ? 1.f : 0.f;
      }
      if (row < B) {
        if constexpr (MODE == 0) {
          put_result(a.out_idx, a.out_p, a.ro, row, S.bi, OVR ? sigmoidf_(S.m) / S.s : 1.f / S.s);
        } else if constexpr (MODE == 4) {
          a.rowstate[row] = make_float4(S.m, S.s, __int_as_float(S.bi), 0.f);
        } else if constexpr (MODE == 2) {
          a.rowstat[row] = make_float2(S.m + __logf(S.s), __int_as_float(S.bi));
        }
      }
    }
  }
  if constexpr (MODE == 5) {
    __syncthreads();  // lse_s / hit_s
    float lse[NT];
    int yr[NT];
    bool live[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int64_t row = row0 + t * 16 + col;
      live[t] = row < B;
      lse[t] = lse_s[t * 16 + col];
      yr[t] = live[t] ? a.y[row] : -1;
    }
    float loss = 0.f;
    const int nchunks_p = a.Kp / CLASS_CHUNK;  // G's padded columns are written too (zeros)
    for (int c = wave; c < nchunks_p; c += nw) {
      const int c0 = c * CLASS_CHUNK;
      f32x4_t acc[NT][4];
      if (a.Zs != nullptr) {  // the first pass's logits: no second GEMM (the X reads and MFMAs)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const float* zr = a.Zs + min(row0 + t * 16 + col, B - 1) * (int64_t)a.Kp + c0 + q * 4;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) acc[t][mt] = *reinterpret_cast<const f32x4_t*>(zr + mt * 16);
        }
      } else {
        chunk_logits(c0, acc);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (!live[t]) continue;
        uint16_t* gr = a.G + (row0 + t * 16 + col) * (int64_t)a.Kp + c0 + q * 4;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          uint16_t gb[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int cls = c0 + mt * 16 + q * 4 + r;
            const float z = acc[t][mt][r];
            float g = 0.f;
            if (cls < K) {
              const bool is_y = cls == yr[t];
              const float p = OVR ? 1.f / (1.f + __expf(-z)) : __expf(z - lse[t]);
              g = p - (is_y ? 1.f : 0.f);
              if constexpr (OVR) loss += fmaxf(z, 0.f) - (is_y ? z : 0.f) + log1pf(__expf(-fabsf(z)));
              else if (is_y) loss += lse[t] - z;
            }
            gb[r] = bf16_rne(g);
          }
          uint2 pk;
          pk.x = (uint32_t)gb[0] | ((uint32_t)gb[1] << 16);
          pk.y = (uint32_t)gb[2] | ((uint32_t)gb[3] << 16);
          *reinterpret_cast<uint2*>(gr + mt * 16) = pk;
        }
      }
    }
    // the block's {loss, correct}: lanes, then waves in order (deterministic)
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) loss += __shfl_xor(loss, off, 64);
    if (lane == 0) wsum_s[wave] = loss;
    __syncthreads();
    if (threadIdx.x == 0) {
      float l = 0.f, h = 0.f;
      for (int w = 0; w < nw; ++w) l += wsum_s[w];
      for (int r = 0; r < ROWS; ++r) h += hit_s[r];
      a.stat_slabs[2 * (int64_t)blockIdx.x] = l;
      a.stat_slabs[2 * (int64_t)blockIdx.x + 1] = h;
    }
  }
}

// MODE 5 with the logits in registers (wide-F training G, F in (512, 1024], K <= 1024): the XLDS
// row-group kernel computed each wave's two class chunks one after the other and parked the first
// pass's logits in an f32 [B][Kp] buffer for the G pass (2 x 268 MB of HBM traffic per F = 1024
// step at B = 65,536). Here a wave accumulates BOTH its chunks in one sweep over F (2 x 64 f32 per
// lane), so the logits never leave the registers: the row stats merge across the waves through LDS
// as before, and the G pass reads the accumulators. The W fragments ping-pong between the two
// chunks - the next fragment's loads are in flight under the other chunk's 32 MFMAs - and X comes
// from the block's LDS copy (staged once, as XLDS).
// W in MFMA-fragment order (pack_w_frag_kernel): the 16 classes x 32 features one fragment load
// needs are ONE contiguous 1 KB block in lane order, block (class block cb, k-step kk) at
// (cb * F / 32 + kk) KB. Each packed load touches 8 full 128-byte lines; the row-major load
// touched 16 class rows x 64 B (16 lines, half of each used) - measured 326-336 -> 202-204 us for
// the launch at F = 1024, K = 1000, B = 65,536 (the data was wrong in that probe; same bytes).
__global__ __launch_bounds__(256) void pack_w_frag_kernel(const uint16_t* __restrict__ W, int K, int F,
                                                          uint16_t* __restrict__ Wp, int64_t pieces) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= pieces) return;
  const int lane = (int)(t & 63);
  const int64_t blk = t >> 6;
  const int nks = F >> 5;
  const int cb = (int)(blk / nks), kk = (int)(blk - (int64_t)cb * nks);
  const int cls = cb * 16 + (lane & 15);
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (cls < K) v = *reinterpret_cast<const uint4*>(W + (int64_t)cls * F + kk * 32 + 8 * (lane >> 4));
  *reinterpret_cast<uint4*>(Wp + t * 8) = v;
}

__host__ __device__ inline size_t packed_w_bytes(int K, int F) { return (size_t)((K + 15) / 16) * (size_t)(F / 32) * 1024; }

template <bool OVR, bool PACKED = false>
__global__ __launch_bounds__(512) void softmax_rows_g2_kernel(RowsArgs a) {
  constexpr int NT = 4, KS = 2, ROWS = 16 * NT, SLICE = KS * 32;
  static_assert(ROWS == XLDS_ROWS, "the X copy holds 64 rows");
  __shared__ __attribute__((aligned(16))) uint16_t xs[XLDS_ROWS][XLDS_PITCH];
  __shared__ float4 part[ROWS_MAX_WAVES][ROWS];
  __shared__ float lse_s[ROWS], hit_s[ROWS], wsum_s[ROWS_MAX_WAVES];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = blockDim.x >> 6;
  const int q = lane >> 4;
  const int col = lane & 15;
  const int64_t B = a.B;
  const int K = a.K;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;
  const int nslices = a.F / SLICE;
  const int nchunks = (K + CLASS_CHUNK - 1) / CLASS_CHUNK;
  const int cc[2] = {wave * CLASS_CHUNK, (wave + nw) * CLASS_CHUNK};
  const bool has_b = wave + nw < nchunks;  // wave-uniform
  stage_rows_dma(xs, a.X, a.ldx, a.F, row0, B, wave, nw, lane);  // lands under the bias loads
  f32x4_t acc[2][NT][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int cb = cc[h] + mt * 16 + q * 4;
      const f32x4_t b0 = {a.bias[min(cb, K - 1)], a.bias[min(cb + 1, K - 1)], a.bias[min(cb + 2, K - 1)],
                          a.bias[min(cb + 3, K - 1)]};
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[h][t][mt] = b0;
    }
  __builtin_amdgcn_s_waitcnt(WAIT_VM0);
  __syncthreads();
  bf16x8_t wa[4][KS], wb[4][KS];
  // W through a range-checked descriptor: ONE per-lane offset (class col, feature group q), the
  // chunk / slice / k-step part a scalar offset, classes past K read as zeros (masked in the
  // epilogue) - no clamped 64-bit address per fragment (those cost the registers the accumulators need)
  const auto wrs = PACKED ? __builtin_amdgcn_make_buffer_rsrc((void*)a.Wp, 0, (int)packed_w_bytes(K, a.F), 0x00020000)
                         : __builtin_amdgcn_make_buffer_rsrc((void*)a.W, 0, K * a.F * 2, 0x00020000);
  // PACKED: one contiguous 1 KB per fragment load (lane-linear); classes past K are out of the
  // packed range (or zero-filled in its last class block) and read as zeros either way
  const uint32_t wlane = PACKED ? (uint32_t)lane * 16u : (uint32_t)(col * a.F + 8 * q) * 2u;
  // k-step major: the first k-step's MFMAs wait for its 4 fragments only (vmcnt counts in order)
  auto load_w = [&](int c0, int sl, bf16x8_t(&wf)[4][KS]) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        wf[mt][ks] = __builtin_bit_cast(
            bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(
                          wrs, wlane,
                          PACKED
                              ? (uint32_t)((((c0 + mt * 16) >> 4) * (a.F >> 5) + sl * KS + ks) * 1024)
                              : (uint32_t)(((c0 + mt * 16) * a.F + sl * SLICE + ks * 32) * 2),
                          0));
  };
  // X fragments one k-step at a time from the LDS copy (16 registers, not 32: the 128 accumulators
  // and both W fragments must fit 256 VGPRs at 2 waves per SIMD); the other wave covers the reads
  auto mma = [&](int sl, const bf16x8_t(&wf)[4][KS], f32x4_t(&ac)[NT][4]) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8_t xk[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        xk[t] = *reinterpret_cast<const bf16x8_t*>(&xs[t * 16 + col][sl * SLICE + ks * 32 + 8 * q]);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          ac[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[mt][ks], xk[t], ac[t][mt], 0, 0, 0);
    }
  };
  // Branch-free: a branch around a load group makes the wait insertion fall back to vmcnt(0) at the
  // join, which waits for the fragments just issued for the OTHER chunk and defeats the ping-pong.
  // So the loads and MFMAs of chunk b run on every wave (past K the range-checked loads return
  // zeros and chunk b's results are never read), and the last slice's look-ahead load of chunk a
  // (out of range or the next class row's features, never used) is issued anyway.
  load_w(cc[0], 0, wa);
  for (int sl = 0; sl < nslices; ++sl) {
    load_w(cc[1], sl, wb);  // in flight under chunk a's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    mma(sl, wa, acc[0]);
    load_w(cc[0], sl + 1, wa);  // in flight under chunk b's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    mma(sl, wb, acc[1]);
  }
  // row stats: online (max, sum, first argmax) over the wave's chunks, then the lanes of a row, then
  // the waves in order (deterministic)
  RowState st[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) st[t] = RowState{-INFINITY, 0.f, 0x7fffffff};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 1 && !has_b) break;
    const int c0 = cc[h];
    const bool partial = c0 + CLASS_CHUNK > K;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = acc[h][t][i >> 2][i & 3];
      if (partial) {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = c0 + (i >> 2) * 16 + q * 4 + (i & 3) < K ? v[i] : -INFINITY;
      }
      online_update<OVR>(v, c0, q, st[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    RowState S = st[t];
    S = merge_state(S, shfl_state(S, 16), OVR);
    S = merge_state(S, shfl_state(S, 32), OVR);
    if (q == 0) part[wave][t * 16 + col] = make_float4(S.m, S.s, __int_as_float(S.bi), 0.f);
  }
  __syncthreads();
  if ((int)threadIdx.x < ROWS) {
    const int r = threadIdx.x;
    const float4 p0 = part[0][r];
    RowState S{p0.x, p0.y, __float_as_int(p0.z)};
    for (int w = 1; w < nw; ++w) {
      const float4 pw = part[w][r];
      S = merge_state(S, RowState{pw.x, pw.y, __float_as_int(pw.z)}, OVR);
    }
    const int64_t row = row0 + r;
    lse_s[r] = S.m + __logf(S.s);
    hit_s[r] = row < B && S.bi == a.y[row] ? 1.f : 0.f;
  }
  __syncthreads();
  // G = softmax(z) - onehot(y) (OvR: sigmoid(z) - onehot) as bf16 [B][Kp], from the accumulators
  float lse[NT];
  int yr[NT];
  bool live[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int64_t row = row0 + t * 16 + col;
    live[t] = row < B;
    lse[t] = lse_s[t * 16 + col];
    yr[t] = live[t] ? a.y[row] : -1;
  }
  float loss = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 1 && !has_b) break;
    const int c0 = cc[h];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (!live[t]) continue;
      uint16_t* gr = a.G + (row0 + t * 16 + col) * (int64_t)a.Kp + c0 + q * 4;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        uint16_t gb[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cls = c0 + mt * 16 + q * 4 + r;
          const float z = acc[h][t][mt][r];
          float g = 0.f;
          if (cls < K) {
            const bool is_y = cls == yr[t];
            const float p = OVR ? 1.f / (1.f + __expf(-z)) : __expf(z - lse[t]);
            g = p - (is_y ? 1.f : 0.f);
            if constexpr (OVR) loss += fmaxf(z, 0.f) - (is_y ? z : 0.f) + log1pf(__expf(-fabsf(z)));
            else if (is_y) loss += lse[t] - z;
          }
          gb[r] = bf16_rne(g);
        }
        uint2 pk;
        pk.x = (uint32_t)gb[0] | ((uint32_t)gb[1] << 16);
        pk.y = (uint32_t)gb[2] | ((uint32_t)gb[3] << 16);
        *reinterpret_cast<uint2*>(gr + mt * 16) = pk;
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) loss += __shfl_xor(loss, off, 64);
  if (lane == 0) wsum_s[wave] = loss;
  __syncthreads();
  if (threadIdx.x == 0) {
    float l = 0.f, h = 0.f;
    for (int w = 0; w < nw; ++w) l += wsum_s[w];
    for (int r = 0; r < ROWS; ++r) h += hit_s[r];
    a.stat_slabs[2 * (int64_t)blockIdx.x] = l;
    a.stat_slabs[2 * (int64_t)blockIdx.x + 1] = h;
  }
}

// Which kernel serves (B, K, F): the row-group kernel only where the tiles kernel has no
// instantiation (F > 512, the only kernel that loops F). At F <= 512 the tiles kernel with class
// splits is faster at every B (profiles/r2_gemm/sweep.log: B <= 4096 rows 17-19 us vs tiles 7-10).
int g_force_kernel = 0;  // benchmark hook: 0 automatic, 1 tiles 16x16, 2 row-group, 3 tiles 32x32
                         // (measurement only: 5 32x32 with the epilogue compiled out, 6 / 7 with
                         // W fragments 1 / 3 k-steps ahead instead of 2)

bool rows_supported(int F) { return F == 32 || F == 64 || F == 128 || F == 256 || (F > 256 && F % 256 == 0); }
bool tiles_supported(int F) { return F == 32 || F == 64 || F == 128 || F == 256 || F == 512; }

bool use_rows(int64_t B, int F) {
  if (!tiles_supported(F)) return true;
  if (g_force_kernel == 1) return false;
  (void)B;
  return g_force_kernel == 2 && rows_supported(F);
}

// 16-row tiles per block of the row-group kernel. Wide F (> 256) at large B: every block streams all
// of W through its waves, so more rows per block mean less L2 traffic - 4 tiles in 128-feature
// slices (KS = 4: 64 rows, half of round 3's 32-row blocks' W traffic), or 6 tiles in 64-feature
// slices (KS = 2, 96 rows; needs >= 2 class chunks: the row merge takes one thread per row).
// MLAPI_ROWS_NT = 2 / 4 / 6 picks (2: round 3's 256-feature slices).
int rows_nt(int64_t B, int F, int K) {
  static const int want = [] {
    const char* e = std::getenv("MLAPI_ROWS_NT");
    return e != nullptr ? std::atoi(e) : 6;  // 6 vs 4: 0.99-1.01 vs 1.05-1.06 ms per F = 1024 step
  }();
  if (B < 16384) return 1;
  if (F <= 256 || want <= 2) return 2;
  return (want >= 6 && K > CLASS_CHUNK) ? 6 : 4;
}

// the LDS-staged-X variant of the row-group kernel: F in (512, 1024] (64 rows x F fit the LDS),
// batches large enough for 64-row blocks, more than one class chunk (the row merge takes one thread
// per row). MLAPI_ROWS_XLDS=0 keeps the register-X kernel (measurement)
bool rows_xlds(int64_t B, int F, int K) {
  static const bool on = [] {
    const char* e = std::getenv("MLAPI_ROWS_XLDS");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on && F > 512 && F <= XLDS_FMAX && F % 256 == 0 && B >= 16384 && K > CLASS_CHUNK;
}

// softmax_rows_g2_kernel serves the wide-F training G launch where the XLDS kernel would (64-row
// blocks, F in (512, 1024]) and every wave has at most two class chunks (K <= 1024) with no padded
// chunk past them (Kp = K rounded up to 64). MLAPI_ROWS_G2=0 keeps the XLDS kernel + logits buffer.
int g_rows_g2 = -1;  // gemm_softmax_set_rows_g2: -1 MLAPI_ROWS_G2 (default on), 0 off, 1 on

bool rows_g2(int64_t B, int F, int K, int Kp) {
  static const bool env = [] {
    const char* e = std::getenv("MLAPI_ROWS_G2");
    return e == nullptr || std::atoi(e) != 0;
  }();
  const bool on = g_rows_g2 < 0 ? env : g_rows_g2 != 0;
  const int nchunks = (K + CLASS_CHUNK - 1) / CLASS_CHUNK;
  return on && rows_xlds(B, F, K) && nchunks <= 2 * ROWS_MAX_WAVES && Kp == nchunks * CLASS_CHUNK;
}

template <int MODE>
void launch_rows(RowsArgs a, int kind, hipStream_t stream) {
  if (!rows_supported(a.F))
    throw std::invalid_argument("gemm_softmax: F must be 32/64/128/256 or a multiple of 256 (pad other widths)");
  if (a.ldx % 8 != 0 || reinterpret_cast<uintptr_t>(a.X) % 16 || reinterpret_cast<uintptr_t>(a.W) % 16)
    throw std::invalid_argument("gemm_softmax: X rows and W must be 16-byte aligned");
  const int nchunks = (a.K + CLASS_CHUNK - 1) / CLASS_CHUNK;
  const int nw = nchunks < ROWS_MAX_WAVES ? nchunks : ROWS_MAX_WAVES;
  const bool ovr = kind == KIND_OVR;
  if (rows_xlds(a.B, a.F, a.K)) {
    const dim3 grid((unsigned)((a.B + XLDS_ROWS - 1) / XLDS_ROWS)), block(64 * nw);
    if (ovr)
      hipLaunchKernelGGL((softmax_rows_kernel<2, 4, MODE, true, true>), grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL((softmax_rows_kernel<2, 4, MODE, false, true>), grid, block, 0, stream, a);
    MLAPI_HIP_CHECK(hipGetLastError());
    return;
  }
  const int nt = rows_nt(a.B, a.F, a.K);
  const dim3 grid((unsigned)((a.B + 16 * nt - 1) / (16 * nt))), block(64 * nw);
#define MLAPI_ROWS_LAUNCH(KSV, NTV)                                                                \
  do {                                                                                             \
    if (ovr)                                                                                       \
      hipLaunchKernelGGL((softmax_rows_kernel<KSV, NTV, MODE, true>), grid, block, 0, stream, a);  \
    else                                                                                           \
      hipLaunchKernelGGL((softmax_rows_kernel<KSV, NTV, MODE, false>), grid, block, 0, stream, a); \
  } while (0)
#define MLAPI_ROWS_NT(KSV)     \
  if (nt == 2)                 \
    MLAPI_ROWS_LAUNCH(KSV, 2); \
  else                         \
    MLAPI_ROWS_LAUNCH(KSV, 1);
  if (a.F == 32) {
    MLAPI_ROWS_NT(1)
  } else if (a.F == 64) {
    MLAPI_ROWS_NT(2)
  } else if (a.F == 128) {
    MLAPI_ROWS_NT(4)
  } else if (nt == 6) {
    MLAPI_ROWS_LAUNCH(2, 6);
  } else if (nt == 4) {
    MLAPI_ROWS_LAUNCH(4, 4);
  } else {
    MLAPI_ROWS_NT(8)
  }
#undef MLAPI_ROWS_NT
#undef MLAPI_ROWS_LAUNCH
  MLAPI_HIP_CHECK(hipGetLastError());
}

RowsArgs rows_args(const void* X, int64_t ldx, const void* W, const float* b, int64_t B, int F, int K) {
  RowsArgs a{};
  a.X = static_cast<const uint16_t*>(X);
  a.ldx = ldx;
  a.W = static_cast<const uint16_t*>(W);
  a.bias = b;
  a.B = B;
  a.K = K;
  a.F = F;
  return a;
}

struct Plan {
  int k32 = 0;            // > 0: the 32x32x16 kernel with this many waves per block
  int rt32 = 1;           // its 32-row tiles per wave
  int nt;                 // 16-row tiles per wave (16x16x32 kernel)
  int splits;
  int classes_per_split;
  int64_t row_blocks;
};

// Benchmark hook (tools/gemm_plan_sweep.py): force (nt, splits); 0 = automatic.
int g_force_nt = 0, g_force_splits = 0;

// rows per block of the tiles kernel (host mirror of tiles_block_waves)
int block_rows(int F, int nt) {
  (void)F;
  return 16 * nt * 4;
}

bool t32_supported(int F) { return F == 64 || F == 128 || F == 256; }

int cus_per_xcd() {  // CUs of the current device / 8 XCDs (the dispatcher round-robins blocks over them)
  static int cache[64] = {0};
  int dev = 0;
  MLAPI_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return 32;
  if (cache[dev] == 0) {
    int n = 0;
    MLAPI_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    cache[dev] = n >= 8 ? n / 8 : 1;
  }
  return cache[dev];
}

// allow32 = false for the logits mode (only the 16x16 kernel writes Z)
Plan make_plan(int64_t B, int K, int F, bool training, bool allow32 = true) {
  Plan p;
  if (allow32 && t32_supported(F)) {
    if (g_force_kernel == 3 || g_force_kernel >= 5) p.k32 = 4;  // 5-9: 32x32 measurement variants
    // B = 8192, K = 1000: 32x32 with 4 splits 10.2-10.4 us vs 16x16 10.8; at K = 100 (2 chunks)
    // the 16x16 kernel keeps it (5.2-5.5 vs 6.7 us; profiles/r4_gemm_merge/)
    else if (g_force_kernel == 0 && (B >= 16384 || (B >= 8192 && K >= 512))) p.k32 = 4;
  }
  // 32 rows per wave (NT = 2) halve the LDS fragment reads per MFMA. It pays once the register
  // staging is gone (LDS-DMA): B=262144 230 -> 172 us, B=8192 about even, B=1024 worse
  // (tools/gemm_plan_sweep.py, profiles/r1_pmc/gemm_plan_sweep_dma.log). KS = 16 at NT = 2 needs
  // all 256 VGPRs.
  (void)training;
  p.nt = (F <= 256 && B >= 16384) ? 2 : 1;
  if (g_force_nt == 1 || g_force_nt == 2) p.nt = g_force_nt;
  if (g_force_splits > 0) {
    const int rows_per_block = p.k32 ? 32 * p.rt32 * p.k32 : block_rows(F, p.nt);
    p.row_blocks = (B + rows_per_block - 1) / rows_per_block;
    const int chunks = (K + CLASS_CHUNK - 1) / CLASS_CHUNK;
    const int sp = g_force_splits > chunks ? chunks : g_force_splits;
    p.classes_per_split = ((chunks + sp - 1) / sp) * CLASS_CHUNK;
    p.splits = (K + p.classes_per_split - 1) / p.classes_per_split;
    if (!(p.splits > 1 && p.row_blocks * 4 > COUNTER_BYTES)) return p;
  }
  const int rows_per_block = p.k32 ? 32 * p.rt32 * p.k32 : block_rows(F, p.nt);
  p.row_blocks = (B + rows_per_block - 1) / rows_per_block;
  const int chunks = (K + CLASS_CHUNK - 1) / CLASS_CHUNK;
  // Splits per row block, measured with the granule merge (profiles/r4_gemm_merge/, F = 256,
  // K = 1000): one block per CU up to 64 row blocks (B = 1024: 16 splits of one 64-class chunk,
  // 6.0 us vs 6.5 at 8 splits; B = 2048: 8), two per CU beyond (B = 8192: 4 splits); the 32x32
  // kernel (128-row blocks) one per CU up to 128 row blocks (B = 16384: 2 splits, 15.4 vs 16.1 us).
  // The round-3 ticket merge wanted >= 2 chunks per block (LDS double buffer) and 2 blocks per CU.
  const int64_t one_per_cu = p.k32 ? 128 : 64;
  int64_t want = p.row_blocks <= one_per_cu ? (256 + p.row_blocks - 1) / p.row_blocks
                                            : (512 + p.row_blocks - 1) / p.row_blocks;
  int splits = (int)(want < 1 ? 1 : (want > chunks ? chunks : want));
  const int chunks_per_split = (chunks + splits - 1) / splits;
  p.classes_per_split = chunks_per_split * CLASS_CHUNK;
  p.splits = (K + p.classes_per_split - 1) / p.classes_per_split;
  if (p.splits > 1 && p.row_blocks * 4 > COUNTER_BYTES) {  // counters do not fit: no split
    p.splits = 1;
    p.classes_per_split = chunks * CLASS_CHUNK;
  }
  return p;
}

template <int MODE, int KS>
void launch32(const GemmArgs& args, const dim3& grid, int rt, hipStream_t stream) {
  if constexpr (MODE != 1) {
    // 4 waves per block, 1 row tile per wave (8-wave blocks and RT = 2 measured slower:
    // profiles/r2_gemm/phase_probe_rt2.log)
    (void)rt;
    const bool o = args.kind == KIND_OVR;
    if constexpr (MODE == 0 && KS == 8) {
      if (!o && g_force_kernel == 5) {  // measurement: epilogue compiled out
        hipLaunchKernelGGL((gemm_softmax32_kernel<KS, 4, 1, MODE, false, false>), grid, dim3(256), 0, stream, args);
        return;
      }
      if (!o && g_force_kernel == 9) {  // measurement: X loaded with the nontemporal hint (round 5's loads)
        hipLaunchKernelGGL((gemm_softmax32_kernel<KS, 4, 1, MODE, false, true, 2, false, true>), grid, dim3(256), 0,
                           stream, args);
        return;
      }
      if (!o && g_force_kernel == 8) {  // measurement: s_setprio around each k-step's MFMAs
        hipLaunchKernelGGL((gemm_softmax32_kernel<KS, 4, 1, MODE, false, true, 2, true>), grid, dim3(256), 0, stream,
                           args);
        return;
      }
      if (!o && (g_force_kernel == 6 || g_force_kernel == 7)) {  // measurement: fragment prefetch depth 1 / 3
        if (g_force_kernel == 6)
          hipLaunchKernelGGL((gemm_softmax32_kernel<KS, 4, 1, MODE, false, true, 1>), grid, dim3(256), 0, stream, args);
        else
          hipLaunchKernelGGL((gemm_softmax32_kernel<KS, 4, 1, MODE, false, true, 3>), grid, dim3(256), 0, stream, args);
        return;
      }
    }
    if (o) hipLaunchKernelGGL((gemm_softmax32_kernel<KS, 4, 1, MODE, true>), grid, dim3(256), 0, stream, args);
    else hipLaunchKernelGGL((gemm_softmax32_kernel<KS, 4, 1, MODE, false>), grid, dim3(256), 0, stream, args);
  }
}

void* g_stamps = nullptr;  // profiling hook (gemm_softmax_set_stamps)

// split-merge granule tags: 28 bits, never 0 (a zero-initialised or cleared granule is never live)
unsigned next_merge_epoch() {
  static std::atomic<unsigned> e{0};
  unsigned v;
  do v = (e.fetch_add(1, std::memory_order_relaxed) + 1) & 0x0fffffffu;
  while (v == 0);
  return v;
}

template <int MODE>
void launch_mode(GemmArgs args, int F, const Plan& plan, hipStream_t stream) {
  args.classes_per_split = plan.classes_per_split;
  args.stamps = static_cast<unsigned long long*>(g_stamps);
  // XCD-local split merge (put_granule / granule_merge): on by default, MLAPI_GEMM_XCD=0 selects the
  // agent-scope protocol. The grid's x extent is padded to a multiple of 8 (blocks past the batch
  // return at once) so that every split of a row block lands on the same XCD.
  static const int xcd_env = [] {
    const char* e = getenv("MLAPI_GEMM_XCD");
    return e ? atoi(e) : 1;
  }();
  const int rb_pad = (plan.row_blocks + 7) / 8 * 8;
  args.xcd_local = (MODE != 1 && xcd_env != 0 && plan.splits > 1 && rb_pad < XCD_ERR_SLOT &&
                    (uint64_t)plan.splits * (uint64_t)args.B * 16u < 0x7fffffffu && xcd_local_allowed(stream))
                       ? 1
                       : 0;
  args.xcd_inject = args.xcd_local ? xcd_local_take_inject() : 0;
  if (MODE != 1 && plan.splits > 1) {
    // granule offsets are 32-bit buffer offsets (automatic plans split only below 512 row blocks)
    if ((uint64_t)plan.splits * (uint64_t)args.B * 16u >= 0x7fffffffu)
      throw std::invalid_argument("gemm_softmax: split plan's partials exceed 2 GiB");
    args.epoch = next_merge_epoch();
  }
  const dim3 grid((unsigned)(args.xcd_local ? rb_pad : plan.row_blocks), (unsigned)plan.splits);
  if (MODE != 1 && plan.k32) {
    if (F == 64) launch32<MODE, 2>(args, grid, plan.rt32, stream);
    else if (F == 128) launch32<MODE, 4>(args, grid, plan.rt32, stream);
    else launch32<MODE, 8>(args, grid, plan.rt32, stream);
    MLAPI_HIP_CHECK(hipGetLastError());
    return;
  }
#define MLAPI_GEMM_LAUNCH(KSV, NTV)                                                                      \
  do {                                                                                                   \
    if (args.kind == KIND_OVR)                                                                           \
      hipLaunchKernelGGL((gemm_softmax_kernel<KSV, NTV, MODE, true>), grid,                             \
                         dim3(64 * tiles_block_waves<KSV, NTV>()), 0, stream, args);                     \
    else                                                                                                 \
      hipLaunchKernelGGL((gemm_softmax_kernel<KSV, NTV, MODE, false>), grid,                            \
                         dim3(64 * tiles_block_waves<KSV, NTV>()), 0, stream, args);                     \
  } while (0)
  const int ks = F / 32;
  if (F != 32 && F != 64 && F != 128 && F != 256 && F != 512)
    throw std::invalid_argument("gemm_softmax: F must be 32, 64, 128, 256 or 512 (pad other widths)");
#define MLAPI_GEMM_NT(KSV)       \
  if (plan.nt == 2)              \
    MLAPI_GEMM_LAUNCH(KSV, 2);   \
  else                           \
    MLAPI_GEMM_LAUNCH(KSV, 1);
  if (ks == 1) {
    MLAPI_GEMM_NT(1)
  } else if (ks == 2) {
    MLAPI_GEMM_NT(2)
  } else if (ks == 4) {
    MLAPI_GEMM_NT(4)
  } else if (ks == 8) {
    MLAPI_GEMM_NT(8)
  } else {
    MLAPI_GEMM_NT(16)
  }
#undef MLAPI_GEMM_NT
#undef MLAPI_GEMM_LAUNCH
  MLAPI_HIP_CHECK(hipGetLastError());
}

GemmArgs base_args(const void* X, const void* W, int64_t B, int F, int K, int kind) {
  GemmArgs a{};
  a.X = static_cast<const uint16_t*>(X);
  a.ldx = F;
  a.W = static_cast<const uint16_t*>(W);
  a.B = B;
  a.K = K;
  a.kind = kind;
  static const int xnt16 = [] {
    const char* e = std::getenv("MLAPI_GEMM_XNT16");
    return e != nullptr && std::atoi(e) != 0 ? 1 : 0;
  }();
  a.x_nt = xnt16;
  return a;
}

}  // namespace

void gemm_softmax_set_stamps(void* stamps) { g_stamps = stamps; }

size_t gemm_softmax_xcd_err_offset() { return (size_t)XCD_ERR_SLOT * 4; }

void gemm_softmax_force_plan(int nt, int splits, int kernel) {
  g_force_nt = nt;
  g_force_splits = splits;
  g_force_kernel = kernel;
}

size_t softmax_rowstats_workspace(int64_t B, int K, int F) {
  const Plan p = make_plan(B, K, F, true);
  return (size_t)COUNTER_BYTES + (p.splits > 1 ? (size_t)p.splits * (size_t)B * sizeof(float4) : 0);
}

void launch_softmax_rowstats(const void* X_aug, int64_t ldx, const void* W, const float* b, int64_t B, int F, int K,
                             int kind, void* rowstat_out, void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (B <= 0) return;
  if (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("softmax_rowstats: multiclass kinds only");
  if (ldx < F || ldx % 8 != 0) throw std::invalid_argument("softmax_rowstats: ldx must be >= F and a multiple of 8");
  if (!tiles_supported(F)) {  // wide models (F a multiple of 256 beyond 512): the row-group kernel
    RowsArgs ra = rows_args(X_aug, ldx, W, b, B, F, K);
    ra.rowstat = static_cast<float2*>(rowstat_out);
    launch_rows<2>(ra, kind, stream);
    return;
  }
  const Plan plan = make_plan(B, K, F, true);
  if (ws_bytes < softmax_rowstats_workspace(B, K, F))
    throw std::invalid_argument("softmax_rowstats: workspace too small (zero it once)");
  GemmArgs args = base_args(X_aug, W, B, F, K, kind);
  args.ldx = ldx;
  args.bias = b;
  args.counters = static_cast<unsigned int*>(workspace);
  args.partials = reinterpret_cast<float4*>(static_cast<unsigned char*>(workspace) + COUNTER_BYTES);
  args.rowstat = static_cast<float2*>(rowstat_out);
  launch_mode<2>(args, F, plan, stream);
}

void gemm_softmax_plan_info(int64_t B, int K, int F, int64_t out[5]) {
  if (use_rows(B, F)) {
    out[0] = 2, out[1] = 0, out[2] = 1, out[3] = K, out[4] = 0;
    return;
  }
  const Plan p = make_plan(B, K, F, false);
  out[0] = p.k32 ? 1 : 0, out[1] = p.nt, out[2] = p.splits, out[3] = p.classes_per_split, out[4] = p.row_blocks;
}

size_t gemm_softmax_workspace(int64_t B, int K, int F) {
  if (use_rows(B, F)) return 0;
  const Plan p = make_plan(B, K, F, false);
  return p.splits > 1 ? (size_t)COUNTER_BYTES + (size_t)p.splits * (size_t)B * sizeof(float4) : 0;
}

// NOTE: every gemm_softmax launch goes through hipLaunchKernelGGL on `stream`; the split merge
// clears its granule tags with plain stores, which is only safe because a HIP stream launch ends
// with a system-scope release. A direct-dispatch path (KernelLauncher, packets without that
// release) must switch these clears to write-through stores first.
void launch_gemm_softmax(const void* X, const void* W, const float* b, int64_t B, int F, int K, int kind,
                         int32_t* out_idx, float* out_p, void* workspace, size_t ws_bytes, hipStream_t stream,
                         RecOut ro) {
  if (B <= 0) return;
  if (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("gemm_softmax: multiclass kinds only (binary models use gemv_binary)");
  if (use_rows(B, F)) {
    RowsArgs ra = rows_args(X, F, W, b, B, F, K);
    ra.out_idx = out_idx;
    ra.out_p = out_p;
    ra.ro = ro;
    launch_rows<0>(ra, kind, stream);
    return;
  }
  const Plan plan = make_plan(B, K, F, false);
  if (plan.splits > 1 && ws_bytes < gemm_softmax_workspace(B, K, F))
    throw std::invalid_argument("gemm_softmax: workspace too small (must be zero-initialised once)");
  GemmArgs args = base_args(X, W, B, F, K, kind);
  args.bias = b;
  args.out_idx = out_idx;
  args.out_p = out_p;
  args.ro = ro;
  if (plan.splits > 1) {
    args.counters = static_cast<unsigned int*>(workspace);
    args.partials = reinterpret_cast<float4*>(static_cast<unsigned char*>(workspace) + COUNTER_BYTES);
  }
  launch_mode<0>(args, F, plan, stream);
}

void launch_gemm_rowstate(const void* X, const void* W, const float* b, int64_t B, int F, int K, int kind,
                          void* out_state, void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (B <= 0) return;
  if (K < 1 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("gemm_rowstate: multiclass kinds only");
  if (use_rows(B, F)) {
    RowsArgs ra = rows_args(X, F, W, b, B, F, K);
    ra.rowstate = static_cast<float4*>(out_state);
    launch_rows<4>(ra, kind, stream);
    return;
  }
  const Plan plan = make_plan(B, K, F, false);
  if (plan.splits > 1 && ws_bytes < gemm_softmax_workspace(B, K, F))
    throw std::invalid_argument("gemm_rowstate: workspace too small (must be zero-initialised once)");
  GemmArgs args = base_args(X, W, B, F, K, kind);
  args.bias = b;
  args.rowstate = static_cast<float4*>(out_state);
  if (plan.splits > 1) {
    args.counters = static_cast<unsigned int*>(workspace);
    args.partials = reinterpret_cast<float4*>(static_cast<unsigned char*>(workspace) + COUNTER_BYTES);
  }
  launch_mode<4>(args, F, plan, stream);
}

int softmax_rows_g_blocks(int64_t B, int F, int K) {  // launch_rows' grid: one {loss, correct} slab per block
  const int rows = rows_xlds(B, F, K) ? XLDS_ROWS : 16 * rows_nt(B, F, K);
  return (int)((B + rows - 1) / rows);
}

bool softmax_rows_g_keeps_logits(int64_t B, int F, int K, int Kp) { return rows_g2(B, F, K, Kp); }

void gemm_softmax_set_rows_g2(int on) { g_rows_g2 = on; }

int g_w_packed = -1;  // gemm_softmax_set_w_packed: -1 MLAPI_G2_PACKED (default on), 0 off, 1 on

bool w_packed_on() {
  static const bool env = [] {
    const char* e = std::getenv("MLAPI_G2_PACKED");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return g_w_packed < 0 ? env : g_w_packed != 0;
}

size_t softmax_rows_g_wpack_bytes(int64_t B, int F, int K, int Kp) {
  return rows_g2(B, F, K, Kp) ? packed_w_bytes(K, F) : 0;
}

void gemm_softmax_set_w_packed(int on) { g_w_packed = on; }

void launch_softmax_rows_g(const void* X_aug, int64_t ldx, const void* W, const float* b, const int32_t* y, int64_t B,
                           int F, int K, int kind, uint16_t* G, int Kp, float* stat_slabs, float* Zs,
                           void* w_packed, hipStream_t stream) {
  if (B <= 0) return;
  if (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("softmax_rows_g: multiclass kinds only");
  if (Kp % CLASS_CHUNK != 0 || Kp < K) throw std::invalid_argument("softmax_rows_g: Kp must be K rounded up to 64");
  RowsArgs ra = rows_args(X_aug, ldx, W, b, B, F, K);
  ra.y = y;
  ra.G = G;
  ra.Kp = Kp;
  ra.stat_slabs = stat_slabs;
  ra.Zs = Zs;
  if (rows_g2(B, F, K, Kp)) {
    // logits kept in registers (no Zs round trip): 8 waves x (at most) 2 class chunks
    const int nchunks = (K + CLASS_CHUNK - 1) / CLASS_CHUNK;
    const dim3 grid((unsigned)((B + XLDS_ROWS - 1) / XLDS_ROWS)), block(64 * std::min(nchunks, ROWS_MAX_WAVES));
    if (w_packed != nullptr && w_packed_on()) {
      // W re-laid in fragment order first (K x F bf16 read once, ~2 MB at F = 1024), then every
      // block's fragment loads are contiguous 1 KB reads
      if (reinterpret_cast<uintptr_t>(w_packed) % 16 != 0)
        throw std::invalid_argument("softmax_rows_g: packed W buffer must be 16-byte aligned");
      const int64_t pieces = (int64_t)packed_w_bytes(K, F) / 16;
      hipLaunchKernelGGL(pack_w_frag_kernel, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0, stream,
                         static_cast<const uint16_t*>(W), K, F, static_cast<uint16_t*>(w_packed), pieces);
      MLAPI_HIP_CHECK(hipGetLastError());
      ra.Wp = static_cast<const uint16_t*>(w_packed);
      if (kind == KIND_OVR)
        hipLaunchKernelGGL((softmax_rows_g2_kernel<true, true>), grid, block, 0, stream, ra);
      else
        hipLaunchKernelGGL((softmax_rows_g2_kernel<false, true>), grid, block, 0, stream, ra);
    } else if (kind == KIND_OVR) {
      hipLaunchKernelGGL(softmax_rows_g2_kernel<true>, grid, block, 0, stream, ra);
    } else {
      hipLaunchKernelGGL(softmax_rows_g2_kernel<false>, grid, block, 0, stream, ra);
    }
    MLAPI_HIP_CHECK(hipGetLastError());
    return;
  }
  launch_rows<5>(ra, kind, stream);
}

void launch_gemm_logits_ld(const void* X, int64_t ldx, const void* W, const float* b, int64_t B, int F, int K, float* Z,
                           hipStream_t stream) {
  if (B <= 0) return;
  RowsArgs ra = rows_args(X, ldx, W, b, B, F, K);
  ra.Z = Z;
  launch_rows<1>(ra, KIND_MULTINOMIAL, stream);
}

void launch_gemm_logits(const void* X, const void* W, const float* b, int64_t B, int F, int K, float* Z,
                        hipStream_t stream) {
  if (B <= 0) return;
  if (use_rows(B, F)) {
    RowsArgs ra = rows_args(X, F, W, b, B, F, K);
    ra.Z = Z;
    launch_rows<1>(ra, KIND_MULTINOMIAL, stream);
    return;
  }
  Plan plan = make_plan(B, K, F, false, false);
  plan.splits = (K + plan.classes_per_split - 1) / plan.classes_per_split;  // no merge needed for logits
  GemmArgs args = base_args(X, W, B, F, K, KIND_MULTINOMIAL);
  args.bias = b;
  args.Z = Z;
  launch_mode<1>(args, F, plan, stream);
}

}  // namespace mlapi
