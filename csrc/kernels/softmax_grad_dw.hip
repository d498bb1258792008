// Fused multiclass training gradient: G = softmax(z) - onehot(y) (OvR: sigmoid(z) - onehot) and
// dW_aug = G^T X_aug in ONE kernel, so the B x K gradient never goes through HBM (SURVEY 2.3 K6 at
// BASELINE config 5 scale; reference: LogisticRegression.fit, `Logistic Regression.ipynb:34`).
//
// v1 of the training step wrote G (bf16, 131 MB at B=65536, K=1000) from the gemm_softmax MODE 3
// tiles and ran dW = G^T X as a split-B hipBLASLt GEMM + a sum over the splits: 72 + 68 + 10 us of
// a 213 us step (profiles/r1_session6/train_softmax_kernel_stats.csv). Here each block owns 64
// classes (16 per wave) and a contiguous range of 64-row tiles:
//
//  1. logits, transposed: Z^T tile = X_tile W_c^T with X as the MFMA A operand (M = rows) and the
//     wave's 16 W rows as B (N = classes; held in VGPRs for the whole kernel), accumulators
//     initialised to the bias. The C layout leaves one CLASS per lane (col = lane & 15) and 4 rows
//     per M-tile in its registers;
//  2. epilogue in registers: with lse per row from the row-stats pass (gemm_softmax MODE 2),
//     g = exp(z - lse) - [y == class], loss and the intercept gradient sum(g) accumulate per lane;
//  3. dW_c += G X_tile: the 4 rows a lane holds in each of two M-tiles ARE the 8 k-values of a
//     16x16x32 A operand (the order of k inside one MFMA is free as long as A and B agree), so G
//     feeds the next MFMA straight from registers; the matching B operand (8 rows of one feature
//     column) comes from the SAME LDS image of the X tile through ds_read_b64_tr_b16
//     (cdna_hip_programming.md T10). 16 N-tiles of f32 accumulators = 64 VGPRs per lane.
//
// X tiles are double-buffered in LDS by global_load_lds DMA (lane-linear destination, swizzle
// applied on the source address: image (b) of T10 - 256-byte rows, 16-byte chunk ch of row r at
// ch ^ (((r & 3) << 2) | ((r >> 2) & 3)) - in 128-column sub-images). The M index -> row map of
// the A operand (grp_row) makes both the row reads and the transposed reads conflict-free. Per-block dW partials go to
// [row group][K][F_aug] slabs folded by the deterministic slab reduction (no atomics: DP replicas
// and reruns stay bitwise identical); XCD-aware block order keeps the class groups that share a
// row range on one XCD's L2.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "mlapi/common.h"
#include "mlapi/kernels.h"
#include "dist/p2p_device.h"

namespace mlapi {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;
typedef __attribute__((ext_vector_type(4))) short i16x4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void glob_void_t;

#ifndef MLAPI_GDW_EXP
#define MLAPI_GDW_EXP 0  // experiment mask for tools/gdw_bench.hip (1 no epilogue math, 2 no dW MFMA,
#endif                   // 4 no logits MFMA, 8 no dW phase, 16 no per-tile DMA/barriers, 64 no dW reads)
constexpr int ROWS = 64;                // rows per tile (4 M-tiles of 16)
constexpr int WAVE_CLASSES = 16;        // classes per MFMA N-tile; a wave owns NC of them
constexpr int SUB_BYTES = ROWS * 256;   // one [64 rows][128 bf16] sub-image
constexpr int META_BYTES = 1024;        // [64 lse] [64 argmax bits] [64 y] [256 B DMA pad]
constexpr float LOG2E_F = 1.4426950408889634f;
constexpr float LN2_F = 0.6931471805599453f;

__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// ds_read_b64_tr_b16 at an immediate offset, invisible to hipcc's wait insertion (see step 3)
template <int OFF>
__device__ __forceinline__ i16x4_t tr_read(uint32_t addr) {
  i16x4_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
// ds_read_b128 at an immediate offset, invisible to hipcc's wait insertion
template <int OFF, typename T>
__device__ __forceinline__ T lds_read_b128(uint32_t addr) {
  T v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int N, typename A>
__device__ __forceinline__ void lgkm_wait(A& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(N));
}
// s_waitcnt lgkmcnt(N) that orders every later use of a and b after it
template <int N, typename A, typename B>
__device__ __forceinline__ void lgkm_wait(A& a, B& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N));
}
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
__device__ __forceinline__ int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
// byte offset of element column c (a multiple of 4) of tile row r
__device__ __forceinline__ int img_off(int r, int c) {
  return (c >> 7) * SUB_BYTES + r * 256 + ((((c >> 3) & 15) ^ swz(r)) << 4) + ((c & 7) << 1);
}
// First tile row of lane group g's 4 C-layout rows inside a 16-row M-tile. Quad q of M indices (i >> 2) maps to tile rows 4 * QROW[q] .. +3 with QROW = {0, 2, 3, 1}: the
// 16-lane groups of the ds_read_b128 A-operand read ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...)
// then hit four different swizzle classes (conflict-free), and each 32-lane half of the transposed
// B-operand read takes two blocks 8 rows apart (conflict-free per T10).
__device__ __forceinline__ int grp_row(int g) { return ((0x1320 >> (4 * g)) & 3) << 2; }
// A-operand M index -> tile row (the same map)
__device__ __forceinline__ int m_row(int i) { return (i & 3) | grp_row(i >> 2); }

struct GradDwArgs {
  const uint16_t* X;  // X_aug [B, ldx] bf16 (first F columns read; column F is the ones column)
  int64_t ldx;
  const uint16_t* W;  // [K, F] bf16
  const float* bias;  // [K]
  const int32_t* y;   // [B]
  const float2* rowstat;  // [B] {lse, argmax bits} from the row-stats pass
  int64_t B;
  int K;
  int tiles;            // ceil(B / 64)
  int tiles_per_group;  // row-group length in tiles
  int row_groups;
  int class_groups;
  int ldw;              // F_aug: slab row stride
  float* dw_slabs;      // [row_groups][K][ldw]
  float* stat_slabs;    // [row_groups * class_groups][2] = {loss_sum, n_correct}
};

// NC = class tiles of 16 per wave. NC = 1: 64 classes per block, <= 256 VGPRs, 2 waves/SIMD (the
// other wave hides the epilogue and the barriers). NC = 2: 128 classes per block, 1 wave/SIMD; every
// X fragment read from LDS feeds two MFMAs, halving the LDS bytes per MFMA (at NC = 1 both phases
// need 256 B/clk/CU, the LDS array's peak).
//
// (A software pipeline across tiles with 3 LDS buffers - the logits of tile t+1 and the epilogue of
// tile t in one basic block - measured equal, 136.9-137.3 vs 136.2-141.9 us per step
// (profiles/r5_train/s35_pipe_ab.log), and left the build in round 5.)
//
// F = 512 (KS = 16): the double-buffered tile is 2 x 65 KB of LDS (one block per CU) and the 32
// dW N-tiles alone take 128 accumulator registers, so it runs NC = 1 at one wave per SIMD
// (512 VGPRs: the accumulators spill into the AGPR half instead of scratch).
template <int KS, int NC>
constexpr int gdw_waves_per_eu() {
  return KS >= 16 ? 1 : 3 - NC;
}

template <int KS, bool OVR, int NC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(gdw_waves_per_eu<KS, NC>(),
                                                                     gdw_waves_per_eu<KS, NC>()))) void
softmax_grad_dw_kernel(GradDwArgs a) {
  static_assert(KS < 16 || NC == 1, "F = 512 runs 16 classes per wave");
  constexpr int NBUF = 2;
  constexpr int CLASSES = 4 * WAVE_CLASSES * NC;
  constexpr int F_ = KS * 32;
  constexpr int X_BYTES = (F_ / 128) * SUB_BYTES;
  constexpr int BUF_BYTES = X_BYTES + META_BYTES;
  constexpr int NT = F_ / 16;  // dW N-tiles (features)
  static_assert(F_ % 128 == 0, "sub-images are 128 columns wide");
  // ALL LDS in one __shared__ object: a second one (even a small reduction array) makes hipcc wait
  // vmcnt(0) before the first ds_read of every tile, draining the in-flight DMA (guide 4(a)).
  __shared__ __attribute__((aligned(16))) unsigned char smem[NBUF * BUF_BYTES];
  float* const red = reinterpret_cast<float*>(smem);  // stats reduction, after the last tile

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform: scalar descriptors
  const int col = lane & 15;
  const int g = lane >> 4;
  const int64_t B = a.B;
  const int K = a.K;

  // XCD-aware block order: hardware block id b runs on XCD b % 8; logical id L puts the class
  // groups of one row range on one XCD (its L2 then serves the 16x reuse of every X tile).
  const int nblk = a.row_groups * a.class_groups;
  int L = blockIdx.x;
  if (nblk % 8 == 0) L = (blockIdx.x & 7) * (nblk >> 3) + (blockIdx.x >> 3);
  const int rg = L / a.class_groups;
  const int cg = L % a.class_groups;
  const int t_begin = rg * a.tiles_per_group;
  const int t_end = min(a.tiles, t_begin + a.tiles_per_group);

  const int cls0 = cg * CLASSES + wave * WAVE_CLASSES * NC + col;  // this lane's class, tile h: + 16 h

  // W rows of the wave's classes: the B operands of every logits MFMA, resident in VGPRs.
  // Padded classes: logits -1e30 (finite: 0 * z stays 0), so p = 0, g = 0 and loss = 0 with no
  // per-element class check.
  bf16x8_t wf[NC][KS];
  float bv[NC];
#pragma unroll
  for (int h = 0; h < NC; ++h) {
    const int cls = cls0 + h * WAVE_CLASSES;
    const int cls_c = min(cls, K - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[h][ks] = *reinterpret_cast<const bf16x8_t*>(a.W + (int64_t)cls_c * F_ + ks * 32 + g * 8);
    bv[h] = cls < K ? a.bias[cls_c] : -1e30f;
  }

  f32x4_t acc[NC][NT];
  // intercept gradient sum_rows g = G^T (ones column of X_aug): one more MFMA per 32 rows with a
  // constant B operand (column 0 = 1, the rest 0) instead of a VALU add per element
  f32x4_t acc_db[NC];
#pragma unroll
  for (int h = 0; h < NC; ++h) {
    acc_db[h] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[h][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8_t ones_b = col == 0 ? bf16x8_t{1, 1, 1, 1, 1, 1, 1, 1} : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  float loss = 0.f, lz = 0.f, correct = 0.f;
  const bool row_wave = cg == 0 && wave == 0;  // one wave per row range: correct count (+ sum lse)

  // ---- tile DMA: KS 16-byte pieces per thread + one dword of row metadata per lane, through
  // buffer_load ... lds with per-tile scalar descriptors (base = the tile's first row, range = its
  // valid rows): rows past B fail the range check instead of being clamped per lane, and the
  // per-lane offsets are tile-invariant (piece i: row (tid >> 4) + 16 (i & 3), sub-image i >> 2).
  uint32_t vo[4];
  {
    const int r = tid >> 4;
    const int c = ((tid & 15) ^ swz(r)) << 3;
#pragma unroll
    for (int k = 0; k < 4; ++k) vo[k] = (uint32_t)(((r + 16 * k) * a.ldx + c) * 2);
  }
  const uint32_t mvo = wave < 2 ? (uint32_t)(lane * 8 + wave * 4) : (uint32_t)(lane * 4);
#define MLAPI_DMA_TILE(T, BUF)                                                                          \
  {                                                                                                     \
    const int64_t row0 = (int64_t)(T) * ROWS;                                                           \
    const int nrows = (int)min<int64_t>(ROWS, B - row0);                                                \
    unsigned char* dst = smem + (BUF) * BUF_BYTES;                                                      \
    const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)(a.X + row0 * a.ldx), 0,                 \
                                                       nrows * (int)a.ldx * 2, 0x00020000);             \
    _Pragma("unroll") for (int i = 0; i < KS; ++i)                                                      \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsx, (lds_void_t*)(dst + (i * 256 + wave * 64) * 16), 16, \
                                               vo[i & 3], (i >> 2) * 256, 0, 0);                        \
    const auto rsm = wave < 2 ? __builtin_amdgcn_make_buffer_rsrc((void*)(a.rowstat + row0), 0, nrows * 8, \
                                                                  0x00020000)                           \
                              : __builtin_amdgcn_make_buffer_rsrc((void*)(a.y + row0), 0, nrows * 4,    \
                                                                  0x00020000);                          \
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsm, (lds_void_t*)(dst + X_BYTES + wave * 256), 4, mvo, 0, 0, 0); \
  }
#define MLAPI_RAW_BARRIER()      \
  asm volatile("" ::: "memory"); \
  __builtin_amdgcn_s_barrier();  \
  asm volatile("" ::: "memory");
  constexpr int kWaitTile = ((KS + 1) & 15) | (7 << 4) | (15 << 8) | (((KS + 1) >> 4) << 14);
  constexpr int kWaitAll = (7 << 4) | (15 << 8);

  // Rows past B are never DMA'd; if this block owns the batch's ragged last tile, zero the LDS once
  // so those rows hold zeros (not stale non-finite bits) where 0-gradients multiply them.
  if ((int64_t)t_end * ROWS > B) {
    for (int o = tid * 16; o < NBUF * BUF_BYTES; o += 256 * 16) *reinterpret_cast<int4*>(smem + o) = int4{0, 0, 0, 0};
    __syncthreads();
  }
  // ---- per-tile pieces (one LDS image at byte offset xo; its row metadata at xo + X_BYTES)
  constexpr int PF = 6;  // A-fragment reads in flight
  constexpr int NA = 4 * KS;
  i32x4_t y4[4], l4[4];  // row metadata of the tile in the epilogue: y and lse of 4 rows per M-tile
  bf16x8_t ga[NC][2];    // G of the tile as the dW A operand
  auto init_z = [&](f32x4_t(&zz)[NC][4]) {
#pragma unroll
    for (int h = 0; h < NC; ++h)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) zz[h][mt] = f32x4_t{bv[h], bv[h], bv[h], bv[h]};
  };
  auto read_meta = [&](uint32_t mb) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const uint32_t rb = mt * 16 + grp_row(g);
      y4[mt] = lds_read_b128<512, i32x4_t>(mb + rb * 4);
      l4[mt] = lds_read_b128<0, i32x4_t>(mb + rb * 4);
    }
  };
  auto wait_meta = [&]() {  // every metadata read landed; one wait on all CFG paths
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(y4[0]), "+v"(y4[1]), "+v"(y4[2]), "+v"(y4[3]), "+v"(l4[0]), "+v"(l4[1]), "+v"(l4[2]),
                   "+v"(l4[3]));
  };
  // 1. Z^T tile (rows x the wave's classes) into zz (bias-initialised by the caller). A fragments
  //    through inline-asm ds_read_b128 with PF reads in flight (counted lgkmcnt waits; 4 per-lane
  //    bases, one per ks & 3, the rest immediate offsets); with_meta: the tile's row metadata
  //    (LDS after the X image: [64 lse][64 argmax bits][64 y]) is read behind the last A read.
  auto logits = [&](uint32_t xo, f32x4_t(&zz)[NC][4], auto with_meta) {
    uint32_t ab[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ab[k] = xo + img_off(m_row(col), k * 32 + g * 8);
    bf16x8_t xa[NA];
    auto issue_a = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int ks = i / 4, mt = i % 4;
      xa[i] = lds_read_b128<(ks >> 2) * SUB_BYTES + mt * 16 * 256, bf16x8_t>(ab[ks & 3]);
    };
    static_for<PF>(issue_a);
    static_for<NA>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr bool meta = decltype(with_meta)::value;
      if constexpr (i + PF < NA) issue_a(std::integral_constant<int, i + PF>{});
      if constexpr (meta && i + PF == NA) read_meta(xo + X_BYTES);
      constexpr int after = (NA - 1 - i < PF ? NA - 1 - i : PF) + (meta && i + PF >= NA ? 8 : 0);
      lgkm_wait<after>(xa[i]);
#pragma unroll
      for (int h = 0; h < NC; ++h) {
        if constexpr (!(MLAPI_GDW_EXP & 4))
          zz[h][i % 4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[i], wf[h][i / 4], zz[h][i % 4], 0, 0, 0);
        else
          zz[h][i % 4] += __builtin_bit_cast(f32x4_t, xa[i]);
      }
    });
  };
  // 2. gradient in registers: lane holds rows mt*16 + grp_row(g) + r of class cls0 + 16 h. Only
  //    the last tile of the batch has padded rows (`partial`); padded classes are -1e30 logits.
  auto epilogue = [&](auto partial, const f32x4_t(&zz)[NC][4], int rows_left) {
    if constexpr (MLAPI_GDW_EXP & 1) {
#pragma unroll
      for (int h = 0; h < NC; ++h)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) ga[h][mt >> 1][(mt & 1) * 4 + r] = (__bf16)zz[h][mt][r];
      return;
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const uint32_t rb = mt * 16 + grp_row(g);
      const int yv[4] = {y4[mt][0], y4[mt][1], y4[mt][2], y4[mt][3]};
      const float lse[4] = {__int_as_float(l4[mt][0]), __int_as_float(l4[mt][1]), __int_as_float(l4[mt][2]),
                            __int_as_float(l4[mt][3])};
#pragma unroll
      for (int h = 0; h < NC; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool hot = cls0 + h * WAVE_CLASSES == yv[r];
          const float zv = zz[h][mt][r];
          float pr;
          if constexpr (OVR) {
            const float e = __builtin_amdgcn_exp2f(-fabsf(zv) * LOG2E_F);  // exp(-|z|)
            const float re = __builtin_amdgcn_rcpf(1.f + e);
            pr = zv >= 0.f ? re : e * re;
            const float l = fmaxf(zv, 0.f) + __builtin_amdgcn_logf(1.f + e) * LN2_F;
            loss += decltype(partial)::value ? (rb + r < (uint32_t)rows_left ? l : 0.f) : l;
          } else {
            pr = __builtin_amdgcn_exp2f((zv - lse[r]) * LOG2E_F);
          }
          // loss = sum(lse) - sum(z_y) (multinomial); OvR: sum(softplus terms) - sum(z_y)
          float msk = hot ? 1.f : 0.f;
          float gv = pr - msk;
          if constexpr (decltype(partial)::value) {
            const bool ok = rb + r < (uint32_t)rows_left;
            gv = ok ? gv : 0.f;
            msk = ok ? msk : 0.f;
          }
          lz = fmaf(msk, zv, lz);
          ga[h][mt >> 1][(mt & 1) * 4 + r] = (__bf16)gv;
        }
    }
  };
  auto row_stats = [&](uint32_t mb, int rows_left) {
    if (row_wave) {  // one row per lane: argmax == y, and sum lse
      int yl, al, ll;
      asm volatile("ds_read_b32 %0, %1 offset:512" : "=v"(yl) : "v"(mb + lane * 4));
      asm volatile("ds_read_b32 %0, %1 offset:256" : "=v"(al) : "v"(mb + lane * 4));
      asm volatile("ds_read_b32 %0, %1" : "=v"(ll) : "v"(mb + lane * 4));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(yl), "+v"(al), "+v"(ll));
      if (lane < rows_left) {
        correct += al == yl ? 1.f : 0.f;
        if constexpr (!OVR) loss += __int_as_float(ll);
      }
    }
  };
  // 3. dW_c += G X_tile: B operand = 8 rows of one feature column via two transposed reads
  //    (lane 4q+p of group g addresses row base + q, columns n*16 + 4p .. +3). Inline asm with
  //    counted waits (DW_PF (j, n) steps in flight): hipcc treats the ds_read_tr builtin as
  //    aliasing the tile DMA in flight and would wait vmcnt(0) before the first one. Row base
  //    + 16 (hi), + 32 (j) and the second 128-column sub-image (n >= 8) keep the swizzle, so they
  //    are immediate offsets from 8 per-lane bases (one per n & 7).
  auto dw = [&](uint32_t xo) {
    uint32_t trb[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) trb[n] = xo + img_off(grp_row(g) + (col >> 2), n * 16 + 4 * (col & 3));
    i16x4_t tl[2 * NT], th[2 * NT];
    auto issue = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int off = (i / NT) * 32 * 256 + ((i % NT) >> 3) * SUB_BYTES;
      tl[i] = tr_read<off>(trb[i & 7]);
      th[i] = tr_read<off + 16 * 256>(trb[i & 7]);
    };
    constexpr int DW_PF = 6;  // (j, n) steps in flight: 2 * DW_PF reads <= 15 (lgkmcnt field)
    if constexpr (!(MLAPI_GDW_EXP & (8 | 64))) static_for<DW_PF>(issue);
    if constexpr (!(MLAPI_GDW_EXP & 8)) static_for<2 * NT>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      bf16x8_t xbf;
      if constexpr (MLAPI_GDW_EXP & 64) {  // experiment: MFMAs only, constant B operand
        xbf = ones_b;
      } else {
        if constexpr (i + DW_PF < 2 * NT) issue(std::integral_constant<int, i + DW_PF>{});
        constexpr int pending = 2 * (2 * NT - 1 - i < DW_PF ? 2 * NT - 1 - i : DW_PF);
        lgkm_wait<pending>(tl[i], th[i]);
        xbf = __builtin_shufflevector(__builtin_bit_cast(bf16x4_t, tl[i]), __builtin_bit_cast(bf16x4_t, th[i]), 0,
                                      1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int h = 0; h < NC; ++h) {
        if constexpr (!(MLAPI_GDW_EXP & 2))
          acc[h][i % NT] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga[h][i / NT], xbf, acc[h][i % NT], 0, 0, 0);
        else
          acc[h][i % NT] += __builtin_bit_cast(f32x4_t, xbf);
        if constexpr (i % NT == NT - 1)
          acc_db[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga[h][i / NT], ones_b, acc_db[h], 0, 0, 0);
      }
    });
  };
  const uint32_t smem_off = lds_off(smem);

  {
    int buf = 0;
    MLAPI_DMA_TILE(t_begin, 0)
    if (t_begin + 1 < t_end) {
      MLAPI_DMA_TILE(t_begin + 1, 1)
      __builtin_amdgcn_s_waitcnt(kWaitTile);  // W, bias and tile 0 landed; tile 1 may still fly
    } else {
      __builtin_amdgcn_s_waitcnt(kWaitAll);
    }
    MLAPI_RAW_BARRIER()
    for (int t = t_begin; t < t_end; ++t) {
      const uint32_t xo = smem_off + buf * BUF_BYTES;
      const int rows_left = (int)min<int64_t>(ROWS, B - (int64_t)t * ROWS);
      f32x4_t z[NC][4];
      init_z(z);
      logits(xo, z, std::true_type{});
      wait_meta();
      if (rows_left == ROWS)
        epilogue(std::false_type{}, z, rows_left);
      else
        epilogue(std::true_type{}, z, rows_left);
      row_stats(xo + X_BYTES, rows_left);
      dw(xo);
      if (MLAPI_GDW_EXP & 16) {
      } else if (t + 2 < t_end) {
        MLAPI_RAW_BARRIER()  // every wave is done reading `buf`
        MLAPI_DMA_TILE(t + 2, buf)
        __builtin_amdgcn_s_waitcnt(kWaitTile);  // tile t+1 landed, t+2 flies
      } else {
        __builtin_amdgcn_s_waitcnt(kWaitAll);
      }
      if (!(MLAPI_GDW_EXP & 16)) {
        MLAPI_RAW_BARRIER()
      }
      buf ^= 1;
    }
  }
#undef MLAPI_RAW_BARRIER
#undef MLAPI_DMA_TILE

  // ---- dW partial of this row group: lane holds dW[class base + 4g + r][n*16 + col]
  float* slab = a.dw_slabs + (int64_t)rg * K * a.ldw;
#pragma unroll
  for (int h = 0; h < NC; ++h) {
    const int cbase = cg * CLASSES + wave * WAVE_CLASSES * NC + h * WAVE_CLASSES + 4 * g;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (cbase + r < K) {
        float* dst = slab + (int64_t)(cbase + r) * a.ldw + col;
#pragma unroll
        for (int n = 0; n < NT; ++n) dst[n * 16] = acc[h][n][r];
      }
    }
    // intercept gradient (column F) and the zero pad columns F+1 .. ldw-1: lane col of acc_db
    // holds G^T e_col, i.e. sum(g) for col 0 and 0 otherwise
    if (col < a.ldw - F_) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (cbase + r < K) slab[(int64_t)(cbase + r) * a.ldw + F_ + col] = acc_db[h][r];
    }
  }
  // ---- [loss, correct] of the block (deterministic tree); padded rows/classes have z_y terms of 0
  loss -= lz;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    loss += __shfl_xor(loss, off, 64);
    correct += __shfl_xor(correct, off, 64);
  }
  __syncthreads();  // every wave is done reading the last tile before `red` overwrites it
  if (lane == 0) {
    red[wave * 2] = loss;
    red[wave * 2 + 1] = correct;
  }
  __syncthreads();
  if (tid < 2) a.stat_slabs[(int64_t)L * 2 + tid] = red[tid] + red[2 + tid] + red[4 + tid] + red[6 + tid];
}

// Slab sums in one launch: blocks 0 .. nb-1 fold the [row group][K * F_aug] dW slabs, one float4
// column per thread over all slabs in a fixed order (coalesced 16-B loads, 4 in flight); the last
// block folds the per-block [loss, correct] pairs with a fixed tree. Deterministic: no atomics.
// Final slab sums (+ fused SGD update). DP: the ranks' sums are exchanged inside this kernel
// (p2p_device.h): block b stores its local f32x4 column sums (the last block: the [loss, correct]
// stats) into the exchange buffer, waits for block b of every rank and sums them in rank order
// before the update. Exchange layout: [width4 f32x4 | loss | correct].
template <bool DP>
__global__ __launch_bounds__(256) void gdw_reduce_kernel(const f32x4_t* __restrict__ slabs, int nslabs, int width4,
                                                         f32x4_t* __restrict__ out, const float* __restrict__ stat_slabs,
                                                         int nstat, float* __restrict__ stats_out, Sgd2D upd,
                                                         P2PBlockArgs dp) {
  if (blockIdx.x == gridDim.x - 1) {
    float l = 0.f, c = 0.f;
    for (int i = threadIdx.x; i < nstat; i += 256) {
      l += stat_slabs[2 * i];
      c += stat_slabs[2 * i + 1];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      l += __shfl_xor(l, off, 64);
      c += __shfl_xor(c, off, 64);
    }
    __shared__ float red[8];
    if ((threadIdx.x & 63) == 0) {
      red[(threadIdx.x >> 6) * 2] = l;
      red[(threadIdx.x >> 6) * 2 + 1] = c;
    }
    __syncthreads();
    float st = 0.f;
    if (threadIdx.x < 2) st = (red[threadIdx.x] + red[2 + threadIdx.x]) + (red[4 + threadIdx.x] + red[6 + threadIdx.x]);
    if (DP && dp.world > 1) {  // one rank: nothing to exchange (the same kernel, no peers)
      float* xs = dp.mine + 4 * (int64_t)width4;
      if (threadIdx.x < 2) xs[threadIdx.x] = st;
      if (!p2p_block_sync(dp, blockIdx.x)) return;
      if (threadIdx.x < 2) {
        const float own = st;  // this rank's slice from registers, not re-read from the buffer
        st = dp.rank == 0 ? own : dp.peer[0][4 * (int64_t)width4 + threadIdx.x];
        for (int r = 1; r < dp.world; ++r) st += r == dp.rank ? own : dp.peer[r][4 * (int64_t)width4 + threadIdx.x];
      }
    }
    if (threadIdx.x < 2) stats_out[threadIdx.x] = st;
    return;
  }
  const int j = blockIdx.x * 256 + threadIdx.x;
  const bool active = j < width4;
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  if (active) {
    int i = 0;
    for (; i + 4 <= nslabs; i += 4) {
      f32x4_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(slabs + (int64_t)(i + u) * width4 + j);
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; i < nslabs; ++i) {
      s += __builtin_nontemporal_load(slabs + (int64_t)i * width4 + j);
    }
  }
  // fused SGD update of the 4 parameters of column j from the reduced gradient s (sgd_update_2d's
  // arithmetic); np / nm: the new parameters and momenta (published by two-shot owners)
  auto update = [&](const f32x4_t& g, f32x4_t& np, f32x4_t& nm) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t e = 4 * (int64_t)j + q;
      const int64_t row = e / upd.cols;
      const int c = (int)(e - row * upd.cols);
      float d = g[q] * upd.inv_n + (c < upd.pen_cols ? upd.l2 * upd.params[e] : 0.f);
      if (upd.mom != nullptr) {
        const float v = upd.momentum * upd.mom[e] + d;
        upd.mom[e] = v;
        nm[q] = v;
        d = v;
      }
      np[q] = upd.params[e] - upd.lr * d;
    }
  };
  // the new parameters (and momenta) of column j into the replica + its shadow copies
  auto store_params = [&](const f32x4_t& np, const f32x4_t* nm) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t e = 4 * (int64_t)j + q;
      const int64_t row = e / upd.cols;
      const int c = (int)(e - row * upd.cols);
      upd.params[e] = np[q];
      if (nm != nullptr && upd.mom != nullptr) upd.mom[e] = (*nm)[q];
      if (upd.shadow_w != nullptr && c < upd.pen_cols)
        upd.shadow_w[row * upd.pen_cols + c] = __builtin_bit_cast(uint16_t, (__bf16)np[q]);
      if (upd.shadow_b != nullptr && c == upd.pen_cols) upd.shadow_b[row] = np[q];
    }
  };
  if (DP && dp.world > 1 && dp.two_shot) {
    // two-shot: rank (b % world) reduces and updates these columns, the others copy its result
    f32x4_t* mine = reinterpret_cast<f32x4_t*>(dp.mine);
    if (active) mine[j] = s;
    const int owner = (int)(blockIdx.x % (unsigned)dp.world);
    p2p_block_publish(dp, blockIdx.x);
    if (dp.rank == owner) {
      if (!p2p_block_wait(dp, blockIdx.x)) return;  // peer missing: status recorded, no update
      if (active) {
        const f32x4_t own = s;
        s = dp.rank == 0 ? own : reinterpret_cast<const f32x4_t*>(dp.peer[0])[j];
        for (int r = 1; r < dp.world; ++r) s += r == dp.rank ? own : reinterpret_cast<const f32x4_t*>(dp.peer[r])[j];
        out[j] = s;
        f32x4_t* pub = reinterpret_cast<f32x4_t*>(dp.mine + dp.pub_off);  // [grad | params | momenta]
        pub[j] = s;
        if (upd.params != nullptr) {
          f32x4_t np = {0.f, 0.f, 0.f, 0.f}, nm = {0.f, 0.f, 0.f, 0.f};
          update(s, np, nm);
          store_params(np, nullptr);
          pub[width4 + j] = np;
          if (upd.mom != nullptr) pub[2 * (int64_t)width4 + j] = nm;
        }
      }
      p2p_block_publish(dp, blockIdx.x, true);
    } else {
      if (!p2p_block_wait(dp, blockIdx.x, owner, true)) return;
      if (active) {
        const f32x4_t* pub = reinterpret_cast<const f32x4_t*>(dp.peer[owner] + dp.pub_off);
        out[j] = pub[j];
        if (upd.params != nullptr) {
          const f32x4_t np = pub[width4 + j];
          if (upd.mom != nullptr) {
            const f32x4_t nm = pub[2 * (int64_t)width4 + j];
            store_params(np, &nm);
          } else {
            store_params(np, nullptr);
          }
        }
      }
    }
    return;
  }
  if (DP && dp.world > 1) {
    if (active) reinterpret_cast<f32x4_t*>(dp.mine)[j] = s;
    if (!p2p_block_sync(dp, blockIdx.x)) return;  // peer missing: status recorded, no update
    if (active) {  // rank order; the own slice from registers (same bits as the published copy)
      const f32x4_t own = s;
      s = dp.rank == 0 ? own : reinterpret_cast<const f32x4_t*>(dp.peer[0])[j];
      for (int r = 1; r < dp.world; ++r) s += r == dp.rank ? own : reinterpret_cast<const f32x4_t*>(dp.peer[r])[j];
    }
  }
  if (!active) return;
  out[j] = s;
  if (upd.params != nullptr) {  // uniform: the fused SGD update of these 4 parameters
    f32x4_t np = {0.f, 0.f, 0.f, 0.f}, nm = {0.f, 0.f, 0.f, 0.f};
    update(s, np, nm);
    store_params(np, nullptr);
  }
}

// The block exchange of one gradient reduce: one-shot (every rank reads every peer's slice) or,
// for large buffers over many ranks, two-shot (P2PBlockArgs). MLAPI_DP_TWO_SHOT: 1 on, 0 off,
// default auto = world >= 4 and a gradient of >= 64 KiB; it needs the exchange buffer to hold the
// published [grad | params | momenta] behind the gradient slice (else one-shot).
P2PBlockArgs gdw_exchange(P2PAllReduce* dp, int width4, int nblocks, int timeout_ms, const Sgd2D* update) {
  const size_t grad_bytes = ((size_t)width4 * 4 + 4) * sizeof(float);
  const int64_t pub_off = ((int64_t)width4 * 4 + 4 + 3) / 4 * 4;  // floats; 16-byte aligned
  const bool mom = update != nullptr && update->mom != nullptr;
  const size_t two_bytes = (size_t)(pub_off + (int64_t)(mom ? 3 : 2) * width4 * 4) * sizeof(float);
  static const int mode = [] {
    const char* e = getenv("MLAPI_DP_TWO_SHOT");
    return e ? atoi(e) : -1;
  }();
  bool two = dp->world() > 1 && (mode == 1 || (mode < 0 && dp->world() >= 4 && grad_bytes >= (64u << 10)));
  if (two && two_bytes > dp->max_bytes()) two = false;
  P2PBlockArgs a = dp->block_exchange(two ? two_bytes : grad_bytes, nblocks, timeout_ms);
  a.two_shot = two ? 1 : 0;
  a.pub_off = pub_off;
  return a;
}

}  // namespace

void launch_gdw_reduce(const float* slabs, int nslabs, int K, int F_aug, float* dW_out, const float* stat_slabs,
                       int nstat, float* stats_out, const Sgd2D* update, P2PAllReduce* dp, int dp_timeout_ms,
                       hipStream_t stream) {
  if ((K * F_aug) % 4 != 0 || reinterpret_cast<uintptr_t>(dW_out) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(slabs) % 16 != 0)
    throw std::invalid_argument("gdw_reduce: K * F_aug must be a multiple of 4 and the buffers 16-byte aligned");
  const int width4 = K * F_aug / 4;
  const int nblocks = (width4 + 255) / 256 + 1;
  if (dp != nullptr) {
    const P2PBlockArgs a = gdw_exchange(dp, width4, nblocks, dp_timeout_ms, update);
    hipLaunchKernelGGL(gdw_reduce_kernel<true>, dim3((unsigned)nblocks), dim3(256), 0, stream,
                       reinterpret_cast<const f32x4_t*>(slabs), nslabs, width4, reinterpret_cast<f32x4_t*>(dW_out),
                       stat_slabs, nstat, stats_out, update != nullptr ? *update : Sgd2D{}, a);
  } else {
    hipLaunchKernelGGL(gdw_reduce_kernel<false>, dim3((unsigned)nblocks), dim3(256), 0, stream,
                       reinterpret_cast<const f32x4_t*>(slabs), nslabs, width4, reinterpret_cast<f32x4_t*>(dW_out),
                       stat_slabs, nstat, stats_out, update != nullptr ? *update : Sgd2D{}, P2PBlockArgs{});
  }
  MLAPI_HIP_CHECK(hipGetLastError());
}

namespace {

struct GdwLayout {
  int nc, tiles, row_groups, tiles_per_group, class_groups;
  size_t rowstat_off, dw_off, stat_off, total;
};

int g_force_row_groups = 0;  // benchmark hooks (softmax_grad_dw_force_plan)
int g_force_nc = 0;

int auto_nc(int K, int F) {
  if (F >= 512) return 1;
  return g_force_nc > 0 ? g_force_nc : (K >= 256 ? 2 : 1);
}

GdwLayout gdw_layout(int64_t B, int K, int F, int nc) {
  GdwLayout L;
  L.nc = nc;
  L.tiles = (int)((B + ROWS - 1) / ROWS);
  const int classes = 4 * WAVE_CLASSES * nc;
  L.class_groups = (K + classes - 1) / classes;
  // resident blocks: 2 per CU at NC = 1, 1 at NC = 2 or F = 512 (unless the rows run out); every
  // row group gets >= 1 tile
  const int target = nc == 1 && F < 512 ? 512 : 256;
  int want = g_force_row_groups > 0 ? g_force_row_groups : (target + L.class_groups - 1) / L.class_groups;
  want = want < 1 ? 1 : (want > L.tiles ? L.tiles : want);
  L.tiles_per_group = (L.tiles + want - 1) / want;
  L.row_groups = (L.tiles + L.tiles_per_group - 1) / L.tiles_per_group;
  auto align = [](size_t v) { return (v + 255) & ~size_t(255); };
  L.rowstat_off = align(softmax_rowstats_workspace(B, K, F));
  L.dw_off = align(L.rowstat_off + (size_t)B * sizeof(float2));
  L.stat_off = align(L.dw_off + (size_t)L.row_groups * K * (F + 8) * sizeof(float));
  L.total = align(L.stat_off + (size_t)L.row_groups * L.class_groups * 2 * sizeof(float));
  return L;
}

}  // namespace

bool softmax_grad_dw_supported(int F) { return F == 128 || F == 256 || F == 512; }

void softmax_grad_dw_force_plan(int row_groups, int nc) {
  g_force_row_groups = row_groups;
  g_force_nc = nc;
}

size_t softmax_grad_dw_workspace(int64_t B, int K, int F) {  // enough for either class-tile plan
  const size_t a = gdw_layout(B, K, F, 1).total, b = gdw_layout(B, K, F, 2).total;
  return a > b ? a : b;
}

void launch_softmax_grad_dw(const void* X_aug, int64_t ldx, const void* W, const float* b, const int32_t* y,
                            int64_t B, int F, int K, int kind, float* dW_out, float* stats_out, void* workspace,
                            size_t ws_bytes, hipStream_t stream, const Sgd2D* update, P2PAllReduce* dp,
                            int dp_timeout_ms) {
  if (B <= 0) return;
  if (dp != nullptr && reinterpret_cast<uintptr_t>(dW_out) % 16 != 0)
    throw std::invalid_argument("softmax_grad_dw: the fused DP exchange needs a 16-byte aligned dW_out");
  if (update != nullptr && (update->params == nullptr || update->cols != F + 8 || update->pen_cols > F))
    throw std::invalid_argument("softmax_grad_dw: fused update needs params [K, F + 8]");
  if (!softmax_grad_dw_supported(F))
    throw std::invalid_argument("softmax_grad_dw: F must be 128, 256 or 512 (pad narrower features)");
  if (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("softmax_grad_dw: multiclass kinds only");
  if (ldx < F + 8 || ldx % 8 != 0)
    throw std::invalid_argument("softmax_grad_dw: X_aug row stride must be >= F + 8 and a multiple of 8");
  if (reinterpret_cast<uintptr_t>(X_aug) % 16 != 0 || reinterpret_cast<uintptr_t>(W) % 16 != 0)
    throw std::invalid_argument("softmax_grad_dw: X_aug and W must be 16-byte aligned");
  const GdwLayout L = gdw_layout(B, K, F, auto_nc(K, F));
  if (ws_bytes < L.total) throw std::invalid_argument("softmax_grad_dw: workspace too small (zero it once)");
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  float2* rowstat = reinterpret_cast<float2*>(ws + L.rowstat_off);
  launch_softmax_rowstats(X_aug, ldx, W, b, B, F, K, kind, rowstat, ws, L.rowstat_off, stream);
  GradDwArgs args{};
  args.X = static_cast<const uint16_t*>(X_aug);
  args.ldx = ldx;
  args.W = static_cast<const uint16_t*>(W);
  args.bias = b;
  args.y = y;
  args.rowstat = rowstat;
  args.B = B;
  args.K = K;
  args.tiles = L.tiles;
  args.tiles_per_group = L.tiles_per_group;
  args.row_groups = L.row_groups;
  args.class_groups = L.class_groups;
  args.ldw = F + 8;
  args.dw_slabs = reinterpret_cast<float*>(ws + L.dw_off);
  args.stat_slabs = reinterpret_cast<float*>(ws + L.stat_off);
  const dim3 grid((unsigned)(L.row_groups * L.class_groups));
  const bool ovr = kind == KIND_OVR;
  auto launch = [&](auto ks, auto nc) {
    constexpr int KS_ = decltype(ks)::value, NC_ = decltype(nc)::value;
    if (ovr)
      hipLaunchKernelGGL((softmax_grad_dw_kernel<KS_, true, NC_>), grid, dim3(256), 0, stream, args);
    else
      hipLaunchKernelGGL((softmax_grad_dw_kernel<KS_, false, NC_>), grid, dim3(256), 0, stream, args);
  };
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  using I16 = std::integral_constant<int, 16>;
  using N1 = std::integral_constant<int, 1>;
  using N2 = std::integral_constant<int, 2>;
  if (F == 128)
    L.nc == 1 ? launch(I4{}, N1{}) : launch(I4{}, N2{});
  else if (F == 256)
    L.nc == 1 ? launch(I8{}, N1{}) : launch(I8{}, N2{});
  else
    launch(I16{}, N1{});
  MLAPI_HIP_CHECK(hipGetLastError());
  if (reinterpret_cast<uintptr_t>(dW_out) % 16 == 0) {
    const int width4 = K * (F + 8) / 4;
    const int nblocks = (width4 + 255) / 256 + 1;
    if (dp != nullptr) {
      const P2PBlockArgs a = gdw_exchange(dp, width4, nblocks, dp_timeout_ms, update);
      hipLaunchKernelGGL(gdw_reduce_kernel<true>, dim3((unsigned)nblocks), dim3(256), 0, stream,
                         reinterpret_cast<const f32x4_t*>(args.dw_slabs), L.row_groups, width4,
                         reinterpret_cast<f32x4_t*>(dW_out), args.stat_slabs, L.row_groups * L.class_groups, stats_out,
                         update != nullptr ? *update : Sgd2D{}, a);
    } else {
      hipLaunchKernelGGL(gdw_reduce_kernel<false>, dim3((unsigned)nblocks), dim3(256), 0, stream,
                         reinterpret_cast<const f32x4_t*>(args.dw_slabs), L.row_groups, width4,
                         reinterpret_cast<f32x4_t*>(dW_out), args.stat_slabs, L.row_groups * L.class_groups, stats_out,
                         update != nullptr ? *update : Sgd2D{}, P2PBlockArgs{});
    }
    MLAPI_HIP_CHECK(hipGetLastError());
  } else {
    launch_reduce_slabs_f32(args.dw_slabs, L.row_groups, K * (F + 8), dW_out, stream);
    launch_reduce_slabs_f32(args.stat_slabs, L.row_groups * L.class_groups, 2, stats_out, stream);
    if (update != nullptr)
      launch_sgd_update_2d(update->params, dW_out, update->mom, K, update->cols, update->pen_cols, update->lr,
                           update->inv_n, update->l2, update->momentum, update->shadow_w, update->shadow_b, stream);
  }
}

}  // namespace mlapi
