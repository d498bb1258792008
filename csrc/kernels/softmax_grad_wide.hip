// Multiclass training gradient for wide models (F > 512) on ONE GPU (reference:
// LogisticRegression.fit on any F, `Logistic Regression.ipynb:33-34`).
//
// The fused kernel (softmax_grad_dw.hip) keeps a 64-row X tile and a wave's 16 W rows in LDS /
// registers for the whole F, which stops at F = 512. Beyond it the step is three launches, all
// hand-written (no vendor GEMM):
//   1. softmax_rows_kernel MODE 5 (gemm_softmax.hip): a block owns 16-64 rows and ALL classes -
//      the row stats {lse, argmax} over the class chunks (each lane storing its f32 logits in the
//      workspace), then (lse held in LDS) the same lanes read their logits back, chunk by chunk,
//      into G = softmax(z) - onehot(y) (OvR: sigmoid(z) - onehot) as bf16 [B][Kp] (Kp = K rounded
//      up to 128, zero padded) plus the block's {loss, correct} - a write + read of the logits
//      instead of a second GEMM over X (F = 1024: 0.914 -> 0.764 ms per step, profiles/r5_train/);
//   2. gdw_gemm_dma_kernel: dW slabs[row group][K][F_aug] = G^T X_aug over the group's rows -
//      v_mfma_f32_16x16x32_bf16 with M = classes, N = features, K = rows: both operands are
//      row-major [rows][*] tiles, DMA'd into LDS (32 rows x 128 columns per k-step, 3 stages)
//      and read transposed with ds_read_b64_tr_b16;
//   3. launch_gdw_reduce: deterministic slab sum + fused SGD update (+ in-kernel DP exchange).
// (Round 3's five launches - row stats, f32 logits through HBM, a wave-per-row G pass - lost to
// this path: 1.79 -> 1.0 ms per step at F = 1024, docs/PERFORMANCE.md; removed in round 5.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 wbf16x8_t;
typedef __attribute__((ext_vector_type(4))) short wi16x4_t;
typedef __attribute__((ext_vector_type(4))) float wf32x4_t;
typedef __attribute__((address_space(3))) wi16x4_t lds_i16x4_t;
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int TILE_ROWS = 32;        // MFMA k-step (rows)


// ---- 2. dW slabs = G^T X_aug per row group, 128 x 128 block tiles: a wave owns 64 classes x 64
// features (4 x 4 tiles of v_mfma_f32_16x16x32_bf16, 64 accumulators); M = classes, N = features,
// K = rows, and both operands are row-major [rows][*] tiles, read transposed from LDS with
// ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group, two reads = a lane's 8-row k-slice).
// The tiles arrive by LDS-DMA (`buffer_load_dwordx4 ... lds`), NS stages deep: NS - 1 k-steps
// stream into LDS while the MFMAs read the oldest. Round 4's kernel staged them through registers
// with one k-step in flight (a second cost registers and a resident block, profiles/r5_train/s42)
// and its waves waited on memory 68 % of their cycles at 19 % MFMA busy (s54); F = 1024 step 0.737
// -> 0.612 ms (s55). A stage is the k-step's G and X tiles, 32 rows x 128 columns
// bf16 each, rows unpadded (the DMA writes 1 KB per wave-instruction, lane-linear); the 16-byte
// chunks of row r sit XOR-permuted by s(r) = 2 (r & 3) + 8 ((r >> 3) & 1), so the transposed reads
// (rows 8g + q (+4), two adjacent chunks per 16-column subtile) touch 64 distinct banks per
// 32-lane group. The source is read through range-checked buffer descriptors: rows past B load 0.
constexpr int TF128 = 128;
constexpr int DMA_ROW_BYTES = TF128 * 2;                 // 256 B: a 128-column bf16 row
constexpr int DMA_TILE_BYTES = TILE_ROWS * DMA_ROW_BYTES;  // 8 KB
__device__ __forceinline__ int dma_swz(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

template <int NS>
__global__ __launch_bounds__(256) void gdw_gemm_dma_kernel(const uint16_t* __restrict__ G, int Kp,
                                                           const uint16_t* __restrict__ X, int64_t ldx, int F_aug,
                                                           int64_t B, int K, int64_t rows_per_group,
                                                           float* __restrict__ slabs, int xcd_tiles,
                                                           int row_groups) {
  constexpr int TC = 128;
  __shared__ __attribute__((aligned(1024))) unsigned char sm[NS][2][DMA_TILE_BYTES];  // [stage][G, X]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wc = wave & 1, wf = wave >> 1;
  int bx, by, bz;
  // a 1-D grid dealt over the 8 XCDs round-robin (block b runs on XCD b % 8, as the dispatcher
  // deals them; a placement hint only, nothing depends on it for correctness): XCD x takes row
  // groups x, x + 8, ..., each as its xcd_tiles = (class tiles x feature tiles) blocks in a row, so
  // an XCD's L2 holds the G and X rows of ITS row groups - every tile of a row group re-reads them
  // there - instead of every XCD streaming all of X (a 3-D grid put class tile x on XCD x: X came
  // from the infinity cache / HBM 8 times; F = 1024 step 0.765 -> 0.737 ms, s52)
  {
    const int j = (int)blockIdx.x >> 3;
    bz = ((int)blockIdx.x & 7) + 8 * (j / xcd_tiles);
    if (bz >= row_groups) return;
    const int tile = j % xcd_tiles, ncb = Kp / TC;
    bx = tile % ncb;
    by = tile / ncb;
  }
  const int c0 = bx * TC, f0 = by * TF128;
  const int64_t r_begin = (int64_t)bz * rows_per_group;
  const int64_t r_end = min(B, r_begin + rows_per_group);
  const int nk = (int)((r_end - r_begin + TILE_ROWS - 1) / TILE_ROWS);
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  // the row group's own descriptors: they end at its last row (the tail k-step's rows past B read
  // as zeros) and keep every offset within 32 bits (wide_layout caps a group's bytes)
  const int64_t nrows = r_end - r_begin;
  const auto grs = __builtin_amdgcn_make_buffer_rsrc((void*)(G + r_begin * Kp), 0, (int)(nrows * Kp * 2), 0x00020000);
  const auto xrs = __builtin_amdgcn_make_buffer_rsrc((void*)(X + r_begin * ldx), 0, (int)(nrows * ldx * 2), 0x00020000);
  // this lane's DMA pieces: wave-instruction j of a tile covers rows 4 (2 wave + j) .. + 3, lane l
  // writes the 16 bytes at chunk position l & 15 of row + (l >> 4), which holds logical chunk
  // (l & 15) ^ s(row)
  uint32_t goff[2], xoff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 4 * (2 * wave + j) + (lane >> 4);
    const int ch = (lane & 15) ^ dma_swz(r);
    goff[j] = (uint32_t)(((int64_t)r * Kp + c0 + ch * 8) * 2);
    xoff[j] = (uint32_t)(((int64_t)r * ldx + f0 + ch * 8) * 2);
  }
  const uint32_t gstep = (uint32_t)(TILE_ROWS * Kp * 2), xstep = (uint32_t)(TILE_ROWS * ldx * 2);
  auto dma = [&](int k, int st) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(grs, (lds_void_t*)(&sm[st][0][(2 * wave + j) * 1024]), 16,
                                               goff[j] + (uint32_t)k * gstep, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void_t*)(&sm[st][1][(2 * wave + j) * 1024]), 16,
                                               xoff[j] + (uint32_t)k * xstep, 0, 0, 0);
    }
  };
  // this lane's transposed-read byte offsets within a tile: rows 8g + q (lo) / + 4 (hi), 4 columns
  // at 16m + 4p of its 64-column half (chunk 2m + (p >> 1) of the half, byte 8 (p & 1))
  uint32_t rdo[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = 8 * g + 4 * h + q;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int ch = (8 * 0 + 2 * m + (p >> 1)) ^ dma_swz(r);  // half offset added per operand below
      rdo[h][m] = (uint32_t)(r * DMA_ROW_BYTES + ch * 16 + (p & 1) * 8);
    }
  }
  wf32x4_t acc[4][4] = {};
  // The transposed reads go through inline asm: the compiler cannot tell the intrinsic's LDS read
  // from the DMA stages still in flight and drained them all (vmcnt(0)) before every read; one
  // lgkmcnt(0) that passes the 16 results through is the reads' only wait.
  const uint32_t sm0 = (uint32_t)(uintptr_t)(lds_void_t*)&sm[0][0][0];
  auto mma_step = [&](int st) {
    const uint32_t gt = sm0 + (uint32_t)(st * 2 * DMA_TILE_BYTES), xt = gt + DMA_TILE_BYTES;
    wi16x4_t r[16];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int h = 0; h < 2; ++h)  // the half's chunks are 8 higher: XOR with s(r) < 16 keeps bit 3
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r[2 * m + h]) : "v"(gt + (rdo[h][m] ^ (wc << 7))));
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r[8 + 2 * n + h]) : "v"(xt + (rdo[h][n] ^ (wf << 7))));
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]),
                   "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]));
    wbf16x8_t a[4], b[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const wi16x4_t v[2] = {r[2 * m], r[2 * m + 1]};
      a[m] = __builtin_bit_cast(wbf16x8_t, v);
      const wi16x4_t w[2] = {r[8 + 2 * m], r[8 + 2 * m + 1]};
      b[m] = __builtin_bit_cast(wbf16x8_t, w);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b[n], acc[m][n], 0, 0, 0);
  };
#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0) dma(min(s0, nk - 1), s0);
  // unrolled by the stages, so every stage index is a constant: with a run-time stage the compiler
  // cannot tell the DMA's LDS target from the stage being read and drains every DMA (vmcnt(0))
  // before the reads
  auto step = [&](int k, auto stc) {
    constexpr int st = decltype(stc)::value;
    // this wave's pieces of step k have landed (NS - 2 later steps may still be in flight: 4 DMA
    // instructions per step and wave, completed in order) ...
    __builtin_amdgcn_s_waitcnt((NS - 2) * 4 == 0 ? ((7 << 4) | (15 << 8)) : (((NS - 2) * 4) | (7 << 4) | (15 << 8)));
    // ... and every other wave's; past this barrier no wave reads step k - 1's stage any more
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    dma(min(k + NS - 1, nk - 1), (st + NS - 1) % NS);  // the tail re-reads the last step into a free stage
    mma_step(st);
  };
  for (int k = 0; k < nk; k += NS) {
    step(k, std::integral_constant<int, 0>{});
    if (k + 1 < nk) step(k + 1, std::integral_constant<int, 1 % NS>{});
    if constexpr (NS > 2)
      if (k + 2 < nk) step(k + 2, std::integral_constant<int, 2 % NS>{});
    if constexpr (NS > 3)
      if (k + 3 < nk) step(k + 3, std::integral_constant<int, 3 % NS>{});
  }
  __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));  // drain the tail's DMAs before the block exits
  // C layout: class c0 + wc*64 + 16m + 4g + i (register i), feature f0 + wf*64 + 16n + (lane & 15)
  float* slab = slabs + (int64_t)bz * K * F_aug;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int f = f0 + wf * 64 + n * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = c0 + wc * 64 + m * 16 + 4 * g + i;
        if (c < K && f < F_aug) slab[(int64_t)c * F_aug + f] = acc[m][n][i];
      }
    }
}

struct WideLayout {
  size_t g_off, dw_off, stat_off, z_off, wp_off, total;
  int Kp, row_groups, g_blocks;
  int64_t rows_per_group;
};

WideLayout wide_layout(int64_t B, int K, int F) {
  WideLayout L{};
  const int F_aug = F + 8;
  const int T = 128;  // G's columns padded to the class tile
  L.Kp = (K + T - 1) / T * T;
  const int TFw = TF128;  // feature tile width
  const int tiles = (L.Kp / T) * ((F_aug + TFw - 1) / TFw);
  // ~1024 G^T X blocks (row groups x tiles): each row group adds a K x F_aug slab to the reduce.
  // F = 1024, K = 1000 (72 tiles): 16 row groups 0.595 ms per step, 8: 0.605, 24: 0.597, 32: 0.613,
  // 48: 0.642 (profiles/r5_train/s61, s62). MLAPI_GDW_TARGET overrides (measurement).
  static const int target = [] {
    const char* e = std::getenv("MLAPI_GDW_TARGET");
    return e != nullptr ? std::atoi(e) : 1024;
  }();
  int64_t rg = (target + tiles - 1) / tiles;
  // a group's G / X bytes stay below 2^31 (the G^T X kernel's buffer offsets are 32-bit)
  // (X rows may be padded to a 64-element multiple: augment_features on the wide path)
  const int64_t cap_rows =
      ((int64_t)INT32_MAX / (2 * std::max<int64_t>(L.Kp, (F_aug + 63) / 64 * 64))) / TILE_ROWS * TILE_ROWS;
  rg = std::max<int64_t>(rg, (B + cap_rows - 1) / cap_rows);
  rg = (rg + 7) / 8 * 8;  // whole rounds of row groups over the 8 XCDs
  const int64_t max_rg = (B + 255) / 256;
  if (rg > max_rg) rg = max_rg;
  if (rg < 1) rg = 1;
  L.rows_per_group = ((B + rg - 1) / rg + TILE_ROWS - 1) / TILE_ROWS * TILE_ROWS;
  L.row_groups = (int)((B + L.rows_per_group - 1) / L.rows_per_group);
  L.g_blocks = softmax_rows_g_blocks(B, F, K);  // the row-stats launch's {loss, correct} slabs
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  size_t o = 0;
  L.g_off = o;
  o = al(o + (size_t)B * L.Kp * sizeof(uint16_t));
  L.dw_off = o;
  o = al(o + (size_t)L.row_groups * K * F_aug * sizeof(float));
  L.stat_off = o;
  o = al(o + (size_t)L.g_blocks * 2 * sizeof(float));
  L.z_off = o;  // the row-stats pass's logits, [B][Kp] f32 (zbuf_on(), unless the kernel keeps them in registers)
  if (!softmax_rows_g_keeps_logits(B, F, K, L.Kp)) o = al(o + (size_t)B * L.Kp * sizeof(float));
  L.wp_off = o;  // W in MFMA-fragment order for the register-resident G kernel (0 bytes when it does not run)
  o = al(o + softmax_rows_g_wpack_bytes(B, F, K, L.Kp));
  L.total = o;
  return L;
}

int g_zbuf = -1;  // softmax_grad_wide_set_zbuf: -1 MLAPI_WIDE_ZBUF (default on), 0 off, 1 on

// The first launch keeps its logits in the workspace for its second pass (off: recomputes them, a
// second GEMM over X instead of a B x Kp f32 write + read)
bool zbuf_on() {
  static const bool env = [] {
    const char* e = std::getenv("MLAPI_WIDE_ZBUF");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return g_zbuf < 0 ? env : g_zbuf != 0;
}

}  // namespace

void softmax_grad_wide_set_zbuf(int mode) { g_zbuf = mode; }

bool softmax_grad_wide_supported(int F) { return F > 512 && F % 256 == 0; }

size_t softmax_grad_wide_workspace(int64_t B, int K, int F) { return wide_layout(B, K, F).total; }

void launch_softmax_grad_wide(const void* X_aug, int64_t ldx, const void* W, const float* b, const int32_t* y,
                              int64_t B, int F, int K, int kind, float* dW_out, float* stats_out, void* workspace,
                              size_t ws_bytes, hipStream_t stream, const Sgd2D* update, P2PAllReduce* dp,
                              int dp_timeout_ms) {
  if (B <= 0) return;
  if (!softmax_grad_wide_supported(F)) throw std::invalid_argument("softmax_grad_wide: F must be a multiple of 256 above 512");
  if (ldx < F + 8 || ldx % 8 != 0)
    throw std::invalid_argument("softmax_grad_wide: X_aug row stride must be >= F + 8 and a multiple of 8");
  if (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("softmax_grad_wide: multiclass kinds only");
  if (update != nullptr && (update->params == nullptr || update->cols != F + 8 || update->pen_cols > F))
    throw std::invalid_argument("softmax_grad_wide: fused update needs params [K, F + 8]");
  if (reinterpret_cast<uintptr_t>(X_aug) % 16 != 0 || reinterpret_cast<uintptr_t>(W) % 16 != 0)
    throw std::invalid_argument("softmax_grad_wide: X_aug and W must be 16-byte aligned");
  const WideLayout L = wide_layout(B, K, F);
  if (ws_bytes < L.total) throw std::invalid_argument("softmax_grad_wide: workspace too small");
  if (L.rows_per_group * ldx * 2 > (int64_t)INT32_MAX)
    throw std::invalid_argument("softmax_grad_wide: X_aug row stride too large for a row group's 32-bit offsets");
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  uint16_t* G = reinterpret_cast<uint16_t*>(ws + L.g_off);
  float* slabs = reinterpret_cast<float*>(ws + L.dw_off);
  float* stat_slabs = reinterpret_cast<float*>(ws + L.stat_off);
  float* Zs = zbuf_on() && !softmax_rows_g_keeps_logits(B, F, K, L.Kp) ? reinterpret_cast<float*>(ws + L.z_off) : nullptr;
  void* wp = softmax_rows_g_wpack_bytes(B, F, K, L.Kp) ? static_cast<void*>(ws + L.wp_off) : nullptr;
  launch_softmax_rows_g(X_aug, ldx, W, b, y, B, F, K, kind, G, L.Kp, stat_slabs, Zs, wp, stream);
  const int g_blocks = L.g_blocks;
  const int F_aug = F + 8;
  const int ncb = L.Kp / 128, nfb = (F_aug + TF128 - 1) / TF128;
  const int rounds = (L.row_groups + 7) / 8;
  hipLaunchKernelGGL((gdw_gemm_dma_kernel<3>), dim3((unsigned)(8 * ncb * nfb * rounds)), dim3(256), 0, stream, G, L.Kp,
                     static_cast<const uint16_t*>(X_aug), ldx, F_aug, B, K, L.rows_per_group, slabs, ncb * nfb,
                     L.row_groups);
  MLAPI_HIP_CHECK(hipGetLastError());
  launch_gdw_reduce(slabs, L.row_groups, K, F_aug, dW_out, stat_slabs, g_blocks, stats_out, update, dp,
                    dp_timeout_ms, stream);
}

}  // namespace mlapi
