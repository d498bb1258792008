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
//   2. gdw_gemm_big_kernel: dW slabs[row group][K][F_aug] = G^T X_aug over the group's rows -
//      v_mfma_f32_16x16x32_bf16 with M = classes, N = features, K = rows: both operands are
//      row-major [rows][*] tiles, so each is staged in LDS (32 rows x 128 columns, 16-byte loads)
//      and read transposed with ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group, two
//      reads = the 8 rows of a lane's k-slice);
//   3. launch_gdw_reduce: deterministic slab sum + fused SGD update (+ in-kernel DP exchange).
// (Round 3's five launches - row stats, f32 logits through HBM, a wave-per-row G pass - lost to
// this path: 1.79 -> 1.0 ms per step at F = 1024, docs/PERFORMANCE.md; removed in round 5.)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <stdexcept>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 wbf16x8_t;
typedef __attribute__((ext_vector_type(4))) short wi16x4_t;
typedef __attribute__((ext_vector_type(4))) float wf32x4_t;
typedef __attribute__((address_space(3))) wi16x4_t lds_i16x4_t;

constexpr int TILE_ROWS = 32;        // MFMA k-step (rows)


// ---- 4. dW slabs = G^T X_aug per row group, (64 WC) x 128 block tiles: a wave owns 64 classes x
// 64 features (4 x 4 MFMA tiles, 64 accumulator VGPRs), the block 2 WC waves, so each 16-byte
// element staged through LDS feeds 2-4x the MFMAs of round 3's 64 x 64 tiles (514 -> 357 us at
// F = 1024; that kernel left the build in round 5) and G / X are re-read from L2 correspondingly
// less often. LDS double buffered (one barrier per 32-row k-step). WC = 2 (128 x 128 tiles, 256
// threads) is the one launched: WC = 4 (256 x 128, 512 threads) measured 1.05 vs 0.99 ms per
// F = 1024 training step (profiles/r4_train/tsm_f1024_t256_*).
// Rows padded by 8 elements. The counters show 1.6 LDS bank conflicts per LDS instruction
// (profiles/r5_pmc/summary_big.md); padding rows to 16 elements instead (8 banks per row) left both
// the count (1.600) and the F = 1024 step (0.971 vs 0.972 ms, interleaved x3) unchanged
// (profiles/r5_train/s37_*), so the conflicts are not the row stride's and not on the critical path.
constexpr int TF128 = 128;
constexpr int LDS_PAD = 8;
constexpr int XROW = TF128 + LDS_PAD;

template <int WC>
__global__ __launch_bounds__(128 * WC) void gdw_gemm_big_kernel(const uint16_t* __restrict__ G, int Kp,
                                                               const uint16_t* __restrict__ X, int64_t ldx, int F_aug,
                                                               int64_t B, int K, int64_t rows_per_group,
                                                               float* __restrict__ slabs, int xcd_tiles,
                                                               int row_groups) {
  constexpr int TC = 64 * WC, NTHR = 128 * WC, GROW = TC + LDS_PAD;
  constexpr int JX = 512 / NTHR;  // X chunks per thread (32 rows x 16 chunks of 8 columns)
  static_assert(32 * TC / 8 == 2 * NTHR, "two G chunks per thread");
  __shared__ __attribute__((aligned(16))) uint16_t gt[2][TILE_ROWS][GROW];
  __shared__ __attribute__((aligned(16))) uint16_t xt[2][TILE_ROWS][XROW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wc = wave % WC, wf = wave / WC;  // the wave's 64-class slice / 64-feature half
  // xcd_tiles > 0: a 1-D grid dealt over the 8 XCDs round-robin (block b runs on XCD b % 8, as the
  // dispatcher deals them; a placement hint only, nothing depends on it for correctness): XCD x
  // takes row groups x, x + 8, ..., each as its xcd_tiles = (class tiles x feature tiles) blocks in
  // a row, so an XCD's L2 holds the G and X rows of ITS row groups - every tile of a row group
  // re-reads them there - instead of every XCD streaming all of X (the 3-D grid put class tile x
  // on XCD x: X came from the infinity cache / HBM 8 times)
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (xcd_tiles > 0) {
    const int j = (int)blockIdx.x >> 3;
    bz = ((int)blockIdx.x & 7) + 8 * (j / xcd_tiles);
    if (bz >= row_groups) return;  // the grid's padding to whole rounds of 8 (uniform per block)
    const int tile = j % xcd_tiles, ncb = Kp / TC;
    bx = tile % ncb;
    by = tile / ncb;
  }
  const int c0 = bx * TC, f0 = by * TF128;
  const int64_t r_begin = (int64_t)bz * rows_per_group;
  const int64_t r_end = min(B, r_begin + rows_per_group);
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto load_tile = [&](int64_t r0, uint4 (&gv)[2], uint4 (&xv)[JX]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = (int)threadIdx.x + NTHR * j, sr = k / (TC / 8), sc = (k % (TC / 8)) * 8;
      const int64_t r = r0 + sr;
      gv[j] = r < r_end ? *reinterpret_cast<const uint4*>(G + r * Kp + c0 + sc) : uint4{0, 0, 0, 0};  // Kp % TC == 0
    }
#pragma unroll
    for (int j = 0; j < JX; ++j) {
      const int k = (int)threadIdx.x + NTHR * j, sr = k >> 4, sc = (k & 15) * 8;
      const int64_t r = r0 + sr;
      xv[j] = uint4{0, 0, 0, 0};
      if (r < r_end) {
        if (f0 + sc + 8 <= ldx) {
          xv[j] = *reinterpret_cast<const uint4*>(X + r * ldx + f0 + sc);
        } else {
          uint16_t tmp[8];
          for (int e = 0; e < 8; ++e) tmp[e] = f0 + sc + e < ldx ? X[r * ldx + f0 + sc + e] : 0;
          __builtin_memcpy(&xv[j], tmp, sizeof(uint4));
        }
      }
    }
  };
  auto store_tile = [&](int buf, const uint4 (&gv)[2], const uint4 (&xv)[JX]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = (int)threadIdx.x + NTHR * j, sr = k / (TC / 8), sc = (k % (TC / 8)) * 8;
      *reinterpret_cast<uint4*>(&gt[buf][sr][sc]) = gv[j];
    }
#pragma unroll
    for (int j = 0; j < JX; ++j) {
      const int k = (int)threadIdx.x + NTHR * j, sr = k >> 4, sc = (k & 15) * 8;
      *reinterpret_cast<uint4*>(&xt[buf][sr][sc]) = xv[j];
    }
  };
  wf32x4_t acc[4][4] = {};
  auto mma_step = [&](int buf) {
    wbf16x8_t a[4], b[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // A: 16 classes x 8 rows per 16-lane group (transposed reads)
      const int cc = wc * 64 + m * 16 + 4 * p;
      const wi16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)&gt[buf][8 * g + q][cc]);
      const wi16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)&gt[buf][8 * g + 4 + q][cc]);
      const wi16x4_t v[2] = {lo, hi};
      a[m] = __builtin_bit_cast(wbf16x8_t, v);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int ff = wf * 64 + n * 16 + 4 * p;
      const wi16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)&xt[buf][8 * g + q][ff]);
      const wi16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)&xt[buf][8 * g + 4 + q][ff]);
      const wi16x4_t v[2] = {lo, hi};
      b[n] = __builtin_bit_cast(wbf16x8_t, v);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b[n], acc[m][n], 0, 0, 0);
  };
  // one k-step of loads in flight. Two (a second register set: tile t + 2 loading while t + 1 waits)
  // took the kernel from 140 to 236 VGPRs, 3 to 2 blocks per CU, and the F = 1024 step from 0.915 to
  // 1.13 ms (profiles/r5_train/s42_depth/): the resident blocks' overlap hides more than the depth
  uint4 gv[2], xv[JX];
  load_tile(r_begin, gv, xv);
  store_tile(0, gv, xv);
  __syncthreads();
  int buf = 0;
  for (int64_t r0 = r_begin; r0 < r_end; r0 += TILE_ROWS) {
    const bool more = r0 + TILE_ROWS < r_end;
    if (more) load_tile(r0 + TILE_ROWS, gv, xv);  // in flight under this step's MFMAs
    mma_step(buf);
    if (more) store_tile(buf ^ 1, gv, xv);  // the other buffer was last read before the previous barrier
    __syncthreads();
    buf ^= 1;
  }
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

// the G^T X launch's XCD-aware block order (gdw_gemm_big_kernel); MLAPI_GDW_XCD=0: the 3-D grid
bool gdw_xcd_on() {
  static const bool on = [] {
    const char* e = std::getenv("MLAPI_GDW_XCD");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}

struct WideLayout {
  size_t g_off, dw_off, stat_off, z_off, total;
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
  int64_t rg = (2048 + tiles - 1) / tiles;
  if (gdw_xcd_on()) rg = (rg + 7) / 8 * 8;  // whole rounds of row groups over the 8 XCDs
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
  L.z_off = o;  // the row-stats pass's logits, [B][Kp] f32 (zbuf_on())
  o = al(o + (size_t)B * L.Kp * sizeof(float));
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
  if (ldx != F + 8) throw std::invalid_argument("softmax_grad_wide: X_aug row stride must be F + 8");
  if (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("softmax_grad_wide: multiclass kinds only");
  if (update != nullptr && (update->params == nullptr || update->cols != F + 8 || update->pen_cols > F))
    throw std::invalid_argument("softmax_grad_wide: fused update needs params [K, F + 8]");
  if (reinterpret_cast<uintptr_t>(X_aug) % 16 != 0 || reinterpret_cast<uintptr_t>(W) % 16 != 0)
    throw std::invalid_argument("softmax_grad_wide: X_aug and W must be 16-byte aligned");
  const WideLayout L = wide_layout(B, K, F);
  if (ws_bytes < L.total) throw std::invalid_argument("softmax_grad_wide: workspace too small");
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  uint16_t* G = reinterpret_cast<uint16_t*>(ws + L.g_off);
  float* slabs = reinterpret_cast<float*>(ws + L.dw_off);
  float* stat_slabs = reinterpret_cast<float*>(ws + L.stat_off);
  float* Zs = zbuf_on() ? reinterpret_cast<float*>(ws + L.z_off) : nullptr;
  launch_softmax_rows_g(X_aug, ldx, W, b, y, B, F, K, kind, G, L.Kp, stat_slabs, Zs, stream);
  const int g_blocks = L.g_blocks;
  const int F_aug = F + 8;
  const int ncb = L.Kp / 128, nfb = (F_aug + TF128 - 1) / TF128;
  if (gdw_xcd_on()) {
    const int rounds = (L.row_groups + 7) / 8;
    hipLaunchKernelGGL((gdw_gemm_big_kernel<2>), dim3((unsigned)(8 * ncb * nfb * rounds)), dim3(256), 0, stream, G,
                       L.Kp, static_cast<const uint16_t*>(X_aug), ldx, F_aug, B, K, L.rows_per_group, slabs, ncb * nfb,
                       L.row_groups);
  } else {
    hipLaunchKernelGGL((gdw_gemm_big_kernel<2>), dim3((unsigned)ncb, (unsigned)nfb, (unsigned)L.row_groups), dim3(256),
                       0, stream, G, L.Kp, static_cast<const uint16_t*>(X_aug), ldx, F_aug, B, K, L.rows_per_group,
                       slabs, 0, L.row_groups);
  }
  MLAPI_HIP_CHECK(hipGetLastError());
  launch_gdw_reduce(slabs, L.row_groups, K, F_aug, dW_out, stat_slabs, g_blocks, stats_out, update, dp,
                    dp_timeout_ms, stream);
}

}  // namespace mlapi
