// Multiclass (softmax / OvR) logistic-regression predict:  Z = X W^T + b  ->  argmax, p_max
// (BASELINE config 3: B=1024, F=256, K=1000 bf16; reference ops K1+K2+K4+K5).
//
// MFMA layout (v_mfma_f32_16x16x32_bf16, cdna_hip_programming.md S3): the class dimension is the
// MFMA "M" (A operand = W rows) and the batch row is "N" (B operand = X rows), so the C/D tile
// puts ONE batch row on each lane (col = lane & 15) and 4 classes in its registers
// (row = (lane >> 4) * 4 + reg). The softmax reduction over classes is then lane-local: each lane
// keeps an online (max, sum-exp, argmax) state over the classes it owns and the 4 lanes that
// share a batch row merge once at the very end (2 xor-shuffles) - no LDS, no per-tile shuffles.
//
// Work split: a 256-thread block = 4 waves x 32 batch rows (2 N-tiles). Each wave keeps its X
// fragments for the whole F in registers (F=256: 64 VGPRs) and streams W fragments (L2-resident,
// 500 KiB at K=1000) for 64 classes (4 M-tiles) per chunk. For small batches (B=1024 -> only 8
// row-blocks) the class range is split over gridDim.y so the launch still fills the chip; each
// split writes a partial (max, sum, argmax) per row and a tiny merge kernel combines them in
// split order (deterministic). For large B there is one split and no merge.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

constexpr int ROWS_PER_WAVE = 32;
constexpr int ROWS_PER_BLOCK = 4 * ROWS_PER_WAVE;
constexpr int CLASS_CHUNK = 64;

struct RowState {
  float m;   // running max logit (-inf if nothing seen yet)
  float s;   // softmax: sum exp(z - m);  OvR: sum sigmoid(z)
  int bi;    // argmax class (first max wins)
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
  RowState r;
  r.m = __shfl_xor(a.m, off, 64);
  r.s = __shfl_xor(a.s, off, 64);
  r.bi = __shfl_xor(a.bi, off, 64);
  return r;
}

// MODE 0: fused argmax/p_max epilogue (partials when gridDim.y > 1). MODE 1: write logits Z.
template <int KS, int MODE>
__global__ __launch_bounds__(256) void gemm_softmax_kernel(const uint16_t* __restrict__ X,
                                                           const uint16_t* __restrict__ W,
                                                           const float* __restrict__ bias, int64_t B, int F, int K,
                                                           int kind, int classes_per_split,
                                                           int32_t* __restrict__ out_idx, float* __restrict__ out_p,
                                                           float4* __restrict__ partials, float* __restrict__ Z) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4;   // k-group of the operand fragments / class quad of the C tile
  const int col = lane & 15;
  const int ksr = F / 32;    // runtime k-steps (<= KS)
  const bool ovr = kind == KIND_OVR;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS_PER_BLOCK + wave * ROWS_PER_WAVE;
  const int c_begin = blockIdx.y * classes_per_split;
  const int c_end = min(K, c_begin + classes_per_split);

  // X fragments for the whole feature range stay in registers.
  bf16x8_t xf[2][KS];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    int64_t r = row0 + t * 16 + col;
    r = r < B ? r : B - 1;
    const uint16_t* xr = X + r * F + 8 * q;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      xf[t][ks] = ks < ksr ? *reinterpret_cast<const bf16x8_t*>(xr + ks * 32) : bf16x8_t{};
  }

  RowState st[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) st[t] = RowState{-INFINITY, 0.f, 0x7fffffff};

  for (int c0 = c_begin; c0 < c_end; c0 += CLASS_CHUNK) {
    f32x4_t acc[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[t][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const uint16_t* wrow[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      int cls = c0 + mt * 16 + col;
      cls = cls < K ? cls : K - 1;
      wrow[mt] = W + (int64_t)cls * F + 8 * q;
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks < ksr) {
        bf16x8_t wf[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) wf[mt] = *reinterpret_cast<const bf16x8_t*>(wrow[mt] + ks * 32);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[mt], xf[t][ks], acc[t][mt], 0, 0, 0);
      }
    }

    // Epilogue for this chunk: lane owns classes c0 + mt*16 + q*4 + reg of batch row (t, col).
    float bv[4][4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cls = c0 + mt * 16 + q * 4 + r;
        bv[mt][r] = cls < c_end ? bias[cls] : 0.f;
      }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if constexpr (MODE == 1) {
        const int64_t row = row0 + t * 16 + col;
        if (row < B) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int cls = c0 + mt * 16 + q * 4 + r;
              if (cls < c_end) Z[row * K + cls] = acc[t][mt][r] + bv[mt][r];
            }
        }
      } else {
        float cm = -INFINITY;
        int ci = 0x7fffffff;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int cls = c0 + mt * 16 + q * 4 + r;
            const float v = acc[t][mt][r] + bv[mt][r];
            if (cls < c_end && v > cm) { cm = v; ci = cls; }
          }
        RowState& S = st[t];
        if (cm > S.m) {
          if (!ovr) S.s = S.m == -INFINITY ? 0.f : S.s * __expf(S.m - cm);
          S.m = cm;
          S.bi = ci;
        }
        float add = 0.f;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int cls = c0 + mt * 16 + q * 4 + r;
            const float v = acc[t][mt][r] + bv[mt][r];
            if (cls < c_end) add += ovr ? sigmoidf_(v) : __expf(v - S.m);
          }
        S.s += add;
      }
    }
  }

  if constexpr (MODE == 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      RowState S = st[t];
      S = merge_state(S, shfl_state(S, 16), ovr);
      S = merge_state(S, shfl_state(S, 32), ovr);
      const int64_t row = row0 + t * 16 + col;
      if (q == 0 && row < B) {
        if (gridDim.y == 1) {
          out_idx[row] = S.bi;
          out_p[row] = ovr ? sigmoidf_(S.m) / S.s : 1.f / S.s;
        } else {
          partials[(int64_t)blockIdx.y * B + row] = make_float4(S.m, S.s, __int_as_float(S.bi), 0.f);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void merge_partials_kernel(const float4* __restrict__ partials, int splits,
                                                             int64_t B, int kind, int32_t* __restrict__ out_idx,
                                                             float* __restrict__ out_p) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  const bool ovr = kind == KIND_OVR;
  float4 p0 = partials[row];
  RowState S{p0.x, p0.y, __float_as_int(p0.z)};
  for (int sp = 1; sp < splits; ++sp) {
    const float4 p = partials[(int64_t)sp * B + row];
    S = merge_state(S, RowState{p.x, p.y, __float_as_int(p.z)}, ovr);
  }
  out_idx[row] = S.bi;
  out_p[row] = ovr ? sigmoidf_(S.m) / S.s : 1.f / S.s;
}

struct Plan {
  int splits;
  int classes_per_split;
};

Plan make_plan(int64_t B, int K) {
  const int64_t row_blocks = (B + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  const int chunks = (K + CLASS_CHUNK - 1) / CLASS_CHUNK;
  int64_t want = (512 + row_blocks - 1) / row_blocks;  // aim for >= 512 blocks (2 per CU)
  int splits = (int)(want < 1 ? 1 : (want > chunks ? chunks : want));
  const int chunks_per_split = (chunks + splits - 1) / splits;
  Plan p;
  p.classes_per_split = chunks_per_split * CLASS_CHUNK;
  p.splits = (K + p.classes_per_split - 1) / p.classes_per_split;
  return p;
}

template <int MODE>
void launch_mode(const void* X, const void* W, const float* b, int64_t B, int F, int K, int kind, int32_t* out_idx,
                 float* out_p, float4* partials, float* Z, const Plan& plan, hipStream_t stream) {
  if (F % 32 != 0 || F > 512) throw std::invalid_argument("gemm_softmax: F must be a multiple of 32 and <= 512");
  const dim3 grid((unsigned)((B + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK), (unsigned)plan.splits);
  auto x = static_cast<const uint16_t*>(X);
  auto w = static_cast<const uint16_t*>(W);
#define MLAPI_GEMM_LAUNCH(KSV)                                                                                    \
  hipLaunchKernelGGL((gemm_softmax_kernel<KSV, MODE>), grid, dim3(256), 0, stream, x, w, b, B, F, K, kind,       \
                     plan.classes_per_split, out_idx, out_p, partials, Z)
  const int ks = F / 32;
  if (ks <= 2)
    MLAPI_GEMM_LAUNCH(2);
  else if (ks <= 4)
    MLAPI_GEMM_LAUNCH(4);
  else if (ks <= 8)
    MLAPI_GEMM_LAUNCH(8);
  else
    MLAPI_GEMM_LAUNCH(16);
#undef MLAPI_GEMM_LAUNCH
  MLAPI_HIP_CHECK(hipGetLastError());
}

}  // namespace

size_t gemm_softmax_workspace(int64_t B, int K, int F) {
  (void)F;
  const Plan p = make_plan(B, K);
  return p.splits > 1 ? (size_t)p.splits * (size_t)B * sizeof(float4) : 0;
}

void launch_gemm_softmax(const void* X, const void* W, const float* b, int64_t B, int F, int K, int kind,
                         int32_t* out_idx, float* out_p, void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (B <= 0) return;
  if (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("gemm_softmax: multiclass kinds only (binary models use gemv_binary)");
  const Plan plan = make_plan(B, K);
  if (plan.splits > 1 && ws_bytes < (size_t)plan.splits * (size_t)B * sizeof(float4))
    throw std::invalid_argument("gemm_softmax: workspace too small");
  launch_mode<0>(X, W, b, B, F, K, kind, out_idx, out_p, static_cast<float4*>(workspace), nullptr, plan, stream);
  if (plan.splits > 1) {
    hipLaunchKernelGGL(merge_partials_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, stream,
                       static_cast<const float4*>(workspace), plan.splits, B, kind, out_idx, out_p);
    MLAPI_HIP_CHECK(hipGetLastError());
  }
}

void launch_gemm_logits(const void* X, const void* W, const float* b, int64_t B, int F, int K, float* Z,
                        hipStream_t stream) {
  if (B <= 0) return;
  const Plan plan = make_plan(B, K);
  launch_mode<1>(X, W, b, B, F, K, KIND_MULTINOMIAL, nullptr, nullptr, nullptr, Z, plan, stream);
}

}  // namespace mlapi
