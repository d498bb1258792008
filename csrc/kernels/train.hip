// Training kernels for logistic / softmax regression.
//
// The reference trains once, offline, with sklearn's full-batch L-BFGS
// (`Logistic Regression.ipynb:33-34`). Here training is a first-class, data-parallel
// workload (BASELINE config 5): every rank computes the gradient SUM of its mini-batch shard with
// these kernels, the sums are all-reduced over RCCL, and the SGD update applies 1/N_global.
//
// train_binary_grad  - binary LR, ONE pass over X (bf16 or f32): forward dot product, sigmoid,
//                      BCE loss, correct count and the dW = sum_i g_i x_i accumulation all happen
//                      while the row is in registers (HBM-bound like the predict GEMV). Per-block
//                      partial slabs + a fixed-order reduce keep the result bitwise deterministic
//                      (no float atomics: cdna_hip_programming.md Guideline 12).
// train_small_grad   - exact fp64 (or fp32) loss + gradient for small models (Iris: F=4, K=3),
//                      all kinds (binary, binary-softmax, multinomial, OvR). Used by the
//                      L-BFGS path that reproduces sklearn's fit, and by small-model SGD.
// sgd_update         - W -= lr * (g / N + l2 * W) (intercept unpenalized), optional momentum.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mlapi/common.h"
#include "mlapi/kernels.h"
#include "mlapi/device.h"
#include "mlapi/rowreduce.h"
#include "dist/p2p_device.h"

namespace mlapi {
namespace {

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// ------------------------------------------------------------------------------------------------
// Binary, large F.
// ------------------------------------------------------------------------------------------------
template <typename T>
struct TChunk;
template <>
struct TChunk<uint16_t> {
  static constexpr int N = 8;
  __device__ static __forceinline__ void unpack(const u32x4_t& v, float (&o)[8]) {
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = __uint_as_float(u[i] << 16);
      o[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  }
};
template <>
struct TChunk<float> {
  static constexpr int N = 4;
  __device__ static __forceinline__ void unpack(const u32x4_t& v, float (&o)[4]) {
    o[0] = __uint_as_float(v.x);
    o[1] = __uint_as_float(v.y);
    o[2] = __uint_as_float(v.z);
    o[3] = __uint_as_float(v.w);
  }
};

template <typename T, int LPR, int CPL, int U>
__global__ __launch_bounds__(256) void train_binary_grad_kernel(const T* __restrict__ X, const float* __restrict__ y,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ bptr, int64_t B, int F,
                                                                float* __restrict__ slabs) {
  constexpr int RPW = 64 / LPR;
  constexpr int NE = TChunk<T>::N;
  __shared__ float red[4 * RPW * CPL * LPR * NE + 4 * 3];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform -> SGPR loop control
  const int sub = lane / LPR;
  const int cl = lane % LPR;
  const int chunks = F / NE;
  const int64_t ld16 = chunks;
  const float bias = *bptr;

  float wv[CPL][NE];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = cl + c * LPR;
#pragma unroll
    for (int e = 0; e < NE; ++e) wv[c][e] = ch < chunks ? w[ch * NE + e] : 0.f;
  }
  float gw[CPL][NE];
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int e = 0; e < NE; ++e) gw[c][e] = 0.f;
  float gb = 0.f, loss = 0.f, correct = 0.f;

  const int64_t rows_per_wave_iter = (int64_t)U * RPW;
  const int64_t waves_total = (int64_t)gridDim.x * 4;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + wave;

  // After reduce_scatter every lane of an LPR group holds the complete dot product of ONE row slot
  // (my_u); the sigmoid / loss / correct epilogue is evaluated once per lane for that slot and only
  // the scalar gradient g is broadcast back for the dW accumulation (evaluating the epilogue for all
  // U slots on every lane made the transcendentals, not HBM, the bottleneck).
  const int my_u = slot_of<LPR, U>(cl);
  const bool my_owner = cl == owner_of<LPR, U>(my_u);  // one lane per row counts the stats
  const int group_base = lane - cl;

  // Chunk column of this lane for each c, clamped into the row: lanes past the last chunk re-read a
  // valid chunk; their forward weights are zero and their dW partials are never written out, so
  // no per-value masking is needed (a select on the loaded data made hipcc wait for each load
  // right after issuing it).
  int coff[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) coff[c] = min(cl + c * LPR, chunks - 1);
  const u32x4_t* X16 = reinterpret_cast<const u32x4_t*>(X);
  const int64_t stride_u = (int64_t)RPW * ld16;  // elements of u32x4 between row slots u and u+1

  for (int64_t base = wave_id * rows_per_wave_iter; base < B; base += waves_total * rows_per_wave_iter) {
    // Loads are unconditional (no per-load guard: a guarded load makes hipcc branch around it and
    // wait vmcnt(0) per load, which serializes the stream). Full iterations (wave-uniform test)
    // use one base pointer + constant strides; only the last, partial iteration clamps rows.
    const int64_t my_row = base + (int64_t)my_u * RPW + sub;
    const float my_y = y[min(my_row, B - 1)];
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
      for (int c = 0; c < CPL; ++c) {
        float xe[NE];
        TChunk<T>::unpack(xv[u][c], xe);
#pragma unroll
        for (int e = 0; e < NE; ++e) acc = fmaf(xe[e], wv[c][e], acc);
      }
      part[u] = acc;
    }
    // Register barrier: make the packed rows opaque here so the compiler re-unpacks them for the
    // backward pass instead of keeping U x NE unpacked floats live across the reduction (that
    // held the kernel at ~200 VGPRs / 2 waves per SIMD).
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < CPL; ++c) asm volatile("" : "+v"(xv[u][c]));
    const float z = reduce_scatter<LPR, U>(part, cl) + bias;
    const bool valid = my_row < B;
    const float yy = valid ? my_y : 0.f;
    const float g_mine = valid ? __builtin_amdgcn_rcpf(1.f + __expf(-z)) - yy : 0.f;
    const bool own = valid && my_owner;
    gb += own ? g_mine : 0.f;
    loss += own ? fmaxf(z, 0.f) - z * yy + log1pf(__expf(-fabsf(z))) : 0.f;
    correct += (own && ((z > 0.f) == (yy > 0.5f))) ? 1.f : 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float g = __shfl(g_mine, group_base + owner_of<LPR, U>(u), 64);
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        float xe[NE];
        TChunk<T>::unpack(xv[u][c], xe);
#pragma unroll
        for (int e = 0; e < NE; ++e) gw[c][e] = fmaf(g, xe[e], gw[c][e]);
      }
    }
  }

  // Deterministic block reduction: [wave][sub][c][cl][e] partials -> fixed-order sum.
  float* gwred = red;
  float* stred = red + 4 * RPW * CPL * LPR * NE;
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int e = 0; e < NE; ++e) gwred[(((wave * RPW + sub) * CPL + c) * LPR + cl) * NE + e] = gw[c][e];
  // wave-level reduce of the scalar stats (fixed xor order)
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    gb += __shfl_xor(gb, off, 64);
    loss += __shfl_xor(loss, off, 64);
    correct += __shfl_xor(correct, off, 64);
  }
  if (lane == 0) {
    stred[wave * 3 + 0] = gb;
    stred[wave * 3 + 1] = loss;
    stred[wave * 3 + 2] = correct;
  }
  __syncthreads();
  float* slab = slabs + (int64_t)blockIdx.x * (F + 3);
  for (int j = threadIdx.x; j < F; j += blockDim.x) {
    const int ch = j / NE, e = j % NE;
    const int c = ch / LPR, l = ch % LPR;
    float s = 0.f;
    for (int wv_ = 0; wv_ < 4; ++wv_)
      for (int sb = 0; sb < RPW; ++sb) s += gwred[(((wv_ * RPW + sb) * CPL + c) * LPR + l) * NE + e];
    slab[j] = s;
  }
  if (threadIdx.x < 3) {
    float s = 0.f;
    for (int wv_ = 0; wv_ < 4; ++wv_) s += stred[wv_ * 3 + threadIdx.x];
    slab[F + threadIdx.x] = s;
  }
}

// Deterministic slab reduction: COLS columns x PARTS partitions per 256-thread block. Partition p
// sums slabs p, p+PARTS, ... in increasing order (each partition row reads COLS consecutive
// columns of a slab), then the PARTS partials are added in fixed order through LDS.
// A single thread per column walking all slabs serially was the bottleneck of the training step
// (232 us vs 22 us for the fused gradient kernel: profiles/r1_first/train_kernel_stats.csv).
// FUSE_SGD: when no all-reduce separates them (one replica), the SGD update of the parameter
// vector is applied by the same thread that produced the column's gradient sum (saves a launch).
// Narrow parameter vectors (binary logistic on a handful of features: width ~5) use 4-column
// groups so 64 partitions share the slab walk instead of 16 (11 of 16 columns would idle).
struct SgdArgs {
  float* params = nullptr;
  float* mom = nullptr;
  int64_t n_params = 0, n_pen = 0;
  float lr = 0.f, inv_n = 0.f, l2 = 0.f, momentum = 0.f;
};

// DP: the data-parallel all-reduce happens here too (p2p_device.h): each block publishes its
// columns' local sums to the IPC-mapped exchange buffer, waits for the same block of every rank,
// and sums the ranks' values in rank order before the update - gradient kernel + this kernel are
// the whole DP step (2 launches at any world size, bitwise-identical replicas).
template <typename T, bool FUSE_SGD, int RED_COLS, bool DP>
__global__ __launch_bounds__(256) void reduce_slabs_kernel(const T* __restrict__ slabs, int nslabs, int width,
                                                           T* __restrict__ out, SgdArgs sgd, P2PBlockArgs dp) {
  constexpr int RED_PARTS = 256 / RED_COLS;
  __shared__ T part[RED_PARTS][RED_COLS];
  const int c = threadIdx.x % RED_COLS;
  const int p = threadIdx.x / RED_COLS;
  const int j = blockIdx.x * RED_COLS + c;
  T s = T(0);
  if (j < width) {
    int i = p;
    for (; i + 3 * RED_PARTS < nslabs; i += 4 * RED_PARTS) {  // 4 independent loads in flight
      const T a0 = slabs[(int64_t)i * width + j];
      const T a1 = slabs[(int64_t)(i + RED_PARTS) * width + j];
      const T a2 = slabs[(int64_t)(i + 2 * RED_PARTS) * width + j];
      const T a3 = slabs[(int64_t)(i + 3 * RED_PARTS) * width + j];
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; i < nslabs; i += RED_PARTS) s += slabs[(int64_t)i * width + j];
  }
  part[p][c] = s;
  __syncthreads();
  T t = T(0);
  if (p == 0 && j < width) {
    t = part[0][c];
#pragma unroll
    for (int q = 1; q < RED_PARTS; ++q) t += part[q][c];
  }
  static_assert(!DP || sizeof(T) == sizeof(float), "fused DP exchange: f32 gradients");
  if (DP && dp.world > 1) {  // one rank: nothing to exchange (the same kernel, no peers)
    if (p == 0 && j < width) dp.mine[j] = (float)t;
    if (!p2p_block_sync(dp, blockIdx.x)) return;  // peer missing: status recorded, no update
    if (p == 0 && j < width) {  // rank order; the own slice from registers (same bits as the published copy)
      const float own = (float)t;
      float g = dp.rank == 0 ? own : dp.peer[0][j];
      for (int r = 1; r < dp.world; ++r) g += r == dp.rank ? own : dp.peer[r][j];
      t = (T)g;
    }
  }
  if (p == 0 && j < width) {
    out[j] = t;
    if constexpr (FUSE_SGD) {
      if (j < sgd.n_params) {
        float d = (float)t * sgd.inv_n + (j < sgd.n_pen ? sgd.l2 * sgd.params[j] : 0.f);
        if (sgd.mom != nullptr) {
          const float v = sgd.momentum * sgd.mom[j] + d;
          sgd.mom[j] = v;
          d = v;
        }
        sgd.params[j] -= sgd.lr * d;
      }
    }
  }
}

template <typename T, int COLS>
void launch_reduce_slabs_cols(const T* slabs, int nslabs, int width, T* out, hipStream_t stream,
                              const SgdArgs* sgd, P2PAllReduce* dp, int dp_timeout_ms) {
  const int nblocks = (width + COLS - 1) / COLS;
  const dim3 grid((unsigned)nblocks);
  if constexpr (sizeof(T) == sizeof(float)) {
    if (dp != nullptr) {
      const P2PBlockArgs a = dp->block_exchange((size_t)width * sizeof(float), nblocks, dp_timeout_ms);
      if (sgd != nullptr)
        hipLaunchKernelGGL((reduce_slabs_kernel<T, true, COLS, true>), grid, dim3(256), 0, stream, slabs, nslabs,
                           width, out, *sgd, a);
      else
        hipLaunchKernelGGL((reduce_slabs_kernel<T, false, COLS, true>), grid, dim3(256), 0, stream, slabs, nslabs,
                           width, out, SgdArgs{}, a);
      MLAPI_HIP_CHECK(hipGetLastError());
      return;
    }
  } else {
    if (dp != nullptr) throw std::invalid_argument("fused DP exchange: f32 gradients only");
  }
  if (sgd != nullptr)
    hipLaunchKernelGGL((reduce_slabs_kernel<T, true, COLS, false>), grid, dim3(256), 0, stream, slabs, nslabs, width,
                       out, *sgd, P2PBlockArgs{});
  else
    hipLaunchKernelGGL((reduce_slabs_kernel<T, false, COLS, false>), grid, dim3(256), 0, stream, slabs, nslabs,
                       width, out, SgdArgs{}, P2PBlockArgs{});
  MLAPI_HIP_CHECK(hipGetLastError());
}

template <typename T>
void launch_reduce_slabs(const T* slabs, int nslabs, int width, T* out, hipStream_t stream,
                         const SgdArgs* sgd = nullptr, P2PAllReduce* dp = nullptr, int dp_timeout_ms = 0) {
  if (width <= 8)
    launch_reduce_slabs_cols<T, 4>(slabs, nslabs, width, out, stream, sgd, dp, dp_timeout_ms);
  else
    launch_reduce_slabs_cols<T, 16>(slabs, nslabs, width, out, stream, sgd, dp, dp_timeout_ms);
}

struct BinPlan {
  int lpr, cpl, u, rows_per_block;
};

BinPlan bin_plan(int chunks) {
  if (chunks <= 8) return {8, 1, 8, 4 * 8 * 8};
  if (chunks <= 16) return {16, 1, 8, 4 * 8 * 4};
  if (chunks <= 32) return {32, 1, 8, 4 * 8 * 2};
  if (chunks <= 64) return {64, 1, 8, 4 * 8};
  if (chunks <= 128) return {64, 2, 4, 4 * 4};
  if (chunks <= 256) return {64, 4, 2, 4 * 2};
  return {0, 0, 0, 0};
}

int g_train_max_blocks = 0;  // benchmark override (train_binary_set_max_blocks); 0 = default

int64_t bin_blocks(int64_t B, const BinPlan& p) {
  int64_t blocks = (B + p.rows_per_block - 1) / p.rows_per_block;
  // Grid cap: more blocks = more bytes in flight (HBM-bound) but more slabs to reduce;
  // 512 was fastest for 64K..1M rows x 256 bf16 (profiles/r1_train_v2/train_sweep.log).
  const int64_t cap = g_train_max_blocks > 0 ? g_train_max_blocks : 512;
  return blocks < 1 ? 1 : (blocks > cap ? cap : blocks);
}

// ------------------------------------------------------------------------------------------------
// Small models, exact objective terms (fp64 or fp32).
// ------------------------------------------------------------------------------------------------
constexpr int SMALL_R = 64;     // rows staged per chunk
constexpr int SMALL_KMAX = 16;  // classes (rows of W)
constexpr int SMALL_FMAX = 64;

template <typename T>
__device__ __forceinline__ T texp(T v);
template <>
__device__ __forceinline__ double texp<double>(double v) { return exp(v); }
template <>
__device__ __forceinline__ float texp<float>(float v) { return expf(v); }
template <typename T>
__device__ __forceinline__ T tlog1p(T v);
template <>
__device__ __forceinline__ double tlog1p<double>(double v) { return log1p(v); }
template <>
__device__ __forceinline__ float tlog1p<float>(float v) { return log1pf(v); }
template <typename T>
__device__ __forceinline__ T tlog(T v);
template <>
__device__ __forceinline__ double tlog<double>(double v) { return log(v); }
template <>
__device__ __forceinline__ float tlog<float>(float v) { return logf(v); }

// Binary cross-entropy with logits: log(1 + exp(-z)) for y=1, log(1 + exp(z)) for y=0.
template <typename T>
__device__ __forceinline__ T bce(T z, T y) {
  return (z > T(0) ? z : T(0)) - z * y + tlog1p<T>(texp<T>(-(z < T(0) ? -z : z)));
}

template <typename T>
__global__ __launch_bounds__(256) void train_small_grad_kernel(const T* __restrict__ X, const int32_t* __restrict__ y,
                                                               const T* __restrict__ W, const T* __restrict__ b,
                                                               int64_t B, int F, int K, int kind,
                                                               T* __restrict__ slabs) {
  __shared__ T gs[SMALL_R * SMALL_KMAX];
  __shared__ T xs[SMALL_R * SMALL_FMAX];
  __shared__ T red[2 * SMALL_R];
  const int tid = threadIdx.x;
  const int KF = K * F;
  T acc[4] = {T(0), T(0), T(0), T(0)};  // owned dW entries: tid, tid+256, ...
  T accb = T(0);
  T loss = T(0), correct = T(0);
  const int64_t nchunks = (B + SMALL_R - 1) / SMALL_R;
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    if (tid < SMALL_R) {
      const int64_t r = ch * SMALL_R + tid;
      const bool valid = r < B;
      T z[SMALL_KMAX];
#pragma unroll
      for (int k = 0; k < SMALL_KMAX; ++k) {
        if (k < K) {
          T a = T(0);
          for (int f = 0; f < F; ++f) a = fma(valid ? X[r * F + f] : T(0), W[k * F + f], a);
          z[k] = a + b[k];
        }
      }
      for (int f = 0; f < F; ++f) xs[tid * SMALL_FMAX + f] = valid ? X[r * F + f] : T(0);
      const int yi = valid ? y[r] : 0;
      T g[SMALL_KMAX];
      if (kind == KIND_BINARY || kind == KIND_BINARY_SOFTMAX) {
        const T sc = kind == KIND_BINARY_SOFTMAX ? T(2) : T(1);
        const T zz = sc * z[0];
        const T yy = T(yi);
        g[0] = sc * (T(1) / (T(1) + texp<T>(-zz)) - yy);
        if (valid) {
          loss += bce<T>(zz, yy);
          correct += ((z[0] > T(0)) == (yi == 1)) ? T(1) : T(0);
        }
      } else if (kind == KIND_MULTINOMIAL) {
        T m = z[0];
        int am = 0;
#pragma unroll
        for (int k = 1; k < SMALL_KMAX; ++k)
          if (k < K && z[k] > m) { m = z[k]; am = k; }
        T s = T(0);
#pragma unroll
        for (int k = 0; k < SMALL_KMAX; ++k)
          if (k < K) { g[k] = texp<T>(z[k] - m); s += g[k]; }
#pragma unroll
        for (int k = 0; k < SMALL_KMAX; ++k)
          if (k < K) g[k] = g[k] / s - (k == yi ? T(1) : T(0));
        if (valid) {
          loss += m + tlog<T>(s) - z[yi];
          correct += am == yi ? T(1) : T(0);
        }
      } else {  // OVR: independent binary problems
        T m = z[0];
        int am = 0;
#pragma unroll
        for (int k = 0; k < SMALL_KMAX; ++k) {
          if (k < K) {
            const T yy = k == yi ? T(1) : T(0);
            g[k] = T(1) / (T(1) + texp<T>(-z[k])) - yy;
            if (valid) loss += bce<T>(z[k], yy);
            if (k > 0 && z[k] > m) { m = z[k]; am = k; }
          }
        }
        if (valid) correct += am == yi ? T(1) : T(0);
      }
#pragma unroll
      for (int k = 0; k < SMALL_KMAX; ++k)
        if (k < K) gs[tid * SMALL_KMAX + k] = valid ? g[k] : T(0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * 256;
      if (e < KF) {
        const int k = e / F, f = e % F;
        T a = acc[i];
        for (int r = 0; r < SMALL_R; ++r) a = fma(gs[r * SMALL_KMAX + k], xs[r * SMALL_FMAX + f], a);
        acc[i] = a;
      }
    }
    if (tid < K) {
      T a = accb;
      for (int r = 0; r < SMALL_R; ++r) a += gs[r * SMALL_KMAX + tid];
      accb = a;
    }
    __syncthreads();
  }
  if (tid < SMALL_R) {
    red[tid] = loss;
    red[SMALL_R + tid] = correct;
  }
  __syncthreads();
  const int width = KF + K + 2;
  T* slab = slabs + (int64_t)blockIdx.x * width;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid + i * 256;
    if (e < KF) slab[e] = acc[i];
  }
  if (tid < K) slab[KF + tid] = accb;
  if (tid == 0) {
    T l = T(0), c = T(0);
    for (int r = 0; r < SMALL_R; ++r) {
      l += red[r];
      c += red[SMALL_R + r];
    }
    slab[KF + K] = l;
    slab[KF + K + 1] = c;
  }
}

int64_t small_blocks(int64_t B) {
  int64_t n = (B + SMALL_R - 1) / SMALL_R;
  return n < 1 ? 1 : (n > 512 ? 512 : n);
}

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sgd_update_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ mom, int64_t n, int64_t n_pen, float lr,
                                                         float inv_n, float l2, float momentum) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float d = g[i] * inv_n + (i < n_pen ? l2 * p[i] : 0.f);
  if (mom != nullptr) {
    const float v = momentum * mom[i] + d;
    mom[i] = v;
    d = v;
  }
  p[i] -= lr * d;
}

// 2-D variant for W_aug = [W | b | 0 pad] (multiclass training): L2 only on the first pen_cols
// columns; writes the bf16 W and the f32 bias the next forward reads (saves a cast launch).
__global__ __launch_bounds__(256) void sgd_update_2d_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                            float* __restrict__ mom, int64_t n, int cols,
                                                            int pen_cols, float lr, float inv_n, float l2,
                                                            float momentum, uint16_t* __restrict__ shadow_w,
                                                            float* __restrict__ shadow_b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t row = i / cols;
  const int c = (int)(i - row * cols);
  float d = g[i] * inv_n + (c < pen_cols ? l2 * p[i] : 0.f);
  if (mom != nullptr) {
    const float v = momentum * mom[i] + d;
    mom[i] = v;
    d = v;
  }
  const float np = p[i] - lr * d;
  p[i] = np;
  if (shadow_w != nullptr && c < pen_cols) shadow_w[row * pen_cols + c] = __builtin_bit_cast(uint16_t, (__bf16)np);
  if (shadow_b != nullptr && c == pen_cols) shadow_b[row] = np;
}

}  // namespace

void train_binary_set_max_blocks(int n) { g_train_max_blocks = n; }

size_t train_binary_workspace(int64_t B, int F) {
  (void)B;
  const int64_t cap = g_train_max_blocks > 0 ? g_train_max_blocks : 512;
  return (size_t)(cap > 4096 ? cap : 4096) * (size_t)(F + 3) * sizeof(float);  // upper bound on slabs
}

namespace {
void train_binary_impl(int dt, const void* X, const float* y, const float* w, const float* bptr, int64_t B, int F,
                       float* out, void* workspace, size_t ws_bytes, hipStream_t stream, const SgdArgs* sgd,
                       P2PAllReduce* dp = nullptr, int dp_timeout_ms = 0) {
  if (B <= 0) return;
  const int ne = dt == DT_BF16 ? 8 : 4;
  if (F % ne != 0) throw std::invalid_argument("train_binary: F must be a multiple of 16 bytes of elements");
  const BinPlan p = bin_plan(F / ne);
  if (p.lpr == 0) throw std::invalid_argument("train_binary: F too large");
  const int64_t blocks = bin_blocks(B, p);
  if (ws_bytes < (size_t)blocks * (F + 3) * sizeof(float)) throw std::invalid_argument("train_binary: workspace");
  float* slabs = static_cast<float*>(workspace);
#define MLAPI_TB(T, L, C, U)                                                                                 \
  hipLaunchKernelGGL((train_binary_grad_kernel<T, L, C, U>), dim3((unsigned)blocks), dim3(256), 0, stream,  \
                     static_cast<const T*>(X), y, w, bptr, B, F, slabs)
#define MLAPI_TB_ALL(T)                                       \
  if (p.lpr == 8) MLAPI_TB(T, 8, 1, 8);                       \
  else if (p.lpr == 16) MLAPI_TB(T, 16, 1, 8);                \
  else if (p.lpr == 32) MLAPI_TB(T, 32, 1, 8);                \
  else if (p.cpl == 1) MLAPI_TB(T, 64, 1, 8);                 \
  else if (p.cpl == 2) MLAPI_TB(T, 64, 2, 4);                 \
  else MLAPI_TB(T, 64, 4, 2);
  if (dt == DT_BF16) {
    MLAPI_TB_ALL(uint16_t)
  } else if (dt == DT_F32) {
    MLAPI_TB_ALL(float)
  } else {
    throw std::invalid_argument("train_binary: dtype must be bf16 or f32");
  }
#undef MLAPI_TB_ALL
#undef MLAPI_TB
  MLAPI_HIP_CHECK(hipGetLastError());
  launch_reduce_slabs<float>(slabs, (int)blocks, F + 3, out, stream, sgd, dp, dp_timeout_ms);
}
}  // namespace

void launch_train_binary_grad(int dt, const void* X, const float* y, const float* w, float /*bias_unused*/,
                              const float* bptr, int64_t B, int F, float* out, void* workspace, size_t ws_bytes,
                              hipStream_t stream) {
  train_binary_impl(dt, X, y, w, bptr, B, F, out, workspace, ws_bytes, stream, nullptr);
}

void launch_train_binary_step(int dt, const void* X, const float* y, float* params, float* mom, int64_t B, int F,
                              float* grad_out, void* workspace, size_t ws_bytes, float lr, float inv_n, float l2,
                              float momentum, hipStream_t stream, P2PAllReduce* dp, int dp_timeout_ms) {
  SgdArgs a;
  a.params = params;
  a.mom = mom;
  a.n_params = F + 1;
  a.n_pen = F;
  a.lr = lr;
  a.inv_n = inv_n;
  a.l2 = l2;
  a.momentum = momentum;
  train_binary_impl(dt, X, y, params, params + F, B, F, grad_out, workspace, ws_bytes, stream, &a, dp, dp_timeout_ms);
}

size_t train_small_workspace(int64_t B, int F, int K) {
  return (size_t)small_blocks(B) * (size_t)(K * F + K + 2) * sizeof(double);
}

void launch_train_small_grad(int dt, const void* X, const int32_t* y, const void* W, const void* b, int64_t B, int F,
                             int K, int kind, void* out, void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (B <= 0) return;
  if (K > SMALL_KMAX || F > SMALL_FMAX || K * F > 1024)
    throw std::invalid_argument("train_small: needs K <= 16, F <= 64");
  const int64_t blocks = small_blocks(B);
  const int width = K * F + K + 2;
  const size_t es = dt == DT_F64 ? 8 : 4;
  if (ws_bytes < (size_t)blocks * width * es) throw std::invalid_argument("train_small: workspace too small");
  if (dt == DT_F64) {
    hipLaunchKernelGGL(train_small_grad_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, stream,
                       static_cast<const double*>(X), y, static_cast<const double*>(W),
                       static_cast<const double*>(b), B, F, K, kind, static_cast<double*>(workspace));
    MLAPI_HIP_CHECK(hipGetLastError());
    launch_reduce_slabs<double>(static_cast<const double*>(workspace), (int)blocks, width, static_cast<double*>(out),
                                stream);
  } else if (dt == DT_F32) {
    hipLaunchKernelGGL(train_small_grad_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, stream,
                       static_cast<const float*>(X), y, static_cast<const float*>(W), static_cast<const float*>(b),
                       B, F, K, kind, static_cast<float*>(workspace));
    MLAPI_HIP_CHECK(hipGetLastError());
    launch_reduce_slabs<float>(static_cast<const float*>(workspace), (int)blocks, width, static_cast<float*>(out),
                               stream);
  } else {
    throw std::invalid_argument("train_small: dtype must be f64 or f32");
  }
  MLAPI_HIP_CHECK(hipGetLastError());
}

void launch_sgd_update(float* params, const float* grad, float* momentum_buf, int64_t n, int64_t n_penalized,
                       float lr, float inv_n, float l2, float momentum, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sgd_update_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, params, grad,
                     momentum_buf, n, n_penalized, lr, inv_n, l2, momentum);
  MLAPI_HIP_CHECK(hipGetLastError());
}

void launch_sgd_update_2d(float* params, const float* grad, float* momentum_buf, int64_t rows, int cols,
                          int pen_cols, float lr, float inv_n, float l2, float momentum, uint16_t* shadow_w,
                          float* shadow_b, hipStream_t stream) {
  const int64_t n = rows * cols;
  if (n <= 0) return;
  hipLaunchKernelGGL(sgd_update_2d_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, params, grad,
                     momentum_buf, n, cols, pen_cols, lr, inv_n, l2, momentum, shadow_w, shadow_b);
  MLAPI_HIP_CHECK(hipGetLastError());
}

void launch_reduce_slabs_f32(const float* slabs, int nslabs, int width, float* out, hipStream_t stream) {
  launch_reduce_slabs<float>(slabs, nslabs, width, out, stream);
}

}  // namespace mlapi
