// Wide-model serving at the reference's precision: z = X W^T + b with
// float64 accumulation on the matrix cores (v_mfma_f64_16x16x4_f64), for rows and weights stored
// as float64 (wide_dtype f64: sklearn's dtype, /root/reference/main.py:21-22 via check_array) or
// float32 (f32 storage, products exact in f64, so the f32 path's only error is the rounding of
// the model and the rows to f32 - no accumulation error), any F, any K, every sklearn kind.
//
// Geometry (serving batches are a few rows, so the kernel is latency bound: spread the weights
// over many CUs and keep every MFMA chain short):
//  * grid = (ncb class blocks x nfs feature splits, row groups of 32 rows); a block = 4 waves;
//    a block owns 16 classes x 32 rows x one feature split, and its 4 waves split that range
//    again, each accumulating the 16 x 16-row tiles of its quarter (NB tiles) in f64 MFMAs;
//  * operands straight from memory to registers, 16 bytes per lane per load (f64: 2 features,
//    f32: 4 features converted exactly to f64): lane l loads class (l & 15) and row (l & 15) at
//    feature offset 4*E*step + (l >> 4)*E, and element e of its load is the MFMA's k = l >> 4
//    for the e-th MFMA of the step - the same k permutation for A (W) and B (X);
//  * loads in chunks of U = 4 steps, two chunks in flight (double buffer);
//  * the 4 waves' tiles are summed through LDS in fixed order; feature splits (nfs > 1) are summed
//    by the last-arriving block of the class block (write-through partials, one ticket, one
//    agent-scope acquire: Guideline 16), in split order;
//  * epilogue per row: bias, then the sklearn epilogue of `kind` (K = 1 binary kinds: z > 0 and
//    sigma(|z|) / the two-class softmax, exactly as linear_rows.h); multiclass kinds reduce the
//    block's 16 classes to a row state {max, sum exp(z - max) | sum sigmoid(z), first argmax} and
//    class blocks are merged either on the host (one 32-byte record per block and row, the
//    engine's completer merges in double in block order) or in-kernel by the last-arriving block
//    of the row group (ticket + acquire), in block order. Everything in f64.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace wide {

typedef __attribute__((ext_vector_type(4))) double wd4_t;
typedef __attribute__((ext_vector_type(2))) double wd2_t;
typedef __attribute__((ext_vector_type(4))) float wf4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t wu4_t;

constexpr int CB = 16;     // classes per block
constexpr int RG = 32;     // rows per row group
constexpr int WAVES = 4;   // waves per block (feature quarters)
constexpr int U = 4;       // steps per load chunk

struct WideArgs {
  const void* X;
  int64_t ldx;             // row stride of X and W (elements): a multiple of the split unit
  const void* W;           // [K][ldx]
  const double* bias;      // [K]
  int32_t B, K, kind, ncb, nfs, fsteps;  // fsteps: steps (4 * E features) per wave per split
  int32_t* out_idx;        // library output (in-kernel class merge) ...
  double* out_p;
  RecOut ro;               // ... or serving records (in-kernel class merge)
  uint4* hrec;             // host class merge: [ncb][32 rows][2] 16-byte units {seq, bi, m} {seq, 0, s}
  uint32_t hseq;
  // Workspace, one region per row group (the layout does not depend on B, so launches of any size
  // share it): [ncb split tickets | 1 class ticket] (zero, re-armed by the last arrivers), then
  // [ncb][nfs][2 * 4 * 64] f64 split partial tiles (nfs > 1), then [ncb][32 rows][4] f64 row
  // states {m, s, argmax bits, 0}.
  unsigned char* ws;
  int64_t rg_bytes, cnt_bytes, part_bytes;
  int32_t row_groups;
  int32_t probe;  // measurement only (linear_wide_set_probe): 1 = stop after the MFMA loop, 2 = after
                  // the block's row states (before the class merge)
};

template <typename T>
__device__ __forceinline__ double elem(const uint4& v, int e) {
  if constexpr (sizeof(T) == 8) {
    return __builtin_bit_cast(wd2_t, v)[e];
  } else {
    return (double)__builtin_bit_cast(wf4_t, v)[e];
  }
}

struct WState {
  double m, s;
  int bi;
};

__device__ __forceinline__ WState wmerge(WState a, WState b, bool ovr) {
  const bool take_b = (b.m > a.m) || (b.m == a.m && b.bi < a.bi);
  WState r;
  r.m = take_b ? b.m : a.m;
  r.bi = take_b ? b.bi : a.bi;
  if (ovr) {
    r.s = a.s + b.s;
  } else {
    const double sa = a.m == -INFINITY ? 0.0 : a.s * exp(a.m - r.m);
    const double sb = b.m == -INFINITY ? 0.0 : b.s * exp(b.m - r.m);
    r.s = sa + sb;
  }
  return r;
}

__device__ __forceinline__ WState wshfl(WState a, int off) {
  return WState{__shfl_xor(a.m, off, 64), __shfl_xor(a.s, off, 64), __shfl_xor(a.bi, off, 64)};
}

__device__ __forceinline__ double wsigmoid(double z) { return 1.0 / (1.0 + exp(-z)); }

// write-through 16-byte store (device-internal hand-off: sc1; host records: sc0 sc1)
__device__ __forceinline__ void st16_sc1(void* dst, wu4_t v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
__device__ __forceinline__ void st16_host(void* dst, wu4_t v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
}
__device__ __forceinline__ wu4_t pack2(uint32_t a, uint32_t b, double d) {
  const uint64_t u = __builtin_bit_cast(uint64_t, d);
  return wu4_t{a, b, (uint32_t)u, (uint32_t)(u >> 32)};
}

// final (label, p) of a merged multiclass state, or of a binary logit
__device__ __forceinline__ void finish_row(const WideArgs& a, int64_t row, int32_t idx, double p) {
  if (a.ro.rec != nullptr) {
    put_record(a.ro.rec + row, a.ro.seq, idx, p);
  } else {
    a.out_idx[row] = idx;
    a.out_p[row] = p;
  }
}

template <typename T, int NB>
__device__ __forceinline__ void wide_predict(const WideArgs& a) {
  constexpr int E = 16 / (int)sizeof(T);  // features per 16-byte load
  constexpr int STEP = 4 * E;             // features per wave step
  __shared__ wd4_t red[WAVES][NB][64];
  __shared__ int bcast;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int cb = blockIdx.x % a.ncb, fs = blockIdx.x / a.ncb, rgi = blockIdx.y;
  const int c0 = cb * CB;
  const int64_t row0 = (int64_t)rgi * RG;
  const int S = a.fsteps;
  const int64_t f0 = ((int64_t)fs * WAVES + wave) * S * STEP + g * E;
  const T* wp = static_cast<const T*>(a.W) + (int64_t)min(c0 + r16, a.K - 1) * a.ldx + f0;
  const T* xp[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t)
    xp[t] = static_cast<const T*>(a.X) + min(row0 + t * 16 + r16, (int64_t)a.B - 1) * a.ldx + f0;

  wd4_t acc[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) acc[t] = wd4_t{0.0, 0.0, 0.0, 0.0};
  uint4 w0[U], x0[NB][U], w1[U], x1[NB][U];
  auto load = [&](uint4(&w)[U], uint4(&x)[NB][U], int s0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s0 + u < S) {  // uniform
        w[u] = *reinterpret_cast<const uint4*>(wp + (int64_t)(s0 + u) * STEP);
#pragma unroll
        for (int t = 0; t < NB; ++t) x[t][u] = *reinterpret_cast<const uint4*>(xp[t] + (int64_t)(s0 + u) * STEP);
      }
    }
  };
  auto mma = [&](const uint4(&w)[U], const uint4(&x)[NB][U], int s0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s0 + u < S) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const double av = elem<T>(w[u], e);
#pragma unroll
          for (int t = 0; t < NB; ++t)
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, elem<T>(x[t][u], e), acc[t], 0, 0, 0);
        }
      }
    }
  };
  load(w0, x0, 0);
  for (int s0 = 0; s0 < S; s0 += 2 * U) {
    load(w1, x1, s0 + U);
    __builtin_amdgcn_sched_barrier(0);  // keep the next chunk's loads in flight over these MFMAs
    mma(w0, x0, s0);
    load(w0, x0, s0 + 2 * U);
    __builtin_amdgcn_sched_barrier(0);
    mma(w1, x1, s0 + U);
  }

  if (a.probe == 1) {  // measurement: keep the accumulators alive, store nothing
    if (acc[0][0] == 12345.678) a.out_p[0] = acc[0][1];
    return;
  }
  // ---- the block's tile: the 4 waves' quarters, summed in wave order
#pragma unroll
  for (int t = 0; t < NB; ++t) red[wave][t][lane] = acc[t];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int t = 0; t < NB; ++t) acc[t] = ((red[0][t][lane] + red[1][t][lane]) + red[2][t][lane]) + red[3][t][lane];
  }
  // ---- feature splits: the last-arriving block of (row group, class block) sums them in order
  if (a.nfs > 1) {
    typedef __attribute__((address_space(1))) unsigned int gu32_t;
    unsigned char* rgw = a.ws + (int64_t)rgi * a.rg_bytes;
    double* part = reinterpret_cast<double*>(rgw + a.cnt_bytes) + ((int64_t)cb * a.nfs) * (2 * 4 * 64);
    if (wave == 0) {
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        double* dst = part + (int64_t)fs * (2 * 4 * 64) + t * 256 + lane * 4;
        st16_sc1(dst, __builtin_bit_cast(wu4_t, wd2_t{acc[t][0], acc[t][1]}));
        st16_sc1(dst + 2, __builtin_bit_cast(wu4_t, wd2_t{acc[t][2], acc[t][3]}));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every partial acknowledged before the ticket
      if (lane == 0) {
        gu32_t* ctr = (gu32_t*)(reinterpret_cast<unsigned int*>(rgw) + cb);
        const unsigned tk = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = tk == (unsigned)a.nfs - 1;
        if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
        bcast = last;
      }
    }
    __syncthreads();
    if (!bcast) return;  // uniform per block
    if (wave == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int t = 0; t < NB; ++t) acc[t] = wd4_t{0.0, 0.0, 0.0, 0.0};
      for (int f = 0; f < a.nfs; ++f) {  // split order: deterministic
#pragma unroll
        for (int t = 0; t < NB; ++t) {
          const double* src = part + (int64_t)f * (2 * 4 * 64) + t * 256 + lane * 4;
          const wd4_t v = *reinterpret_cast<const wd4_t*>(src);
          acc[t] += v;
        }
      }
    }
  }
  const bool ovr = a.kind == KIND_OVR;
  const bool binary = a.kind == KIND_BINARY || a.kind == KIND_BINARY_SOFTMAX;
  // the other waves are only needed for an in-kernel class merge (they join its barriers)
  if (wave != 0 && (binary || a.ncb == 1 || a.hrec != nullptr || a.probe == 2)) return;
  // ---- epilogue (wave 0): lane holds classes c0 + g + 4r of row r16 of each tile
  WState st[NB];
  if (wave == 0) {
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int64_t row = row0 + t * 16 + r16;
      if (binary) {
        if (g == 0 && row < a.B) {  // class 0 = the single logit
          const double z = acc[t][0] + a.bias[0];
          double pm;
          if (a.kind == KIND_BINARY) {
            const double p1 = 1.0 / (1.0 + exp(-z)), p0 = 1.0 - p1;
            pm = isnan(p1) ? p1 : (p0 > p1 ? p0 : p1);
          } else {
            const double mm = fabs(z), e0 = exp(-z - mm), e1 = exp(z - mm), s = e0 + e1;
            const double q0 = e0 / s, q1 = e1 / s;
            pm = isnan(s) ? s : (q0 > q1 ? q0 : q1);
          }
          finish_row(a, row, z > 0.0 ? 1 : 0, pm);
        }
        continue;
      }
      double z[4];
      bool nan = false;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = c0 + g + 4 * r;
        z[r] = c < a.K ? acc[t][r] + a.bias[c] : -INFINITY;
        nan |= isnan(z[r]);
      }
      WState S0{z[0], 0.0, c0 + g};
#pragma unroll
      for (int r = 1; r < 4; ++r)
        if (z[r] > S0.m) {
          S0.m = z[r];
          S0.bi = c0 + g + 4 * r;
        }
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) s += ovr ? (z[r] == -INFINITY ? 0.0 : wsigmoid(z[r])) : (S0.m == -INFINITY ? 0.0 : exp(z[r] - S0.m));
      S0.s = s;
      if (S0.m == -INFINITY) S0.bi = 0x7fffffff;
      if (nan) S0.m = NAN;  // a NaN logit makes the row's probability NaN (500, like sklearn -> json)
      S0 = wmerge(S0, wshfl(S0, 16), ovr);
      S0 = wmerge(S0, wshfl(S0, 32), ovr);
      st[t] = S0;
    }
    if (binary) return;
    if (a.probe == 2) {
      if (st[0].m == 12345.678) a.out_p[0] = st[0].s;
      return;
    }
    if (a.hrec != nullptr) {  // host merge: one 32-byte record per (class block, row)
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        const int rl = t * 16 + r16;
        if (g == 0 && row0 + rl < a.B) {
          uint4* dst = a.hrec + ((int64_t)cb * RG + rl) * 2;
          st16_host(dst, pack2(a.hseq, (uint32_t)st[t].bi, st[t].m));
          st16_host(dst + 1, pack2(a.hseq, 0u, st[t].s));
        }
      }
      return;
    }
    if (a.ncb == 1) {
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        const int64_t row = row0 + t * 16 + r16;
        if (g == 0 && row < a.B) finish_row(a, row, st[t].bi, ovr ? wsigmoid(st[t].m) / st[t].s : 1.0 / st[t].s);
      }
      return;
    }
  }
  // ---- class blocks: the last-arriving block of the row group merges them in block order
  unsigned char* rgw2 = a.ws + (int64_t)rgi * a.rg_bytes;
  double* states = reinterpret_cast<double*>(rgw2 + a.cnt_bytes + a.part_bytes);
  if (wave == 0) {
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int rl = t * 16 + r16;
      if (g == 0) {
        double* dst = states + ((int64_t)cb * RG + rl) * 4;
        st16_sc1(dst, __builtin_bit_cast(wu4_t, wd2_t{st[t].m, st[t].s}));
        st16_sc1(dst + 2, wu4_t{(uint32_t)st[t].bi, 0u, 0u, 0u});
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      typedef __attribute__((address_space(1))) unsigned int gu32_t;
      gu32_t* ctr = (gu32_t*)(reinterpret_cast<unsigned int*>(rgw2) + a.ncb);
      const unsigned tk = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = tk == (unsigned)a.ncb - 1;
      if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bcast = last;
    }
  }
  __syncthreads();
  if (!bcast) return;
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // 256 threads: row = tid & 31, part = tid >> 5 merges class blocks part, part + 8, ... in order
  __shared__ double mrg[8][RG][3];
  const int rl = threadIdx.x & 31, part = threadIdx.x >> 5;
  WState M{-INFINITY, 0.0, 0x7fffffff};
  for (int b0 = part; b0 < a.ncb; b0 += 8 * 8) {
    wd2_t ms[8];
    uint32_t bis[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = min(b0 + u * 8, a.ncb - 1);
      const double* src = states + ((int64_t)b * RG + rl) * 4;
      ms[u] = *reinterpret_cast<const wd2_t*>(src);
      bis[u] = *reinterpret_cast<const uint32_t*>(src + 2);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (b0 + u * 8 < a.ncb) M = wmerge(M, WState{ms[u][0], ms[u][1], (int)bis[u]}, ovr);
  }
  mrg[part][rl][0] = M.m;
  mrg[part][rl][1] = M.s;
  mrg[part][rl][2] = __builtin_bit_cast(double, (uint64_t)(uint32_t)M.bi);
  __syncthreads();
  if (threadIdx.x >= RG) return;
  // parts hold interleaved block sets; merging them in part order is a fixed order (deterministic)
  WState R{mrg[0][rl][0], mrg[0][rl][1], (int)(uint32_t)__builtin_bit_cast(uint64_t, mrg[0][rl][2])};
#pragma unroll
  for (int p = 1; p < 8; ++p)
    R = wmerge(R, WState{mrg[p][rl][0], mrg[p][rl][1], (int)(uint32_t)__builtin_bit_cast(uint64_t, mrg[p][rl][2])},
               ovr);
  const int64_t row = row0 + rl;
  if (row < a.B) finish_row(a, row, R.bi, ovr ? wsigmoid(R.m) / R.s : 1.0 / R.s);
}

}  // namespace wide
}  // namespace mlapi
