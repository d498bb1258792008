// Wide-model serving at the reference's precision: z = X W^T + b with
// float64 accumulation on the matrix cores (v_mfma_f64_16x16x4_f64), for rows and weights stored
// as float64 (wide_dtype f64: sklearn's dtype, /root/reference/main.py:21-22 via check_array) or
// float32 (f32 storage, products exact in f64, so the f32 path's only error is the rounding of
// the model and the rows to f32 - no accumulation error), any F, any K, every sklearn kind.
//
// Geometry (serving batches are a few rows, so the kernel is latency bound: spread the weights
// over many CUs and keep every MFMA chain short):
//  * grid = (ncb class blocks x nfs feature splits, row groups of NB 16-row tiles: NB = 1 while
//    that grid fits one block per CU, else 2); a block = 4 waves; a block owns 16 classes x
//    16 NB rows x one feature split, and its 4 waves split that range again, each accumulating
//    the 16 x 16-row tiles of its quarter in f64 MFMAs;
//  * operands straight from memory to registers, 16 bytes per lane per load (f64: 2 features,
//    f32: 4 features converted exactly to f64): lane l loads class (l & 15) and row (l & 15) at
//    feature offset 4*E*step + (l >> 4)*E, and element e of its load is the MFMA's k = l >> 4
//    for the e-th MFMA of the step - the same k permutation for A (W) and B (X);
//  * loads in chunks of U = 4 steps, two chunks in flight (double buffer);
//  * the 4 waves' tiles meet in LDS; feature splits (nfs > 1) are summed by the last-arriving
//    block of the class block (write-through partials, one ticket, agent-coherent sc1 loads of
//    them: Guideline 16), in split order;
//  * epilogue on every wave (the serving batch is latency bound, and one wave running it alone
//    measured ~1.5 us of issue for the block's states and ~2.3 us for the class merge - the
//    per-block timeline of tools/wide_trace.py): wave w takes 4 rows of each tile, one row per
//    16-lane DPP row and one class per lane, so a row's max / first argmax / sum are 4-step DPP
//    all-reductions and every lane evaluates one exponential. Then bias and the sklearn epilogue
//    of `kind` (K = 1 binary kinds: z > 0 and sigma(|z|) / the two-class softmax, exactly as
//    linear_rows.h); multiclass kinds reduce the block's 16 classes to a row state {max,
//    sum exp(z - max) | sum sigmoid(z), first argmax}, and class blocks are merged either on the
//    host (one 32-byte record per block and row, the engine's completer merges in double) or
//    in-kernel by the row group's highest class blocks: 16 / 32 / 64 lanes per row by the number
//    of class blocks (one block per lane at K = 1000; sc1 polls of tagged granules), DPP plus
//    permlane-swap all-reductions, every block's rescaled sum in parallel. Everything in f64,
//    fixed orders.
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
constexpr int RG = 32;     // row slots of a row group's workspace region (a launch's groups use 16 or 32)
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
  // share it): [ncb split tickets | 1 spare] (zero, re-armed by the last arrivers), then
  // [ncb][nfs][2 * 4 * 64] f64 split partial tiles (nfs > 1), then [ncb][32 rows] 32-byte row
  // state granules {m, argmax, epoch} {s, epoch, 0}.
  unsigned char* ws;
  int64_t rg_bytes, cnt_bytes, part_bytes;
  int32_t row_groups;
  int32_t clear_tags; // the merger clears the tags it consumed (set for HIP-graph captures only)
  uint32_t epoch;     // != 0, distinct per launch: the tag of this launch's class-merge granules
  int32_t probe;  // linear_wide_set_probe: measurement 1 = stop after the MFMA loop, 2 = after the
                  // block's row states (before the class merge); fault injection 3 = the merging
                  // block never sees the states (its rows time out after 1 s)
  uint64_t* trace;  // linear_wide_set_trace (measurement, nullptr in production): per block 8 wall-clock
                    // stamps (100 MHz) at entry, MFMA loop done, states published, merge poll begin /
                    // end, rows written, first operands landed, kernel arguments arrived
};

// measurement timeline: lane 0 of the calling wave stamps slot i of its block (vector stores)
__device__ __forceinline__ void wstamp(const WideArgs& a, int i) {
  if (a.trace != nullptr && (threadIdx.x & 63) == 0)
    a.trace[((int64_t)blockIdx.y * (a.ncb * a.nfs) + blockIdx.x) * 8 + i] = wall_clock64();  // no gridDim: the
  // direct-dispatched entries read no implicit argument (direct_dispatch.cpp launch_kernel)
}

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

// all-reductions over the 16 lanes of a DPP row (xor 1 and xor 2 in the quad, then rotations by 4
// and 8 within the row): VALU data movement, no LDS round trip; every lane of the row ends with the
// row's result, in a fixed order per lane (deterministic). Call with the whole wave active.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint64_t lo = dpp_u32<CTRL>((uint32_t)u), hi = dpp_u32<CTRL>((uint32_t)(u >> 32));
  return __builtin_bit_cast(double, lo | (hi << 32));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_ROR4 = 0x124, DPP_ROR8 = 0x128;
__device__ __forceinline__ double row16_max(double v) {  // fmax: a NaN lane is skipped
  v = fmax(v, dpp_f64<DPP_XOR1>(v));
  v = fmax(v, dpp_f64<DPP_XOR2>(v));
  v = fmax(v, dpp_f64<DPP_ROR4>(v));
  return fmax(v, dpp_f64<DPP_ROR8>(v));
}
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_f64<DPP_XOR1>(v);
  v += dpp_f64<DPP_XOR2>(v);
  v += dpp_f64<DPP_ROR4>(v);
  return v + dpp_f64<DPP_ROR8>(v);
}
__device__ __forceinline__ int row16_min(int v) {
  v = min(v, (int)dpp_u32<DPP_XOR1>((uint32_t)v));
  v = min(v, (int)dpp_u32<DPP_XOR2>((uint32_t)v));
  v = min(v, (int)dpp_u32<DPP_ROR4>((uint32_t)v));
  return min(v, (int)dpp_u32<DPP_ROR8>((uint32_t)v));
}
// the value of lane ^ 16 / lane ^ 32 (gfx950 v_permlane16/32_swap with both operands v: each lane
// gets back its own value and its partner's, in an order the test below does not need to know)
__device__ __forceinline__ uint32_t xchg16(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return r[0] == v ? r[1] : r[0];
}
__device__ __forceinline__ uint32_t xchg32(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return r[0] == v ? r[1] : r[0];
}
template <bool X32>
__device__ __forceinline__ double xchg_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint64_t lo = X32 ? xchg32((uint32_t)u) : xchg16((uint32_t)u);
  const uint64_t hi = X32 ? xchg32((uint32_t)(u >> 32)) : xchg16((uint32_t)(u >> 32));
  return __builtin_bit_cast(double, lo | (hi << 32));
}
// all-reductions over groups of lpr = 16 / 32 / 64 lanes (lpr wave-uniform)
__device__ __forceinline__ double lanes_max(double v, int lpr) {
  v = row16_max(v);
  if (lpr >= 32) v = fmax(v, xchg_f64<false>(v));
  if (lpr == 64) v = fmax(v, xchg_f64<true>(v));
  return v;
}
__device__ __forceinline__ double lanes_sum(double v, int lpr) {
  v = row16_sum(v);
  if (lpr >= 32) v += xchg_f64<false>(v);
  if (lpr == 64) v += xchg_f64<true>(v);
  return v;
}
__device__ __forceinline__ int lanes_min(int v, int lpr) {
  v = row16_min(v);
  if (lpr >= 32) v = min(v, (int)xchg16((uint32_t)v));
  if (lpr == 64) v = min(v, (int)xchg32((uint32_t)v));
  return v;
}

typedef __attribute__((address_space(1))) unsigned int gu32_t;
typedef __attribute__((address_space(1))) unsigned long long gu64_t;

// agent-coherent 8-byte load (global_load_dwordx2 sc1): bypasses this CU's L1, so bytes another
// workgroup stored sc1 and drained before its ticket add need no acquire fence (MI355X_MICROARCH.md
// visibility table, first row: sc1 stores, one agent-scope ticket counter, last arriver loads)
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load((gu64_t*)const_cast<double*>(p), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
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
  __shared__ double red[WAVES][NB][64][4];
  __shared__ int bcast;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int cb = blockIdx.x % a.ncb, fs = blockIdx.x / a.ncb, rgi = blockIdx.y;
  const int c0 = cb * CB;
  const int64_t row0 = (int64_t)rgi * (16 * NB);  // a launch's row groups are its NB-tile groups
  if (threadIdx.x < 64) wstamp(a, 0);
  if (a.trace != nullptr && threadIdx.x < 64) {  // measurement only: the kernel arguments arrived
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wstamp(a, 7);
  }
  const int S = a.fsteps;
  const int64_t f0 = ((int64_t)fs * WAVES + wave) * S * STEP + g * E;
  const T* wp = static_cast<const T*>(a.W) + (int64_t)min(c0 + r16, a.K - 1) * a.ldx + f0;
  const T* xp[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t)
    xp[t] = static_cast<const T*>(a.X) + min(row0 + t * 16 + r16, (int64_t)a.B - 1) * a.ldx + f0;

  // the bias of this lane's classes, loaded now so its latency hides under the MFMA loop
  const double bcl = a.bias[min(c0 + (lane & 15), a.K - 1)];
  // one accumulator chain per tile: two chains (even / odd k) measured no faster - the SIMD's f64
  // MFMA pipe, not the chain's dependency, paces the loop (16 MFMAs per wave ~0.88 us after the
  // operands land at F = 256; tools/wide_trace.py, profiles/r5_wide/)
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
  if (a.trace != nullptr && wave == 0) {  // measurement only: the first chunk's operands landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wstamp(a, 6);
  }
  for (int s0 = 0; s0 < S; s0 += 2 * U) {
    load(w1, x1, s0 + U);
    __builtin_amdgcn_sched_barrier(0);  // keep the next chunk's loads in flight over these MFMAs
    mma(w0, x0, s0);
    load(w0, x0, s0 + 2 * U);
    __builtin_amdgcn_sched_barrier(0);
    mma(w1, x1, s0 + U);
  }

  if (wave == 0) wstamp(a, 1);
  if (a.probe == 1) {  // measurement: keep the accumulators alive, store nothing
    if (acc[0][0] == 12345.678) a.out_p[0] = acc[0][1];
    return;
  }
  // ---- the block's tile: the waves' feature quarters meet in LDS
#pragma unroll
  for (int t = 0; t < NB; ++t) *reinterpret_cast<wd4_t*>(&red[wave][t][lane][0]) = acc[t];
  __syncthreads();
  int nred = WAVES;  // partial tiles to sum per element
  // ---- feature splits: the last-arriving block of (row group, class block) sums them in order
  if (a.nfs > 1) {
    unsigned char* rgw = a.ws + (int64_t)rgi * a.rg_bytes;
    double* part = reinterpret_cast<double*>(rgw + a.cnt_bytes) + ((int64_t)cb * a.nfs) * (2 * 4 * 64);
    if (wave == 0) {
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        wd4_t v = *reinterpret_cast<const wd4_t*>(&red[0][t][lane][0]);
#pragma unroll
        for (int w2 = 1; w2 < WAVES; ++w2) v += *reinterpret_cast<const wd4_t*>(&red[w2][t][lane][0]);
        double* dst = part + (int64_t)fs * (2 * 4 * 64) + t * 256 + lane * 4;
        st16_sc1(dst, __builtin_bit_cast(wu4_t, wd2_t{v[0], v[1]}));
        st16_sc1(dst + 2, __builtin_bit_cast(wu4_t, wd2_t{v[2], v[3]}));
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
    if (wave == 0) {  // only wave 0 (the adder) reads the partials
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        wd4_t v = wd4_t{0.0, 0.0, 0.0, 0.0};
        for (int f = 0; f < a.nfs; ++f) {  // split order: deterministic
          const double* src = part + (int64_t)f * (2 * 4 * 64) + t * 256 + lane * 4;
          wd4_t u;  // agent-coherent sc1 loads: no acquire fence (the partials bypass this CU's L1)
#pragma unroll
          for (int k = 0; k < 4; ++k) u[k] = ld_sc1(src + k);
          v += u;
        }
        *reinterpret_cast<wd4_t*>(&red[0][t][lane][0]) = v;
      }
    }
    __syncthreads();
    nred = 1;
  }
  // ---- epilogue, every wave: wave w takes rows 4w .. 4w + 3 of each 16-row tile, one row per
  // 16-lane DPP row (rs = lane >> 4), one class per lane (cl = lane & 15). The tile element of
  // (class cl, row r) sits in lane r + 16 (cl & 3), component cl >> 2, of each wave's accumulator.
  const bool ovr = a.kind == KIND_OVR;
  const bool binary = a.kind == KIND_BINARY || a.kind == KIND_BINARY_SOFTMAX;
  const int rs = lane >> 4, cl = lane & 15;
  const int rows = (int)min<int64_t>((int64_t)a.B - row0, 16 * NB);  // rows of this row group in the launch
  const bool cvalid = c0 + cl < a.K;
  double z[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) {
    const int src = 4 * wave + rs + 16 * (cl & 3);
    double v = red[0][t][src][cl >> 2];
#pragma unroll
    for (int w2 = 1; w2 < WAVES; ++w2)
      if (w2 < nred) v += red[w2][t][src][cl >> 2];
    z[t] = cvalid ? v + bcl : -INFINITY;
  }
  if (binary) {  // K = 1: class 0 is the single logit (z > 0 and the sklearn probabilities, as linear_rows.h)
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int rl = t * 16 + 4 * wave + rs;
      if (cl == 0 && rl < rows) {
        double pm;
        if (a.kind == KIND_BINARY) {
          const double p1 = 1.0 / (1.0 + exp(-z[t])), p0 = 1.0 - p1;
          pm = isnan(p1) ? p1 : (p0 > p1 ? p0 : p1);
        } else {
          const double mm = fabs(z[t]), e0 = exp(-z[t] - mm), e1 = exp(z[t] - mm), s = e0 + e1;
          const double q0 = e0 / s, q1 = e1 / s;
          pm = isnan(s) ? s : (q0 > q1 ? q0 : q1);
        }
        finish_row(a, row0 + rl, z[t] > 0.0 ? 1 : 0, pm);
      }
    }
    return;
  }
  // the row's block state {max, sum over the block's classes of exp(z - max) | sigmoid(z), first
  // argmax}: 16-lane DPP all-reductions in a fixed order (deterministic), one exponential per lane
  // and tile. A NaN logit makes s NaN (fmax skips it), and the row's probability NaN (500, like
  // sklearn -> json); masked classes (z = -inf) add 0.
  WState st[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) {
    const double m = row16_max(z[t]);
    const int bi = row16_min(cvalid && z[t] == m ? c0 + cl : 0x7fffffff);
    // one exponential per lane for either kind (OvR: sigmoid(z) = 1 / (1 + exp(-z)))
    const double e = exp(ovr ? -z[t] : z[t] - m);
    const double s = row16_sum(ovr ? 1.0 / (1.0 + e) : e);
    st[t] = WState{m, s, bi};
  }
  if (a.probe == 2) {
    if (st[0].m == 12345.678) a.out_p[0] = st[0].s;
    return;
  }
  if (a.hrec != nullptr) {  // host merge: one 32-byte record per (class block, row)
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int rl = t * 16 + 4 * wave + rs;
      if (cl == 0 && rl < rows) {
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
      const int rl = t * 16 + 4 * wave + rs;
      if (cl == 0 && rl < rows) finish_row(a, row0 + rl, st[t].bi, ovr ? wsigmoid(st[t].m) / st[t].s : 1.0 / st[t].s);
    }
    return;
  }
  // ---- class blocks: every block publishes its rows' states as two tagged 16-byte granules
  // {m, argmax, epoch} {s, epoch, 0} (write-through sc1 stores; the data is the flag, so no drain,
  // ticket or fence: Guideline 16 R2)
  unsigned char* rgw2 = a.ws + (int64_t)rgi * a.rg_bytes;
  double* states = reinterpret_cast<double*>(rgw2 + a.cnt_bytes + a.part_bytes);
#pragma unroll
  for (int t = 0; t < NB; ++t) {
    const int rl = t * 16 + 4 * wave + rs;
    if (cl == 0 && rl < rows) {
      double* dst = states + ((int64_t)cb * RG + rl) * 4;
      const uint64_t mu = __builtin_bit_cast(uint64_t, st[t].m), su = __builtin_bit_cast(uint64_t, st[t].s);
      st16_sc1(dst, wu4_t{(uint32_t)mu, (uint32_t)(mu >> 32), (uint32_t)st[t].bi, a.epoch});
      st16_sc1(dst + 2, wu4_t{(uint32_t)su, (uint32_t)(su >> 32), 0u, a.epoch});
    }
  }
  if (wave == 0) wstamp(a, 2);
  // ---- the class merge, by the row group's highest class blocks: lpr lanes per row (16 / 32 / 64
  // by the number of class blocks, so a lane takes at most ceil(ncb / lpr) <= 4 blocks - one at
  // K = 1000), lane lb of a row taking blocks lb, lb + lpr, ...; one wave per 64 / lpr rows, 4 waves
  // per merging block, nm = min(ncb, ceil(waves / 4)) merging blocks (rows <= 32: enough, since lpr
  // grows with ncb). The mergers sit at the highest block indices: blocks are dispatched in index
  // order in practice, so their producers are already resident when they poll; the poll is bounded
  // (1 s, then the rows fail with WIDE_TIMEOUT_IDX).
  const int lpr = a.ncb > 32 ? 64 : (a.ncb > 16 ? 32 : 16);
  const int rpw = 64 / lpr;
  const int units = (rows + rpw - 1) / rpw;
  const int nm = min(a.ncb, (units + WAVES - 1) / WAVES);
  const int j = a.ncb - 1 - cb;
  if (j >= nm) return;
  const int unit = j + nm * wave;
  if (unit >= units) return;  // wave-uniform
  const int lb = lane & (lpr - 1);
  const int rl = unit * rpw + lane / lpr;
  const bool live = rl < rows;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)states, 0, a.ncb * RG * 32, 0x00020000);
  auto ldg = [&](int b, int h) -> wu4_t {  // sc1 (aux 16): past this CU's L1, agent-coherent
    return __builtin_bit_cast(wu4_t, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (b * RG + rl) * 32 + h * 16, 0, 16));
  };
  auto gm = [](const wu4_t& v) { return __builtin_bit_cast(double, (uint64_t)v[0] | ((uint64_t)v[1] << 32)); };
  constexpr int MU = 4;  // granule pairs per lane held in registers (ncb <= 4 lpr: one pass)
  const uint64_t t0 = wall_clock64();
  if (wave == 0) wstamp(a, 3);
  bool timeout = false;
  wu4_t g1[MU], g2[MU];
  double m = -INFINITY;  // lane-local first max over its blocks (increasing b), and its class
  int bi = 0x7fffffff;
  for (int b0 = 0; b0 < a.ncb && !timeout; b0 += lpr * MU) {
    for (;;) {  // until every granule of this chunk carries this launch's epoch
      bool ok = true;
#pragma unroll
      for (int u = 0; u < MU; ++u) {
        const int b = b0 + lb + lpr * u;
        if (live && b < a.ncb) {
          g1[u] = ldg(b, 0);
          g2[u] = ldg(b, 1);
        }
      }
#pragma unroll
      for (int u = 0; u < MU; ++u) {
        const int b = b0 + lb + lpr * u;
        if (live && b < a.ncb) ok &= g1[u][3] == a.epoch && g2[u][3] == a.epoch;
      }
      if (__all(ok) && a.probe != 3) break;  // probe 3 (fault injection): the states never arrive
      if (wall_clock64() - t0 > 100000000ull) {  // 1 s at 100 MHz: a block never ran
        timeout = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");  // the next pass loads again
    }
#pragma unroll
    for (int u = 0; u < MU; ++u) {
      const int b = b0 + lb + lpr * u;
      const double mu = live && b < a.ncb ? gm(g1[u]) : -INFINITY;
      const bool take = mu > m;
      m = take ? mu : m;
      bi = take ? (int)g1[u][2] : bi;
    }
  }
  if (wave == 0) wstamp(a, 4);
  const double M = lanes_max(m, lpr);
  const int BI = lanes_min(m == M ? bi : 0x7fffffff, lpr);
  double sl = 0.0;
  if (a.ncb <= lpr * MU) {  // the last poll's granules are the states
#pragma unroll
    for (int u = 0; u < MU; ++u) {
      const int b = lb + lpr * u;
      if (live && b < a.ncb) sl += ovr ? gm(g2[u]) : gm(g2[u]) * exp(gm(g1[u]) - M);  // OvR: no exp
    }
  } else if (live && !timeout) {  // very wide K: every granule has arrived; the sums reloaded
    for (int b = lb; b < a.ncb; b += lpr) sl += ovr ? gm(ldg(b, 1)) : gm(ldg(b, 1)) * exp(gm(ldg(b, 0)) - M);
  }
  const double SS = lanes_sum(sl, lpr);
  // graph captures: clear the consumed tags with write-through stores (no dirty line is left behind
  // to be written back over a later launch's granule) - also after a timeout (the rows already
  // fail) - so the next replay, one epoch baked into its arguments, never merges this replay's
  // states. Captured launches only: an eager launch has an epoch of its own.
  if (a.clear_tags && live) {
    for (int b = lb; b < a.ncb; b += lpr) {
      gu32_t* const tg = (gu32_t*)(states + ((int64_t)b * RG + rl) * 4);
      __hip_atomic_store(tg + 3, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(tg + 7, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (lb == 0 && live) {
    if (timeout) {
      finish_row(a, row0 + rl, WIDE_TIMEOUT_IDX, NAN);
    } else if (ovr) {
      finish_row(a, row0 + rl, BI, wsigmoid(M) / SS);
    } else {  // a branch of its own: the softmax row does not also pay the OvR sigmoid's exp and division
      finish_row(a, row0 + rl, BI, 1.0 / SS);
    }
  }
  if (wave == 0) wstamp(a, 5);
}

}  // namespace wide
}  // namespace mlapi
