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
//    by the last-arriving block of the class block (write-through partials, one ticket, and
//    agent-coherent sc1 loads of them - or one agent-scope acquire: Guideline 16), in split order;
//  * epilogue per row: bias, then the sklearn epilogue of `kind` (K = 1 binary kinds: z > 0 and
//    sigma(|z|) / the two-class softmax, exactly as linear_rows.h); multiclass kinds reduce the
//    block's 16 classes to a row state {max, sum exp(z - max) | sum sigmoid(z), first argmax} and
//    class blocks are merged either on the host (one 32-byte record per block and row, the
//    engine's completer merges in double in block order) or in-kernel by the last-arriving block
//    of the row group (ticket + sc1 loads), 8 lanes per row: max by compares first, then every
//    block's rescaled sum in parallel and a fixed-order sum tree. Everything in f64.
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

  // the bias of this lane's classes, loaded now so its latency hides under the MFMA loop
  double bz[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bz[r] = a.bias[min(c0 + g + 4 * r, a.K - 1)];
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
    if (wave == 0) {  // only wave 0 (the adder) reads the partials
#pragma unroll
      for (int t = 0; t < NB; ++t) acc[t] = wd4_t{0.0, 0.0, 0.0, 0.0};
      for (int f = 0; f < a.nfs; ++f) {  // split order: deterministic
#pragma unroll
        for (int t = 0; t < NB; ++t) {
          const double* src = part + (int64_t)f * (2 * 4 * 64) + t * 256 + lane * 4;
          wd4_t v;  // agent-coherent sc1 loads: no acquire fence (the partials bypass this CU's L1)
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = ld_sc1(src + k);
          acc[t] += v;
        }
      }
    }
  }
  const bool ovr = a.kind == KIND_OVR;
  const bool binary = a.kind == KIND_BINARY || a.kind == KIND_BINARY_SOFTMAX;
  // the other waves are only needed for an in-kernel class merge (they join its barriers)
  if (wave != 0 && (binary || a.ncb == 1 || a.hrec != nullptr || a.probe == 2 || cb != a.ncb - 1)) return;
  // ---- epilogue (wave 0): lane holds classes c0 + g + 4r of row r16 of each tile. The row's
  // block state {max, sum over the block's classes of exp(z - max) | sigmoid(z), first argmax}:
  // the max (and argmax) first, by compares only, then the 16 exponentials in parallel against
  // it and a fixed-order sum - no dependent chain of exponentials.
  WState st[NB];
  if (wave == 0) {
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int64_t row = row0 + t * 16 + r16;
      if (binary) {
        if (g == 0 && row < a.B) {  // class 0 = the single logit
          const double z = acc[t][0] + bz[0];
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
        z[r] = c0 + g + 4 * r < a.K ? acc[t][r] + bz[r] : -INFINITY;
        nan |= isnan(z[r]);
      }
      double m = z[0];
      int bi = c0 + g;
#pragma unroll
      for (int r = 1; r < 4; ++r)
        if (z[r] > m) {
          m = z[r];
          bi = c0 + g + 4 * r;
        }
#pragma unroll
      for (int off = 16; off <= 32; off <<= 1) {  // the row's 16 classes sit in lanes r16 + 16 g
        const double om = __shfl_xor(m, off, 64);
        const int ob = __shfl_xor(bi, off, 64);
        if (om > m || (om == m && ob < bi)) {
          m = om;
          bi = ob;
        }
      }
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) s += ovr ? wsigmoid(z[r]) : exp(z[r] - m);  // masked classes: z = -inf -> 0
      // a NaN logit makes the row's probability NaN (500, like sklearn -> json)
      const uint64_t nanm = __ballot(nan) >> r16;
      if (nanm & 0x0001000100010001ull) s = NAN;
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      st[t] = WState{m, s, bi};
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
  // ---- class blocks: every block publishes its rows' states as two tagged 16-byte granules
  // {m, argmax, epoch} {s, epoch, 0} (write-through sc1 stores; the data is the flag, so no drain,
  // ticket or fence: Guideline 16 R2), and the row group's LAST class block polls them with sc1 loads
  // and merges. All blocks of a serving launch are co-resident (<= a few hundred blocks of 4
  // waves), and the poll is bounded (1 s, then the rows fail with WIDE_TIMEOUT_IDX).
  unsigned char* rgw2 = a.ws + (int64_t)rgi * a.rg_bytes;
  double* states = reinterpret_cast<double*>(rgw2 + a.cnt_bytes + a.part_bytes);
  if (wave == 0) {
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int rl = t * 16 + r16;
      if (g == 0) {
        double* dst = states + ((int64_t)cb * RG + rl) * 4;
        const uint64_t mu = __builtin_bit_cast(uint64_t, st[t].m), su = __builtin_bit_cast(uint64_t, st[t].s);
        st16_sc1(dst, wu4_t{(uint32_t)mu, (uint32_t)(mu >> 32), (uint32_t)st[t].bi, a.epoch});
        st16_sc1(dst + 2, wu4_t{(uint32_t)su, (uint32_t)(su >> 32), 0u, a.epoch});
      }
    }
  }
  // the merger is the highest block index of the row group: blocks are dispatched in index order in
  // practice, so its producers are already resident when it starts, and a grid far larger than the
  // chip (library calls with huge B) never parks a spinning merger ahead of its own producers
  if (cb != a.ncb - 1) return;
  // merging block, 256 threads: row rl = tid >> 3 (8 rows per wave), part = tid & 7 takes class blocks
  // part, part + 8, ...: the row max by compares and 3 xor shuffles, then every block's
  // s * exp(m - max) in parallel, summed per lane in block order and over the 8 lanes in a
  // fixed xor tree (deterministic).
  const int rows = (int)min<int64_t>((int64_t)a.B - row0, 16 * NB);
  if (8 * wave >= rows) return;  // wave-uniform: no rows of this wave in the launch
  const int rl = threadIdx.x >> 3, part = threadIdx.x & 7;
  const bool live = rl < rows;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)states, 0, a.ncb * RG * 32, 0x00020000);
  auto ldg = [&](int b, int h) -> wu4_t {  // sc1 (aux 16): past this CU's L1, agent-coherent
    return __builtin_bit_cast(wu4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, (b * RG + rl) * 32 + h * 16, 0, 16));
  };
  constexpr int MU = 8;  // states per lane held in registers (ncb <= 64: one pass)
  const uint64_t t0 = wall_clock64();
  bool timeout = false;
  // wait until every granule this wave merges carries this launch's epoch
  wu4_t g1[MU], g2[MU];
  for (int b0 = 0; b0 < a.ncb; b0 += 8 * MU) {
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int u = 0; u < MU; ++u) {
        const int b = b0 + part + 8 * u;
        if (live && b < a.ncb) {
          g1[u] = ldg(b, 0);
          g2[u] = ldg(b, 1);
        }
      }
#pragma unroll
      for (int u = 0; u < MU; ++u) {
        const int b = b0 + part + 8 * u;
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
    if (timeout) break;
  }
  auto gm = [](const wu4_t& v) { return __builtin_bit_cast(double, (uint64_t)v[0] | ((uint64_t)v[1] << 32)); };
  double M = -INFINITY, SS = 0.0;
  int BI = 0x7fffffff;
  bool nan = false;
  auto reduce_max = [&]() {
#pragma unroll
    for (int off = 1; off <= 4; off <<= 1) {
      const double om = __shfl_xor(M, off, 64);
      const int ob = __shfl_xor(BI, off, 64);
      if (om > M || (om == M && ob < BI)) {
        M = om;
        BI = ob;
      }
    }
  };
  if (a.ncb <= 8 * MU) {  // the last poll's granules are the states
#pragma unroll
    for (int u = 0; u < MU; ++u) {
      const int b = part + 8 * u;
      if (live && b < a.ncb) {
        const double m = gm(g1[u]);
        const int bi = (int)g1[u][2];
        nan |= isnan(m);
        if (m > M || (m == M && bi < BI)) {
          M = m;
          BI = bi;
        }
      }
    }
    reduce_max();
#pragma unroll
    for (int u = 0; u < MU; ++u)
      if (live && part + 8 * u < a.ncb) SS += ovr ? gm(g2[u]) : gm(g2[u]) * exp(gm(g1[u]) - M);
  } else if (live) {  // very wide K: every granule has arrived; a max pass, then a sum pass
    for (int b = part; b < a.ncb; b += 8) {
      const wu4_t v = ldg(b, 0);
      const double m = gm(v);
      nan |= isnan(m);
      if (m > M || (m == M && (int)v[2] < BI)) {
        M = m;
        BI = (int)v[2];
      }
    }
    reduce_max();
    for (int b = part; b < a.ncb; b += 8) SS += ovr ? gm(ldg(b, 1)) : gm(ldg(b, 1)) * exp(gm(ldg(b, 0)) - M);
  } else {
    reduce_max();
  }
  // consumed: clear the granules' tags with write-through stores (no dirty line is left behind to
  // be written back over a later launch's granule), so a HIP-graph replay - one epoch baked into
  // its arguments - never merges the previous replay's states. Captured launches only: an eager
  // launch has an epoch of its own, and the kernel's end waits for these stores (+1.1 us at B = 8,
  // profiles/r4_wide_merge/s39_summary.txt)
  // graph captures: clear the consumed tags - also after a timeout (the rows already fail), so the
  // next replay never reads this replay's granules as its own
  if (a.clear_tags && live) {
    for (int b = part; b < a.ncb; b += 8) {
      gu32_t* const t = (gu32_t*)(states + ((int64_t)b * RG + rl) * 4);
      __hip_atomic_store(t + 3, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(t + 7, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (nan) SS = NAN;
  SS += __shfl_xor(SS, 1, 64);
  SS += __shfl_xor(SS, 2, 64);
  SS += __shfl_xor(SS, 4, 64);
  const int64_t row = row0 + rl;
  if (part == 0 && live) {
    if (timeout)
      finish_row(a, row, WIDE_TIMEOUT_IDX, NAN);
    else
      finish_row(a, row, BI, ovr ? wsigmoid(M) / SS : 1.0 / SS);
  }
}

}  // namespace wide
}  // namespace mlapi
