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
//    fills the chip; the splits are merged IN THE SAME LAUNCH by the last-arriving block of each
//    row block (partials stored write-through (sc1) + relaxed ticket, acquire fence in the reducer:
//    Guideline 16 R1), replacing v1's separate merge kernel (7.3 us of a 18.6 us total);
//  * the epilogue is branch-free per element (kind is a template parameter; a split's partial
//    last chunk is masked to -inf) and uses exp2/rcp; accumulators start at the bias.
//
// Training (multinomial / OvR mini-batch SGD, SURVEY 2.3 K6 at BASELINE config 5 scale) reuses the
// same tiles for its row-stats pass (MODE 2): the online (max, sum-exp, argmax) state, merged
// across class splits like MODE 0, is published as {lse = m + log s, argmax} per row; the fused
// gradient kernel (softmax_grad_dw.hip) consumes it. X_aug may carry extra columns (row stride
// ldx >= F; the forward reads only its first F columns).
#include <hip/hip_runtime.h>

#include <cmath>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

constexpr int CLASS_CHUNK = 64;
constexpr float LOG2E_F = 1.4426950408889634f;
constexpr float LN2_F = 0.6931471805599453f;
constexpr int COUNTER_BYTES = 4096;  // per-row-block arrival counters live at the start of the workspace
constexpr int MERGE_MAX = 8;         // split partials the merging block loads at once (automatic plans: <= 8)

struct RowState {
  float m;  // running max logit (-inf if nothing seen yet)
  float s;  // softmax: sum exp(z - m);  OvR: sum sigmoid(z)
  int bi;   // argmax class (first max wins)
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
  return RowState{__shfl_xor(a.m, off, 64), __shfl_xor(a.s, off, 64), __shfl_xor(a.bi, off, 64)};
}

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

typedef __attribute__((address_space(3))) void lds_void_t;
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
  unsigned int* counters;  // split merge (MODE 0/2)
  float4* partials;        // split merge (MODE 0/2)
  float* Z;                // MODE 1
  float2* rowstat;         // MODE 2 output: {lse, argmax bits}
  float4* rowstate;        // MODE 4 output: {max, sum, argmax bits, 0} (class-sharded TP)
};

// One 64-class chunk against the LDS image `wb`: MFMAs into bias-initialised accumulators, then the
// mode's epilogue. Inlined into the kernel (reference parameters stay in registers).
template <int KS, int NT, int MODE, bool OVR>
__device__ __forceinline__ void compute_chunk(const unsigned char* wb, const bf16x8_t (&xf)[NT][KS], int c0, int c_end,
                                              int q, int col, int64_t row0, int64_t B, int K, const float* bias_lds,
                                              const GemmArgs& a, RowState (&st)[NT]) {
  constexpr bool ovr = OVR;
  // The accumulators start at the bias, which was DMA'd into LDS next to the W chunk (clamped
  // index; classes past the split are masked later), so the epilogue needs no per-element add and
  // no global load sits between the counted waits of the staging pipeline.
  f32x4_t acc[NT][4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const f32x4_t b0 = *reinterpret_cast<const f32x4_t*>(bias_lds + mt * 16 + q * 4);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t][mt] = b0;
  }
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

  // Epilogue: lane owns classes c0 + mt*16 + q*4 + r (i = mt*4 + r, increasing class order) of
  // batch row (t, col). Only a split's last chunk can hold classes >= c_end (wave-uniform test);
  // they are masked to -inf, which every reduction below maps to "absent" (exp2 -> 0,
  // sigmoid -> 0, never the max). No per-element branches: a runtime kind or bound check here
  // made hipcc emit exec-mask branches around every element (SQ_INSTS_VALU 5.4k per wave).
  const bool partial = c0 + CLASS_CHUNK > c_end;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = acc[t][i >> 2][i & 3];
    if (partial) {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = c0 + (i >> 2) * 16 + q * 4 + (i & 3) < c_end ? v[i] : -INFINITY;
    }
    if constexpr (MODE == 1) {
      const int64_t row = row0 + t * 16 + col;
      if (row < B) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int cls = c0 + (i >> 2) * 16 + q * 4 + (i & 3);
          if (cls < c_end) a.Z[row * K + cls] = v[i];
        }
      }
    } else {  // MODE 0 / 2: online (max, sum, first argmax)
      float cm = v[0];
      int ci = 0;
#pragma unroll
      for (int i = 1; i < 16; ++i) {
        const bool gt = v[i] > cm;  // strict: the first (lowest class) maximum wins
        cm = gt ? v[i] : cm;
        ci = gt ? i : ci;
      }
      RowState& S = st[t];
      const bool take = cm > S.m;
      const float m_new = take ? cm : S.m;
      if constexpr (OVR) {
        float add = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float e = __builtin_amdgcn_exp2f(-v[i] * LOG2E_F);  // -inf -> +inf -> sigmoid 0
          add += __builtin_amdgcn_rcpf(1.f + e);
        }
        S.s += add;
      } else {
        const float m2 = m_new * LOG2E_F;
        float add = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) add += __builtin_amdgcn_exp2f(fmaf(v[i], LOG2E_F, -m2));
        // rescale the running sum to the new max (S.m = -inf: nothing accumulated yet)
        const float scale = S.m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(fmaf(S.m, LOG2E_F, -m2));
        S.s = fmaf(S.s, scale, add);
      }
      S.bi = take ? c0 + (ci >> 2) * 16 + q * 4 + (ci & 3) : S.bi;
      S.m = m_new;
    }
  }
}

// KS = F/32 (exact), NT = 16-row N-tiles per wave, MODE: 0 = fused predict epilogue,
// 1 = write logits, 2 = training row stats (see header), 4 = raw online softmax state per row
// (class-sharded TP, merged across ranks by shard.hip).
template <int KS, int NT, int MODE, bool OVR>
__global__ __launch_bounds__(256) void gemm_softmax_kernel(GemmArgs a) {
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
  constexpr int ROWS_PER_BLOCK = 4 * ROWS_PER_WAVE;
  constexpr int F_ = KS * 32;
  constexpr int NCH = F_ / 8;                          // 16-byte chunks per W row
  constexpr int W_BYTES = CLASS_CHUNK * lds_row_stride<KS>();
  constexpr int BUF_BYTES = W_BYTES + CLASS_CHUNK * 4;  // [W chunk][64 f32 bias]
  constexpr int PIECES = CLASS_CHUNK * NCH / 256;      // 16-byte pieces per thread per chunk (== KS)
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF_BYTES + 16];
  int* const flag = reinterpret_cast<int*>(smem + 2 * BUF_BYTES);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int q = lane >> 4;
  const int col = lane & 15;
  constexpr bool ovr = OVR;
  (void)kind;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS_PER_BLOCK + wave * ROWS_PER_WAVE;
  const int c_begin = blockIdx.y * classes_per_split;
  const int c_end = min(K, c_begin + classes_per_split);
  const int c_last = c_begin + ((c_end - 1 - c_begin) / CLASS_CHUNK) * CLASS_CHUNK;  // last chunk start

  bf16x8_t xf[NT][KS];

  // ---- W chunk staging: global -> registers (issue early) -> LDS (write late). Plain unrolled
  // code with ext_vector registers: a lambda capture or HIP_vector_type array goes to scratch.
  // W staging: chunk c + 1 is DMA'd into the idle buffer while chunk c computes (no staging
  // VGPRs, no ds_write pass); the barrier's vmcnt(0) retires it. On the last chunk the (valid)
  // last chunk address is re-loaded instead of branching around the loads.
  // Lane-linear destination: 16-B position P = i*256 + wave*64 + lane holds row P / NCH, in-row
  // position P % NCH, i.e. source chunk lds_pos(row, P % NCH).
#define MLAPI_DMA_CHUNK(C0, BUF)                                                                        \
  _Pragma("unroll") for (int i = 0; i < PIECES; ++i) {                                                  \
    const int p = tid + i * 256;                                                                        \
    const int r = p / NCH;                                                                              \
    const int cls = min((C0) + r, K - 1);                                                               \
    const uint16_t* src = W + (int64_t)cls * F_ + lds_pos<KS>(r, p % NCH) * 8;                          \
    __builtin_amdgcn_global_load_lds((glob_void_t*)src,                                                 \
                                     (lds_void_t*)(smem + (BUF) * BUF_BYTES + (i * 256 + wave * 64) * 16), \
                                     16, 0, 0);                                                         \
  }                                                                                                     \
  /* bias: each wave DMAs 16 floats (lanes 0-15), one more VM op per wave (uniform count) */            \
  if (lane < 16)                                                                                        \
    __builtin_amdgcn_global_load_lds((glob_void_t*)(bias + min((C0) + wave * 16 + lane, K - 1)),       \
                                     (lds_void_t*)(smem + (BUF) * BUF_BYTES + W_BYTES + wave * 64), 4, 0, 0);

  RowState st[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) st[t] = RowState{-INFINITY, 0.f, 0x7fffffff};

  // Two chunks in flight: the prologue DMAs chunks 0 and 1 together (a split of B=1024 has only
  // two, so their latencies overlap instead of adding up); in the loop the DMA of chunk c+2 goes
  // into the buffer chunk c was just read from (after a barrier: WAR), and a COUNTED wait retires
  // chunk c+1 while c+2 stays in flight. Raw s_barrier, not __syncthreads(): the latter's fence
  // waits vmcnt(0) and would drain the in-flight DMA (cdna_hip_programming.md "Pipelining across
  // barriers"); the empty asm statements keep the compiler from moving LDS accesses across it.
#define MLAPI_RAW_BARRIER()          \
  asm volatile("" ::: "memory");     \
  __builtin_amdgcn_s_barrier();      \
  asm volatile("" ::: "memory");
  int buf = 0;
  MLAPI_DMA_CHUNK(c_begin, 0)
  // X fragments for the whole feature range, straight to registers, issued between the DMAs of
  // chunks 0 and 1 so that ONE counted wait retires chunk 0 + X while chunk 1 stays in flight
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int64_t r = row0 + t * 16 + col;
    r = r < B ? r : B - 1;
    const uint16_t* xr = X + r * a.ldx + 8 * q;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)  // X is streamed once: non-temporal, keep the L2 for W
      xf[t][ks] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8_t*>(xr + ks * 32));
  }
  // (the builtin form of s_waitcnt is visible to the compiler's wait insertion, so it does not
  // add a vmcnt(0) for the X registers before the loop; encoding: vmcnt[3:0,15:14], expcnt[6:4],
  // lgkmcnt[11:8] with the other two counters left at "no wait")
  constexpr int kWaitChunk = ((PIECES + 1) & 15) | (7 << 4) | (15 << 8) | (((PIECES + 1) >> 4) << 14);
  constexpr int kWaitAll = (7 << 4) | (15 << 8);
  if (c_begin + CLASS_CHUNK < c_end) {
    MLAPI_DMA_CHUNK(c_begin + CLASS_CHUNK, 1)
    __builtin_amdgcn_s_waitcnt(kWaitChunk);  // chunk 0 + X landed, chunk 1 may still fly
  } else {
    __builtin_amdgcn_s_waitcnt(kWaitAll);
  }
  MLAPI_RAW_BARRIER()
  for (int c0 = c_begin; c0 < c_end; c0 += CLASS_CHUNK) {
    compute_chunk<KS, NT, MODE, OVR>(smem + buf * BUF_BYTES, xf, c0, c_end, q, col, row0, B, K,
                                     reinterpret_cast<const float*>(smem + buf * BUF_BYTES + W_BYTES), a, st);
    if (c0 + 2 * CLASS_CHUNK < c_end) {
      MLAPI_RAW_BARRIER()  // every wave is done reading `buf`
      MLAPI_DMA_CHUNK(c0 + 2 * CLASS_CHUNK, buf)
      __builtin_amdgcn_s_waitcnt(kWaitChunk);  // chunk c+1 landed, c+2 flies
    } else {
      __builtin_amdgcn_s_waitcnt(kWaitAll);
    }
    MLAPI_RAW_BARRIER()
    buf ^= 1;
  }
#undef MLAPI_RAW_BARRIER
#undef MLAPI_DMA_CHUNK
  if constexpr (MODE == 0 || MODE == 2 || MODE == 4) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      RowState S = st[t];
      S = merge_state(S, shfl_state(S, 16), ovr);
      S = merge_state(S, shfl_state(S, 32), ovr);
      st[t] = S;
    }
    if (gridDim.y == 1) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int64_t row = row0 + t * 16 + col;
        if (q == 0 && row < B) {
          if constexpr (MODE == 0) {
            a.out_idx[row] = st[t].bi;
            a.out_p[row] = ovr ? sigmoidf_(st[t].m) / st[t].s : 1.f / st[t].s;
          } else if constexpr (MODE == 4) {
            a.rowstate[row] = make_float4(st[t].m, st[t].s, __int_as_float(st[t].bi), 0.f);
          } else {
            a.rowstat[row] = make_float2(st[t].m + __logf(st[t].s), __int_as_float(st[t].bi));
          }
        }
      }
      return;
    }
    // ---- split classes: publish partials, last-arriving block of this row block merges them.
    // Partials are stored write-through (sc1: agent-scope atomic stores into global memory), so
    // no release fence (buffer_wbl2, ~1.7 us per block on the critical path) is needed before the
    // ticket: every storing wave drains (vmcnt(0)), the workgroup barrier orders the waves, then one
    // lane takes the ticket; the merging block keeps its agent acquire (cdna_hip_programming.md
    // Guideline 16, R1).
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int64_t row = row0 + t * 16 + col;
      if (q == 0 && row < B) {
        typedef __attribute__((address_space(1))) unsigned long long gu64_t;
        typedef __attribute__((address_space(1))) unsigned int gu32_t;
        float4* dst = a.partials + (int64_t)blockIdx.y * B + row;
        const unsigned long long ms =
            (unsigned long long)__float_as_uint(st[t].m) | ((unsigned long long)__float_as_uint(st[t].s) << 32);
        __hip_atomic_store((gu64_t*)dst, ms, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((gu32_t*)dst + 2, (unsigned)st[t].bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();
    if (tid == 0) {
      const unsigned ticket =
          __hip_atomic_fetch_add(&a.counters[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = ticket == gridDim.y - 1;
    }
    __syncthreads();
    if (*flag == 0) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&a.counters[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    __syncthreads();
    if (tid < ROWS_PER_BLOCK) {
      const int64_t row = (int64_t)blockIdx.x * ROWS_PER_BLOCK + tid;
      if (row < B) {
        // All splits' partials are issued before the first merge: a load-merge-load chain made each
        // split one more dependent round trip to the memory-side cache (the partials were written
        // by CUs of other XCDs), ~7 of them at B=1024.
        const unsigned ns = gridDim.y;
        float4 p[MERGE_MAX];
#pragma unroll
        for (int sp = 0; sp < MERGE_MAX; ++sp)
          p[sp] = a.partials[(int64_t)min((unsigned)sp, ns - 1) * B + row];  // clamped: unconditional
        RowState S{p[0].x, p[0].y, __float_as_int(p[0].z)};
#pragma unroll
        for (int sp = 1; sp < MERGE_MAX; ++sp)  // fixed split order: deterministic
          if ((unsigned)sp < ns) S = merge_state(S, RowState{p[sp].x, p[sp].y, __float_as_int(p[sp].z)}, ovr);
        for (unsigned sp = MERGE_MAX; sp < ns; ++sp) {  // plans with more splits (forced sweeps)
          const float4 q = a.partials[(int64_t)sp * B + row];
          S = merge_state(S, RowState{q.x, q.y, __float_as_int(q.z)}, ovr);
        }
        if constexpr (MODE == 0) {
          a.out_idx[row] = S.bi;
          a.out_p[row] = ovr ? sigmoidf_(S.m) / S.s : 1.f / S.s;
        } else if constexpr (MODE == 4) {
          a.rowstate[row] = make_float4(S.m, S.s, __int_as_float(S.bi), 0.f);
        } else {
          a.rowstat[row] = make_float2(S.m + __logf(S.s), __int_as_float(S.bi));
        }
      }
    }
  }
}

struct Plan {
  int nt;                 // 16-row tiles per wave
  int splits;
  int classes_per_split;
  int64_t row_blocks;
};

// Benchmark hook (tools/gemm_plan_sweep.py): force (nt, splits); 0 = automatic.
int g_force_nt = 0, g_force_splits = 0;

Plan make_plan(int64_t B, int K, int F, bool training) {
  Plan p;
  // 32 rows per wave (NT = 2) halve the LDS fragment reads per MFMA. It pays once the register
  // staging is gone (LDS-DMA): B=262144 230 -> 172 us, B=8192 about even, B=1024 worse
  // (tools/gemm_plan_sweep.py, profiles/r1_pmc/gemm_plan_sweep_dma.log). KS = 16 at NT = 2 needs
  // all 256 VGPRs.
  (void)training;
  p.nt = (F <= 256 && B >= 16384) ? 2 : 1;
  if (g_force_nt == 1 || g_force_nt == 2) p.nt = g_force_nt;
  if (g_force_splits > 0) {
    const int rows_per_block = 64 * p.nt;
    p.row_blocks = (B + rows_per_block - 1) / rows_per_block;
    const int chunks = (K + CLASS_CHUNK - 1) / CLASS_CHUNK;
    const int sp = g_force_splits > chunks ? chunks : g_force_splits;
    p.classes_per_split = ((chunks + sp - 1) / sp) * CLASS_CHUNK;
    p.splits = (K + p.classes_per_split - 1) / p.classes_per_split;
    if (!(p.splits > 1 && p.row_blocks * 4 > COUNTER_BYTES)) return p;
  }
  const int rows_per_block = 64 * p.nt;
  p.row_blocks = (B + rows_per_block - 1) / rows_per_block;
  const int chunks = (K + CLASS_CHUNK - 1) / CLASS_CHUNK;
  // measured best: B=1024 -> 8 splits (128 blocks), B=8192 -> 4 (512 blocks): fill the chip, but
  // keep >= 2 chunks per block so the LDS double buffer overlaps (the split merge is not free).
  int64_t want = (512 + p.row_blocks - 1) / p.row_blocks;
  if (want > chunks / 2) want = chunks / 2;
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

template <int MODE>
void launch_mode(GemmArgs args, int F, const Plan& plan, hipStream_t stream) {
  const dim3 grid((unsigned)plan.row_blocks, (unsigned)plan.splits);
  args.classes_per_split = plan.classes_per_split;
#define MLAPI_GEMM_LAUNCH(KSV, NTV)                                                                      \
  do {                                                                                                   \
    if (args.kind == KIND_OVR)                                                                           \
      hipLaunchKernelGGL((gemm_softmax_kernel<KSV, NTV, MODE, true>), grid, dim3(256), 0, stream, args); \
    else                                                                                                 \
      hipLaunchKernelGGL((gemm_softmax_kernel<KSV, NTV, MODE, false>), grid, dim3(256), 0, stream, args); \
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
  return a;
}

}  // namespace

void gemm_softmax_force_plan(int nt, int splits) {
  g_force_nt = nt;
  g_force_splits = splits;
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

size_t gemm_softmax_workspace(int64_t B, int K, int F) {
  (void)F;
  const Plan p = make_plan(B, K, F, false);
  return p.splits > 1 ? (size_t)COUNTER_BYTES + (size_t)p.splits * (size_t)B * sizeof(float4) : 0;
}

void launch_gemm_softmax(const void* X, const void* W, const float* b, int64_t B, int F, int K, int kind,
                         int32_t* out_idx, float* out_p, void* workspace, size_t ws_bytes, hipStream_t stream) {
  if (B <= 0) return;
  if (K < 2 || (kind != KIND_MULTINOMIAL && kind != KIND_OVR))
    throw std::invalid_argument("gemm_softmax: multiclass kinds only (binary models use gemv_binary)");
  const Plan plan = make_plan(B, K, F, false);
  if (plan.splits > 1 && ws_bytes < gemm_softmax_workspace(B, K, F))
    throw std::invalid_argument("gemm_softmax: workspace too small (must be zero-initialised once)");
  GemmArgs args = base_args(X, W, B, F, K, kind);
  args.bias = b;
  args.out_idx = out_idx;
  args.out_p = out_p;
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

void launch_gemm_logits(const void* X, const void* W, const float* b, int64_t B, int F, int K, float* Z,
                        hipStream_t stream) {
  if (B <= 0) return;
  Plan plan = make_plan(B, K, F, false);
  plan.splits = (K + plan.classes_per_split - 1) / plan.classes_per_split;  // no merge needed for logits
  GemmArgs args = base_args(X, W, B, F, K, KIND_MULTINOMIAL);
  args.bias = b;
  args.Z = Z;
  launch_mode<1>(args, F, plan, stream);
}

}  // namespace mlapi
