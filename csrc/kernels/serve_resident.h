// The resident SMALL-path serving kernel (layouts and protocol: csrc/include/mlapi/resident.h).
// HIP device code, included by serve_direct.hip (entries mlapi_resident_<dt>_r<LPE>_d<D>, launched
// by the engine's supervisor onto a queue of their own: csrc/runtime/direct_dispatch.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "linear_rows.h"
#include "mlapi/kernels.h"
#include "mlapi/resident.h"

namespace mlapi {
namespace resident {

typedef __attribute__((ext_vector_type(4))) uint32_t ru32x4_t;

// One wave per ring (blockIdx.x = the IO thread's ring). T: compute dtype (the SMALL path's f64 =
// sklearn parity, or f32); LPE: lanes per row (F <= LPE); D: polls in flight; KMAX: K bound.
template <typename T, int LPE, int D, int KMAX>
__device__ __forceinline__ void resident_serve(const ResidentArgs& a) {
  static_assert(LPE == 4 || LPE == 8 || LPE == 16 || LPE == 32, "lanes per row");
  constexpr int EPL = 64 / LPE;  // rows per poll (the window)
  constexpr uint64_t LMASK = LPE == 64 ? ~0ull : ((1ull << LPE) - 1);
  __shared__ T s_wb[RESIDENT_FMAX * KMAX + KMAX];  // W [K][F] then b [K]
  __shared__ T s_x[EPL][LPE];                      // the rows of one poll
  const int r = blockIdx.x, l = threadIdx.x;
  const int ent = l / LPE, f = l % LPE;
  const int F = a.F, K = a.K, kind = a.kind;
  {
    const T* W = static_cast<const T*>(a.W);
    const T* b = static_cast<const T*>(a.b);
    for (int i = l; i < K * F; i += 64) s_wb[i] = W[i];
    for (int i = l; i < K; i += 64) s_wb[K * F + i] = b[i];
  }
  __syncthreads();
  const unsigned char* ring = a.rings + (size_t)r * RESIDENT_RING * RESIDENT_ENTRY_BYTES;
  ServeRecord* rec = static_cast<ServeRecord*>(a.recs) + (size_t)r * RESIDENT_RING;
  // aux 17 = sc0 sc1: system scope, past every GPU cache (the rows are host memory a CPU rewrites)
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)ring, 0, RESIDENT_RING * RESIDENT_ENTRY_BYTES, 0x00020000);
  const auto cs = __builtin_amdgcn_make_buffer_rsrc((void*)a.ctl, 0, (int)sizeof(ResidentCtl), 0x00020000);
  uint32_t head = __builtin_amdgcn_readfirstlane(
      __builtin_amdgcn_raw_buffer_load_b32(cs, (int)offsetof(ResidentCtl, heads) + 4 * r, 0, 17));
  uint32_t done = 0;  // bit i: row head + i answered (EPL <= 16 bits)
  uint64_t polls = 0, rows = 0;
  const uint64_t t0 = wall_clock64();
  uint64_t t_lease = t0, t_row = t0;
  uint32_t lease = 0xffffffffu, idle = 0;
  uint32_t fault = RES_FAULT_NONE;  // injected fault (tests), re-read with the stop word
  const bool fetch = f < F;  // lanes past F carry no feature: they do not load and always match
  ru32x4_t g[D];
  uint32_t base[D];
  auto issue = [&](int d) {
    base[d] = head;
    const uint32_t e = (head + (uint32_t)ent) & (RESIDENT_RING - 1);
    g[d] = fetch ? __builtin_bit_cast(ru32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rs, (int)(e * RESIDENT_ENTRY_BYTES + f * 16), 0, 17))
                 : ru32x4_t{0u, 0u, 0u, 0u};
  };
#pragma unroll
  for (int d = 0; d < D; ++d) issue(d);
  bool quit = false;
  while (!quit) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      ++polls;
      const uint32_t pos = base[d] + (uint32_t)ent;
      // The row's width comes from its leader granule (meta & 0xff): lanes past it carry nothing
      // for this row. A stale leader fails its own tag, so a garbage width cannot complete a row.
      const uint32_t row_f = __shfl(g[d][3], l - f) & 0xffu;
      const bool tag_ok = g[d][2] == pos;
      const bool lane_ok = !fetch || (f > 0 && (uint32_t)f >= row_f) || tag_ok;
      const uint64_t mt = __ballot(lane_ok);
      // this instance's model (and so its width): the leader's version matches
      const uint64_t mv = __ballot(f == 0 && fetch && tag_ok && (g[d][3] >> 8) == a.mver);
      uint32_t full = 0, good = 0;  // per row of the poll: every granule written / and for this model
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        full |= (((mt >> (LPE * j)) & LMASK) == LMASK ? 1u : 0u) << j;
        good |= (uint32_t)((mv >> (LPE * j)) & 1ull) << j;
      }
      const uint32_t sh = head - base[d];  // the poll was issued at base[d] <= head
      const uint32_t fresh = sh >= (uint32_t)EPL ? 0u : (full >> sh) & ~done & ((1u << EPL) - 1u);
      if (fresh != 0 && fault != RES_FAULT_STALL) {  // wave-uniform
        const int wpos = ent - (int)sh;  // window position of this lane's row
        const bool mine = wpos >= 0 && ((fresh >> wpos) & 1u);
        if (fetch) s_x[ent][f] = (T)__builtin_bit_cast(double, (uint64_t)g[d][0] | ((uint64_t)g[d][1] << 32));
        __syncthreads();  // one wave: orders the LDS row writes before the leaders' reads
        if (mine && f == 0) {
          int32_t idx = RESIDENT_STALE_IDX;
          T p = T(0);
          if ((good >> ent) & 1u)
            rows::row_predict<T, LPE, KMAX>(&s_x[ent][0], s_wb, s_wb + K * F, F, K, kind, idx, p);
          put_record(rec + (pos & (RESIDENT_RING - 1)), pos, idx, (double)p);
        }
        __syncthreads();  // the next poll's row writes wait for these reads
        rows += (uint64_t)__popc(fresh);
        done |= fresh;
        const int adv = __builtin_ctz(~done);  // done < 2^16: ~done != 0
        head += (uint32_t)adv;
        done >>= adv;
        idle = 0;
        t_row = wall_clock64();
      } else if (++idle > a.idle_polls) {
        // no row for a while (an idle server): slow the polling down, ~3.4 us per s_sleep round
        for (uint32_t s = 0; s < a.idle_sleep; ++s) __builtin_amdgcn_s_sleep(127);
      }
      issue(d);
      if ((polls & 63) == 0) {
        const uint32_t stop = __builtin_amdgcn_raw_buffer_load_b32(cs, (int)offsetof(ResidentCtl, stop), 0, 17);
        const uint32_t ls = __builtin_amdgcn_raw_buffer_load_b32(cs, (int)offsetof(ResidentCtl, lease), 0, 17);
        fault = __builtin_amdgcn_readfirstlane(
            __builtin_amdgcn_raw_buffer_load_b32(cs, (int)offsetof(ResidentCtl, fault), 0, 17));
        const uint64_t now = wall_clock64();
        if (ls != lease) {
          lease = ls;
          t_lease = now;
        }
        if ((stop != 0 && fault != RES_FAULT_IGNORE_STOP) || now - t_lease > a.lease_ticks ||
            (a.idle_exit_ticks != 0 && now - t_row > a.idle_exit_ticks))
          quit = true;
        if (fault == RES_FAULT_EXIT_RING &&
            (uint32_t)r == __builtin_amdgcn_raw_buffer_load_b32(cs, (int)offsetof(ResidentCtl, fault_arg), 0, 17))
          quit = true;
        if (r == 0 && (polls & 1023) == 0 && l == 0 && fault != RES_FAULT_STALL) {
          __hip_atomic_store(&a.ctl->heartbeat, polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(&a.ctl->rows, rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
  // every record of this wave is out before the head that the next instance starts from
  __threadfence_system();
  if (l == 0) {
    __hip_atomic_store(&a.ctl->heads[r], head, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (r == 0) {
      __hip_atomic_store(&a.ctl->heartbeat, polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&a.ctl->rows, rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace resident
}  // namespace mlapi
