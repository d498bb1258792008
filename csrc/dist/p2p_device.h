// Device side of the fused per-block P2P exchange (P2PBlockArgs, p2p.h).
//
// A gradient-reduction kernel block that owns columns [c0, c1) of the flat gradient:
//   1. stores its local column sums into a.mine[c0..c1) (uncached memory: the stores reach HBM,
//      where a peer GPU reads them over xGMI);
//   2. p2p_block_sync(a, b): all threads' stores acknowledged (uncached buffer: they are in memory),
//      then one thread per rank stores the epoch into THAT rank's block-flag word for (b, this rank);
//      then threads 0..world-1 spin (bounded) until every rank's flag for block b reached the
//      epoch, followed by a system-scope acquire;
//   3. reads a.peer[0..world)[c0..c1) and sums them in rank order - bitwise the same result on
//      every rank - and applies the optimizer step to its columns.
// Only block b's flags are involved: no grid-wide barrier, the blocks of different ranks pair up
// independently. Double buffering (the epoch parity picks the data half) makes a trailing barrier
// unnecessary: a rank rewrites half (e & 1) at epoch e + 2 only after its block b saw every rank's
// flag e + 1 for block b, which each rank published after its epoch-e kernel (and so its reads of
// that half) had completed in stream order.
// Timeout: the block records status = 1 (sticky; NativeComm / P2PComm check it) and skips its
// update, so a missing peer can never hang the GPU.
#pragma once
#include <hip/hip_runtime.h>

#include "p2p.h"

namespace mlapi {

// Publish this block's slice: every thread's stores acknowledged (the exchange buffer is uncached
// fine-grained memory: an acknowledged store is in memory, where peers read it, so no L2
// write-back is needed before the flag store; P2P_RELEASE_FENCE, mode bit 0, restores the fenced
// protocol for A/B measurements), then one thread per rank stores the epoch into that rank's flag
// word for (block, this rank). phase2: the two-shot result flags instead.
__device__ inline void p2p_block_publish(const P2PBlockArgs& a, int block, bool phase2 = false) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (block == a.fault_block && !phase2) return;  // injected fault: the peers see a stale flag
  if (a.mode & 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if ((int)threadIdx.x < a.world) {
    uint32_t* f = (phase2 ? a.peer_bflags2 : a.peer_bflags)[threadIdx.x] + (size_t)block * P2PBlockArgs::MAX_RANKS + a.rank;
    if (a.mode & 1)
      __hip_atomic_store(f, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      __hip_atomic_store(f, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Wait until every rank's flag for `block` (only_rank >= 0: that rank's) reached the epoch, with a
// bounded spin (timeout: sticky status word, false), then a system-scope acquire so the peer reads
// that follow see this epoch's slices. Every thread of the block calls it.
__device__ inline bool p2p_block_wait(const P2PBlockArgs& a, int block, int only_rank = -1, bool phase2 = false) {
  __shared__ int p2p_ok;
  if (threadIdx.x == 0) p2p_ok = 1;
  __syncthreads();
  const int r = only_rank >= 0 ? only_rank : (int)threadIdx.x;
  if (only_rank >= 0 ? threadIdx.x == 0 : (int)threadIdx.x < a.world) {
    // poll with system-coherent relaxed loads (each acquire load would invalidate the L2 again);
    // one acquire fence after the loop orders the peer reads
    const uint32_t* f = (phase2 ? a.my_bflags2 : a.my_bflags) + (size_t)block * P2PBlockArgs::MAX_RANKS + r;
    const uint64_t t0 = wall_clock64();
    for (;;) {
      const uint32_t v = (a.mode & 2) ? __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)
                                      : __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((int32_t)(v - a.epoch) >= 0) break;
      if (wall_clock64() - t0 > a.timeout_ticks) {
        p2p_ok = 0;
        __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  // system scope: invalidates cached copies of peer lines (an IPC mapping of a peer's buffer may be
  // cacheable on this GPU) so the reads below see this epoch's slices
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return p2p_ok != 0;
}

__device__ inline bool p2p_block_sync(const P2PBlockArgs& a, int block) {
  p2p_block_publish(a, block);
  return p2p_block_wait(a, block);
}

}  // namespace mlapi
