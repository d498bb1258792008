// One-shot peer-to-peer all-reduce over IPC-mapped device memory ("a custom
// one-shot P2P all-reduce over IPC peer pointers for the <= 1 MiB training gradients").
//
// Why: every DP collective of this framework is small (the fused [dW | b | loss | correct] buffer
// is <= ~1 MiB), so it is latency bound. RCCL's ring pays 2(N-1) = 14 sequential hops
// on 8 GPUs; on MI355X's full xGMI mesh each rank can instead read all N peers' buffers directly
// (7 links in parallel) and reduce them itself: one hop, one launch.
//
// Protocol (per call, epoch e = 1, 2, ...):
//   1. the caller's tensor is copied into this rank's IPC-exported buffer half (e & 1)
//      (uncached memory: the stores reach HBM, so a peer reading over xGMI sees them);
//   2. one kernel: block 0 publishes e into every peer's flag array (slot = this rank, system-scope
//      release), every block waits until all N flags of its own array reached e (bounded spin:
//      after timeout_ms it records a timeout in the status word and exits - never a hang), then
//      sums the N peers' halves IN RANK ORDER (bitwise-identical results on every rank) into the
//      caller's tensor.
//   Double buffering makes a second barrier unnecessary: a rank overwrites half (e & 1) at epoch
//   e + 2 only after its kernel for e + 1 saw every peer's flag e + 1, which each peer published
//   after its kernel for e (the reads of half (e & 1)) had completed.
//
// Handles (hipIpcMemHandle_t, 64 bytes) are exchanged by the caller over the job's TCP store
// (mlapi_amd/parallel/p2p.py). Peers on the SAME device (several ranks sharing one GPU, as in the
// 1-GPU test box) work through the same code path.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace mlapi {

// Kernel-side view of one fused exchange (p2p_device.h): gradient-reduction kernels store their
// local slice into `mine`, publish it per BLOCK, wait for the same block of every rank and sum the
// ranks' slices in rank order - the all-reduce happens inside the kernel that produced the
// gradient, and the SGD update runs right after it in the same kernel (DP training, VERDICT r2
// next 2). Block b's flag of rank r lives at bflags[b * MAX_RANKS + r] of the receiving rank.
struct P2PBlockArgs {
  static constexpr int MAX_RANKS = 16;
  float* mine = nullptr;                          // this rank's data half of this epoch
  const float* peer[MAX_RANKS] = {};              // every rank's same half (peer[rank] == mine)
  uint32_t* peer_bflags[MAX_RANKS] = {};          // every rank's block-flag array
  const uint32_t* my_bflags = nullptr;
  // Two-shot exchange (large buffers, many ranks): block b's columns are reduced and updated by
  // rank b % world only (reads N-1 peer slices of 1/N of the columns), which publishes the result
  // into `mine + pub_off` and raises its phase-2 flag; the other ranks copy that one slice. Per
  // rank 2 (N-1) / N of the buffer cross xGMI instead of (N-1) x.
  uint32_t* peer_bflags2[MAX_RANKS] = {};         // every rank's phase-2 flag array
  const uint32_t* my_bflags2 = nullptr;
  int64_t pub_off = 0;                            // floats from `mine` / `peer[r]` to the published result
  int two_shot = 0;
  uint32_t* status = nullptr;                     // sticky: 1 = a peer did not arrive in time (host-mapped)
  int rank = 0, world = 1;
  uint32_t epoch = 0;
  uint64_t timeout_ticks = 0;                     // wall_clock64() ticks (100 MHz)
  uint32_t mode = 0;  // bit 0: release fence + release flag store; bit 1: acquire polling (A/B: MLAPI_P2P_MODE)
  int fault_block = -1;  // fault injection (P2PAllReduce::inject_skip_publish): this block never publishes
};

class P2PAllReduce {
 public:
  static constexpr int MAX_RANKS = 16;
  static constexpr int MAX_FLAG_BLOCKS = 4096;  // blocks of a fused-exchange kernel
  P2PAllReduce(int rank, int world, int device, size_t max_bytes);
  ~P2PAllReduce();
  P2PAllReduce(const P2PAllReduce&) = delete;
  P2PAllReduce& operator=(const P2PAllReduce&) = delete;

  // This rank's exported handles: data buffer, flag array (64 bytes each).
  std::string data_handle() const;
  std::string flag_handle() const;
  // Map every peer's buffers (handles indexed by rank; this rank's own entry is ignored).
  void open_peers(const std::vector<std::string>& data_handles, const std::vector<std::string>& flag_handles);

  // In-place sum of `count` elements (dtype: 7 = float32, 9 = bfloat16; RCCL enum values) on
  // `stream`. count * elem_size <= max_bytes.
  void all_reduce(void* buf, size_t count, int dtype, hipStream_t stream, int timeout_ms);
  // 0 = every call so far completed; 1 = a call timed out waiting for a peer (sticky). Syncs.
  int status();
  // The same word as the kernels have published it so far, without synchronising (it lives in
  // host-mapped memory): trainers check it every step and stop at the first missed exchange
  // instead of running on with partly updated replicas.
  int status_now() const;
  // Start-up self-check of the IPC mappings (every rank, between the two calls a host barrier):
  // selftest_write stores a rank-tagged pattern into this rank's buffer (corrupt != 0: a wrong one,
  // for tests); selftest_verify reads every peer's pattern through the mappings with the same
  // uncached / system-scope loads the exchange uses and returns the number of wrong words.
  void selftest_write(int corrupt);
  int selftest_verify();
  // One fused exchange for a kernel of `nblocks` blocks whose slices total `bytes` (advances the
  // epoch; every rank must issue the same sequence of calls).
  P2PBlockArgs block_exchange(size_t bytes, int nblocks, int timeout_ms);
  // Fault injection for the exchange verification (mlapi_amd/parallel/p2p.py): the next
  // block_exchange's block `block` skips its flag publish on this rank (a stale flag for its peers).
  void inject_skip_publish(int block) { fault_next_ = block; }
  uint32_t epoch() const { return epoch_; }
  int world() const { return world_; }
  size_t max_bytes() const { return max_bytes_; }

 private:
  int rank_, world_, device_;
  size_t max_bytes_;
  void* data_ = nullptr;        // 2 halves of max_bytes (uncached, IPC-exported)
  uint32_t* flags_ = nullptr;   // FLAG_WORDS_ALLREDUCE epoch words + block flags (uncached, IPC-exported)
  uint32_t* status_ = nullptr;   // host-mapped word (status_d_ on the device)
  uint32_t* status_d_ = nullptr;
  int fault_next_ = -1;
  uint32_t* selftest_h_ = nullptr;  // host-mapped mismatch counter of selftest_verify
  uint32_t* selftest_d_ = nullptr;
  void* peer_data_[MAX_RANKS] = {};
  uint32_t* peer_flags_[MAX_RANKS] = {};
  bool opened_[MAX_RANKS] = {};
  uint32_t epoch_ = 0;
  bool ready_ = false;

 public:
  static constexpr size_t FLAG_WORDS_ALLREDUCE = 64;  // all_reduce(): one word per source rank
  // [all-reduce epoch words][phase-1 block flags][phase-2 block flags]
  static constexpr size_t FLAG_BYTES = (FLAG_WORDS_ALLREDUCE + 2 * (size_t)MAX_RANKS * MAX_FLAG_BLOCKS) * 4;
  static constexpr int SELFTEST_WORDS = 4096;
};

}  // namespace mlapi
