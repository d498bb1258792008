// Native RCCL communicator ("RCCL over xGMI, called directly from C++").
//
// One process per GPU; rank 0 creates the 128-byte unique id and publishes it over a host channel
// (the launcher's TCP store, see mlapi_amd/parallel/rccl.py); every rank then joins with
// ncclCommInitRank on its own device. Collectives run on the HIP stream PyTorch hands us.
//
// librccl is resolved at runtime with dlopen: if PyTorch already loaded its librccl.so.1 the
// SAME library is used (one RCCL per process, so its proxy threads and our comms coexist), else the
// ROCm install's copy. Failure handling: wait() polls the stream with a deadline and,
// on timeout or an asynchronous RCCL error, aborts the communicator (ncclCommAbort) so a dead peer
// turns into an exception instead of a hang.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace mlapi {

struct RcclApi;

class RcclComm {
 public:
  // 128 raw bytes of an ncclUniqueId (call on ONE rank, share with all).
  static std::string unique_id();
  // RCCL version as reported by the loaded library (e.g. 22704), and its path.
  static int version();
  static std::string library_path();

  RcclComm(const std::string& id, int rank, int world, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // dtype / op are RCCL's enum values (ncclFloat32 = 7, ncclSum = 0, ...). In-place when send == recv.
  void all_reduce(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t stream);
  void broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t stream);
  void all_gather(const void* send, void* recv, size_t count_per_rank, int dtype, hipStream_t stream);
  void reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op, hipStream_t stream);
  void group_start();
  void group_end();

  // Block until `stream` drains. Returns false (after aborting the communicator) on timeout or an
  // asynchronous RCCL error; timeout_ms <= 0 waits forever.
  bool wait(hipStream_t stream, int timeout_ms);
  // Device barrier: 1-element all-reduce on a private scratch word + wait().
  bool barrier(hipStream_t stream, int timeout_ms);
  void abort();

  // What RCCL itself reports for this communicator (ncclCommCount / ncclCommCuDevice /
  // ncclCommUserRank): the evidence that a job really runs `world` RCCL ranks.
  int comm_count() const;
  int comm_device() const;
  int comm_rank() const;

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  bool aborted() const { return aborted_; }

 private:
  void check(int result, const char* what);
  const RcclApi* api_;
  void* comm_ = nullptr;
  int rank_, world_, device_;
  bool aborted_ = false;
  int* scratch_ = nullptr;  // barrier word (device memory)
};

}  // namespace mlapi
