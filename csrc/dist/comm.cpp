// Native RCCL communicator; see comm.h.
#include "comm.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "mlapi/common.h"

namespace mlapi {

struct RcclApi {
  void* handle = nullptr;
  std::string path;
  decltype(&::ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&::ncclCommInitRank) CommInitRank = nullptr;
  decltype(&::ncclCommDestroy) CommDestroy = nullptr;
  decltype(&::ncclCommAbort) CommAbort = nullptr;
  decltype(&::ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&::ncclGetErrorString) GetErrorString = nullptr;
  decltype(&::ncclGetVersion) GetVersion = nullptr;
  decltype(&::ncclAllReduce) AllReduce = nullptr;
  decltype(&::ncclBroadcast) Broadcast = nullptr;
  decltype(&::ncclAllGather) AllGather = nullptr;
  decltype(&::ncclReduceScatter) ReduceScatter = nullptr;
  decltype(&::ncclGroupStart) GroupStart = nullptr;
  decltype(&::ncclGroupEnd) GroupEnd = nullptr;
  decltype(&::ncclCommCount) CommCount = nullptr;
  decltype(&::ncclCommCuDevice) CommCuDevice = nullptr;
  decltype(&::ncclCommUserRank) CommUserRank = nullptr;
};

namespace {

template <typename F>
void bind(void* h, F& fn, const char* name) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  if (fn == nullptr) throw std::runtime_error(std::string("RCCL: missing symbol ") + name);
}

const RcclApi& api() {
  static RcclApi a;
  static std::once_flag once;
  static std::string error;
  std::call_once(once, [] {
    // Prefer the copy PyTorch already mapped (same soname), then the ROCm install.
    const char* candidates[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    for (int i = 0; h == nullptr && i < 3; ++i) h = dlopen(candidates[i], RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) {
      error = std::string("RCCL: cannot load librccl (") + dlerror() + ")";
      return;
    }
    a.handle = h;
    Dl_info info;
    void* sym = dlsym(h, "ncclGetUniqueId");
    if (sym != nullptr && dladdr(sym, &info) && info.dli_fname) a.path = info.dli_fname;
    try {
      bind(h, a.GetUniqueId, "ncclGetUniqueId");
      bind(h, a.CommInitRank, "ncclCommInitRank");
      bind(h, a.CommDestroy, "ncclCommDestroy");
      bind(h, a.CommAbort, "ncclCommAbort");
      bind(h, a.CommGetAsyncError, "ncclCommGetAsyncError");
      bind(h, a.GetErrorString, "ncclGetErrorString");
      bind(h, a.GetVersion, "ncclGetVersion");
      bind(h, a.AllReduce, "ncclAllReduce");
      bind(h, a.Broadcast, "ncclBroadcast");
      bind(h, a.AllGather, "ncclAllGather");
      bind(h, a.ReduceScatter, "ncclReduceScatter");
      bind(h, a.GroupStart, "ncclGroupStart");
      bind(h, a.GroupEnd, "ncclGroupEnd");
      bind(h, a.CommCount, "ncclCommCount");
      bind(h, a.CommCuDevice, "ncclCommCuDevice");
      bind(h, a.CommUserRank, "ncclCommUserRank");
    } catch (const std::exception& e) {
      error = e.what();
      a.handle = nullptr;
    }
  });
  if (a.handle == nullptr) throw std::runtime_error(error.empty() ? "RCCL: unavailable" : error);
  return a;
}

inline ncclComm_t as_comm(void* c) { return static_cast<ncclComm_t>(c); }

}  // namespace

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  const ncclResult_t r = api().GetUniqueId(&id);
  if (r != ncclSuccess) throw std::runtime_error(std::string("ncclGetUniqueId: ") + api().GetErrorString(r));
  return std::string(id.internal, sizeof(id.internal));
}

int RcclComm::version() {
  int v = 0;
  api().GetVersion(&v);
  return v;
}

std::string RcclComm::library_path() { return api().path; }

RcclComm::RcclComm(const std::string& id, int rank, int world, int device)
    : api_(&api()), rank_(rank), world_(world), device_(device) {
  if (id.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("RcclComm: unique id must be 128 bytes");
  if (rank < 0 || rank >= world) throw std::invalid_argument("RcclComm: bad rank");
  MLAPI_HIP_CHECK(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(uid.internal, id.data(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  check(api_->CommInitRank(&c, world, uid, rank), "ncclCommInitRank");
  comm_ = c;
  MLAPI_HIP_CHECK(hipMalloc(&scratch_, sizeof(int)));
  MLAPI_HIP_CHECK(hipMemset(scratch_, 0, sizeof(int)));
}

RcclComm::~RcclComm() {
  if (comm_ != nullptr && !aborted_) api_->CommDestroy(as_comm(comm_));  // abort() already released it
  if (scratch_ != nullptr) (void)hipFree(scratch_);
}

void RcclComm::check(int result, const char* what) {
  if (result != ncclSuccess && result != ncclInProgress)
    throw std::runtime_error(std::string(what) + ": " + api_->GetErrorString(static_cast<ncclResult_t>(result)));
}

void RcclComm::all_reduce(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t stream) {
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  check(api_->AllReduce(send, recv, count, static_cast<ncclDataType_t>(dtype), static_cast<ncclRedOp_t>(op),
                        as_comm(comm_), stream),
        "ncclAllReduce");
}

void RcclComm::broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t stream) {
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  check(api_->Broadcast(send, recv, count, static_cast<ncclDataType_t>(dtype), root, as_comm(comm_), stream),
        "ncclBroadcast");
}

void RcclComm::all_gather(const void* send, void* recv, size_t count_per_rank, int dtype, hipStream_t stream) {
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  check(api_->AllGather(send, recv, count_per_rank, static_cast<ncclDataType_t>(dtype), as_comm(comm_), stream),
        "ncclAllGather");
}

void RcclComm::reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op,
                              hipStream_t stream) {
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  check(api_->ReduceScatter(send, recv, recv_count, static_cast<ncclDataType_t>(dtype),
                            static_cast<ncclRedOp_t>(op), as_comm(comm_), stream),
        "ncclReduceScatter");
}

int RcclComm::comm_count() const {
  int n = 0;
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  const_cast<RcclComm*>(this)->check(api_->CommCount(as_comm(comm_), &n), "ncclCommCount");
  return n;
}

int RcclComm::comm_device() const {
  int d = -1;
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  const_cast<RcclComm*>(this)->check(api_->CommCuDevice(as_comm(comm_), &d), "ncclCommCuDevice");
  return d;
}

int RcclComm::comm_rank() const {
  int r = -1;
  if (aborted_) throw std::runtime_error("RcclComm: communicator aborted");
  const_cast<RcclComm*>(this)->check(api_->CommUserRank(as_comm(comm_), &r), "ncclCommUserRank");
  return r;
}

void RcclComm::group_start() { check(api_->GroupStart(), "ncclGroupStart"); }
void RcclComm::group_end() { check(api_->GroupEnd(), "ncclGroupEnd"); }

bool RcclComm::wait(hipStream_t stream, int timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  int spins = 0;
  for (;;) {
    const hipError_t q = hipStreamQuery(stream);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) MLAPI_HIP_CHECK(q);
    ncclResult_t async = ncclSuccess;
    api_->CommGetAsyncError(as_comm(comm_), &async);
    if ((async != ncclSuccess && async != ncclInProgress) ||
        (timeout_ms > 0 && std::chrono::steady_clock::now() > deadline)) {
      abort();
      return false;
    }
    if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

bool RcclComm::barrier(hipStream_t stream, int timeout_ms) {
  all_reduce(scratch_, scratch_, 1, ncclInt32, ncclSum, stream);
  return wait(stream, timeout_ms);
}

void RcclComm::abort() {
  if (!aborted_ && comm_ != nullptr) {
    api_->CommAbort(as_comm(comm_));
    aborted_ = true;
  }
}

}  // namespace mlapi
