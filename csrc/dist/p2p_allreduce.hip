// One-shot P2P all-reduce over IPC-mapped peer buffers; protocol in p2p.h.
#include "p2p.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "mlapi/common.h"

namespace mlapi {
namespace {

constexpr int THREADS = 256;
constexpr int MAX_BLOCKS = 64;  // small grid: ranks sharing one GPU must all be resident at once

struct P2PArgs {
  const unsigned char* peer[P2PAllReduce::MAX_RANKS];  // this epoch's half of every rank's buffer
  uint32_t* peer_flags[P2PAllReduce::MAX_RANKS];       // every rank's flag array (slot = our rank)
  const uint32_t* my_flags;
  uint32_t* status;
  void* out;
  int64_t n;
  int rank, world;
  uint32_t epoch;
  uint64_t timeout_ticks;  // wall_clock64() ticks (100 MHz)
};

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {  // round to nearest even (finite inputs)
  const uint32_t u = __float_as_uint(f);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

// Signal + wait. Returns false when a peer did not arrive within the timeout.
__device__ bool p2p_barrier(const P2PArgs& a) {
  if (blockIdx.x == 0 && (int)threadIdx.x < a.world)
    __hip_atomic_store(a.peer_flags[threadIdx.x] + a.rank, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  if ((int)threadIdx.x < a.world) {
    const uint64_t t0 = wall_clock64();
    while ((int32_t)(__hip_atomic_load(a.my_flags + threadIdx.x, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) -
                     a.epoch) < 0) {
      if (wall_clock64() - t0 > a.timeout_ticks) {
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: peers' data before the reads below
  return ok != 0;
}

// float32: float4 per thread and step, peers summed in rank order (identical on every rank).
__global__ __launch_bounds__(THREADS) void p2p_allreduce_f32(P2PArgs a) {
  if (!p2p_barrier(a)) {
    if (threadIdx.x == 0) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  float* out = static_cast<float*>(a.out);
  const int64_t nv = a.n / 4;
  const int64_t stride = (int64_t)gridDim.x * THREADS;
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < nv; i += stride) {
    float4 s = reinterpret_cast<const float4*>(a.peer[0])[i];
    for (int j = 1; j < a.world; ++j) {
      const float4 v = reinterpret_cast<const float4*>(a.peer[j])[i];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    reinterpret_cast<float4*>(out)[i] = s;
  }
  for (int64_t i = nv * 4 + (int64_t)blockIdx.x * THREADS + threadIdx.x; i < a.n; i += stride) {
    float s = reinterpret_cast<const float*>(a.peer[0])[i];
    for (int j = 1; j < a.world; ++j) s += reinterpret_cast<const float*>(a.peer[j])[i];
    out[i] = s;
  }
}

// bfloat16: 8 elements (16 B) per thread and step, fp32 accumulation, one rounding at the end.
__global__ __launch_bounds__(THREADS) void p2p_allreduce_bf16(P2PArgs a) {
  if (!p2p_barrier(a)) {
    if (threadIdx.x == 0) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  uint16_t* out = static_cast<uint16_t*>(a.out);
  const int64_t nv = a.n / 8;
  const int64_t stride = (int64_t)gridDim.x * THREADS;
  for (int64_t i = (int64_t)blockIdx.x * THREADS + threadIdx.x; i < nv; i += stride) {
    float s[8];
    {
      const uint4 v = reinterpret_cast<const uint4*>(a.peer[0])[i];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s[2 * k] = __uint_as_float(w[k] << 16);
        s[2 * k + 1] = __uint_as_float(w[k] & 0xFFFF0000u);
      }
    }
    for (int j = 1; j < a.world; ++j) {
      const uint4 v = reinterpret_cast<const uint4*>(a.peer[j])[i];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s[2 * k] += __uint_as_float(w[k] << 16);
        s[2 * k + 1] += __uint_as_float(w[k] & 0xFFFF0000u);
      }
    }
    uint4 o;
    o.x = f32_to_bf16(s[0]) | ((uint32_t)f32_to_bf16(s[1]) << 16);
    o.y = f32_to_bf16(s[2]) | ((uint32_t)f32_to_bf16(s[3]) << 16);
    o.z = f32_to_bf16(s[4]) | ((uint32_t)f32_to_bf16(s[5]) << 16);
    o.w = f32_to_bf16(s[6]) | ((uint32_t)f32_to_bf16(s[7]) << 16);
    reinterpret_cast<uint4*>(out)[i] = o;
  }
  for (int64_t i = nv * 8 + (int64_t)blockIdx.x * THREADS + threadIdx.x; i < a.n; i += stride) {
    float s = bf16_to_f32(reinterpret_cast<const uint16_t*>(a.peer[0])[i]);
    for (int j = 1; j < a.world; ++j) s += bf16_to_f32(reinterpret_cast<const uint16_t*>(a.peer[j])[i]);
    out[i] = f32_to_bf16(s);
  }
}

// Self-test: a rank-tagged pattern (exact in f32) into this rank's half 0, and a check of every
// peer's pattern with the exchange's own load path (uncached buffer, system-scope acquire).
__device__ __forceinline__ float selftest_word(int rank, int i) { return (float)(rank * 8192 + (i ^ 0x5a5)); }

__global__ __launch_bounds__(THREADS) void p2p_selftest_write(float* mine, int rank, int corrupt, int nwords) {
  for (int i = blockIdx.x * THREADS + threadIdx.x; i < nwords; i += gridDim.x * THREADS)
    mine[i] = selftest_word(rank, i) + (corrupt && i == 77 ? 1.0f : 0.0f);
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

struct SelftestArgs {
  const float* peer[P2PAllReduce::MAX_RANKS];
  uint32_t* bad;
  int world, nwords;
};

__global__ __launch_bounds__(THREADS) void p2p_selftest_verify(SelftestArgs a) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  uint32_t bad = 0;
  for (int r = 0; r < a.world; ++r)
    for (int i = blockIdx.x * THREADS + threadIdx.x; i < a.nwords; i += gridDim.x * THREADS)
      bad += __hip_atomic_load(a.peer[r] + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != selftest_word(r, i);
  if (bad) __hip_atomic_fetch_add(a.bad, bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

P2PAllReduce::P2PAllReduce(int rank, int world, int device, size_t max_bytes)
    : rank_(rank), world_(world), device_(device), max_bytes_((max_bytes + 255) & ~size_t(255)) {
  if (world < 1 || world > MAX_RANKS || rank < 0 || rank >= world)
    throw std::invalid_argument("P2PAllReduce: need 0 <= rank < world <= 16");
  if (max_bytes == 0) throw std::invalid_argument("P2PAllReduce: max_bytes must be > 0");
  MLAPI_HIP_CHECK(hipSetDevice(device));
  // Uncached: stores go to HBM, so a peer GPU reading over xGMI never sees a stale L2 line.
  MLAPI_HIP_CHECK(hipExtMallocWithFlags(&data_, 2 * max_bytes_, hipDeviceMallocUncached));
  MLAPI_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), FLAG_BYTES, hipDeviceMallocUncached));
  MLAPI_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&status_), 64, hipHostMallocMapped | hipHostMallocCoherent));
  MLAPI_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&status_d_), status_, 0));
  MLAPI_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&selftest_h_), 64, hipHostMallocMapped | hipHostMallocCoherent));
  MLAPI_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&selftest_d_), selftest_h_, 0));
  std::memset(status_, 0, 64);
  std::memset(selftest_h_, 0, 64);
  MLAPI_HIP_CHECK(hipMemset(data_, 0, 2 * max_bytes_));
  MLAPI_HIP_CHECK(hipMemset(flags_, 0, FLAG_BYTES));
  MLAPI_HIP_CHECK(hipDeviceSynchronize());
  peer_data_[rank] = data_;
  peer_flags_[rank] = flags_;
  if (world == 1) ready_ = true;
}

P2PAllReduce::~P2PAllReduce() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (int j = 0; j < world_; ++j) {
    if (!opened_[j]) continue;
    (void)hipIpcCloseMemHandle(peer_data_[j]);
    (void)hipIpcCloseMemHandle(peer_flags_[j]);
  }
  (void)hipFree(data_);
  (void)hipFree(flags_);
  (void)hipHostFree(status_);
  (void)hipHostFree(selftest_h_);
}

int P2PAllReduce::status_now() const { return (int)__atomic_load_n(status_, __ATOMIC_ACQUIRE); }

void P2PAllReduce::selftest_write(int corrupt) {
  MLAPI_HIP_CHECK(hipSetDevice(device_));
  const int nw = (int)std::min<size_t>(SELFTEST_WORDS, max_bytes_ / sizeof(float));
  hipLaunchKernelGGL(p2p_selftest_write, dim3(4), dim3(THREADS), 0, 0, static_cast<float*>(data_), rank_, corrupt, nw);
  MLAPI_HIP_CHECK(hipGetLastError());
  MLAPI_HIP_CHECK(hipDeviceSynchronize());
}

int P2PAllReduce::selftest_verify() {
  if (!ready_) throw std::runtime_error("P2PAllReduce: open_peers() first");
  MLAPI_HIP_CHECK(hipSetDevice(device_));
  SelftestArgs a{};
  for (int j = 0; j < world_; ++j) a.peer[j] = static_cast<const float*>(peer_data_[j]);
  a.bad = selftest_d_;
  a.world = world_;
  a.nwords = (int)std::min<size_t>(SELFTEST_WORDS, max_bytes_ / sizeof(float));
  __atomic_store_n(selftest_h_, 0u, __ATOMIC_RELEASE);
  hipLaunchKernelGGL(p2p_selftest_verify, dim3(4), dim3(THREADS), 0, 0, a);
  MLAPI_HIP_CHECK(hipGetLastError());
  MLAPI_HIP_CHECK(hipDeviceSynchronize());
  return (int)__atomic_load_n(selftest_h_, __ATOMIC_ACQUIRE);
}

static std::string export_handle(void* p) {
  hipIpcMemHandle_t h;
  MLAPI_HIP_CHECK(hipIpcGetMemHandle(&h, p));
  return std::string(reinterpret_cast<const char*>(&h), sizeof h);
}

std::string P2PAllReduce::data_handle() const { return export_handle(data_); }
std::string P2PAllReduce::flag_handle() const { return export_handle(flags_); }

void P2PAllReduce::open_peers(const std::vector<std::string>& data_handles,
                              const std::vector<std::string>& flag_handles) {
  if ((int)data_handles.size() != world_ || (int)flag_handles.size() != world_)
    throw std::invalid_argument("P2PAllReduce::open_peers: one handle per rank expected");
  MLAPI_HIP_CHECK(hipSetDevice(device_));
  for (int j = 0; j < world_; ++j) {
    if (j == rank_ || opened_[j]) continue;
    hipIpcMemHandle_t hd, hf;
    if (data_handles[j].size() != sizeof hd || flag_handles[j].size() != sizeof hf)
      throw std::invalid_argument("P2PAllReduce::open_peers: malformed handle");
    std::memcpy(&hd, data_handles[j].data(), sizeof hd);
    std::memcpy(&hf, flag_handles[j].data(), sizeof hf);
    MLAPI_HIP_CHECK(hipIpcOpenMemHandle(&peer_data_[j], hd, hipIpcMemLazyEnablePeerAccess));
    void* f = nullptr;
    MLAPI_HIP_CHECK(hipIpcOpenMemHandle(&f, hf, hipIpcMemLazyEnablePeerAccess));
    peer_flags_[j] = static_cast<uint32_t*>(f);
    if (peer_data_[j] == nullptr || peer_flags_[j] == nullptr)
      throw std::runtime_error("P2PAllReduce::open_peers: null peer mapping");
    opened_[j] = true;
  }
  ready_ = true;
}

void P2PAllReduce::all_reduce(void* buf, size_t count, int dtype, hipStream_t stream, int timeout_ms) {
  if (!ready_) throw std::runtime_error("P2PAllReduce: open_peers() first");
  const size_t es = dtype == 7 ? 4 : dtype == 9 ? 2 : 0;
  if (es == 0) throw std::invalid_argument("P2PAllReduce: float32 (7) or bfloat16 (9) only");
  const size_t bytes = count * es;
  if (bytes > max_bytes_) throw std::invalid_argument("P2PAllReduce: tensor larger than max_bytes");
  if (reinterpret_cast<uintptr_t>(buf) % 16 != 0) throw std::invalid_argument("P2PAllReduce: 16-byte aligned buffers only");
  if (count == 0) return;
  ++epoch_;
  const size_t half = (size_t)(epoch_ & 1u) * max_bytes_;
  MLAPI_HIP_CHECK(hipSetDevice(device_));
  MLAPI_HIP_CHECK(hipMemcpyAsync(static_cast<unsigned char*>(data_) + half, buf, bytes, hipMemcpyDeviceToDevice, stream));
  P2PArgs a{};
  for (int j = 0; j < world_; ++j) {
    a.peer[j] = static_cast<const unsigned char*>(peer_data_[j]) + half;
    a.peer_flags[j] = peer_flags_[j];
  }
  a.my_flags = flags_;
  a.status = status_d_;
  a.out = buf;
  a.n = (int64_t)count;
  a.rank = rank_;
  a.world = world_;
  a.epoch = epoch_;
  a.timeout_ticks = (uint64_t)(timeout_ms > 0 ? timeout_ms : 60000) * 100000ull;
  const int64_t vec = (int64_t)(count / (es == 4 ? 4 : 8)) + 1;
  const int blocks = (int)std::min<int64_t>(MAX_BLOCKS, (vec + THREADS - 1) / THREADS);
  if (es == 4)
    hipLaunchKernelGGL(p2p_allreduce_f32, dim3(blocks), dim3(THREADS), 0, stream, a);
  else
    hipLaunchKernelGGL(p2p_allreduce_bf16, dim3(blocks), dim3(THREADS), 0, stream, a);
  MLAPI_HIP_CHECK(hipGetLastError());
}

P2PBlockArgs P2PAllReduce::block_exchange(size_t bytes, int nblocks, int timeout_ms) {
  if (!ready_) throw std::runtime_error("P2PAllReduce: open_peers() first");
  if (bytes > max_bytes_) throw std::invalid_argument("P2PAllReduce::block_exchange: slice larger than max_bytes");
  if (nblocks < 1 || nblocks > MAX_FLAG_BLOCKS) throw std::invalid_argument("P2PAllReduce::block_exchange: too many blocks");
  ++epoch_;
  const size_t half = (size_t)(epoch_ & 1u) * max_bytes_;
  P2PBlockArgs a;
  a.mine = reinterpret_cast<float*>(static_cast<unsigned char*>(data_) + half);
  for (int j = 0; j < world_; ++j) {
    a.peer[j] = reinterpret_cast<const float*>(static_cast<const unsigned char*>(peer_data_[j]) + half);
    a.peer_bflags[j] = peer_flags_[j] + FLAG_WORDS_ALLREDUCE;
  }
  a.my_bflags = flags_ + FLAG_WORDS_ALLREDUCE;
  for (int j = 0; j < world_; ++j) a.peer_bflags2[j] = peer_flags_[j] + FLAG_WORDS_ALLREDUCE + (size_t)MAX_RANKS * MAX_FLAG_BLOCKS;
  a.my_bflags2 = flags_ + FLAG_WORDS_ALLREDUCE + (size_t)MAX_RANKS * MAX_FLAG_BLOCKS;
  a.status = status_d_;
  a.rank = rank_;
  a.world = world_;
  a.epoch = epoch_;
  a.timeout_ticks = (uint64_t)(timeout_ms > 0 ? timeout_ms : 60000) * 100000ull;
  static const uint32_t mode = [] {
    const char* e = getenv("MLAPI_P2P_MODE");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  a.mode = mode;
  a.fault_block = fault_next_;
  fault_next_ = -1;
  return a;
}

int P2PAllReduce::status() {
  MLAPI_HIP_CHECK(hipSetDevice(device_));
  MLAPI_HIP_CHECK(hipDeviceSynchronize());
  return status_now();
}

}  // namespace mlapi
