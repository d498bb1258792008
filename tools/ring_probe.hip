// Probe for the resident serving kernel (round 5): how fast can a GPU-resident wave pick up rows
// that CPU threads write into host memory, and answer them through host-mapped records?
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ring_probe.hip -o /tmp/ring_probe -lpthread
//   ring_probe <mode> <threads> <outstanding per thread> <seconds> [hdr_only 0|1] [window]
//     mode pingpong: each thread keeps `outstanding` rows in flight (1 = batch-1 ping-pong) and
//                    prints the completion latency distribution and rows/s
//   ring_probe v2 <waves> 0 <seconds> [depth]: poll-only waves (no rows ever written), e.g. the
//                    host-memory polling load of 8 GPUs x 8 rings on one box
//
// One workgroup (one wave) per ring; ring t belongs to host thread t. A row is F = 4 granules of
// 16 bytes {x_f (f64), pos (u32), 0}: every granule carries the row's ring position, so a wave
// that reads a row while the CPU is still writing it sees a mixed tag and skips it (no header,
// no second round trip). hdr_only = 1 polls granule 0 of each entry first and reads the rest
// only for entries whose granule 0 matched (F x less polling traffic, one more round trip).
// The wave exits on the stop word, when the host's lease word has not moved for 200 ms, or after
// 120 s of wall clock, whichever comes first.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <pthread.h>
#include <x86intrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int F = 4, K = 3, N = 256;  // ring entries per thread (power of two)

struct alignas(16) Granule {
  double x;
  uint32_t pos, pad;
};
struct alignas(16) Rec {
  uint32_t seq;
  int32_t idx;
  double p;
};
struct Ctl {
  uint32_t stop;
  uint32_t lease;
  uint32_t pad[14];
  uint64_t iters[64];  // per ring: poll iterations at exit
  uint64_t rows[64];
};

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

__global__ __launch_bounds__(64) void ring_kernel(const Granule* in, Rec* out, Ctl* ctl, int hdr_only, int window) {
  const int r = blockIdx.x, l = threadIdx.x;
  const Granule* ring = in + (size_t)r * N * F;
  Rec* rec = out + (size_t)r * N;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)ring, 0, N * F * (int)sizeof(Granule), 0x00020000);
  const auto cs = __builtin_amdgcn_make_buffer_rsrc((void*)ctl, 0, (int)sizeof(Ctl), 0x00020000);
  const double W[K][F] = {{0.4, 1.3, -2.1, -1.0}, {0.5, -0.3, -0.2, -0.9}, {-0.9, -1.0, 2.3, 1.9}};
  const double b[K] = {9.4, 1.6, -11.1};
  uint32_t head = 0;
  uint64_t done = 0;  // bit i: entry head + i answered
  uint64_t iters = 0, nrows = 0;
  const uint64_t t_start = wall_clock64();
  uint64_t t_lease = t_start;
  uint32_t lease = 0xffffffffu;
  for (;;) {
    ++iters;
    const uint32_t pos = head + (uint32_t)l;
    const uint32_t e = pos & (N - 1);
    bool want = l < window && !((done >> l) & 1);
    u32x4 g[F];
    bool ok = false;
    if (want) {
      if (hdr_only) {
        g[0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (e * F) * 16, 0, 17));
        ok = g[0][2] == pos;
        if (ok) {
#pragma unroll
          for (int f = 1; f < F; ++f)
            g[f] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (e * F + f) * 16, 0, 17));
#pragma unroll
          for (int f = 1; f < F; ++f) ok = ok && g[f][2] == pos;
        }
      } else {
#pragma unroll
        for (int f = 0; f < F; ++f)
          g[f] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (e * F + f) * 16, 0, 17));
        ok = true;
#pragma unroll
        for (int f = 0; f < F; ++f) ok = ok && g[f][2] == pos;
      }
    }
    const uint64_t m = __ballot(ok);
    if (m) {
      if (ok) {
        double x[F];
#pragma unroll
        for (int f = 0; f < F; ++f) x[f] = __builtin_bit_cast(double, (uint64_t)g[f][0] | ((uint64_t)g[f][1] << 32));
        double z[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          double acc = 0;
#pragma unroll
          for (int f = 0; f < F; ++f) acc = fma(x[f], W[k][f], acc);
          z[k] = acc + b[k];
        }
        int idx = 0;
        double mx = z[0];
        for (int k = 1; k < K; ++k)
          if (z[k] > mx) { mx = z[k]; idx = k; }
        double s = 0;
        for (int k = 0; k < K; ++k) s += exp(z[k] - mx);
        const double p = 1.0 / s;
        const uint64_t pb = __builtin_bit_cast(uint64_t, p);
        const u32x4 v = {pos, (uint32_t)idx, (uint32_t)pb, (uint32_t)(pb >> 32)};
        Rec* dst = rec + e;
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
      }
      nrows += __popcll(m);
      done |= m;
      const uint64_t nd = ~done;
      const int adv = nd == 0 ? 64 : __builtin_ctzll(nd);
      head += (uint32_t)adv;
      done = adv == 64 ? 0 : done >> adv;
    } else {
      __builtin_amdgcn_s_sleep(1);
    }
    if ((iters & 63) == 0) {
      const uint32_t stop = __builtin_amdgcn_raw_buffer_load_b32(cs, 0, 0, 17);
      const uint32_t ls = __builtin_amdgcn_raw_buffer_load_b32(cs, 4, 0, 17);
      const uint64_t now = wall_clock64();
      if (ls != lease) {
        lease = ls;
        t_lease = now;
      }
      // wall_clock64: 100 MHz
      if (stop != 0 || now - t_lease > 20000000ull || now - t_start > 12000000000ull) break;
    }
  }
  if (l == 0) {
    __hip_atomic_store(&ctl->iters[r], iters, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&ctl->rows[r], nrows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}


// v2: one 16-byte granule per lane, 4 lanes per entry (16 entries per wave load: one load
// instruction per poll carries the rows themselves), D polls in flight (a poll issued every RT / D)
template <int D>
__global__ __launch_bounds__(64) void ring2_kernel(const Granule* in, Rec* out, Ctl* ctl, int window) {
  const int r = blockIdx.x, l = threadIdx.x;
  const int ent = l >> 2, f = l & 3;
  Rec* rec = out + (size_t)r * N;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(in + (size_t)r * N * F), 0, N * F * (int)sizeof(Granule), 0x00020000);
  const auto cs = __builtin_amdgcn_make_buffer_rsrc((void*)ctl, 0, (int)sizeof(Ctl), 0x00020000);
  const double W[K][F] = {{0.4, 1.3, -2.1, -1.0}, {0.5, -0.3, -0.2, -0.9}, {-0.9, -1.0, 2.3, 1.9}};
  const double b[K] = {9.4, 1.6, -11.1};
  uint32_t head = 0;
  uint32_t done = 0;  // bit i: entry head + i answered (window <= 16)
  uint64_t iters = 0, nrows = 0;
  const uint64_t t_start = wall_clock64();
  uint64_t t_lease = t_start;
  uint32_t lease = 0xffffffffu;
  u32x4 g[D];
  uint32_t base[D];
  auto issue = [&](int d) {
    base[d] = head;
    const uint32_t e = (head + (uint32_t)ent) & (N - 1);
    g[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (e * F + f) * 16, 0, 17));
  };
#pragma unroll
  for (int d = 0; d < D; ++d) issue(d);
  bool quit = false;
  while (!quit) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      ++iters;
      const uint32_t pos = base[d] + (uint32_t)ent;
      const bool ok = g[d][2] == pos && ent < window;
      const uint64_t m = __ballot(ok);
      // entry j complete iff its 4 lanes matched
      uint32_t full = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) full |= (((m >> (4 * j)) & 0xfull) == 0xfull ? 1u : 0u) << j;
      // relative to the current head (the load was issued at base[d] <= head)
      const uint32_t sh = head - base[d];
      uint32_t fresh = sh >= 16 ? 0u : (full >> sh) & ~done;
      if (fresh) {
        // the entry's leader lane gathers its row
        double x[F];
#pragma unroll
        for (int q = 0; q < F; ++q) {
          const uint32_t lo = __shfl(g[d][0], (l & ~3) + q), hi = __shfl(g[d][1], (l & ~3) + q);
          x[q] = __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
        }
        const int wpos = ent - (int)sh;  // window position of this lane's entry
        if (f == 0 && wpos >= 0 && ((fresh >> wpos) & 1)) {
          double z[K];
#pragma unroll
          for (int k = 0; k < K; ++k) {
            double acc = 0;
#pragma unroll
            for (int q = 0; q < F; ++q) acc = fma(x[q], W[k][q], acc);
            z[k] = acc + b[k];
          }
          int idx = 0;
          double mx = z[0];
          for (int k = 1; k < K; ++k)
            if (z[k] > mx) { mx = z[k]; idx = k; }
          double s = 0;
          for (int k = 0; k < K; ++k) s += exp(z[k] - mx);
          const double p = 1.0 / s;
          const uint64_t pb = __builtin_bit_cast(uint64_t, p);
          const u32x4 v = {pos, (uint32_t)idx, (uint32_t)pb, (uint32_t)(pb >> 32)};
          Rec* dst = rec + (pos & (N - 1));
          asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(dst), "v"(v) : "memory");
        }
        nrows += __popc(fresh);
        done |= fresh;
        const uint32_t nd = ~done;
        const int adv = __builtin_ctz(nd);  // done < 2^16: nd != 0
        head += (uint32_t)adv;
        done >>= adv;
      }
      issue(d);
      if ((iters & 63) == 0) {
        const uint32_t stop = __builtin_amdgcn_raw_buffer_load_b32(cs, 0, 0, 17);
        const uint32_t ls = __builtin_amdgcn_raw_buffer_load_b32(cs, 4, 0, 17);
        const uint64_t now = wall_clock64();
        if (ls != lease) {
          lease = ls;
          t_lease = now;
        }
        if (stop != 0 || now - t_lease > 20000000ull || now - t_start > 12000000000ull) quit = true;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (l == 0) {
    __hip_atomic_store(&ctl->iters[r], iters, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&ctl->rows[r], nrows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double ns_per_tick() {
  auto t0 = std::chrono::steady_clock::now();
  uint64_t c0 = __rdtsc();
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  auto t1 = std::chrono::steady_clock::now();
  uint64_t c1 = __rdtsc();
  return std::chrono::duration<double, std::nano>(t1 - t0).count() / (double)(c1 - c0);
}

// device-memory ring (v2 devmem=1): uncached HBM the CPU writes through the BAR, pushed past the
// host data path with an HDP flush (no read-back: the GPU polls, it sees the rows when they land)
static hsa_agent_t g_gpu, g_cpu;
static bool g_have_gpu = false, g_have_cpu = false;
static hsa_status_t find_agents(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_have_gpu) g_gpu = a, g_have_gpu = true;
  if (t == HSA_DEVICE_TYPE_CPU && !g_have_cpu) g_cpu = a, g_have_cpu = true;
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_dpool(hsa_amd_memory_pool_t p, void* data) {
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) {
    *static_cast<hsa_amd_memory_pool_t*>(data) = p;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: ring_probe v1 <threads> <outstanding> <seconds> [hdr_only] [window]\n"
                    "       ring_probe v2 <threads> <outstanding> <seconds> [depth 1|2|4] [window<=16] [devmem]\n");
    return 2;
  }
  const bool v2 = strcmp(argv[1], "v2") == 0;
  const int T = atoi(argv[2]), OUT = atoi(argv[3]);
  const double secs = atof(argv[4]);
  const int opt = argc > 5 ? atoi(argv[5]) : (v2 ? 1 : 0);  // v1: hdr_only, v2: depth
  const int window = argc > 6 ? atoi(argv[6]) : (v2 ? 16 : 64);
  const int devmem = v2 && argc > 7 ? atoi(argv[7]) : 0;
  // v2 with outstanding 0: poll-only waves (no host writer threads) - the host-memory read load of
  // T busy resident rings, e.g. 64 to stand in for 8 GPUs x 8 rings next to a serving process
  if (T < 1 || T > 64 || OUT < (v2 ? 0 : 1) || OUT > N / 2 || (v2 && (window < 1 || window > 16))) return 2;
  if (v2 && opt != 1 && opt != 2 && opt != 4) return 2;
  Granule* in = nullptr;
  Rec* out;
  Ctl* ctl;
  uint32_t* hdp = nullptr;
  const size_t in_bytes = sizeof(Granule) * N * F * T;
  Granule* din = nullptr;
  if (devmem) {
    CHECK(hipFree(nullptr));
    if (hsa_init() != HSA_STATUS_SUCCESS) return 3;
    hsa_iterate_agents(find_agents, nullptr);
    hsa_amd_hdp_flush_t h{};
    hsa_amd_memory_pool_t pool{};
    if (!g_have_gpu || !g_have_cpu ||
        hsa_agent_get_info(g_gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &h) != HSA_STATUS_SUCCESS ||
        hsa_amd_agent_iterate_memory_pools(g_gpu, find_dpool, &pool) != HSA_STATUS_INFO_BREAK ||
        hsa_amd_memory_pool_allocate(pool, in_bytes, HSA_AMD_MEMORY_POOL_UNCACHED_FLAG, (void**)&in) != HSA_STATUS_SUCCESS ||
        hsa_amd_agents_allow_access(1, &g_cpu, nullptr, in) != HSA_STATUS_SUCCESS) {
      fprintf(stderr, "device ring unavailable\n");
      return 3;
    }
    hdp = h.HDP_MEM_FLUSH_CNTL;
    din = in;
  } else {
    CHECK(hipHostMalloc((void**)&in, in_bytes, hipHostMallocMapped | hipHostMallocCoherent));
  }
  CHECK(hipHostMalloc((void**)&out, sizeof(Rec) * N * T, hipHostMallocMapped | hipHostMallocCoherent));
  CHECK(hipHostMalloc((void**)&ctl, sizeof(Ctl), hipHostMallocMapped | hipHostMallocCoherent));
  memset(in, 0xff, in_bytes);  // pos 0xffffffff never matches a live position
  if (hdp) {
    _mm_sfence();
    *reinterpret_cast<volatile uint32_t*>(hdp) = 1u;
    (void)*reinterpret_cast<volatile uint32_t*>(hdp);
  }
  memset(out, 0xff, sizeof(Rec) * N * T);
  memset(ctl, 0, sizeof(Ctl));
  Rec* dout;
  Ctl* dctl;
  if (!devmem) CHECK(hipHostGetDevicePointer((void**)&din, in, 0));
  CHECK(hipHostGetDevicePointer((void**)&dout, out, 0));
  CHECK(hipHostGetDevicePointer((void**)&dctl, ctl, 0));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  if (!v2)
    hipLaunchKernelGGL(ring_kernel, dim3(T), dim3(64), 0, st, din, dout, dctl, opt, window);
  else if (opt == 1)
    hipLaunchKernelGGL(ring2_kernel<1>, dim3(T), dim3(64), 0, st, din, dout, dctl, window);
  else if (opt == 2)
    hipLaunchKernelGGL(ring2_kernel<2>, dim3(T), dim3(64), 0, st, din, dout, dctl, window);
  else
    hipLaunchKernelGGL(ring2_kernel<4>, dim3(T), dim3(64), 0, st, din, dout, dctl, window);
  CHECK(hipGetLastError());
  const double npt = ns_per_tick();
  std::atomic<bool> go{false}, quit{false};
  std::vector<std::vector<uint32_t>> lat(T);
  std::vector<uint64_t> done(T * 8, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < T && OUT > 0; ++t) {
    th.emplace_back([&, t] {
      Granule* ring = in + (size_t)t * N * F;
      volatile Rec* rec = out + (size_t)t * N;
      std::vector<uint64_t> t0(N);
      lat[t].reserve(1 << 22);
      while (!go.load()) _mm_pause();
      uint32_t next = 0, tail = 0;  // [tail, next) in flight
      auto submit = [&](uint32_t pos) {
        const uint32_t e = pos & (N - 1);
        t0[e] = __rdtsc();
        for (int f = 0; f < F; ++f) {
          alignas(16) Granule g{1.0 + 0.1 * ((pos + f) % 37), pos, 0};
          _mm_store_si128(reinterpret_cast<__m128i*>(&ring[e * F + f]), _mm_load_si128(reinterpret_cast<__m128i*>(&g)));
        }
        if (hdp) {
          _mm_sfence();
          *reinterpret_cast<volatile uint32_t*>(hdp) = 1u;
        }
      };
      for (int i = 0; i < OUT; ++i) submit(next++);
      while (!quit.load(std::memory_order_relaxed)) {
        // completions arrive in any order within the window: scan the in-flight ones
        for (uint32_t p = tail; p != next; ++p) {
          const uint32_t e = p & (N - 1);
          if (t0[e] == 0) continue;
          asm volatile("" ::: "memory");
          if (rec[e].seq == p) {
            lat[t].push_back((uint32_t)(__rdtsc() - t0[e]));
            t0[e] = 0;
            ++done[t * 8];
          }
        }
        while (tail != next && t0[tail & (N - 1)] == 0) ++tail;
        while (next - tail < (uint32_t)OUT) submit(next++);
        _mm_pause();
      }
    });
  }
  go.store(true);
  const auto tb = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count() < secs) {
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
    __atomic_fetch_add(&ctl->lease, 1u, __ATOMIC_RELEASE);
  }
  quit.store(true);
  for (auto& x : th) x.join();
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count();
  __atomic_store_n(&ctl->stop, 1u, __ATOMIC_RELEASE);
  CHECK(hipStreamSynchronize(st));
  std::vector<uint32_t> all;
  uint64_t tot = 0, it = 0;
  for (int t = 0; t < T; ++t) {
    all.insert(all.end(), lat[t].begin(), lat[t].end());
    tot += done[t * 8];
    it += ctl->iters[t];
  }
  std::sort(all.begin(), all.end());
  auto q = [&](double f) { return all.empty() ? 0.0 : all[(size_t)(f * (all.size() - 1))] * npt * 1e-3; };
  printf("{\"kernel\": \"%s\", \"threads\": %d, \"outstanding\": %d, \"opt\": %d, \"window\": %d, \"devmem\": %d, "
         "\"rows_per_s\": %.0f, \"p10_us\": %.2f, \"p50_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f, "
         "\"gpu_polls_per_s_per_ring\": %.0f}\n",
         v2 ? "v2" : "v1", T, OUT, opt, window, devmem, tot / el, q(0.1), q(0.5), q(0.9), q(0.99), it / el / T);
  return 0;
}
