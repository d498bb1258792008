// How many tiny serving kernels can one HSA queue take, and does per-IO-thread dispatch scale?
//
// Question behind it: if every HTTP IO thread dispatched its own
// epoll round's rows (instead of handing them to the engine's batcher thread), the GPU would see
// one small launch per IO-thread round - ~1 M launches/s at the node's target rate. This probe
// measures, for a one-wave kernel that writes a 16-byte record to host memory (the serving
// kernels' completion shape) with its kernarg block in device HBM written through the BAR:
//   open:   one thread, M back-to-back packets, no waiting -> packets/s the CP sustains
//   closed: T threads, each in a closed loop (dispatch, spin on its own record, repeat),
//           sharing ONE queue (ticketed packet publication) or each with its OWN queue
//           -> aggregate launches/s and per-launch latency
//   hipcc --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -O3 tools/hsa_probe_kernel.hip -o /tmp/probe.hsaco
//   hipcc -O2 -std=c++17 tools/dispatch_rate_probe.cpp -o /tmp/rate_probe -lhsa-runtime64 -lpthread
//   /tmp/rate_probe /tmp/probe.hsaco
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <mutex>
#include <thread>
#include <vector>

#define HC(x)                                                      \
  do {                                                             \
    hsa_status_t s_ = (x);                                         \
    if (s_ != HSA_STATUS_SUCCESS) {                                \
      const char* m_ = nullptr;                                    \
      hsa_status_string(s_, &m_);                                  \
      std::fprintf(stderr, "%s failed: %s\n", #x, m_ ? m_ : "?"); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Env {
  hsa_agent_t gpu{}, cpu{};
  hsa_amd_memory_pool_t fine{}, dev{};
  bool have_fine = false, have_dev = false;
  uint64_t kobj = 0;
  uint32_t grp = 0, prv = 0;
  volatile uint32_t* hdp = nullptr;
};

struct Args {
  unsigned* rec;
  unsigned seq;
  unsigned pad;
};

// one producer's view of a queue: its kernarg entries (device HBM via the BAR)
struct Producer {
  hsa_queue_t* q = nullptr;
  std::atomic<uint64_t>* publish = nullptr;  // shared queue: next packet id allowed to publish
  char* ka = nullptr;
  uint32_t nka = 0, next = 0;
};

static void dispatch(const Env& e, Producer& p, unsigned* rec, unsigned seq) {
  char* k = p.ka + (size_t)(p.next++ % p.nka) * 256;
  Args a{rec, seq, 0};
  std::memcpy(k, &a, sizeof a);
  _mm_sfence();
  *e.hdp = 1u;
  (void)*e.hdp;
  const uint64_t wi = hsa_queue_add_write_index_relaxed(p.q, 1);
  while (wi - hsa_queue_load_read_index_scacquire(p.q) >= p.q->size) _mm_pause();
  auto* pkt = reinterpret_cast<hsa_kernel_dispatch_packet_t*>(p.q->base_address) + (wi & (p.q->size - 1));
  pkt->workgroup_size_x = 64;
  pkt->workgroup_size_y = 1;
  pkt->workgroup_size_z = 1;
  pkt->reserved0 = 0;
  pkt->grid_size_x = 64;
  pkt->grid_size_y = 1;
  pkt->grid_size_z = 1;
  pkt->private_segment_size = e.prv;
  pkt->group_segment_size = e.grp;
  pkt->kernel_object = e.kobj;
  pkt->kernarg_address = k;
  pkt->reserved2 = 0;
  pkt->completion_signal.handle = 0;
  const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                          (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                          (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  // shared queue: headers (and doorbells) go out in packet order, so the doorbell value the
  // packet processor sees never moves backwards
  if (p.publish)
    while (p.publish->load(std::memory_order_acquire) != wi) _mm_pause();
  __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | (1u << 16), __ATOMIC_RELEASE);
  hsa_signal_store_relaxed(p.q->doorbell_signal, (hsa_signal_value_t)wi);
  if (p.publish) p.publish->store(wi + 1, std::memory_order_release);
}

static bool wait_rec(volatile unsigned* r, unsigned seq, double limit_us) {
  const double t0 = now_us();
  while (*r != seq) {
    if (now_us() - t0 > limit_us) return false;
    _mm_pause();
  }
  return true;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s probe.hsaco\n", argv[0]);
    return 2;
  }
  if (hipSetDevice(0) != hipSuccess) return 1;
  HC(hsa_init());
  Env e;
  HC(hsa_iterate_agents(
      [](hsa_agent_t a, void* d) -> hsa_status_t {
        auto* e = static_cast<Env*>(d);
        hsa_device_type_t t;
        hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
        static bool g = false, c = false;
        if (t == HSA_DEVICE_TYPE_GPU && !g) e->gpu = a, g = true;
        if (t == HSA_DEVICE_TYPE_CPU && !c) e->cpu = a, c = true;
        return HSA_STATUS_SUCCESS;
      },
      &e));
  HC(hsa_amd_agent_iterate_memory_pools(
      e.cpu,
      [](hsa_amd_memory_pool_t p, void* d) -> hsa_status_t {
        auto* e = static_cast<Env*>(d);
        hsa_amd_segment_t seg;
        hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
        uint32_t fl = 0;
        hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
        if (seg == HSA_AMD_SEGMENT_GLOBAL && (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !e->have_fine)
          e->fine = p, e->have_fine = true;
        return HSA_STATUS_SUCCESS;
      },
      &e));
  HC(hsa_amd_agent_iterate_memory_pools(
      e.gpu,
      [](hsa_amd_memory_pool_t p, void* d) -> hsa_status_t {
        auto* e = static_cast<Env*>(d);
        hsa_amd_segment_t seg;
        hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
        uint32_t fl = 0;
        hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
        if (seg == HSA_AMD_SEGMENT_GLOBAL && (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !e->have_dev)
          e->dev = p, e->have_dev = true;
        return HSA_STATUS_SUCCESS;
      },
      &e));
  hsa_amd_hdp_flush_t hdp{};
  HC(hsa_agent_get_info(e.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp));
  if (!e.have_fine || !e.have_dev || !hdp.HDP_MEM_FLUSH_CNTL) {
    std::fprintf(stderr, "missing pool / HDP register\n");
    return 1;
  }
  e.hdp = hdp.HDP_MEM_FLUSH_CNTL;
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  hsa_code_object_reader_t rd;
  HC(hsa_code_object_reader_create_from_memory(blob.data(), blob.size(), &rd));
  hsa_executable_t ex;
  HC(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex));
  HC(hsa_executable_load_agent_code_object(ex, e.gpu, rd, nullptr, nullptr));
  HC(hsa_executable_freeze(ex, nullptr));
  hsa_executable_symbol_t sym;
  HC(hsa_executable_get_symbol_by_name(ex, "probe_rec.kd", &e.gpu, &sym));
  HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &e.kobj));
  HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &e.grp));
  HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &e.prv));

  const int TMAX = 16;
  const uint32_t NKA = 256;  // kernarg entries per producer
  char* ka = nullptr;
  HC(hsa_amd_memory_pool_allocate(e.dev, (size_t)TMAX * NKA * 256, 0, (void**)&ka));
  HC(hsa_amd_agents_allow_access(1, &e.cpu, nullptr, ka));
  const size_t NREC = 1 << 16;
  unsigned* rec = nullptr;
  HC(hsa_amd_memory_pool_allocate(e.fine, NREC * 64, 0, (void**)&rec));
  HC(hsa_amd_agents_allow_access(1, &e.gpu, nullptr, rec));
  std::memset(rec, 0, NREC * 64);
  std::vector<hsa_queue_t*> qs(TMAX);
  for (int t = 0; t < TMAX; ++t)
    HC(hsa_queue_create(e.gpu, 1024, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &qs[t]));
  unsigned seq = 1000;

  // ---- open loop: one thread, M packets, each to its own record
  for (int rep = 0; rep < 2; ++rep) {
    const int M = 20000;
    Producer p;
    p.q = qs[0];
    p.ka = ka;
    p.nka = NKA;
    const unsigned base = ++seq;
    seq += M;
    const double t0 = now_us();
    double issue = 0;
    for (int i = 0; i < M; ++i) {
      // kernarg entry reuse: wait for the packet 256 launches back to have completed
      if (i >= (int)NKA && !wait_rec(rec + (size_t)((i - NKA) % NREC) * 16, base + i - NKA, 1e6)) {
        std::printf("open: timeout at %d\n", i);
        return 1;
      }
      dispatch(e, p, rec + (size_t)(i % NREC) * 16, base + i);
    }
    issue = now_us() - t0;
    bool ok = true;
    for (int i = std::max(0, M - (int)NKA); i < M; ++i) ok &= wait_rec(rec + (size_t)(i % NREC) * 16, base + i, 1e6);
    const double dt = now_us() - t0;
    std::printf("open loop 1 thread : %d packets in %.0f us (issue %.0f us) -> %.2f M packets/s %s\n", M, dt, issue,
                M / dt, ok ? "" : "TIMEOUT");
  }

  // ---- closed loops: T threads, shared queue vs own queues
  for (int shared = 1; shared >= 0; --shared) {
    for (int T : {1, 2, 4, 8, 12, 16}) {
      std::atomic<uint64_t> publish{hsa_queue_load_write_index_scacquire(qs[0])};
      std::atomic<bool> go{false}, stop{false};
      std::vector<std::thread> th;
      std::vector<long> count(T, 0), to(T, 0);
      std::vector<std::vector<double>> lat(T);
      for (int t = 0; t < T; ++t) {
        th.emplace_back([&, t] {
          Producer p;
          p.q = shared ? qs[0] : qs[t];
          p.publish = shared ? &publish : nullptr;
          p.ka = ka + (size_t)t * NKA * 256;
          p.nka = NKA;
          unsigned* r = rec + (size_t)t * 16;
          unsigned s = 1u + (unsigned)t * 100000000u;
          while (!go.load()) _mm_pause();
          while (!stop.load(std::memory_order_relaxed)) {
            ++s;
            const double a = now_us();
            dispatch(e, p, r, s);
            if (!wait_rec(r, s, 2e5)) {
              ++to[t];
              break;
            }
            lat[t].push_back(now_us() - a);
            ++count[t];
          }
        });
      }
      const double t0 = now_us();
      go.store(true);
      std::this_thread::sleep_for(std::chrono::milliseconds(300));
      stop.store(true);
      for (auto& x : th) x.join();
      const double dt = now_us() - t0;
      long n = 0, tos = 0;
      std::vector<double> all;
      for (int t = 0; t < T; ++t) {
        n += count[t];
        tos += to[t];
        all.insert(all.end(), lat[t].begin(), lat[t].end());
      }
      std::sort(all.begin(), all.end());
      auto q = [&](double x) { return all.empty() ? 0.0 : all[(size_t)(x * (all.size() - 1))]; };
      std::printf("closed %-6s queue T=%2d: %.3f M launches/s  latency p50 %.2f p90 %.2f p99 %.2f us  timeouts %ld\n",
                  shared ? "shared" : "own", T, n / dt, q(0.5), q(0.9), q(0.99), tos);
      if (tos) return 1;
    }
  }
  for (auto* q : qs) hsa_queue_destroy(q);
  return 0;
}
