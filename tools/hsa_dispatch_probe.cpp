// Direct AQL dispatch vs hipLaunchKernel for a one-wave serving-style kernel (outputs + done word in
// host memory, host spins on the done word). Same process uses HIP too, like the engine would.
//   hipcc --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -O3 tools/hsa_probe_kernel.hip -o /tmp/probe.hsaco
//   hipcc -O2 tools/hsa_dispatch_probe.cpp -o /tmp/hsa_probe -lhsa-runtime64 && /tmp/hsa_probe /tmp/probe.hsaco
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#define HC(x)                                                                     \
  do {                                                                            \
    hsa_status_t s_ = (x);                                                        \
    if (s_ != HSA_STATUS_SUCCESS) {                                               \
      const char* m_ = nullptr;                                                   \
      hsa_status_string(s_, &m_);                                                 \
      std::fprintf(stderr, "%s failed: %s\n", #x, m_ ? m_ : "?");                \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Found {
  hsa_agent_t gpu{}, cpu{};
  bool have_gpu = false, have_cpu = false;
};

static hsa_status_t find_agents(hsa_agent_t a, void* data) {
  auto* f = static_cast<Found*>(data);
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !f->have_gpu) f->gpu = a, f->have_gpu = true;
  if (t == HSA_DEVICE_TYPE_CPU && !f->have_cpu) f->cpu = a, f->have_cpu = true;
  return HSA_STATUS_SUCCESS;
}

struct Pools {
  hsa_amd_memory_pool_t kernarg{}, fine{};
  bool have_kernarg = false, have_fine = false;
};

static hsa_status_t find_pools(hsa_amd_memory_pool_t p, void* data) {
  auto* f = static_cast<Pools*>(data);
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !f->have_kernarg) f->kernarg = p, f->have_kernarg = true;
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !f->have_fine) f->fine = p, f->have_fine = true;
  return HSA_STATUS_SUCCESS;
}

struct BigArgsH {
  unsigned long long* out;
  unsigned* done;
  unsigned seq;
  unsigned pad;
  unsigned long long payload[440];
};
__global__ void big_hip(const BigArgsH) {
  const BigArgsH* a = (const BigArgsH*)__builtin_amdgcn_kernarg_segment_ptr();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < 440; i += 64) s += a->payload[i];
  a->out[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(a->done, a->seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void hip_flag(int* idx, double* p, unsigned* done, unsigned seq) {
  idx[threadIdx.x] = (int)(threadIdx.x + seq);
  p[threadIdx.x] = 0.5 * threadIdx.x + seq;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s probe.hsaco [iters]\n", argv[0]);
    return 2;
  }
  const int iters = argc > 2 ? std::atoi(argv[2]) : 3000;
  // HIP first (as in the engine), then HSA on the same runtime
  if (hipSetDevice(0) != hipSuccess) return 1;
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  HC(hsa_init());
  Found ag;
  HC(hsa_iterate_agents(find_agents, &ag));
  if (!ag.have_gpu || !ag.have_cpu) return 1;
  Pools pl;
  HC(hsa_amd_agent_iterate_memory_pools(ag.cpu, find_pools, &pl));
  if (!pl.have_kernarg || !pl.have_fine) {
    std::fprintf(stderr, "no kernarg / fine-grained pool\n");
    return 1;
  }
  // code object
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  hsa_code_object_reader_t rd;
  HC(hsa_code_object_reader_create_from_memory(blob.data(), blob.size(), &rd));
  hsa_executable_t ex;
  HC(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex));
  HC(hsa_executable_load_agent_code_object(ex, ag.gpu, rd, nullptr, nullptr));
  HC(hsa_executable_freeze(ex, nullptr));
  hsa_executable_symbol_t sym;
  HC(hsa_executable_get_symbol_by_name(ex, "probe_flag.kd", &ag.gpu, &sym));
  uint64_t kobj = 0;
  uint32_t ka_size = 0, grp = 0, prv = 0;
  HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
  HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &ka_size));
  HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &grp));
  HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &prv));
  std::printf("kernarg segment %u B, group %u, private %u\n", ka_size, grp, prv);
  hsa_queue_t* q;
  HC(hsa_queue_create(ag.gpu, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  // memory: kernarg ring + host-visible outputs
  const int NKA = 64;
  const uint32_t ka_stride = (std::max<uint32_t>(ka_size, 64) + 63) / 64 * 64;
  char* ka = nullptr;
  HC(hsa_amd_memory_pool_allocate(pl.kernarg, (size_t)ka_stride * NKA, 0, (void**)&ka));
  HC(hsa_amd_agents_allow_access(1, &ag.gpu, nullptr, ka));
  int* idx = nullptr;
  double* p = nullptr;
  unsigned* done = nullptr;
  HC(hsa_amd_memory_pool_allocate(pl.fine, 4096, 0, (void**)&idx));
  HC(hsa_amd_memory_pool_allocate(pl.fine, 4096, 0, (void**)&p));
  HC(hsa_amd_memory_pool_allocate(pl.fine, 4096, 0, (void**)&done));
  for (void* m : {(void*)idx, (void*)p, (void*)done}) HC(hsa_amd_agents_allow_access(1, &ag.gpu, nullptr, m));
  std::memset(done, 0, 64);
  unsigned seq = 0;
  long bad = 0;
  // modes: 0 hipLaunchKernel; 1..4 direct AQL with (acquire, release) fence scopes
  const char* names[] = {"hipLaunch", "AQL acq=system rel=agent", "AQL acq=agent rel=agent", "AQL acq=agent rel=none",
                         "AQL acq=none rel=none"};
  const int acq[] = {0, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_NONE};
  const int rel[] = {0, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE};
  std::vector<double> lat[5], api[5];
  long timeouts[5] = {0, 0, 0, 0, 0};
  for (int mode = 0; mode < 5; ++mode) {
    for (int i = 0; i < iters + 50; ++i) {
      ++seq;
      const double t0 = now_us();
      if (mode != 0) {
        char* k = ka + (size_t)(seq % NKA) * ka_stride;
        struct Args {
          int* idx;
          double* p;
          unsigned* done;
          unsigned seq;
        } a{idx, p, done, seq};
        std::memset(k, 0, ka_stride);
        std::memcpy(k, &a, sizeof a);
        const uint64_t wi = hsa_queue_add_write_index_relaxed(q, 1);
        auto* pkt = reinterpret_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (wi & (q->size - 1));
        pkt->setup = 1;  // dimensions
        pkt->workgroup_size_x = 64;
        pkt->workgroup_size_y = 1;
        pkt->workgroup_size_z = 1;
        pkt->reserved0 = 0;
        pkt->grid_size_x = 64;
        pkt->grid_size_y = 1;
        pkt->grid_size_z = 1;
        pkt->private_segment_size = prv;
        pkt->group_segment_size = grp;
        pkt->kernel_object = kobj;
        pkt->kernarg_address = k;
        pkt->reserved2 = 0;
        pkt->completion_signal.handle = 0;
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                (acq[mode] << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (rel[mode] << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | (1u << 16), __ATOMIC_RELEASE);
        hsa_signal_store_relaxed(q->doorbell_signal, (hsa_signal_value_t)wi);
      } else {
        hipLaunchKernelGGL(hip_flag, dim3(1), dim3(64), 0, s, idx, p, done, seq);
      }
      const double t1 = now_us();
      bool to = false;
      while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != seq) {
        if (now_us() - t1 > 200000) {  // a stale kernel argument would never publish this seq
          to = true;
          break;
        }
      }
      const double t2 = now_us();
      if (to) {
        ++timeouts[mode];
        continue;
      }
      for (int l = 0; l < 64; ++l) bad += (idx[l] != (int)(l + seq)) || (p[l] != 0.5 * l + seq);
      if (i >= 50) {
        lat[mode].push_back(t2 - t0);
        api[mode].push_back(t1 - t0);
      }
    }
    if (mode == 0) hipStreamSynchronize(s);
  }
  auto med = [](std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (v.size() - 1))];
  };
  for (int m = 0; m < 5; ++m)
    if (!lat[m].empty())
      std::printf("%-26s: submit %.2f us  launch->done p50 %.2f us  p10 %.2f  p90 %.2f  timeouts %ld\n", names[m],
                  med(api[m], 0.5), med(lat[m], 0.5), med(lat[m], 0.1), med(lat[m], 0.9), timeouts[m]);
    else
      std::printf("%-26s: every launch timed out (%ld)\n", names[m], timeouts[m]);
  std::printf("outputs not visible at done: %ld\n", bad);

  // ---- serving-sized kernel argument (3.5 KB): where the kernarg block lives matters -------------
  struct BigArgs {
    unsigned long long* out;
    unsigned* done;
    unsigned seq;
    unsigned pad;
    unsigned long long payload[440];
  };
  hsa_executable_symbol_t bsym;
  HC(hsa_executable_get_symbol_by_name(ex, "probe_big.kd", &ag.gpu, &bsym));
  uint64_t bobj = 0;
  uint32_t bka = 0;
  HC(hsa_executable_symbol_get_info(bsym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &bobj));
  HC(hsa_executable_symbol_get_info(bsym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &bka));
  const uint32_t bstride = (bka + 255) / 256 * 256;
  char* ka_host = nullptr;
  HC(hsa_amd_memory_pool_allocate(pl.kernarg, (size_t)bstride * NKA, 0, (void**)&ka_host));
  HC(hsa_amd_agents_allow_access(1, &ag.gpu, nullptr, ka_host));
  // device-local kernarg ring the CPU writes through the BAR
  struct GpuPool {
    hsa_amd_memory_pool_t pool{};
    bool have = false;
  } gp;
  HC(hsa_amd_agent_iterate_memory_pools(
      ag.gpu,
      [](hsa_amd_memory_pool_t p, void* d) -> hsa_status_t {
        auto* g = static_cast<GpuPool*>(d);
        hsa_amd_segment_t seg;
        hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
        uint32_t flags = 0;
        hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
        if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !g->have) {
          g->pool = p;
          g->have = true;
        }
        return HSA_STATUS_SUCCESS;
      },
      &gp));
  char* ka_dev = nullptr;
  bool dev_ok = gp.have && hsa_amd_memory_pool_allocate(gp.pool, (size_t)bstride * NKA, 0, (void**)&ka_dev) ==
                               HSA_STATUS_SUCCESS;
  if (dev_ok) dev_ok = hsa_amd_agents_allow_access(1, &ag.cpu, nullptr, ka_dev) == HSA_STATUS_SUCCESS;
  hsa_amd_hdp_flush_t hdp{};
  hsa_agent_get_info(ag.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp);
  std::printf("device kernarg ring: %s, HDP flush register: %s\n", dev_ok ? "yes" : "no",
              hdp.HDP_MEM_FLUSH_CNTL ? "yes" : "no");
  unsigned long long* out = nullptr;
  HC(hsa_amd_memory_pool_allocate(pl.fine, 4096, 0, (void**)&out));
  HC(hsa_amd_agents_allow_access(1, &ag.gpu, nullptr, out));
  const char* bnames[] = {"hipLaunch 3.5KB", "AQL 3.5KB host kernarg", "AQL 3.5KB dev kernarg+hdp",
                          "AQL 3.5KB dev kernarg+hdp+rb"};
  for (int mode = 0; mode < 4; ++mode) {
    if (mode >= 2 && !dev_ok) continue;
    std::vector<double> L, A;
    long wrong = 0, tos = 0;
    for (int i = 0; i < iters + 50; ++i) {
      ++seq;
      BigArgs b{};
      b.out = out;
      b.done = done;
      b.seq = seq;
      unsigned long long expect[64] = {0};
      for (int j = 0; j < 440; ++j) {
        b.payload[j] = (unsigned long long)seq * 1000003ull + (unsigned long long)j * 7919ull;
        expect[j % 64] += b.payload[j];
      }
      const double t0 = now_us();
      if (mode == 0) {
        hipLaunchKernelGGL(HIP_KERNEL_NAME(big_hip), dim3(1), dim3(64), 0, s, *reinterpret_cast<BigArgsH*>(&b));
      } else {
        char* base = mode == 1 ? ka_host : ka_dev;
        char* k = base + (size_t)(seq % NKA) * bstride;
        std::memcpy(k, &b, sizeof b);
        if (mode >= 2) {
          __builtin_ia32_sfence();
          if (hdp.HDP_MEM_FLUSH_CNTL) {
            *(volatile uint32_t*)hdp.HDP_MEM_FLUSH_CNTL = 1u;
            if (mode == 3) (void)*(volatile uint32_t*)hdp.HDP_MEM_FLUSH_CNTL;
          }
        }
        const uint64_t wi = hsa_queue_add_write_index_relaxed(q, 1);
        auto* pkt = reinterpret_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (wi & (q->size - 1));
        pkt->workgroup_size_x = 64;
        pkt->workgroup_size_y = 1;
        pkt->workgroup_size_z = 1;
        pkt->reserved0 = 0;
        pkt->grid_size_x = 64;
        pkt->grid_size_y = 1;
        pkt->grid_size_z = 1;
        pkt->private_segment_size = 0;
        pkt->group_segment_size = 0;
        pkt->kernel_object = bobj;
        pkt->kernarg_address = k;
        pkt->reserved2 = 0;
        pkt->completion_signal.handle = 0;
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | (1u << 16), __ATOMIC_RELEASE);
        hsa_signal_store_relaxed(q->doorbell_signal, (hsa_signal_value_t)wi);
      }
      const double t1 = now_us();
      bool to = false;
      while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != seq) {
        if (now_us() - t1 > 200000) {
          to = true;
          break;
        }
      }
      const double t2 = now_us();
      if (to) {
        ++tos;
        continue;
      }
      for (int l = 0; l < 64; ++l) wrong += out[l] != expect[l];
      if (i >= 50) {
        L.push_back(t2 - t0);
        A.push_back(t1 - t0);
      }
    }
    if (mode == 0) hipStreamSynchronize(s);
    if (L.empty())
      std::printf("%-30s: all timed out\n", bnames[mode]);
    else
      std::printf("%-30s: submit %.2f us  launch->done p50 %.2f us  p90 %.2f  wrong %ld  timeouts %ld\n", bnames[mode],
                  med(A, 0.5), med(L, 0.5), med(L, 0.9), wrong, tos);
  }
  hsa_queue_destroy(q);
  hsa_executable_destroy(ex);
  hsa_code_object_reader_destroy(rd);
  return 0;
}
