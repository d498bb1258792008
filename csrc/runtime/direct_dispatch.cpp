// HSA side of the engine's direct dispatch (see direct_dispatch.h).
#include "direct_dispatch.h"

#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <fstream>
#include <iterator>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace mlapi {
namespace {

struct Kernel {
  uint64_t object = 0;
  uint32_t group = 0, priv = 0, kernarg = 0;
};

struct AgentSearch {
  uint32_t bdf = 0, domain = 0;  // bdf = bus << 8 | device << 3 | function
  hsa_agent_t gpu{}, cpu{};
  bool have_gpu = false, have_cpu = false;
  int matches = 0;  // GPU agents with this exact domain:bus:device.function (must be 1)
};

hsa_status_t pick_agents(hsa_agent_t a, void* data) {
  auto* s = static_cast<AgentSearch*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !s->have_cpu) {
    s->cpu = a;
    s->have_cpu = true;
  } else if (t == HSA_DEVICE_TYPE_GPU) {
    uint32_t bdf = 0, dom = 0;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
    if (bdf == s->bdf && dom == s->domain) {
      ++s->matches;
      if (!s->have_gpu) {
        s->gpu = a;
        s->have_gpu = true;
      }
    }
  }
  return HSA_STATUS_SUCCESS;
}

// the code object's "mlapi_split_*" / "mlapi_gemv_*" kernels (serve_direct.hip), by name without ".kd"
hsa_status_t collect_split_kernels(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t sym, void* data) {
  hsa_symbol_kind_t kind;
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
      kind != HSA_SYMBOL_KIND_KERNEL)
    return HSA_STATUS_SUCCESS;
  uint32_t len = 0;
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
  std::string name(len, '\0');
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &name[0]);
  if (name.size() > 3 && name.compare(name.size() - 3, 3, ".kd") == 0) name.resize(name.size() - 3);
  if (name.rfind("mlapi_split_", 0) != 0 && name.rfind("mlapi_gemv_", 0) != 0 && name.rfind("mlapi_wide_", 0) != 0 &&
      name.rfind("mlapi_resident_", 0) != 0)
    return HSA_STATUS_SUCCESS;
  Kernel k;
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg);
  (*static_cast<std::unordered_map<std::string, Kernel>*>(data))[name] = k;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t pick_kernarg_pool(hsa_amd_memory_pool_t p, void* data) {
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT)) {
    *static_cast<hsa_amd_memory_pool_t*>(data) = p;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// The GPU's own (coarse-grained) HBM pool: the kernarg ring lives there, written by the CPU
// through the BAR, so the kernel's scalar loads of the 3.6 KB argument block stay on the device.
hsa_status_t pick_device_pool(hsa_amd_memory_pool_t p, void* data) {
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

void queue_error(hsa_status_t, hsa_queue_t*, void* data);
void resident_queue_error(hsa_status_t, hsa_queue_t*, void* data);

class HsaInlineDispatcher final : public InlineDispatcher {
 public:
  ~HsaInlineDispatcher() override {
    // a resident kernel still running (its owner waited and gave up): leave its queue and memory
    // alone - destroying them under a live wave is what the lease rule exists to avoid
    if (rqueue_ && !resident_wait(0)) rqueue_ = nullptr, rkernarg_ = nullptr, rsig_.handle = 0;
    (void)resident_abandoned_done();  // frees the abandoned instances that have ended since
    if (rqueue_) hsa_queue_destroy(rqueue_);
    if (rkernarg_) hsa_amd_memory_pool_free(rkernarg_);
    if (rsig_.handle) hsa_signal_destroy(rsig_);
    if (queue_) hsa_queue_destroy(queue_);
    if (kernargs_) hsa_amd_memory_pool_free(kernargs_);
    for (void* p : bar_bufs_) hsa_amd_memory_pool_free(p);
    if (exe_.handle) hsa_executable_destroy(exe_);
    if (reader_.handle) hsa_code_object_reader_destroy(reader_);
    if (inited_) hsa_shut_down();
  }

  bool init(int device, const std::string& path, int max_in_flight, std::string* why) {
    ka_slots_ = std::max<uint32_t>(64u, 8u * (uint32_t)std::max(1, max_in_flight));
    const uint32_t ka_total = ka_slots_;
    if (const char* e = getenv("MLAPI_HDP_READBACK")) hdp_readback_ = atoi(e) != 0;
    auto fail = [&](const std::string& m) {
      if (why) *why = m;
      return false;
    };
    int bus = 0, dev = 0, dom = 0;
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess)
      return fail("no PCI id for the HIP device");
    (void)hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device);
    // The PCI function matters in partitioned modes (several agents behind one bus:device, each
    // its own function): the full "dddd:bb:dd.f" id names exactly one agent.
    int fn = 0;
    char pci[64] = {0};
    if (hipDeviceGetPCIBusId(pci, sizeof pci, device) == hipSuccess) {
      unsigned d0 = 0, b0 = 0, v0 = 0, f0 = 0;
      if (sscanf(pci, "%x:%x:%x.%x", &d0, &b0, &v0, &f0) == 4 && (int)b0 == bus && (int)v0 == dev) fn = (int)f0;
    }
    if (hsa_init() != HSA_STATUS_SUCCESS) return fail("hsa_init failed");
    inited_ = true;
    AgentSearch s;
    s.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3) | ((uint32_t)fn & 7u);
    s.domain = (uint32_t)dom;
    hsa_iterate_agents(pick_agents, &s);
    if (!s.have_gpu || !s.have_cpu) return fail("HSA agent of the HIP device not found");
    if (s.matches != 1) return fail("HIP device matches " + std::to_string(s.matches) + " HSA agents");
    gpu_ = s.gpu;
    hsa_amd_memory_pool_t pool{};
    if (hsa_amd_agent_iterate_memory_pools(s.cpu, pick_kernarg_pool, &pool) != HSA_STATUS_INFO_BREAK)
      return fail("no kernarg memory pool");
    kpool_ = pool;
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail("code object " + path + " not found");
    blob_.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    if (hsa_code_object_reader_create_from_memory(blob_.data(), blob_.size(), &reader_) != HSA_STATUS_SUCCESS)
      return fail("unreadable code object");
    if (hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe_) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_load_agent_code_object(exe_, gpu_, reader_, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        hsa_executable_freeze(exe_, nullptr) != HSA_STATUS_SUCCESS)
      return fail("code object does not load for this GPU");
    const char* names[6] = {"mlapi_inline_f64_s.kd", "mlapi_inline_f64_w.kd", "mlapi_inline_f32_s.kd",
                            "mlapi_inline_f32_w.kd", "mlapi_inline_f64_4x3.kd", "mlapi_inline_f32_4x3.kd"};
    for (int i = 0; i < 6; ++i) {
      hsa_executable_symbol_t sym;
      if (hsa_executable_get_symbol_by_name(exe_, names[i], &gpu_, &sym) != HSA_STATUS_SUCCESS)
        return fail(std::string("kernel ") + names[i] + " missing");
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k_[i].object);
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k_[i].group);
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k_[i].priv);
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k_[i].kernarg);
      if (k_[i].kernarg < sizeof(InlineBatch) || k_[i].kernarg > stride_) return fail("unexpected kernarg layout");
    }
    hsa_executable_iterate_agent_symbols(exe_, gpu_, collect_split_kernels, &named_);
    if (hsa_queue_create(gpu_, QUEUE_SIZE, HSA_QUEUE_TYPE_SINGLE, queue_error,
                         this, UINT32_MAX, UINT32_MAX, &queue_) != HSA_STATUS_SUCCESS)
      return fail("hsa_queue_create failed");
    // Kernarg ring: a buffer is rewritten KA_SLOTS launches later; the engine keeps at most
    // `slots` (a handful) batches in flight, so its previous kernel has long finished reading it.
    // Preferred home: device HBM (CPU-writable through the BAR; the writes are pushed past the
    // host data path with an HDP flush before the doorbell). Measured on MI355X
    // (profiles/r2_signal/hsa_probe_kernarg.txt), batch-1 launch -> done with a 3.5 KB argument:
    // device ring 6.9 us, hipLaunchKernel 9.5 us, host kernarg pool 14.0 us.
    // MLAPI_KERNARG_HOST=1: the ring in host memory instead - no HDP flush + read-back on the
    // launching (batcher) thread, at the price of the packet processor reading the block over the
    // host link.
    const char* kh = getenv("MLAPI_KERNARG_HOST");
    const bool host_ring = kh != nullptr && atoi(kh) != 0;
    hsa_amd_hdp_flush_t hdp{};
    hsa_amd_memory_pool_t dpool{};
    if (!host_ring && hsa_agent_get_info(gpu_, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp) == HSA_STATUS_SUCCESS &&
        hdp.HDP_MEM_FLUSH_CNTL != nullptr &&
        hsa_amd_agent_iterate_memory_pools(gpu_, pick_device_pool, &dpool) == HSA_STATUS_INFO_BREAK &&
        hsa_amd_memory_pool_allocate(dpool, (size_t)stride_ * ka_total, 0, (void**)&kernargs_) == HSA_STATUS_SUCCESS) {
      if (hsa_amd_agents_allow_access(1, &s.cpu, nullptr, kernargs_) == HSA_STATUS_SUCCESS) {
        hdp_flush_ = hdp.HDP_MEM_FLUSH_CNTL;
        dpool_ = dpool;
        cpu_ = s.cpu;
      } else {
        hsa_amd_memory_pool_free(kernargs_);
        kernargs_ = nullptr;
      }
    }
    if (kernargs_ == nullptr &&
        (hsa_amd_memory_pool_allocate(pool, (size_t)stride_ * ka_total, 0, (void**)&kernargs_) != HSA_STATUS_SUCCESS ||
         hsa_amd_agents_allow_access(1, &gpu_, nullptr, kernargs_) != HSA_STATUS_SUCCESS))
      return fail("kernarg allocation failed");
    std::memset(kernargs_, 0, (size_t)stride_ * ka_total);
    ring_.base = kernargs_;
    ring_.entries = ka_slots_;
    ring_.wi.assign(ka_slots_, ~uint64_t(0));
    return true;
  }

  void launch(int dt, const InlineBatch& a) override {
    if (dt != DT_F64 && dt != DT_F32) throw std::invalid_argument("direct dispatch: f64 / f32 batches only");
    if (faulted()) throw std::runtime_error("direct dispatch: queue error");
    const Kernel& k = (a.F == 4 && a.K == 3) ? k_[dt == DT_F64 ? 4 : 5]  // exact shape: one load batch
                                              : k_[(dt == DT_F64 ? 0 : 2) + (a.F <= 8 && a.K <= 4 ? 0 : 1)];
    uint64_t* wi_slot = nullptr;
    char* ka = next_kernarg(ring_, &wi_slot);
    // Only the bytes the kernel reads: header + W/b of this model + n rows.
    const size_t es = dt == DT_F64 ? 8 : 4;
    const size_t wb_end = offsetof(InlineBatch, wb) + (size_t)a.K * (a.F + 1) * es;
    std::memcpy(ka, &a, wb_end);
    std::memcpy(ka + offsetof(InlineBatch, x), a.x, (size_t)a.n * a.F * es);
    if (a.rec_scatter) std::memcpy(ka + offsetof(InlineBatch, rec_idx), a.rec_idx, (size_t)a.n * sizeof(uint32_t));
    flush_kernargs();
    const uint16_t threads = a.n <= 64 ? 64 : 128;
    // Acquire at agent scope invalidates the caches the kernel reads its (host-written) kernarg
    // block through; no release fence: the kernel publishes its outputs at system scope itself.
    submit(k, ka, threads, 1, threads, false, HSA_FENCE_SCOPE_NONE, wi_slot);
  }

  bool launch_kernel(const char* name, const void* args, size_t bytes, unsigned grid_x, unsigned grid_y,
                     unsigned block, bool ordered) override {
    if (named_.empty()) return false;
    const auto it = named_.find(name);
    if (it == named_.end()) return false;
    const Kernel& k = it->second;
    // the entries read no implicit argument: their kernarg segment is exactly the argument block
    if (bytes != k.kernarg || bytes > stride_ || block == 0 || block > 1024 || grid_x == 0 || grid_y == 0 ||
        (uint64_t)grid_x * block > UINT32_MAX)
      throw std::invalid_argument(std::string("direct dispatch: bad launch of ") + name);
    if (faulted()) throw std::runtime_error("direct dispatch: queue error");
    uint64_t* wi_slot = nullptr;
    char* ka = next_kernarg(ring_, &wi_slot);
    std::memcpy(ka, args, bytes);
    flush_kernargs();
    // ordered: barrier bit (the kernel starts after every earlier packet of this queue has
    // finished: the order of hipLaunchKernel's stream, for launches that share a workspace) and a
    // system-scope release at kernel end, as a HIP stream's; unordered: neither - the kernel's
    // results are write-through records and it may overlap the batch before it
    submit(k, ka, grid_x * block, grid_y, (uint16_t)block, ordered,
           ordered ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_NONE, wi_slot);
    ++named_launches_;
    return true;
  }

  void* bar_alloc(size_t bytes) override {
    if (hdp_flush_ == nullptr || bytes == 0) return nullptr;
    void* p = nullptr;
    // uncached (MTYPE UC): the GPU never keeps a line of it in L2, so a row the CPU rewrote through
    // the BAR for the slot's next batch cannot be shadowed by a stale cached copy of the last one
    if (hsa_amd_memory_pool_allocate(dpool_, (bytes + 255) & ~size_t(255), HSA_AMD_MEMORY_POOL_UNCACHED_FLAG, &p) !=
        HSA_STATUS_SUCCESS)
      return nullptr;
    if (hsa_amd_agents_allow_access(1, &cpu_, nullptr, p) != HSA_STATUS_SUCCESS) {
      hsa_amd_memory_pool_free(p);
      return nullptr;
    }
    bar_bufs_.push_back(p);
    return p;
  }
  void bar_flush() override {
    if (hdp_flush_ == nullptr) return;
    _mm_sfence();
    *reinterpret_cast<volatile uint32_t*>(hdp_flush_) = 1u;
    (void)*reinterpret_cast<volatile uint32_t*>(hdp_flush_);  // the flush is posted: wait for it
  }

  bool resident_launch(const char* name, const void* args, size_t bytes, unsigned grid_blocks, unsigned block) override {
    const auto it = named_.find(name);
    if (it == named_.end()) return false;
    const Kernel& k = it->second;
    if (bytes != k.kernarg || bytes > RESIDENT_KERNARG || block == 0 || block > 1024 || grid_blocks == 0) return false;
    if (rqueue_ != nullptr && !resident_wait(0)) return false;  // one at a time
    if (rqueue_ == nullptr) {
      if (hsa_queue_create(gpu_, 64, HSA_QUEUE_TYPE_SINGLE, resident_queue_error, this, UINT32_MAX, UINT32_MAX, &rqueue_) !=
          HSA_STATUS_SUCCESS) {
        rqueue_ = nullptr;
        return false;
      }
      if (hsa_amd_memory_pool_allocate(kpool_, RESIDENT_KERNARG, 0, (void**)&rkernarg_) != HSA_STATUS_SUCCESS ||
          hsa_amd_agents_allow_access(1, &gpu_, nullptr, rkernarg_) != HSA_STATUS_SUCCESS ||
          hsa_signal_create(0, 0, nullptr, &rsig_) != HSA_STATUS_SUCCESS) {
        hsa_queue_destroy(rqueue_);
        rqueue_ = nullptr;
        if (rkernarg_) hsa_amd_memory_pool_free(rkernarg_);
        rkernarg_ = nullptr;
        rsig_.handle = 0;
        return false;
      }
    }
    // the previous resident kernel has ended (checked above): its argument block is free
    std::memcpy(rkernarg_, args, bytes);
    hsa_signal_store_screlease(rsig_, 1);
    const uint64_t wi = hsa_queue_add_write_index_scacq_screl(rqueue_, 1);
    auto* pkt = reinterpret_cast<hsa_kernel_dispatch_packet_t*>(rqueue_->base_address) + (wi & (rqueue_->size - 1));
    pkt->workgroup_size_x = (uint16_t)block;
    pkt->workgroup_size_y = 1;
    pkt->workgroup_size_z = 1;
    pkt->reserved0 = 0;
    pkt->grid_size_x = grid_blocks * block;
    pkt->grid_size_y = 1;
    pkt->grid_size_z = 1;
    pkt->private_segment_size = k.priv;
    pkt->group_segment_size = k.group;
    pkt->kernel_object = k.object;
    pkt->kernarg_address = rkernarg_;
    pkt->reserved2 = 0;
    pkt->completion_signal = rsig_;
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            (1 << HSA_PACKET_HEADER_BARRIER) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | (1u << 16), __ATOMIC_RELEASE);
    hsa_signal_store_relaxed(rqueue_->doorbell_signal, (hsa_signal_value_t)wi);
    return true;
  }

  bool resident_wait(int timeout_ms) override {
    if (rsig_.handle == 0) return true;
    const uint64_t ns = (uint64_t)std::max(0, timeout_ms) * 1000000ull;
    // blocked wait (interrupt signal): the supervisor sleeps while the kernel serves
    return hsa_signal_wait_scacquire(rsig_, HSA_SIGNAL_CONDITION_LT, 1, ns == 0 ? 1 : ns,
                                     ns == 0 ? HSA_WAIT_STATE_ACTIVE : HSA_WAIT_STATE_BLOCKED) < 1;
  }

  bool resident_faulted() const override { return rfault_.load(std::memory_order_relaxed); }

  void resident_abandon(bool track) override {
    rfault_.store(false);
    // a queue in error never signals: forget it; a kernel that only ignored its stop word ends on
    // its lease: keep watching its signal, and free its queue once it has ended
    if (track && rqueue_ != nullptr) abandoned_.push_back(Abandoned{rqueue_, rkernarg_, rsig_});
    rqueue_ = nullptr;
    rkernarg_ = nullptr;
    rsig_.handle = 0;
  }

  bool resident_abandoned_done() override {
    for (size_t i = 0; i < abandoned_.size();) {
      Abandoned& a = abandoned_[i];
      if (hsa_signal_load_scacquire(a.sig) >= 1) {
        ++i;
        continue;
      }
      hsa_queue_destroy(a.queue);
      if (a.kernarg) hsa_amd_memory_pool_free(a.kernarg);
      hsa_signal_destroy(a.sig);
      abandoned_.erase(abandoned_.begin() + (long)i);
    }
    return abandoned_.empty();
  }

  void inject_resident_fault() override { rfault_.store(true); }

  bool faulted() const override { return fault_.load(std::memory_order_relaxed); }
  uint64_t named_launches() const override { return named_launches_; }
  bool device_kernargs() const override { return hdp_flush_ != nullptr; }
  void set_fault() { fault_.store(true); }
  void set_resident_fault() { rfault_.store(true); }

 private:
  // The kernarg ring: `entries` argument blocks used round robin; wi[e] is the packet id that last
  // used entry e (~0: never).
  struct alignas(64) Ring {
    char* base = nullptr;
    uint32_t entries = 0;
    uint64_t launches = 0;
    std::vector<uint64_t> wi;
  };

  // Ring entry reuse: the packet that last used this entry must have been consumed by the packet
  // processor (its read index passed it). With at most a few batches in flight and
  // the region several times deeper, its kernel has finished as well; after a watchdog failure (a
  // batch given up while its packet may still be queued) this wait is what keeps live arguments
  // from being overwritten.
  char* next_kernarg(Ring& p, uint64_t** slot) {
    const uint32_t e = (uint32_t)(p.launches++ % p.entries);
    const uint64_t last = p.wi[e];
    if (last != ~uint64_t(0)) {
      const auto t0 = std::chrono::steady_clock::now();
      while (hsa_queue_load_read_index_scacquire(queue_) <= last) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200))
          throw std::runtime_error("direct dispatch: kernarg ring entry still owned by a queued packet");
        _mm_pause();
      }
    }
    *slot = &p.wi[e];  // submit() records the packet id here
    return p.base + (size_t)e * stride_;
  }

  void flush_kernargs() {
    if (hdp_flush_ == nullptr) return;
    _mm_sfence();  // drain the write-combined BAR writes, then flush the HDP ahead of the doorbell
    *reinterpret_cast<volatile uint32_t*>(hdp_flush_) = 1u;
    // The flush register write is posted: read it back so the flush has completed before the
    // packet (and so the kernel's kernarg loads) can be seen. MLAPI_HDP_READBACK=0 skips it
    // (measured ~0.9 us per launch, tools/hsa_dispatch_probe.cpp mode 3) at the risk of stale
    // kernargs.
    if (hdp_readback_) (void)*reinterpret_cast<volatile uint32_t*>(hdp_flush_);
  }

  // grid_x in work-items (AQL), grid_y in blocks of height 1. One producer at a time (the engine's
  // launch lock): reserve the slot, fill the packet, publish the header, ring the doorbell.
  void submit(const Kernel& k, const char* ka, uint32_t grid_x, uint32_t grid_y, uint16_t block, bool barrier,
              int release_scope, uint64_t* wi_slot) {
    const uint64_t wi = hsa_queue_add_write_index_scacq_screl(queue_, 1);
    *wi_slot = wi;
    while (wi - hsa_queue_load_read_index_scacquire(queue_) >= queue_->size) {
      // full (cannot happen with a few batches in flight): wait for the packet processor
      _mm_pause();
    }
    auto* pkt = reinterpret_cast<hsa_kernel_dispatch_packet_t*>(queue_->base_address) + (wi & (queue_->size - 1));
    pkt->workgroup_size_x = block;
    pkt->workgroup_size_y = 1;
    pkt->workgroup_size_z = 1;
    pkt->reserved0 = 0;
    pkt->grid_size_x = grid_x;
    pkt->grid_size_y = grid_y;
    pkt->grid_size_z = 1;
    pkt->private_segment_size = k.priv;
    pkt->group_segment_size = k.group;
    pkt->kernel_object = k.object;
    pkt->kernarg_address = const_cast<char*>(ka);
    pkt->reserved2 = 0;
    pkt->completion_signal.handle = 0;  // completion: the kernel's own done word / records
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                            (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (release_scope << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint32_t setup = grid_y > 1 ? 2 : 1;  // grid dimensions
    __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | (setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_relaxed(queue_->doorbell_signal, (hsa_signal_value_t)wi);
  }

  static constexpr uint32_t QUEUE_SIZE = 256;
  static constexpr size_t RESIDENT_KERNARG = 4096;
  hsa_amd_memory_pool_t kpool_{};  // host kernarg pool (the resident kernel's block: read once)
  hsa_queue_t* rqueue_ = nullptr;  // resident kernel queue
  void* rkernarg_ = nullptr;
  hsa_signal_t rsig_{};
  struct Abandoned {  // resident instances that did not stop when told (resident_abandon(true))
    hsa_queue_t* queue;
    void* kernarg;
    hsa_signal_t sig;
  };
  std::vector<Abandoned> abandoned_;
  uint32_t ka_slots_ = 64;
  bool hdp_readback_ = true;
  const uint32_t stride_ = (uint32_t)((sizeof(InlineBatch) + 255) / 256 * 256);
  bool inited_ = false;
  hsa_agent_t gpu_{};
  std::vector<char> blob_;
  hsa_code_object_reader_t reader_{};
  hsa_executable_t exe_{};
  Kernel k_[6];
  std::unordered_map<std::string, Kernel> named_;  // launch_kernel's kernels
  uint64_t named_launches_ = 0;
  hsa_queue_t* queue_ = nullptr;
  char* kernargs_ = nullptr;
  uint32_t* hdp_flush_ = nullptr;  // non-null: the ring is in device memory
  hsa_amd_memory_pool_t dpool_{};
  hsa_agent_t cpu_{};
  std::vector<void*> bar_bufs_;
  Ring ring_;
  std::atomic<bool> fault_{false};
  std::atomic<bool> rfault_{false};  // the resident queue reported an error
};

void queue_error(hsa_status_t, hsa_queue_t*, void* data) { static_cast<HsaInlineDispatcher*>(data)->set_fault(); }
void resident_queue_error(hsa_status_t, hsa_queue_t*, void* data) {
  static_cast<HsaInlineDispatcher*>(data)->set_resident_fault();
}

}  // namespace

std::unique_ptr<InlineDispatcher> make_direct_dispatcher(int device, const std::string& hsaco_path, int max_in_flight,
                                                         std::string* why) {
  auto d = std::make_unique<HsaInlineDispatcher>();
  if (!d->init(device, hsaco_path, max_in_flight, why)) return nullptr;
  return d;
}

}  // namespace mlapi
