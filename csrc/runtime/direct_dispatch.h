// Direct AQL dispatch of the serving kernels ("hsaco loader, direct-launch wrappers").
//
// hipLaunchKernel spends ~2.5 us of the calling thread per launch and its path from launch to a
// kernel-written done word is ~7.5 us for a one-wave kernel on MI355X; writing the AQL packet into
// an HSA queue of our own costs ~0.03 us and that path ~5.3 us (tools/hsa_dispatch_probe.cpp,
// profiles/r2_signal/hsa_probe.txt). The engine uses it for kernel-argument batches (InlineBatch:
// the whole batch travels in the kernarg segment, so a dispatch is one memcpy + one packet).
// Where that segment lives decides the latency: with a 3.5 KB block, a kernarg ring in host memory
// made the path 14.0 us (the kernel's scalar loads cross the host link), one in device HBM written
// through the BAR + HDP flush 6.9 us, hipLaunchKernel 9.5 us (profiles/r2_signal/hsa_probe_kernarg.txt).
#pragma once

#include <memory>
#include <string>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {

// KernelLauncher: the wide serving kernels of the same code object (linear_split's class-split
// predict, the binary GEMV) by name, through the same queue and kernarg ring; the ring entry is written through the
// BAR and one HDP flush covers it and any BAR-staged rows written before it.
class InlineDispatcher : public KernelLauncher {
 public:
  ~InlineDispatcher() override = default;
  // Enqueue one kernel-argument batch (dt: DT_F64 / DT_F32); completion is the batch's done word
  // or its records. One caller at a time: the engine's launch path (batcher / run_idle, serialised
  // by the engine's launch lock; also the only user of launch_kernel). Round 4's per-IO-thread
  // dispatch lanes (a multi-producer queue) lost their A/B (profiles/r4_lanes/) and were removed in
  // round 5; the resident kernel replaced the per-batch packet instead. Throws on failure.
  virtual void launch(int dt, const InlineBatch& a) = 0;
  // true once the queue reported an error (the engine then fails the batches instead of waiting)
  virtual bool faulted() const = 0;
  // launches made through launch_kernel (wide serving batches dispatched without hipLaunchKernel)
  virtual uint64_t named_launches() const = 0;
  // true if the kernarg ring is in device memory (else the host kernarg pool)
  virtual bool device_kernargs() const = 0;
  // Device HBM the CPU writes directly through the BAR (the kernarg ring's mechanism), for rows
  // of small wide batches: the kernel then reads them from HBM / L2 instead of pulling them over
  // the host link once per wave. nullptr if the device has no HDP flush (no BAR staging). Freed
  // with the dispatcher.
  virtual void* bar_alloc(size_t bytes) = 0;
  // Make BAR writes visible to the device: sfence, HDP flush, read-back. Call before the launch.
  virtual void bar_flush() = 0;
  // Resident kernels (the SMALL path's serve_resident.h): a kernel of the code object that runs
  // until its own stop / lease rule ends it, on a second HSA queue of its own (it must not sit in
  // front of the serving packets), one at a time, with a completion signal. false: the kernel is
  // not in the code object, the argument block does not match it, or the queue failed.
  virtual bool resident_launch(const char* name, const void* args, size_t bytes, unsigned grid_blocks,
                               unsigned block) = 0;
  // Wait up to timeout_ms for the resident kernel to end: true = ended (or none running).
  virtual bool resident_wait(int timeout_ms) = 0;
  // A resident kernel that did not end when told to, or whose queue failed: the next launch gets a
  // fresh queue, and the old one is never destroyed under a live wave. track = true (a kernel that
  // still runs and ends on its lease): its signal is watched by resident_abandoned_done(), which
  // frees the queue once the kernel has ended; false (a queue in error): forgotten.
  virtual void resident_abandon(bool track) = 0;
  // true once every tracked abandoned instance has ended (their queues are then freed)
  virtual bool resident_abandoned_done() = 0;
  // the resident queue reported an error (its kernel faulted): abandon it and launch afresh
  virtual bool resident_faulted() const = 0;
  // fault injection (tests): report the resident queue as failed
  virtual void inject_resident_fault() = 0;
};

// Loads `hsaco_path` (csrc/kernels/serve_direct.hip) for the GPU behind HIP device `device` and
// creates the queue; nullptr with the reason in *why if anything is missing (the engine then keeps
// using hipLaunchKernel).
// `max_in_flight`: the engine's slot count. The kernarg ring is sized to a multiple of it (at least
// 64 entries), and an entry is rewritten only after the packet processor has consumed the packet
// that last used it (bounded wait, then an error instead of overwriting live arguments).
std::unique_ptr<InlineDispatcher> make_direct_dispatcher(int device, const std::string& hsaco_path, int max_in_flight,
                                                         std::string* why);

}  // namespace mlapi
