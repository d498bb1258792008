// The resident SMALL-path serving kernel (round 5): host/device layouts.
//
// One workgroup (one wave) per HTTP IO thread stays on the GPU and polls that thread's submission
// ring in host memory; the IO thread writes each parsed /predict row into the ring and later finds
// the answer in the ring's record array. No AQL packet, no kernel-argument copy, no batcher or
// completer thread per request: one HSA queue takes only ~0.7 M tiny dispatches/s
// (profiles/r4_lanes/), a resident wave takes rows as fast as it can read host memory.
//
//  * A row is F granules of 16 bytes {x_f (f64), pos (u32), meta (u32)}: every granule carries the
//    row's ring position and the model version it was parsed for, so a wave that reads a row while
//    the CPU is still writing it sees a mixed tag and simply reads it again on its next poll - no
//    header word, no second host round trip. (Aligned 16-byte stores are single-copy atomic on
//    x86-64 with AVX; the GPU reads each granule with one 16-byte load.)
//  * The wave reads a window of rows with ONE load instruction: LPE lanes per row (LPE = F rounded
//    up to 4 / 8 / 32), 64 / LPE rows per poll, D polls in flight (a poll issued every round trip /
//    D: tools/ring_probe.hip measured ~2 us per host-memory round trip). Rows may be written out
//    of order; a done mask over the window keeps each one answered exactly once.
//  * The row's leader lane runs the same sklearn-exact row code as the launched kernels
//    (linear_rows.h row_predict: bit-identical logits) and writes the record {pos, idx, p} with
//    one write-through 16-byte store.
//  * A row parsed for another model version (hot reload raced the submit) is answered
//    RESIDENT_STALE_IDX; the IO thread re-submits it through the engine queue.
//  * Lifecycle: the engine's supervisor thread bumps `lease` every ~10 ms; a wave exits on the
//    stop word, or by itself when the lease has not moved for lease_ticks (the process died or hung:
//    the kernel never outlives it by more than that). At exit every wave publishes its ring head so
//    the next instance (reload, restart) continues where it stopped. A heartbeat word (block 0's
//    poll count) feeds the engine's watchdog.
#pragma once
#include <cstdint>

namespace mlapi {

constexpr int RESIDENT_RING = 256;          // entries per ring (power of two)
constexpr int RESIDENT_MAX_RINGS = 32;      // IO threads with a ring (the rest use the engine queue)
constexpr int RESIDENT_FMAX = 32;           // features per row (the SMALL path's F <= 32)
constexpr int RESIDENT_ENTRY_BYTES = RESIDENT_FMAX * 16;  // entry stride: F granules
constexpr int32_t RESIDENT_STALE_IDX = -4;  // the row's model version is not the kernel's

// meta = mver << 8 | F: the row's model version (24 bits, never 0) and its feature count, so an
// instance can recognise - and bounce - a row of any earlier model, whatever its width
struct alignas(16) ResidentGranule {
  double x;
  uint32_t pos;
  uint32_t meta;
};
inline uint32_t resident_mver(uint64_t model_version) { return (uint32_t)(model_version % 0xffffffu) + 1u; }

// Fault injection (tests): ResidentCtl::fault, read by every wave with the stop word.
// Each mode keeps the lease rule, so no injected fault can keep a wave alive past its process.
enum ResidentFault : uint32_t {
  RES_FAULT_NONE = 0,
  RES_FAULT_STALL = 1,        // waves stop answering rows and block 0 stops its heartbeat (a hung instance)
  RES_FAULT_EXIT_RING = 2,    // the wave of ring fault_arg exits at once (publishing its head)
  RES_FAULT_IGNORE_STOP = 3,  // waves ignore the stop word (only the lease ends them)
};

// Control block (host-coherent memory). Host -> GPU words first, GPU -> host words after.
struct alignas(64) ResidentCtl {
  uint32_t stop;       // non-zero: every wave exits at its next check
  uint32_t lease;      // bumped by the supervisor every ~10 ms
  uint32_t fault;      // ResidentFault (0 in service)
  uint32_t fault_arg;  // ... its argument (RES_FAULT_EXIT_RING: the ring)
  uint32_t pad0[12];
  uint32_t heads[RESIDENT_MAX_RINGS];  // ring heads: read at start, written back at exit
  uint64_t heartbeat;                  // block 0: polls so far (published every 1024 polls)
  uint64_t rows;                       // block 0: rows answered (same cadence)
  uint32_t pad1[12];
};

// Kernel arguments of mlapi_resident_<dt>_r<LPE>_d<D> (serve_direct.hip). No implicit argument is
// read: the kernarg block is this struct alone.
struct ResidentArgs {
  const unsigned char* rings;  // [nrings][RESIDENT_RING][RESIDENT_ENTRY_BYTES], device address of host memory
  void* recs;                  // ServeRecord [nrings][RESIDENT_RING]
  ResidentCtl* ctl;
  const void* W;               // device: [K][F] in the model dtype
  const void* b;               // device: [K]
  int32_t F, K, kind;
  uint32_t mver;               // 24-bit model version the rows must carry (0: bounce every row as stale)
  uint64_t lease_ticks;        // wall_clock64 ticks (100 MHz) without a lease bump before a wave exits
  uint64_t idle_exit_ticks;    // exit after this long without a row (0 = never; the bounce instance)
  uint32_t idle_polls;         // polls without a row before a wave backs off to slow polling
  uint32_t idle_sleep;         // s_sleep rounds per slow poll (each ~3.4 us)
};

}  // namespace mlapi
