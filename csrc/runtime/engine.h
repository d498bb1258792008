// Per-GPU serving engine: request queue -> continuous batcher -> fused HIP kernel -> completions.
//
// Replaces the reference's per-request model execution (main.py:19-22: unpickle + two sklearn
// calls, serialized on the event loop) with a server-side batcher (BASELINE north star): every
// request submitted while the previous batch is on the GPU is coalesced into the next launch.
//
//   submit() (any thread, short mutex, one lock per epoll round of an IO thread)
//     -> batcher thread: drains up to max_batch rows and launches ONE kernel for them on a
//        high-priority stream; the kernel is picked per model at load time (Model::path):
//          SMALL   (F <= 32, K <= 16; the Iris shape): linear_small, fp64 (sklearn bit parity) or
//                  fp32. Batches that fit 3 KB travel inside the kernel-argument block
//                  (launch_linear_inline: no host-link read at all); larger ones are read
//                  zero-copy from the pinned slot;
//          GEMV    (binary, wide F): rows packed as bf16 (or fp32) into the pinned slot, read
//                  zero-copy by the gemv_binary kernel (stage_wide: one hipMemcpyAsync H2D
//                  into a device buffer first);
//          GEMM    (multiclass, wide F / many classes): bf16 rows (F zero-padded to the MFMA
//                  width), the MFMA gemm_softmax kernel with its online softmax/argmax epilogue
//                  (workspace per model, zeroed once);
//          GENERIC (wide models served in fp32/fp64): one-row-per-lane scalar kernel;
//        the (idx, p) results are written by the kernel straight into host-mapped memory, and
//        the kernel (or, on the GEMV / GEMM paths, a one-wave signal kernel behind it) publishes
//        the batch's sequence number into the slot's host-coherent done word (ServeSignal);
//        up to `slots` batches are in flight;
//     -> completer thread: spins on the oldest slot's done word (no HIP event: launch-to-
//        observed drops from ~12 to ~7 us, tools/launch_probe.hip), groups results by Sink and
//        hands them over (HTTP IO threads, Python futures, blocking callers).
//
// The CPU backend (device = -1) runs the same math in C++ float64 (a "FakeDevice" for tests and
// GPU-less hosts). Models are immutable and swapped atomically (hot reload): an in-flight batch
// keeps the model it was launched with alive through its shared_ptr.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mlapi/common.h"
#include "mlapi/kernels.h"
#include "direct_dispatch.h"
#include "mlapi/resident.h"

namespace mlapi {

enum Status : int32_t {
  ST_OK = 0,
  ST_NONFINITE = 1,     // NaN / inf probability (reference: json.dumps raises -> HTTP 500)
  ST_NO_MODEL = 2,      // checkpoint missing (reference: open() raises -> HTTP 500)
  ST_SHAPE = 3,         // feature count mismatch
  ST_DEVICE_ERROR = 4,  // launch failure / injected fault / a row the kernel refused to answer
                        // (misplaced XCD-local merge, wide class-merge timeout)
  ST_SHUTDOWN = 5,
};

// how a launched batch completes (Slot::rec_mode): per-row records, class-split records merged on
// the host (linear_split), f64 class-block records merged on the host (linear_wide)
enum RecMode : int { REC_ROWS = 1, REC_SPLITS = 2, REC_WIDE = 3 };

// WIDE: linear_wide.h, f64 accumulation on the matrix cores for f64 / f32 storage, any F and K
enum ServePath : int32_t {
  PATH_SMALL = 0, PATH_GEMV = 1, PATH_GEMM = 2, PATH_GENERIC = 3, PATH_WIDE = 4, PATH_COUNT = 5
};

struct Model {
  int kind = KIND_MULTINOMIAL;
  int F = 0;          // features
  int K = 0;          // rows of W (1 for binary kinds)
  int dtype = DT_F64; // small-path compute dtype (f64 / f32)
  int path = PATH_SMALL;
  int xdt = DT_F64;   // dtype of the rows as the kernel reads them (f64 / f32 / bf16)
  int ldx = 0;        // row stride of the packed rows (F, or F zero-padded for GEMV / GEMM)
  int pdt = DT_F64;   // dtype of the kernel's p output (f32 on the GEMV / GEMM paths)
  float bias0 = 0.f;  // GEMV: scalar intercept
  uint64_t version = 0;
  std::vector<double> W, b;             // host float64 copies (CPU backend + reload)
  std::vector<std::string> label_json;  // pre-rendered JSON per class index
  int device = -1;
  void* dW = nullptr;
  void* db = nullptr;
  void* ws = nullptr;  // GEMM: gemm_softmax workspace (zeroed once; split-merge counters re-arm)
  size_t ws_bytes = 0;
  void* ws_split = nullptr;  // GEMM: linear_split workspace (small batches; every f32 batch)
  size_t ws_split_bytes = 0;
  WidePlan wplan{};          // WIDE: the kernel's plan (class blocks, feature splits, padded width)
  void* ws_wide = nullptr;   // WIDE: linear_wide workspace (zeroed once)
  size_t ws_wide_bytes = 0;
  ~Model();
};

struct Completion {
  uint64_t tag;
  int32_t idx;
  int32_t status;
  double p;
  int64_t latency_ns;  // submit -> completion
};

class Engine;

class Sink {
 public:
  virtual ~Sink() = default;
  // Called on the engine's completion thread; must not block for long.
  virtual void on_complete(const Completion* c, size_t n, const std::shared_ptr<const Model>& model) = 0;
};

// Per-IO-thread submission ring of the resident SMALL-path kernel (csrc/include/mlapi/resident.h,
// the request path without an HSA packet, a batcher or a completer). The IO
// thread that parsed an epoll round's rows writes them into its ring (plain stores into host
// memory: no lock, no syscall) and later finds each answer in the ring's record array from its
// own event loop. The resident wave of that ring (one per IO thread) reads the rows, runs the
// SMALL kernel's row code and writes the records. One thread per ring.
class ServeRing {
 public:
  ServeRing(const ServeRing&) = delete;
  ServeRing& operator=(const ServeRing&) = delete;
  // Write n rows (nf features each) for the resident kernel. true = accepted (completions come
  // from poll()); false = not eligible now (no resident kernel live for the current model, ring
  // full, a row of another width, fault injection on): the caller submits them to the engine queue.
  bool submit(const double* X, int n, int nf, const uint64_t* tags);
  struct Seg {
    size_t begin;  // first completion of a run of one model in poll()'s output
    std::shared_ptr<const Model> model;
  };
  // Appends the completions of answered rows to `out` (runs of one model in segs). A row answered
  // stale (a hot reload raced its submit) goes through the engine queue to `sink` instead; the
  // number of those is added to *requeued. Returns the rows still pending.
  int poll(std::vector<Completion>& out, std::vector<Seg>& segs, Sink* sink, int* requeued);
  // rows submitted and not yet answered (given-up rows are not counted: nothing waits for them)
  int pending() const { return live_n_; }
  // Give up on every pending row (the owning thread leaves the ring): their slots stay out of
  // reuse until their records land, and no answer of theirs is ever rendered. Returns the rows.
  int abandon_pending();
  // Spin (user space, no syscall) until a pending row's record lands or `ns` passed: true if one did.
  bool wait_any(int64_t ns) const;

 private:
  friend class Engine;
  ServeRing(Engine* e, int index);
  bool landed(uint32_t pos) const;
  Engine* eng_;
  int idx_;
  ResidentGranule* ring_;  // this ring's entries (host view)
  ServeRecord* rec_;       // this ring's records (host view)
  uint32_t next_ = 0, tail_ = 0;  // positions: [tail_, next_) submitted, not yet consumed or given up
  int live_n_ = 0;                // live rows (pending())
  struct Pend {
    uint64_t tag = 0;
    int64_t t_enq = 0;
    std::shared_ptr<const Model> model;
    uint32_t pos = 0;       // ring position of the row last written into this slot
    int32_t nf = 0;
    bool live = false;      // submitted, answer not yet consumed
    bool poisoned = false;  // given up on (watchdog / ring closed): not rewritten until its record lands
  };
  // a poisoned slot whose record has landed since (the GPU answered late) is free again
  bool reclaim(Pend& p);
  Pend pend_[RESIDENT_RING];
};


struct EngineConfig {
  int device = -1;        // HIP device ordinal, -1 = CPU backend
  int max_batch = 256;    // rows per launch
  int max_wait_us = 0;    // 0 = continuous batching; >0 = also wait up to this long to fill a batch
  int slots = 4;          // batches in flight
  int dtype = DT_F64;     // SMALL-path compute dtype (f64 = bit parity with sklearn, or f32)
  int wide_dtype = DT_F64;   // dtype of models too wide for the SMALL path: f64 (default) -> WIDE (f64
                             // storage, f64 MFMA accumulation: the reference's precision, any F / K /
                             // kind); f32 -> WIDE (f32 storage, f64 accumulation; f32_gemv: binary
                             // F <= 2048 on the f32 GEMV); bf16 -> GEMV / bf16 MFMA GEMM (F <= 4096),
                             // WIDE beyond
  // WIDE multiclass batches of <= host_merge_rows rows from models with at most this many 16-class
  // blocks end in per-block records merged by the completer; 0 (default) = always the in-kernel
  // class merge. Off: the completer polls 2 records per block and row (126 per row at K = 1000;
  // measured 52 us GPU legs, profiles/r4_s4/), and the served p_max then depends on the batch
  // size (host vs device exp, another merge order), which breaks the f64 path's byte-exact bodies.
  int wide_host_merge_blocks = 0;
  bool f32_gemv = false;     // f32 binary F <= 2048: the f32-accumulating GEMV instead of WIDE (A/B)
  int bar_rows = 32;         // wide paths: batches of at most this many rows are written straight into
                             // device HBM through the BAR (direct dispatch's HDP-flushed mapping) instead
                             // of being read by every wave over the host link (0 = off)
  int host_merge_rows = 16;  // class-split launches of at most this many rows publish per-block states
                             // and the completer merges them (no in-kernel merge round trips; 0 = off)
  int split_max_rows = 32;   // bf16 GEMM path: batches of at most this many rows take the
                             // class-split kernel (linear_split.h; 0 = always the tiles kernel)
  int max_features = 256; // per-request feature cap (sizes the slot buffers)
  bool inline_args = true;  // SMALL path: batches that fit travel in the kernel-argument block
  // ... and complete through per-row 16-byte records {seq, idx, p} (one store per row, no fence,
  // no done word) instead of outputs + a fenced done word
  bool record_completion = true;
  bool direct_wide = true;   // class-split / record GEMV batches dispatched into the direct queue (needs record_completion)
  int64_t direct_wide_max_weight_bytes = 256 << 10;  // ... for models with at most this many bytes of W
  int gemv_record_rows = 2;  // GEMV batches of at least this many rows complete through records (0 = never)
  bool stage_wide = false;  // GEMV / GEMM / GENERIC: H2D-copy the rows first (default: zero-copy reads)
  int watchdog_ms = 2000; // batch not complete after this -> engine marked unhealthy
  int fail_every = 0;     // fault injection: fail every N-th batch with ST_DEVICE_ERROR
  int delay_us = 0;       // fault injection: extra per-batch delay
  int spin_us = 0;        // batcher / completer poll their queues this long before sleeping on a condvar
                          // (saves the futex wake-up on the request path under load)
  // Completer threads: each takes the oldest in-flight slot, waits for its done word and delivers
  // it (grouping by sink, one eventfd wake per IO thread); with several, the delivery of batch k
  // overlaps the wait for batch k+1. Per-connection order is safe: a connection has at most one
  // request outstanding.
  int completers = 1;
  // Batcher threads: each drains the queue and launches (packing + dispatch serialised on the
  // launch lock); with two, one batch's queue take / slot wait / bookkeeping overlaps the other's
  // launch. The batcher is a single-server queue at ~80 % utilisation under the c=64 load, which
  // is what the rows' queue wait is made of (engine stage clocks).
  int batchers = 1;
  int max_queue = 1 << 20;  // backpressure: rows waiting for the batcher; beyond it submit is refused
  // Kernel-argument batches go through the engine's own HSA queue (direct_dispatch.h) when the
  // serving code object loads; empty path or failure -> hipLaunchKernel.
  bool direct_dispatch = true;
  std::string hsaco_path;
  // Idle-engine fast path (run_idle): when nothing is queued or in flight, the submitting thread
  // launches its rows itself and waits for the done word, skipping the batcher and completer
  // wake-ups (two futex hand-offs on a batch=1 request). SMALL-path models, batches of at most
  // this many rows; 0 = off. On the CPU backend the calling thread runs the float64 oracle.
  int idle_inline_rows = 8;
  // The resident SMALL-path kernel (ServeRing, mlapi/resident.h): IO threads write SMALL-model rows
  // into per-thread rings that resident waves poll, no packet or engine thread per request; 0 = off
  // (every row through the batcher). Needs the direct dispatcher's code object on a GPU; on the CPU
  // backend a host thread plays the kernel's part (tests).
  int resident = 1;
  int resident_depth = 2;        // host-memory polls in flight per wave (1, 2, 4)
  int resident_lease_ms = 200;   // a wave exits when the supervisor's lease has not moved for this long
  int resident_idle_polls = 20000;  // polls without a row before a wave slows down (an idle server)
  int resident_idle_sleep = 4;      // ... to one poll per this many ~3.4 us sleeps
};

struct EngineStats {
  uint64_t requests = 0, batches = 0, errors = 0;
  uint64_t rejected = 0;            // rows refused by backpressure (max_queue)
  uint64_t batch_hist[12] = {0};    // batch size buckets: 1,2,4,...,2048+
  uint64_t latency_hist[24] = {0};  // latency buckets in powers of two of 1us: <1us .. >=2^23us
  uint64_t path_batches[PATH_COUNT] = {0};  // GPU batches per kernel path
  uint64_t inline_batches = 0;      // SMALL batches launched through the kernel-argument block
  uint64_t direct_batches = 0;      // ... of which written straight into the HSA queue
  uint64_t direct_wide_batches = 0; // class-split (wide multiclass) batches dispatched into that queue
  uint64_t idle_batches = 0;        // batches run by the submitting thread (run_idle)
  uint64_t resident_rows = 0;       // rows answered by the resident kernel (ServeRing)
  uint64_t resident_stale = 0;      // ... bounced to the engine queue (a hot reload raced them)
  uint64_t resident_launches = 0;   // resident kernel instances launched (start, reload, restart)
  uint64_t resident_hb_restarts = 0;    // ... stopped and relaunched: block 0's heartbeat stalled
  uint64_t resident_ring_restarts = 0;  // ... stopped and relaunched: a ring's row waited past the watchdog
  uint64_t resident_self_exits = 0;     // instances that ended by themselves (lease expiry, early exit)
  uint64_t resident_queue_faults = 0;   // ... on a queue error (relaunched on a fresh queue)
  uint64_t resident_abandoned = 0;      // instances that did not stop when told (left to their lease)
  uint64_t resident_heartbeat = 0;      // block 0's poll count (liveness; GPU instances)
  int resident_rings = 0;           // rings the running instance polls (0: none running)
  bool resident_live = false;       // IO threads may submit to their rings now
  uint64_t generic_models = 0;      // models loaded onto the scalar GENERIC kernel (a warning is logged)
  uint64_t xcd_errors = 0;          // rows failed because an XCD-local split merge read a misplaced partial
                                    // (the protocol is then off for the device: linear_split.h, xcd.hip)
  uint64_t bar_batches = 0;         // wide batches whose rows were written into HBM through the BAR
  bool direct_dispatch = false;     // the direct queue is up
  bool direct_device_kernargs = false;  // ... and its kernarg ring is in device memory
  double latency_sum_us = 0;
  double device_us_sum = 0;         // launch -> completion observed by the completer
  double queue_wait_us_sum = 0;     // per row: submit -> its batch's launch (batcher queue + packing)
  // Engine-thread stage clocks (ns, summed over GPU batches): batcher - take (queue swap + model
  // ref), slot (wait for a free slot), launch (pack + dispatch), book (stats, in-flight hand-off,
  // wake); completer - wait_gpu (launch -> records seen), deliver (collect + per-sink delivery +
  // slot return). Sleeping on an empty queue is in neither.
  double batcher_ns[4] = {0, 0, 0, 0};
  // inside `launch` for zero-copy / BAR batches (not kernel-argument ones): pack (rows -> the
  // model dtype, into the slot or through the BAR), flush (HDP flush + read-back of BAR rows),
  // kernel (the launch call(s))
  double launch_ns[3] = {0, 0, 0};
  double completer_ns[2] = {0, 0};
  uint64_t queue_depth = 0;
  uint64_t model_version = 0;
  bool healthy = true;
  bool dropped = false;             // fault injection: every batch fails (drop-a-rank)
};

class Engine {
 public:
  explicit Engine(const EngineConfig& cfg);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  // Installs a new model (atomic swap). W: K x F row-major float64. Returns the new version.
  uint64_t load_model(int kind, int F, int K, const double* W, const double* b,
                      const std::vector<std::string>& label_json);
  void unload_model();  // subsequent requests complete with ST_NO_MODEL
  std::shared_ptr<const Model> model() const;

  // Thread-safe. Returns false if the engine is stopping or nf exceeds max_features.
  bool submit(const double* x, int nf, uint64_t tag, Sink* sink);
  // n rows (row-major, nf features each) under one lock. Returns the number k of rows accepted:
  // rows [0, k) are queued, rows [k, n) were refused because the queue reached max_queue
  // (k < n only under backpressure); SUBMIT_BUSY if none fits, 0 if the engine is stopping (or
  // the request is malformed).
  static constexpr int SUBMIT_BUSY = -1;
  int submit_many(const double* X, int n, int nf, const uint64_t* tags, Sink* sink);
  // Idle-engine fast path: if the engine has nothing queued or in flight (and the rows fit
  // cfg.idle_inline_rows), launch the rows from the calling thread, wait for their done word and
  // append their completions to `out` (model in `m_out`); true = done, the caller must not submit
  // them. false = not eligible (busy, CPU backend, fault injection on, no model): submit normally.
  // allow_wide: also for GEMV / GEMM / GENERIC models (the caller knows the load is low, e.g. one
  // open connection; under concurrency their IO threads are better spent parsing).
  bool run_idle(const double* X, int n, int nf, const uint64_t* tags, std::vector<Completion>& out,
                std::shared_ptr<const Model>& m_out, bool allow_wide = false);
  // Blocking convenience API (tests / bulk scoring through the batcher).
  void predict(const double* X, int64_t B, int F, int32_t* idx, double* p, int32_t* status);

  // The calling IO thread's submission ring for the resident kernel (owned by the engine, valid until
  // it is destroyed), or nullptr: resident off / unavailable, or every ring taken.
  ServeRing* open_ring();
  // The thread is done with the ring: its pending rows are waited for (bounded) and the ring goes
  // back to the engine's pool for the next open_ring().
  void close_ring(ServeRing* ring);
  // Stop the resident kernel for good (process exit): no relaunch, wait up to timeout_ms for it.
  void resident_halt(int timeout_ms);
  // Fault injection into the resident path (tests). Kernel-side (the running instance,
  // cleared when the supervisor relaunches): RES_FAULT_STALL, RES_FAULT_EXIT_RING (arg = ring),
  // RES_FAULT_IGNORE_STOP; RES_FAULT_NONE clears. Host-side: RES_INJECT_LEASE_STARVE (the supervisor stops bumping the
  // lease for arg ms), RES_INJECT_QUEUE_FAULT (the running instance is stopped and its queue
  // treated as faulted). false: no resident instance to inject into.
  static constexpr int RES_INJECT_LEASE_STARVE = 16;
  static constexpr int RES_INJECT_QUEUE_FAULT = 17;
  static constexpr int RES_INJECT_STALL_STICKY = 18;  // RES_FAULT_STALL kept across relaunches (until NONE)
  bool resident_inject(int mode, int arg);

  EngineStats stats() const;
  const EngineConfig& config() const { return cfg_; }
  bool healthy() const { return healthy_.load(std::memory_order_relaxed); }
  // Health probe succeeded (HttpServer's health thread): the engine serves again.
  void mark_healthy() { healthy_.store(!drop_.load()); }
  // Fault injection "drop this rank": while on, every batch fails with ST_DEVICE_ERROR and the
  // engine reports unhealthy (DP dispatch takes the rank out of its SO_REUSEPORT group).
  void inject_drop(bool on) {
    drop_.store(on);
    if (on) healthy_.store(false);
  }
  void stop();

 private:
  struct Meta {
    uint64_t tag;
    Sink* sink;
    int64_t t_enq;
    int32_t nf;
    int32_t off;  // offset into the feature arena
  };
  struct Slot {
    void* hx = nullptr;       // host pinned, device mapped: packed rows (model xdt)
    void* dx = nullptr;       // device address of hx (zero-copy reads)
    void* dstage = nullptr;   // device buffer: H2D destination of the GEMV / GEMM / GENERIC paths
    void* xbar = nullptr;     // device HBM written by the CPU through the BAR: rows of small wide batches
    int32_t* hidx = nullptr;  // host pinned outputs, written by the kernel over the host link
    int32_t* didx = nullptr;
    void* hp = nullptr;
    void* dp = nullptr;
    ServeRecord* hrec = nullptr;  // host pinned per-row completion records (kernel-argument batches)
    ServeRecord* drec = nullptr;
    int rec_mode = 0;         // 0: done word; REC_ROWS: per-row records (hrec); REC_SPLITS: per-split records (hsrec)
    SplitRecord* hsrec = nullptr;  // host-merge class-split launches: [64 splits][32 rows]
    SplitRecord* dsrec = nullptr;
    int rec_nsplit = 0;
    uint32_t seq = 0;         // sequence number the launch publishes into the done word
    std::vector<Meta> metas;
    std::vector<int32_t> pre_status;  // per-row status decided before launch
    std::shared_ptr<const Model> model;
    int64_t t_launch = 0;
    int n = 0;
    bool launched = false;
    bool failed = false;
  };

  void batcher_loop();
  void completer_loop();
  void pack_rows(Slot& s, const std::vector<double>& xs, const Model& m, void* dst);
  void launch_batch(Slot& s, const Model& m, const std::vector<double>& xs);
  void run_cpu(std::vector<Meta>& metas, const std::vector<double>& xs, const std::shared_ptr<const Model>& m);
  void finish(Slot& s, const int32_t* idx, const double* p, const int32_t* status);
  void deliver(std::vector<Meta>& metas, const int32_t* idx, const double* p, const int32_t* st,
               const std::shared_ptr<const Model>& m, int64_t now);
  void record_batch(size_t n);
  friend class ServeRing;
  void kick_resident();  // reload / ring open: wake the supervisor
  void resident_register(bool on);  // the at-exit halt list
  // Resident kernel supervisor (one thread): launches an instance for the current SMALL model over
  // the open rings, bumps the lease, restarts it on reload / new rings / a stalled heartbeat, and on
  // the CPU backend plays the kernel itself (resident_cpu_poll).
  void resident_loop();
  bool resident_launch(const std::shared_ptr<const Model>& m, uint32_t mver, int nrings, bool bounce);
  bool resident_stop_instance(int timeout_ms);
  int resident_cpu_poll(const std::shared_ptr<const Model>& m, uint32_t mver, int nrings, bool bounce);
  // Wait for a launched slot's done word (spin, then back off; fault and watchdog checks).
  void wait_done(Slot& s);
  // The launched slot's results -> idx / p (from the records or the output arrays).
  const int32_t* collect(Slot& s, std::vector<int32_t>& st, std::vector<double>& pd, std::vector<int32_t>& idx);
  void xcd_check(const int32_t* idx, std::vector<int32_t>& st, std::vector<double>& pd);

  EngineConfig cfg_;
  std::shared_ptr<const Model> model_;
  mutable std::mutex model_mu_;
  std::atomic<uint64_t> next_version_{1};

  // submission queue (double-buffered arenas)
  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::vector<Meta> q_meta_;
  std::vector<double> q_x_;
  bool stopping_ = false;
  int batchers_sleeping_ = 0;  // guarded by q_mu_: submit wakes a batcher only if one sleeps
  std::atomic<int> q_count_{0};    // rows queued (lock-free hint for the batcher's spin phase)

  // GPU slots
  hipStream_t stream_ = nullptr;
  std::unique_ptr<InlineDispatcher> direct_;  // direct AQL dispatch of kernel-argument batches
  std::vector<Slot> slots_;
  std::mutex s_mu_;
  std::condition_variable s_cv_;
  std::deque<int> free_slots_;
  std::deque<int> inflight_;
  std::atomic<int> inflight_n_{0};  // inflight_.size(), readable without s_mu_ (completer spin)
  int batchers_done_ = 0;  // guarded by s_mu_: the completers exit once every batcher has

  size_t slot_row_bytes_ = 0;  // capacity of one packed row in a slot (any path)
  uint32_t* done_h_ = nullptr;  // per-slot done words (host-coherent, SIGNAL_STRIDE apart)
  uint32_t* done_d_ = nullptr;
  uint32_t* sig_counter_ = nullptr;  // device word for multi-block signalled launches
  static constexpr int SIGNAL_STRIDE = 16;  // 64 bytes: one cache line per slot
  InlineBatch inline_{};        // guarded by launch_mu_
  std::mutex launch_mu_;        // launch_batch: batcher thread and run_idle callers

  // resident kernel (ServeRing): host-coherent rings [RESIDENT_MAX_RINGS][RESIDENT_RING] entries,
  // records, control block; the supervisor thread and its wake-up
  unsigned char* res_rings_h_ = nullptr;
  unsigned char* res_rings_d_ = nullptr;
  ServeRecord* res_recs_h_ = nullptr;
  ServeRecord* res_recs_d_ = nullptr;
  ResidentCtl* res_ctl_h_ = nullptr;
  ResidentCtl* res_ctl_d_ = nullptr;
  bool res_cpu_ = false;              // CPU backend: the supervisor polls the rings itself
  bool res_leaked_ = false;           // an instance never ended: its memory is not freed
  std::mutex rings_mu_;
  std::vector<std::unique_ptr<ServeRing>> rings_;
  std::vector<ServeRing*> free_rings_;
  std::atomic<int> rings_open_{0};    // rings handed out so far (the instance's grid)
  std::mutex res_mu_;
  std::condition_variable res_cv_;
  bool res_stop_ = false;
  uint64_t res_kick_ = 0;             // bumped on reload / ring open: the supervisor re-plans
  std::atomic<bool> res_live_{false};
  std::atomic<bool> res_halt_{false};   // resident_halt: never launch again
  std::atomic<uint32_t> res_mver_{0};   // 24-bit version of the model the running instance serves
  std::atomic<int> res_nrings_{0};      // rings the running instance polls
  // launch / stop / halt / abandon of the instance: one at a time (the at-exit halt runs on another
  // thread than the supervisor)
  std::mutex res_inst_mu_;
  std::atomic<bool> res_ring_stall_{false};     // ServeRing::poll: a row waited past the watchdog
  std::atomic<int64_t> res_starve_until_{0};    // injection: no lease bump before this (now_ns)
  std::atomic<bool> res_fault_queue_{false};    // injection: treat the ending instance's queue as faulted
  std::atomic<bool> res_fault_sticky_{false};   // injection: the fault word survives relaunches
  std::thread res_thread_;

  std::vector<std::thread> batchers_;
  std::vector<std::thread> completers_;
  std::atomic<bool> healthy_{true};
  std::atomic<bool> drop_{false};

  mutable std::mutex st_mu_;
  EngineStats stats_;
  std::atomic<uint64_t> batch_counter_{0};  // fault injection (fail_every), any batcher
};

// Reference float64 implementation of the fused epilogue (CPU backend + host-side oracle).
void cpu_linear_predict(const Model& m, const double* X, int64_t B, int32_t* idx, double* p);

int64_t now_ns();

}  // namespace mlapi
