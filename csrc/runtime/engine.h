// Per-GPU serving engine: request queue -> continuous batcher -> fused HIP kernel -> completions.
//
// Replaces the reference's per-request model execution (main.py:19-22: unpickle + two sklearn
// calls, serialized on the event loop) with a server-side batcher (BASELINE north star): every
// request submitted while the previous batch is on the GPU is coalesced into the next launch.
//
//   submit() (any thread, lock-free fast append under a short mutex)
//     -> batcher thread: drains up to max_batch rows, packs them into a host-pinned,
//        device-mapped slot (zero-copy: the kernel reads x and writes (idx, p) over the host
//        link directly, no hipMemcpy), launches launch_linear_small on a high-priority stream,
//        records an event; up to `slots` batches are in flight;
//     -> completer thread: polls the oldest slot's event, groups results by Sink and hands them
//        over (HTTP IO threads, Python futures, blocking callers).
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

namespace mlapi {

enum Status : int32_t {
  ST_OK = 0,
  ST_NONFINITE = 1,     // NaN / inf probability (reference: json.dumps raises -> HTTP 500)
  ST_NO_MODEL = 2,      // checkpoint missing (reference: open() raises -> HTTP 500)
  ST_SHAPE = 3,         // feature count mismatch
  ST_DEVICE_ERROR = 4,  // launch failure / injected fault
  ST_SHUTDOWN = 5,
};

struct Model {
  int kind = KIND_MULTINOMIAL;
  int F = 0;          // features
  int K = 0;          // rows of W (1 for binary kinds)
  int dtype = DT_F64; // device compute dtype (f64 / f32)
  uint64_t version = 0;
  std::vector<double> W, b;             // host float64 copies (CPU backend + reload)
  std::vector<std::string> label_json;  // pre-rendered JSON per class index
  int device = -1;
  void* dW = nullptr;
  void* db = nullptr;
  ~Model();
};

struct Completion {
  uint64_t tag;
  int32_t idx;
  int32_t status;
  double p;
  int64_t latency_ns;  // submit -> completion
};

class Sink {
 public:
  virtual ~Sink() = default;
  // Called on the engine's completion thread; must not block for long.
  virtual void on_complete(const Completion* c, size_t n, const std::shared_ptr<const Model>& model) = 0;
};

struct EngineConfig {
  int device = -1;        // HIP device ordinal, -1 = CPU backend
  int max_batch = 256;    // rows per launch
  int max_wait_us = 0;    // 0 = continuous batching; >0 = also wait up to this long to fill a batch
  int slots = 4;          // batches in flight
  int dtype = DT_F64;     // device compute dtype for served models (f64 = bit parity with sklearn)
  int max_features = 256; // per-request feature cap
  int watchdog_ms = 2000; // batch not complete after this -> engine marked unhealthy
  int fail_every = 0;     // fault injection: fail every N-th batch with ST_DEVICE_ERROR
  int delay_us = 0;       // fault injection: extra per-batch delay
  int spin_us = 0;        // batcher polls the queue this long before sleeping on the condvar
                          // (saves the futex wake-up on the request path under load)
  int max_queue = 1 << 20;  // backpressure: rows waiting for the batcher; beyond it submit is refused
  bool persistent = false;  // GPU: one resident kernel fed through a host mailbox instead of a
                            // launch per batch (serve_persistent_kernel, linear_small.hip)
  int persistent_idle_ms = 5;  // the resident kernel exits after this long without work
};

struct EngineStats {
  uint64_t requests = 0, batches = 0, errors = 0;
  uint64_t kernel_launches = 0;     // persistent mode: (re)launches of the resident kernel
  uint64_t rejected = 0;            // rows refused by backpressure (max_queue)
  uint64_t batch_hist[12] = {0};    // batch size buckets: 1,2,4,...,2048+
  uint64_t latency_hist[24] = {0};  // latency buckets in powers of two of 1us: <1us .. >=2^23us
  double latency_sum_us = 0;
  double device_us_sum = 0;         // launch -> completion observed by the completer
  uint64_t queue_depth = 0;
  uint64_t model_version = 0;
  bool healthy = true;
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
  // Blocking convenience API (tests / bulk scoring through the batcher).
  void predict(const double* X, int64_t B, int F, int32_t* idx, double* p, int32_t* status);

  EngineStats stats() const;
  const EngineConfig& config() const { return cfg_; }
  bool healthy() const { return healthy_.load(std::memory_order_relaxed); }
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
    void* hx = nullptr;       // host pinned, device mapped (inputs, model dtype)
    void* dx = nullptr;
    int32_t* hidx = nullptr;  // host pinned outputs
    int32_t* didx = nullptr;
    void* hp = nullptr;
    void* dp = nullptr;
    hipEvent_t ev = nullptr;
    std::vector<Meta> metas;
    std::vector<int32_t> pre_status;  // per-row status decided before launch
    std::shared_ptr<const Model> model;
    int64_t t_launch = 0;
    uint64_t batch = 0;  // persistent mode: global batch index (mailbox sequence - 1)
    int n = 0;
    bool launched = false;
    bool failed = false;
  };

  void batcher_loop();
  void completer_loop();
  bool wait_persistent(Slot& s, int si);
  void run_cpu(std::vector<Meta>& metas, const std::vector<double>& xs, const std::shared_ptr<const Model>& m);
  void finish(Slot& s, const int32_t* idx, const double* p, const int32_t* status);
  void deliver(std::vector<Meta>& metas, const int32_t* idx, const double* p, const int32_t* st,
               const std::shared_ptr<const Model>& m, int64_t now);
  void record_batch(size_t n);

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
  bool batcher_sleeping_ = false;  // guarded by q_mu_: submit wakes the batcher only if true
  std::atomic<int> q_count_{0};    // rows queued (lock-free hint for the batcher's spin phase)

  // GPU slots
  hipStream_t stream_ = nullptr;
  std::vector<Slot> slots_;
  std::mutex s_mu_;
  std::condition_variable s_cv_;
  std::deque<int> free_slots_;
  std::deque<int> inflight_;
  bool batcher_done_ = false;

  // persistent mode: host-pinned mailbox (device-visible), its stop word, the resident kernel's
  // stream; kernel_running_ / relaunch bookkeeping are owned by the completer thread
  ServeMailSlot* mail_h_ = nullptr;
  ServeMailSlot* mail_d_ = nullptr;
  uint32_t* done_h_ = nullptr;  // one word per slot, 64 B apart
  uint32_t* done_d_ = nullptr;
  uint32_t* stop_h_ = nullptr;
  uint32_t* stop_d_ = nullptr;
  hipStream_t pstream_ = nullptr;
  bool kernel_running_ = false;
  uint64_t idle_ticks_ = 0;
  uint64_t next_batch_ = 0;     // batcher thread only
  int64_t last_done_ns_ = 0;   // completer thread only

  std::thread batcher_, completer_;
  std::atomic<bool> healthy_{true};

  mutable std::mutex st_mu_;
  EngineStats stats_;
  uint64_t batch_counter_ = 0;
};

// Reference float64 implementation of the fused epilogue (CPU backend + host-side oracle).
void cpu_linear_predict(const Model& m, const double* X, int64_t B, int32_t* idx, double* p);

int64_t now_ns();

}  // namespace mlapi
