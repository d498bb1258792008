// Native HTTP/1.1 front end for the serving engine.
//
// The reference spends ~80% of every request in uvicorn/h11 + FastAPI + pydantic,
// and its multi-worker mode stalls 44 ms per response on Nagle/delayed-ACK. This
// server keeps the reference's HTTP surface but moves the hot path native:
//
//  * N IO threads, each with its own SO_REUSEPORT listener + epoll loop (the kernel spreads
//    connections; DP ranks can share one port the same way), TCP_NODELAY on every socket, every
//    response emitted with a single send();
//  * fast path: `POST /predict`, JSON content type, body that is a plain JSON object whose
//    required keys are finite JSON numbers (extra keys ignored) -> parsed straight into the
//    engine queue; the response {"prediction":...,"probability":repr(p)} is rendered natively,
//    byte-identical to FastAPI's JSONResponse;
//  * everything else (validation errors, /files/, /docs, /openapi.json, 404/405, anything a
//    strict parser would have to guess about) is handed to the Python ASGI app through
//    next_slow()/respond(), so error bodies stay exactly FastAPI's.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../runtime/engine.h"

namespace mlapi {

struct ServerConfig {
  std::string host = "127.0.0.1";
  int port = 8000;
  int io_threads = 2;
  bool reuseport = true;
  std::vector<std::string> feature_names;  // JSON keys of the /predict body, in W's column order
  std::string predict_path = "/predict";
  std::string server_header = "uvicorn";
  bool fast_path = true;
  size_t max_body = 64u << 20;
  size_t max_header = 64u << 10;
  size_t pipeline_cap = 1u << 20;  // unparsed bytes buffered behind an outstanding request (then EPOLLIN off)
  int backlog = 4096;
  bool access_log = false;         // uvicorn-format access log lines
  int access_log_fd = 2;
  // DP serving: while the engine is unhealthy, close this rank's SO_REUSEPORT listeners so the
  // kernel routes new connections to the healthy ranks; a probe row every health_probe_ms
  // re-admits the rank once a batch succeeds again.
  bool health_dispatch = false;
  int health_probe_ms = 100;
  // Busy-poll window: after activity an IO thread polls epoll (timeout 0) and its completion
  // queue for this long before blocking, and the engine's completer then hands it batches
  // without an eventfd write (no wake-up on the request path). 0 = always block.
  int io_spin_us = 0;
  // Wait-spin: an IO thread with rows in the engine watches its hand-off flag in user space for up
  // to this long before blocking in epoll_wait (no eventfd write for the completer, no wake-up on
  // the request path). 0 = off. 1-5 us measured +4-21 % c=64 req/s over 0 on three boxes, 15-30
  // us lost (the spinning threads take the load generator's CPU): profiles/r4_waitspin/.
  int io_wait_spin_us = 3;
  // Rows of this thread on the resident kernel (ServeRing) and no socket event: watch their records
  // in user space this long before the next epoll_wait(0) (no syscall per check). 0 = never spin.
  int io_ring_spin_us = 5;
  // ... or, when > 0, sleep in epoll_pwait2 for this long instead of spinning (a socket event
  // still wakes the thread; timer slack set to 1 us): a context switch instead of a spin.
  int io_ring_sleep_us = 0;
  int idle_max_conns = 0;  // idle-engine path only while <= this many connections are open (0 = any)
  // Low-load busy-poll: while the whole server holds at most io_spin_max_conns open connections
  // (a batch=1 client), an IO thread that just had activity polls for this long before blocking,
  // so the client's next request does not pay an idle-thread wake-up. Under concurrency (more
  // connections) the threads block as usual and no CPU is spent spinning. 0 = off.
  int io_spin_lowload_us = 50;
  int io_spin_max_conns = 2;
  // Connection steering by SO_INCOMING_CPU: every steer_every requests an IO thread reads the CPU
  // that last processed a connection's incoming segments (for loopback, the client thread's CPU;
  // for a NIC, its RX queue's). A plan (recomputed every 100 ms from the connections' stable CPUs)
  // gives each such CPU one IO thread, or two when its connections exceed a thread's share, and an
  // idle connection whose CPU is planned elsewhere moves there: connections driven from one CPU
  // share one IO thread, so a burst of their requests lands in one epoll round (one wake-up)
  // instead of one per thread. A churn guard pauses it when client CPUs keep moving. 0 = off.
  int io_steer = 1;
  int steer_every = 32;
  int steer_stable = 3;  // samples in a row on one CPU before a connection may move
  // IO thread i runs on CPU io_cpus[i] (threads past the list: wherever the scheduler puts them). A NIC
  // deployment pins them next to the RX queues' CPUs; bench.py gives them physical cores of their
  // own beside the load generator's (an unpinned IO thread sharing a core with another one or a
  // client thread is what made the same binary measure 1.3 or 2.3 M req/s run to run).
  std::vector<int> io_cpus;
  bool stage_timing = true;  // per-stage CPU accounting + HTTP latency histogram (a few rdtsc per request)
  // Connection dispatch (dispatch.h): "acceptor" (default) = one acceptor per serving group hands
  // every new connection to the next healthy replica / IO thread, round robin; "source" = the same
  // with source-address affinity (a client address keeps its replica); "reuseport" = every IO
  // thread listens on the port itself and the kernel hashes connections over the listeners.
  std::string dispatch = "acceptor";
  std::string dispatch_group;  // "" = named after host:port
  int dispatch_rank = 0;       // this replica's rank (reported to the group's leader)
  // dispatch = source: a client address this replica claims - its connections come here from the
  // first on (e.g. the co-located load generator's address), instead of round robin ("" = none)
  std::string dispatch_claim;
};

struct SlowRequest {
  uint64_t token = 0;
  std::string method, target, http_version;
  std::vector<std::pair<std::string, std::string>> headers;  // names lower-cased
  std::string body;
  std::string client_host, server_host;
  int client_port = 0, server_port = 0;
};

// Where the IO threads spend their time (exclusive, per stage; rdtsc-clocked, summed over the
// threads): the per-request CPU breakdown of the serving front end. Also the
// names of the roctx ranges emitted under MLAPI_ROCTX=1 ("mlapi.http.<stage>").
enum ServerStage : int {
  SS_POLL = 0,   // epoll_wait (blocking: idle, not CPU) + loop overhead
  SS_RECV,       // recv() syscalls
  SS_PARSE,      // HTTP + JSON parse of requests
  SS_SUBMIT,     // handing parsed rows to the engine (submit_many)
  SS_IDLE_GPU,   // waiting for the GPU in this thread: idle-engine launches (run_idle), ring record watch
  SS_RENDER,     // JSON response rendering
  SS_SEND,       // send() syscalls
  SS_HANDOFF,    // completion / slow-path hand-offs drained from other threads
  SS_COUNT
};
const char* server_stage_name(int s);
constexpr int HTTP_LAT_BUCKETS = 24;  // power-of-two microsecond buckets: <1us .. >=2^23us

struct ServerStats {
  uint64_t fast = 0, slow = 0, responses = 0, connections = 0, errors = 0, bad_requests = 0;
  uint64_t steered = 0;        // connections moved between IO threads by io_steer
  uint64_t steer_pauses = 0;   // ... times its churn guard paused it
  std::vector<int> conns_per_thread;  // open connections per IO thread
  std::vector<std::vector<int>> steer_plan;  // io_steer: {cpu, connections, thread 1, thread 2, thread 3}
  uint64_t listen_closes = 0;  // health_dispatch: times this rank left its dispatch group
  bool accepting = true;
  uint64_t stage_ns[SS_COUNT] = {};
  // end-to-end inside the server: request fully parsed -> its response handed to send()
  uint64_t http_latency_hist[HTTP_LAT_BUCKETS] = {};
  uint64_t http_latency_sum_ns = 0, http_latency_count = 0;
};

class ConnDispatcher;

class IoThread;

class HttpServer {
 public:
  HttpServer(Engine* engine, const ServerConfig& cfg);
  ~HttpServer();
  void start();
  void stop();
  int port() const { return bound_port_; }
  bool next_slow(SlowRequest* out, int timeout_ms);
  void respond(uint64_t token, int status, const std::string& reason,
               const std::vector<std::pair<std::string, std::string>>& headers, const std::string& body,
               bool close);
  ServerStats stats() const;
  const ServerConfig& config() const { return cfg_; }
  std::atomic<int> open_conns{0};  // keep-alive connections open across all IO threads
  Engine* engine() const { return engine_; }
  // false while health_dispatch has taken this rank out of its SO_REUSEPORT group
  bool accepting() const { return accepting_.load(std::memory_order_relaxed); }
  int listeners() const;  // IO threads currently holding a listening socket

  // internal, used by IoThread
  void push_slow(SlowRequest&& r);
  // io_steer: the IO thread that owns connections whose segments arrive on `cpu` (claimed for the
  // least-loaded thread on first sight; claims not seen for a second expire)
  int steer_target(int cpu, int self, uint32_t key);
  void steer_moved();  // a connection moved (churn guard)
  void steer_count(int old_cpu, int new_cpu);  // a connection's stable CPU changed (-1: none)
  IoThread* io_thread(int i) const { return threads_[(size_t)i].get(); }
  int io_thread_count() const { return (int)threads_.size(); }
  bool acceptor_mode() const { return acceptor_; }
  ConnDispatcher* dispatcher() const { return dispatcher_.get(); }

 private:
  Engine* engine_;
  ServerConfig cfg_;
  int bound_port_ = 0;
  std::vector<std::unique_ptr<IoThread>> threads_;
  std::mutex slow_mu_;
  std::condition_variable slow_cv_;
  std::deque<SlowRequest> slow_q_;
  bool stopping_ = false;
  bool started_ = false;
  std::atomic<bool> accepting_{true};
  std::atomic<bool> health_stop_{false};
  std::thread health_;
  void health_loop();
  bool acceptor_ = false;
  std::unique_ptr<ConnDispatcher> dispatcher_;
  std::atomic<uint64_t> adopt_rr_{0};
  std::atomic<uint64_t> leaves_{0};  // acceptor mode: healthy -> unhealthy transitions
  void steer_replan(int64_t now_ms);
  std::unique_ptr<std::atomic<int>[]> cpu_conns_;   // connections whose stable incoming CPU is c
  std::unique_ptr<std::atomic<uint64_t>[]> plan_;   // per CPU: up to three IO threads (+1, 8 bits each)
  std::vector<int> home_;  // per CPU: the IO thread pinned on its physical core (io_cpus), -1 = none
  std::atomic<int64_t> plan_ms_{0};
  std::atomic<int> steer_share_{1};  // the plan's connections per IO thread
  std::mutex plan_mu_;
  std::atomic<int64_t> steer_win_ms_{0}, steer_win_moves_{0}, steer_pause_until_ms_{0};
  std::atomic<uint64_t> steer_pauses_{0};
  int steer_ncpu_ = 0;
};

// HTTP date (RFC 7231 IMF-fixdate), cached per second.
const std::string& http_date_now();  // per-thread cache

}  // namespace mlapi
