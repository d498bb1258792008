// Native HTTP/1.1 server (see server.h).
#include "server.h"

#include "dispatch.h"
#include "json_body.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sched.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/prctl.h>
#include <sys/socket.h>
#include <unistd.h>
#include <x86intrin.h>

#include <cerrno>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <algorithm>
#include <chrono>
#include <cstring>
#include <ctime>
#include <stdexcept>
#include <unordered_map>

#include "../runtime/float_repr.h"
#include "../runtime/trace.h"

namespace mlapi {

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
const std::string& http_date_now() {  // per-thread cache, re-rendered once a second
  thread_local time_t cached_t = 0;
  thread_local std::string cached;
  const time_t t = time(nullptr);
  if (t != cached_t) {
    struct tm g;
    gmtime_r(&t, &g);
    char buf[64];
    strftime(buf, sizeof buf, "%a, %d %b %Y %H:%M:%S GMT", &g);
    cached = buf;
    cached_t = t;
  }
  return cached;
}

static inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

static inline void lower_inplace(std::string& s) {
  for (char& c : s)
    if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
}

static inline std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t')) --b;
  return s.substr(a, b - a);
}

namespace {

inline bool is_hex(char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

}  // namespace

// ------------------------------------------------------------------------------------------------
// IO thread
// ------------------------------------------------------------------------------------------------
namespace {
inline int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

// rdtsc ticks -> ns, calibrated once (HttpServer::start, off the request path)
double tsc_ns_per_tick() {
  static const double r = [] {
    const int64_t n0 = mono_ns();
    const uint64_t t0 = __rdtsc();
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    const int64_t n1 = mono_ns();
    const uint64_t t1 = __rdtsc();
    return t1 > t0 ? (double)(n1 - n0) / (double)(t1 - t0) : 1.0;
  }();
  return r;
}

const char* const kStageRange[SS_COUNT] = {"mlapi.http.poll",   "mlapi.http.recv",   "mlapi.http.parse",
                                           "mlapi.http.submit", "mlapi.http.idle_gpu", "mlapi.http.render",
                                           "mlapi.http.send",   "mlapi.http.handoff"};
}  // namespace

const char* server_stage_name(int s) {
  static const char* const names[SS_COUNT] = {"poll", "recv", "parse", "submit", "idle_gpu", "render", "send",
                                              "handoff"};
  return s >= 0 && s < SS_COUNT ? names[s] : "?";
}

namespace {

constexpr uint64_t ID_LISTEN = 0;
constexpr uint64_t ID_EVENT = 1;

struct Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in;
  size_t in_pos = 0;
  std::string out;
  size_t out_pos = 0;
  bool waiting = false;       // a request is outstanding (engine or Python)
  bool close_after = false;   // close once `out` is flushed
  bool sent_continue = false;
  bool epollout = false;
  bool paused = false;        // EPOLLIN dropped: too many unparsed bytes behind an outstanding request
  std::string client_host, server_host;
  int client_port = 0, server_port = 0;
  std::string req_line;       // access log: request line of the outstanding request
  uint64_t t_req = 0;         // rdtsc when the outstanding request was fully parsed
  // io_steer
  uint32_t nreq = 0;          // fast-path requests parsed on this connection
  int in_cpu = -1;            // SO_INCOMING_CPU at the last sample ...
  int same_n = 0;             // ... and on how many samples in a row
  int stable_cpu = -1;        // the CPU it counts for in the steering plan
  uint32_t key = 0;           // (reserved) a per-connection key that survives moves
  int flips = 0;              // stable-CPU changes within 5 s of each other ...
  int64_t flip_ns = 0;
  int64_t unsteered_until = 0;  // ... 3 of them: not steered until then
  int move_to = -1;           // IO thread to hand the connection to once it is idle
  int64_t moved_ns = 0;       // when it last moved (at most one move per 50 ms)
};

// A run of engine completions that share one model (render_fast's unit).
struct FastSeg {
  size_t begin;  // index of the run's first completion
  std::shared_ptr<const Model> model;
};

struct SlowResp {
  uint64_t conn_id;
  std::string bytes;
  bool close;
};

void addr_to_str(const sockaddr_storage& ss, std::string& host, int& port) {
  char buf[INET6_ADDRSTRLEN] = {0};
  if (ss.ss_family == AF_INET) {
    const auto* a = reinterpret_cast<const sockaddr_in*>(&ss);
    inet_ntop(AF_INET, &a->sin_addr, buf, sizeof buf);
    port = ntohs(a->sin_port);
  } else {
    const auto* a = reinterpret_cast<const sockaddr_in6*>(&ss);
    inet_ntop(AF_INET6, &a->sin6_addr, buf, sizeof buf);
    port = ntohs(a->sin6_port);
  }
  host = buf;
}

int make_listener(const std::string& host, int port, bool reuseport, int backlog, int* bound_port) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE | AI_NUMERICSERV;
  addrinfo* res = nullptr;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host.empty() ? nullptr : host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("getaddrinfo failed for " + host);
  int fd = socket(res->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, IPPROTO_TCP);
  if (fd < 0) {
    freeaddrinfo(res);
    throw std::runtime_error("socket() failed");
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (reuseport) setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  if (bind(fd, res->ai_addr, res->ai_addrlen) != 0) {
    const int e = errno;
    freeaddrinfo(res);
    close(fd);
    throw std::runtime_error("bind(" + host + ":" + ps + ") failed: " + strerror(e));
  }
  freeaddrinfo(res);
  if (listen(fd, backlog) != 0) {
    close(fd);
    throw std::runtime_error("listen() failed");
  }
  sockaddr_storage ss{};
  socklen_t sl = sizeof ss;
  getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &sl);
  std::string h;
  addr_to_str(ss, h, *bound_port);
  return fd;
}

}  // namespace

class IoThread : public Sink {
 public:
  IoThread(HttpServer* srv, int index, int listen_fd) : srv_(srv), index_(index), lfd_(listen_fd) {
    epfd_ = epoll_create1(EPOLL_CLOEXEC);
    evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (epfd_ < 0 || evfd_ < 0) throw std::runtime_error("epoll/eventfd creation failed");
    epoll_event ev{};
    ev.events = EPOLLIN;
    if (lfd_ >= 0) {  // reuseport mode: this thread's own listener; acceptor mode: adopt() hands connections
      ev.data.u64 = ID_LISTEN;
      epoll_ctl(epfd_, EPOLL_CTL_ADD, lfd_, &ev);
    }
    listening_.store(lfd_ >= 0);
    ev.data.u64 = ID_EVENT;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
    const auto& cfg = srv_->config();
    nfeat_ = cfg.feature_names.size();
    body_parser_ = std::make_unique<PredictBodyParser>(cfg.feature_names);
  }
  ~IoThread() override {
    for (auto& kv : conns_) close(kv.second->fd);
    if (lfd_ >= 0) close(lfd_);
    close(evfd_);
    close(epfd_);
  }

  void start() { th_ = std::thread([this] { loop(); }); }
  void stop() {
    stop_.store(true);
    wake();
    if (th_.joinable()) th_.join();
  }

  // Sink: engine completer thread -> this IO thread.
  void on_complete(const Completion* c, size_t n, const std::shared_ptr<const Model>& model) override {
    {
      std::lock_guard<std::mutex> lk(mu_);
      // appended to reusable buffers (no allocation per hand-off once they have grown)
      if (fast_seg_.empty() || fast_seg_.back().model != model) fast_seg_.push_back(FastSeg{fast_c_.size(), model});
      fast_c_.insert(fast_c_.end(), c, c + n);
    }
    wake();
  }

  // Acceptor mode: a connected socket from the group's dispatcher (any thread).
  void adopt(int fd) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      adopted_.push_back(fd);
    }
    wake();
  }

  // io_steer: an idle connection handed over by another IO thread (a new id is assigned here)
  void adopt_conn(std::unique_ptr<Conn> c) {
    n_open_.fetch_add(1, std::memory_order_relaxed);  // counted now: io_steer's cap sees moves in flight
    {
      std::lock_guard<std::mutex> lk(mu_);
      moved_in_.push_back(std::move(c));
    }
    wake();
  }

  void post_slow(uint64_t conn_id, std::string&& bytes, bool close) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      slow_.push_back(SlowResp{conn_id, std::move(bytes), close});
    }
    wake();
  }

  std::atomic<uint64_t> n_fast{0}, n_slow{0}, n_resp{0}, n_conn{0}, n_err{0}, n_bad{0}, n_listen_close{0};
  std::atomic<uint64_t> n_steered{0};
  int open_count() const { return n_open_.load(std::memory_order_relaxed); }
  // published copies of the stage clock / latency histogram (ticks; see ServerStats)
  std::atomic<uint64_t> pub_stage[SS_COUNT] = {};
  std::atomic<uint64_t> pub_lat[HTTP_LAT_BUCKETS] = {};
  std::atomic<uint64_t> pub_lat_sum{0}, pub_lat_n{0};

 private:
  // Hand-off from other threads: a spinning IO thread sees `pending_` on its next poll; a blocked
  // one needs the eventfd. Both flags are seq_cst so the spin -> block transition cannot lose a
  // wake (the IO thread clears spinning_ and then re-reads pending_ before it blocks).
  void wake() {
    pending_.store(true);
    if (spinning_.load()) return;
    // Only a thread blocked (or about to block) in epoll_wait needs the eventfd: a running one
    // sees `pending_` before it blocks again. Dekker pair with loop(): it stores blocked_ and then
    // loads pending_, this stores pending_ and then loads blocked_ (all seq_cst), so at least one
    // side sees the other and no hand-off is lost. Under load most IO threads are running, and
    // each eventfd write that wakes a sleeping reader costs the completer ~1 us.
    if (!blocked_.load()) return;
    if (!signaled_.exchange(true)) {
      const uint64_t one = 1;
      ssize_t r = write(evfd_, &one, sizeof one);
      (void)r;
    }
  }

  // ---- stage clock: exclusive time per stage (ServerStage), rdtsc between transitions
  void stage(int st) {
    if (!timing_) return;
    const uint64_t t = __rdtsc();
    st_acc_[st_cur_] += t - st_last_;
    st_last_ = t;
    st_cur_ = st;
  }
  struct Stage {
    IoThread* io;
    int prev;
    bool rtx;
    Stage(IoThread* i, int st) : io(i), prev(i->st_cur_), rtx(Roctx::get().enabled) {
      io->stage(st);
      if (rtx) Roctx::get().push(kStageRange[st]);
    }
    ~Stage() {
      if (rtx) Roctx::get().pop();
      io->stage(prev);
    }
  };
  void publish_clock() {
    if (!timing_) return;
    stage(st_cur_);
    for (int i = 0; i < SS_COUNT; ++i) pub_stage[i].store(st_acc_[i], std::memory_order_relaxed);
    for (int i = 0; i < HTTP_LAT_BUCKETS; ++i) pub_lat[i].store(lat_hist_[i], std::memory_order_relaxed);
    pub_lat_sum.store(lat_sum_, std::memory_order_relaxed);
    pub_lat_n.store(lat_n_, std::memory_order_relaxed);
  }
  // the response to c's outstanding request was just handed to send()
  void note_latency(uint64_t t_req) {
    if (!timing_ || t_req == 0) return;
    const uint64_t d = __rdtsc() - t_req;
    const uint64_t us = (uint64_t)((double)d * ns_per_tick_ * 1e-3);
    const int b = us == 0 ? 0 : std::min(HTTP_LAT_BUCKETS - 1, 64 - __builtin_clzll(us));
    ++lat_hist_[b];
    lat_sum_ += d;
    ++lat_n_;
  }

  // Rows of this thread's resident-kernel ring whose records have landed: render them (rows bounced
  // stale by a hot reload went to the engine queue: their answers come as hand-offs).
  void harvest_ring() {
    if (ring_ == nullptr || ring_->pending() == 0) return;
    ring_c_.clear();
    ring_seg_.clear();
    int requeued = 0;
    ring_->poll(ring_c_, ring_seg_, this, &requeued);
    outstanding_ += requeued;
    for (size_t k = 0; k < ring_seg_.size(); ++k) {
      const size_t b = ring_seg_[k].begin, e = k + 1 < ring_seg_.size() ? ring_seg_[k + 1].begin : ring_c_.size();
      render_fast(ring_seg_[k].model, ring_c_.data() + b, e - b);
    }
  }

  void flush_submits() {
    if (pend_tags_.empty()) return;
    Stage sg(this, SS_SUBMIT);
    const int n = (int)pend_tags_.size();
    // the round's rows go into this thread's ring for the resident kernel (no packet, no batcher /
    // completer hop); not eligible (wide model, no resident kernel, ...) -> the idle path or the queue
    if (ring_ != nullptr && ring_->submit(pend_x_.data(), n, (int)nfeat_, pend_tags_.data())) {
      pend_x_.clear();
      pend_tags_.clear();
      return;
    }
    {
      // idle engine: this thread launches the rows itself and renders the responses right away
      // (no batcher / completer hand-off, no eventfd round trip)
      idle_done_.clear();
      std::shared_ptr<const Model> m;
      // wide models too while the server is at low load (a batch=1 client)
      const int conns = srv_->open_conns.load(std::memory_order_relaxed);
      const bool low = conns <= srv_->config().io_spin_max_conns;
      const int idle_max = srv_->config().idle_max_conns;
      bool ran = false;
      if (idle_max <= 0 || conns <= idle_max) {
        Stage sg2(this, SS_IDLE_GPU);
        ran = srv_->engine()->run_idle(pend_x_.data(), n, (int)nfeat_, pend_tags_.data(), idle_done_, m, low);
      }
      if (ran) {
        pend_x_.clear();
        pend_tags_.clear();
        render_fast(m, idle_done_.data(), idle_done_.size());  // may parse pipelined requests into
                                                               // pend_*: flushed on the next round
        return;
      }
    }
    const int r = srv_->engine()->submit_many(pend_x_.data(), n, (int)nfeat_, pend_tags_.data(), this);
    if (r > 0) outstanding_ += r;
    if (r != n) {
      // rows [0, r) were queued; the rest: overloaded -> 503 + Retry-After, engine stopping -> 500
      for (int i = r > 0 ? r : 0; i < n; ++i) {
        const uint64_t id = pend_tags_[i];
        auto it = conns_.find(id);
        if (it == conns_.end()) continue;
        it->second->waiting = false;
        if (r != 0) {  // SUBMIT_BUSY, or a partial accept
          service_unavailable(it->second.get());
          log_access(it->second.get(), 503, "Service Unavailable");
        } else {
          internal_error(it->second.get());
          log_access(it->second.get(), 500, "Internal Server Error");
        }
        flush(it->second.get());
      }
    }
    pend_x_.clear();
    pend_tags_.clear();
  }

  void loop() {
    char name[16];
    snprintf(name, sizeof name, "mlapi-io-%d", index_);
    pthread_setname_np(pthread_self(), name);
    if ((size_t)index_ < srv_->config().io_cpus.size()) {
      cpu_set_t set;
      CPU_ZERO(&set);
      const int cpu = srv_->config().io_cpus[(size_t)index_];
      if (cpu >= 0 && cpu < CPU_SETSIZE) {
        CPU_SET(cpu, &set);
        if (pthread_setaffinity_np(pthread_self(), sizeof set, &set) != 0)
          fprintf(stderr, "mlapi: io thread %d: cannot pin to cpu %d (left unpinned)\n", index_, cpu);
      }
    }
    timing_ = srv_->config().stage_timing;
    ns_per_tick_ = tsc_ns_per_tick();
    st_last_ = __rdtsc();
    st_cur_ = SS_POLL;
    epoll_event evs[256];
    const int64_t always_spin_ns = (int64_t)srv_->config().io_spin_us * 1000;
    const int64_t lowload_spin_ns = (int64_t)srv_->config().io_spin_lowload_us * 1000;
    const int lowload_conns = srv_->config().io_spin_max_conns;
    const int64_t wait_spin_ns = (int64_t)srv_->config().io_wait_spin_us * 1000;
    const int64_t ring_spin_ns = (int64_t)srv_->config().io_ring_spin_us * 1000;
    const int64_t ring_sleep_ns = (int64_t)srv_->config().io_ring_sleep_us * 1000;
    if (ring_sleep_ns > 0) prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // us-scale epoll_pwait2 timeouts
    bool ring_sleep = false;  // this pass waits for the ring's records in epoll_pwait2
    bool ring_spun = false;   // spun since the last epoll_wait: poll the sockets before spinning again
    int64_t last_active = 0;
    int last_n = 0;  // events of the previous epoll_wait
    ring_ = srv_->engine() != nullptr ? srv_->engine()->open_ring() : nullptr;
    while (!stop_.load()) {
      harvest_ring();
      flush_submits();
      flush_log();
      publish_clock();
      int timeout = 200;
      // busy-poll window: always (io_spin_us), or at low load only (a batch=1 client)
      const int64_t spin_ns =
          always_spin_ns > 0 ? always_spin_ns
                             : (lowload_spin_ns > 0 && srv_->open_conns.load(std::memory_order_relaxed) <= lowload_conns
                                    ? lowload_spin_ns
                                    : 0);
      if (spin_ns > 0) {
        const int64_t now = mono_ns();
        if (now - last_active < spin_ns) {
          spinning_.store(true);
          timeout = 0;
        } else {
          spinning_.store(false);
          if (pending_.load()) timeout = 0;  // a hand-off raced with the transition
        }
      } else if (spinning_.load(std::memory_order_relaxed)) {
        spinning_.store(false);  // left the low-load regime: hand-offs need the eventfd again
        if (pending_.load()) timeout = 0;
      }
      if (ring_ != nullptr && ring_->pending() > 0) {
        // rows of this thread are on the GPU: no blocking wait. With nothing else to do (the last
        // poll found no event), watch their records in user space for a while first - the GPU leg
        // is a few us, an epoll_wait per check would be a syscall per pass
        timeout = 0;
        if (last_n == 0 && ring_sleep_ns > 0 && !pending_.load(std::memory_order_relaxed)) {
          // io_ring_sleep_us: sleep in the kernel for that long instead (a socket event still
          // wakes the thread at once); costs a context switch, saves the spin's CPU
          ring_sleep = true;
        } else if (last_n == 0 && !ring_spun && ring_spin_ns > 0 && !pending_.load(std::memory_order_relaxed)) {
          // one spin per epoll_wait: a steady trickle of landing records must not keep this thread
          // from reading its other connections' requests
          ring_spun = true;
          Stage sg(this, SS_IDLE_GPU);
          if (ring_->wait_any(ring_spin_ns)) continue;  // harvest first
        }
      }
      stage(SS_POLL);
      if (timeout != 0 && wait_spin_ns > 0 && outstanding_ > 0 && !spinning_.load(std::memory_order_relaxed)) {
        // rows of this thread are in the engine: watch for their hand-off in user space for a
        // bounded while before blocking (the completer then skips the eventfd write and this
        // thread its wake-up); `spinning_` tells wake() not to write it, and is cleared before
        // blocked_ is set below, so a hand-off that raced with the end of the spin is still seen
        spinning_.store(true);
        const int64_t until = mono_ns() + wait_spin_ns;
        while (!pending_.load(std::memory_order_acquire) && mono_ns() < until) _mm_pause();
        spinning_.store(false);
        if (pending_.load()) timeout = 0;
      }
      if (timeout != 0) {
        blocked_.store(true);
        if (pending_.load()) timeout = 0;  // a hand-off that did not write the eventfd
      }
      int n;
      if (ring_sleep) {
        ring_sleep = false;
        const timespec ts{0, (long)ring_sleep_ns};
        n = epoll_pwait2(epfd_, evs, 256, &ts, nullptr);
      } else {
        n = epoll_wait(epfd_, evs, 256, timeout);
      }
      ring_spun = false;
      blocked_.store(false);
      last_n = n;
      const bool spin_enabled = always_spin_ns > 0 || lowload_spin_ns > 0;
      if (n > 0 && spin_enabled) last_active = mono_ns();
      // hand-offs posted while spinning come without an eventfd write (also the ones that raced
      // with leaving the spin regime); with an eventfd pending too, its later drain finds nothing
      if (pending_.load()) {
        pending_.store(false);
        drain_pending();
        if (spin_enabled) last_active = mono_ns();
      }
      for (int i = 0; i < n; ++i) {
        const uint64_t id = evs[i].data.u64;
        if (id == ID_LISTEN) {
          if (lfd_ >= 0) accept_all();
        } else if (id == ID_EVENT) {
          uint64_t v;
          ssize_t r = read(evfd_, &v, sizeof v);
          (void)r;
          signaled_.store(false);
          pending_.store(false);
          drain_pending();
        } else {
          auto it = conns_.find(id);
          if (it == conns_.end()) continue;
          Conn* c = it->second.get();
          // One misbehaving connection (e.g. an allocation failure while buffering its request)
          // must never take the process down: drop that connection and keep serving.
          try {
            bool alive = true;
            if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR | EPOLLRDHUP)) alive = on_readable(c);
            if (alive && (evs[i].events & EPOLLOUT)) alive = flush(c);
          } catch (const std::exception&) {
            n_bad.fetch_add(1, std::memory_order_relaxed);
            if (conns_.count(id)) close_conn(c);
          }
        }
      }
      apply_listen_state();
    }
    if (ring_ != nullptr) srv_->engine()->close_ring(ring_);
    ring_ = nullptr;
  }

  // Health-aware dispatch (SO_REUSEPORT group membership): an IO thread whose engine is unhealthy
  // closes its listening socket, so the kernel stops routing new connections of the shared port
  // to this rank; it re-binds once the engine is healthy again. Connections already accepted keep
  // being served (their requests complete with 500 while the engine is down).
  void apply_listen_state() {
    if (srv_->acceptor_mode()) return;  // the group's dispatcher skips unhealthy replicas instead
    const bool want = srv_->accepting();
    if (want == listening_.load(std::memory_order_relaxed)) return;
    if (!want) {
      epoll_ctl(epfd_, EPOLL_CTL_DEL, lfd_, nullptr);
      close(lfd_);
      lfd_ = -1;
      listening_ = false;
      n_listen_close.fetch_add(1, std::memory_order_relaxed);
      return;
    }
    try {
      int bp = 0;
      const auto& cfg = srv_->config();
      lfd_ = make_listener(cfg.host, srv_->port(), true, cfg.backlog, &bp);
    } catch (const std::exception&) {
      return;  // retried on the next loop iteration (<= 200 ms)
    }
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = ID_LISTEN;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, lfd_, &ev);
    listening_ = true;
  }

 public:
  bool listening() const { return listening_.load(std::memory_order_relaxed); }

 private:
  // uvicorn-format access log ('INFO:     127.0.0.1:5000 - "POST /predict HTTP/1.1" 200 OK'),
  // buffered per IO thread and written with one write(2) per epoll round.
  void log_access(Conn* c, int status, const char* reason) {
    if (!srv_->config().access_log || c->req_line.empty()) return;
    log_ += "INFO:     ";
    log_ += c->client_host;
    log_ += ':';
    log_ += std::to_string(c->client_port);
    log_ += " - \"";
    log_ += c->req_line;
    log_ += "\" ";
    log_ += std::to_string(status);
    log_ += ' ';
    log_ += reason;
    log_ += '\n';
    c->req_line.clear();
  }
  void flush_log() {
    if (log_.empty()) return;
    size_t off = 0;
    while (off < log_.size()) {
      const ssize_t w = write(srv_->config().access_log_fd, log_.data() + off, log_.size() - off);
      if (w <= 0) break;
      off += (size_t)w;
    }
    log_.clear();
  }

  // EPOLLIN is dropped while a request is outstanding and more than pipeline_cap bytes of later
  // requests are already buffered (a client that keeps writing cannot grow server memory).
  void update_events(Conn* c) {
    epoll_event ev{};
    ev.events = EPOLLRDHUP | (c->paused ? 0u : (uint32_t)EPOLLIN) | (c->epollout ? (uint32_t)EPOLLOUT : 0u);
    ev.data.u64 = c->id;
    epoll_ctl(epfd_, EPOLL_CTL_MOD, c->fd, &ev);
  }

  void accept_all() {
    for (;;) {
      sockaddr_storage ss{};
      socklen_t sl = sizeof ss;
      const int fd = accept4(lfd_, reinterpret_cast<sockaddr*>(&ss), &sl, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      register_conn(fd, ss);
    }
  }

  void register_conn(int fd, const sockaddr_storage& ss) {
    {
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);  // never Nagle
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      c->id = next_id_++;
      {  // a per-connection key that survives moves (splitmix64 of the fd and the clock)
        uint64_t z = (uint64_t)fd * 0x9E3779B97F4A7C15ull + (uint64_t)mono_ns();
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        c->key = (uint32_t)(z ^ (z >> 31));
      }
      addr_to_str(ss, c->client_host, c->client_port);
      sockaddr_storage ls{};
      socklen_t ll = sizeof ls;
      getsockname(fd, reinterpret_cast<sockaddr*>(&ls), &ll);
      addr_to_str(ls, c->server_host, c->server_port);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = c->id;
      epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
      conns_.emplace(c->id, std::move(c));
      n_open_.fetch_add(1, std::memory_order_relaxed);
      n_conn.fetch_add(1, std::memory_order_relaxed);
      srv_->open_conns.fetch_add(1, std::memory_order_relaxed);
    }
  }

  void close_conn(Conn* c) {
    if (c->stable_cpu >= 0) srv_->steer_count(c->stable_cpu, -1);
    epoll_ctl(epfd_, EPOLL_CTL_DEL, c->fd, nullptr);
    close(c->fd);
    conns_.erase(c->id);  // destroys c
    n_open_.fetch_sub(1, std::memory_order_relaxed);
    srv_->open_conns.fetch_sub(1, std::memory_order_relaxed);
  }

  // returns false if the connection was closed
  bool on_readable(Conn* c) {
    char buf[65536];
    bool eof = false;
    Stage sg(this, SS_RECV);
    for (;;) {
      const ssize_t r = recv(c->fd, buf, sizeof buf, 0);
      if (r > 0) {
        c->in.append(buf, (size_t)r);
        if ((size_t)r < sizeof buf) break;
      } else if (r == 0) {
        eof = true;
        break;
      } else {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        if (errno == EINTR) continue;
        eof = true;
        break;
      }
    }
    if (eof) {
      close_conn(c);
      return false;
    }
    if (c->waiting && !c->paused && c->in.size() - c->in_pos > srv_->config().pipeline_cap) {
      c->paused = true;
      update_events(c);
    }
    stage(SS_PARSE);  // the rest of this call is parsing (process() switches to SEND itself)
    return process(c);
  }

  bool flush(Conn* c) {
    Stage sg(this, SS_SEND);
    while (c->out_pos < c->out.size()) {
      const ssize_t w = send(c->fd, c->out.data() + c->out_pos, c->out.size() - c->out_pos, MSG_NOSIGNAL);
      if (w > 0) {
        c->out_pos += (size_t)w;
      } else if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (!c->epollout) {
          c->epollout = true;
          update_events(c);
        }
        return true;
      } else if (w < 0 && errno == EINTR) {
        continue;
      } else {
        close_conn(c);
        return false;
      }
    }
    c->out.clear();
    c->out_pos = 0;
    if (c->epollout) {
      c->epollout = false;
      update_events(c);
    }
    if (c->close_after && !c->waiting) {
      close_conn(c);
      return false;
    }
    return true;
  }

  void append_response(Conn* c, int status, const char* reason, const char* ctype, const std::string& body,
                       const char* extra_headers = "") {
    std::string& o = c->out;
    o.reserve(o.size() + 160 + body.size());
    o += "HTTP/1.1 ";
    o += std::to_string(status);
    o += ' ';
    o += reason;
    o += "\r\ndate: ";
    o += http_date_now();
    o += "\r\nserver: ";
    o += srv_->config().server_header;
    o += "\r\ncontent-length: ";
    o += std::to_string(body.size());
    o += "\r\ncontent-type: ";
    o += ctype;
    if (c->close_after) o += "\r\nconnection: close";
    o += "\r\n";
    o += extra_headers;  // each "name: value\r\n"
    o += "\r\n";
    o += body;
    n_resp.fetch_add(1, std::memory_order_relaxed);
  }

  void internal_error(Conn* c) {
    append_response(c, 500, "Internal Server Error", "text/plain; charset=utf-8", "Internal Server Error");
    n_err.fetch_add(1, std::memory_order_relaxed);
  }

  // Backpressure (engine queue over max_queue): the request was not queued; the client may retry.
  void service_unavailable(Conn* c) {
    append_response(c, 503, "Service Unavailable", "application/json",
                     "{\"detail\":\"server overloaded, retry later\"}", "retry-after: 1\r\n");
    n_err.fetch_add(1, std::memory_order_relaxed);
  }

  void bad_request(Conn* c, int status, const char* reason) {
    c->close_after = true;
    append_response(c, status, reason, "text/plain; charset=utf-8", reason);
    n_bad.fetch_add(1, std::memory_order_relaxed);
  }

  // Responses of one batch of fast-path completions (each one then dispatches its connection's
  // pipelined requests and flushes).
  void render_fast(const std::shared_ptr<const Model>& model, const Completion* comps, size_t ncomp) {
    std::string& body = body_;
    Stage sg(this, SS_RENDER);
    for (size_t ci = 0; ci < ncomp; ++ci) {
      const Completion& cp = comps[ci];
      auto it = conns_.find(cp.tag);
      if (it == conns_.end()) continue;  // client went away
      Conn* c = it->second.get();
      c->waiting = false;
      const uint64_t t_req = c->t_req;
      bool ok = cp.status == ST_OK && model && cp.idx >= 0 && (size_t)cp.idx < model->label_json.size();
      if (ok) {
        body.clear();
        body += "{\"prediction\":";
        body += model->label_json[cp.idx];
        body += ",\"probability\":";
        ok = append_py_float(body, cp.p);
        body += '}';
      }
      if (ok) {
        append_response(c, 200, "OK", "application/json", body);
        log_access(c, 200, "OK");
      } else {
        internal_error(c);
        log_access(c, 500, "Internal Server Error");
      }
      {
        Stage sp(this, SS_PARSE);  // pipelined requests behind this one, then the flush (SEND)
        process(c);                // (may close c)
      }
      note_latency(t_req);
    }
  }

  void drain_pending() {
    Stage sg(this, SS_HANDOFF);
    // double-buffered: the spare vectors keep their capacity, so a hand-off allocates nothing
    std::vector<Completion>& fast_c = spare_c_;
    std::vector<FastSeg>& fast_seg = spare_seg_;
    fast_c.clear();
    fast_seg.clear();
    std::vector<SlowResp> slow;
    std::vector<int> adopted;
    std::vector<std::unique_ptr<Conn>> moved;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fast_c.swap(fast_c_);
      fast_seg.swap(fast_seg_);
      if (!slow_.empty()) slow.swap(slow_);
      if (!adopted_.empty()) adopted.swap(adopted_);
      if (!moved_in_.empty()) moved.swap(moved_in_);
    }
    for (int fd : adopted) {
      sockaddr_storage ss{};
      socklen_t sl = sizeof ss;
      getpeername(fd, reinterpret_cast<sockaddr*>(&ss), &sl);
      register_conn(fd, ss);
    }
    for (auto& c : moved) {
      // idle when it left its old thread; level-triggered EPOLLIN reports bytes that arrived meanwhile
      c->id = next_id_++;
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = c->id;
      epoll_ctl(epfd_, EPOLL_CTL_ADD, c->fd, &ev);
      const uint64_t id = c->id;
      conns_.emplace(id, std::move(c));  // n_open_ was counted by adopt_conn
    }
    outstanding_ = std::max<int64_t>(0, outstanding_ - (int64_t)fast_c.size());
    for (size_t k = 0; k < fast_seg.size(); ++k) {
      const size_t b = fast_seg[k].begin, e = k + 1 < fast_seg.size() ? fast_seg[k + 1].begin : fast_c.size();
      render_fast(fast_seg[k].model, fast_c.data() + b, e - b);
    }
    for (SlowResp& sr : slow) {
      auto it = conns_.find(sr.conn_id);
      if (it == conns_.end()) continue;
      Conn* c = it->second.get();
      c->waiting = false;
      if (!c->req_line.empty() && sr.bytes.size() > 12) {  // "HTTP/1.1 NNN reason\r\n..."
        const size_t le = sr.bytes.find("\r\n");
        const std::string st = sr.bytes.substr(13, le == std::string::npos ? 0 : le - 13);
        log_access(c, atoi(sr.bytes.c_str() + 9), st.c_str());
      }
      c->out += sr.bytes;
      if (sr.close) c->close_after = true;
      n_resp.fetch_add(1, std::memory_order_relaxed);
      const uint64_t t_req = c->t_req;
      process(c);  // dispatches pipelined requests, then flushes (may close c)
      note_latency(t_req);
    }
  }

  // Parse and dispatch as many complete requests as possible (one outstanding at a time).
  // Returns false if the connection was closed.
  bool process(Conn* c) {
    while (!c->waiting && !c->close_after) {
      const int r = parse_one(c);
      if (r == 0) break;  // need more bytes
      if (r < 0) break;   // error response queued, close_after set
    }
    if (c->in_pos > 0 && (c->in_pos == c->in.size() || c->in_pos > (1u << 16))) {
      c->in.erase(0, c->in_pos);
      c->in_pos = 0;
    }
    if (c->paused && (!c->waiting || c->in.size() - c->in_pos <= srv_->config().pipeline_cap)) {
      c->paused = false;
      update_events(c);
    }
    if (!flush(c)) return false;
    if (c->move_to >= 0 && !c->waiting && !c->close_after && c->in_pos == c->in.size() && c->out.empty() &&
        !c->epollout)
      return migrate(c);
    return true;
  }

  // io_steer: sample the connection's incoming CPU every steer_every fast-path requests; seen twice
  // in a row on a CPU another IO thread owns, the connection moves there once it is idle
  void steer_sample(Conn* c) {
    const int every = srv_->config().steer_every;
    if (srv_->config().io_steer <= 0 || every <= 0 || ++c->nreq % (uint32_t)every != 0) return;
    int cpu = -1;
    socklen_t l = sizeof cpu;
    if (getsockopt(c->fd, SOL_SOCKET, SO_INCOMING_CPU, &cpu, &l) != 0 || cpu < 0) return;
    if (cpu != c->in_cpu) {
      c->in_cpu = cpu;
      c->same_n = 1;
      return;
    }
    // only a CPU seen on steer_stable samples in a row counts (a client thread the scheduler keeps
    // moving gives no stable CPU, and its connections stay where they are)
    if (++c->same_n < std::max(2, srv_->config().steer_stable)) return;
    const int64_t now = mono_ns();
    if (now < c->unsteered_until) return;
    if (cpu != c->stable_cpu) {
      // a connection whose client keeps changing CPU (an unpinned client thread the scheduler
      // moves around) has no CPU to be grouped by: it leaves the plan for 10 s instead of chasing it
      c->flips = now - c->flip_ns < 5000000000LL ? c->flips + 1 : 1;
      c->flip_ns = now;
      if (c->flips >= 3) {
        srv_->steer_count(c->stable_cpu, -1);
        c->stable_cpu = -1;
        c->move_to = -1;
        c->flips = 0;
        c->unsteered_until = now + 10000000000LL;
        return;
      }
      srv_->steer_count(c->stable_cpu, cpu);
      c->stable_cpu = cpu;
    }
    const int t = srv_->steer_target(cpu, index_, c->key);
    if (t != index_ && t >= 0 && now - c->moved_ns > 50000000) c->move_to = t;
  }

  // hand an idle connection to another IO thread (returns false: it is no longer this thread's)
  bool migrate(Conn* c) {
    const int t = c->move_to;
    c->move_to = -1;
    if (t < 0 || t >= srv_->io_thread_count() || t == index_) return true;
    epoll_ctl(epfd_, EPOLL_CTL_DEL, c->fd, nullptr);
    auto it = conns_.find(c->id);
    std::unique_ptr<Conn> up = std::move(it->second);
    conns_.erase(it);
    n_open_.fetch_sub(1, std::memory_order_relaxed);
    up->moved_ns = mono_ns();
    up->nreq = 0;
    up->same_n = 0;
    n_steered.fetch_add(1, std::memory_order_relaxed);
    srv_->steer_moved();
    srv_->io_thread(t)->adopt_conn(std::move(up));
    return false;
  }

  static bool ieq(const char* a, size_t n, const char* lower_lit, size_t m) {
    if (n != m) return false;
    for (size_t i = 0; i < n; ++i) {
      char ch = a[i];
      if (ch >= 'A' && ch <= 'Z') ch = (char)(ch | 0x20);
      if (ch != lower_lit[i]) return false;
    }
    return true;
  }
  static bool icontains(const char* a, size_t n, const char* lower_lit, size_t m) {
    for (size_t i = 0; i + m <= n; ++i)
      if (ieq(a + i, m, lower_lit, m)) return true;
    return false;
  }
  // FastAPI's JSON content-type rule (json_ctype) on a view
  static bool json_ctype_view(const char* p, size_t n) {
    const char* semi = static_cast<const char*>(memchr(p, ';', n));
    if (semi) n = (size_t)(semi - p);
    while (n && (p[0] == ' ' || p[0] == '\t')) ++p, --n;
    while (n && (p[n - 1] == ' ' || p[n - 1] == '\t')) --n;
    if (n < 12 || !ieq(p, 12, "application/", 12)) return false;
    p += 12;
    n -= 12;
    return ieq(p, n, "json", 4) || (n > 5 && ieq(p + n - 5, 5, "+json", 5));
  }

  // Zero-allocation parse of the common request: `POST <predict_path>[?q] HTTP/1.1` with a
  // Content-Length, a JSON content type, no Expect / Transfer-Encoding, and a body the strict
  // parser accepts - parsed straight into the pending arena. 1 = queued for the engine,
  // 0 = incomplete (wait for bytes), -2 = anything else: the full parser below decides (and
  // produces the exact same responses it always did).
  int parse_fast(Conn* c) {
    const auto& cfg = srv_->config();
    if (!cfg.fast_path || cfg.access_log || nfeat_ == 0) return -2;
    const char* base = c->in.data() + c->in_pos;
    const size_t avail = c->in.size() - c->in_pos;
    if (avail < 5 || memcmp(base, "POST ", 5) != 0) return -2;
    const char* hend = static_cast<const char*>(memmem(base, avail, "\r\n\r\n", 4));
    if (hend == nullptr) return avail > cfg.max_header ? -2 : 0;
    const size_t hlen = (size_t)(hend - base) + 4;
    const char* le = static_cast<const char*>(memmem(base, hlen, "\r\n", 2));
    const char* t0 = base + 5;
    const char* sp = static_cast<const char*>(memchr(t0, ' ', (size_t)(le - t0)));
    if (sp == nullptr || (size_t)(le - sp - 1) != 8 || memcmp(sp + 1, "HTTP/1.1", 8) != 0) return -2;
    const char* q = static_cast<const char*>(memchr(t0, '?', (size_t)(sp - t0)));
    const char* pe = q ? q : sp;
    if ((size_t)(pe - t0) != cfg.predict_path.size() || memcmp(t0, cfg.predict_path.data(), (size_t)(pe - t0)) != 0)
      return -2;
    int64_t clen = -1;
    bool close = false, json = false, seen_ctype = false;
    const char* hp = le + 2;
    const char* hlim = base + hlen - 2;
    while (hp < hlim) {
      const char* e = static_cast<const char*>(memmem(hp, (size_t)(hlim - hp) + 2, "\r\n", 2));
      if (e == nullptr) return -2;
      const char* colon = static_cast<const char*>(memchr(hp, ':', (size_t)(e - hp)));
      if (colon == nullptr) return -2;
      const char* v = colon + 1;
      const char* ve = e;
      while (v < ve && (*v == ' ' || *v == '\t')) ++v;
      while (ve > v && (ve[-1] == ' ' || ve[-1] == '\t')) --ve;
      const size_t nl = (size_t)(colon - hp), vl = (size_t)(ve - v);
      if (ieq(hp, nl, "content-length", 14)) {
        if (vl == 0 || vl > 18) return -2;
        int64_t x = 0;
        for (size_t i = 0; i < vl; ++i) {
          if (v[i] < '0' || v[i] > '9') return -2;
          x = x * 10 + (v[i] - '0');
        }
        if (clen >= 0 && clen != x) return -2;
        clen = x;
      } else if (ieq(hp, nl, "transfer-encoding", 17) || ieq(hp, nl, "expect", 6)) {
        return -2;
      } else if (ieq(hp, nl, "connection", 10)) {
        close = close || icontains(v, vl, "close", 5);  // any Connection header (h11 joins them)
      } else if (ieq(hp, nl, "content-type", 12)) {
        if (!seen_ctype) json = json_ctype_view(v, vl);  // the first one (Starlette's headers[...])
        seen_ctype = true;
      }
      hp = e + 2;
    }
    if (clen < 0 || !json || (size_t)clen > cfg.max_body) return -2;
    if (avail - hlen < (size_t)clen) return 0;
    const size_t at = pend_x_.size();
    pend_x_.resize(at + nfeat_);
    if (!body_parser_->parse(base + hlen, (size_t)clen, pend_x_.data() + at)) {
      pend_x_.resize(at);
      return -2;
    }
    c->in_pos += hlen + (size_t)clen;
    c->sent_continue = false;
    if (close) c->close_after = true;
    c->waiting = true;
    c->t_req = timing_ ? __rdtsc() : 0;
    pend_tags_.push_back(c->id);
    n_fast.fetch_add(1, std::memory_order_relaxed);
    steer_sample(c);
    return 1;
  }

  // 1 = dispatched a request, 0 = incomplete, -1 = protocol error (response queued)
  int parse_one(Conn* c) {
    {
      const int f = parse_fast(c);
      if (f != -2) return f;
    }
    const auto& cfg = srv_->config();
    const char* base = c->in.data() + c->in_pos;
    const size_t avail = c->in.size() - c->in_pos;
    if (avail == 0) return 0;
    // tolerate stray CRLFs between requests (RFC 7230 3.5)
    size_t lead = 0;
    while (lead < avail && (base[lead] == '\r' || base[lead] == '\n')) ++lead;
    if (lead) {
      c->in_pos += lead;
      return avail > lead ? 1 : 0;
    }
    const void* hend_p = memmem(base, avail, "\r\n\r\n", 4);
    if (!hend_p) {
      if (avail > cfg.max_header) {
        bad_request(c, 431, "Request Header Fields Too Large");
        return -1;
      }
      return 0;
    }
    const size_t hlen = (size_t)(static_cast<const char*>(hend_p) - base) + 4;
    // request line
    const char* le = static_cast<const char*>(memmem(base, hlen, "\r\n", 2));
    std::string line(base, (size_t)(le - base));
    const size_t s1 = line.find(' ');
    const size_t s2 = s1 == std::string::npos ? std::string::npos : line.find(' ', s1 + 1);
    if (s1 == std::string::npos || s2 == std::string::npos) {
      bad_request(c, 400, "Bad Request");
      return -1;
    }
    std::string method = line.substr(0, s1), target = line.substr(s1 + 1, s2 - s1 - 1),
                version = line.substr(s2 + 1);
    if (cfg.access_log) c->req_line = line;
    if (version != "HTTP/1.1" && version != "HTTP/1.0") {
      bad_request(c, 400, "Bad Request");
      return -1;
    }
    // headers
    std::vector<std::pair<std::string, std::string>> headers;
    int64_t clen = -1;
    bool chunked = false, expect100 = false, have_ctype = false;
    std::string conn_hdr, ctype;
    const char* hp = le + 2;
    const char* hlim = base + hlen - 2;
    while (hp < hlim) {
      const char* e = static_cast<const char*>(memmem(hp, (size_t)(hlim - hp) + 2, "\r\n", 2));
      if (!e) break;
      const char* colon = static_cast<const char*>(memchr(hp, ':', (size_t)(e - hp)));
      if (!colon) {
        bad_request(c, 400, "Bad Request");
        return -1;
      }
      std::string name(hp, (size_t)(colon - hp)), value(colon + 1, (size_t)(e - colon - 1));
      lower_inplace(name);
      value = trim(value);
      if (name == "content-length") {
        char* endp = nullptr;
        const long long v = strtoll(value.c_str(), &endp, 10);
        if (value.empty() || *endp != '\0' || v < 0 || (clen >= 0 && clen != v)) {
          bad_request(c, 400, "Bad Request");
          return -1;
        }
        clen = v;
      } else if (name == "transfer-encoding") {
        std::string v = value;
        lower_inplace(v);
        if (v.find("chunked") != std::string::npos) chunked = true;
      } else if (name == "connection") {
        std::string v = value;  // every Connection header counts (h11 joins them)
        lower_inplace(v);
        conn_hdr += conn_hdr.empty() ? v : "," + v;
      } else if (name == "content-type") {
        if (!have_ctype) ctype = value;  // the first one: what FastAPI (Starlette headers[...]) reads
        have_ctype = true;
      } else if (name == "expect") {
        std::string v = value;
        lower_inplace(v);
        expect100 = v == "100-continue";
      }
      headers.emplace_back(std::move(name), std::move(value));
      hp = e + 2;
    }
    // body
    std::string body;
    size_t consumed = hlen;
    if (chunked) {
      size_t pos = hlen;
      for (;;) {
        const void* ce = memmem(base + pos, avail - pos, "\r\n", 2);
        if (!ce) {
          if (expect100 && !c->sent_continue) send_continue(c);
          return 0;
        }
        // chunk-size = 1*HEXDIG [ ; ext ]: at most 15 hex digits (no sign, no 0x, no overflow)
        const char* sp = base + pos;
        const char* se = static_cast<const char*>(ce);
        size_t sz = 0;
        int ndig = 0;
        while (sp < se && is_hex(*sp) && ndig < 16) {
          const char h = *sp++;
          sz = (sz << 4) | (size_t)(h <= '9' ? h - '0' : (h | 0x20) - 'a' + 10);
          ++ndig;
        }
        if (ndig == 0 || ndig > 15 || (sp < se && *sp != ';' && *sp != ' ' && *sp != '\t')) {
          bad_request(c, 400, "Bad Request");
          return -1;
        }
        pos = (size_t)(se - base) + 2;
        if (sz == 0) {
          // trailers until empty line
          const void* te = memmem(base + pos, avail - pos, "\r\n", 2);
          if (!te) return 0;
          while (static_cast<const char*>(te) != base + pos) {
            pos = (size_t)(static_cast<const char*>(te) - base) + 2;
            te = memmem(base + pos, avail - pos, "\r\n", 2);
            if (!te) return 0;
          }
          pos += 2;
          break;
        }
        if (sz > cfg.max_body - std::min(body.size(), cfg.max_body)) {  // no overflow: sz < 2^60
          bad_request(c, 413, "Payload Too Large");
          return -1;
        }
        if (avail - pos < sz + 2) {
          if (expect100 && !c->sent_continue) send_continue(c);
          return 0;
        }
        if (base[pos + sz] != '\r' || base[pos + sz + 1] != '\n') {
          bad_request(c, 400, "Bad Request");
          return -1;
        }
        body.append(base + pos, sz);
        pos += sz + 2;
      }
      consumed = pos;
    } else if (clen > 0) {
      if ((size_t)clen > cfg.max_body) {
        bad_request(c, 413, "Payload Too Large");
        return -1;
      }
      if (avail - hlen < (size_t)clen) {
        if (expect100 && !c->sent_continue) send_continue(c);
        return 0;
      }
      body.assign(base + hlen, (size_t)clen);
      consumed = hlen + (size_t)clen;
    }
    c->in_pos += consumed;
    c->sent_continue = false;
    const bool keep_alive = version == "HTTP/1.1" ? conn_hdr.find("close") == std::string::npos
                                                  : conn_hdr.find("keep-alive") != std::string::npos;
    if (!keep_alive) c->close_after = true;

    // ---- fast path
    if (cfg.fast_path && method == "POST") {
      const size_t q = target.find('?');
      const std::string path = q == std::string::npos ? target : target.substr(0, q);
      if (path == cfg.predict_path && json_ctype(ctype) && nfeat_ > 0) {
        // parsed straight into the pending arena; the whole epoll round goes to the engine in
        // one submit_many()
        const size_t at = pend_x_.size();
        pend_x_.resize(at + nfeat_);
        if (body_parser_->parse(body.data(), body.size(), pend_x_.data() + at)) {
          c->waiting = true;
          c->t_req = timing_ ? __rdtsc() : 0;
          pend_tags_.push_back(c->id);
          n_fast.fetch_add(1, std::memory_order_relaxed);
          steer_sample(c);
          return 1;
        }
        pend_x_.resize(at);
      }
    }
    // ---- slow path: hand to the Python ASGI app
    SlowRequest sr;
    sr.token = ((uint64_t)index_ << 56) | c->id;
    sr.method = std::move(method);
    sr.target = std::move(target);
    sr.http_version = version.substr(5);
    sr.headers = std::move(headers);
    sr.body = std::move(body);
    sr.client_host = c->client_host;
    sr.client_port = c->client_port;
    sr.server_host = c->server_host;
    sr.server_port = c->server_port;
    c->waiting = true;
    c->t_req = timing_ ? __rdtsc() : 0;
    n_slow.fetch_add(1, std::memory_order_relaxed);
    srv_->push_slow(std::move(sr));
    return 1;
  }

  static bool json_ctype(const std::string& ct) {
    // FastAPI: maintype 'application' and subtype 'json' or '*+json' (routing.py), params ignored.
    std::string v = ct.substr(0, ct.find(';'));
    v = trim(v);
    lower_inplace(v);
    if (v.compare(0, 12, "application/") != 0) return false;
    const std::string sub = v.substr(12);
    return sub == "json" || (sub.size() > 5 && sub.compare(sub.size() - 5, 5, "+json") == 0);
  }

  void send_continue(Conn* c) {
    c->sent_continue = true;
    static const char kCont[] = "HTTP/1.1 100 Continue\r\n\r\n";
    ssize_t w = send(c->fd, kCont, sizeof(kCont) - 1, MSG_NOSIGNAL);
    (void)w;
  }

  HttpServer* srv_;
  int index_;
  int lfd_;
  int epfd_ = -1, evfd_ = -1;
  size_t nfeat_ = 0;
  std::unique_ptr<PredictBodyParser> body_parser_;  // /predict JSON keys -> feature columns
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> signaled_{false};
  std::atomic<bool> pending_{false};   // completions / slow responses queued for this thread
  std::atomic<bool> spinning_{false};  // inside the busy-poll window (no eventfd needed)
  std::atomic<bool> blocked_{true};    // in (or about to enter) a blocking epoll_wait: hand-offs need the eventfd
  std::mutex mu_;
  std::vector<int> adopted_;  // acceptor mode: connections handed over by the dispatcher
  std::vector<std::unique_ptr<Conn>> moved_in_;  // io_steer: connections handed over by other IO threads
  std::atomic<int> n_open_{0};                   // connections this thread holds (io_steer's balance)
  bool timing_ = false;
  double ns_per_tick_ = 1.0;
  uint64_t st_acc_[SS_COUNT] = {};
  uint64_t st_last_ = 0;
  int st_cur_ = SS_POLL;
  uint64_t lat_hist_[HTTP_LAT_BUCKETS] = {};
  uint64_t lat_sum_ = 0, lat_n_ = 0;
  std::vector<Completion> fast_c_;  // completions handed over by the engine (guarded by mu_) ...
  std::vector<FastSeg> fast_seg_;   // ... in runs of one model each
  std::vector<Completion> spare_c_;  // drain_pending's side of the double buffer (this thread only)
  std::vector<FastSeg> spare_seg_;
  std::vector<Completion> idle_done_;  // run_idle completions (this thread only)
  ServeRing* ring_ = nullptr;          // this thread's resident-kernel ring (engine-owned), or none
  int64_t outstanding_ = 0;            // rows this thread queued in the engine, not yet handed back
  std::vector<Completion> ring_c_;     // harvest_ring scratch (this thread only)
  std::vector<ServeRing::Seg> ring_seg_;
  std::string body_;                   // response body scratch (this thread only)
  std::vector<SlowResp> slow_;
  std::vector<double> pend_x_;      // fast-path rows parsed in this epoll round (IO thread only)
  std::vector<uint64_t> pend_tags_;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns_;
  uint64_t next_id_ = 16;
  std::atomic<bool> listening_{true};
  std::string log_;  // access-log lines of this epoll round
};

// ------------------------------------------------------------------------------------------------
HttpServer::HttpServer(Engine* engine, const ServerConfig& cfg) : engine_(engine), cfg_(cfg) {
  if (cfg_.io_threads < 1) cfg_.io_threads = 1;
  if (cfg_.io_threads > 64) cfg_.io_threads = 64;
  steer_ncpu_ = (int)std::min<long>(4096, std::max<long>(1, sysconf(_SC_NPROCESSORS_CONF)));
  cpu_conns_.reset(new std::atomic<int>[(size_t)steer_ncpu_]);
  plan_.reset(new std::atomic<uint64_t>[(size_t)steer_ncpu_]);
  for (int c = 0; c < steer_ncpu_; ++c) {
    cpu_conns_[c].store(0);
    plan_[c].store(0);
  }
  // io_cpus: each CPU's home IO thread = the one pinned to a CPU of the same physical core (the CPU
  // itself or its SMT sibling, from sysfs); the steering plan prefers it for that CPU's connections
  home_.assign((size_t)steer_ncpu_, -1);
  for (size_t i = 0; i < cfg_.io_cpus.size() && i < (size_t)cfg_.io_threads; ++i) {
    const int cpu = cfg_.io_cpus[i];
    if (cpu < 0 || cpu >= steer_ncpu_) continue;
    std::vector<int> sib{cpu};
    char path[96];
    snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", cpu);
    if (FILE* f = fopen(path, "r")) {
      char buf[128];
      if (fgets(buf, sizeof buf, f)) {
        sib.clear();
        char* save = nullptr;
        for (char* tok = strtok_r(buf, ",\n", &save); tok; tok = strtok_r(nullptr, ",\n", &save)) {
          int a = 0, b = 0;
          const int nf = sscanf(tok, "%d-%d", &a, &b);
          if (nf == 1) b = a;
          for (int c = a; nf >= 1 && c <= b; ++c) sib.push_back(c);
        }
      }
      fclose(f);
    }
    for (int c : sib)
      if (c >= 0 && c < steer_ncpu_ && home_[(size_t)c] < 0) home_[(size_t)c] = (int)i;
  }
}

// io_steer plan: every CPU that drives connections is assigned to its home IO thread (io_cpus: the
// one pinned on the same physical core) or else the least-loaded IO thread, and
// a CPU whose connections exceed that thread's room spills into the next least-loaded ones (at most
// three threads per CPU; water-filling by group size, ties to the lowest index, so equal counts give
// an equal plan). A CPU keeps its previous first thread while that one still has room (a re-plan
// with slightly different counts must not shuffle every group). Encoding per CPU: three owners + 1,
// 8 bits each (0 = none).
void HttpServer::steer_replan(int64_t now_ms) {
  std::unique_lock<std::mutex> lk(plan_mu_, std::try_to_lock);
  if (!lk.owns_lock()) return;
  if (now_ms - plan_ms_.load(std::memory_order_relaxed) < 100) return;
  plan_ms_.store(now_ms, std::memory_order_relaxed);
  const int n = std::min(255, (int)threads_.size());
  std::vector<std::pair<int, int>> groups;  // (count, cpu)
  int total = 0;
  for (int c = 0; c < steer_ncpu_; ++c) {
    const int k = cpu_conns_[c].load(std::memory_order_relaxed);
    if (k > 0) {
      groups.emplace_back(k, c);
      total += k;
    }
  }
  std::sort(groups.begin(), groups.end(), [](const std::pair<int, int>& a, const std::pair<int, int>& b) {
    return a.first != b.first ? a.first > b.first : a.second < b.second;
  });
  const int share = std::max(1, (total + n - 1) / n);
  steer_share_.store(share, std::memory_order_relaxed);
  std::vector<int> load((size_t)n, 0);
  std::vector<uint64_t> prev((size_t)steer_ncpu_);
  for (int c = 0; c < steer_ncpu_; ++c) prev[(size_t)c] = plan_[c].exchange(0, std::memory_order_relaxed);
  for (const auto& g : groups) {
    int left = g.first;
    uint64_t e = 0;
    int used[3] = {-1, -1, -1};
    for (int k = 0; k < 3 && left > 0; ++k) {
      int t = -1;
      // first choice: the CPU's home thread (pinned on its core), then its previous thread
      const int home = home_[(size_t)g.second];
      if (k == 0 && home >= 0 && home < n && load[(size_t)home] < share) t = home;
      const int p1 = (int)(prev[(size_t)g.second] & 0xff) - 1;
      if (t < 0 && k == 0 && p1 >= 0 && p1 < n && load[(size_t)p1] < share) t = p1;
      if (t < 0)
        for (int i = 0; i < n; ++i)
          if (i != used[0] && i != used[1] && (t < 0 || load[(size_t)i] < load[(size_t)t])) t = i;
      const int room = std::max(1, share - load[(size_t)t]);
      const int take = k == 2 ? left : std::min(left, room);
      load[(size_t)t] += take;
      left -= take;
      used[k] = t;
      e |= (uint64_t)(t + 1) << (8 * k);
    }
    plan_[g.second].store(e, std::memory_order_relaxed);
  }
}

int HttpServer::steer_target(int cpu, int self, uint32_t key) {
  (void)key;
  if (cpu < 0 || cpu >= steer_ncpu_) return self;
  const int64_t now = mono_ns() / 1000000;
  if (now < steer_pause_until_ms_.load(std::memory_order_relaxed)) return self;  // churn guard
  if (now - plan_ms_.load(std::memory_order_relaxed) >= 100) steer_replan(now);
  const uint64_t e = plan_[cpu].load(std::memory_order_relaxed);
  const int n = (int)threads_.size();
  int owners[3], no = 0;
  for (int k = 0; k < 3; ++k) {
    const int o = (int)((e >> (8 * k)) & 0xff) - 1;
    if (o >= 0 && o < n) owners[no++] = o;
  }
  if (no == 0) return self;  // not planned yet
  const int share = steer_share_.load(std::memory_order_relaxed);
  for (int k = 0; k < no; ++k)
    if (owners[k] == self) {
      // already on one of its CPU's threads: stays, unless this one is over its share and another
      // of them is under it (the split then evens out)
      if (threads_[(size_t)self]->open_count() > share)
        for (int j = 0; j < no; ++j)
          if (owners[j] != self && threads_[(size_t)owners[j]]->open_count() < share) return owners[j];
      return self;
    }
  // the first of its CPU's threads with room (moves in flight counted by adopt_conn): connections of
  // other CPUs parked there leave for their own threads as those make room
  const int cap = share + 1;
  for (int k = 0; k < no; ++k)
    if (threads_[(size_t)owners[k]]->open_count() < cap) return owners[k];
  return self;
}

void HttpServer::steer_count(int old_cpu, int new_cpu) {
  if (old_cpu >= 0 && old_cpu < steer_ncpu_) cpu_conns_[old_cpu].fetch_sub(1, std::memory_order_relaxed);
  if (new_cpu >= 0 && new_cpu < steer_ncpu_) cpu_conns_[new_cpu].fetch_add(1, std::memory_order_relaxed);
}

void HttpServer::steer_moved() {
  // churn guard: a scheduler that keeps moving client threads between CPUs makes connections chase
  // them; more than 2 moves per open connection in a second pauses steering for 5 s
  const int64_t now = mono_ns() / 1000000;
  int64_t w = steer_win_ms_.load(std::memory_order_relaxed);
  if (now - w >= 1000 && steer_win_ms_.compare_exchange_strong(w, now)) steer_win_moves_.store(0);
  if (steer_win_moves_.fetch_add(1) + 1 > 2 * (int64_t)std::max(8, open_conns.load(std::memory_order_relaxed))) {
    steer_pause_until_ms_.store(now + 5000, std::memory_order_relaxed);
    steer_pauses_.fetch_add(1, std::memory_order_relaxed);
    steer_win_moves_.store(0);
  }
}

HttpServer::~HttpServer() {
  stop();
  for (auto& t : threads_) (void)t;  // IO threads are joined by stop()
}

namespace {
// Completion of a health probe row: a successful batch re-admits the rank.
struct ProbeSink : Sink {
  Engine* eng;
  std::atomic<int> state{0};  // 0 idle, 1 outstanding
  explicit ProbeSink(Engine* e) : eng(e) {}
  void on_complete(const Completion* c, size_t n, const std::shared_ptr<const Model>&) override {
    if (n > 0 && c[0].status == ST_OK) eng->mark_healthy();
    state.store(0);
  }
};
}  // namespace

void HttpServer::health_loop() {
  pthread_setname_np(pthread_self(), "mlapi-health");
  ProbeSink probe(engine_);
  std::vector<double> row;
  while (!health_stop_.load()) {
    const bool ok = engine_->healthy();
    if (accepting_.load() != ok) {
      if (!ok) leaves_.fetch_add(1);
      accepting_.store(ok);
    }
    if (!ok && probe.state.load() == 0) {
      auto m = engine_->model();
      if (m) {
        row.assign((size_t)m->F, 0.0);
        probe.state.store(1);
        if (!engine_->submit(row.data(), m->F, 0, &probe)) probe.state.store(0);
      }
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(std::max(5, cfg_.health_probe_ms)));
  }
  // the engine outlives the server: wait for an outstanding probe so its sink stays valid
  for (int i = 0; i < 2000 && probe.state.load() != 0; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(5));
}

int HttpServer::listeners() const {
  if (acceptor_) return accepting() ? (int)threads_.size() : 0;
  int n = 0;
  for (const auto& t : threads_) n += t->listening() ? 1 : 0;
  return n;
}

void HttpServer::start() {
  if (started_) return;
  (void)tsc_ns_per_tick();  // calibrate the stage clock before any IO thread needs it
  if (cfg_.dispatch == "acceptor" || cfg_.dispatch == "source") {
    acceptor_ = true;
    for (int i = 0; i < cfg_.io_threads; ++i) threads_.push_back(std::make_unique<IoThread>(this, i, -1));
    for (auto& t : threads_) t->start();
    dispatcher_ = std::make_unique<ConnDispatcher>(
        cfg_.dispatch_group, cfg_.host, cfg_.port, cfg_.backlog, cfg_.dispatch_rank,
        [this](int fd) { threads_[adopt_rr_.fetch_add(1, std::memory_order_relaxed) % threads_.size()]->adopt(fd); },
        [this] { return accepting(); }, cfg_.dispatch == "source", cfg_.dispatch_claim);
    try {
      dispatcher_->start();
    } catch (...) {
      for (auto& t : threads_) t->stop();
      threads_.clear();
      dispatcher_.reset();
      throw;
    }
    bound_port_ = dispatcher_->port();
    if (cfg_.health_dispatch) health_ = std::thread([this] { health_loop(); });
    started_ = true;
    return;
  }
  if (cfg_.dispatch != "reuseport") throw std::invalid_argument("dispatch must be acceptor, source or reuseport");
  int port = cfg_.port;
  std::vector<int> fds;
  try {
    for (int i = 0; i < cfg_.io_threads; ++i) {
      int bp = 0;
      fds.push_back(make_listener(cfg_.host, port, cfg_.reuseport || cfg_.io_threads > 1, cfg_.backlog, &bp));
      if (i == 0) {
        bound_port_ = bp;
        port = bp;
      }
    }
  } catch (...) {
    for (int fd : fds) close(fd);
    throw;
  }
  for (int i = 0; i < cfg_.io_threads; ++i) threads_.push_back(std::make_unique<IoThread>(this, i, fds[i]));
  for (auto& t : threads_) t->start();
  if (cfg_.health_dispatch) health_ = std::thread([this] { health_loop(); });
  started_ = true;
}

void HttpServer::stop() {
  {
    std::lock_guard<std::mutex> lk(slow_mu_);
    if (stopping_) return;
    stopping_ = true;
  }
  slow_cv_.notify_all();
  health_stop_.store(true);
  if (health_.joinable()) health_.join();
  if (dispatcher_) dispatcher_->stop();  // no new connections while the IO threads wind down
  for (auto& t : threads_) t->stop();
  threads_.clear();
}

void HttpServer::push_slow(SlowRequest&& r) {
  {
    std::lock_guard<std::mutex> lk(slow_mu_);
    slow_q_.push_back(std::move(r));
  }
  slow_cv_.notify_one();
}

bool HttpServer::next_slow(SlowRequest* out, int timeout_ms) {
  std::unique_lock<std::mutex> lk(slow_mu_);
  if (!slow_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return stopping_ || !slow_q_.empty(); }))
    return false;
  if (slow_q_.empty()) return false;
  *out = std::move(slow_q_.front());
  slow_q_.pop_front();
  return true;
}

void HttpServer::respond(uint64_t token, int status, const std::string& reason,
                         const std::vector<std::pair<std::string, std::string>>& headers, const std::string& body,
                         bool close) {
  const int ti = (int)(token >> 56);
  const uint64_t cid = token & ((uint64_t(1) << 56) - 1);
  if (ti < 0 || ti >= (int)threads_.size()) return;
  std::string o;
  o.reserve(256 + body.size());
  o += "HTTP/1.1 ";
  o += std::to_string(status);
  o += ' ';
  o += reason;
  o += "\r\ndate: ";
  o += http_date_now();
  o += "\r\nserver: ";
  o += cfg_.server_header;
  bool has_len = false;
  for (const auto& h : headers) {
    if (h.first == "content-length") has_len = true;
    o += "\r\n";
    o += h.first;
    o += ": ";
    o += h.second;
  }
  if (!has_len) {
    o += "\r\ncontent-length: ";
    o += std::to_string(body.size());
  }
  if (close) o += "\r\nconnection: close";
  o += "\r\n\r\n";
  o += body;
  threads_[ti]->post_slow(cid, std::move(o), close);
}

ServerStats HttpServer::stats() const {
  ServerStats s;
  for (const auto& t : threads_) {
    s.fast += t->n_fast.load();
    s.slow += t->n_slow.load();
    s.responses += t->n_resp.load();
    s.connections += t->n_conn.load();
    s.errors += t->n_err.load();
    s.bad_requests += t->n_bad.load();
    s.listen_closes += t->n_listen_close.load();
    s.steered += t->n_steered.load();
    s.conns_per_thread.push_back(t->open_count());
  }
  s.steer_pauses = steer_pauses_.load();
  for (int c = 0; c < steer_ncpu_; ++c) {
    const int k = cpu_conns_[c].load(std::memory_order_relaxed);
    const uint64_t e = plan_[c].load(std::memory_order_relaxed);
    if (k != 0 || e != 0)
      s.steer_plan.push_back({c, k, (int)(e & 0xff) - 1, (int)((e >> 8) & 0xff) - 1, (int)((e >> 16) & 0xff) - 1});
  }
  s.listen_closes += leaves_.load();
  s.accepting = accepting_.load();
  const double k = tsc_ns_per_tick();
  for (const auto& t : threads_) {
    for (int i = 0; i < SS_COUNT; ++i) s.stage_ns[i] += (uint64_t)((double)t->pub_stage[i].load() * k);
    for (int i = 0; i < HTTP_LAT_BUCKETS; ++i) s.http_latency_hist[i] += t->pub_lat[i].load();
    s.http_latency_sum_ns += (uint64_t)((double)t->pub_lat_sum.load() * k);
    s.http_latency_count += t->pub_lat_n.load();
  }
  return s;
}

}  // namespace mlapi
