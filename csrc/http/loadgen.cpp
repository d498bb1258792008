// Closed-loop HTTP/1.1 load generator (no wrk/ab/hey in the image; a single aiohttp
// client caps at ~7.4k req/s, far below what the native server sustains).
//
// `threads` epoll loops share `conns` keep-alive connections; every connection cycles through the
// workload's requests, waits for the complete response (status line + content-length body),
// checks the body byte for byte against the expected one (a wrong label or probability at HTTP
// 200 is a failure, not throughput), records the latency, and immediately sends the next one
// until it has completed `n` requests. One send() per request, TCP_NODELAY, so the client itself
// never introduces Nagle stalls.
#include "loadgen.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cmath>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <numeric>
#include <random>

namespace mlapi {

namespace {
int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

struct LgConn {
  int fd = -1;
  std::string in;
  size_t sent = 0;
  size_t next = 0;  // workload entry of the outstanding request
  int64_t t_send = 0;
  int64_t remaining = 0;
  bool active = false;
};

Loadgen::Loadgen(const std::string& host, int port, const std::string& request, int conns, int threads,
                 double timeout_s, const std::string& source)
    : host_(host), port_(port), requests_{request}, timeout_s_(timeout_s) {
  if (conns < 1) conns = 1;
  if (threads < 1) threads = 1;
  if (threads > conns) threads = conns;
  threads_ = threads;
  conns_.resize(conns);
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) != 0 || !res) throw std::runtime_error("loadgen: resolve");
  for (auto& c : conns_) {
    c = std::make_unique<LgConn>();
    c->fd = socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, IPPROTO_TCP);
    if (c->fd >= 0 && !source.empty()) {
      sockaddr_in src{};
      src.sin_family = AF_INET;
      src.sin_port = 0;
      if (res->ai_family != AF_INET || inet_pton(AF_INET, source.c_str(), &src.sin_addr) != 1 ||
          bind(c->fd, reinterpret_cast<sockaddr*>(&src), sizeof src) != 0) {
        const int e = errno;
        freeaddrinfo(res);
        throw std::runtime_error("loadgen: bind to source " + source + " failed: " + strerror(e));
      }
    }
    if (c->fd < 0 || connect(c->fd, res->ai_addr, res->ai_addrlen) != 0) {
      const int e = errno;
      freeaddrinfo(res);
      throw std::runtime_error(std::string("loadgen: connect failed: ") + strerror(e));
    }
    int one = 1;
    setsockopt(c->fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  }
  freeaddrinfo(res);
  order_.resize(conns);
  std::iota(order_.begin(), order_.end(), 0);
}

Loadgen::~Loadgen() { close_all(); }

void Loadgen::set_thread_cpus(const std::vector<int>& cpus) {
  for (int c : cpus)
    if (c < 0 || c >= CPU_SETSIZE) throw std::invalid_argument("loadgen: bad CPU in the thread list");
  thread_cpus_ = cpus;
}

void Loadgen::set_conn_map(const std::string& mode, uint64_t seed) {
  std::iota(order_.begin(), order_.end(), 0);
  if (mode == "shuffle") {
    std::mt19937_64 rng(seed);
    std::shuffle(order_.begin(), order_.end(), rng);
  } else if (mode != "rr") {
    throw std::invalid_argument("loadgen: conn map must be rr or shuffle");
  }
}

void Loadgen::set_workload(const std::vector<std::string>& requests, const std::vector<std::string>& expected,
                           double rel_tol) {
  rel_tol_ = rel_tol;
  if (requests.empty()) throw std::invalid_argument("loadgen: empty workload");
  if (!expected.empty() && expected.size() != requests.size())
    throw std::invalid_argument("loadgen: one expected body per request");
  requests_ = requests;
  expected_ = expected;
}

void Loadgen::close_all() {
  for (auto& c : conns_)
    if (c && c->fd >= 0) {
      close(c->fd);
      c->fd = -1;
    }
}

// Parses one complete response at the front of `in`. Returns bytes consumed (0 if incomplete),
// -1 on protocol error. *status receives the HTTP status code.
// Body check: exact bytes, or (rel_tol > 0) exact up to the last ':' and the trailing number
// (up to the closing brace) within rel_tol.
static bool body_matches(const char* b, size_t n, const std::string& ex, double rel_tol) {
  if (rel_tol <= 0) return n == ex.size() && memcmp(b, ex.data(), n) == 0;
  const size_t ce = ex.rfind(':');
  if (ce == std::string::npos || n <= ce || memcmp(b, ex.data(), ce + 1) != 0) return false;
  const std::string got(b + ce + 1, n - ce - 1), want = ex.substr(ce + 1);
  char* e1 = nullptr;
  char* e2 = nullptr;
  const double x = strtod(got.c_str(), &e1), y = strtod(want.c_str(), &e2);
  if (e1 == got.c_str() || e2 == want.c_str() || std::strcmp(e1, e2) != 0) return false;
  return std::fabs(x - y) <= rel_tol * std::fabs(y);
}

static int64_t parse_response(const std::string& in, int* status, size_t* body_off) {
  const size_t he = in.find("\r\n\r\n");
  if (he == std::string::npos) return 0;
  if (in.size() < 12 || in.compare(0, 5, "HTTP/") != 0) return -1;
  *status = atoi(in.c_str() + 9);
  int64_t clen = 0;
  size_t pos = in.find("\r\n") + 2;
  while (pos < he) {
    const size_t e = in.find("\r\n", pos);
    if (e - pos > 15 && strncasecmp(in.c_str() + pos, "content-length:", 15) == 0) clen = atoll(in.c_str() + pos + 15);
    pos = e + 2;
  }
  const int64_t total = (int64_t)he + 4 + clen;
  if ((int64_t)in.size() < total) return 0;
  *body_off = he + 4;
  return total;
}

LoadgenResult Loadgen::run(int64_t requests_per_conn, bool record) {
  LoadgenResult R;
  const int nc = (int)conns_.size();
  std::vector<std::vector<int64_t>> lats(threads_);
  std::vector<std::vector<uint64_t>> statuses(threads_, std::vector<uint64_t>(600, 0));
  std::vector<uint64_t> errs(threads_, 0), mism(threads_, 0);
  std::atomic<int> failed{0};
  const int64_t t0 = mono_ns();
  auto worker = [&](int ti) {
    pthread_setname_np(pthread_self(), "mlapi-loadgen");
    if (!thread_cpus_.empty()) {
      // this client thread on its own CPU (like a NIC whose RX queues' interrupts are pinned: every
      // connection's segments then arrive from one stable CPU)
      cpu_set_t one;
      CPU_ZERO(&one);
      CPU_SET(thread_cpus_[(size_t)ti % thread_cpus_.size()], &one);
      pthread_setaffinity_np(pthread_self(), sizeof one, &one);
    }
    const int ep = epoll_create1(EPOLL_CLOEXEC);
    std::vector<LgConn*> mine;
    for (int i = ti; i < nc; i += threads_) mine.push_back(conns_[order_[i]].get());
    if (record) lats[ti].reserve((size_t)(requests_per_conn * (int64_t)mine.size()));
    int live = 0;
    const size_t nw = requests_.size();
    auto send_req = [&](LgConn* c) -> bool {
      c->t_send = mono_ns();
      const std::string& rq = requests_[c->next];
      size_t off = 0;
      while (off < rq.size()) {
        const ssize_t w = send(c->fd, rq.data() + off, rq.size() - off, MSG_NOSIGNAL);
        if (w <= 0) {
          if (w < 0 && errno == EINTR) continue;
          return false;
        }
        off += (size_t)w;
      }
      return true;
    };
    for (size_t k = 0; k < mine.size(); ++k) {
      LgConn* c = mine[k];
      c->remaining = requests_per_conn;
      c->in.clear();
      c->next = (size_t)(ti + k * threads_) % nw;  // = connection index mod workload size
      if (c->remaining <= 0) continue;
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.u64 = k;
      epoll_ctl(ep, EPOLL_CTL_ADD, c->fd, &ev);
      c->active = true;
      ++live;
      if (!send_req(c)) {
        failed.store(1);
        break;
      }
    }
    epoll_event evs[256];
    char buf[65536];
    int64_t last_progress = mono_ns();
    while (live > 0 && !failed.load()) {
      // spin_us: poll (timeout 0) for this long after the last response before sleeping in
      // epoll_wait - a closed-loop client whose responses arrive every few us then never pays a
      // sleep / wake-up per response (and the server's send() never has to wake it)
      const int n = epoll_wait(ep, evs, 256, spin_ns_ > 0 && mono_ns() - last_progress < spin_ns_ ? 0 : 1000);
      if (n > 0) last_progress = mono_ns();
      if (n == 0 && mono_ns() - last_progress > (int64_t)timeout_s_ * 1000000000LL) {
        failed.store(2);  // no progress for timeout_s: give up
        break;
      }
      for (int i = 0; i < n; ++i) {
        LgConn* c = mine[evs[i].data.u64];
        const ssize_t r = recv(c->fd, buf, sizeof buf, 0);
        if (r <= 0) {
          if (r < 0 && (errno == EAGAIN || errno == EINTR)) continue;
          errs[ti]++;
          failed.store(3);
          break;
        }
        c->in.append(buf, (size_t)r);
        for (;;) {
          int st = 0;
          size_t boff = 0;
          const int64_t used = parse_response(c->in, &st, &boff);
          if (used == 0) break;
          if (used < 0) {
            failed.store(4);
            break;
          }
          const int64_t now = mono_ns();
          if (st == 200 && !expected_.empty()) {
            const std::string& ex = expected_[c->next];
            if (!body_matches(c->in.data() + boff, (size_t)used - boff, ex, rel_tol_)) {
              mism[ti]++;
              errs[ti]++;
            }
          }
          c->in.erase(0, (size_t)used);
          c->next = c->next + 1 == nw ? 0 : c->next + 1;
          if (st >= 0 && st < 600) statuses[ti][st]++;
          if (st != 200) errs[ti]++;
          if (record) lats[ti].push_back(now - c->t_send);
          if (--c->remaining > 0) {
            if (!send_req(c)) {
              failed.store(5);
              break;
            }
          } else {
            epoll_ctl(ep, EPOLL_CTL_DEL, c->fd, nullptr);
            c->active = false;
            --live;
          }
        }
      }
    }
    close(ep);
  };
  std::vector<std::thread> ths;
  for (int t = 0; t < threads_; ++t) ths.emplace_back(worker, t);
  for (auto& t : ths) t.join();
  R.elapsed_s = (double)(mono_ns() - t0) * 1e-9;
  R.failed = failed.load();
  for (int t = 0; t < threads_; ++t) {
    R.errors += errs[t];
    R.body_mismatches += mism[t];
    R.latencies_ns.insert(R.latencies_ns.end(), lats[t].begin(), lats[t].end());
    for (int s = 0; s < 600; ++s) R.status_counts[s] += statuses[t][s];
  }
  R.completed = 0;
  for (int s = 0; s < 600; ++s) R.completed += R.status_counts[s];
  return R;
}

}  // namespace mlapi
