// Host-side stress test of the native runtime under AddressSanitizer/UBSan or ThreadSanitizer
// ("host C++ built with -fsanitize=address,undefined in a debug target; TSAN-style
// stress tests of the batcher"). Runs on the CPU backend (device = -1), so it needs no GPU:
//
//   0. resident rings: an injected hang (rows given up after 10 x watchdog, no busy loop after),
//      a ring closed with rows pending and handed to its next owner, restarts by the watchdogs;
//   1. engine: 8 submitter threads x random batch sizes, results checked against the float64
//      oracle, while another thread hot-swaps the model (version-tagged results must match the
//      model they were computed with), polls stats() and unloads/reloads;
//   2. HTTP: the epoll server + native load generator over loopback (keep-alive, 32 connections,
//      4+4 threads) with a slow-path consumer thread answering everything the fast path rejects;
//      raw sockets send pipelined, chunked, malformed and half-closed requests meanwhile.
//
// Built and run by tools/sanitize.sh (hipcc -Xarch_host -fsanitize=...); exits non-zero on any
// mismatch; the sanitizers abort on memory errors / data races.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "http/loadgen.h"
#include "http/server.h"
#include "http/dispatch.h"
#include "runtime/engine.h"

using namespace mlapi;

namespace {

std::atomic<int> g_fail{0};
#define CHECK(cond, ...)                                      \
  do {                                                        \
    if (!(cond)) {                                            \
      std::fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                      \
      std::fprintf(stderr, "\n");                             \
      g_fail.fetch_add(1);                                    \
    }                                                         \
  } while (0)

struct ModelSpec {
  int kind, F, K;
  std::vector<double> W, b;
};

ModelSpec make_model(uint64_t seed, int kind) {
  std::mt19937_64 rng(seed);
  std::normal_distribution<double> nd;
  ModelSpec m{kind, 4, kind == KIND_BINARY ? 1 : 3, {}, {}};
  m.W.resize((size_t)m.K * m.F);
  m.b.resize(m.K);
  for (auto& v : m.W) v = nd(rng);
  for (auto& v : m.b) v = nd(rng);
  return m;
}

// Checks every completion against the model version it reports.
class CheckingSink : public Sink {
 public:
  explicit CheckingSink(std::map<uint64_t, std::vector<double>>* rows) : rows_(rows) {}
  void on_complete(const Completion* c, size_t n, const std::shared_ptr<const Model>& m) override {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < n; ++i) {
      ++done;
      if (c[i].status == ST_NO_MODEL) {
        ++no_model;
        continue;
      }
      CHECK(c[i].status == ST_OK, "status %d", c[i].status);
      if (!m) continue;
      auto it = rows_->find(c[i].tag);
      CHECK(it != rows_->end(), "unknown tag");
      if (it == rows_->end()) continue;
      int32_t idx;
      double p;
      cpu_linear_predict(*m, it->second.data(), 1, &idx, &p);
      CHECK(idx == c[i].idx && p == c[i].p, "tag %llu: got (%d, %.17g) want (%d, %.17g) v%llu",
            (unsigned long long)c[i].tag, c[i].idx, c[i].p, idx, p, (unsigned long long)m->version);
    }
  }
  std::mutex mu_;
  uint64_t done = 0, no_model = 0;

 private:
  std::map<uint64_t, std::vector<double>>* rows_;
};

void engine_stress() {
  EngineConfig cfg;
  cfg.device = -1;
  cfg.max_batch = 64;
  cfg.batchers = 2;  // two batcher threads draining one queue
  Engine eng(cfg);
  auto m0 = make_model(1, KIND_MULTINOMIAL);
  eng.load_model(m0.kind, m0.F, m0.K, m0.W.data(), m0.b.data(), {"\"a\"", "\"b\"", "\"c\""});

  constexpr int kThreads = 8, kPerThread = 4000;
  std::vector<std::map<uint64_t, std::vector<double>>> rows(kThreads);
  std::vector<std::unique_ptr<CheckingSink>> sinks;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd;
  for (int t = 0; t < kThreads; ++t) {
    for (int i = 0; i < kPerThread; ++i) {
      std::vector<double> x(4);
      for (auto& v : x) v = nd(rng);
      rows[t][(uint64_t)t << 32 | (uint64_t)i] = x;
    }
    sinks.emplace_back(new CheckingSink(&rows[t]));
  }
  std::atomic<bool> done{false};
  std::thread swapper([&] {  // hot reload + unload while requests fly
    uint64_t s = 100;
    while (!done.load()) {
      ++s;
      auto m = make_model(s, (s % 3 == 0) ? KIND_OVR : KIND_MULTINOMIAL);
      eng.load_model(m.kind, m.F, m.K, m.W.data(), m.b.data(), {"1", "2", "3"});
      if (s % 17 == 0) eng.unload_model();
      (void)eng.stats();
      std::this_thread::sleep_for(std::chrono::microseconds(300));
    }
  });
  std::vector<std::thread> subs;
  for (int t = 0; t < kThreads; ++t) {
    subs.emplace_back([&, t] {
      std::mt19937 r(t);
      std::vector<uint64_t> tags;
      std::vector<double> X;
      int i = 0;
      while (i < kPerThread) {
        const int n = std::min(kPerThread - i, 1 + (int)(r() % 40));
        tags.clear();
        X.clear();
        for (int j = 0; j < n; ++j, ++i) {
          const uint64_t tag = (uint64_t)t << 32 | (uint64_t)i;
          tags.push_back(tag);
          const auto& x = rows[t][tag];
          X.insert(X.end(), x.begin(), x.end());
        }
        CHECK(eng.submit_many(X.data(), n, 4, tags.data(), sinks[t].get()) == n, "submit_many");
      }
    });
  }
  for (auto& th : subs) th.join();
  for (int spin = 0; spin < 20000; ++spin) {
    uint64_t total = 0;
    for (auto& s : sinks) {
      std::lock_guard<std::mutex> lk(s->mu_);
      total += s->done;
    }
    if (total == (uint64_t)kThreads * kPerThread) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  done = true;
  swapper.join();
  uint64_t total = 0, nm = 0;
  for (auto& s : sinks) {
    std::lock_guard<std::mutex> lk(s->mu_);
    total += s->done;
    nm += s->no_model;
  }
  CHECK(total == (uint64_t)kThreads * kPerThread, "completed %llu", (unsigned long long)total);
  eng.stop();
  std::printf("engine stress: %llu completions (%llu during unload windows)\n", (unsigned long long)total,
              (unsigned long long)nm);
}

int connect_to(int port) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
    close(fd);
    return -1;
  }
  return fd;
}

std::string read_some(int fd, size_t want_responses) {
  std::string got;
  char buf[4096];
  timeval tv{2, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  size_t seen = 0;
  while (seen < want_responses) {
    const ssize_t r = recv(fd, buf, sizeof buf, 0);
    if (r <= 0) break;
    got.append(buf, (size_t)r);
    seen = 0;
    for (size_t p = got.find("HTTP/1.1 "); p != std::string::npos; p = got.find("HTTP/1.1 ", p + 1)) ++seen;
  }
  return got;
}

void http_stress() {
  EngineConfig ecfg;
  ecfg.device = -1;
  Engine eng(ecfg);
  auto m = make_model(3, KIND_MULTINOMIAL);
  eng.load_model(m.kind, m.F, m.K, m.W.data(), m.b.data(), {"\"x\"", "\"y\"", "\"z\""});
  ServerConfig scfg;
  scfg.port = 0;
  scfg.io_threads = 4;
  scfg.feature_names = {"sepal_length", "sepal_width", "petal_length", "petal_width"};
  HttpServer srv(&eng, scfg);
  srv.start();
  // a second replica joins srv's dispatch group (same port): the leader deals connections to both
  // over the SCM_RIGHTS channel while the load below runs
  ServerConfig mcfg = scfg;
  mcfg.port = srv.port();
  mcfg.dispatch_rank = 1;
  mcfg.io_threads = 2;
  HttpServer member(&eng, mcfg);
  member.start();
  CHECK(srv.dispatcher() && srv.dispatcher()->leader() && member.dispatcher() && !member.dispatcher()->leader(),
        "dispatch roles");
  for (int i = 0; i < 500 && srv.dispatcher()->targets().size() < 2; ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  std::atomic<bool> stop{false};
  std::atomic<int> slow_seen{0};
  std::thread slow([&] {  // stands in for the Python ASGI app
    SlowRequest r;
    while (!stop.load()) {
      for (HttpServer* h : {&srv, &member}) {  // each replica has its own slow-path queue
        if (!h->next_slow(&r, 10)) continue;
        slow_seen.fetch_add(1);
        h->respond(r.token, 422, "Unprocessable Entity", {{"content-type", "application/json"}}, "{\"detail\":[]}",
                   false);
      }
    }
  });
  const std::string body = "{\"sepal_length\":5.1,\"sepal_width\":3.5,\"petal_length\":1.4,\"petal_width\":0.2}";
  const std::string req = "POST /predict HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nContent-Length: " +
                          std::to_string(body.size()) + "\r\n\r\n" + body;
  std::thread raw([&] {  // odd clients alongside the load
    for (int round = 0; round < 50 && !stop.load(); ++round) {
      int fd = connect_to(srv.port());
      if (fd < 0) continue;
      std::string pip = req + req + req;  // pipelined
      send(fd, pip.data(), pip.size(), MSG_NOSIGNAL);
      std::string got = read_some(fd, 3);
      CHECK(got.find("HTTP/1.1 200") != std::string::npos, "pipelined: %s", got.substr(0, 80).c_str());
      const std::string chunked =
          "POST /predict HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n" +
          [&] {
            char h[16];
            std::snprintf(h, sizeof h, "%zx\r\n", body.size());
            return std::string(h);
          }() + body + "\r\n0\r\n\r\n";
      send(fd, chunked.data(), chunked.size(), MSG_NOSIGNAL);
      got = read_some(fd, 1);
      CHECK(got.find("HTTP/1.1 ") != std::string::npos, "chunked: no response");
      const std::string bad = "POST /predict HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                              "Content-Length: 9\r\n\r\n{\"a\": 1}x";
      send(fd, bad.data(), bad.size(), MSG_NOSIGNAL);  // strict parser rejects -> slow path
      got = read_some(fd, 1);
      CHECK(got.find("HTTP/1.1 422") != std::string::npos, "slow path: %s", got.substr(0, 80).c_str());
      const std::string half = req.substr(0, req.size() / 2);
      send(fd, half.data(), half.size(), MSG_NOSIGNAL);  // then vanish mid-request
      close(fd);
      fd = connect_to(srv.port());
      if (fd >= 0) {
        const std::string junk = "GARBAGE\r\n\r\n";
        send(fd, junk.data(), junk.size(), MSG_NOSIGNAL);
        got = read_some(fd, 1);
        CHECK(got.find("HTTP/1.1 400") != std::string::npos, "garbage: %s", got.substr(0, 80).c_str());
        close(fd);
      }
    }
  });
  {
    Loadgen lg("127.0.0.1", srv.port(), req, 32, 4, 20.0);
    LoadgenResult res = lg.run(300, true);
    CHECK(res.failed == 0 && res.status_counts[200] == 32u * 300u, "loadgen: failed=%d ok=%llu", res.failed,
          (unsigned long long)res.status_counts[200]);
    // reload during load
    std::thread reloader([&] {
      for (int i = 0; i < 20; ++i) {
        auto mm = make_model(50 + i, KIND_MULTINOMIAL);
        eng.load_model(mm.kind, mm.F, mm.K, mm.W.data(), mm.b.data(), {"\"x\"", "\"y\"", "\"z\""});
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
    });
    LoadgenResult res2 = lg.run(300, false);
    reloader.join();
    CHECK(res2.failed == 0 && res2.status_counts[200] == 32u * 300u, "loadgen under reload: failed=%d",
          res2.failed);
    lg.close_all();
    std::printf("http stress: %llu + %llu responses\n", (unsigned long long)res.completed,
                (unsigned long long)res2.completed);
  }
  raw.join();
  stop = true;
  slow.join();
  CHECK(slow_seen.load() > 0, "slow path never used");
  const auto tg = srv.dispatcher()->targets();
  CHECK(tg.size() == 2 && tg[1].conns > 0 && (tg[0].conns > tg[1].conns ? tg[0].conns - tg[1].conns
                                                                        : tg[1].conns - tg[0].conns) <= 1,
        "round robin: %llu vs %llu", (unsigned long long)tg[0].conns,
        (unsigned long long)(tg.size() > 1 ? tg[1].conns : 0));
  member.stop();
  srv.stop();
  eng.stop();
}

}  // namespace

// The resident rings' failure paths on the CPU backend (the supervisor thread plays the kernel):
// a sticky injected hang makes rows give up after 10 x watchdog (a 500, never a hang, and no busy
// IO loop afterwards: pending() drops to 0); a ring closed with rows pending hands its next owner
// none of the old rows' answers; after the hang clears, the reopened ring serves correct answers.
void ring_stress() {
  EngineConfig cfg;
  cfg.device = -1;
  cfg.resident = 1;
  cfg.watchdog_ms = 300;  // rows give up after 3 s: past close_ring's 2 s wait
  Engine eng(cfg);
  auto m0 = make_model(3, KIND_MULTINOMIAL);
  eng.load_model(m0.kind, m0.F, m0.K, m0.W.data(), m0.b.data(), {"\"a\"", "\"b\"", "\"c\""});
  ServeRing* ring = eng.open_ring();
  CHECK(ring != nullptr, "no ring");
  if (ring == nullptr) return;
  std::vector<Completion> out;
  std::vector<ServeRing::Seg> segs;
  int rq = 0;
  const double x[8] = {5.1, 3.5, 1.4, 0.2, 6.7, 3.0, 5.2, 2.3};
  auto submit = [&](uint64_t tag0, int n) {  // retried while an instance (re)starts
    const uint64_t tags[2] = {tag0, tag0 + 1};
    for (int i = 0; i < 4000; ++i) {
      if (ring->submit(x, n, 4, tags)) return true;
      std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
    return false;
  };
  auto drain = [&](int want, int ms) {
    out.clear();
    segs.clear();
    const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(ms);
    while ((int)out.size() < want && std::chrono::steady_clock::now() < until) {
      ring->poll(out, segs, nullptr, &rq);
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  };
  auto check_answers = [&](uint64_t tag0) {
    for (const Completion& c : out) {
      int32_t idx;
      double p;
      cpu_linear_predict(*eng.model(), x + 4 * (c.tag - tag0), 1, &idx, &p);
      CHECK(c.status == ST_OK && c.idx == idx && c.p == p, "ring answer tag %llu", (unsigned long long)c.tag);
    }
  };
  CHECK(submit(10, 2), "submit (healthy)");
  drain(2, 2000);
  CHECK(out.size() == 2, "healthy ring answered %zu of 2", out.size());
  check_answers(10);
  // sticky hang: the rows give up after 10 x watchdog as device errors; nothing stays pending
  CHECK(eng.resident_inject(Engine::RES_INJECT_STALL_STICKY, 0), "inject");
  std::this_thread::sleep_for(std::chrono::milliseconds(20));  // the poller has seen the hang
  CHECK(submit(20, 2), "submit (stalled)");
  drain(2, 6000);
  CHECK(out.size() == 2 && out[0].status == ST_DEVICE_ERROR && out[1].status == ST_DEVICE_ERROR,
        "given-up rows: %zu completions (status %d, %d)", out.size(), out.empty() ? -1 : (int)out[0].status,
        out.size() < 2 ? -1 : (int)out[1].status);
  CHECK(ring->pending() == 0, "pending after give-up: %d", ring->pending());
  // close with rows pending (still hung): the next owner sees none of them
  CHECK(submit(30, 2), "submit (before close)");
  eng.close_ring(ring);  // waits 2 s, then abandons them
  CHECK(!eng.healthy(), "closing a ring with rows unanswered marks the engine unhealthy");
  CHECK(eng.resident_inject(RES_FAULT_NONE, 0), "clear");
  std::this_thread::sleep_for(std::chrono::milliseconds(50));  // the old rows' records land now
  ServeRing* again = eng.open_ring();
  CHECK(again == ring, "the pooled ring comes back");
  ring = again;
  out.clear();
  segs.clear();
  ring->poll(out, segs, nullptr, &rq);
  CHECK(out.empty() && ring->pending() == 0, "reopened ring rendered %zu old answers", out.size());
  CHECK(submit(40, 2), "submit (reopened)");
  drain(2, 2000);
  CHECK(out.size() == 2 && out[0].tag == 40 && out[1].tag == 41, "reopened ring answered %zu", out.size());
  check_answers(40);
  const EngineStats s = eng.stats();
  CHECK(s.resident_hb_restarts + s.resident_ring_restarts >= 1, "no watchdog restart counted");
  eng.close_ring(ring);
  eng.stop();
  std::printf("ring stress: give-up, close-with-pending and reopen OK (%llu restarts)\n",
              (unsigned long long)(s.resident_hb_restarts + s.resident_ring_restarts));
}

int main() {
  ring_stress();
  engine_stress();
  http_stress();
  if (g_fail.load() != 0) {
    std::fprintf(stderr, "%d checks failed\n", g_fail.load());
    return 1;
  }
  std::printf("stress OK\n");
  return 0;
}
