#pragma once
#include <cstdlib>
#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace mlapi {

struct LoadgenResult {
  double elapsed_s = 0;
  uint64_t completed = 0, errors = 0;
  uint64_t body_mismatches = 0;  // 200 responses whose body differs from the expected bytes
  int failed = 0;  // nonzero: connection error / timeout code
  std::vector<int64_t> latencies_ns;
  uint64_t status_counts[600] = {0};
};

struct LgConn;

class Loadgen {
 public:
  // Opens `conns` keep-alive connections (distributed over `threads` epoll loops: connection c on
  // loop c % threads), one after the other, from local address `source` when it is not empty (an
  // IPv4 literal: on loopback every 127.x.y.z works, so several load generators on one host look
  // like several client hosts to a source-affinity dispatcher).
  Loadgen(const std::string& host, int port, const std::string& request, int conns, int threads,
          double timeout_s = 30.0, const std::string& source = "");
  ~Loadgen();
  // Distinct requests cycled per connection (connection c starts at entry c % n), each with the
  // exact response body it must produce; empty `expected` = status-only checking.
  // `rel_tol` > 0: the text after the body's last ':' (the probability) is compared as a number
  // within rel_tol, the bytes before it exactly (batch-size-dependent reduction orders of the
  // bf16 GEMM path change the last bits); 0 = the whole body byte for byte.
  void set_workload(const std::vector<std::string>& requests, const std::vector<std::string>& expected,
                    double rel_tol = 0.0);
  // Which epoll loop drives which connection: "rr" (default) = connection c on loop c % threads,
  // i.e. in connect order; "shuffle" = a seeded random permutation of the connections dealt round
  // robin - a client thread's connections then land wherever the server's dispatcher put them, as
  // independent clients' would (not paired with the server's IO threads by connect order).
  void set_conn_map(const std::string& mode, uint64_t seed = 1);
  // Thread i of the next run() pins itself to cpus[i % size] (empty: threads keep the process mask).
  void set_thread_cpus(const std::vector<int>& cpus);
  // Every connection completes `requests_per_conn` closed-loop requests.
  LoadgenResult run(int64_t requests_per_conn, bool record = true);
  void close_all();

 private:
  std::string host_;
  int port_;
  std::vector<std::string> requests_;
  std::vector<std::string> expected_;
  double rel_tol_ = 0.0;
  double timeout_s_ = 30.0;
  // MLAPI_LOADGEN_SPIN_US (default 0): each thread polls its sockets this long after its last
  // response before it sleeps in epoll_wait (no sleep / wake-up per response in a closed loop)
  int64_t spin_ns_ = [] {
    const char* e = std::getenv("MLAPI_LOADGEN_SPIN_US");
    return e ? (int64_t)std::atoll(e) * 1000 : (int64_t)0;
  }();
  std::vector<int> thread_cpus_;  // set_thread_cpus
  int threads_;
  std::vector<int> order_;  // connection index of slot i (thread i % threads_ drives it)
  std::vector<std::unique_ptr<LgConn>> conns_;
};

}  // namespace mlapi
