#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace mlapi {

struct LoadgenResult {
  double elapsed_s = 0;
  uint64_t completed = 0, errors = 0;
  int failed = 0;  // nonzero: connection error / timeout code
  std::vector<int64_t> latencies_ns;
  uint64_t status_counts[600] = {0};
};

struct LgConn;

class Loadgen {
 public:
  // Opens `conns` keep-alive connections (distributed over `threads` epoll loops).
  Loadgen(const std::string& host, int port, const std::string& request, int conns, int threads,
          double timeout_s = 30.0);
  ~Loadgen();
  // Every connection completes `requests_per_conn` closed-loop requests.
  LoadgenResult run(int64_t requests_per_conn, bool record = true);
  void close_all();

 private:
  std::string host_;
  int port_;
  std::string request_;
  double timeout_s_ = 30.0;
  int threads_;
  std::vector<std::unique_ptr<LgConn>> conns_;
};

}  // namespace mlapi
