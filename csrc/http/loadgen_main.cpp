// mlapi-loadgen: the closed-loop load generator (loadgen.cpp) as its own process, so a benchmark
// rank can drive its server from CPUs apart from the server's threads (and so a DP bench drives
// the shared SO_REUSEPORT port like real clients). Line commands on stdin, one JSON line per
// command on stdout:
//
//   pin <cpu>,<cpu>,...                        sched_setaffinity (threads created later inherit it)
//   workload <path> [rel_tol]                  "MLW1\n" then per entry "<req_len> <exp_len>\n" + bytes
//   connect <host> <port> <conns> <threads> <timeout_s> [<source address>]
//   connmap <rr|shuffle> [seed]                which loop drives which connection (after connect)
//   threadcpus <cpu>,<cpu>,... | -             one CPU per client thread (after connect; - = none)
//   run <requests_per_conn> <record 0|1>       -> {"completed":..,"p50_ns":..,...}
//   close | quit
#include <sched.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "loadgen.h"

using namespace mlapi;

namespace {

bool read_workload(const std::string& path, std::vector<std::string>& req, std::vector<std::string>& exp) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::string magic;
  std::getline(f, magic);
  if (magic != "MLW1") return false;
  for (;;) {
    size_t a = 0, b = 0;
    std::string line;
    if (!std::getline(f, line)) break;
    if (sscanf(line.c_str(), "%zu %zu", &a, &b) != 2) return false;
    std::string r(a, '\0'), e(b, '\0');
    if (!f.read(&r[0], (std::streamsize)a) || (b && !f.read(&e[0], (std::streamsize)b))) return false;
    req.push_back(std::move(r));
    exp.push_back(std::move(e));
  }
  return !req.empty();
}

int64_t pct(std::vector<int64_t>& v, double q) {
  if (v.empty()) return 0;
  const size_t i = std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5));
  std::nth_element(v.begin(), v.begin() + (long)i, v.end());
  return v[i];
}

void reply(const std::string& s) {
  std::fputs(s.c_str(), stdout);
  std::fputc('\n', stdout);
  std::fflush(stdout);
}

}  // namespace

int main() {
  std::unique_ptr<Loadgen> lg;
  std::vector<std::string> req, exp;
  double rel_tol = 0.0;
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream in(line);
    std::string cmd;
    in >> cmd;
    try {
      if (cmd == "pin") {
        std::string list;
        in >> list;
        cpu_set_t set;
        CPU_ZERO(&set);
        std::stringstream ss(list);
        std::string tok;
        int n = 0;
        while (std::getline(ss, tok, ','))
          if (!tok.empty()) {
            CPU_SET(std::atoi(tok.c_str()), &set);
            ++n;
          }
        const int rc = n ? sched_setaffinity(0, sizeof set, &set) : 0;
        reply(std::string("{\"ok\":") + (rc == 0 ? "true" : "false") + ",\"cpus\":" + std::to_string(n) + "}");
      } else if (cmd == "workload") {
        std::string path;
        in >> path;
        if (!(in >> rel_tol)) rel_tol = 0.0;
        req.clear();
        exp.clear();
        if (!read_workload(path, req, exp)) throw std::runtime_error("bad workload file " + path);
        bool any_exp = false;
        for (auto& e : exp) any_exp |= !e.empty();
        if (!any_exp) exp.clear();
        if (lg) lg->set_workload(req, exp, rel_tol);
        reply("{\"ok\":true,\"entries\":" + std::to_string(req.size()) + "}");
      } else if (cmd == "connect") {
        std::string host;
        int port = 0, conns = 1, threads = 1;
        double timeout_s = 30;
        std::string source;
        in >> host >> port >> conns >> threads >> timeout_s;
        if (!(in >> source) || source == "-") source.clear();  // optional local (source) address
        if (req.empty()) throw std::runtime_error("connect before workload");
        lg = std::make_unique<Loadgen>(host, port, req[0], conns, threads, timeout_s, source);
        lg->set_workload(req, exp, rel_tol);
        reply("{\"ok\":true}");
      } else if (cmd == "connmap") {
        std::string mode;
        unsigned long long seed = 1;
        in >> mode;
        if (!(in >> seed)) seed = 1;
        if (!lg) throw std::runtime_error("connmap before connect");
        lg->set_conn_map(mode, seed);
        reply("{\"ok\":true}");
      } else if (cmd == "threadcpus") {
        std::string list;
        in >> list;
        if (!lg) throw std::runtime_error("threadcpus before connect");
        std::vector<int> cpus;
        std::stringstream ss(list == "-" ? std::string() : list);
        std::string tok;
        while (std::getline(ss, tok, ','))
          if (!tok.empty()) cpus.push_back(std::atoi(tok.c_str()));
        lg->set_thread_cpus(cpus);
        reply("{\"ok\":true,\"cpus\":" + std::to_string(cpus.size()) + "}");
      } else if (cmd == "run") {
        long long n = 0;
        int record = 1;
        in >> n >> record;
        if (!lg) throw std::runtime_error("run before connect");
        LoadgenResult r = lg->run(n, record != 0);
        std::ostringstream o;
        o << "{\"ok\":true,\"completed\":" << r.completed << ",\"errors\":" << r.errors
          << ",\"failed\":" << r.failed << ",\"body_mismatches\":" << r.body_mismatches
          << ",\"elapsed_s\":" << r.elapsed_s << ",\"ok200\":" << r.status_counts[200];
        if (record) {
          double sum = 0;
          for (int64_t v : r.latencies_ns) sum += (double)v;
          o << ",\"n_lat\":" << r.latencies_ns.size()
            << ",\"mean_ns\":" << (r.latencies_ns.empty() ? 0.0 : sum / (double)r.latencies_ns.size())
            << ",\"p50_ns\":" << pct(r.latencies_ns, 0.50) << ",\"p99_ns\":" << pct(r.latencies_ns, 0.99);
        }
        o << ",\"status\":{";
        bool first = true;
        for (int s = 0; s < 600; ++s)
          if (r.status_counts[s]) {
            o << (first ? "" : ",") << "\"" << s << "\":" << r.status_counts[s];
            first = false;
          }
        o << "}}";
        reply(o.str());
      } else if (cmd == "close") {
        lg.reset();
        reply("{\"ok\":true}");
      } else if (cmd == "quit") {
        reply("{\"ok\":true}");
        break;
      } else if (!cmd.empty()) {
        throw std::runtime_error("unknown command " + cmd);
      }
    } catch (const std::exception& e) {
      std::string msg = e.what();
      for (auto& ch : msg)
        if (ch == '"' || ch == '\\' || ch < 0x20) ch = ' ';
      reply("{\"ok\":false,\"error\":\"" + msg + "\"}");
    }
  }
  return 0;
}
