// Connection dispatcher: ONE acceptor per serving group hands every new TCP connection to the
// next healthy replica, round robin (BASELINE config 4: "round-robin dispatch").
//
// Why not SO_REUSEPORT alone: the kernel picks a listener by hashing the connection 4-tuple, so
// with 64 keep-alive clients per GPU the per-rank (and per-IO-thread) connection counts differ by
// +-5-17%, and the whole-node number is set by the most loaded rank.
//
// Protocol (all ranks of one host; no GPU involvement):
//  * the group is named by an abstract unix socket ("\0mlapi-dispatch/<host>:<port>" unless the
//    config names one). Binding that name is the election: the process that binds it is the
//    LEADER, owns the TCP listener and runs the acceptor; every other process connects to it as
//    a MEMBER (SOCK_SEQPACKET: hello {rank, pid} -> reply {tcp port}).
//  * leader: accept4() -> next target in round-robin order over [itself, members in join order],
//    skipping unhealthy ones -> its own IO threads (in-process hand-off) or the member's channel
//    (sendmsg SCM_RIGHTS, then the leader closes its copy). A failed send drops the member and
//    the same connection goes to the next target.
//  * member: recvmsg -> the fd goes to its next IO thread; it reports health changes as one byte
//    ('H' healthy / 'U' unhealthy), so an unhealthy replica stops receiving connections and is
//    re-admitted when its health probe succeeds (the round-2 leave/rejoin semantics).
//  * source affinity (optional, `source_affinity`): the first connection from a client address
//    takes the next target in round-robin order, and later connections from that address go to
//    the same target while it stays healthy (IPVS's "source hashing", kept as a table: a client
//    host's keep-alive connections land together, in their connect order). A host with many
//    clients behind one address then loads one replica: off by default, `bench.py` turns it on
//    with one source address per rank's load generator.
//  * failover: a member whose channel breaks (the leader died or stopped) runs the election again;
//    the winner re-binds the TCP port and the others re-join it. A restarted replica simply joins.
//  * trust: both ends check SO_PEERCRED - a member must run as the leader's user (the abstract
//    name is visible to every process of the network namespace), and a member only accepts
//    sockets from a leader of its own user.
//  * port 0: the process binds an ephemeral TCP port first and names the group after it (it is
//    the leader by construction; the others are given the bound port).
#pragma once
#include <atomic>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace mlapi {

struct DispatchTarget {
  int rank = -1;       // -1 = the leader's own IO threads
  uint64_t conns = 0;  // connections handed to this target
  bool healthy = true;
};

class ConnDispatcher {
 public:
  // adopt(fd): give a connected TCP socket to this process's IO threads. healthy(): may this
  // process receive new connections.
  ConnDispatcher(std::string group, std::string host, int port, int backlog, int rank,
                 std::function<void(int)> adopt, std::function<bool()> healthy, bool source_affinity = false,
                 std::string claim = "");
  ~ConnDispatcher();
  ConnDispatcher(const ConnDispatcher&) = delete;
  ConnDispatcher& operator=(const ConnDispatcher&) = delete;

  // Decides the role and binds (leader) or joins (member); returns once port() is known.
  void start();
  void stop();
  int port() const { return port_.load(); }
  bool leader() const { return leader_.load(); }
  uint64_t received() const { return received_.load(); }  // connections this process adopted
  uint64_t elections() const { return elections_.load(); }
  std::vector<DispatchTarget> targets() const;  // leader only (empty on members)
  std::string group() const;

 private:
  struct Member {
    int fd;
    int rank;
    bool healthy;
    uint64_t conns;
  };
  bool try_lead();        // bind the group name (+ TCP) -> true if this process is now the leader
  bool try_join();        // connect to the leader -> true if joined
  void run();
  void lead_loop();
  void member_loop();
  void dispatch(int fd, const std::string& source);
  bool deliver(size_t i, int fd);  // target i (0 = this process): true once the fd is handed over
  bool send_fd(Member& m, int fd);
  void drop_member(size_t i);

  std::string group_, host_;
  int want_port_, backlog_, rank_;
  std::function<void(int)> adopt_;
  std::function<bool()> healthy_;
  std::atomic<int> port_{0};
  std::atomic<bool> leader_{false}, stop_{false};
  std::atomic<uint64_t> received_{0}, elections_{0};
  int wake_fd_ = -1;   // eventfd: stop()
  int tcp_fd_ = -1;    // leader: TCP listener
  int unix_fd_ = -1;   // leader: group socket
  int chan_fd_ = -1;   // member: channel to the leader
  bool self_healthy_ = true;
  uint64_t self_conns_ = 0;
  size_t rr_ = 0;
  std::string claim_;  // client address this process claims (source affinity; sent in its hello)
  bool source_affinity_ = false;
  std::unordered_map<std::string, int> affinity_;  // client address -> target rank (-1 = leader)
  mutable std::mutex mu_;  // members_, self_* (read by targets())
  std::vector<Member> members_;
  std::thread th_;
  std::mutex start_mu_;
  bool started_ = false;
};

}  // namespace mlapi
