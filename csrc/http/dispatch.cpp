// Round-robin connection dispatcher for a serving group; protocol in dispatch.h.
#include "dispatch.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <chrono>
#include <cstddef>
#include <cstring>
#include <stdexcept>

namespace mlapi {
namespace {

constexpr uint32_t MAGIC = 0x4d4c4450u;  // "MLDP"
struct Hello {
  uint32_t magic;
  int32_t rank;
  int32_t pid;
  char claim[48];  // client address this member claims (source affinity), "" = none
};
struct Reply {
  uint32_t magic;
  int32_t port;
};

std::string default_group(const std::string& host, int port) {
  return "mlapi-dispatch/" + host + ":" + std::to_string(port);
}

socklen_t abstract_addr(const std::string& name, sockaddr_un* a) {
  std::memset(a, 0, sizeof *a);
  a->sun_family = AF_UNIX;
  const size_t n = std::min(name.size(), sizeof(a->sun_path) - 1);
  std::memcpy(a->sun_path + 1, name.data(), n);  // sun_path[0] = 0: Linux abstract namespace
  return (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
}

// Plain TCP listener (no SO_REUSEPORT: exactly one acceptor per port). -1 + errno on failure.
int tcp_listen(const std::string& host, int port, int backlog, int* bound) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE | AI_NUMERICSERV;
  addrinfo* res = nullptr;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host.empty() ? nullptr : host.c_str(), ps.c_str(), &hints, &res) != 0 || !res) {
    errno = EINVAL;
    return -1;
  }
  const int fd = socket(res->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, IPPROTO_TCP);
  if (fd < 0) {
    freeaddrinfo(res);
    return -1;
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (bind(fd, res->ai_addr, res->ai_addrlen) != 0 || listen(fd, backlog) != 0) {
    const int e = errno;
    freeaddrinfo(res);
    close(fd);
    errno = e;
    return -1;
  }
  freeaddrinfo(res);
  sockaddr_storage ss{};
  socklen_t sl = sizeof ss;
  getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &sl);
  *bound = ss.ss_family == AF_INET ? ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port)
                                   : ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port);
  return fd;
}

int unix_listen(const std::string& name) {
  const int fd = socket(AF_UNIX, SOCK_SEQPACKET | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  sockaddr_un a;
  const socklen_t len = abstract_addr(name, &a);
  if (bind(fd, reinterpret_cast<sockaddr*>(&a), len) != 0 || listen(fd, 256) != 0) {
    const int e = errno;
    close(fd);
    errno = e;
    return -1;
  }
  return fd;
}

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

// The abstract unix name is visible to every process in the network namespace: only a peer running
// as this user may join the group (receive client sockets) or act as its leader (send us sockets).
bool same_user(int fd) {
  ucred cr{};
  socklen_t len = sizeof cr;
  if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &len) != 0 || len != sizeof cr) return false;
  return cr.uid == geteuid();
}

}  // namespace

ConnDispatcher::ConnDispatcher(std::string group, std::string host, int port, int backlog, int rank,
                               std::function<void(int)> adopt, std::function<bool()> healthy, bool source_affinity,
                               std::string claim)
    : group_(std::move(group)),
      host_(std::move(host)),
      want_port_(port),
      backlog_(backlog),
      rank_(rank),
      adopt_(std::move(adopt)),
      healthy_(std::move(healthy)),
      claim_(claim.size() < sizeof(Hello::claim) ? std::move(claim) : std::string()),
      source_affinity_(source_affinity) {
  wake_fd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (wake_fd_ < 0) throw std::runtime_error("dispatch: eventfd failed");
}

ConnDispatcher::~ConnDispatcher() {
  stop();
  close(wake_fd_);
}

std::string ConnDispatcher::group() const {
  std::lock_guard<std::mutex> lk(mu_);
  return group_;
}

bool ConnDispatcher::try_lead() {
  int bound = 0;
  if (want_port_ == 0 && group_.empty()) {
    // ephemeral port: this process is the leader by construction; the group is named after it
    const int t = tcp_listen(host_, 0, backlog_, &bound);
    if (t < 0) throw std::runtime_error(std::string("dispatch: TCP bind failed: ") + strerror(errno));
    {
      std::lock_guard<std::mutex> lk(mu_);
      group_ = default_group(host_, bound);
    }
    const int u = unix_listen(group_);
    if (u < 0) {
      close(t);
      throw std::runtime_error("dispatch: group " + group_ + " already has a leader");
    }
    tcp_fd_ = t;
    unix_fd_ = u;
  } else {
    if (group_.empty()) {
      std::lock_guard<std::mutex> lk(mu_);
      group_ = default_group(host_, want_port_);
    }
    const int u = unix_listen(group_);
    if (u < 0) return false;  // someone else holds the name: join it
    // the previous leader's listener may still be closing (failover): retry the TCP bind briefly
    int t = -1;
    for (int i = 0; i < 100 && t < 0 && !stop_.load(); ++i) {
      t = tcp_listen(host_, want_port_, backlog_, &bound);
      if (t < 0) std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    if (t < 0) {
      close(u);  // give the name back; the election runs again
      return false;
    }
    tcp_fd_ = t;
    unix_fd_ = u;
  }
  port_.store(bound);
  leader_.store(true);
  elections_.fetch_add(1);
  if (source_affinity_ && !claim_.empty()) {
    std::lock_guard<std::mutex> lk(mu_);
    affinity_[claim_] = -1;  // the leader's own clients stay here
  }
  return true;
}

bool ConnDispatcher::try_join() {
  const int c = socket(AF_UNIX, SOCK_SEQPACKET | SOCK_CLOEXEC, 0);
  if (c < 0) return false;
  sockaddr_un a;
  const socklen_t len = abstract_addr(group_, &a);
  if (connect(c, reinterpret_cast<sockaddr*>(&a), len) != 0 || !same_user(c)) {
    close(c);
    return false;
  }
  timeval tv{2, 0};
  setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  Hello h{MAGIC, rank_, (int32_t)getpid(), {}};
  memcpy(h.claim, claim_.c_str(), claim_.size() + 1);
  Reply r{};
  if (send(c, &h, sizeof h, MSG_NOSIGNAL) != (ssize_t)sizeof h || recv(c, &r, sizeof r, 0) != (ssize_t)sizeof r ||
      r.magic != MAGIC) {
    close(c);
    return false;
  }
  set_nonblock(c);
  chan_fd_ = c;
  port_.store(r.port);
  leader_.store(false);
  return true;
}

void ConnDispatcher::start() {
  std::lock_guard<std::mutex> lk(start_mu_);
  if (started_) return;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(30);
  for (;;) {
    if (try_lead() || try_join()) break;
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("dispatch: could not lead or join group " + group_);
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  stop_.store(false);
  th_ = std::thread([this] { run(); });
  started_ = true;
}

void ConnDispatcher::stop() {
  std::lock_guard<std::mutex> lk(start_mu_);
  if (!started_) return;
  stop_.store(true);
  const uint64_t one = 1;
  ssize_t w = write(wake_fd_, &one, sizeof one);
  (void)w;
  if (th_.joinable()) th_.join();
  if (tcp_fd_ >= 0) close(tcp_fd_);
  if (unix_fd_ >= 0) close(unix_fd_);
  if (chan_fd_ >= 0) close(chan_fd_);
  tcp_fd_ = unix_fd_ = chan_fd_ = -1;
  {
    std::lock_guard<std::mutex> l2(mu_);
    for (auto& m : members_) close(m.fd);
    members_.clear();
  }
  started_ = false;
}

void ConnDispatcher::run() {
  pthread_setname_np(pthread_self(), "mlapi-dispatch");
  while (!stop_.load()) {
    if (leader_.load()) {
      lead_loop();
      continue;
    }
    member_loop();  // returns on stop or when the channel to the leader broke
    while (!stop_.load()) {  // failover: run the election again
      if (try_lead() || try_join()) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
}

std::vector<DispatchTarget> ConnDispatcher::targets() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<DispatchTarget> out;
  if (!leader_.load()) return out;
  out.push_back(DispatchTarget{rank_, self_conns_, self_healthy_});
  for (const auto& m : members_)
    if (m.rank >= 0) out.push_back(DispatchTarget{m.rank, m.conns, m.healthy});
  return out;
}

void ConnDispatcher::drop_member(size_t i) {
  std::lock_guard<std::mutex> lk(mu_);
  close(members_[i].fd);
  members_.erase(members_.begin() + (ptrdiff_t)i);
}

bool ConnDispatcher::send_fd(Member& m, int fd) {
  char b = 'C';
  iovec iov{&b, 1};
  alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(int))];
  std::memset(cbuf, 0, sizeof cbuf);
  msghdr msg{};
  msg.msg_iov = &iov;
  msg.msg_iovlen = 1;
  msg.msg_control = cbuf;
  msg.msg_controllen = sizeof cbuf;
  cmsghdr* c = CMSG_FIRSTHDR(&msg);
  c->cmsg_level = SOL_SOCKET;
  c->cmsg_type = SCM_RIGHTS;
  c->cmsg_len = CMSG_LEN(sizeof(int));
  std::memcpy(CMSG_DATA(c), &fd, sizeof(int));
  for (;;) {
    const ssize_t r = sendmsg(m.fd, &msg, MSG_NOSIGNAL | MSG_DONTWAIT);
    if (r == 1) return true;
    if (r < 0 && errno == EINTR) continue;
    return false;
  }
}

// Hand fd to target i (0 = this process, i > 0 = members_[i - 1]) if it is healthy; a member
// whose channel fails for good is dropped.
bool ConnDispatcher::deliver(size_t i, int fd) {
  if (i == 0) {
    if (!self_healthy_) return false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      ++self_conns_;
    }
    received_.fetch_add(1, std::memory_order_relaxed);
    adopt_(fd);
    return true;
  }
  Member& m = members_[i - 1];
  if (m.rank < 0 || !m.healthy) return false;
  if (send_fd(m, fd)) {
    std::lock_guard<std::mutex> lk(mu_);
    ++m.conns;
    close(fd);  // the member holds its own descriptor of the socket now
    return true;
  }
  if (errno != EAGAIN && errno != EWOULDBLOCK) drop_member(i - 1);  // peer gone
  return false;
}

// One connection to the next healthy target in round-robin order (source affinity: to the target
// its client address already uses, while that one is healthy); a target whose channel fails is
// dropped and the connection goes to the next one. No healthy target: the connection is closed
// (what a client of an all-unhealthy SO_REUSEPORT group saw: refused).
void ConnDispatcher::dispatch(int fd, const std::string& source) {
  if (source_affinity_ && !source.empty()) {
    const auto it = affinity_.find(source);
    if (it != affinity_.end()) {
      size_t i = 0;  // the target's current index (members come and go)
      if (it->second >= 0) {
        i = SIZE_MAX;
        for (size_t k = 0; k < members_.size(); ++k)
          if (members_[k].rank == it->second) i = k + 1;
      }
      if (i != SIZE_MAX && deliver(i, fd)) return;
      affinity_.erase(it);  // gone or unhealthy: the address moves on with its next connection
    }
  }
  for (size_t attempt = 0; attempt < 2 * (members_.size() + 1) + 2; ++attempt) {
    const size_t n = members_.size() + 1;
    const size_t i = rr_++ % n;
    const int rank = i == 0 ? -1 : members_[i - 1].rank;
    if (deliver(i, fd)) {
      if (source_affinity_ && !source.empty()) {
        if (affinity_.size() >= 65536) affinity_.clear();  // bounded: a full table starts over
        affinity_[source] = rank;
      }
      return;
    }
  }
  close(fd);
}

void ConnDispatcher::lead_loop() {
  std::vector<pollfd> pf;
  while (!stop_.load()) {
    {
      const bool h = healthy_();
      std::lock_guard<std::mutex> lk(mu_);
      self_healthy_ = h;
    }
    pf.clear();
    pf.push_back(pollfd{wake_fd_, POLLIN, 0});
    pf.push_back(pollfd{tcp_fd_, POLLIN, 0});
    pf.push_back(pollfd{unix_fd_, POLLIN, 0});
    for (const auto& m : members_) pf.push_back(pollfd{m.fd, POLLIN, 0});
    const int n = poll(pf.data(), pf.size(), 50);
    if (n < 0 && errno != EINTR) break;
    if (n <= 0) continue;
    if (pf[0].revents) return;  // stop()
    // membership and health first, so a connection accepted in this round sees them
    for (size_t k = pf.size(); k-- > 3;) {
      const size_t i = k - 3;
      if (!pf[k].revents) continue;
      Member& m = members_[i];
      if (m.rank < 0 && (pf[k].revents & POLLIN)) {  // pending hello
        Hello h{};
        const ssize_t r = recv(m.fd, &h, sizeof h, MSG_DONTWAIT);
        if (r == (ssize_t)sizeof h && h.magic == MAGIC) {
          // a claimed client address goes to this member from its first connection on (the
          // replica beside those clients: its IO threads run next to their CPUs). Recorded before
          // the reply, so the claim is in place when the member's start() returns; a member that
          // then fails leaves a claim to a rank no member has, which dispatch() drops
          h.claim[sizeof h.claim - 1] = '\0';
          if (source_affinity_ && h.claim[0] != '\0') {
            std::lock_guard<std::mutex> lk(mu_);
            affinity_[std::string(h.claim)] = h.rank;
          }
          const Reply rep{MAGIC, port_.load()};
          if (send(m.fd, &rep, sizeof rep, MSG_NOSIGNAL) == (ssize_t)sizeof rep) {
            std::lock_guard<std::mutex> lk(mu_);
            m.rank = h.rank;
            continue;
          }
        } else if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
          continue;
        }
        drop_member(i);
        continue;
      }
      if (pf[k].revents & POLLIN) {
        char buf[64];
        const ssize_t r = recv(m.fd, buf, sizeof buf, MSG_DONTWAIT);
        if (r > 0) {
          std::lock_guard<std::mutex> lk(mu_);
          m.healthy = buf[r - 1] == 'H';  // the latest report wins
          continue;
        }
        if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) continue;
        drop_member(i);
        continue;
      }
      if (pf[k].revents & (POLLHUP | POLLERR | POLLNVAL)) drop_member(i);
    }
    if (pf[2].revents & POLLIN) {
      for (;;) {
        const int c = accept4(unix_fd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
        if (c < 0) break;
        if (!same_user(c)) {  // another user's process: never hand it client sockets
          close(c);
          continue;
        }
        std::lock_guard<std::mutex> lk(mu_);
        members_.push_back(Member{c, -1, true, 0});
      }
    }
    if (pf[1].revents & POLLIN) {
      for (;;) {
        sockaddr_storage ss{};
        socklen_t sl = sizeof ss;
        const int c = accept4(tcp_fd_, reinterpret_cast<sockaddr*>(&ss), &sl, SOCK_NONBLOCK | SOCK_CLOEXEC);
        if (c < 0) break;
        int one = 1;
        setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);  // never Nagle
        std::string source;  // the client's address without its port (source affinity)
        if (source_affinity_) {
          char txt[INET6_ADDRSTRLEN] = {0};
          if (ss.ss_family == AF_INET)
            inet_ntop(AF_INET, &reinterpret_cast<sockaddr_in*>(&ss)->sin_addr, txt, sizeof txt);
          else if (ss.ss_family == AF_INET6)
            inet_ntop(AF_INET6, &reinterpret_cast<sockaddr_in6*>(&ss)->sin6_addr, txt, sizeof txt);
          source = txt;
        }
        dispatch(c, source);
      }
    }
  }
}

void ConnDispatcher::member_loop() {
  char sent = 0;
  while (!stop_.load()) {
    const char h = healthy_() ? 'H' : 'U';
    if (h != sent) {
      if (send(chan_fd_, &h, 1, MSG_NOSIGNAL | MSG_DONTWAIT) == 1) sent = h;
    }
    pollfd pf[2] = {{wake_fd_, POLLIN, 0}, {chan_fd_, POLLIN, 0}};
    const int n = poll(pf, 2, 20);  // health changes reach the leader within one period
    if (n < 0 && errno != EINTR) break;
    if (n <= 0) continue;
    if (pf[0].revents) return;
    bool broken = (pf[1].revents & (POLLHUP | POLLERR | POLLNVAL)) != 0;
    if (pf[1].revents & POLLIN) {
      for (;;) {
        char b;
        iovec iov{&b, 1};
        alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(int))];
        msghdr msg{};
        msg.msg_iov = &iov;
        msg.msg_iovlen = 1;
        msg.msg_control = cbuf;
        msg.msg_controllen = sizeof cbuf;
        const ssize_t r = recvmsg(chan_fd_, &msg, MSG_DONTWAIT | MSG_CMSG_CLOEXEC);
        if (r > 0) {
          for (cmsghdr* c = CMSG_FIRSTHDR(&msg); c != nullptr; c = CMSG_NXTHDR(&msg, c)) {
            if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS) {
              int fd;
              std::memcpy(&fd, CMSG_DATA(c), sizeof fd);
              set_nonblock(fd);
              received_.fetch_add(1, std::memory_order_relaxed);
              adopt_(fd);
            }
          }
          continue;
        }
        if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
        if (r < 0 && errno == EINTR) continue;
        broken = true;  // EOF: the leader went away
        break;
      }
    }
    if (broken) {
      close(chan_fd_);
      chan_fd_ = -1;
      return;
    }
  }
}

}  // namespace mlapi
