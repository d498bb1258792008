// Host syscall costs on the serving box (what the IO threads pay per request): a bare syscall,
// eventfd write+read, epoll_wait(0) on a quiet set, a 150-byte loopback TCP send (+ the peer's
// recv), and io_uring availability (io_uring_setup). Single-threaded, no GPU.
//
//   g++ -O2 -std=c++17 tools/syscall_probe.cpp -o /tmp/syscall_probe && /tmp/syscall_probe
#include <arpa/inet.h>
#include <linux/io_uring.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>

namespace {
double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
template <typename F>
double per_call_ns(int n, F&& f) {
  for (int i = 0; i < n / 10; ++i) f();
  const double t0 = now_us();
  for (int i = 0; i < n; ++i) f();
  return (now_us() - t0) * 1e3 / n;
}
}  // namespace

int main() {
  const int N = 200000;
  printf("getppid            %7.1f ns\n", per_call_ns(N, [] { (void)syscall(SYS_getppid); }));
  const int efd = eventfd(0, EFD_NONBLOCK);
  uint64_t v = 1;
  printf("eventfd write+read %7.1f ns\n", per_call_ns(N, [&] {
           (void)!write(efd, &v, 8);
           (void)!read(efd, &v, 8);
         }));
  const int ep = epoll_create1(0);
  epoll_event ev{};
  ev.events = EPOLLIN;
  epoll_ctl(ep, EPOLL_CTL_ADD, efd, &ev);
  epoll_event out[16];
  printf("epoll_wait(0) idle %7.1f ns\n", per_call_ns(N, [&] { (void)epoll_wait(ep, out, 16, 0); }));

  // loopback TCP pair
  const int ls = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof a);
  socklen_t al = sizeof a;
  getsockname(ls, reinterpret_cast<sockaddr*>(&a), &al);
  listen(ls, 4);
  const int c = socket(AF_INET, SOCK_STREAM, 0);
  connect(c, reinterpret_cast<sockaddr*>(&a), sizeof a);
  const int s = accept(ls, nullptr, nullptr);
  setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  char msg[150];
  memset(msg, 'x', sizeof msg);
  char buf[4096];
  const int M = 50000;
  printf("tcp send 150 B     %7.1f ns  (send only; recv below)\n", [&] {
    double tot = 0;
    for (int i = 0; i < M; ++i) {
      const double t0 = now_us();
      (void)!send(s, msg, sizeof msg, MSG_NOSIGNAL);
      tot += now_us() - t0;
      (void)!recv(c, buf, sizeof buf, 0);
    }
    return tot * 1e3 / M;
  }());
  printf("tcp send+recv      %7.1f ns\n", per_call_ns(M, [&] {
           (void)!send(s, msg, sizeof msg, MSG_NOSIGNAL);
           (void)!recv(c, buf, sizeof buf, 0);
         }));
  io_uring_params p{};
  const long fd = syscall(__NR_io_uring_setup, 8, &p);
  printf("io_uring_setup     %s\n", fd >= 0 ? "ok" : strerror(errno));
  if (fd >= 0) close((int)fd);
  return 0;
}
