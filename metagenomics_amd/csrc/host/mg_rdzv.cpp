// mg_rdzv.cpp — mgh_rendezvous (include/mg_host.h): rank 0 hands a small blob
// (the RCCL unique id of the exchange mode's communicator, mg_xchg.cpp) to the
// other ranks of one job over TCP.  MASTER_ADDR may be a dotted address or a
// host name (getaddrinfo); every wait is bounded by one deadline, so a peer
// that never shows up ends the call with -4 instead of a hang (the peers'
// connects are non-blocking too, so an address that drops SYNs cannot hold a
// rank past its deadline), and every descriptor is closed on every path (RAII).
// A peer opens with a header (magic, its rank); rank 0 serves each rank 1..P-1
// exactly once and drops a connection that sends no header, a wrong magic,
// rank 0, an out-of-range rank or a rank already served (a port probe, a
// health check, a duplicate).  It does not authenticate: a client that sends
// the magic and a rank not yet served is served as that rank, and the real
// rank is then dropped and ends with -4 / -5 at its deadline.  The id only
// names a communicator; the job is expected to run on one trusted node.
#include <netdb.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>

#include "mg_host.h"

namespace {

using Clock = std::chrono::steady_clock;
constexpr uint32_t kMagic = 0x4d47525aU;  // "MGRZ"
constexpr int kHeaderMs = 2000;           // a connection that sends no header within this is dropped

struct Fd {
  int fd = -1;
  explicit Fd(int f = -1) : fd(f) {}
  Fd(const Fd&) = delete;
  Fd& operator=(const Fd&) = delete;
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

struct AddrList {
  addrinfo* ai = nullptr;
  ~AddrList() {
    if (ai) freeaddrinfo(ai);
  }
};

int remaining_ms(Clock::time_point deadline) {
  const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
  return ms > 0 ? (int)ms : 0;
}

// wait until fd is readable (POLLIN) or writable (POLLOUT); false on the deadline or an error
bool wait_fd(int fd, short ev, Clock::time_point deadline) {
  for (;;) {
    pollfd p{fd, ev, 0};
    const int r = ::poll(&p, 1, remaining_ms(deadline));
    if (r > 0) return (p.revents & ev) != 0;
    if (r == 0) return false;
    if (errno != EINTR) return false;
  }
}

bool send_all(int fd, const char* p, size_t n, Clock::time_point deadline) {
  while (n) {
    if (!wait_fd(fd, POLLOUT, deadline)) return false;
    const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0 && (errno == EINTR || errno == EAGAIN || errno == EWOULDBLOCK)) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, char* p, size_t n, Clock::time_point deadline) {
  while (n) {
    if (!wait_fd(fd, POLLIN, deadline)) return false;
    const ssize_t k = ::recv(fd, p, n, 0);
    if (k < 0 && (errno == EINTR || errno == EAGAIN || errno == EWOULDBLOCK)) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

// non-blocking connect bounded by the deadline; true once connected
bool connect_by(int fd, const sockaddr* a, socklen_t len, Clock::time_point deadline) {
  if (::connect(fd, a, len) == 0) return true;
  if (errno != EINPROGRESS && errno != EINTR) return false;
  if (!wait_fd(fd, POLLOUT, deadline)) return false;
  int err = 0;
  socklen_t el = sizeof err;
  return ::getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el) == 0 && err == 0;
}

}  // namespace

extern "C" int mgh_rendezvous(int rank, int world, const char* addr, int port, void* blob, uint64_t n,
                              int timeout_ms) {
  if (world < 1 || rank < 0 || rank >= world || !addr || port <= 0 || port > 65535 || (n && !blob)) return -1;
  if (world == 1) return 0;
  const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 600000);
  AddrList res;
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (rank == 0) hints.ai_flags = AI_PASSIVE;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(addr, ps.c_str(), &hints, &res.ai) != 0 || !res.ai) return -2;
  char* data = static_cast<char*>(blob);
  if (rank == 0) {
    Fd lfd;
    for (addrinfo* a = res.ai; a && lfd.fd < 0; a = a->ai_next) {
      Fd s(::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol));
      if (s.fd < 0) continue;
      const int one = 1;
      (void)::setsockopt(s.fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
      if (::bind(s.fd, a->ai_addr, a->ai_addrlen) == 0 && ::listen(s.fd, world) == 0) std::swap(lfd.fd, s.fd);
    }
    if (lfd.fd < 0) return -3;
    std::string done((size_t)world, 0);
    for (int served = 1; served < world;) {
      if (!wait_fd(lfd.fd, POLLIN, deadline)) return -4;  // a peer never connected
      Fd c(::accept4(lfd.fd, nullptr, nullptr, SOCK_CLOEXEC | SOCK_NONBLOCK));
      if (c.fd < 0) {
        if (errno == EINTR || errno == ECONNABORTED || errno == EAGAIN) continue;
        return -5;
      }
      uint32_t hdr[2];
      const auto hd = std::min(deadline, Clock::now() + std::chrono::milliseconds(kHeaderMs));
      if (!recv_all(c.fd, reinterpret_cast<char*>(hdr), sizeof hdr, hd)) continue;  // not a peer: drop it
      if (hdr[0] != kMagic || hdr[1] < 1 || hdr[1] >= (uint32_t)world || done[hdr[1]]) continue;
      if (!send_all(c.fd, data, n, deadline)) continue;  // that peer went away: it may connect again
      done[hdr[1]] = 1;
      ++served;
    }
    return 0;
  }
  // other ranks: rank 0 may not listen yet, so connect until the deadline
  for (;;) {
    for (addrinfo* a = res.ai; a; a = a->ai_next) {
      Fd s(::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC | SOCK_NONBLOCK, a->ai_protocol));
      if (s.fd < 0) continue;
      if (!connect_by(s.fd, a->ai_addr, a->ai_addrlen, deadline)) continue;
      const uint32_t hdr[2] = {kMagic, (uint32_t)rank};
      if (!send_all(s.fd, reinterpret_cast<const char*>(hdr), sizeof hdr, deadline)) continue;
      return recv_all(s.fd, data, n, deadline) ? 0 : -5;
    }
    if (remaining_ms(deadline) == 0) return -4;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}
