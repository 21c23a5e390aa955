// mg_rdzv.cpp — mgh_rendezvous (include/mg_host.h): rank 0 hands a small blob
// (the RCCL unique id of the exchange mode's communicator, mg_xchg.cpp) to the
// other ranks of one job over TCP.  MASTER_ADDR may be a dotted address or a
// host name (getaddrinfo); every wait is bounded by one deadline, so a peer
// that never shows up ends the call with -4 instead of a hang, and every
// descriptor is closed on every path (RAII).
#include <netdb.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>

#include "mg_host.h"

namespace {

using Clock = std::chrono::steady_clock;

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
    if (k < 0 && errno == EINTR) continue;
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
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
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
    for (int served = 1; served < world;) {
      if (!wait_fd(lfd.fd, POLLIN, deadline)) return -4;  // a peer never connected
      Fd c(::accept4(lfd.fd, nullptr, nullptr, SOCK_CLOEXEC));
      if (c.fd < 0) {
        if (errno == EINTR || errno == ECONNABORTED) continue;
        return -5;
      }
      if (!send_all(c.fd, data, n, deadline)) return -5;
      ++served;
    }
    return 0;
  }
  // other ranks: rank 0 may not listen yet, so connect until the deadline
  for (;;) {
    for (addrinfo* a = res.ai; a; a = a->ai_next) {
      Fd s(::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol));
      if (s.fd < 0) continue;
      if (::connect(s.fd, a->ai_addr, a->ai_addrlen) == 0) return recv_all(s.fd, data, n, deadline) ? 0 : -5;
    }
    if (remaining_ms(deadline) == 0) return -4;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}
