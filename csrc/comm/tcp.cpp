// TCP rendezvous + TCP host halo transport (see mdfx/bootstrap.hpp).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "mdfx/bootstrap.hpp"

namespace mdfx {

ProcEnv detect_proc_env() {
  ProcEnv e;
  auto get = [](const char* k) -> const char* {
    const char* v = std::getenv(k);
    return (v && *v) ? v : nullptr;
  };
  const char* triples[][3] = {{"RANK", "WORLD_SIZE", "LOCAL_RANK"},
                              {"OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"},
                              {"PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"}};
  for (auto& t : triples) {
    if (get(t[0]) && get(t[1])) {
      e.rank = std::atoi(get(t[0]));
      e.world = std::atoi(get(t[1]));
      e.local_rank = get(t[2]) ? std::atoi(get(t[2])) : e.rank;
      e.launched = e.world > 1;
      break;
    }
  }
  if (get("MASTER_ADDR")) e.addr = get("MASTER_ADDR");
  if (get("MDFX_PORT")) e.port = std::atoi(get("MDFX_PORT"));
  else if (get("MASTER_PORT")) e.port = std::atoi(get("MASTER_PORT")) + 7;  // stay off torch's store port
  return e;
}

namespace {

void send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n > 0) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) MDFX_FAIL(std::string("tcp send failed: ") + std::strerror(errno));
    c += k;
    n -= (size_t)k;
  }
}

void recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n > 0) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) MDFX_FAIL(std::string("tcp recv failed (peer gone?): ") + (k == 0 ? "eof" : std::strerror(errno)));
    c += k;
    n -= (size_t)k;
  }
}

void send_str(int fd, const std::string& s) {
  const uint64_t n = s.size();
  send_all(fd, &n, 8);
  send_all(fd, s.data(), s.size());
}

std::string recv_str(int fd) {
  uint64_t n = 0;
  recv_all(fd, &n, 8);
  std::string s(n, '\0');
  recv_all(fd, &s[0], n);
  return s;
}

void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

int listen_on(const std::string& addr, int port, int backlog) {
  const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  MDFX_CHECK(fd >= 0, "socket()");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = addr.empty() ? htonl(INADDR_ANY) : inet_addr(addr.c_str());
  if (::bind(fd, (sockaddr*)&a, sizeof(a)) != 0) {
    ::close(fd);
    MDFX_FAIL(format("bind %s:%d failed: %s", addr.c_str(), port, std::strerror(errno)));
  }
  MDFX_CHECK(::listen(fd, backlog) == 0, "listen()");
  return fd;
}

int connect_to(const std::string& addr, int port, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = inet_addr(addr.c_str());
    if (::connect(fd, (sockaddr*)&a, sizeof(a)) == 0) {
      tune(fd);
      return fd;
    }
    ::close(fd);
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      MDFX_FAIL(format("could not connect to %s:%d within %.0f s", addr.c_str(), port, timeout_s));
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

int local_port(int fd) {
  sockaddr_in a{};
  socklen_t l = sizeof(a);
  getsockname(fd, (sockaddr*)&a, &l);
  return ntohs(a.sin_port);
}

}  // namespace

Rendezvous::Rendezvous(const ProcEnv& env, double timeout_s) : env_(env) {
  if (env_.world <= 1) return;
  if (env_.rank == 0) {
    listen_fd_ = listen_on("", env_.port, env_.world);
    peers_.assign(env_.world, -1);
    for (int i = 1; i < env_.world; ++i) {
      const int fd = ::accept(listen_fd_, nullptr, nullptr);
      MDFX_CHECK(fd >= 0, "accept()");
      tune(fd);
      int32_t r = -1;
      recv_all(fd, &r, 4);
      MDFX_CHECK(r > 0 && r < env_.world && peers_[r] < 0, "bad rendezvous hello");
      peers_[r] = fd;
    }
  } else {
    const int fd = connect_to(env_.addr, env_.port, timeout_s);
    const int32_t r = env_.rank;
    send_all(fd, &r, 4);
    peers_.assign(1, fd);
  }
}

Rendezvous::~Rendezvous() {
  for (int fd : peers_)
    if (fd >= 0) ::close(fd);
  if (listen_fd_ >= 0) ::close(listen_fd_);
}

std::string Rendezvous::bcast(const std::string& root_data) {
  if (env_.world <= 1) return root_data;
  if (env_.rank == 0) {
    for (int i = 1; i < env_.world; ++i) send_str(peers_[i], root_data);
    return root_data;
  }
  return recv_str(peers_[0]);
}

std::vector<std::string> Rendezvous::allgather(const std::string& mine) {
  std::vector<std::string> all(env_.world);
  if (env_.world <= 1) {
    all[0] = mine;
    return all;
  }
  if (env_.rank == 0) {
    all[0] = mine;
    for (int i = 1; i < env_.world; ++i) all[i] = recv_str(peers_[i]);
    std::string packed;
    for (auto& s : all) {
      const uint64_t n = s.size();
      packed.append((const char*)&n, 8);
      packed.append(s);
    }
    for (int i = 1; i < env_.world; ++i) send_str(peers_[i], packed);
  } else {
    send_str(peers_[0], mine);
    const std::string packed = recv_str(peers_[0]);
    size_t p = 0;
    for (int i = 0; i < env_.world; ++i) {
      uint64_t n = 0;
      std::memcpy(&n, packed.data() + p, 8);
      p += 8;
      all[i] = packed.substr(p, n);
      p += n;
    }
  }
  return all;
}

double Rendezvous::allreduce_max(double v) {
  const auto all = allgather(std::string((const char*)&v, 8));
  double m = v;
  for (auto& s : all) {
    double x;
    std::memcpy(&x, s.data(), 8);
    m = std::max(m, x);
  }
  return m;
}

double Rendezvous::allreduce_sum(double v) {
  const auto all = allgather(std::string((const char*)&v, 8));
  double m = 0;
  for (auto& s : all) {  // rank order: deterministic
    double x;
    std::memcpy(&x, s.data(), 8);
    m += x;
  }
  return m;
}

void Rendezvous::barrier() { (void)allgather(std::string()); }

namespace {

class TcpTransport final : public Transport {
 public:
  explicit TcpTransport(Rendezvous& rv) : rv_(rv) {}
  ~TcpTransport() override {
    if (lo_fd_ >= 0) ::close(lo_fd_);
    if (hi_fd_ >= 0) ::close(hi_fd_);
  }
  const char* name() const override { return "tcp"; }
  bool in_process_only() const override { return false; }
  void setup(const std::vector<LocalSlab>& locals, int nranks) override {
    require_slabs(locals, "tcp");
    MDFX_CHECK(locals.size() == 1, "tcp transport: one slab per process");
    MDFX_CHECK(locals[0].be->kind() == DeviceKind::CPU, "tcp transport carries host memory (CPU backend)");
    MDFX_CHECK(nranks == rv_.world() && locals[0].rank == rv_.rank(), "tcp transport: slab index = process rank");
    slab_ = locals[0];
    nranks_ = nranks;
    // every rank listens on an ephemeral port; ports are shared through the rendezvous
    const int lfd = listen_on("", 0, 2);
    const int port = local_port(lfd);
    const char* host = std::getenv("MDFX_HOST");
    const std::string me = std::string(host ? host : "127.0.0.1") + ":" + std::to_string(port);
    const auto all = rv_.allgather(me);
    const int r = slab_.rank;
    if (r + 1 < nranks) {  // connect up
      const std::string& hp = all[r + 1];
      const size_t c = hp.rfind(':');
      hi_fd_ = connect_to(hp.substr(0, c), std::atoi(hp.c_str() + c + 1), 60.0);
    }
    if (r > 0) {  // accept from below
      lo_fd_ = ::accept(lfd, nullptr, nullptr);
      MDFX_CHECK(lo_fd_ >= 0, "accept()");
      tune(lo_fd_);
    }
    ::close(lfd);
    for (int fd : {lo_fd_, hi_fd_})
      if (fd >= 0) fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
  }

  void exchange(int b) override {
    struct Xfer {
      int fd;
      char* p;
      size_t left;
      bool send;
    };
    std::vector<Xfer> xs;
    for (int side = 0; side < 2; ++side) {
      const HaloSpan h = halo_span(slab_, b, side, nranks_);
      if (h.peer < 0) continue;
      const int fd = side == 0 ? lo_fd_ : hi_fd_;
      xs.push_back({fd, (char*)h.send, h.bytes, true});
      xs.push_back({fd, (char*)h.recv, h.bytes, false});
    }
    // full duplex on both sockets until every transfer is done
    for (;;) {
      std::vector<pollfd> pf;
      for (int fd : {lo_fd_, hi_fd_}) {
        if (fd < 0) continue;
        short ev = 0;
        for (auto& x : xs)
          if (x.fd == fd && x.left) ev |= x.send ? POLLOUT : POLLIN;
        if (ev) pf.push_back({fd, ev, 0});
      }
      if (pf.empty()) break;
      static const int timeout_ms = [] {
        const char* v = std::getenv("MDFX_TCP_TIMEOUT_S");
        return (int)(1000 * ((v && *v) ? std::atof(v) : 120.0));
      }();
      const int k = ::poll(pf.data(), pf.size(), timeout_ms);
      if (k < 0 && errno == EINTR) continue;
      MDFX_CHECK(k > 0, format("tcp halo exchange timed out after %.1f s (peer hung?)", timeout_ms / 1000.0));
      for (auto& q : pf) {
        if (q.revents & (POLLERR | POLLHUP | POLLNVAL)) MDFX_FAIL("tcp halo peer closed the connection");
        for (auto& x : xs) {
          if (x.fd != q.fd || !x.left) continue;
          if (x.send && (q.revents & POLLOUT)) {
            const ssize_t n = ::send(x.fd, x.p, x.left, MSG_NOSIGNAL);
            if (n > 0) {
              x.p += n;
              x.left -= (size_t)n;
            } else if (n < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
              MDFX_FAIL(std::string("tcp send: ") + std::strerror(errno));
            }
          } else if (!x.send && (q.revents & POLLIN)) {
            const ssize_t n = ::recv(x.fd, x.p, x.left, 0);
            if (n > 0) {
              x.p += n;
              x.left -= (size_t)n;
            } else if (n == 0) {
              MDFX_FAIL("tcp halo peer closed the connection");
            } else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
              MDFX_FAIL(std::string("tcp recv: ") + std::strerror(errno));
            }
          }
        }
      }
    }
  }
  double allreduce_sum(double v) override { return rv_.allreduce_sum(v); }
  double allreduce_max(double v) override { return rv_.allreduce_max(v); }
  void barrier() override { rv_.barrier(); }

 private:
  Rendezvous& rv_;
  LocalSlab slab_;
  int nranks_ = 1;
  int lo_fd_ = -1, hi_fd_ = -1;
};

}  // namespace

std::unique_ptr<Transport> make_tcp_transport(Rendezvous& rv) {
  return std::unique_ptr<Transport>(new TcpTransport(rv));
}

}  // namespace mdfx
