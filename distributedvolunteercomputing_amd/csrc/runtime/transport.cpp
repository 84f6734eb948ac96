#include "transport.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <stdexcept>

namespace vcxrt {

namespace {

constexpr uint32_t kMagic = 0x56435846u;  // "VCXF"

struct WireHeader {
  uint32_t magic;
  uint32_t header_len;
  uint64_t payload_len;
};

// Waits until fd is readable/writable or the deadline passes. deadline < 0: no deadline.
bool wait_fd(int fd, short ev, double timeout_s) {
  if (timeout_s < 0) return true;
  struct pollfd p{fd, ev, 0};
  int ms = (int)(timeout_s * 1000.0);
  for (;;) {
    int r = ::poll(&p, 1, ms);
    if (r > 0) return true;
    if (r == 0) return false;
    if (errno != EINTR) return false;
  }
}

bool write_all(int fd, const void* buf, size_t n, double timeout_s) {
  const uint8_t* p = (const uint8_t*)buf;
  auto t0 = std::chrono::steady_clock::now();
  while (n > 0) {
    double left = -1;
    if (timeout_s >= 0) {
      left = timeout_s - std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (left <= 0) return false;
    }
    if (!wait_fd(fd, POLLOUT, left)) return false;
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

// Reads exactly n bytes. Returns false on EOF / error / timeout / stop flag.
bool read_all(int fd, void* buf, size_t n, const std::atomic<bool>* stop, double timeout_s = -1) {
  uint8_t* p = (uint8_t*)buf;
  auto t0 = std::chrono::steady_clock::now();
  while (n > 0) {
    if (stop && stop->load()) return false;
    // poll in short slices so close() is noticed promptly
    double slice = 0.2;
    if (timeout_s >= 0) {
      double left = timeout_s - std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (left <= 0) return false;
      slice = left < slice ? left : slice;
    }
    if (!wait_fd(fd, POLLIN, slice)) continue;
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;
      return false;
    }
    p += r;
    n -= (size_t)r;
  }
  return true;
}

void tune_socket(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 8 << 20;
  ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

}  // namespace

// ============================================================================ Hub
Hub::Hub(const std::string& bind_host, int port, size_t capacity, bool ack, uint64_t max_payload, uint32_t max_header)
    : capacity_(capacity ? capacity : 1), ack_(ack), max_payload_(max_payload), max_header_(max_header) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("Hub: socket() failed");
  int one = 1;
  ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (bind_host.empty() || bind_host == "*" || bind_host == "0.0.0.0") {
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
  } else if (::inet_pton(AF_INET, bind_host.c_str(), &addr.sin_addr) != 1) {
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
  }
  if (::bind(listen_fd_, (sockaddr*)&addr, sizeof(addr)) != 0) {
    ::close(listen_fd_);
    throw std::runtime_error("Hub: bind() failed on port " + std::to_string(port) + ": " + strerror(errno));
  }
  if (::listen(listen_fd_, 64) != 0) {
    ::close(listen_fd_);
    throw std::runtime_error("Hub: listen() failed");
  }
  socklen_t len = sizeof(addr);
  ::getsockname(listen_fd_, (sockaddr*)&addr, &len);
  port_ = ntohs(addr.sin_port);
  acceptor_ = std::thread([this] { accept_loop(); });
}

Hub::~Hub() { close(); }

void Hub::close() {
  bool was = closed_.exchange(true);
  if (was) return;
  cv_not_empty_.notify_all();
  cv_not_full_.notify_all();
  if (listen_fd_ >= 0) {
    ::shutdown(listen_fd_, SHUT_RDWR);
  }
  if (acceptor_.joinable()) acceptor_.join();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
  std::vector<std::thread> conns;
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
    conns.swap(conns_);
  }
  for (auto& t : conns)
    if (t.joinable()) t.join();
  std::lock_guard<std::mutex> g(conn_mu_);
  for (int fd : conn_fds_) ::close(fd);
  conn_fds_.clear();
}

void Hub::accept_loop() {
  while (!closed_.load()) {
    if (!wait_fd(listen_fd_, POLLIN, 0.2)) continue;
    sockaddr_in peer{};
    socklen_t len = sizeof(peer);
    int fd = ::accept(listen_fd_, (sockaddr*)&peer, &len);
    if (fd < 0) continue;
    tune_socket(fd);
    char ip[64];
    ::inet_ntop(AF_INET, &peer.sin_addr, ip, sizeof(ip));
    std::string who = std::string(ip) + ":" + std::to_string(ntohs(peer.sin_port));
    std::lock_guard<std::mutex> g(conn_mu_);
    conn_fds_.push_back(fd);
    conns_.emplace_back([this, fd, who] { conn_loop(fd, who); });
  }
}

void Hub::conn_loop(int fd, std::string peer) {
  // Everything on this socket comes from an untrusted volunteer: lengths are checked against
  // the configured caps BEFORE anything is allocated, and no exception may escape the thread
  // (std::terminate would take the whole coordinator down).
  try {
    conn_frames(fd, peer);
  } catch (const std::exception&) {
    rejected_ += 1;
  }
  ::shutdown(fd, SHUT_RDWR);
}

void Hub::conn_frames(int fd, const std::string& peer) {
  while (!closed_.load()) {
    WireHeader wh{};
    if (!read_all(fd, &wh, sizeof(wh), &closed_)) break;
    if (wh.magic != kMagic || wh.header_len > max_header_ || wh.payload_len > max_payload_) {
      rejected_ += 1;  // protocol error or oversized frame: drop the connection, allocate nothing
      break;
    }
    Frame f;
    f.peer = peer;
    f.header.resize(wh.header_len);
    if (wh.header_len && !read_all(fd, &f.header[0], wh.header_len, &closed_)) break;
    f.payload.resize(wh.payload_len);
    if (wh.payload_len && !read_all(fd, f.payload.data(), wh.payload_len, &closed_)) break;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_not_full_.wait(lk, [&] { return closed_.load() || q_.size() < capacity_; });
      if (closed_.load()) break;
      bytes_ += wh.payload_len;
      frames_ += 1;
      q_.push_back(std::move(f));
    }
    cv_not_empty_.notify_one();
    if (ack_) {
      if (!write_all(fd, "OK", 2, 30.0)) break;
    }
  }
}

bool Hub::recv(Frame* out, double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return closed_.load() || !q_.empty(); };
  if (timeout_s < 0) {
    cv_not_empty_.wait(lk, ready);
  } else if (!cv_not_empty_.wait_for(lk, std::chrono::duration<double>(timeout_s), ready)) {
    return false;
  }
  if (q_.empty()) return false;
  *out = std::move(q_.front());
  q_.pop_front();
  lk.unlock();
  cv_not_full_.notify_one();
  return true;
}

size_t Hub::pending() {
  std::lock_guard<std::mutex> g(mu_);
  return q_.size();
}

// ============================================================================ Sender
Sender::Sender(const std::string& host, int port, bool ack, double connect_timeout_s) : ack_(ack) {
  addrinfo hints{};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  std::string h = (host.empty() || host == "*" || host == "localhost") ? "127.0.0.1" : host;
  if (::getaddrinfo(h.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("Sender: cannot resolve " + h);
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) break;
    if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
      tune_socket(fd);
      fd_ = fd;
      break;
    }
    ::close(fd);
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (connect_timeout_s >= 0 && el > connect_timeout_s) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));  // receiver may not be up yet
  }
  ::freeaddrinfo(res);
  if (fd_ < 0) throw std::runtime_error("Sender: connect to " + h + ":" + std::to_string(port) + " failed");
}

Sender::~Sender() { close(); }

void Sender::close() {
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ >= 0) {
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
  }
  fd_ = -1;
}

bool Sender::send(const std::string& header, const uint8_t* data, size_t n, double timeout_s) {
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ < 0) return false;
  WireHeader wh{kMagic, (uint32_t)header.size(), (uint64_t)n};
  bool ok = write_all(fd_, &wh, sizeof(wh), timeout_s) && write_all(fd_, header.data(), header.size(), timeout_s) &&
            (n == 0 || write_all(fd_, data, n, timeout_s));
  if (ok && ack_) {
    char rep[2];
    ok = read_all(fd_, rep, 2, nullptr, timeout_s) && rep[0] == 'O' && rep[1] == 'K';
  }
  if (!ok) {
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    fd_ = -1;
  } else {
    bytes_ += n;
  }
  return ok;
}

}  // namespace vcxrt
