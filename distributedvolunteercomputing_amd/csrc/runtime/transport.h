// Framed point-to-point message transport over TCP (host side of the data plane).
//
// Replaces the reference's imagezmq/ZeroMQ ImageHub/ImageSender pair
// (/root/reference/server.py:43,112 and worker.py:64,164): a message is (header, payload)
// where the header is a small UTF-8 string (the python layer puts JSON {msg,dtype,shape}
// there) and the payload is a raw byte buffer (a C-contiguous ndarray). In "ack" mode a
// receiver answers every frame with a 2-byte "OK" after it has been queued, which is the
// reference's REQ/REP flow control; without ack the sender streams (PUB/SUB analog).
//
// Differences from the reference, by design:
//  * a Hub accepts MANY senders on one port (the reference needs a port per client);
//  * the receive queue is bounded (credits): when full the Hub stops reading sockets, so TCP
//    back-pressure throttles the sender instead of silently growing a python list;
//  * all blocking I/O happens without the GIL, and every call takes a timeout so a dead
//    peer cannot hang the caller forever.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace vcxrt {

struct Frame {
  std::string header;
  std::vector<uint8_t> payload;
  std::string peer;  // "ip:port" of the sending socket
};

class Hub {
 public:
  // max_payload / max_header bound what ONE frame from an untrusted volunteer may make this
  // process allocate; a frame announcing more drops its connection before any allocation.
  Hub(const std::string& bind_host, int port, size_t capacity, bool ack, uint64_t max_payload = kDefaultMaxPayload,
      uint32_t max_header = kDefaultMaxHeader);
  static constexpr uint64_t kDefaultMaxPayload = 2ull << 30;  // 2 GiB: a raw 100-frame 1440p chunk
  static constexpr uint32_t kDefaultMaxHeader = 64u << 10;
  ~Hub();
  int port() const { return port_; }
  // Blocks up to timeout_s (<0: forever). Returns false on timeout / closed.
  bool recv(Frame* out, double timeout_s);
  size_t pending();
  void close();
  bool closed() const { return closed_.load(); }
  uint64_t frames_received() const { return frames_; }
  uint64_t bytes_received() const { return bytes_; }
  uint64_t frames_rejected() const { return rejected_; }

 private:
  void accept_loop();
  void conn_loop(int fd, std::string peer);
  void conn_frames(int fd, const std::string& peer);
  int listen_fd_ = -1;
  int port_ = 0;
  size_t capacity_;
  bool ack_;
  uint64_t max_payload_;
  uint32_t max_header_;
  std::atomic<bool> closed_{false};
  std::mutex mu_;
  std::condition_variable cv_not_empty_, cv_not_full_;
  std::deque<Frame> q_;
  std::thread acceptor_;
  std::mutex conn_mu_;
  std::vector<std::thread> conns_;
  std::vector<int> conn_fds_;
  std::atomic<uint64_t> frames_{0}, bytes_{0}, rejected_{0};
};

class Sender {
 public:
  Sender(const std::string& host, int port, bool ack, double connect_timeout_s);
  ~Sender();
  // Sends one frame; in ack mode waits (up to timeout_s) for the receiver's "OK".
  // Returns false on timeout / broken connection (the sender is then closed).
  bool send(const std::string& header, const uint8_t* data, size_t n, double timeout_s);
  void close();
  bool connected() const { return fd_ >= 0; }
  uint64_t bytes_sent() const { return bytes_; }

 private:
  int fd_ = -1;
  bool ack_;
  std::mutex mu_;  // one frame at a time per socket (fixes the shared-REQ-socket race)
  uint64_t bytes_ = 0;
};

}  // namespace vcxrt
