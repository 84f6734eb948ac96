// Race / memory-error stress driver for the host runtime (the reference has no
// locks and real races — one ZMQ REQ socket shared by two threads, a worker pool iterated while
// another thread mutates it). tests/test_native_sanitizers_cpu.py builds this file together with
// csrc/runtime/{scheduler,transport}.cpp once under -fsanitize=thread and once under
// -fsanitize=address,undefined and runs it; any sanitizer report or failed check fails the test.
//   1. ChunkScheduler: dispatcher threads racing membership churn (leave + rejoin, heartbeats,
//      lease expiry, request/stop toggles): every chunk must complete exactly once, and a chunk
//      is never dispatched to its own requester.
//   2. Hub/Sender: several sender threads stream framed messages into ONE bounded Hub in ack
//      mode (back-pressure blocks them): every frame arrives intact and in per-sender order.
//   3. ReorderIndex: random arrival orders with duplicates release every key once, in order.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "scheduler.h"
#include "transport.h"

using namespace vcxrt;
using Clock = std::chrono::steady_clock;

static std::atomic<int> g_errors{0};
#define EXPECT(c, msg)                                                             \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "CHECK FAILED: %s (%s:%d)\n", msg, __FILE__, __LINE__); \
      g_errors.fetch_add(1);                                                       \
    }                                                                              \
  } while (0)

static void scheduler_stress() {
  ChunkScheduler s(ChunkScheduler::ROUND_ROBIN, 3);
  const int kChunks = 3000;
  const auto deadline = Clock::now() + std::chrono::seconds(90);
  for (int w = 0; w < 4; ++w) s.add_worker("w" + std::to_string(w), 0.0);
  std::vector<std::atomic<int>> completions(kChunks);
  for (auto& c : completions) c.store(0);
  std::atomic<int> done{0};
  // requesters: two external clients and one volunteer that is also a worker (w0)
  const char* reqs[3] = {"reqA", "reqB", "w0"};
  std::thread producer([&] {
    for (int c = 0; c < kChunks; ++c) s.submit(c, reqs[c % 3]);
  });
  std::vector<std::thread> disp;
  for (int t = 0; t < 3; ++t)
    disp.emplace_back([&] {
      while (done.load() < kChunks && Clock::now() < deadline) {
        Assignment a = s.next();
        if (!a.valid()) {
          std::this_thread::yield();
          continue;
        }
        EXPECT(a.worker != a.requester, "scheduler: chunk dispatched to its own requester");
        if (s.complete(a.chunk)) {
          completions[a.chunk].fetch_add(1);
          done.fetch_add(1);
        }
      }
    });
  std::thread churn([&] {
    double now = 1.0;
    while (done.load() < kChunks && Clock::now() < deadline) {
      s.remove_worker("w3");  // its in-flight chunks go back to the front of the queue
      s.add_worker("w3", now);
      for (int w = 0; w < 4; ++w) s.heartbeat("w" + std::to_string(w), now);
      s.expire(now, 1e9);
      s.set_available("w2", false);
      s.set_available("w2", true);
      (void)s.queued();
      (void)s.inflight();
      (void)s.workers();
      (void)s.available_workers();
      (void)s.inflight_of("w1");
      now += 1e-3;
    }
  });
  producer.join();
  for (auto& t : disp) t.join();
  churn.join();
  EXPECT(done.load() == kChunks, "scheduler: not every chunk completed before the deadline");
  for (int c = 0; c < kChunks; ++c) EXPECT(completions[c].load() <= 1, "scheduler: a chunk completed twice");
  EXPECT(s.queued() == 0 && s.inflight() == 0, "scheduler: work left over");
}

static void transport_stress() {
  Hub hub("127.0.0.1", 0, 8, /*ack=*/true);
  const int kSenders = 4, kFrames = 120;
  std::atomic<int> send_fail{0};
  std::vector<std::thread> ss;
  for (int i = 0; i < kSenders; ++i)
    ss.emplace_back([&, i] {
      Sender snd("127.0.0.1", hub.port(), true, 10.0);
      std::mt19937 rng(i);
      std::vector<uint8_t> buf;
      for (int f = 0; f < kFrames; ++f) {
        const size_t n = rng() % 65536;
        buf.resize(n);
        for (size_t k = 0; k < n; ++k) buf[k] = (uint8_t)(i * 31 + f * 7 + k);
        const std::string h = std::to_string(i) + ":" + std::to_string(f) + ":" + std::to_string(n);
        if (!snd.send(h, buf.data(), n, 60.0)) send_fail.fetch_add(1);
      }
      snd.close();
    });
  int got = 0;
  std::vector<int> next(kSenders, 0);
  Frame fr;
  while (got < kSenders * kFrames) {
    if (!hub.recv(&fr, 60.0)) break;
    int i = -1, f = -1;
    size_t n = 0;
    std::sscanf(fr.header.c_str(), "%d:%d:%zu", &i, &f, &n);
    if (i < 0 || i >= kSenders) {
      EXPECT(false, "transport: bad header");
      break;
    }
    EXPECT(f == next[i], "transport: frames of one sender out of order");
    EXPECT(fr.payload.size() == n, "transport: payload length");
    bool intact = fr.payload.size() == n;
    for (size_t k = 0; intact && k < n; ++k) intact = fr.payload[k] == (uint8_t)(i * 31 + f * 7 + k);
    EXPECT(intact, "transport: payload corrupted");
    next[i] = f + 1;
    ++got;
  }
  for (auto& t : ss) t.join();
  hub.close();
  EXPECT(got == kSenders * kFrames, "transport: frames lost");
  EXPECT(send_fail.load() == 0, "transport: a send failed");
}

static void reorder_property() {
  std::mt19937 rng(7);
  for (int trial = 0; trial < 200; ++trial) {
    const int n = 1 + (int)(rng() % 300);
    std::vector<int64_t> keys;
    for (int k = 1; k <= n; ++k) keys.push_back(k);
    for (int d = 0; d < n / 5; ++d) keys.push_back(1 + (int64_t)(rng() % n));  // duplicates
    std::shuffle(keys.begin(), keys.end(), rng);
    ReorderIndex ri(1);
    std::vector<int64_t> out;
    for (auto k : keys)
      for (auto r : ri.push(k)) out.push_back(r);
    EXPECT((int)out.size() == n, "reorder: every key released exactly once");
    for (int k = 0; k < (int)out.size(); ++k)
      if (out[k] != k + 1) {
        EXPECT(false, "reorder: keys released out of order");
        break;
      }
  }
}

int main() {
  scheduler_stress();
  transport_stress();
  reorder_property();
  if (g_errors.load()) {
    std::fprintf(stderr, "%d check(s) failed\n", g_errors.load());
    return 1;
  }
  std::printf("OK\n");
  return 0;
}
