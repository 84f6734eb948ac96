// Chunk scheduler: the coordinator's dispatch policy, lease table and in-flight ledger.
//
// Reference behaviour kept (server.py:77-91): chunks are dispatched FIFO to the
// pool of available volunteers minus the chunk's requester, round-robin by a global counter.
// Fixed by design:
//  * a chunk with no eligible worker stays queued (the reference pops and silently drops it);
//  * every dispatched chunk is recorded in an in-flight ledger, so a worker that leaves or
//    whose lease expires has its chunks re-queued at the FRONT and re-dispatched;
//  * per-worker credits bound the chunks in flight on one volunteer (flow control that the
//    reference gets only from a blocking 2-byte ack);
//  * all state sits behind one mutex — the reference iterates `clients` while another thread
//    mutates it (server.py:85-87 vs 106-150).
#pragma once
#include <cstdint>
#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

namespace vcxrt {

struct Assignment {
  int64_t chunk = -1;
  std::string worker;
  std::string requester;
  bool valid() const { return chunk >= 0; }
};

class ChunkScheduler {
 public:
  enum Policy { ROUND_ROBIN = 0, LEAST_LOADED = 1 };
  explicit ChunkScheduler(int policy = ROUND_ROBIN, int credits = 2) : policy_(policy), credits_(credits) {}

  // membership (the `clients` pool of server.py)
  void add_worker(const std::string& w, double now);
  // Removes w from the pool; returns the chunk ids it had in flight (re-queued at the front).
  std::vector<int64_t> remove_worker(const std::string& w);
  void set_available(const std::string& w, bool avail);  // request/stop verbs toggle this
  bool has_worker(const std::string& w);
  std::vector<std::string> workers();
  std::vector<std::string> available_workers();

  // leases
  void heartbeat(const std::string& w, double now);
  // Workers whose last heartbeat is older than lease_s are removed; their chunks re-queued.
  std::vector<std::string> expire(double now, double lease_s);

  // work
  void submit(int64_t chunk, const std::string& requester);
  void requeue_front(int64_t chunk, const std::string& requester);
  Assignment next();  // invalid Assignment when nothing is dispatchable
  bool complete(int64_t chunk);  // returns false for an unknown / duplicate completion
  // The transfer of `chunk` to `worker` failed (p2p plane): if it is still in flight there, take
  // it back and re-queue it at the front. Returns false when the chunk is not w's any more.
  bool fail(int64_t chunk, const std::string& worker);
  std::vector<int64_t> cancel_requester(const std::string& requester);  // drop (and return) its queued chunks

  size_t queued();
  size_t inflight();
  size_t inflight_of(const std::string& w);
  uint64_t dispatched() const { return dispatched_; }
  uint64_t requeued() const { return requeued_; }  // chunks re-queued by worker removal / expiry

 private:
  struct Pending {
    int64_t chunk;
    std::string requester;
  };
  struct WorkerState {
    bool available = true;
    double last_seen = 0;
    std::set<int64_t> inflight;
  };
  std::vector<int64_t> drop_worker_locked(const std::string& w);

  std::mutex mu_;
  int policy_;
  int credits_;
  uint64_t rr_ = 0;
  uint64_t dispatched_ = 0;
  uint64_t requeued_ = 0;
  std::vector<std::string> order_;  // join order (round-robin order)
  std::unordered_map<std::string, WorkerState> ws_;
  std::deque<Pending> q_;
  std::unordered_map<int64_t, std::pair<std::string, std::string>> owner_;  // chunk -> (worker, requester)
};

// In-order sink (reference worker.py:210-239 does an O(n^2) list scan; this is O(log n)).
// push() returns the run of consecutive keys that became writable.
class ReorderIndex {
 public:
  explicit ReorderIndex(int64_t first = 1) : next_(first) {}
  // Returns keys ready in order. Duplicates and already-emitted keys are ignored.
  std::vector<int64_t> push(int64_t key);
  int64_t next_expected() const { return next_; }
  size_t stashed() const { return stash_.size(); }
  void reset(int64_t first) {
    next_ = first;
    stash_.clear();
  }

 private:
  int64_t next_;
  std::set<int64_t> stash_;
};

}  // namespace vcxrt
