#include "scheduler.h"

#include <algorithm>

namespace vcxrt {

void ChunkScheduler::add_worker(const std::string& w, double now) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = ws_.find(w);
  if (it != ws_.end()) {  // idempotent re-join (a lost `ok||port` reply must not double-insert);
    it->second.last_seen = now;  // it changes nothing else: a requester stays out of the worker pool
    return;
  }
  WorkerState s;
  s.last_seen = now;
  ws_.emplace(w, s);
  order_.push_back(w);
}

std::vector<int64_t> ChunkScheduler::drop_worker_locked(const std::string& w) {
  std::vector<int64_t> back;
  auto it = ws_.find(w);
  if (it == ws_.end()) return back;
  // re-queue in ascending chunk order at the front, so the earliest frames go out first
  std::vector<int64_t> ids(it->second.inflight.begin(), it->second.inflight.end());
  for (auto r = ids.rbegin(); r != ids.rend(); ++r) {
    auto o = owner_.find(*r);
    std::string req = o != owner_.end() ? o->second.second : std::string();
    owner_.erase(*r);
    q_.push_front(Pending{*r, req});
  }
  back = ids;
  requeued_ += ids.size();
  ws_.erase(it);
  order_.erase(std::remove(order_.begin(), order_.end(), w), order_.end());
  return back;
}

std::vector<int64_t> ChunkScheduler::remove_worker(const std::string& w) {
  std::lock_guard<std::mutex> g(mu_);
  return drop_worker_locked(w);
}

void ChunkScheduler::set_available(const std::string& w, bool avail) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = ws_.find(w);
  if (it != ws_.end()) it->second.available = avail;
}

bool ChunkScheduler::has_worker(const std::string& w) {
  std::lock_guard<std::mutex> g(mu_);
  return ws_.count(w) > 0;
}

std::vector<std::string> ChunkScheduler::workers() {
  std::lock_guard<std::mutex> g(mu_);
  return order_;
}

std::vector<std::string> ChunkScheduler::available_workers() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> r;
  for (auto& w : order_)
    if (ws_[w].available) r.push_back(w);
  return r;
}

void ChunkScheduler::heartbeat(const std::string& w, double now) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = ws_.find(w);
  if (it != ws_.end()) it->second.last_seen = now;
}

std::vector<std::string> ChunkScheduler::expire(double now, double lease_s) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> dead;
  for (auto& w : order_)
    if (now - ws_[w].last_seen > lease_s) dead.push_back(w);
  for (auto& w : dead) drop_worker_locked(w);
  return dead;
}

void ChunkScheduler::submit(int64_t chunk, const std::string& requester) {
  std::lock_guard<std::mutex> g(mu_);
  q_.push_back(Pending{chunk, requester});
}

void ChunkScheduler::requeue_front(int64_t chunk, const std::string& requester) {
  std::lock_guard<std::mutex> g(mu_);
  auto o = owner_.find(chunk);
  if (o != owner_.end()) {
    auto w = ws_.find(o->second.first);
    if (w != ws_.end()) w->second.inflight.erase(chunk);
    owner_.erase(o);
  }
  q_.push_front(Pending{chunk, requester});
}

Assignment ChunkScheduler::next() {
  std::lock_guard<std::mutex> g(mu_);
  Assignment a;
  // Scan the FIFO for the first chunk that has an eligible worker (head-of-line blocking
  // would otherwise stall every requester behind one whose only peer is itself).
  for (auto qi = q_.begin(); qi != q_.end(); ++qi) {
    std::vector<std::string> elig;
    for (auto& w : order_) {
      auto& s = ws_[w];
      if (!s.available || w == qi->requester) continue;
      if (credits_ > 0 && (int)s.inflight.size() >= credits_) continue;
      elig.push_back(w);
    }
    if (elig.empty()) continue;
    std::string pick;
    if (policy_ == LEAST_LOADED) {
      size_t best = SIZE_MAX;
      for (auto& w : elig) {
        size_t l = ws_[w].inflight.size();
        if (l < best) {
          best = l;
          pick = w;
        }
      }
    } else {
      pick = elig[rr_ % elig.size()];
      rr_++;
    }
    a.chunk = qi->chunk;
    a.worker = pick;
    a.requester = qi->requester;
    ws_[pick].inflight.insert(a.chunk);
    owner_[a.chunk] = {pick, a.requester};
    q_.erase(qi);
    dispatched_++;
    return a;
  }
  return a;
}

bool ChunkScheduler::complete(int64_t chunk) {
  std::lock_guard<std::mutex> g(mu_);
  auto o = owner_.find(chunk);
  if (o == owner_.end()) return false;
  auto w = ws_.find(o->second.first);
  if (w != ws_.end()) w->second.inflight.erase(chunk);
  owner_.erase(o);
  return true;
}

bool ChunkScheduler::fail(int64_t chunk, const std::string& worker) {
  std::lock_guard<std::mutex> g(mu_);
  auto o = owner_.find(chunk);
  if (o == owner_.end() || o->second.first != worker) return false;
  auto w = ws_.find(worker);
  if (w != ws_.end()) w->second.inflight.erase(chunk);
  q_.push_front(Pending{chunk, o->second.second});
  owner_.erase(o);
  ++requeued_;
  return true;
}

std::vector<int64_t> ChunkScheduler::cancel_requester(const std::string& requester) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<int64_t> dropped;
  for (const Pending& p : q_)
    if (p.requester == requester) dropped.push_back(p.chunk);
  q_.erase(std::remove_if(q_.begin(), q_.end(), [&](const Pending& p) { return p.requester == requester; }),
           q_.end());
  return dropped;  // the caller frees the payloads it holds for these chunks
}

size_t ChunkScheduler::queued() {
  std::lock_guard<std::mutex> g(mu_);
  return q_.size();
}

size_t ChunkScheduler::inflight() {
  std::lock_guard<std::mutex> g(mu_);
  return owner_.size();
}

size_t ChunkScheduler::inflight_of(const std::string& w) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = ws_.find(w);
  return it == ws_.end() ? 0 : it->second.inflight.size();
}

std::vector<int64_t> ReorderIndex::push(int64_t key) {
  std::vector<int64_t> out;
  if (key < next_) return out;  // late duplicate
  if (key != next_) {
    stash_.insert(key);
    return out;
  }
  out.push_back(key);
  next_++;
  while (!stash_.empty() && *stash_.begin() == next_) {
    out.push_back(next_);
    stash_.erase(stash_.begin());
    next_++;
  }
  // drop any stale entries below next_ (duplicates that slipped in)
  while (!stash_.empty() && *stash_.begin() < next_) stash_.erase(stash_.begin());
  return out;
}

}  // namespace vcxrt
