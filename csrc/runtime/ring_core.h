// RingCore: the scheduling core of the native batch ring (runtime.cpp: BatchRing), free of
// torch and HIP so the host sanitizers can run it (tests/test_ring_sanitizers_cpu.py builds
// csrc/runtime/ring_stress.cpp against it with -fsanitize=thread and
// -fsanitize=address,undefined).
//
// A fixed set of slots cycles empty -> (producer fills) -> ready -> (consumer) -> empty.
// Producers take batch indices start, start + stride, ... in order but may finish in any
// order; the consumer always receives the slot holding the NEXT index (deterministic data
// order).  Two producer kinds: native threads (run_producers: take an index and an empty
// slot, fill, commit) and external ones (acquire_empty / commit from other threads, e.g.
// Python PIL decode threads).  stop() wakes and ends every waiter.
//
// Reference data path it replaces: DataLoader(num_workers=0) in the training loop
// (/root/reference/main.py:99-102) and the eval pipeline's read stage
// (evaluation_pipeline.py:53-71).
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mpa_runtime {

class RingCore {
 public:
  RingCore(int depth, int64_t start_index, int64_t stride)
      : index_(depth, -1), count_(depth, 0), next_index_(start_index),
        next_consume_(start_index), stride_(stride) {
    for (int i = 0; i < depth; ++i) empty_.push_back(i);
  }
  ~RingCore() { stop(); }

  int depth() const { return (int)index_.size(); }

  // Native producers: `threads` workers each loop {next index, an empty slot, fill, commit}
  // until stop() or, with num_batches >= 0, until the indices pass num_batches.  fill(id,
  // bidx) writes the slot's payload and returns its valid item count.
  void run_producers(int threads, std::function<int(int, int64_t)> fill,
                     int64_t num_batches = -1) {
    fill_ = std::move(fill);
    limit_ = num_batches;
    for (int t = 0; t < std::max(1, threads); ++t) workers_.emplace_back([this] { produce(); });
  }

  // Consumer: block until the slot holding the next batch index is ready; -1 once stopped.
  // (starvation counters: calls that found their batch not ready yet, and the time they
  // blocked - read by stats())
  int acquire() {
    std::unique_lock<std::mutex> lk(mu_);
    ++acquires_;
    if (find_ready() < 0 && !stopping_) {
      ++waits_;
      const auto t0 = std::chrono::steady_clock::now();
      cv_.wait(lk, [&] { return find_ready() >= 0 || stopping_; });
      blocked_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::steady_clock::now() - t0)
                         .count();
    }
    const int id = find_ready();
    if (id < 0) return -1;
    ready_.erase(std::find(ready_.begin(), ready_.end(), id));
    next_consume_ += stride_;
    return id;
  }

  void release(int id) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      index_[id] = -1;
      empty_.push_back(id);
    }
    cv_.notify_all();
  }

  // External producers: an empty slot to fill (-1 once stopped), then commit it.
  int acquire_empty() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !empty_.empty() || stopping_; });
    if (empty_.empty()) return -1;
    const int id = empty_.front();
    empty_.pop_front();
    return id;
  }

  void commit(int id, int64_t batch_index, int count) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      index_[id] = batch_index;
      count_[id] = count;
      ready_.push_back(id);
    }
    cv_.notify_all();
  }

  // batch index / item count of a slot the caller holds (acquired by it)
  int64_t batch_index(int id) const {
    std::lock_guard<std::mutex> lk(mu_);
    return index_[id];
  }
  int count(int id) const {
    std::lock_guard<std::mutex> lk(mu_);
    return count_[id];
  }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stopping_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_)
      if (t.joinable()) t.join();
    workers_.clear();
  }

  bool producing() const { return !workers_.empty(); }

  // consumer starvation since the last reset: {acquire calls, calls that had to wait for
  // a producer, nanoseconds spent waiting}
  void stats(int64_t out[3], bool reset) {
    std::lock_guard<std::mutex> lk(mu_);
    out[0] = acquires_;
    out[1] = waits_;
    out[2] = blocked_ns_;
    if (reset) acquires_ = waits_ = blocked_ns_ = 0;
  }

 private:
  int find_ready() const {  // the ready slot holding batch next_consume_, or -1
    for (int id : ready_)
      if (index_[id] == next_consume_) return id;
    return -1;
  }

  void produce() {
    while (true) {
      int id;
      int64_t bidx;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !empty_.empty() || stopping_; });
        if (stopping_) return;
        bidx = next_index_;
        if (limit_ >= 0 && bidx >= limit_) return;  // source exhausted
        id = empty_.front();
        empty_.pop_front();
        next_index_ += stride_;
      }
      const int n = fill_(id, bidx);  // outside the lock: producers fill in parallel
      commit(id, bidx, n);
    }
  }

  std::vector<int64_t> index_;
  std::vector<int> count_;
  int64_t next_index_, next_consume_, stride_;
  int64_t limit_ = -1;
  std::function<int(int, int64_t)> fill_;
  std::deque<int> empty_, ready_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  bool stopping_ = false;
  int64_t acquires_ = 0, waits_ = 0, blocked_ns_ = 0;
  std::vector<std::thread> workers_;
};

}  // namespace mpa_runtime
