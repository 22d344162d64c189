// FakePartDevice: a CPU stand-in for HipPartDevice (gpu_sha1.hip) behind PartDispatcher
// (part_dispatch.h), for selftest.cpp under TSan / ASan.
//
// Copy streams and compute streams are host threads with FIFO task queues, like HIP streams:
// a "DMA" is a memcpy into the slot's host memory after a random delay, a "kernel" waits for
// the copy markers (close_copies) of every slot of its launch, sleeps a random time and SHA-1s
// every lane, slot after slot. Events are
// shared atomic flags. On top of the device's own timing:
//   * `lag`: probability that a completed copy still reads as not ready - the dispatcher then
//     sees the slot's kernel finish before that copy, the order commit 363d26c had to handle;
//   * `fail_launch_at` / `fail_query_at`: the Nth launch / event query throws, as a HIP error
//     would (the hasher goes broken; parts it had finished must still be told).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "native.h"

namespace stager {

struct FakeDeviceKnobs {
  int copy_us_max = 200;       // random DMA latency per part
  int kernel_us_max = 1500;    // random kernel latency per launch
  double lag = 0.3;            // share of ready copies that still read as not ready
  int fail_launch_at = 0;      // the Nth launch throws (0: never)
  int fail_query_at = 0;       // the Nth copied()/finished() query throws (0: never)
  uint32_t seed = 1;
};

class FakePartDevice {
 public:
  using Event = std::shared_ptr<std::atomic<int>>;

  FakePartDevice(int64_t slot_bytes, int slots, int compute_streams, int copy_streams,
                 int max_lanes, FakeDeviceKnobs k)
      : max_lanes_(max_lanes), k_(k), rng_(k.seed) {
    slots_.resize((size_t)slots);
    for (auto& s : slots_) {
      s.mem.assign((size_t)slot_bytes, 0);
      s.lanes.assign((size_t)max_lanes * 2, 0);
      s.markers.resize((size_t)copy_streams);
    }
    runs_.resize((size_t)compute_streams);
    for (auto& r : runs_) r.done = std::make_shared<std::atomic<int>>(0);
    for (int i = 0; i < copy_streams; ++i) copies_.emplace_back(new Queue(k.seed * 7 + i));
    for (int i = 0; i < compute_streams; ++i) computes_.emplace_back(new Queue(k.seed * 13 + i));
  }
  ~FakePartDevice() {
    for (auto& q : copies_) q->stop();
    for (auto& q : computes_) q->stop();
  }
  FakePartDevice(const FakePartDevice&) = delete;
  FakePartDevice& operator=(const FakePartDevice&) = delete;

  int copy_streams() const { return (int)copies_.size(); }
  int compute_streams() const { return (int)computes_.size(); }
  int slots() const { return (int)slots_.size(); }
  void bind_thread() {}
  int64_t* lane_table(int s) { return slots_[(size_t)s].lanes.data(); }

  Event copy(int s, int64_t off, const uint8_t* host, int64_t len, int cs) {
    Event e = std::make_shared<std::atomic<int>>(0);
    uint8_t* dst = slots_[(size_t)s].mem.data() + off;
    const int us = k_.copy_us_max;
    Queue* q = copies_[(size_t)cs].get();
    q->push([dst, host, len, e, us, q] {
      q->nap(us);
      memcpy(dst, host, (size_t)len);
      e->store(1, std::memory_order_release);
    });
    return e;
  }
  bool copied(const Event& e) {
    tick();
    if (!e->load(std::memory_order_acquire)) return false;
    return !chance(k_.lag);
  }
  void recycle(const Event&) {}
  void close_copies(int s) {
    Slot& sl = slots_[(size_t)s];
    for (size_t k = 0; k < copies_.size(); ++k) {
      Event m = std::make_shared<std::atomic<int>>(0);
      sl.markers[k] = m;
      copies_[k]->push([m] { m->store(1, std::memory_order_release); });
    }
  }
  int64_t launch_lanes() const { return (int64_t)max_lanes_ * (int64_t)slots_.size(); }
  // One kernel over the lanes of several slots, in order (PartDispatcher's multi-slot launch).
  void launch(int stream, const int* slots, const int* lanes, int nslots, int total,
              bool /*align16*/) {
    if (k_.fail_launch_at && ++launches_ == k_.fail_launch_at)
      throw std::runtime_error("injected device fault (launch)");
    Run* run = &runs_[(size_t)stream];
    run->done->store(0, std::memory_order_relaxed);
    std::vector<std::pair<Slot*, int>> group;
    std::vector<Event> markers;
    for (int k = 0; k < nslots; ++k) {
      Slot* sl = &slots_[(size_t)slots[k]];
      group.push_back({sl, lanes[k]});
      markers.insert(markers.end(), sl->markers.begin(), sl->markers.end());
    }
    const int us = k_.kernel_us_max, ml = max_lanes_;
    Queue* q = computes_[(size_t)stream].get();
    run->dig.assign((size_t)total * 20, 0);
    q->push([run, group, markers, us, ml, q] {
      for (auto& m : markers)
        while (m && !m->load(std::memory_order_acquire)) std::this_thread::yield();
      q->nap(us);
      size_t i = 0;
      for (auto& g : group) {
        Slot* sl = g.first;
        for (int k = 0; k < g.second; ++k, ++i) {
          const int64_t off = sl->lanes[(size_t)k], len = sl->lanes[(size_t)(ml + k)];
          const std::string d = digest("sha1", sl->mem.data() + off, (size_t)len);
          memcpy(run->dig.data() + i * 20, d.data(), 20);
        }
      }
      run->done->store(1, std::memory_order_release);
    });
  }
  bool finished(int stream) {
    tick();
    return runs_[(size_t)stream].done->load(std::memory_order_acquire) != 0;
  }
  const uint8_t* digests(int stream) { return runs_[(size_t)stream].dig.data(); }
  void drain_copies() noexcept {
    for (auto& q : copies_) q->drain();
  }
  int reg(void*, size_t) { return 0; }
  void unreg(void*) {}

 private:
  // One "stream": a thread running its tasks in order.
  struct Queue {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> tasks;
    bool stopping = false, busy = false;
    std::mt19937 rng;
    std::thread th;
    explicit Queue(uint32_t seed) : rng(seed) {
      th = std::thread([this] {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
          cv.wait(lk, [&] { return stopping || !tasks.empty(); });
          if (tasks.empty()) return;
          auto f = std::move(tasks.front());
          tasks.pop_front();
          busy = true;
          lk.unlock();
          f();
          lk.lock();
          busy = false;
          cv.notify_all();
        }
      });
    }
    void push(std::function<void()> f) {
      std::lock_guard<std::mutex> g(mu);
      tasks.push_back(std::move(f));
      cv.notify_all();
    }
    void nap(int us_max) {   // on this queue's own thread
      const int us = us_max > 0 ? (int)(rng() % (uint32_t)us_max) : 0;
      if (us) std::this_thread::sleep_for(std::chrono::microseconds(us));
    }
    void drain() {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return tasks.empty() && !busy; });
    }
    void stop() {
      {
        std::lock_guard<std::mutex> g(mu);
        stopping = true;
      }
      cv.notify_all();
      if (th.joinable()) th.join();
    }
  };
  struct Slot {
    std::vector<uint8_t> mem;
    std::vector<int64_t> lanes;
    std::vector<Event> markers;
  };
  struct Run {                   // a compute stream's current launch
    std::vector<uint8_t> dig;
    Event done;
  };

  void tick() {
    if (k_.fail_query_at && ++queries_ == k_.fail_query_at)
      throw std::runtime_error("injected device fault (query)");
  }
  bool chance(double p) {   // dispatcher thread only
    return p > 0 && std::uniform_real_distribution<double>(0, 1)(rng_) < p;
  }

  int max_lanes_;
  FakeDeviceKnobs k_;
  std::mt19937 rng_;
  int launches_ = 0, queries_ = 0;
  std::vector<Slot> slots_;
  std::vector<Run> runs_;
  std::vector<std::unique_ptr<Queue>> copies_, computes_;
};

}  // namespace stager
