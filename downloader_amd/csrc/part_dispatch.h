// PartDispatcher<Dev>: the scheduling state machine of the GPU part hasher (gpu_part_api.h),
// independent of the device it drives.
//
// gpu_sha1.hip instantiates it with HipPartDevice (hipMemcpyAsync on copy streams, sha1_lanes
// launches on compute streams, hipEvent polling) for gfx950; selftest.cpp instantiates it with
// a fake device made of host threads with random copy / kernel latencies, so the same queue /
// slot / stream / notify logic runs under TSan and ASan on a CPU (the
// reference's shared singletons, /root/reference/lib/download.js:19,27, are the race class it
// guards against).
//
// The flow: submit() queues a part (a page-locked host buffer holding whole pieces); the
// dispatcher thread DMAs it into the open device slot at once on a copy stream, and the relay's
// lease on the buffer ends when that copy completes (COPIED) - not when the hash does; a slot
// (up to slot_bytes / max_lanes pieces of any number of parts) is launched as ONE kernel as
// soon as a compute stream is idle - together with every other slot closed meanwhile, so one
// launch spans all the slots that filled while the streams were busy and a launch is no longer
// capped at one slot's lanes (1 GiB = 256 pieces of 4 MiB: ~15 GB/s per stream);
// while all streams are busy the open slot keeps filling, so batches grow with the arrival
// rate; digests come back per launch and are handed out per slot (DONE). notify is called without mu_,
// on the dispatcher thread, for every phase a job reaches - including, when the device fails,
// the phases the loop had already reached but not yet told (a waiter must never be left
// without news: its buffer, budget and permit would leak).
//
// Dev interface (Event is a copyable handle):
//   int copy_streams() const; int compute_streams() const; int slots() const;
//   void bind_thread();                            // dispatcher thread start (hipSetDevice)
//   int64_t* lane_table(int slot);                 // host [off x max_lanes][len x max_lanes]
//   Event copy(int slot, int64_t off, const uint8_t* host, int64_t len, int copy_stream);
//   bool copied(Event e);                          // that DMA completed; throws on device error
//   void recycle(Event e);
//   void close_copies(int slot);                   // end of the slot's copies on every stream
//   int64_t launch_lanes() const;                  // lanes one launch may carry
//   void launch(int stream, const int* slots, const int* lanes, int nslots, int total,
//               bool align16);                     // after the slots' copies; lanes in order
//   bool finished(int stream);                     // its launch completed; throws on error
//   const uint8_t* digests(int stream);            // 20 B per lane of the launch, in order
//   void drain_copies() noexcept;                  // failure path: queued DMAs still read
//   int reg(void* p, size_t n); void unreg(void* p);
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <exception>
#include <mutex>
#include <pthread.h>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "gpu_part_api.h"

namespace stager {

struct PartDispatchStats {
  uint64_t submitted = 0, launches = 0, lanes = 0, max_batch_lanes = 0;
  uint64_t multi_slot_launches = 0, max_launch_slots = 0;
  uint64_t registered = 0, unregistered = 0;
  double register_s = 0;
  bool broken = false;
  size_t pending = 0;
  int copy_streams = 0, compute_streams = 0;
};

template <class Dev>
class PartDispatcher {
 public:
  template <class... A>
  PartDispatcher(int64_t slot_bytes, int max_lanes, A&&... dev_args)
      : dev_(std::forward<A>(dev_args)...), slot_bytes_(slot_bytes), max_lanes_(max_lanes) {
    slots_.resize((size_t)dev_.slots());
    running_.resize((size_t)dev_.compute_streams());
    api_.abi = GPU_PART_API_ABI;
    api_.ctx = this;
    api_.reg = [](void* c, void* p, size_t n) { return ((PartDispatcher*)c)->reg(p, n); };
    api_.unreg = [](void* c, void* p) { ((PartDispatcher*)c)->unreg(p); };
    api_.submit = [](void* c, const uint8_t* d, int64_t len, int64_t pl) {
      return ((PartDispatcher*)c)->submit(d, len, pl);
    };
    api_.wait = [](void* c, uint64_t t, int ph, uint8_t* out, size_t ol, char* err, size_t el) {
      return ((PartDispatcher*)c)->wait(t, ph, out, ol, err, el);
    };
    api_.set_notify = [](void* c, gpu_part_notify_fn fn, void* arg) {
      PartDispatcher* h = (PartDispatcher*)c;
      std::lock_guard<std::mutex> g(h->mu_);
      h->notify_ = fn;
      h->notify_arg_ = arg;
    };
    thread_ = std::thread([this] { run(); });
    pthread_setname_np(thread_.native_handle(), "gpu-part-disp");
  }

  ~PartDispatcher() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (thread_.joinable()) thread_.join();
  }

  PartDispatcher(const PartDispatcher&) = delete;
  PartDispatcher& operator=(const PartDispatcher&) = delete;

  const GpuPartHashApi* api() const { return &api_; }
  Dev& device() { return dev_; }

  int reg(void* p, size_t n) {
    const auto t0 = std::chrono::steady_clock::now();
    const bool ok = dev_.reg(p, n) == 0;
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::lock_guard<std::mutex> g(mu_);
    stats_.registered++;
    stats_.register_s += dt;
    return ok ? 0 : -1;
  }
  void unreg(void* p) {
    dev_.unreg(p);
    std::lock_guard<std::mutex> g(mu_);
    stats_.unregistered++;
  }

  uint64_t submit(const uint8_t* data, int64_t len, int64_t piece_len) {
    if (len <= 0 || piece_len <= 0) return 0;
    const int64_t np = (len + piece_len - 1) / piece_len;
    if (np > max_lanes_ || len > slot_bytes_) return 0;
    std::lock_guard<std::mutex> g(mu_);
    if (broken_ || stop_) return 0;
    uint64_t t = ++seq_;
    Job& j = jobs_[t];
    j.host = data;
    j.len = len;
    j.piece_len = piece_len;
    j.np = (int)np;
    queue_.push_back(t);
    stats_.submitted++;
    cv_.notify_all();
    return t;
  }

  int wait(uint64_t t, int phase, uint8_t* out, size_t out_len, char* err, size_t errlen) {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = jobs_.find(t);
    if (it == jobs_.end()) return fail(err, errlen, "unknown ticket");
    Job* j = &it->second;   // elements of an unordered_map keep their address across rehashes
    wcv_.wait(lk, [&] {
      return !j->err.empty() || j->done || (phase == GPU_PART_COPIED && j->copied);
    });
    if (!j->err.empty()) {
      std::string e = j->err;
      // nobody waits again for a failed copy (the relay hashes on the host), and once broken
      // the dispatcher thread has exited: the job can go (by key: `it` may be stale)
      if (phase == GPU_PART_DONE || j->done || broken_) jobs_.erase(t);
      return fail(err, errlen, e.c_str());
    }
    if (phase == GPU_PART_DONE) {
      if (out_len < j->digests.size()) return fail(err, errlen, "digest buffer too small");
      memcpy(out, j->digests.data(), j->digests.size());
      jobs_.erase(t);
    }
    return 0;
  }

  PartDispatchStats stats() {
    std::lock_guard<std::mutex> g(mu_);
    PartDispatchStats s = stats_;
    s.broken = broken_;
    s.pending = jobs_.size();
    s.copy_streams = dev_.copy_streams();
    s.compute_streams = dev_.compute_streams();
    return s;
  }

 private:
  using Event = typename Dev::Event;
  struct Job {
    const uint8_t* host = nullptr;
    int64_t len = 0, piece_len = 0;
    int np = 0;
    int slot = -1, lane0 = 0;
    Event copy_ev{};
    bool copied = false, done = false;
    std::string err, digests;
  };
  struct Slot {
    int64_t used = 0;
    int lanes = 0;
    bool align16 = true;
    std::vector<uint64_t> jobs;
    int state = 0;               // 0 free, 1 filling, 2 closed (waiting for a stream), 3 running
    std::chrono::steady_clock::time_point opened;
  };

  static int fail(char* err, size_t errlen, const char* msg) {
    if (err && errlen) {
      strncpy(err, msg, errlen - 1);
      err[errlen - 1] = 0;
    }
    return -1;
  }

  // Tell the relay module about the phases in `owed` (and clear it): outside mu_ (the
  // callback calls wait() and may unregister buffers), on this dispatcher thread.
  void tell(std::vector<uint64_t>& owed, int phase) {
    if (owed.empty()) return;
    std::vector<uint64_t> tickets;
    tickets.swap(owed);
    gpu_part_notify_fn fn;
    void* arg;
    {
      std::lock_guard<std::mutex> g(mu_);
      fn = notify_;
      arg = notify_arg_;
    }
    if (fn)
      for (uint64_t t : tickets) fn(arg, t, phase);
  }

  Job& job(uint64_t t) {
    std::lock_guard<std::mutex> g(mu_);
    return jobs_.at(t);
  }

  // Everything below runs on the dispatcher thread; mu_ guards jobs_ / queue_ / flags.
  void run() {
    // phases reached (under mu_) but not yet told: kept across a device error so the failure
    // path still delivers them before it fails the rest
    std::vector<uint64_t> owed_copied, owed_done;
    std::deque<uint64_t> copying;                // tickets whose H2D is in flight, in order
    try {
      dev_.bind_thread();
      int filling = -1;
      for (;;) {
        std::deque<uint64_t> fresh;
        {
          std::unique_lock<std::mutex> lk(mu_);
          const bool idle = queue_.empty() && copying.empty() && !any_running() &&
                            !any_closed() && !(filling >= 0 && slots_[(size_t)filling].lanes > 0);
          if (idle) cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
          if (stop_ && idle && queue_.empty()) return;
          fresh.swap(queue_);
        }
        bool progressed = false;
        // 1. DMA new parts into the open slot (a new one when it is full)
        while (!fresh.empty()) {
          const uint64_t t = fresh.front();
          Job* j = &job(t);
          if (filling >= 0) {
            Slot& f = slots_[(size_t)filling];
            const int64_t off = (f.used + 255) & ~(int64_t)255;
            if (off + j->len > slot_bytes_ || f.lanes + j->np > max_lanes_) {
              f.state = 2;                    // full: closed, launched when a stream frees
              dev_.close_copies(filling);
              filling = -1;
            }
          }
          if (filling < 0) {
            filling = free_slot();
            if (filling < 0) break;            // every slot busy: the part waits queued
            Slot& f = slots_[(size_t)filling];
            f.state = 1;
            f.used = 0;
            f.lanes = 0;
            f.align16 = true;
            f.jobs.clear();
            f.opened = std::chrono::steady_clock::now();
          }
          Slot& f = slots_[(size_t)filling];
          const int64_t off = (f.used + 255) & ~(int64_t)255;
          const int cs = (int)(next_copy_++ % (size_t)dev_.copy_streams());
          Event ev = dev_.copy(filling, off, j->host, j->len, cs);
          int64_t* lt = dev_.lane_table(filling);
          for (int k = 0; k < j->np; ++k) {
            const int64_t po = (int64_t)k * j->piece_len;
            lt[f.lanes + k] = off + po;
            lt[max_lanes_ + f.lanes + k] = std::min(j->piece_len, j->len - po);
          }
          {
            std::lock_guard<std::mutex> g(mu_);
            j->copy_ev = ev;
            j->slot = filling;
            j->lane0 = f.lanes;
          }
          if (j->piece_len % 16) f.align16 = false;
          f.lanes += j->np;
          f.used = off + j->len;
          f.jobs.push_back(t);
          copying.push_back(t);
          fresh.pop_front();
          progressed = true;
        }
        const bool slot_bound = !fresh.empty();
        if (slot_bound) {                       // no free slot: back to the head of the queue
          std::lock_guard<std::mutex> g(mu_);
          for (auto it = fresh.rbegin(); it != fresh.rend(); ++it) queue_.push_front(*it);
        }
        // 2. completed copies: the relay may reuse those buffers (copies on different
        // streams finish out of order: every pending one is checked)
        for (auto it = copying.begin(); it != copying.end();) {
          Job* j = &job(*it);
          if (!dev_.copied(j->copy_ev)) {
            ++it;
            continue;
          }
          Event ev;
          {
            std::lock_guard<std::mutex> g(mu_);
            j->copied = true;
            ev = j->copy_ev;
            j->copy_ev = Event{};
            owed_copied.push_back(*it);
          }
          dev_.recycle(ev);
          wcv_.notify_all();
          it = copying.erase(it);
          progressed = true;
        }
        tell(owed_copied, GPU_PART_COPIED);
        // 3. finished kernels: publish digests, free the launch's slots and its stream
        for (size_t s = 0; s < running_.size(); ++s) {
          std::vector<int>& group = running_[s];
          if (group.empty()) continue;
          if (!dev_.finished((int)s)) continue;
          const uint8_t* dig = dev_.digests((int)s);
          std::vector<Event> late;
          {
            std::lock_guard<std::mutex> g(mu_);
            size_t base = 0;                  // first lane of each slot inside the launch
            for (int si : group) {
              Slot& sl = slots_[(size_t)si];
              for (uint64_t t : sl.jobs) {
                Job& j = jobs_.at(t);
                j.digests.assign((const char*)dig + (base + (size_t)j.lane0) * 20, (size_t)j.np * 20);
                j.done = true;
                if (!j.copied) {
                  // its copy ended after step 2 looked (the kernel waited for it): a DONE
                  // implies COPIED, and a job the relay may now erase must leave `copying`
                  j.copied = true;
                  late.push_back(j.copy_ev);
                  j.copy_ev = Event{};
                  auto c = std::find(copying.begin(), copying.end(), t);
                  if (c != copying.end()) copying.erase(c);
                  owed_copied.push_back(t);
                }
                owed_done.push_back(t);
              }
              base += (size_t)sl.lanes;
            }
          }
          for (Event e : late) dev_.recycle(e);
          wcv_.notify_all();
          for (int si : group) {
            slots_[(size_t)si].state = 0;
            slots_[(size_t)si].jobs.clear();
          }
          group.clear();
          progressed = true;
        }
        tell(owed_copied, GPU_PART_COPIED);
        // 4. launch on each idle stream: every closed slot (oldest first), then the open one,
        // as ONE kernel - up to the device's lanes per launch
        for (size_t s = 0; s < running_.size(); ++s) {
          if (!running_[s].empty()) continue;
          std::vector<int> group, lanes;
          int total = 0;
          bool a16 = true;
          for (int pick : closed_by_age()) {
            const Slot& sl = slots_[(size_t)pick];
            if (total + sl.lanes > dev_.launch_lanes()) break;
            group.push_back(pick);
            lanes.push_back(sl.lanes);
            total += sl.lanes;
            a16 = a16 && sl.align16;
          }
          if (filling >= 0 && slots_[(size_t)filling].lanes > 0 &&
              total + slots_[(size_t)filling].lanes <= dev_.launch_lanes()) {
            Slot& f = slots_[(size_t)filling];
            dev_.close_copies(filling);
            group.push_back(filling);
            lanes.push_back(f.lanes);
            total += f.lanes;
            a16 = a16 && f.align16;
            filling = -1;
          }
          if (group.empty()) break;
          dev_.launch((int)s, group.data(), lanes.data(), (int)group.size(), total, a16);
          for (int si : group) slots_[(size_t)si].state = 3;
          running_[s] = group;
          std::lock_guard<std::mutex> g(mu_);
          stats_.launches++;
          stats_.lanes += (uint64_t)total;
          stats_.max_batch_lanes = std::max<uint64_t>(stats_.max_batch_lanes, (uint64_t)total);
          stats_.max_launch_slots = std::max<uint64_t>(stats_.max_launch_slots, group.size());
          if (group.size() > 1) stats_.multi_slot_launches++;
          progressed = true;
        }
        tell(owed_done, GPU_PART_DONE);
        if (!progressed) {
          // nothing moved: poll the device again after a short sleep. New parts only end the
          // sleep early when there is a slot to put them in - with every slot busy the
          // predicate would be true at once and the thread would spin on mu_ and the device
          // queries against submit() / wait().
          // (system_clock on purpose: libstdc++ turns a steady_clock wait into
          // pthread_cond_clockwait, which GCC 11's TSan does not intercept - the mutex then
          // looks held through the wait and every submit() a double lock; a 200 us poll does
          // not care about wall-clock steps)
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::microseconds(200),
                         [&] { return stop_ || (!slot_bound && !queue_.empty()); });
        }
      }
    } catch (const std::exception& e) {
      // DMAs already queued on the copy streams may still read part buffers: let them end
      // before any waiter learns of the failure and hands its buffer back to the pool (which
      // may unmap it)
      dev_.drain_copies();
      // what the loop had reached but not told yet is real news, not a failure
      tell(owed_copied, GPU_PART_COPIED);
      tell(owed_done, GPU_PART_DONE);
      std::vector<uint64_t> failed_copy, failed_hash;
      {
        std::lock_guard<std::mutex> g(mu_);
        broken_ = true;
        for (auto& kv : jobs_)
          if (!kv.second.done) {
            kv.second.err = std::string("GPU part hasher: ") + e.what();
            (kv.second.copied ? failed_hash : failed_copy).push_back(kv.first);
          }
        queue_.clear();
        wcv_.notify_all();
      }
      tell(failed_copy, GPU_PART_COPIED);
      tell(failed_hash, GPU_PART_DONE);
    }
  }

  bool any_running() const {
    for (auto& g : running_)
      if (!g.empty()) return true;
    return false;
  }
  bool any_closed() const {
    for (auto& sl : slots_)
      if (sl.state == 2) return true;
    return false;
  }
  int free_slot() const {
    for (size_t i = 0; i < slots_.size(); ++i)
      if (slots_[i].state == 0) return (int)i;
    return -1;
  }
  std::vector<int> closed_by_age() const {
    std::vector<int> out;
    for (size_t i = 0; i < slots_.size(); ++i)
      if (slots_[i].state == 2) out.push_back((int)i);
    std::sort(out.begin(), out.end(),
              [&](int a, int b) { return slots_[(size_t)a].opened < slots_[(size_t)b].opened; });
    return out;
  }

  Dev dev_;                        // first member: destroyed last, after the thread joined
  int64_t slot_bytes_;
  int max_lanes_;
  size_t next_copy_ = 0;
  std::vector<std::vector<int>> running_;   // slots of the launch on each compute stream
  std::vector<Slot> slots_;
  std::mutex mu_;
  std::condition_variable cv_, wcv_;
  std::deque<uint64_t> queue_;
  std::unordered_map<uint64_t, Job> jobs_;
  uint64_t seq_ = 0;
  bool stop_ = false, broken_ = false;
  PartDispatchStats stats_;
  GpuPartHashApi api_{};
  gpu_part_notify_fn notify_ = nullptr;
  void* notify_arg_ = nullptr;
  std::thread thread_;
};

}  // namespace stager
