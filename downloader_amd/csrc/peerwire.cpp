// Native BitTorrent peer-wire receive path (BEP-3 framing) for swarm downloads.
//
// The reference downloads swarm pieces inside webtorrent (bittorrent-protocol framing, piece
// assembly, simple-sha1 verification, fs-chunk-store writes; /root/reference/lib/download.js:64,
// yarn.lock:389-398). In torrent/peer.py each 16 KiB block used to be framed, copied and
// bookkept in Python, and every piece SHA-1'd by one single-buffer chain: ~1 worker CPU-s per
// GB (round 2). Here the bytes stay native:
//   * a few I/O threads (`io_threads`, epoll, non-blocking sockets; connections spread over
//     them, fewest first) read and write every connection - not two threads per connection:
//     with 32 peers a job and 4 jobs a worker that was ~260 threads, each polling every 500 ms
//     (VERDICT r5). Each connection's messages are framed out of its own receive buffer; PIECE
//     payloads are copied once, straight into the assembling piece's buffer (first arrival of a
//     block wins); every other message goes up to Python, which stays the protocol and
//     state-machine owner (torrent/peer.py, torrent/session.py);
//   * a piece Python assigns to a connection (assign) is requested by the wire itself: the
//     I/O thread that takes a block answering one of that connection's requests queues the
//     next REQUEST, so `depth` stay in flight without Python, whose work per 4 MiB piece is one
//     assignment and one result instead of 256 block bookings (~0.1 CPU-s/GB on the event
//     loop); NEED tells Python when a connection's queue runs low, release / release_piece
//     hand a choked, closed or endgame piece back to per-block requesting;
//   * for the other pieces, Python learns which blocks arrived from one BLOCKS event per
//     receive batch (coalesced while Python has not polled: the busier the loop, the bigger
//     the batches);
//   * complete pieces are verified 16 at a time on the AVX-512 multi-buffer SHA-1 (sha1_mb),
//     written to the storage files with pwrite by one writer thread, and reported as PIECE
//     events;
//   * the same I/O thread sends, in one FIFO per connection, what Python queues (requests,
//     control messages), the refill REQUESTs (behind anything Python queued earlier, so the
//     wire keeps Python's message order) and the blocks asked for by peers Python has unchoked,
//     for pieces we have: the PIECE header, then the block straight from the storage files
//     with sendfile (no copy through user space; Python only decides who is unchoked). At most
//     kMaxServeQueue blocks wait per connection - a peer flooding REQUESTs is disconnected -
//     and a CANCEL drops its queued block.
// Events reach the event loop through an eventfd, like gpu_part_poll.
#include "native.h"
#include "gpu_part_api.h"

#include <poll.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <unistd.h>

#include <fcntl.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace stager {

namespace {

constexpr uint32_t kBlock = 16384;
constexpr uint32_t kMaxMsg = 2u << 20;     // torrent/peer.py MAX_MSG
constexpr uint8_t kPiece = 7;
constexpr uint8_t kRequest = 6;
constexpr uint8_t kCancel = 8;
constexpr uint32_t kMaxServe = 131072;     // session.py serve_request's bound
// blocks queued to serve on one connection (advertised as BEP-10 reqq, torrent/peer.py): a
// leecher sizing its pipeline to a fast, distant link keeps up to ~1,000 out (ours: 1,024;
// libtorrent allows 2,000); more is a flood (the queue grew without bound).
// 12 bytes of request each: 2,048 is ~100 KiB a connection.
constexpr size_t kMaxServeQueue = 2048;
constexpr size_t kRecvBatch = 1u << 20;    // receive room kept per connection (plus kMaxMsg)

uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
void put32(std::string& s, uint32_t v) {
  char b[4] = {(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
  s.append(b, 4);
}

// Piece buffers, process-wide: reused across pieces and sessions (no page faults per piece),
// and in GPU mode page-locked once for the hasher (hipHostRegister costs milliseconds per 4 MiB
// buffer - paid per session, it landed inside short jobs). Never destroyed: pieces may be
// released by a wire's threads during interpreter shutdown.
struct PiecePool {
  std::mutex mu;
  std::unordered_map<size_t, std::vector<std::pair<uint8_t*, const void*>>> idle;
  size_t in_use = 0, idle_count = 0, idle_bytes = 0;
  uint64_t allocs = 0, frees = 0, locks = 0;
  // Idle buffers kept (download.swarm_pool_mb): enough for the pieces in flight of a fast
  // swarm - ~250 x 4 MiB at 7 GB/s behind the GPU's ~150 ms - or every new one costs ~1,000
  // page faults in the reader that fills it and, in GPU mode, a page-locking.
  size_t max_idle_bytes = (size_t)1 << 30;

  // locked_for: the hasher the piece will most likely go to (GPU mode), else nullptr - an
  // idle buffer already page-locked for it is taken first (for a host piece, one that is not):
  // a LIFO of mixed buffers handed device pieces unlocked ones while locked ones sat idle,
  // ~30 page-lockings of a few ms each per 2 GB job after the first (config 6, r6/tail)
  uint8_t* take(size_t n, const void** reg, const void* locked_for) {
    {
      std::lock_guard<std::mutex> g(mu);
      in_use++;
      auto it = idle.find(n);
      if (it != idle.end() && !it->second.empty()) {
        auto& v = it->second;
        size_t k = v.size() - 1;
        // newest first, among the last 64 (the search stays short)
        for (size_t j = v.size(); j-- > 0 && j + 64 >= v.size();)
          if (v[j].second == locked_for) {
            k = j;
            break;
          }
        auto b = v[k];
        v[k] = v.back();
        v.pop_back();
        idle_count--;
        idle_bytes -= n;
        *reg = b.second;
        return b.first;
      }
    }
    void* b = aligned_alloc(4096, n);
    {
      std::lock_guard<std::mutex> g(mu);
      if (!b) {
        in_use--;
        throw std::bad_alloc();
      }
      allocs++;
    }
    *reg = nullptr;
    return (uint8_t*)b;
  }
  void give(uint8_t* b, size_t n, const void* reg) {
    {
      std::lock_guard<std::mutex> g(mu);
      in_use--;
      // a buffer locked for a hasher no longer installed goes (the API stays valid: retired
      // hashers are kept alive, ops/hashing.py)
      if (idle_bytes + n <= max_idle_bytes && (!reg || reg == gpu_part_hasher_current())) {
        idle[n].push_back({b, reg});
        idle_count++;
        idle_bytes += n;
        return;
      }
      frees++;
    }
    if (reg) ((const GpuPartHashApi*)reg)->unreg(((const GpuPartHashApi*)reg)->ctx, b);
    free(b);
  }
  // Idle buffers page-locked for `api` (the hasher is going away; all == nullptr: every idle
  // buffer), or beyond a new limit, are unlocked and freed.
  void drop_idle(bool all, const void* api, size_t limit) {
    std::vector<std::pair<uint8_t*, const void*>> drop;
    {
      std::lock_guard<std::mutex> g(mu);
      max_idle_bytes = limit;
      for (auto& kv : idle) {
        auto& v = kv.second;
        for (size_t i = 0; i < v.size();) {
          if ((all && v[i].second == api) || idle_bytes > max_idle_bytes) {
            drop.push_back(v[i]);
            v[i] = v.back();
            v.pop_back();
            idle_count--;
            idle_bytes -= kv.first;
            frees++;
          } else {
            ++i;
          }
        }
      }
    }
    for (auto& b : drop) {
      if (b.second)
        ((const GpuPartHashApi*)b.second)->unreg(((const GpuPartHashApi*)b.second)->ctx, b.first);
      free(b.first);
    }
  }
};

PiecePool& piece_pool() {
  static PiecePool* p = new PiecePool();
  return *p;
}

}  // namespace

void swarm_piece_pool_forget(const void* api) {
  PiecePool& p = piece_pool();
  size_t limit;
  {
    std::lock_guard<std::mutex> g(p.mu);
    limit = p.max_idle_bytes;
  }
  if (api) p.drop_idle(true, api, limit);
}

void swarm_piece_pool_limit(size_t bytes) { piece_pool().drop_idle(false, nullptr, bytes); }

struct SwarmWire::Piece {
  uint32_t idx = 0;
  uint32_t size = 0, nblocks = 0;
  uint8_t* data = nullptr;               // from the process-wide PiecePool
  size_t cap = 0;
  const void* reg = nullptr;             // hasher API the buffer is page-locked for (GPU mode)
  std::vector<uint8_t> claimed;          // per block: taken by a reader (under mu_)
  std::atomic<uint32_t> filled{0};       // blocks copied in
  uint64_t epoch = 0;                    // begin_piece generation (a re-begun piece is new)
  uint64_t owner = 0;                    // connection requesting it natively (under mu_)
  ~Piece() {
    if (data) piece_pool().give(data, cap, reg);
  }
};

// FIFO entry of what to send: bytes (Python's messages, refill REQUESTs), or (serve) a block
// to serve from storage: piece, begin, length packed into `data`. `off`: bytes of the item
// (serve: of its 13-byte PIECE header) already sent; `fdone`: serve, block bytes sent.
struct SwarmWire::OutItem {
  std::string data;
  bool serve = false;
  size_t off = 0;
  int64_t fdone = 0;
};

struct SwarmWire::Conn {
  uint64_t id = 0;
  int fd = -1;
  IoLoop* loop = nullptr;                // the I/O thread that reads and writes it
  std::mutex wmu;                        // out / out_bytes / serve_queued / stop
  using Item = OutItem;
  std::deque<Item> out;
  size_t out_bytes = 0, serve_queued = 0;
  bool stop = false;                     // under wmu
  std::atomic<bool> kicked{false};       // queued output the I/O thread has not looked at yet
  std::atomic<bool> serving{false};      // Python unchoked the peer: REQUESTs served natively
  std::atomic<uint64_t> served{0};
  std::atomic<bool> dead{false};
  std::string prefix;                    // bytes read before the handoff (asyncio buffer)
  std::atomic<int64_t> last_rx_ns{0};    // steady clock of the last receive
  std::atomic<uint64_t> rx{0};           // bytes received (Python's per-peer rate)
  // I/O thread only
  std::unique_ptr<uint8_t[]> rbuf;
  size_t rcap = 0, rstart = 0, rend = 0;
  bool out_armed = false;                // EPOLLOUT wanted (a send would have blocked)
  bool removed = false;                  // under the wire's lmu_: off its I/O thread for good
  // native request pipeline of its owned pieces (under the wire's mu_): blocks still to
  // request (piece << 32 | begin) and blocks requested and not answered yet
  std::deque<uint64_t> todo;
  std::unordered_set<uint64_t> asked;
  bool need_sent = false;
  uint32_t depth = 0;                    // requests in flight (0: the wire's set_pipeline)
};

// One I/O thread: an epoll set of connections plus an eventfd for commands (new connection,
// detach, output queued from Python, stop).
struct SwarmWire::IoLoop {
  int ep = -1, cmd = -1;
  std::thread th;
  std::mutex mu;                         // the command lists
  std::vector<std::shared_ptr<Conn>> adds, removes, kicks;
  bool stop = false;
  std::atomic<int> nconns{0};
  std::unordered_map<uint64_t, std::shared_ptr<Conn>> conns;   // I/O thread only

  void wake() {
    const uint64_t one = 1;
    ssize_t w = ::write(cmd, &one, sizeof one);
    (void)w;
  }
};

namespace {
inline uint64_t block_key(uint32_t idx, uint32_t begin) { return (uint64_t)idx << 32 | begin; }
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

SwarmWire::SwarmWire(int verify_threads, int io_threads) : io_threads_(std::max(1, io_threads)) {
  efd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (efd_ < 0) throw std::runtime_error("eventfd failed");
  for (int i = 0; i < std::max(1, verify_threads); ++i) {
    verifiers_.emplace_back([this] { verify_loop(); });
    pthread_setname_np(verifiers_.back().native_handle(), "wire-verify");
  }
  // digest collectors: each takes the oldest submitted piece, waits for it and compares
  for (int i = 0; i < std::max(1, verify_threads); ++i) {
    gthreads_.emplace_back([this] { gpu_loop(); });
    pthread_setname_np(gthreads_.back().native_handle(), "wire-gpu");
  }
  // one writer: page-cache writes into a file serialise on its inode anyway, and verifiers
  // that wrote themselves spun on that lock (4 of them: 2x the write CPU of one)
  sthread_ = std::thread([this] { store_loop(); });
  pthread_setname_np(sthread_.native_handle(), "wire-store");
}

SwarmWire::~SwarmWire() { close(); }

void SwarmWire::close() {
  std::vector<uint64_t> ids;
  {
    std::lock_guard<std::mutex> g(cmu_);
    for (auto& kv : conns_) ids.push_back(kv.first);
  }
  for (uint64_t id : ids) detach(id);
  std::vector<std::unique_ptr<IoLoop>> loops;
  {
    std::lock_guard<std::mutex> g(cmu_);
    loops.swap(loops_);
  }
  for (auto& l : loops) {
    {
      std::lock_guard<std::mutex> g(l->mu);
      l->stop = true;
    }
    l->wake();
    if (l->th.joinable()) l->th.join();
    ::close(l->ep);
    ::close(l->cmd);
  }
  {
    std::lock_guard<std::mutex> g(vmu_);
    vstop_ = true;
  }
  vcv_.notify_all();
  for (auto& t : verifiers_)
    if (t.joinable()) t.join();
  verifiers_.clear();
  {
    std::lock_guard<std::mutex> g(gmu_);
    gstop_ = true;
  }
  gcv_.notify_all();
  for (auto& t : gthreads_)                 // after the verifiers: nothing submits any more
    if (t.joinable()) t.join();
  gthreads_.clear();
  {
    std::lock_guard<std::mutex> g(smu_);
    sstop_ = true;                          // (the writer drains its queue first)
  }
  scv_.notify_all();
  if (sthread_.joinable()) sthread_.join();
  {
    std::lock_guard<std::mutex> g(mu_);
    pieces_.clear();                        // their pooled buffers go back before the pool
  }
  // (piece buffers go back to the process-wide pool, kept for the next session)
  if (efd_ >= 0) {
    ::close(efd_);
    efd_ = -1;
  }
}

void SwarmWire::set_storage(int64_t piece_length, int64_t total, const std::string& hashes,
                            const std::vector<std::pair<int, int64_t>>& files) {
  if (piece_length <= 0 || total < 0) throw std::invalid_argument("bad torrent geometry");
  const int64_t n = (total + piece_length - 1) / piece_length;
  if ((int64_t)hashes.size() != n * 20) throw std::invalid_argument("piece hashes do not match");
  std::lock_guard<std::mutex> g(mu_);
  piece_length_ = piece_length;
  total_ = total;
  hashes_ = hashes;
  files_ = files;
}

uint32_t SwarmWire::piece_size(uint32_t idx) const {
  const int64_t off = (int64_t)idx * piece_length_;
  return (uint32_t)std::min<int64_t>(piece_length_, total_ - off);
}

void SwarmWire::set_have(const std::string& bits) {
  std::lock_guard<std::mutex> g(mu_);
  have_.assign(bits.begin(), bits.end());
}

void SwarmWire::set_have_piece(uint32_t idx) {
  std::lock_guard<std::mutex> g(mu_);
  if (have_.size() <= idx / 8) have_.resize(idx / 8 + 1, 0);
  have_[idx / 8] |= (uint8_t)(0x80 >> (idx % 8));
}

bool SwarmWire::has(uint32_t idx) {      // mu_ held
  return idx / 8 < have_.size() && (have_[idx / 8] & (0x80 >> (idx % 8)));
}

void SwarmWire::set_serving(uint64_t id, bool on) {
  std::lock_guard<std::mutex> g(cmu_);
  auto it = conns_.find(id);
  if (it != conns_.end()) it->second->serving.store(on);
}

void SwarmWire::begin_piece(uint32_t idx) {
  std::lock_guard<std::mutex> g(mu_);
  if (piece_length_ <= 0 || (int64_t)idx * piece_length_ >= total_)
    throw std::out_of_range("begin_piece: no such piece");
  auto p = std::make_shared<Piece>();
  p->idx = idx;
  p->size = piece_size(idx);
  p->nblocks = (p->size + kBlock - 1) / kBlock;
  // pooled and reused: a fresh 4 MiB buffer per piece cost ~1,000 page faults in the reader
  // that first writes it; in GPU mode the pool's buffers are also page-locked once
  p->cap = ((size_t)piece_length_ + 4095) & ~(size_t)4095;
  p->data = piece_pool().take(p->cap, &p->reg,
                              gpu_.load() && !host_tail_.load() ? gpu_part_hasher_current()
                                                                : nullptr);
  p->claimed.assign(p->nblocks, 0);
  p->epoch = ++epoch_;
  pieces_[idx] = std::move(p);          // a re-begun piece (failed its check) starts over
  stats_.begun++;
}

void SwarmWire::drop_piece(uint32_t idx) {
  std::lock_guard<std::mutex> g(mu_);
  pieces_.erase(idx);
}

// 0 not taken (no such active piece, a duplicate, a bad offset / length), 1 taken, 2 taken and
// the piece is complete (queued for verification).
int SwarmWire::take_block(uint32_t idx, uint32_t begin, const uint8_t* p, uint32_t len) {
  bool owned = false, need = false;
  return take_from(nullptr, idx, begin, p, len, &owned, nullptr, &need);
}

// A block that arrived on connection `c` (nullptr: handed in by Python). An answer to one of
// the connection's own requests makes room in its pipeline: the next REQUESTs are appended to
// `reqs`, and `need` set when its queue fell below a pipeline.
int SwarmWire::take_from(Conn* c, uint32_t idx, uint32_t begin, const uint8_t* p, uint32_t len,
                         bool* owned, std::string* reqs, bool* need) {
  std::shared_ptr<Piece> pc;
  {
    std::lock_guard<std::mutex> g(mu_);
    // an answer to the wire's own request: not reported unless it lands in an ordinary piece
    // (a released one, whose blocks Python books again)
    const bool ours = c && c->asked.erase(block_key(idx, begin));
    if (ours && pump(*c, reqs)) *need = true;
    *owned = ours;
    auto it = pieces_.find(idx);
    if (it == pieces_.end()) {
      stats_.blocks_ignored++;
      return 0;
    }
    pc = it->second;
    const uint32_t b = begin / kBlock;
    // an owned piece takes blocks from its owner only: bytes nobody asked that peer for must
    // not mix into a piece whose hash failure is blamed on the owner
    if (pc->owner && (!c || pc->owner != c->id)) {
      *owned = true;        // (not reported either: Python did not ask this peer for it)
      stats_.blocks_ignored++;
      return 0;
    }
    if (begin % kBlock || b >= pc->nblocks || len != std::min(kBlock, pc->size - b * kBlock) ||
        pc->claimed[b]) {
      stats_.blocks_ignored++;
      return 0;
    }
    *owned = pc->owner != 0;
    pc->claimed[b] = 1;
    stats_.blocks++;
    stats_.block_bytes += len;
  }
  memcpy(pc->data + begin, p, len);        // outside the lock: readers copy in parallel
  const uint32_t f = pc->filled.fetch_add(1, std::memory_order_acq_rel) + 1;
  if (f < pc->nblocks) return 1;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = pieces_.find(idx);
    if (it != pieces_.end() && it->second == pc) pieces_.erase(it);
  }
  backlog_bytes_.fetch_add(pc->size);      // until its result is reported
  {
    std::lock_guard<std::mutex> g(vmu_);
    vq_.push_back(std::move(pc));
  }
  vcv_.notify_one();
  return 2;
}

// Next REQUESTs of `c`'s owned pieces, up to depth_ in flight (mu_ held). True the first time
// the queue of blocks to request drops below a pipeline since Python last filled it.
bool SwarmWire::pump(Conn& c, std::string* reqs) {
  const uint32_t depth = c.depth ? c.depth : depth_;
  while (c.asked.size() < depth && !c.todo.empty()) {
    const uint64_t k = c.todo.front();
    c.todo.pop_front();
    const uint32_t idx = (uint32_t)(k >> 32), begin = (uint32_t)k;
    auto it = pieces_.find(idx);
    if (it == pieces_.end() || it->second->owner != c.id) continue;   // complete or released
    const Piece& p = *it->second;
    if (p.claimed[begin / kBlock]) continue;
    c.asked.insert(k);
    stats_.requests++;
    if (reqs) {
      put32(*reqs, 13);
      reqs->push_back((char)kRequest);
      put32(*reqs, idx);
      put32(*reqs, begin);
      put32(*reqs, std::min(kBlock, p.size - begin));
    }
  }
  if (c.todo.size() < depth && !c.need_sent) {
    c.need_sent = true;
    return true;
  }
  return false;
}

// Output from any thread but the connection's I/O thread (Python's messages, assign's first
// REQUESTs): queued, and the I/O thread told once until it has looked.
void SwarmWire::queue_out(Conn& c, std::string data) {
  {
    std::lock_guard<std::mutex> g(c.wmu);
    if (c.stop) return;
    c.out_bytes += data.size();
    c.out.push_back(Conn::Item{std::move(data), false, 0, 0});
  }
  kick(c);
}

void SwarmWire::kick(Conn& c) {
  if (c.kicked.exchange(true)) return;
  IoLoop* l = c.loop;
  std::shared_ptr<Conn> sp = conn(c.id);
  if (!sp || !l) return;
  {
    std::lock_guard<std::mutex> g(l->mu);
    l->kicks.push_back(std::move(sp));
  }
  l->wake();
}

std::shared_ptr<SwarmWire::Conn> SwarmWire::conn(uint64_t id) {
  std::lock_guard<std::mutex> g(cmu_);
  auto it = conns_.find(id);
  return it == conns_.end() ? nullptr : it->second;
}

void SwarmWire::set_pipeline(uint32_t depth) {
  std::lock_guard<std::mutex> g(mu_);
  depth_ = std::max<uint32_t>(1, depth);
}

// One connection's requests in flight (its bandwidth-delay product, sized by Python from the
// peer's measured rate); a deeper pipeline is filled at once.
void SwarmWire::set_conn_pipeline(uint64_t id, uint32_t depth) {
  std::shared_ptr<Conn> c = conn(id);
  if (!c) return;
  std::string reqs;
  bool need;
  {
    std::lock_guard<std::mutex> g(mu_);
    c->depth = std::max<uint32_t>(1, depth);
    need = pump(*c, &reqs);
  }
  if (!reqs.empty()) queue_out(*c, std::move(reqs));
  // a deeper pipeline drains the queue below it: Python must hear so (pump marked NEED sent;
  // dropping it left the connection idle for good - config 6 stopped at 160 MiB)
  if (need) push(c->id, kEvNeed, std::string());
}

size_t SwarmWire::assign(uint64_t id, uint32_t idx) {
  std::shared_ptr<Conn> c = conn(id);
  if (!c) throw std::invalid_argument("assign: no such connection");
  std::string reqs;
  size_t n;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = pieces_.find(idx);
    if (it == pieces_.end()) throw std::out_of_range("assign: piece not active");
    Piece& p = *it->second;
    if (p.owner && p.owner != id) throw std::invalid_argument("assign: piece owned elsewhere");
    if (p.owner != id) stats_.assigned++;
    p.owner = id;
    for (uint32_t b = 0; b < p.nblocks; ++b) {
      const uint64_t k = block_key(idx, b * kBlock);
      if (!p.claimed[b] && !c->asked.count(k)) c->todo.push_back(k);
    }
    pump(*c, &reqs);
    n = c->todo.size();
    // Python sees the queue length in the return value: kEvNeed next when it falls below a
    // pipeline again, not while Python is still the one filling it
    c->need_sent = n < (c->depth ? c->depth : depth_);
  }
  if (!reqs.empty()) queue_out(*c, std::move(reqs));
  return n;
}

size_t SwarmWire::todo(uint64_t id) {
  std::shared_ptr<Conn> c = conn(id);
  if (!c) return 0;
  std::lock_guard<std::mutex> g(mu_);
  return c->todo.size();
}

std::string SwarmWire::block_states(const Piece& p, const Conn* owner) {
  std::string s(p.nblocks, '\0');
  for (uint32_t b = 0; b < p.nblocks; ++b)
    s[b] = p.claimed[b] ? 2 : (owner && owner->asked.count(block_key(p.idx, b * kBlock)) ? 1 : 0);
  return s;
}

std::vector<std::pair<uint32_t, std::string>> SwarmWire::release(uint64_t id) {
  std::shared_ptr<Conn> c = conn(id);   // (gone after detach: its requests count as unanswered)
  std::vector<std::pair<uint32_t, std::string>> out;
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : pieces_) {
    Piece& p = *kv.second;
    if (p.owner != id) continue;
    out.emplace_back(p.idx, block_states(p, c.get()));
    p.owner = 0;
  }
  if (c) {
    c->todo.clear();
    c->asked.clear();      // a choking peer drops what we asked for (BEP-3)
    c->need_sent = false;
  }
  return out;
}

bool SwarmWire::release_piece(uint32_t idx, uint64_t* owner, std::string* states) {
  uint64_t id;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = pieces_.find(idx);
    if (it == pieces_.end() || !it->second->owner) return false;
    id = it->second->owner;
  }
  std::shared_ptr<Conn> c = conn(id);
  std::lock_guard<std::mutex> g(mu_);
  auto it = pieces_.find(idx);
  if (it == pieces_.end() || it->second->owner != id) return false;
  *owner = id;
  *states = block_states(*it->second, c.get());
  it->second->owner = 0;      // its entries left in the owner's queue are skipped by pump
  return true;
}

double SwarmWire::rx_idle(uint64_t id) {
  std::shared_ptr<Conn> c = conn(id);
  if (!c) return 0.0;
  return (double)(now_ns() - c->last_rx_ns.load(std::memory_order_relaxed)) / 1e9;
}

void SwarmWire::verify_loop() {
  for (;;) {
    std::vector<std::shared_ptr<Piece>> batch;
    {
      std::unique_lock<std::mutex> lk(vmu_);
      vcv_.wait(lk, [&] { return vstop_ || !vq_.empty(); });
      if (vq_.empty()) return;               // stopping, nothing left
      // sha1_mb costs the same for 1 lane as for 16: let more pieces complete (at 4 GB/s a
      // 4 MiB piece completes every ~1 ms) before hashing a short batch - a piece's HAVE is
      // late by at most this much (system_clock: steady-clock waits are invisible to GCC 11's
      // TSan, part_dispatch.h). The GPU batches by itself: no wait there.
      if (vq_.size() < 16 && !vstop_ && !(gpu_.load() && !host_tail_.load()))
        vcv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(20),
                        [&] { return vstop_ || vq_.size() >= 16; });
      while (!vq_.empty() && batch.size() < 16) {
        batch.push_back(std::move(vq_.front()));
        vq_.pop_front();
      }
    }
    // GPU mode: submit each piece to the installed hasher, the collector finishes it
    const GpuPartHashApi* api =
        gpu_.load() && !host_tail_.load() ? (const GpuPartHashApi*)gpu_part_hasher_current()
                                          : nullptr;
    std::vector<std::shared_ptr<Piece>> host;
    for (auto& p : batch) {
      uint64_t t = 0;
      // the device takes pieces while fewer than gpu_cap_ are in flight on it (a 4 MiB piece
      // spends ~75 ms there): past that the download outruns it, and the host hashes the
      // rest instead of the pieces queueing (and their buffers piling up) behind the device
      if (api && gpu_inflight_.load() < gpu_cap_.load()) {
        if (p->reg != api) {
          if (p->reg) ((const GpuPartHashApi*)p->reg)->unreg(((const GpuPartHashApi*)p->reg)->ctx, p->data);
          p->reg = api->reg(api->ctx, p->data, p->cap) == 0 ? api : nullptr;
          if (p->reg) {
            std::lock_guard<std::mutex> g(piece_pool().mu);
            piece_pool().locks++;
          }
        }
        if (p->reg == api) t = api->submit(api->ctx, p->data, p->size, p->size);
      }
      if (t) {
        gpu_inflight_.fetch_add(1);
        std::lock_guard<std::mutex> g(gmu_);
        gq_.push_back({std::move(p), t, now_ns()});
        gcv_.notify_one();
      } else {
        if (api) {
          std::lock_guard<std::mutex> g(mu_);
          if (gpu_inflight_.load() < gpu_cap_.load()) stats_.gpu_refused++;
          else stats_.gpu_overflow++;
        }
        host.push_back(std::move(p));
      }
    }
    if (host.empty()) continue;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<const uint8_t*> ptrs;
    std::vector<size_t> lens;
    for (auto& p : host) {
      ptrs.push_back(p->data);
      lens.push_back(p->size);
    }
    std::string dig(host.size() * 20, '\0');
    if (sha1_mb_supported() && host.size() >= 4) {   // below 4 lanes one SHA-NI chain each wins
      sha1_mb(ptrs.data(), lens.data(), host.size(), (uint8_t*)&dig[0]);
    } else {
      for (size_t i = 0; i < host.size(); ++i) {
        std::string d = digest("sha1", ptrs[i], lens[i]);
        memcpy(&dig[i * 20], d.data(), 20);
      }
    }
    const auto t1 = std::chrono::steady_clock::now();
    {
      std::lock_guard<std::mutex> g(mu_);
      stats_.verify_batches++;
      stats_.sha_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    }
    for (size_t i = 0; i < host.size(); ++i)
      finish_piece(std::move(host[i]), (const uint8_t*)&dig[i * 20]);
  }
}

// The GPU's digests: each collector takes the oldest piece submitted and not yet claimed (the
// device hashes them in parallel anyway), so results come back in about submission order.
void SwarmWire::gpu_loop() {
  for (;;) {
    GpuJob job;
    {
      std::unique_lock<std::mutex> lk(gmu_);
      gcv_.wait(lk, [&] { return gstop_ || !gq_.empty(); });
      if (gq_.empty()) return;
      job = std::move(gq_.front());
      gq_.pop_front();
    }
    Piece& p = *job.piece;
    const GpuPartHashApi* api = (const GpuPartHashApi*)p.reg;
    uint8_t dig[20];
    char err[256] = {0};
    if (api->wait(api->ctx, job.ticket, GPU_PART_DONE, dig, sizeof dig, err, sizeof err) != 0) {
      // the device failed: the bytes are still in the buffer - hash them here
      std::string d = digest("sha1", p.data, p.size);
      memcpy(dig, d.data(), 20);
      std::lock_guard<std::mutex> g(mu_);
      stats_.gpu_errors++;
    } else {
      const int64_t lat = now_ns() - job.submit_ns;
      const int64_t prev = gpu_lat_ewma_ns_.load();
      gpu_lat_ewma_ns_.store(prev ? (prev * 7 + lat) / 8 : lat);
      std::lock_guard<std::mutex> g(mu_);
      stats_.gpu_pieces++;
      stats_.gpu_latency_ns_sum += lat;
      stats_.gpu_latency_ns_max = std::max(stats_.gpu_latency_ns_max, lat);
    }
    gpu_inflight_.fetch_sub(1);
    finish_piece(std::move(job.piece), dig);
  }
}

// A hashed piece: a mismatch is reported at once, a good one goes to the writer.
void SwarmWire::finish_piece(std::shared_ptr<Piece> p, const uint8_t* dig) {
  bool ok;
  {
    std::lock_guard<std::mutex> g(mu_);
    ok = memcmp(dig, hashes_.data() + (size_t)p->idx * 20, 20) == 0;
  }
  if (!ok) {
    report(p->idx, 0, std::string());
    return;
  }
  {
    std::lock_guard<std::mutex> g(smu_);
    sq_.push_back(std::move(p));
  }
  scv_.notify_one();
}

void SwarmWire::store_loop() {
  for (;;) {
    std::shared_ptr<Piece> p;
    {
      std::unique_lock<std::mutex> lk(smu_);
      scv_.wait(lk, [&] { return sstop_ || !sq_.empty(); });
      if (sq_.empty()) return;
      p = std::move(sq_.front());
      sq_.pop_front();
    }
    const auto w0 = std::chrono::steady_clock::now();
    std::string err = write_piece(*p);
    {
      std::lock_guard<std::mutex> g(mu_);
      stats_.write_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
          std::chrono::steady_clock::now() - w0).count();
    }
    report(p->idx, err.empty() ? 1 : 2, err);
  }
}

// PIECE event: 1 verified + written, 0 hash mismatch, 2 I/O error (+ message).
void SwarmWire::report(uint32_t idx, int status, const std::string& err) {
  std::string ev;
  put32(ev, idx);
  ev.push_back((char)status);
  ev += err;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (status == 1) {
      stats_.verified++;
      if (have_.size() <= idx / 8) have_.resize(idx / 8 + 1, 0);
      have_[idx / 8] |= (uint8_t)(0x80 >> (idx % 8));   // servable from now on
    } else if (status == 0) {
      stats_.hash_fails++;
    }
  }
  // (off the backlog before the result is out: a session that ends on it sees it drained)
  const int64_t left = backlog_bytes_.fetch_sub(piece_size(idx)) - piece_size(idx);
  push(0, kEvPiece, std::move(ev));
  // back-pressure off: half the cap drained since backlogged() said full -> NEED on conn 0
  if (backlog_full_.load() && left < backlog_cap_.load() / 2 && backlog_full_.exchange(false))
    push(0, kEvNeed, std::string());
}

void SwarmWire::set_backlog_cap(int64_t bytes) { backlog_cap_.store(std::max<int64_t>(0, bytes)); }

bool SwarmWire::backlogged() {
  const int64_t cap = backlog_cap_.load();
  if (cap <= 0 || backlog_bytes_.load() < cap) return false;
  backlog_full_.store(true);
  return true;
}

void SwarmWire::set_host_tail(bool on) { host_tail_.store(on); }

void SwarmWire::set_gpu(bool on, int max_inflight) {
  gpu_cap_.store(std::max(1, max_inflight));
  gpu_.store(on);
}


// The piece's bytes into the files it spans (pwrite; the storage owns the fds).
std::string SwarmWire::write_piece(const Piece& p) {
  int64_t off = (int64_t)p.idx * piece_length_;
  int64_t left = p.size;
  const uint8_t* src = p.data;
  int64_t fstart = 0;
  std::vector<std::pair<int, int64_t>> files;
  {
    std::lock_guard<std::mutex> g(mu_);
    files = files_;
  }
  for (auto& f : files) {
    const int64_t fend = fstart + f.second;
    if (left > 0 && off < fend && off >= fstart) {
      const int64_t k = std::min<int64_t>(left, fend - off);
      int64_t done = 0;
      while (done < k) {
        ssize_t w = ::pwrite(f.first, src + done, (size_t)(k - done), off - fstart + done);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) return std::string("pwrite: ") + strerror(w < 0 ? errno : EIO);
        done += w;
      }
      src += k;
      off += k;
      left -= k;
    }
    fstart = fend;
  }
  return left > 0 ? "piece past the end of the storage" : "";
}

void SwarmWire::push(uint64_t conn, int kind, std::string data) {
  {
    std::lock_guard<std::mutex> g(emu_);
    // BLOCKS of a connection coalesce while nobody polled: one event per poll, not per recv
    if (kind == kEvBlocks && !events_.empty() && events_.back().conn == conn &&
        events_.back().kind == kEvBlocks) {
      events_.back().data += data;
      return;
    }
    events_.push_back(WireEvent{conn, kind, std::move(data)});
  }
  const uint64_t one = 1;
  if (efd_ >= 0) {
    ssize_t w = write(efd_, &one, sizeof one);
    (void)w;
  }
}

std::vector<WireEvent> SwarmWire::poll() {
  uint64_t cnt;
  if (efd_ >= 0) {
    ssize_t r = read(efd_, &cnt, sizeof cnt);
    (void)r;
  }
  std::vector<WireEvent> out;
  std::lock_guard<std::mutex> g(emu_);
  out.reserve(events_.size());
  for (auto& e : events_) out.push_back(std::move(e));
  events_.clear();
  return out;
}

// ---- connections and their I/O threads

SwarmWire::IoLoop* SwarmWire::pick_loop() {   // cmu_ held
  if ((int)loops_.size() < io_threads_) {
    std::unique_ptr<IoLoop> l(new IoLoop());
    l->ep = ::epoll_create1(EPOLL_CLOEXEC);
    l->cmd = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (l->ep < 0 || l->cmd < 0) {
      if (l->ep >= 0) ::close(l->ep);
      if (l->cmd >= 0) ::close(l->cmd);
      if (loops_.empty()) throw std::runtime_error("epoll / eventfd failed");
    } else {
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.u64 = 0;                        // (connection ids start at 1)
      ::epoll_ctl(l->ep, EPOLL_CTL_ADD, l->cmd, &ev);
      IoLoop* raw = l.get();
      l->th = std::thread([this, raw] { io_loop(*raw); });
      pthread_setname_np(l->th.native_handle(), "wire-io");
      loops_.push_back(std::move(l));
      return raw;
    }
  }
  IoLoop* best = loops_.front().get();
  for (auto& l : loops_)
    if (l->nconns.load() < best->nconns.load()) best = l.get();
  return best;
}

void SwarmWire::attach(int fd, uint64_t id, const std::string& prefix) {
  if (id == 0) throw std::invalid_argument("connection id 0 is reserved");
  auto c = std::make_shared<Conn>();
  c->id = id;
  c->fd = fd;
  c->prefix = prefix;
  c->last_rx_ns.store(now_ns());
  const int fl = ::fcntl(fd, F_GETFL);           // (the asyncio socket's is; do not rely on it)
  if (fl >= 0 && !(fl & O_NONBLOCK)) ::fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  IoLoop* l;
  {
    std::lock_guard<std::mutex> g(cmu_);
    if (conns_.count(id)) throw std::invalid_argument("connection already attached");
    l = pick_loop();
    c->loop = l;
    l->nconns++;
    conns_[id] = c;
  }
  {
    std::lock_guard<std::mutex> g(l->mu);
    l->adds.push_back(c);
  }
  l->wake();
}

void SwarmWire::io_loop(IoLoop& l) {
  epoll_event evs[64];
  for (;;) {
    const int n = ::epoll_wait(l.ep, evs, 64, -1);
    if (n < 0) {
      if (errno == EINTR) continue;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));   // (EBADF etc. cannot happen
      continue;                                                    //  before close() joins)
    }
    for (int i = 0; i < n; ++i) {
      const uint64_t key = evs[i].data.u64;
      if (key == 0) {
        if (!commands(l)) return;
        continue;
      }
      auto it = l.conns.find(key);
      if (it == l.conns.end()) continue;          // killed or removed earlier in this batch
      std::shared_ptr<Conn> c = it->second;       // (kill() erases the map's reference)
      if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR | EPOLLRDHUP)) on_readable(l, *c);
      if (!c->dead.load() && (evs[i].events & EPOLLOUT)) flush(l, *c);
    }
  }
}

// The command eventfd fired: new connections, output queued by Python, detaches, stop.
bool SwarmWire::commands(IoLoop& l) {
  uint64_t cnt;
  ssize_t r = ::read(l.cmd, &cnt, sizeof cnt);
  (void)r;
  std::vector<std::shared_ptr<Conn>> adds, kicks, removes;
  bool stop;
  {
    std::lock_guard<std::mutex> g(l.mu);
    adds.swap(l.adds);
    kicks.swap(l.kicks);
    removes.swap(l.removes);
    stop = l.stop;
  }
  for (auto& c : adds) {
    // room for the largest message plus a receive batch; not value-initialised, so a
    // connection's pages are only touched as far as its data reaches
    c->rcap = (size_t)kMaxMsg + 64 + kRecvBatch;
    c->rbuf.reset(new uint8_t[c->rcap]);
    const size_t k = std::min(c->prefix.size(), c->rcap);
    if (k) memcpy(c->rbuf.get(), c->prefix.data(), k);
    c->rend = k;
    c->prefix.clear();
    l.conns[c->id] = c;
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u64 = c->id;
    if (::epoll_ctl(l.ep, EPOLL_CTL_ADD, c->fd, &ev) != 0) {
      kill(l, *c, std::string("epoll_ctl: ") + strerror(errno));
      continue;
    }
    if (c->rend) process(l, *c);                  // what asyncio had read already
    if (!c->dead.load()) flush(l, *c);
  }
  for (auto& c : kicks) {
    c->kicked.store(false);
    if (!c->dead.load() && l.conns.count(c->id)) flush(l, *c);
  }
  for (auto& c : removes) {
    if (l.conns.count(c->id)) {
      ::epoll_ctl(l.ep, EPOLL_CTL_DEL, c->fd, nullptr);
      if (!c->dead.exchange(true)) push(c->id, kEvClosed, "closed");
      l.conns.erase(c->id);
      l.nconns--;
    }
    {
      std::lock_guard<std::mutex> g(lmu_);
      c->removed = true;                          // the I/O thread is done with it
    }
    lcv_.notify_all();
  }
  return !stop;
}

// The connection is over (peer closed, error, protocol violation): out of the epoll set and
// this thread's map, the reason to Python. detach() still closes the fd.
void SwarmWire::kill(IoLoop& l, Conn& c, const std::string& reason) {
  if (c.dead.exchange(true)) return;
  ::epoll_ctl(l.ep, EPOLL_CTL_DEL, c.fd, nullptr);
  {
    std::lock_guard<std::mutex> g(c.wmu);
    c.stop = true;
  }
  if (l.conns.erase(c.id)) l.nconns--;
  push(c.id, kEvClosed, reason);
}

void SwarmWire::arm_out(IoLoop& l, Conn& c, bool on) {
  if (c.out_armed == on) return;
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP | (on ? EPOLLOUT : 0);
  ev.data.u64 = c.id;
  ::epoll_ctl(l.ep, EPOLL_CTL_MOD, c.fd, &ev);
  c.out_armed = on;
}

void SwarmWire::on_readable(IoLoop& l, Conn& c) {
  if (c.rstart == c.rend) {
    c.rstart = c.rend = 0;
  } else if (c.rstart > 0 && c.rcap - c.rend < kRecvBatch) {
    memmove(c.rbuf.get(), c.rbuf.get() + c.rstart, c.rend - c.rstart);
    c.rend -= c.rstart;
    c.rstart = 0;
  }
  const ssize_t r = ::recv(c.fd, c.rbuf.get() + c.rend, c.rcap - c.rend, MSG_DONTWAIT);
  if (r == 0) {
    kill(l, c, "closed");
    return;
  }
  if (r < 0) {
    if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) return;
    kill(l, c, std::string("recv: ") + strerror(errno));
    return;
  }
  c.rend += (size_t)r;
  c.last_rx_ns.store(now_ns(), std::memory_order_relaxed);
  c.rx.fetch_add((uint64_t)r, std::memory_order_relaxed);
  rx_bytes_.fetch_add((uint64_t)r, std::memory_order_relaxed);
  recvs_.fetch_add(1, std::memory_order_relaxed);
  process(l, c);
}

// Frame every complete message in the receive buffer.
void SwarmWire::process(IoLoop& l, Conn& c) {
  std::string blocks;                     // records of this batch: idx, begin, len, status
  std::string reqs;                       // REQUESTs the batch's answers made room for
  bool need = false;
  std::string bad;
  auto flush_blocks = [&] {
    if (!blocks.empty()) {
      push(c.id, kEvBlocks, std::move(blocks));
      blocks.clear();
    }
  };
  uint8_t* const buf = c.rbuf.get();
  while (c.rend - c.rstart >= 4) {
    const uint32_t n = be32(buf + c.rstart);
    if (n > kMaxMsg) {
      bad = "message too large (" + std::to_string(n) + ")";
      break;
    }
    if (c.rend - c.rstart < 4 + (size_t)n) break;
    const uint8_t* m = buf + c.rstart + 4;
    if (n > 0) {
      if (m[0] == kPiece && n >= 9) {
        const uint32_t idx = be32(m + 1), begin = be32(m + 5), len = n - 9;
        bool owned = false;
        const int st = take_from(&c, idx, begin, m + 9, len, &owned, &reqs, &need);
        if (!owned) {                     // an owned piece's blocks are the wire's business
          put32(blocks, idx);
          put32(blocks, begin);
          put32(blocks, len);
          put32(blocks, (uint32_t)st);
        }
      } else if (m[0] == kRequest && n == 13 && c.serving.load() &&
                 servable(be32(m + 1), be32(m + 5), be32(m + 9))) {
        std::lock_guard<std::mutex> g(c.wmu);
        if (c.serve_queued >= kMaxServeQueue) {
          bad = "request flood (" + std::to_string(c.serve_queued) + " blocks queued)";
          serve_floods_.fetch_add(1, std::memory_order_relaxed);
          break;
        }
        c.out.push_back(Conn::Item{std::string((const char*)m + 1, 12), true, 0, 0});
        c.serve_queued++;
      } else {
        if (m[0] == kCancel && n == 13) {   // a block we were going to serve: dropped
          std::lock_guard<std::mutex> g(c.wmu);
          for (auto it = c.out.begin(); it != c.out.end(); ++it) {
            if (it->serve && it->off == 0 && it->fdone == 0 && memcmp(it->data.data(), m + 1, 12) == 0) {
              c.out.erase(it);
              c.serve_queued--;
              serve_cancels_.fetch_add(1, std::memory_order_relaxed);
              break;
            }
          }
        }
        flush_blocks();                   // keep the order of blocks and control messages
        push(c.id, kEvMsg, std::string((const char*)m, n));
      }
    }
    c.rstart += 4 + (size_t)n;
  }
  flush_blocks();
  if (!reqs.empty()) {                    // behind whatever Python queued before
    std::lock_guard<std::mutex> g(c.wmu);
    if (!c.stop) {
      c.out_bytes += reqs.size();
      c.out.push_back(Conn::Item{std::move(reqs), false, 0, 0});
    }
  }
  if (need) push(c.id, kEvNeed, std::string());
  if (!bad.empty()) {
    kill(l, c, bad);
    return;
  }
  flush(l, c);
}

// Send the connection's queue until it is empty or the socket is full (then EPOLLOUT).
void SwarmWire::flush(IoLoop& l, Conn& c) {
  for (;;) {
    Conn::Item* it;
    {
      std::lock_guard<std::mutex> g(c.wmu);
      if (c.out.empty() || c.stop) break;
      it = &c.out.front();                  // (push_back elsewhere keeps it valid)
    }
    int st;
    if (it->serve) {
      st = serve_step(c, *it);
      if (st == 1) {
        std::lock_guard<std::mutex> g(c.wmu);
        c.serve_queued--;
        c.out.pop_front();
        continue;
      }
    } else {
      const ssize_t w = ::send(c.fd, it->data.data() + it->off, it->data.size() - it->off,
                               MSG_DONTWAIT | MSG_NOSIGNAL);
      if (w > 0) {
        it->off += (size_t)w;
        if (it->off == it->data.size()) {
          std::lock_guard<std::mutex> g(c.wmu);
          c.out_bytes -= it->data.size();
          c.out.pop_front();
        }
        continue;
      }
      if (w < 0 && errno == EINTR) continue;
      st = (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) ? 0 : -1;
    }
    if (st == 0) {
      arm_out(l, c, true);
      return;
    }
    kill(l, c, std::string("send: ") + strerror(errno ? errno : EPIPE));
    return;
  }
  arm_out(l, c, false);
}

bool SwarmWire::servable(uint32_t idx, uint32_t begin, uint32_t len) {
  std::lock_guard<std::mutex> g(mu_);
  if (piece_length_ <= 0 || (int64_t)idx * piece_length_ >= total_ || !has(idx)) return false;
  return len > 0 && len <= kMaxServe && (uint64_t)begin + len <= piece_size(idx);
}

// One serve item: the PIECE header, then the block from the storage files (sendfile: page
// cache -> socket), resumable. 1 done, 0 the socket is full, -1 error (errno).
int SwarmWire::serve_step(Conn& c, OutItem& item) {
  const uint8_t* q = (const uint8_t*)item.data.data();
  const uint32_t idx = be32(q), begin = be32(q + 4), len = be32(q + 8);
  while (item.off < 13) {
    std::string hdr;
    put32(hdr, len + 9);
    hdr.push_back((char)kPiece);
    put32(hdr, idx);
    put32(hdr, begin);
    const ssize_t w = ::send(c.fd, hdr.data() + item.off, 13 - item.off,
                             MSG_DONTWAIT | MSG_NOSIGNAL | MSG_MORE);
    if (w > 0) {
      item.off += (size_t)w;
      continue;
    }
    if (w < 0 && errno == EINTR) continue;
    return (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) ? 0 : -1;
  }
  std::vector<std::pair<int, int64_t>> files;
  int64_t off;
  {
    std::lock_guard<std::mutex> g(mu_);
    files = files_;
    off = (int64_t)idx * piece_length_ + begin + item.fdone;
  }
  int64_t fstart = 0;
  for (auto& f : files) {
    const int64_t fend = fstart + f.second;
    while (item.fdone < (int64_t)len && off >= fstart && off < fend) {
      off_t fo = (off_t)(off - fstart);
      const size_t k = (size_t)std::min<int64_t>((int64_t)len - item.fdone, fend - off);
      const ssize_t w = ::sendfile(c.fd, f.first, &fo, k);
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return 0;
      if (w <= 0) {
        if (w == 0) errno = EIO;
        return -1;
      }
      off += w;
      item.fdone += w;
    }
    fstart = fend;
  }
  if (item.fdone < (int64_t)len) {
    errno = EIO;                            // the block runs past the storage files
    return -1;
  }
  c.served.fetch_add(len, std::memory_order_relaxed);
  served_bytes_.fetch_add(len, std::memory_order_relaxed);
  return 1;
}

size_t SwarmWire::send(uint64_t id, std::string data) {
  std::shared_ptr<Conn> c = conn(id);
  if (!c) return 0;
  size_t n;
  {
    std::lock_guard<std::mutex> g(c->wmu);
    if (c->stop || c->dead.load()) return 0;
    c->out_bytes += data.size();
    c->out.push_back(Conn::Item{std::move(data), false, 0, 0});
    n = c->out_bytes;
  }
  kick(*c);
  return n;
}

size_t SwarmWire::pending_out(uint64_t id) {
  std::shared_ptr<Conn> c = conn(id);
  if (!c) return 0;
  std::lock_guard<std::mutex> g(c->wmu);
  return c->out_bytes;
}

uint64_t SwarmWire::conn_rx(uint64_t id) {
  std::shared_ptr<Conn> c = conn(id);
  return c ? c->rx.load(std::memory_order_relaxed) : 0;
}

void SwarmWire::detach(uint64_t id) {
  std::shared_ptr<Conn> c;
  {
    std::lock_guard<std::mutex> g(cmu_);
    auto it = conns_.find(id);
    if (it == conns_.end()) return;
    c = it->second;
    conns_.erase(it);
  }
  {
    std::lock_guard<std::mutex> g(c->wmu);
    c->stop = true;
  }
  ::shutdown(c->fd, SHUT_RDWR);
  IoLoop* l = c->loop;
  {
    std::lock_guard<std::mutex> g(l->mu);
    l->removes.push_back(c);
  }
  l->wake();
  {
    std::unique_lock<std::mutex> lk(lmu_);
    lcv_.wait(lk, [&] { return c->removed; });   // the I/O thread will not touch it again
  }
  ::close(c->fd);
}

SwarmWireStats SwarmWire::stats() {
  std::lock_guard<std::mutex> g(mu_);
  SwarmWireStats s = stats_;
  s.active_pieces = pieces_.size();
  s.rx_bytes = rx_bytes_.load();
  s.recvs = recvs_.load();
  s.served_bytes = served_bytes_.load();
  s.backlog_bytes = backlog_bytes_.load();
  s.serve_floods = serve_floods_.load();
  s.serve_cancels = serve_cancels_.load();
  {
    std::lock_guard<std::mutex> g2(cmu_);
    s.io_threads = loops_.size();
  }
  {
    PiecePool& pp = piece_pool();
    std::lock_guard<std::mutex> g2(pp.mu);
    s.pool_in_use = pp.in_use;
    s.pool_idle = pp.idle_count;
    s.pool_idle_bytes = pp.idle_bytes;
    s.pool_allocs = pp.allocs;
    s.pool_frees = pp.frees;
    s.pool_locks = pp.locks;
  }
  return s;
}

}  // namespace stager
