// Shared declarations of the stager native module (_native).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

typedef struct evp_md_ctx_st EVP_MD_CTX;
typedef struct evp_md_st EVP_MD;
typedef struct ssl_st SSL;
typedef struct ssl_ctx_st SSL_CTX;

namespace stager {

// ---- hashing.cpp -----------------------------------------------------------------------
const EVP_MD* md_for(const std::string& algo);
size_t digest_size(const std::string& algo);
int effective_cpus();
int resolve_threads(int threads, size_t work_items);

class Hasher {
 public:
  explicit Hasher(const std::string& algo);
  ~Hasher();
  Hasher(const Hasher&) = delete;
  Hasher& operator=(const Hasher&) = delete;
  void update(const uint8_t* p, size_t n);
  void update_fd(int fd, int64_t offset, int64_t length);
  std::string digest() const;
  // Digest of everything fed so far, then start over (one EVP final, no context copy).
  std::string finish_and_reset();
  std::unique_ptr<Hasher> copy() const;
  const std::string& algo() const { return algo_; }

 private:
  std::string algo_;
  EVP_MD_CTX* ctx_;
};

std::string digest(const std::string& algo, const uint8_t* p, size_t n);
// CRC32C of S3 flexible checksums (x-amz-checksum-crc32c): continue `crc` over p[0, n).
uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc = 0);
// CRC32C of a file range (pread through an L2-sized buffer).
uint32_t crc32c_fd(int fd, int64_t off, int64_t len);
std::string crc32c_base64(uint32_t crc);
// "avx512-vpclmulqdq" (folding, >= 1 KiB) or "sse4.2-3way": the CRC32C path this CPU runs.
const char* crc32c_impl();
std::string hash_pieces(const std::string& algo, const uint8_t* p, size_t n, size_t piece_len,
                        int threads);

// ---- sha1_mb.cpp (AVX-512 16-lane multi-buffer SHA-1) --------------------------------
bool sha1_mb_supported();
// SHA-1 of n independent messages, 20 bytes each into out (16 lanes per group).
void sha1_mb(const uint8_t* const* msgs, const size_t* lens, size_t n, uint8_t* out);
// Streaming form for 16 messages of EQUAL length: init, absorb whole blocks (lanes whose
// `active` bit is clear are untouched), finish with each lane's last tail_len (< 64) bytes;
// digests of active lanes go to out + 20 * lane.
void sha1x16_init(uint32_t st[5][16]);
void sha1_mb16_blocks(uint32_t state[5][16], const uint8_t* const ptr[16], size_t nblocks,
                      uint16_t active);
void sha1x16_finish(uint32_t st[5][16], const uint8_t* const tails[16], size_t tail_len,
                    uint64_t total_len, uint16_t active, uint8_t* out);

struct Storage {
  struct Entry {
    std::string path;
    int64_t length;
    int64_t offset;
    int fd;
  };
  explicit Storage(const std::vector<std::pair<std::string, int64_t>>& files);
  ~Storage();
  void open_all(bool missing_ok);
  void close_all();
  bool read(int64_t off, int64_t len, uint8_t* buf) const;
  std::vector<Entry> entries;
  int64_t total = 0;
};

std::vector<uint8_t> verify_pieces(const std::vector<std::pair<std::string, int64_t>>& files,
                                   int64_t piece_len, const std::string& hashes,
                                   const std::vector<int64_t>& which, int threads);
std::string hash_storage_pieces(const std::vector<std::pair<std::string, int64_t>>& files,
                                int64_t piece_len, const std::string& algo, int threads);
std::vector<std::string> hash_file_ranges(const std::string& path,
                                          const std::vector<std::pair<int64_t, int64_t>>& ranges,
                                          const std::string& algo, int threads);

// ---- tls.cpp ---------------------------------------------------------------------------
// One client SSL_CTX per trust setting, shared by every connection (and thread) of a transport.
class TlsContext {
 public:
  TlsContext(bool verify, const std::string& ca_file);
  ~TlsContext();
  TlsContext(const TlsContext&) = delete;
  TlsContext& operator=(const TlsContext&) = delete;
  SSL_CTX* ctx() const { return ctx_; }
  bool verify() const { return verify_; }

 private:
  SSL_CTX* ctx_ = nullptr;
  bool verify_;
};
// Client handshake on a connected blocking socket: SNI for DNS names, host name / IP checked
// against the certificate when verifying. Throws with the verification error on failure.
SSL* tls_handshake(TlsContext& ctx, int fd, const std::string& name);
// Message for a failed SSL_read / SSL_write / SSL_connect (drains the thread's error queue).
std::string tls_error(SSL* s, int r, const std::string& what);

// ---- transfer.cpp ----------------------------------------------------------------------
// Parts up to this size are relayed through a pooled buffer and hashed with the multi-buffer
// SHA-1; larger ones take the chunked (L2-sized, single-chain) path.
constexpr int64_t kMaxBufferedPart = (int64_t)64 << 20;

// Pipes of splice transfers (leased per transfer from a process-wide pool): created, created
// smaller than asked (the user's pipe page budget is spent), in use / idle and their capacity.
struct PipeStats {
  uint64_t created, short_pipes;
  size_t in_use, in_use_bytes, idle, idle_bytes;
};
PipeStats pipe_stats();
// Per-phase counters of relay_body_to (process-wide, since start): where a checksummed
// relay's CPU goes next to the plain splice one. Modes: 0 splice (no user-space copy),
// 1 dup (recv(MSG_PEEK) or tee() copy + CRC, splice), 2 copy (recv + send: TLS, no pipe).
// `cpu_ns` is the relaying thread's own CPU (CLOCK_THREAD_CPUTIME_ID around the call).
struct RelayCounters {
  uint64_t relays[4], bytes[4], cpu_ns[4];      // splice, dup, copy, hashed (torrent parts)
  uint64_t splice_in_calls, splice_out_calls;   // socket -> pipe, pipe -> socket (all modes)
  uint64_t dup_calls, dup_bytes;                // recv(MSG_PEEK) / read(tee) copies
  uint64_t crc_ns, crc_bytes;                   // CRC32C over the copied bytes
  uint64_t sha1_ns;                             // host piece SHA-1 inside hashed relays
  uint64_t nt_bytes;                            // hashed parts staged in L2 + streamed (NT)
};
RelayCounters relay_counters();
// Capacity asked for new pipes: the splice pipe, and the tee() duplicate pipe (0 = keep).
void set_pipe_sizes(size_t main, size_t tee);
// Tests: refuse every pipe, as when the budget is spent (transfers fall back to copying).
void set_pipes_refused(bool on);
// How relays that need the bytes in user space (CRC, piece hashing) get them: "peek"
// (recv(MSG_PEEK), one pipe; default) or "tee" (tee() into a second pipe).
void set_relay_dup(const std::string& mode);
std::string relay_dup_mode();

struct RelayPoolStats {
  size_t idle_buffers, idle_bytes, in_use, max_idle;
  uint64_t created;
  size_t in_use_bytes, budget, peak_bytes;   // peak of in_use_bytes + idle_bytes
  uint64_t evicted, over_budget;             // idle buffers unmapped to stay in budget; leases past it
};
// GPU piece hashing of relayed parts (gpu_part_api.h, implemented by _gpuhash): when set,
// relay_body_hashed_mb hands parts of >= min_pieces whole pieces to the GPU instead of the
// host multi-buffer SHA-1 and returns a part id. The part's buffer goes back to the pool as
// soon as its DMA has completed (the hasher's COPIED notification); the digests arrive with
// DONE. Completions are reported through an eventfd (gpu_part_eventfd) and drained with
// gpu_part_poll, or waited for with gpu_part_wait. Part ids are this module's own (never a
// hasher's ticket), so replacing the hasher cannot make two pending parts collide.
void set_gpu_part_hasher(const void* api, int min_pieces);
const void* gpu_part_hasher_current();        // the installed hasher's API (null: none)
// The swarm wire's idle piece buffers page-locked for this hasher API are unlocked and freed
// (peerwire.cpp); set_gpu_part_hasher calls it for the hasher it replaces.
void swarm_piece_pool_forget(const void* api);
// At most this many bytes of idle piece buffers are kept (beyond it they are freed now and on
// release; download.swarm_pool_mb).
void swarm_piece_pool_limit(size_t bytes);
struct GpuPartStats {
  uint64_t submitted, host_fallbacks, refused, pending;
};
GpuPartStats gpu_part_stats();
// Blocks until part `id` is hashed; its digests (throws when the device failed after the DMA).
// A part is consumed once: by gpu_part_wait (which claims it - gpu_part_poll then skips it)
// or by gpu_part_poll (a wait called after the poll collected it throws "already collected").
std::string gpu_part_wait(uint64_t id);
// A part nobody will ask for (the relay failed after queueing it): blocks until its buffer is
// back in the pool, then drops its result when it arrives.
void gpu_part_forget(uint64_t id);
// Readable (eventfd counter) whenever gpu_part_poll has something new.
int gpu_part_eventfd();
struct GpuPartEvent {
  uint64_t id;
  int kind;                 // 1 copied (buffer released), 2 done (digests), 3 failed (error)
  std::string data;         // digests / error message
};
std::vector<GpuPartEvent> gpu_part_poll();
// gpu_part_api.h served by a host thread (copy, then multi-buffer SHA-1, each after
// `delay_s`): the asynchronous relay-hashing path without a HIP device (tests).
class CpuPartHasher {
 public:
  // fail_copy_every / fail_done_every (0 = never): every Nth job's COPIED / DONE wait
  // fails, as a device that dies before / after the DMA out of the part buffer would.
  explicit CpuPartHasher(double delay_s, int fail_copy_every = 0, int fail_done_every = 0);
  ~CpuPartHasher();
  const void* api() const;
  uint64_t registered() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};
// ---- peerwire.cpp: native BitTorrent peer-wire receive path ---------------------------
// One per torrent session. Connections are handed over after the handshake (attach: the fd is
// owned from then on); a reader thread per connection frames messages, copies PIECE payloads
// into the piece being assembled (begin_piece), and queues every other message for Python; a
// writer thread sends what Python queues. Complete pieces are SHA-1'd 16 at a time (sha1_mb),
// written to the storage files (set_storage: the torrent's (fd, length) list in order) and
// reported. Events (poll(), signalled on eventfd()): kEvMsg = one message (id byte +
// payload), kEvBlocks = 16-byte records (piece, begin, length, status: 0 not taken, 1 taken, 2
// taken and the piece is complete) in wire order, coalesced while not polled, kEvClosed =
// reason; kEvPiece (conn 0) = piece index + status byte (1 verified and written, 0 hash
// mismatch, 2 write error + message).
struct WireEvent {
  uint64_t conn;
  int kind;
  std::string data;
};
struct SwarmWireStats {
  uint64_t begun = 0, blocks = 0, block_bytes = 0, blocks_ignored = 0, verified = 0,
           hash_fails = 0, rx_bytes = 0, recvs = 0;
  uint64_t verify_batches = 0, sha_ns = 0, write_ns = 0;   // verifier: batches, time hashing /
                                                            // writing
  uint64_t served_bytes = 0;                                // blocks served with sendfile
  uint64_t assigned = 0, requests = 0;                      // owned pieces, REQUESTs the wire sent
  uint64_t gpu_pieces = 0, gpu_refused = 0, gpu_errors = 0; // pieces SHA-1'd on the GPU hasher
  uint64_t gpu_overflow = 0;        // hashed on the host: max_inflight pieces on the device
  int64_t gpu_latency_ns_sum = 0, gpu_latency_ns_max = 0;   // submission -> digest, device pieces
  int64_t backlog_bytes = 0;        // complete pieces not yet reported
  size_t pool_in_use = 0, pool_idle = 0, pool_idle_bytes = 0;   // process-wide piece buffers
  uint64_t pool_allocs = 0, pool_frees = 0, pool_locks = 0; // since start: buffers made /
                                                            // unmade, page-locked for a hasher
  size_t active_pieces = 0;
  size_t io_threads = 0;            // I/O threads (epoll) serving the connections
  uint64_t serve_floods = 0;        // connections dropped for flooding REQUESTs
  uint64_t serve_cancels = 0;       // queued blocks a CANCEL removed
};
class SwarmWire {
 public:
  // kEvNeed: the connection's native request queue fell below one pipeline (assign more)
  static constexpr int kEvMsg = 1, kEvBlocks = 2, kEvClosed = 3, kEvPiece = 4, kEvNeed = 5;
  // io_threads: epoll threads reading and writing the connections (spread, fewest first)
  explicit SwarmWire(int verify_threads = 2, int io_threads = 4);
  ~SwarmWire();
  void set_storage(int64_t piece_length, int64_t total, const std::string& hashes,
                   const std::vector<std::pair<int, int64_t>>& files);
  void begin_piece(uint32_t idx);
  void drop_piece(uint32_t idx);
  // Owned pieces: a piece assigned to a connection is requested by the wire itself, block by
  // block, keeping `depth` requests in flight on that connection (refilled as blocks arrive,
  // on the reader thread); only its owner may fill it, and its blocks are not reported one by
  // one (the PIECE result is the first Python hears of it). assign returns the connection's
  // queue of blocks still to request; kEvNeed fires once when that queue drops below a
  // pipeline. release (the peer choked us, or closed) and release_piece (endgame) turn owned
  // pieces back into ordinary ones and return their per-block state: 2 received, 1 requested
  // from the owner and not answered yet, 0 neither.
  void set_pipeline(uint32_t depth);
  void set_conn_pipeline(uint64_t conn, uint32_t depth);   // per connection (0: the default)
  size_t assign(uint64_t conn, uint32_t idx);
  size_t todo(uint64_t conn);
  std::vector<std::pair<uint32_t, std::string>> release(uint64_t conn);
  bool release_piece(uint32_t idx, uint64_t* owner, std::string* states);
  double rx_idle(uint64_t conn);                // seconds since the connection last received
  // Serving: pieces we have (storage recheck; natively verified ones are added as they pass)
  // are served to connections Python unchoked, straight from the storage files.
  void set_have(const std::string& bits);
  void set_have_piece(uint32_t idx);
  void set_serving(uint64_t id, bool on);
  // Verify complete pieces on the installed GPU part hasher (gpu_part_api.h, the gfx950
  // PartHasher) instead of sha1_mb: piece buffers come from a pool page-locked for it, each
  // complete piece is submitted at once (the device batches them into sha1_lanes launches),
  // collector threads (one per verifier) take the digests in order and compare, the writer
  // stores. At most max_inflight pieces are on the device at once: the rest, a piece the
  // hasher refuses, or no hasher installed: sha1_mb as before.
  void set_gpu(bool on, int max_inflight = 64);
  // GPU mode, the end of the download: pieces completing from now on are hashed on the host
  // (the last ~100 ms of download would otherwise wait out the device's per-piece latency).
  void set_host_tail(bool on);
  // GPU mode: a piece's time from its submission to its digest on the device (EWMA, seconds;
  // 0 before the first one) - the session sizes the host-hashed tail of the download by it
  double gpu_latency() const { return gpu_lat_ewma_ns_.load() / 1e9; }
  uint64_t rx_total() const { return rx_bytes_.load(std::memory_order_relaxed); }
  // Back-pressure: complete pieces not yet reported (verifying, on the device, waiting for the
  // writer) hold their buffers. backlogged() is true at `bytes` or more (Python then starts no
  // new piece); when half has drained since, NEED arrives on conn 0 (refill every connection).
  void set_backlog_cap(int64_t bytes);
  bool backlogged();
  void attach(int fd, uint64_t id, const std::string& prefix);
  size_t send(uint64_t id, std::string data);   // queued bytes after this one (0: closed)
  size_t pending_out(uint64_t id);
  uint64_t conn_rx(uint64_t id);                // bytes the connection received so far
  void detach(uint64_t id);                     // shut down, off its I/O thread, close the fd
  int eventfd() const { return efd_; }
  std::vector<WireEvent> poll();
  SwarmWireStats stats();
  void close();                                 // every connection, then the verifiers
  int take_block(uint32_t idx, uint32_t begin, const uint8_t* p, uint32_t len);

 private:
  struct Piece;
  struct Conn;
  struct OutItem;
  struct IoLoop;
  uint32_t piece_size(uint32_t idx) const;
  void verify_loop();
  std::string write_piece(const Piece& p);
  void push(uint64_t conn, int kind, std::string data);
  IoLoop* pick_loop();                          // cmu_ held
  void io_loop(IoLoop& l);
  bool commands(IoLoop& l);
  void kill(IoLoop& l, Conn& c, const std::string& reason);
  void arm_out(IoLoop& l, Conn& c, bool on);
  void on_readable(IoLoop& l, Conn& c);
  void process(IoLoop& l, Conn& c);
  void flush(IoLoop& l, Conn& c);
  void kick(Conn& c);
  int serve_step(Conn& c, OutItem& item);
  bool has(uint32_t idx);
  bool servable(uint32_t idx, uint32_t begin, uint32_t len);
  void finish_piece(std::shared_ptr<Piece> p, const uint8_t* dig);   // compare, then store
  void store_loop();                                                  // the writer
  void report(uint32_t idx, int status, const std::string& err);
  void gpu_loop();
  int take_from(Conn* c, uint32_t idx, uint32_t begin, const uint8_t* p, uint32_t len,
                bool* owned, std::string* reqs, bool* need);
  bool pump(Conn& c, std::string* reqs);        // mu_ held
  void queue_out(Conn& c, std::string data);
  std::shared_ptr<Conn> conn(uint64_t id);
  std::string block_states(const Piece& p, const Conn* owner);   // mu_ held

  std::mutex mu_;                               // pieces_, geometry, stats_, request queues
  uint32_t depth_ = 64;
  int64_t piece_length_ = 0, total_ = 0;
  std::string hashes_;
  std::vector<std::pair<int, int64_t>> files_;
  std::unordered_map<uint32_t, std::shared_ptr<Piece>> pieces_;
  std::vector<uint8_t> have_;                   // bitfield (BEP-3 bit order)
  std::atomic<bool> gpu_{false};
  std::atomic<int> gpu_cap_{64}, gpu_inflight_{0};
  std::atomic<bool> host_tail_{false};
  std::atomic<int64_t> backlog_bytes_{0}, backlog_cap_{0};
  std::atomic<bool> backlog_full_{false};
  std::mutex gmu_;
  std::condition_variable gcv_;
  struct GpuJob {
    std::shared_ptr<Piece> piece;
    uint64_t ticket;
    int64_t submit_ns;
  };
  std::deque<GpuJob> gq_;                       // submitted, in order
  std::atomic<int64_t> gpu_lat_ewma_ns_{0};
  bool gstop_ = false;
  std::vector<std::thread> gthreads_;
  std::mutex smu_;
  std::condition_variable scv_;
  std::deque<std::shared_ptr<Piece>> sq_;       // verified pieces waiting for the writer
  bool sstop_ = false;
  std::thread sthread_;
  std::atomic<uint64_t> served_bytes_{0};
  uint64_t epoch_ = 0;
  SwarmWireStats stats_;
  std::atomic<uint64_t> rx_bytes_{0}, recvs_{0};
  std::mutex cmu_;                              // conns_, loops_
  std::unordered_map<uint64_t, std::shared_ptr<Conn>> conns_;
  int io_threads_ = 4;
  std::vector<std::unique_ptr<IoLoop>> loops_;
  std::mutex lmu_;                              // Conn::removed (detach waits for it)
  std::condition_variable lcv_;
  std::atomic<uint64_t> serve_floods_{0}, serve_cancels_{0};
  std::mutex vmu_;
  std::condition_variable vcv_;
  std::deque<std::shared_ptr<Piece>> vq_;
  bool vstop_ = false;
  std::vector<std::thread> verifiers_;
  std::mutex emu_;
  std::deque<WireEvent> events_;
  int efd_ = -1;
};

// Idle part buffers beyond `keep_bytes` are unmapped (returns the bytes freed); max_idle
// bounds the idle list. A budget (bytes, 0 = none) bounds leased + idle buffers: idle ones are
// unmapped first to make room for a new lease; a lease past the budget is counted
// (over_budget) - admission is the caller's job (torrent/stream.py's PartBudget).
size_t relay_pool_trim(size_t keep_bytes = 0);
void relay_pool_set_max_idle(size_t n);
void relay_pool_set_budget(size_t bytes);
void relay_pool_reset_peak();
RelayPoolStats relay_pool_stats();

// Byte counter shared between a transfer running on a worker thread and the asyncio side
// (progress telemetry, stall watchdog, cancellation).
struct Progress {
  std::atomic<int64_t> bytes{0};
  std::atomic<bool> cancelled{false};
};

struct ResponseHead {
  int status = 0;
  std::string reason;
  std::vector<std::pair<std::string, std::string>> headers;  // lower-cased names
  int64_t content_length = -1;
  bool chunked = false;
  bool keep_alive = true;
};

class HttpConn {
 public:
  // `tls` non-null: TLS over the socket (server name = host). Every body path below then
  // moves bytes through user space (SSL_read / SSL_write) instead of splice / sendfile.
  HttpConn(const std::string& host, int port, double connect_timeout_s, double io_timeout_s,
           std::shared_ptr<TlsContext> tls = nullptr);
  ~HttpConn();
  HttpConn(const HttpConn&) = delete;
  HttpConn& operator=(const HttpConn&) = delete;

  // Send `head` (request line + headers + CRLFCRLF) and an optional in-memory body.
  void send_request(const std::string& head, const uint8_t* body, size_t body_len);
  // Send `head` and then `len` bytes of file `fd` from `off` with sendfile(2).
  void send_request_fd(const std::string& head, int fd, int64_t off, int64_t len,
                       Progress* prog);
  ResponseHead read_head();
  // This socket is connected to a forward proxy: open a CONNECT tunnel to "host:port"
  // (`auth` = Proxy-Authorization value or ""). Throws unless the proxy answers 200.
  void connect_tunnel(const std::string& target, const std::string& auth);
  // TLS handshake on the (possibly tunnelled) socket; `name` is the server's host name.
  void start_tls(std::shared_ptr<TlsContext> tls, const std::string& name);
  // Body into memory (bounded by max_bytes).
  std::string read_body(const ResponseHead& h, int64_t max_bytes);
  // Body into fd at `offset` (splice for Content-Length bodies, read/pwrite for chunked).
  int64_t read_body_to_fd(const ResponseHead& h, int fd, int64_t offset, int64_t max_bytes,
                          Progress* prog);
  // Drain and discard a body (keeps the connection reusable).
  void discard_body(const ResponseHead& h);
  // Move exactly `n` body bytes of the response being read on *this to `dst`'s socket
  // (bytes already buffered first, then socket -> pipe -> socket with splice).
  // `crc` non-null: the bytes are CRC32C'd on the way (S3 trailing checksum of an aws-chunked
  // PUT): each spliced chunk is tee()d into a second pipe whose copy is read and CRC'd, the
  // original pages still go to `dst` by splice (one user-space copy instead of recv + send).
  int64_t relay_body_to(HttpConn& dst, int64_t n, Progress* prog, uint32_t* crc = nullptr);
  // Same relay, but through a user-space chunk that is also hashed: body bytes [skip,
  // skip + full_len) are SHA-1'd as consecutive pieces of `piece_len` (the last may be
  // short) into `digests`; bytes before `skip` go to `head`, bytes after to `tail` (the
  // fragments of pieces that straddle the body's ends). One pass, L2-resident chunks.
  // `gpu_ticket` non-null: the part may go to the GPU hasher; then *gpu_ticket != 0 and
  // `digests` stays empty (gpu_part_wait).
  int64_t relay_body_hashed(HttpConn& dst, int64_t n, int64_t skip, int64_t full_len,
                            int64_t piece_len, Progress* prog, std::string* digests,
                            std::string* head, std::string* tail, uint32_t* crc = nullptr,
                            uint64_t* gpu_ticket = nullptr);
  // relay_body_hashed for parts of >= 8 pieces: buffer the part, then multi-buffer SHA-1.
  int64_t relay_body_hashed_mb(HttpConn& dst, int64_t n, int64_t skip, int64_t full_len,
                               int64_t piece_len, Progress* prog, std::string* digests,
                               std::string* head, std::string* tail, uint32_t* crc = nullptr,
                               uint64_t* gpu_ticket = nullptr);
  void send_raw(const std::string& s) { send_all((const uint8_t*)s.data(), s.size()); }
  int fd() const { return fd_; }
  void mark_unusable() { reusable_ = false; }
  void close();
  // Unblock a transfer running on another thread (cancelled job, shutdown): shut the
  // socket down in both directions; the owner's recv/splice/send then fails fast and
  // the owner closes the fd as usual.
  void abort();
  bool is_open() const { return fd_ >= 0; }
  bool is_tls() const { return ssl_ != nullptr; }
  bool reusable() const { return fd_ >= 0 && reusable_; }
  const std::string& host() const { return host_; }
  int port() const { return port_; }

 private:
  size_t recv_some(uint8_t* p, size_t n);
  void send_all(const uint8_t* p, size_t n);
  std::string read_line();
  int64_t take_buffered(uint8_t* p, int64_t n);
  // Relay through a user-space buffer (either side is TLS).
  int64_t relay_copy(HttpConn& dst, int64_t n, int64_t moved, Progress* prog,
                     uint32_t* crc = nullptr);
  // Plain sockets, bytes needed in user space (CRC, piece hashing): splice socket -> pipe ->
  // socket and read a tee()d duplicate of every chunk into memory the caller names
  // (room(len) -> where up to len bytes go, may lower len; got(p, k) after each read).
  template <class Room, class Got>
  int64_t relay_tee(HttpConn& dst, int64_t n, int64_t moved, Progress* prog, Room&& room,
                    Got&& got);
  // The same contract with recv(MSG_PEEK) into `room` and a splice of exactly the peeked
  // bytes: one copy like tee, one pipe instead of two (csrc/relaybench.cpp at 8 relay
  // threads: 38.7 vs 29.9 GB/s on one MI355X box, 37.5 vs 38.4 on another - the copy costs
  // the same; the pipe is what peek saves).
  template <class Room, class Got>
  int64_t relay_peek(HttpConn& dst, int64_t n, int64_t moved, Progress* prog, Room&& room,
                     Got&& got);
  // relay_peek, or relay_tee with STAGER_RELAY_DUP=tee
  template <class Room, class Got>
  int64_t relay_dup(HttpConn& dst, int64_t n, int64_t moved, Progress* prog, Room&& room,
                    Got&& got);
  std::string host_;
  int port_;
  int fd_ = -1;
  SSL* ssl_ = nullptr;
  std::shared_ptr<TlsContext> tls_;  // keeps the SSL_CTX alive as long as ssl_
  bool reusable_ = true;
  std::vector<uint8_t> rbuf_;
  size_t rpos_ = 0, rend_ = 0;
};

}  // namespace stager
