// Native HTTP/1.1 transport for the staging hot loops (SURVEY.md §3 "hot loops"):
//   (1) network -> disk: response bodies are spliced socket -> pipe -> file, so the payload
//       never crosses into user space (the reference pipes `request` into a write stream,
//       lib/download.js:159-160).
//   (2) disk -> network: request bodies go file -> socket with sendfile(2) (the reference's
//       minio-js fPutObject reads the file into JS buffers, lib/upload.js:45).
// The Python side owns protocol logic (URLs, SigV4, retries); this layer owns bytes. Every
// call blocks its calling thread and is invoked with the GIL released.
#include "native.h"
#include "gpu_part_api.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <thread>
#include <arpa/inet.h>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <mutex>
#include <new>
#include <stdexcept>
#include <sys/mman.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>
#include <unordered_map>
#include <immintrin.h>
#include <map>
#include <sys/eventfd.h>

#include <openssl/err.h>
#include <openssl/ssl.h>

namespace stager {

namespace {

struct IoError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

std::string errstr(const char* what) { return std::string(what) + ": " + strerror(errno); }

// ---- pipes for splice transfers ----------------------------------------------------------
// Leased per transfer from a process-wide pool instead of living on every connection: an
// unprivileged user's pipes share one page budget (fs.pipe-user-pages-soft, 16384 pages =
// 64 MiB by default, counted by capacity, not by bytes held). Past it F_SETPIPE_SZ is refused
// and new pipes get two pages, and 1 MiB pipes kept on every pooled connection - idle ones
// included, in the workers and in the S3 peer alike - ran a busy 16-relay worker into it.
// Now only running transfers hold pipes (plus a few idle ones for reuse).
std::atomic<size_t> g_pipe_main{size_t(1) << 20}, g_pipe_tee{size_t(1) << 20};

// ---- relay counters (RelayCounters) ---------------------------------------------------------
// The hot loops bump a thread_local tally (no shared cache line per syscall); relay_body_to
// folds it into the process-wide atomics once per relay.
struct RelayTally {
  uint64_t splice_in = 0, splice_out = 0, dup_calls = 0, dup_bytes = 0, crc_ns = 0, crc_bytes = 0;
  uint64_t sha1_ns = 0;   // host piece SHA-1 inside hashed relays
};
thread_local RelayTally t_tally;
// modes: 0 splice, 1 dup (peek / tee copy + CRC), 2 copy, 3 hashed (piece-hashed torrent part)
struct {
  std::atomic<uint64_t> relays[4], bytes[4], cpu_ns[4];
  std::atomic<uint64_t> splice_in{0}, splice_out{0}, dup_calls{0}, dup_bytes{0}, crc_ns{0},
      crc_bytes{0}, sha1_ns{0}, nt_bytes{0};
} g_rc;

uint64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// Scope of one relay_body_to: thread CPU and the tally's growth go to mode `mode`.
struct RelayScope {
  int mode = 0;
  int64_t* moved;
  uint64_t cpu0 = thread_cpu_ns();
  RelayTally t0 = t_tally;
  explicit RelayScope(int64_t* m) : moved(m) {}
  ~RelayScope() {
    const RelayTally& t = t_tally;
    g_rc.relays[mode].fetch_add(1, std::memory_order_relaxed);
    g_rc.bytes[mode].fetch_add((uint64_t)std::max<int64_t>(0, *moved), std::memory_order_relaxed);
    g_rc.cpu_ns[mode].fetch_add(thread_cpu_ns() - cpu0, std::memory_order_relaxed);
    g_rc.splice_in.fetch_add(t.splice_in - t0.splice_in, std::memory_order_relaxed);
    g_rc.splice_out.fetch_add(t.splice_out - t0.splice_out, std::memory_order_relaxed);
    g_rc.dup_calls.fetch_add(t.dup_calls - t0.dup_calls, std::memory_order_relaxed);
    g_rc.dup_bytes.fetch_add(t.dup_bytes - t0.dup_bytes, std::memory_order_relaxed);
    g_rc.crc_ns.fetch_add(t.crc_ns - t0.crc_ns, std::memory_order_relaxed);
    g_rc.crc_bytes.fetch_add(t.crc_bytes - t0.crc_bytes, std::memory_order_relaxed);
    g_rc.sha1_ns.fetch_add(t.sha1_ns - t0.sha1_ns, std::memory_order_relaxed);
  }
};
std::atomic<uint64_t> g_pipes_created{0}, g_pipes_short{0};
std::atomic<bool> g_pipes_refused{false};   // tests: behave as if the budget were spent

struct Pipe {
  int r = -1, w = -1;
  size_t cap = 0;
};

class PipePool {
 public:
  // A pipe of `want` bytes, or the largest power-of-two step down to 64 KiB the budget still
  // allows; IoError when not even that (the caller copies through user space instead: a
  // two-page pipe would cost a pair of syscalls per 8 KiB).
  Pipe acquire(size_t want) {
    {
      std::lock_guard<std::mutex> g(mu_);
      // an idle pipe of exactly this size, else any large enough (or any, once short)
      size_t pick = idle_.size();
      for (size_t i = idle_.size(); i-- > 0 && !g_pipes_refused.load();) {
        if (idle_[i].cap == want) {
          pick = i;
          break;
        }
        if (pick == idle_.size() && (idle_[i].cap >= want || short_seen_)) pick = i;
      }
      if (pick < idle_.size()) {
        Pipe p = idle_[pick];
        idle_.erase(idle_.begin() + (ptrdiff_t)pick);
        ++in_use_;
        in_use_bytes_ += p.cap;
        return p;
      }
    }
    if (g_pipes_refused.load()) throw IoError("pipe page budget exhausted (test)");
    int fds[2];
    if (pipe2(fds, O_CLOEXEC) != 0) throw IoError(errstr("pipe2"));
    Pipe p{fds[0], fds[1], 0};
    for (size_t sz = want; sz >= kMinPipe; sz >>= 1)
      if (fcntl(p.w, F_SETPIPE_SZ, (int)sz) >= 0) break;
    int got = fcntl(p.w, F_GETPIPE_SZ);
    p.cap = got > 0 ? (size_t)got : 4096;
    g_pipes_created++;
    std::lock_guard<std::mutex> g(mu_);
    if (p.cap < want) {
      g_pipes_short++;
      short_seen_ = true;      // the budget is spent: take what an idle pipe has from now on
    }
    if (p.cap < kMinPipe) {
      ::close(p.r);
      ::close(p.w);
      throw IoError("pipe page budget exhausted (fs.pipe-user-pages-soft)");
    }
    ++in_use_;
    in_use_bytes_ += p.cap;
    return p;
  }
  // `clean`: the transfer drained the pipe (an aborted one may leave bytes: closed instead)
  void release(Pipe p, bool clean) {
    {
      std::lock_guard<std::mutex> g(mu_);
      --in_use_;
      in_use_bytes_ -= p.cap;
      if (clean && idle_.size() < kMaxIdle) {
        idle_.push_back(p);
        return;
      }
    }
    ::close(p.r);
    ::close(p.w);
  }
  // Close the idle pipes (their capacity was asked for under other settings).
  void drop_idle() {
    std::vector<Pipe> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      drop.swap(idle_);
      short_seen_ = false;
    }
    for (auto& p : drop) {
      ::close(p.r);
      ::close(p.w);
    }
  }
  PipeStats stats() {
    std::lock_guard<std::mutex> g(mu_);
    size_t idle_bytes = 0;
    for (auto& p : idle_) idle_bytes += p.cap;
    return PipeStats{g_pipes_created.load(), g_pipes_short.load(), in_use_, in_use_bytes_,
                     idle_.size(), idle_bytes};
  }

 private:
  static constexpr size_t kMaxIdle = 32;   // a tee()d relay holds two: 16 relays in flight
  static constexpr size_t kMinPipe = size_t(64) << 10;
  std::mutex mu_;
  std::vector<Pipe> idle_;
  size_t in_use_ = 0, in_use_bytes_ = 0;
  bool short_seen_ = false;
};

PipePool& pipe_pool() {
  static PipePool* p = new PipePool();   // never destroyed: transfer threads may outlive exit
  return *p;
}

struct PipeLease {
  Pipe p;
  bool clean = false;
  explicit PipeLease(size_t want) : p(pipe_pool().acquire(want)) {}
  ~PipeLease() { pipe_pool().release(p, clean); }
  PipeLease(const PipeLease&) = delete;
  PipeLease& operator=(const PipeLease&) = delete;
};

void set_timeouts(int fd, double s) {
  if (s <= 0) return;
  timeval tv;
  tv.tv_sec = (time_t)s;
  tv.tv_usec = (suseconds_t)((s - (double)tv.tv_sec) * 1e6);
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
}

std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t");
  size_t b = s.find_last_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  return s.substr(a, b - a + 1);
}

// Size line of a chunked body ("1a2b[;ext]\r\n"): hex digits only, no sign, no overflow.
int64_t chunk_size(const std::string& line) {
  int64_t n = 0;
  size_t i = 0;
  for (; i < line.size() && isxdigit((unsigned char)line[i]); ++i) {
    if (n > ((int64_t)1 << 58)) throw IoError("chunk size too large");
    const char c = (char)tolower((unsigned char)line[i]);
    n = n * 16 + (c <= '9' ? c - '0' : c - 'a' + 10);
  }
  if (i == 0) throw IoError("malformed chunk size line");
  return n;
}

// Content-Length value: decimal digits only (a list of identical values is tolerated, as RFC
// 9110 allows); anything else - sign, hex, overflow, conflicting values - is an error rather
// than a guess at the body's end.
int64_t content_length(const std::string& v) {
  int64_t out = -1;
  size_t i = 0;
  while (i <= v.size()) {
    size_t j = v.find(',', i);
    if (j == std::string::npos) j = v.size();
    std::string t = trim(v.substr(i, j - i));
    if (t.empty() || t.size() > 18 || t.find_first_not_of("0123456789") != std::string::npos)
      throw IoError("malformed Content-Length: " + v.substr(0, 64));
    const int64_t n = std::stoll(t);
    if (out >= 0 && n != out) throw IoError("conflicting Content-Length values");
    out = n;
    i = j + 1;
  }
  return out;
}

// A response head (or chunked trailer) larger than this is refused instead of buffered.
constexpr size_t kMaxHeadBytes = 256 * 1024;
constexpr size_t kMaxHeadLines = 1024;

}  // namespace

HttpConn::HttpConn(const std::string& host, int port, double connect_timeout_s,
                   double io_timeout_s, std::shared_ptr<TlsContext> tls)
    : host_(host), port_(port), rbuf_(64 * 1024) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  std::string ps = std::to_string(port);
  int rc = getaddrinfo(host.c_str(), ps.c_str(), &hints, &res);
  if (rc != 0) throw IoError("getaddrinfo(" + host + "): " + gai_strerror(rc));
  std::string last = "connect failed";
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    int fd = socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC | SOCK_NONBLOCK, ai->ai_protocol);
    if (fd < 0) continue;
    int r = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (r < 0 && errno == EINPROGRESS) {
      pollfd p{fd, POLLOUT, 0};
      int to = connect_timeout_s > 0 ? (int)(connect_timeout_s * 1000) : -1;
      int pr = poll(&p, 1, to);
      int soerr = 0;
      socklen_t sl = sizeof(soerr);
      if (pr == 1) getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl);
      if (pr != 1 || soerr != 0) {
        last = pr == 0 ? "connect timeout" : std::string("connect: ") + strerror(soerr ? soerr : errno);
        ::close(fd);
        continue;
      }
    } else if (r < 0) {
      last = errstr("connect");
      ::close(fd);
      continue;
    }
    int fl = fcntl(fd, F_GETFL);
    fcntl(fd, F_SETFL, fl & ~O_NONBLOCK);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int big = 4 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
    set_timeouts(fd, io_timeout_s);
    fd_ = fd;
    break;
  }
  freeaddrinfo(res);
  if (fd_ < 0) throw IoError(last + " (" + host + ":" + ps + ")");
  if (tls) {
    try {
      start_tls(std::move(tls), host);
    } catch (...) {
      close();  // the destructor does not run for a throwing constructor
      throw;
    }
  }
}

void HttpConn::start_tls(std::shared_ptr<TlsContext> tls, const std::string& name) {
  if (fd_ < 0) throw IoError("connection closed");
  if (ssl_) throw IoError("TLS already started");
  if (rpos_ != rend_) throw IoError("unread bytes before the TLS handshake");
  try {
    ssl_ = tls_handshake(*tls, fd_, name);
  } catch (const std::exception& e) {
    reusable_ = false;
    throw IoError(e.what());
  }
  tls_ = std::move(tls);
  // Coalesce outgoing records: SSL_write emits one 16 KiB record per socket write; a buffer
  // BIO in front of the socket turns them into 256 KiB sends, flushed by send_all. (An A/B on
  // the build box measured it CPU-neutral for relays: one memcpy traded for 15 sends.)
  BIO* sock = SSL_get_wbio(ssl_);
  BIO* buf = BIO_new(BIO_f_buffer());
  if (buf && BIO_set_write_buffer_size(buf, 256 * 1024) == 1) {
    BIO_up_ref(sock);  // the chain holds its own reference; SSL drops the old wbio's
    SSL_set0_wbio(ssl_, BIO_push(buf, sock));
  } else if (buf) {
    BIO_free(buf);
  }
}

void HttpConn::connect_tunnel(const std::string& target, const std::string& auth) {
  std::string req = "CONNECT " + target + " HTTP/1.1\r\nHost: " + target + "\r\n";
  if (!auth.empty()) req += "Proxy-Authorization: " + auth + "\r\n";
  req += "\r\n";
  send_all((const uint8_t*)req.data(), req.size());
  ResponseHead h = read_head();
  if (h.status != 200) {
    reusable_ = false;
    throw IoError("proxy CONNECT " + target + ": HTTP " + std::to_string(h.status) + " " +
                  h.reason);
  }
  // A 2xx to CONNECT has no body: the socket is the tunnel from here on (read_head judged
  // it by HTTP framing rules, which do not apply).
  reusable_ = true;
}

HttpConn::~HttpConn() { close(); }

void HttpConn::close() {
  if (ssl_) {
    SSL_free(ssl_);  // no close_notify: the socket may be dead or mid-body
    ssl_ = nullptr;
  }
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

void HttpConn::abort() {
  reusable_ = false;
  const int fd = fd_;
  if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
}

void HttpConn::send_all(const uint8_t* p, size_t n) {
  if (ssl_) {
    while (n) {
      ERR_clear_error();
      int w = SSL_write(ssl_, p, (int)std::min<size_t>(n, (size_t)1 << 30));
      if (w <= 0) {
        const int e = SSL_get_error(ssl_, w);
        if ((e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_WANT_READ) && errno == EINTR) continue;
        reusable_ = false;
        throw IoError(tls_error(ssl_, w, "send"));
      }
      p += w;
      n -= (size_t)w;
    }
    while (BIO_flush(SSL_get_wbio(ssl_)) <= 0) {
      if (BIO_should_retry(SSL_get_wbio(ssl_)) && errno == EINTR) continue;
      reusable_ = false;
      throw IoError(errno == EAGAIN ? std::string("send timeout") : errstr("send"));
    }
    return;
  }
  while (n) {
    ssize_t w = ::send(fd_, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      reusable_ = false;
      throw IoError(errstr("send"));
    }
    p += w;
    n -= (size_t)w;
  }
}

size_t HttpConn::recv_some(uint8_t* p, size_t n) {
  while (ssl_) {
    ERR_clear_error();
    int r = SSL_read(ssl_, p, (int)std::min<size_t>(n, (size_t)1 << 30));
    if (r > 0) {
      // SSL_read returns one record (<= 16 KiB); take whatever else is already buffered
      // (read-ahead) so callers move 100s of KiB per call, not one record.
      size_t got = (size_t)r;
      while (got < n && SSL_has_pending(ssl_)) {
        int k = SSL_read(ssl_, p + got, (int)std::min<size_t>(n - got, (size_t)1 << 30));
        if (k <= 0) {
          ERR_clear_error();  // reported by the next call, after these bytes are consumed
          break;
        }
        got += (size_t)k;
      }
      return got;
    }
    const int e = SSL_get_error(ssl_, r);
    if (e == SSL_ERROR_ZERO_RETURN) return 0;  // close_notify, or EOF (IGNORE_UNEXPECTED_EOF)
    if ((e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) && errno == EINTR) continue;
    reusable_ = false;
    if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) throw IoError("recv timeout");
    throw IoError(tls_error(ssl_, r, "recv"));
  }
  for (;;) {
    ssize_t r = ::recv(fd_, p, n, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      reusable_ = false;
      if (errno == EAGAIN || errno == EWOULDBLOCK) throw IoError("recv timeout");
      throw IoError(errstr("recv"));
    }
    return (size_t)r;
  }
}

void HttpConn::send_request(const std::string& head, const uint8_t* body, size_t body_len) {
  if (fd_ < 0) throw IoError("connection closed");
  if (body_len && body_len <= 64 * 1024) {
    std::string all = head;
    all.append((const char*)body, body_len);
    send_all((const uint8_t*)all.data(), all.size());
    return;
  }
  send_all((const uint8_t*)head.data(), head.size());
  if (body_len) send_all(body, body_len);
}

void HttpConn::send_request_fd(const std::string& head, int fd, int64_t off, int64_t len,
                               Progress* prog) {
  if (fd_ < 0) throw IoError("connection closed");
  int cork = 1;
  setsockopt(fd_, IPPROTO_TCP, TCP_CORK, &cork, sizeof(cork));
  send_all((const uint8_t*)head.data(), head.size());
  off_t o = (off_t)off;
  int64_t left = len;
  if (ssl_) {  // no sendfile through TLS: pread L2-sized chunks and encrypt them
    thread_local std::vector<uint8_t> buf(256 * 1024);
    while (left > 0) {
      if (prog && prog->cancelled.load(std::memory_order_relaxed)) {
        reusable_ = false;
        throw IoError("cancelled");
      }
      ssize_t k = ::pread(fd, buf.data(), (size_t)std::min<int64_t>(left, (int64_t)buf.size()), o);
      if (k < 0) {
        if (errno == EINTR) continue;
        reusable_ = false;
        throw IoError(errstr("pread"));
      }
      if (k == 0) {
        reusable_ = false;
        throw IoError("pread: source file shorter than declared length");
      }
      send_all(buf.data(), (size_t)k);
      o += k;
      left -= k;
      if (prog) prog->bytes.fetch_add(k, std::memory_order_relaxed);
    }
  }
  while (left > 0) {
    if (prog && prog->cancelled.load(std::memory_order_relaxed)) {
      reusable_ = false;
      throw IoError("cancelled");
    }
    size_t chunk = (size_t)std::min<int64_t>(left, 8 << 20);
    ssize_t w = ::sendfile(fd_, fd, &o, chunk);
    if (w < 0) {
      if (errno == EINTR) continue;
      reusable_ = false;
      throw IoError(errstr("sendfile"));
    }
    if (w == 0) {
      reusable_ = false;
      throw IoError("sendfile: source file shorter than declared length");
    }
    left -= w;
    if (prog) prog->bytes.fetch_add(w, std::memory_order_relaxed);
  }
  cork = 0;
  setsockopt(fd_, IPPROTO_TCP, TCP_CORK, &cork, sizeof(cork));
}

std::string HttpConn::read_line() {
  std::string line;
  for (;;) {
    while (rpos_ < rend_) {
      char c = (char)rbuf_[rpos_++];
      line.push_back(c);
      if (c == '\n') return line;
      if (line.size() > 64 * 1024) throw IoError("header line too long");
    }
    rpos_ = rend_ = 0;
    size_t r = recv_some(rbuf_.data(), rbuf_.size());
    if (r == 0) {
      reusable_ = false;
      if (line.empty()) throw IoError("connection closed by peer");
      return line;
    }
    rend_ = r;
  }
}

ResponseHead HttpConn::read_head() {
  ResponseHead h;
  std::string status;
  do {
    status = read_line();
  } while (status == "\r\n");  // tolerate stray CRLF
  // HTTP/1.1 200 OK
  if (status.compare(0, 5, "HTTP/") != 0) {
    reusable_ = false;
    throw IoError("malformed status line: " + trim(status));
  }
  // "HTTP/x.y NNN reason": exactly three digits, 100 - 599
  const size_t sp = status.find(' ');
  const std::string code = sp == std::string::npos ? "" : status.substr(sp + 1, 3);
  if (code.size() != 3 || code.find_first_not_of("0123456789") != std::string::npos ||
      (status.size() > sp + 4 && !isspace((unsigned char)status[sp + 4])) || code < "100" ||
      code > "599") {
    reusable_ = false;
    throw IoError("malformed status line: " + trim(status).substr(0, 128));
  }
  h.status = std::stoi(code);
  size_t sp2 = status.find(' ', sp + 1);
  h.reason = sp2 == std::string::npos ? "" : trim(status.substr(sp2 + 1));
  bool http10 = status.compare(0, 8, "HTTP/1.0") == 0;
  h.keep_alive = !http10;
  size_t head_bytes = status.size();
  for (;;) {
    std::string line = read_line();
    if (line == "\r\n" || line == "\n" || line.empty()) break;
    head_bytes += line.size();
    if (head_bytes > kMaxHeadBytes || h.headers.size() >= kMaxHeadLines) {
      reusable_ = false;
      throw IoError("response head too large");
    }
    size_t c = line.find(':');
    if (c == std::string::npos) continue;
    std::string k = lower(trim(line.substr(0, c)));
    std::string v = trim(line.substr(c + 1));
    if (k == "content-length") {
      int64_t n;
      try {
        n = content_length(v);
      } catch (...) {
        reusable_ = false;
        throw;
      }
      if (h.content_length >= 0 && n != h.content_length) {
        reusable_ = false;
        throw IoError("conflicting Content-Length values");
      }
      h.content_length = n;
    }
    if (k == "transfer-encoding" && lower(v).find("chunked") != std::string::npos) h.chunked = true;
    if (k == "connection") {
      std::string lv = lower(v);
      if (lv.find("close") != std::string::npos) h.keep_alive = false;
      if (lv.find("keep-alive") != std::string::npos) h.keep_alive = true;
    }
    h.headers.emplace_back(k, v);
  }
  if (!h.keep_alive) reusable_ = false;
  if (h.content_length < 0 && !h.chunked && h.status != 204 && h.status != 304) {
    // Body delimited by connection close.
    reusable_ = false;
  }
  return h;
}

int64_t HttpConn::take_buffered(uint8_t* p, int64_t n) {
  int64_t k = std::min<int64_t>(n, (int64_t)(rend_ - rpos_));
  if (k > 0) {
    memcpy(p, rbuf_.data() + rpos_, (size_t)k);
    rpos_ += (size_t)k;
  }
  return k;
}

std::string HttpConn::read_body(const ResponseHead& h, int64_t max_bytes) {
  std::string out;
  auto append = [&](int64_t n, bool until_close) {
    int64_t got = 0;
    std::vector<uint8_t> tmp(64 * 1024);
    while (until_close || got < n) {
      int64_t want = until_close ? (int64_t)tmp.size() : std::min<int64_t>(n - got, (int64_t)tmp.size());
      int64_t k = take_buffered(tmp.data(), want);
      if (k == 0) {
        size_t r = recv_some(tmp.data(), (size_t)want);
        if (r == 0) {
          if (until_close) break;
          reusable_ = false;
          throw IoError("connection closed mid-body");
        }
        k = (int64_t)r;
      }
      if ((int64_t)out.size() + k > max_bytes) {
        reusable_ = false;
        throw IoError("response body exceeds limit");
      }
      out.append((const char*)tmp.data(), (size_t)k);
      got += k;
    }
  };
  if (h.chunked) {
    for (;;) {
      std::string line = read_line();
      int64_t n = chunk_size(line);
      if (n == 0) {
        size_t trailer = 0;
        while (true) {
          std::string t = read_line();
          if (t == "\r\n" || t.empty()) break;
          if ((trailer += t.size()) > kMaxHeadBytes) throw IoError("chunked trailer too large");
        }
        break;
      }
      append(n, false);
      read_line();
    }
  } else if (h.content_length >= 0) {
    append(h.content_length, false);
  } else if (h.status != 204 && h.status != 304) {
    append(0, true);
  }
  return out;
}

int64_t HttpConn::read_body_to_fd(const ResponseHead& h, int fd, int64_t offset,
                                  int64_t max_bytes, Progress* prog) {
  int64_t written = 0;
  auto check_cancel = [&] {
    if (prog && prog->cancelled.load(std::memory_order_relaxed)) {
      reusable_ = false;
      throw IoError("cancelled");
    }
  };
  auto pwrite_all = [&](const uint8_t* p, int64_t n) {
    while (n > 0) {
      ssize_t w = ::pwrite(fd, p, (size_t)n, offset + written);
      if (w < 0) {
        if (errno == EINTR) continue;
        reusable_ = false;
        throw IoError(errstr("pwrite"));
      }
      p += w;
      n -= w;
      written += w;
      if (prog) prog->bytes.fetch_add(w, std::memory_order_relaxed);
    }
  };
  // Copy exactly n bytes (or until EOF when n < 0) from the socket into fd.
  auto copy_n = [&](int64_t n) {
    if (written + std::max<int64_t>(n, 0) > max_bytes) {
      reusable_ = false;
      throw IoError("response body exceeds limit");
    }
    // 1) bytes already buffered after the header.
    if (rpos_ < rend_) {
      int64_t k = n < 0 ? (int64_t)(rend_ - rpos_) : std::min<int64_t>(n, (int64_t)(rend_ - rpos_));
      pwrite_all(rbuf_.data() + rpos_, k);
      rpos_ += (size_t)k;
      if (n >= 0) n -= k;
    }
    if (n == 0) return;
    // 2) zero-copy: socket -> pipe -> file (plain sockets only: TLS bytes need decrypting).
    std::unique_ptr<PipeLease> pl;
    if (!ssl_) {
      try {
        pl.reset(new PipeLease(g_pipe_main.load()));
      } catch (const IoError&) {
      }
    }
    if (pl) {
      const int pr = pl->p.r, pw = pl->p.w;
      const size_t psz = pl->p.cap;
      while (n != 0) {
        check_cancel();
        size_t want = n < 0 ? psz : (size_t)std::min<int64_t>(n, (int64_t)psz);
        ssize_t in = ::splice(fd_, nullptr, pw, nullptr, want, SPLICE_F_MOVE | SPLICE_F_MORE);
        if (in < 0) {
          if (errno == EINTR) continue;
          if (errno == EINVAL) break;  // fs does not support splice: fall back below
          reusable_ = false;
          if (errno == EAGAIN) throw IoError("recv timeout");
          throw IoError(errstr("splice(sock)"));
        }
        if (in == 0) {
          if (n < 0) return;
          reusable_ = false;
          throw IoError("connection closed mid-body");
        }
        ssize_t left = in;
        while (left > 0) {
          loff_t o = offset + written;
          ssize_t out = ::splice(pr, nullptr, fd, &o, (size_t)left, SPLICE_F_MOVE);
          if (out < 0) {
            if (errno == EINTR) continue;
            reusable_ = false;
            throw IoError(errstr("splice(file)"));
          }
          if (out == 0) {                // nothing taken: a retry would spin
            reusable_ = false;
            throw IoError("splice(file) made no progress");
          }
          left -= out;
          written += out;
          if (prog) prog->bytes.fetch_add(out, std::memory_order_relaxed);
        }
        if (n > 0) n -= in;
        if (written > max_bytes) {
          reusable_ = false;
          throw IoError("response body exceeds limit");
        }
      }
      pl->clean = true;        // every spliced byte went on to the file
      if (n == 0) return;
    }
    // 3) fallback: recv + pwrite.
    std::vector<uint8_t> tmp(1 << 20);
    while (n != 0) {
      check_cancel();
      size_t want = n < 0 ? tmp.size() : (size_t)std::min<int64_t>(n, (int64_t)tmp.size());
      size_t r = recv_some(tmp.data(), want);
      if (r == 0) {
        if (n < 0) return;
        reusable_ = false;
        throw IoError("connection closed mid-body");
      }
      pwrite_all(tmp.data(), (int64_t)r);
      if (n > 0) n -= (int64_t)r;
    }
  };
  if (h.chunked) {
    for (;;) {
      std::string line = read_line();
      int64_t n = chunk_size(line);
      if (n == 0) {
        size_t trailer = 0;
        while (true) {
          std::string t = read_line();
          if (t == "\r\n" || t.empty()) break;
          if ((trailer += t.size()) > kMaxHeadBytes) throw IoError("chunked trailer too large");
        }
        break;
      }
      copy_n(n);
      read_line();
    }
  } else if (h.content_length >= 0) {
    copy_n(h.content_length);
  } else {
    copy_n(-1);
    reusable_ = false;
  }
  return written;
}

// STAGER_RELAY_TEE=0: user-space relays recv + send instead (A/B of the tee path).
static bool relay_tee_on() {
  static const bool on = [] {
    const char* e = getenv("STAGER_RELAY_TEE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// CRC staging, L2-sized: relaybench peekcrc at 8 threads, 64 / 128 / 256 / 512 / 1024 KiB:
// 36.3 / 36.7 / 37.5 / 39.4 / 38.1 GB/s (profiles/archive/r4/peekbuf/); STAGER_PEEK_KB: A/B knob
static size_t peek_stage_bytes() {
  static const size_t bytes = [] {
    const char* e = getenv("STAGER_PEEK_KB");
    long kb = e ? atol(e) : 0;
    return (size_t)(kb >= 16 && kb <= 8192 ? kb : 512) * 1024;
  }();
  return bytes;
}

int64_t HttpConn::relay_body_to(HttpConn& dst, int64_t n, Progress* prog, uint32_t* crc) {
  int64_t moved = 0, done = 0;
  RelayScope scope(&done);
  auto fin = [&](int mode, int64_t m) {
    scope.mode = mode;
    done = m;
    return m;
  };
  if (rpos_ < rend_) {
    int64_t k = std::min<int64_t>(n, (int64_t)(rend_ - rpos_));
    if (crc) *crc = stager::crc32c(rbuf_.data() + rpos_, (size_t)k, *crc);
    dst.send_all(rbuf_.data() + rpos_, (size_t)k);
    rpos_ += (size_t)k;
    moved += k;
    if (prog) prog->bytes.fetch_add(k, std::memory_order_relaxed);
  }
  if (moved == n) return fin(0, moved);
  if (ssl_ || dst.ssl_ || (crc && !relay_tee_on()))
    return fin(2, relay_copy(dst, n, moved, prog, crc));
  if (crc) {
    thread_local std::vector<uint8_t> cbuf(peek_stage_bytes());
    int64_t m = relay_dup(
        dst, n, moved, prog,
        [&](size_t& len) {
          len = std::min(len, cbuf.size());
          return cbuf.data();
        },
        [&](const uint8_t* p, size_t k) {
          uint64_t t0 = mono_ns();
          *crc = stager::crc32c(p, k, *crc);
          t_tally.crc_ns += mono_ns() - t0;
          t_tally.crc_bytes += k;
        });
    return m >= 0 ? fin(1, m) : fin(2, relay_copy(dst, n, moved, prog, crc));
  }
  std::unique_ptr<PipeLease> lease;
  try {
    lease.reset(new PipeLease(g_pipe_main.load()));
  } catch (const IoError&) {
    return fin(2, relay_copy(dst, n, moved, prog, nullptr));   // no pipe to be had: copy
  }
  PipeLease& pl = *lease;
  const int pr = pl.p.r, pw = pl.p.w;
  while (moved < n) {
    if (prog && prog->cancelled.load(std::memory_order_relaxed)) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("cancelled");
    }
    size_t want = (size_t)std::min<int64_t>(n - moved, (int64_t)pl.p.cap);
    ssize_t in = ::splice(fd_, nullptr, pw, nullptr, want, SPLICE_F_MOVE | SPLICE_F_MORE);
    ++t_tally.splice_in;
    if (in < 0) {
      if (errno == EINTR) continue;
      reusable_ = false;
      dst.reusable_ = false;
      if (errno == EAGAIN) throw IoError("recv timeout");
      throw IoError(errstr("splice(src)"));
    }
    if (in == 0) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("source closed mid-body");
    }
    ssize_t left = in;
    while (left > 0) {
      ssize_t out = ::splice(pr, nullptr, dst.fd_, nullptr, (size_t)left,
                             SPLICE_F_MOVE | SPLICE_F_MORE);
      ++t_tally.splice_out;
      if (out < 0) {
        if (errno == EINTR) continue;
        reusable_ = false;
        dst.reusable_ = false;
        throw IoError(errstr("splice(dst)"));
      }
      if (out == 0) {                    // nothing taken: a retry would spin
        reusable_ = false;
        dst.reusable_ = false;
        throw IoError("splice(dst) made no progress");
      }
      left -= out;
    }
    moved += in;
    if (prog) prog->bytes.fetch_add(in, std::memory_order_relaxed);
  }
  pl.clean = true;
  return fin(0, moved);
}

// The bytes sent and the bytes the caller sees are the same pipe pages: splice moves page
// references socket -> pipe -> socket, tee() duplicates the references into a second pipe and
// only that duplicate is copied out (one user-space copy, where recv + send made two and
// allocated fresh socket-buffer pages for the send). -1 (nothing moved) when no pipes can be
// had: the caller copies instead.
template <class Room, class Got>
int64_t HttpConn::relay_tee(HttpConn& dst, int64_t n, int64_t moved, Progress* prog,
                            Room&& room, Got&& got) {
  std::unique_ptr<PipeLease> main_l, dup_l;
  try {
    main_l.reset(new PipeLease(g_pipe_main.load()));
    dup_l.reset(new PipeLease(g_pipe_tee.load()));
  } catch (const IoError&) {
    if (main_l) main_l->clean = true;
    return -1;                       // no pipes to be had: the caller copies (recv + send)
  }
  PipeLease& main = *main_l;
  PipeLease& dup = *dup_l;
  auto fail = [&](const char* what) {
    reusable_ = false;
    dst.reusable_ = false;
    throw IoError(errstr(what));
  };
  // bytes that arrived with the response head
  while (moved < n && rpos_ < rend_) {
    size_t len = (size_t)std::min<int64_t>(n - moved, (int64_t)(rend_ - rpos_));
    uint8_t* p = room(len);
    memcpy(p, rbuf_.data() + rpos_, len);
    rpos_ += len;
    got(p, len);
    try {
      dst.send_all(p, len);
    } catch (...) {
      reusable_ = false;
      throw;
    }
    moved += (int64_t)len;
    if (prog) prog->bytes.fetch_add((int64_t)len, std::memory_order_relaxed);
  }
  if (moved == n) {
    main.clean = dup.clean = true;
    return moved;
  }
  while (moved < n) {
    if (prog && prog->cancelled.load(std::memory_order_relaxed)) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("cancelled");
    }
    size_t want = (size_t)std::min<int64_t>(n - moved, (int64_t)main.p.cap);
    ssize_t in = ::splice(fd_, nullptr, main.p.w, nullptr, want, SPLICE_F_MOVE | SPLICE_F_MORE);
    ++t_tally.splice_in;
    if (in < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        reusable_ = false;
        dst.reusable_ = false;
        throw IoError("recv timeout");
      }
      fail("splice(src)");
    }
    if (in == 0) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("source closed mid-body");
    }
    ssize_t left = in;
    while (left > 0) {
      ssize_t t = ::tee(main.p.r, dup.p.w, (size_t)left, 0);
      if (t < 0) {
        if (errno == EINTR) continue;
        fail("tee");
      }
      if (t == 0) {
        reusable_ = false;
        dst.reusable_ = false;
        throw IoError("tee: no data");
      }
      for (ssize_t seen = 0; seen < t;) {
        size_t len = (size_t)(t - seen);
        uint8_t* p = room(len);
        ssize_t r = ::read(dup.p.r, p, len);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) fail("read(tee)");
        ++t_tally.dup_calls;
        t_tally.dup_bytes += (uint64_t)r;
        got(p, (size_t)r);
        seen += r;
      }
      for (ssize_t chunk = t; chunk > 0;) {
        ssize_t out = ::splice(main.p.r, nullptr, dst.fd_, nullptr, (size_t)chunk,
                               SPLICE_F_MOVE | SPLICE_F_MORE);
        ++t_tally.splice_out;
        if (out < 0) {
          if (errno == EINTR) continue;
          fail("splice(dst)");
        }
        if (out == 0) {                  // nothing taken: a retry would spin
          errno = EPIPE;
          fail("splice(dst)");
        }
        chunk -= out;
      }
      left -= t;
    }
    moved += in;
    if (prog) prog->bytes.fetch_add(in, std::memory_order_relaxed);
  }
  main.clean = dup.clean = true;
  return moved;
}

// STAGER_RELAY_DUP=tee (or set_relay_dup("tee")): the tee() duplicate instead of
// recv(MSG_PEEK) (A/B knob).
static std::atomic<int> g_relay_peek{[] {
  const char* e = getenv("STAGER_RELAY_DUP");
  return (e && strcmp(e, "tee") == 0) ? 0 : 1;
}()};
static bool relay_peek_on() { return g_relay_peek.load(std::memory_order_relaxed) != 0; }

template <class Room, class Got>
int64_t HttpConn::relay_dup(HttpConn& dst, int64_t n, int64_t moved, Progress* prog,
                            Room&& room, Got&& got) {
  return relay_peek_on() ? relay_peek(dst, n, moved, prog, room, got)
                         : relay_tee(dst, n, moved, prog, room, got);
}

// recv(MSG_PEEK) copies the next bytes of the receive queue into the caller's memory without
// consuming them, then exactly those bytes are spliced socket -> pipe -> socket: the S3 leg
// still moves page references, the one copy is the peek, and only one pipe is leased (the
// tee() path needs a second one, which a uid's 64 MiB pipe budget feels at 8 ranks).
template <class Room, class Got>
int64_t HttpConn::relay_peek(HttpConn& dst, int64_t n, int64_t moved, Progress* prog,
                             Room&& room, Got&& got) {
  std::unique_ptr<PipeLease> main_l;
  try {
    main_l.reset(new PipeLease(g_pipe_main.load()));
  } catch (const IoError&) {
    return -1;                       // no pipe to be had: the caller copies (recv + send)
  }
  PipeLease& main = *main_l;
  auto fail = [&](const char* what) {
    reusable_ = false;
    dst.reusable_ = false;
    throw IoError(errstr(what));
  };
  // bytes that arrived with the response head
  while (moved < n && rpos_ < rend_) {
    size_t len = (size_t)std::min<int64_t>(n - moved, (int64_t)(rend_ - rpos_));
    uint8_t* p = room(len);
    memcpy(p, rbuf_.data() + rpos_, len);
    rpos_ += len;
    got(p, len);
    try {
      dst.send_all(p, len);
    } catch (...) {
      reusable_ = false;
      throw;
    }
    moved += (int64_t)len;
    if (prog) prog->bytes.fetch_add((int64_t)len, std::memory_order_relaxed);
  }
  // The peek waits for 256 KiB (or the rest of the body) instead of waking on every segment
  // that lands: 53.4 / 51.7 vs 50.3 / 51.5 GB/s for the checked headline, worker + peer CPU
  // 0.287 - 0.296 vs 0.293 - 0.300 CPU-s/GB (profiles/r6/check2/lowat*). STAGER_RCVLOWAT_KB:
  // another mark (0: off)
  static const int lowat = [] {
    const char* e = getenv("STAGER_RCVLOWAT_KB");
    long kb = e ? atol(e) : 256;
    return (int)(kb > 0 && kb <= 4096 ? kb * 1024 : 0);
  }();
  // (TCP wakes a sleeping reader only once sk_rcvlowat bytes are queued, whatever it asked
  // for: the mark must drop back to 1 before fewer than that are left to come)
  struct LowatScope {
    int fd, on;
    LowatScope(int f, int v) : fd(f), on(v) {
      if (on) setsockopt(fd, SOL_SOCKET, SO_RCVLOWAT, &on, sizeof on);
    }
    void off() {
      if (on) {
        int one = 1;
        setsockopt(fd, SOL_SOCKET, SO_RCVLOWAT, &one, sizeof one);
        on = 0;
      }
    }
    ~LowatScope() { off(); }
  } lowat_scope(fd_, n - moved > 2 * (int64_t)lowat ? lowat : 0);
  while (moved < n) {
    if (lowat_scope.on && n - moved < 2 * (int64_t)lowat) lowat_scope.off();
    if (prog && prog->cancelled.load(std::memory_order_relaxed)) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("cancelled");
    }
    size_t len = (size_t)std::min<int64_t>(n - moved, (int64_t)main.p.cap);
    uint8_t* p = room(len);
    ssize_t k = ::recv(fd_, p, len, MSG_PEEK);
    ++t_tally.dup_calls;
    if (k < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        reusable_ = false;
        dst.reusable_ = false;
        throw IoError("recv timeout");
      }
      fail("recv(peek)");
    }
    if (k == 0) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("source closed mid-body");
    }
    t_tally.dup_bytes += (uint64_t)k;
    got(p, (size_t)k);
    for (ssize_t left = k; left > 0;) {
      // the peeked bytes are queued already: this splice moves them without waiting
      ssize_t in = ::splice(fd_, nullptr, main.p.w, nullptr, (size_t)left,
                            SPLICE_F_MOVE | SPLICE_F_MORE);
      ++t_tally.splice_in;
      if (in < 0) {
        if (errno == EINTR) continue;
        fail("splice(src)");
      }
      if (in == 0) {
        reusable_ = false;
        dst.reusable_ = false;
        throw IoError("source closed mid-body");
      }
      for (ssize_t chunk = in; chunk > 0;) {
        ssize_t out = ::splice(main.p.r, nullptr, dst.fd_, nullptr, (size_t)chunk,
                               SPLICE_F_MOVE | SPLICE_F_MORE);
        ++t_tally.splice_out;
        if (out < 0) {
          if (errno == EINTR) continue;
          fail("splice(dst)");
        }
        if (out == 0) {                  // nothing taken: a retry would spin
          errno = EPIPE;
          fail("splice(dst)");
        }
        chunk -= out;
      }
      left -= in;
    }
    moved += k;
    if (prog) prog->bytes.fetch_add(k, std::memory_order_relaxed);
  }
  main.clean = true;
  return moved;
}

int64_t HttpConn::relay_copy(HttpConn& dst, int64_t n, int64_t moved, Progress* prog,
                             uint32_t* crc) {
  thread_local std::vector<uint8_t> buf(256 * 1024);
  while (moved < n) {
    if (prog && prog->cancelled.load(std::memory_order_relaxed)) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("cancelled");
    }
    size_t r;
    try {
      r = recv_some(buf.data(), (size_t)std::min<int64_t>(n - moved, (int64_t)buf.size()));
    } catch (...) {
      dst.reusable_ = false;
      throw;
    }
    if (r == 0) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("source closed mid-body");
    }
    if (crc) *crc = stager::crc32c(buf.data(), r, *crc);
    try {
      dst.send_all(buf.data(), r);
    } catch (...) {
      reusable_ = false;
      throw;
    }
    moved += (int64_t)r;
    if (prog) prog->bytes.fetch_add((int64_t)r, std::memory_order_relaxed);
  }
  return moved;
}

int64_t HttpConn::relay_body_hashed(HttpConn& dst, int64_t n, int64_t skip, int64_t full_len,
                                    int64_t piece_len, Progress* prog, std::string* digests,
                                    std::string* head, std::string* tail, uint32_t* crc,
                                    uint64_t* gpu_ticket) {
  if (skip < 0 || full_len < 0 || skip + full_len > n || piece_len <= 0)
    throw IoError("relay_body_hashed: bad piece split");
  int64_t scoped = n;               // (counted as moved: a failed relay throws past it)
  RelayScope scope(&scoped);
  scope.mode = 3;
  const int64_t npieces = (full_len + piece_len - 1) / piece_len;
  if (npieces >= 8 && n <= kMaxBufferedPart && sha1_mb_supported())
    return relay_body_hashed_mb(dst, n, skip, full_len, piece_len, prog, digests, head, tail, crc,
                                gpu_ticket);
  // Chunk size: 512 KiB stays in a Zen 5 core's 1 MiB L2 between the copy in (a tee()d
  // duplicate on plain sockets, recv on TLS), the send copy (TLS) and the SHA-1 pass, so the
  // payload is read from DRAM once.
  thread_local std::vector<uint8_t> buf(512 * 1024);
  Hasher h("sha1");
  const int64_t full_end = skip + full_len;
  int64_t pos = 0;        // body offset of the next byte
  int64_t in_piece = 0;   // bytes of the current piece hashed so far
  auto consume = [&](const uint8_t* p, int64_t k) {
    while (k > 0) {
      int64_t t;
      if (pos < skip) {
        t = std::min(k, skip - pos);
        head->append((const char*)p, (size_t)t);
      } else if (pos < full_end) {
        t = std::min({k, piece_len - in_piece, full_end - pos});
        h.update(p, (size_t)t);
        in_piece += t;
        if (in_piece == piece_len || pos + t == full_end) {
          *digests += h.finish_and_reset();
          in_piece = 0;
        }
      } else {
        t = k;
        tail->append((const char*)p, (size_t)t);
      }
      pos += t;
      p += t;
      k -= t;
    }
  };
  if (!ssl_ && !dst.ssl_ && relay_tee_on() &&
      relay_dup(
          dst, n, 0, prog,
          [&](size_t& len) {
            len = std::min(len, buf.size());
            return buf.data();
          },
          [&](const uint8_t* p, size_t k) {
            uint64_t t0 = mono_ns();
            if (crc) *crc = stager::crc32c(p, k, *crc);
            uint64_t t1 = mono_ns();
            consume(p, (int64_t)k);
            t_tally.crc_ns += t1 - t0;
            t_tally.sha1_ns += mono_ns() - t1;
          }) >= 0)
    return pos;
  while (pos < n) {
    if (prog && prog->cancelled.load(std::memory_order_relaxed)) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("cancelled");
    }
    const int64_t want = std::min<int64_t>(n - pos, (int64_t)buf.size());
    int64_t k = take_buffered(buf.data(), want);   // bytes that arrived with the header
    if (k == 0) {
      size_t r;
      try {
        r = recv_some(buf.data(), (size_t)want);
      } catch (...) {
        dst.reusable_ = false;
        throw;
      }
      if (r == 0) {
        reusable_ = false;
        dst.reusable_ = false;
        throw IoError("source closed mid-body");
      }
      k = (int64_t)r;
    }
    if (crc) *crc = stager::crc32c(buf.data(), (size_t)k, *crc);
    try {
      dst.send_all(buf.data(), (size_t)k);
    } catch (...) {
      reusable_ = false;
      throw;
    }
    consume(buf.data(), k);
    if (prog) prog->bytes.fetch_add(k, std::memory_order_relaxed);
  }
  return pos;
}

namespace {
// Part buffers for relay_body_hashed_mb: anonymous memory on 2 MiB boundaries with
// MADV_HUGEPAGE and no value-initialisation. A std::vector resize zero-filled every 4 KiB page
// of a 64 MiB part and faulted them one by one: ~280k minor faults (0.7 CPU-s) the first time
// 16 relay threads ran, i.e. the first torrent a worker staged ran at half speed.
// The part hasher the hashed relay hands parts to (set_gpu_part_hasher), or null.
std::atomic<const GpuPartHashApi*> g_gpu_api{nullptr};

struct PartBuffer {
  static constexpr size_t kHuge = size_t(2) << 20;
  uint8_t* base = nullptr;
  size_t mapped = 0, cap = 0;
  uint8_t* data = nullptr;
  const GpuPartHashApi* reg_api = nullptr;   // page-locked for the GPU hasher's DMA
  explicit PartBuffer(size_t n) {
    const size_t c = (n + kHuge - 1) & ~(kHuge - 1);
    void* m = mmap(nullptr, c + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) throw std::bad_alloc();
    base = (uint8_t*)m;
    mapped = c + kHuge;
    data = (uint8_t*)(((uintptr_t)m + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
    madvise(data, c, MADV_HUGEPAGE);  // best effort: THP "never" just keeps 4 KiB pages
    cap = c;
  }
  ~PartBuffer() {
    if (reg_api) reg_api->unreg(reg_api->ctx, data);
    munmap(base, mapped);
  }
  PartBuffer(const PartBuffer&) = delete;
  PartBuffer& operator=(const PartBuffer&) = delete;
};

// One process-wide pool instead of a buffer per transfer thread: a thread_local buffer as
// large as the biggest part ever relayed stayed resident on each of the 32 transfer threads
// (up to 4-8 GiB per worker after one torrent job). Buffers in use are bounded by the
// caller's admission (torrent/stream.py's PartBudget: relays in flight and parts awaiting
// their DMA draw bytes from one process-wide budget); idle buffers are kept for the next
// part only while leased + idle stays within that budget - an idle buffer is unmapped to make
// room before a new one is mapped - and trim() unmaps the idle ones down to what the caller
// keeps warm.
class PartPool {
 public:
  static size_t need(size_t n) { return (n + PartBuffer::kHuge - 1) & ~(PartBuffer::kHuge - 1); }

  std::unique_ptr<PartBuffer> acquire(size_t n) {
    const size_t want = need(n);
    std::vector<std::unique_ptr<PartBuffer>> drop;   // unmapped outside the lock
    {
      std::lock_guard<std::mutex> g(mu_);
      // reuse an idle buffer of about the asked size: a much larger one would lease more
      // bytes than the caller's budget accounted for
      size_t best = idle_.size();
      for (size_t i = 0; i < idle_.size(); ++i) {
        const size_t c = idle_[i]->cap;
        if (c >= want && c - want <= std::max(want / 4, PartBuffer::kHuge) &&
            (best == idle_.size() || c < idle_[best]->cap))
          best = i;
      }
      if (best < idle_.size()) {
        std::unique_ptr<PartBuffer> b = std::move(idle_[best]);
        idle_.erase(idle_.begin() + (ptrdiff_t)best);
        idle_bytes_ -= b->cap;
        lease(b->cap);
        return b;
      }
      // a new mapping: unmap idle buffers (largest first) until it fits in the budget
      while (budget_ && !idle_.empty() && in_use_bytes_ + idle_bytes_ + want > budget_) {
        size_t big = 0;
        for (size_t i = 1; i < idle_.size(); ++i)
          if (idle_[i]->cap > idle_[big]->cap) big = i;
        idle_bytes_ -= idle_[big]->cap;
        drop.push_back(std::move(idle_[big]));
        idle_.erase(idle_.begin() + (ptrdiff_t)big);
        evicted_++;
      }
      lease(want);
    }
    drop.clear();
    try {
      created_.fetch_add(1, std::memory_order_relaxed);
      return std::unique_ptr<PartBuffer>(new PartBuffer(n));
    } catch (...) {
      std::lock_guard<std::mutex> g(mu_);
      in_use_ -= 1;
      in_use_bytes_ -= want;
      throw;
    }
  }
  void release(std::unique_ptr<PartBuffer> b) {
    std::unique_ptr<PartBuffer> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      in_use_ -= 1;
      in_use_bytes_ -= b->cap;
      if (b->reg_api && b->reg_api != g_gpu_api.load()) {
        drop = std::move(b);         // registered with a hasher no longer in use: unlock
      } else if (idle_.size() < max_idle_ &&
                 (!budget_ || in_use_bytes_ + idle_bytes_ + b->cap <= budget_)) {
        idle_bytes_ += b->cap;
        idle_.push_back(std::move(b));
      } else {
        drop = std::move(b);
      }
    }
  }  // `drop` unmapped outside the lock
  // Idle buffers page-locked for another hasher than `keep` are unregistered and unmapped
  // (set_gpu_part_hasher: the previous hasher is still alive when this runs).
  void drop_foreign(const GpuPartHashApi* keep) {
    std::vector<std::unique_ptr<PartBuffer>> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t i = 0; i < idle_.size();) {
        if (idle_[i]->reg_api && idle_[i]->reg_api != keep) {
          idle_bytes_ -= idle_[i]->cap;
          drop.push_back(std::move(idle_[i]));
          idle_.erase(idle_.begin() + (ptrdiff_t)i);
        } else {
          ++i;
        }
      }
    }
  }
  size_t trim(size_t keep_bytes) {
    std::vector<std::unique_ptr<PartBuffer>> drop;
    size_t freed = 0;
    {
      std::lock_guard<std::mutex> g(mu_);
      while (!idle_.empty() && idle_bytes_ > keep_bytes) {
        idle_bytes_ -= idle_.back()->cap;
        freed += idle_.back()->cap;
        drop.push_back(std::move(idle_.back()));
        idle_.pop_back();
      }
    }
    return freed;
  }
  void set_max_idle(size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    max_idle_ = n;
  }
  void set_budget(size_t bytes) {
    std::vector<std::unique_ptr<PartBuffer>> drop;   // unmapped outside the lock
    std::lock_guard<std::mutex> g(mu_);
    budget_ = bytes;
    // idle buffers beyond the new budget go at once
    while (bytes && !idle_.empty() && in_use_bytes_ + idle_bytes_ > budget_) {
      idle_bytes_ -= idle_.back()->cap;
      drop.push_back(std::move(idle_.back()));
      idle_.pop_back();
      evicted_++;
    }
  }
  void reset_peak() {
    std::lock_guard<std::mutex> g(mu_);
    peak_ = in_use_bytes_ + idle_bytes_;
    over_budget_ = 0;
  }
  RelayPoolStats stats() {
    std::lock_guard<std::mutex> g(mu_);
    return RelayPoolStats{idle_.size(), idle_bytes_, in_use_, max_idle_, created_.load(),
                          in_use_bytes_, budget_, peak_, evicted_, over_budget_};
  }

 private:
  void lease(size_t bytes) {   // mu_ held
    in_use_ += 1;
    in_use_bytes_ += bytes;
    if (budget_ && in_use_bytes_ > budget_) over_budget_++;
    peak_ = std::max(peak_, in_use_bytes_ + idle_bytes_);
  }
  std::mutex mu_;
  std::vector<std::unique_ptr<PartBuffer>> idle_;
  size_t idle_bytes_ = 0, in_use_ = 0, max_idle_ = 16;
  size_t in_use_bytes_ = 0, budget_ = 0, peak_ = 0;
  uint64_t evicted_ = 0, over_budget_ = 0;
  std::atomic<uint64_t> created_{0};   // buffers mapped (each one faulted in, maybe page-locked)
};

PartPool& part_pool() {
  static PartPool* p = new PartPool();  // never destroyed: transfer threads may outlive exit
  return *p;
}

struct PartLease {
  std::unique_ptr<PartBuffer> b;
  explicit PartLease(size_t n) : b(part_pool().acquire(n)) {}
  ~PartLease() {
    if (b) part_pool().release(std::move(b));
  }
};

// ---- GPU part hashing (gpu_part_api.h) -------------------------------------------------
// The hasher notifies each part's COPIED / DONE from its own thread (gpu_notify); the part's
// buffer goes back to the pool right there, and the news is queued for gpu_part_poll (the
// asyncio side reads the eventfd) or for a blocked gpu_part_wait. No thread waits per part.
std::atomic<int> g_gpu_min_pieces{8};
std::atomic<uint64_t> g_gpu_submitted{0}, g_gpu_fallbacks{0}, g_gpu_refused{0};

struct GpuPending {
  std::unique_ptr<PartBuffer> buf;   // leased until the DMA out of it completed
  const GpuPartHashApi* api = nullptr;
  uint64_t ticket = 0;
  int64_t skip = 0, full_len = 0, piece_len = 0;
  bool copied = false, finished = false, failed = false;
  bool forgotten = false, copied_reported = false;
  bool waited = false;               // claimed by gpu_part_wait: gpu_part_poll leaves it alone
  std::string result;                // digests, or the error
};
std::mutex g_gpu_mu;
std::condition_variable g_gpu_cv;
std::unordered_map<uint64_t, GpuPending> g_gpu_parts;                      // by part id
std::map<std::pair<const GpuPartHashApi*, uint64_t>, uint64_t> g_gpu_ids;  // (hasher, ticket)
std::deque<uint64_t> g_gpu_news;                                           // ids for gpu_part_poll
uint64_t g_gpu_next_id = 0;

int gpu_efd() {
  static int fd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  return fd;
}

void gpu_signal(uint64_t id) {   // g_gpu_mu held
  g_gpu_news.push_back(id);
  g_gpu_cv.notify_all();
  const uint64_t one = 1;
  if (gpu_efd() >= 0) {
    ssize_t w = write(gpu_efd(), &one, sizeof one);
    (void)w;   // EAGAIN: the counter is saturated, the reader wakes anyway
  }
}

void host_digests_impl(const uint8_t* p, int64_t full_len, int64_t piece_len, std::string* out);
void host_digests(const uint8_t* p, int64_t full_len, int64_t piece_len, std::string* out) {
  const uint64_t t0 = mono_ns();
  host_digests_impl(p, full_len, piece_len, out);
  t_tally.sha1_ns += mono_ns() - t0;
}
void host_digests_impl(const uint8_t* p, int64_t full_len, int64_t piece_len, std::string* out) {
  const int64_t np = (full_len + piece_len - 1) / piece_len;
  std::vector<const uint8_t*> ptrs((size_t)np);
  std::vector<size_t> lens((size_t)np);
  for (int64_t i = 0; i < np; ++i) {
    ptrs[(size_t)i] = p + i * piece_len;
    lens[(size_t)i] = (size_t)std::min<int64_t>(piece_len, full_len - i * piece_len);
  }
  out->resize((size_t)np * 20);
  sha1_mb(ptrs.data(), lens.data(), (size_t)np, (uint8_t*)&(*out)[0]);
}

// COPIED: the buffer returns to the pool (or, when the device failed before the DMA ended,
// the bytes are still ours: hashed here and the part finishes at once).
void gpu_copied(const GpuPartHashApi* a, uint64_t ticket, uint64_t id) {
  char err[256] = {0};
  const int rc = a->wait(a->ctx, ticket, GPU_PART_COPIED, nullptr, 0, err, sizeof err);
  std::unique_ptr<PartBuffer> buf;
  int64_t skip = 0, full = 0, plen = 0;
  {
    std::lock_guard<std::mutex> g(g_gpu_mu);
    auto it = g_gpu_parts.find(id);
    if (it == g_gpu_parts.end() || it->second.copied || !it->second.buf) return;
    buf = std::move(it->second.buf);
    skip = it->second.skip;
    full = it->second.full_len;
    plen = it->second.piece_len;
  }
  std::string digests;
  if (rc != 0) {
    host_digests(buf->data + skip, full, plen, &digests);
    g_gpu_fallbacks++;
  }
  part_pool().release(std::move(buf));
  std::lock_guard<std::mutex> g(g_gpu_mu);
  auto it = g_gpu_parts.find(id);
  if (it == g_gpu_parts.end()) return;   // only a finished part is ever erased: not this one
  GpuPending& p = it->second;
  p.copied = true;
  if (rc != 0) {            // the hasher forgets a job whose copy failed: no DONE follows
    p.finished = true;
    p.result.swap(digests);
    g_gpu_ids.erase({a, ticket});
  }
  if (p.forgotten && p.finished)
    g_gpu_parts.erase(it);          // (a failed copy finishes the part at once)
  else if (!p.forgotten)
    gpu_signal(id);
  // a gpu_part_forget blocked on this part wakes on any change, the erase included (the
  // selftest's fault section hung here when a forgotten part's copy failed)
  g_gpu_cv.notify_all();
}

void gpu_done(const GpuPartHashApi* a, uint64_t ticket, uint64_t id) {
  int64_t np = 0;
  {
    std::lock_guard<std::mutex> g(g_gpu_mu);
    auto it = g_gpu_parts.find(id);
    if (it == g_gpu_parts.end() || it->second.finished) return;
    np = (it->second.full_len + it->second.piece_len - 1) / it->second.piece_len;
  }
  std::string out((size_t)np * 20, '\0');
  char err[256] = {0};
  const int rc = a->wait(a->ctx, ticket, GPU_PART_DONE, (uint8_t*)&out[0], out.size(), err,
                         sizeof err);
  std::lock_guard<std::mutex> g(g_gpu_mu);
  g_gpu_ids.erase({a, ticket});
  auto it = g_gpu_parts.find(id);
  if (it == g_gpu_parts.end()) return;
  GpuPending& p = it->second;
  p.finished = true;
  p.failed = rc != 0;
  p.result = rc ? std::string("GPU piece hashing failed: ") + err : out;
  if (p.forgotten) {
    g_gpu_parts.erase(it);
    g_gpu_cv.notify_all();
  } else {
    gpu_signal(id);
  }
}

// gpu_notify_fn: called on the hasher's thread without its lock held.
void gpu_notify(void* arg, uint64_t ticket, int phase) {
  const GpuPartHashApi* a = (const GpuPartHashApi*)arg;
  uint64_t id;
  bool copied;
  {
    std::lock_guard<std::mutex> g(g_gpu_mu);
    auto it = g_gpu_ids.find({a, ticket});
    if (it == g_gpu_ids.end()) return;
    id = it->second;
    // never throw on the hasher's thread (its dispatcher would take it for a device error)
    auto p = g_gpu_parts.find(id);
    if (p == g_gpu_parts.end()) return;
    copied = p->second.copied;
  }
  if (!copied) gpu_copied(a, ticket, id);   // a DONE implies the copy is over
  if (phase == GPU_PART_DONE) gpu_done(a, ticket, id);
}
}  // namespace

const void* gpu_part_hasher_current() { return g_gpu_api.load(); }

void set_gpu_part_hasher(const void* api, int min_pieces) {
  const GpuPartHashApi* a = (const GpuPartHashApi*)api;
  if (a && a->abi != GPU_PART_API_ABI) throw std::invalid_argument("gpu_part_api ABI mismatch");
  if (a) a->set_notify(a->ctx, &gpu_notify, (void*)a);
  g_gpu_min_pieces.store(std::max(1, min_pieces));
  const GpuPartHashApi* old = g_gpu_api.exchange(a);
  part_pool().drop_foreign(a);
  // idle swarm piece buffers page-locked for the hasher being replaced are unlocked and freed
  // now, not whenever a verifier happens to touch them (retired hashers stay alive,
  // ops/hashing.py, so `old` is still callable)
  if (old && old != a) swarm_piece_pool_forget(old);
}

// ---- CpuPartHasher: the gpu_part_api.h contract served by a host thread ------------------
// A test double with the device's timing shape: the "DMA" (a copy into its own buffer) and
// the "kernel" (multi-buffer SHA-1) each complete after a delay on a worker thread, which
// notifies COPIED / DONE like the device's dispatcher, so the stream stager's asynchronous
// GPU path (part ids, buffer release at copy completion, eventfd completions) runs and is
// tested on hosts without a HIP device.
namespace {
struct CpuJob {
  const uint8_t* host;
  int64_t len, piece_len;
  std::string copy, digests;
  bool copied = false, done = false;
  bool fail_copy = false, fail_done = false;
  bool abandoned = false;   // its copy "failed": the relay hashed on the host, nobody waits
};
}  // namespace

struct CpuPartHasher::Impl {
  std::mutex mu;
  std::condition_variable cv, wcv;
  std::unordered_map<uint64_t, CpuJob> jobs;
  std::deque<uint64_t> queue;
  uint64_t seq = 0;
  bool stop = false;
  double delay_s;
  int fail_copy_every = 0, fail_done_every = 0;
  std::thread th;
  GpuPartHashApi api{};
  uint64_t registered = 0;
  gpu_part_notify_fn notify = nullptr;
  void* notify_arg = nullptr;

  void tell(uint64_t t, int phase, std::unique_lock<std::mutex>& lk) {
    gpu_part_notify_fn fn = notify;
    void* arg = notify_arg;
    lk.unlock();
    if (fn) fn(arg, t, phase);
    lk.lock();
  }

  void run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || !queue.empty(); });
      if (stop && queue.empty()) return;
      uint64_t t = queue.front();
      queue.pop_front();
      CpuJob* j = &jobs.at(t);
      lk.unlock();
      std::this_thread::sleep_for(std::chrono::duration<double>(delay_s));
      std::string c((const char*)j->host, (size_t)j->len);
      lk.lock();
      j->copy.swap(c);
      j->copied = true;
      wcv.notify_all();
      tell(t, GPU_PART_COPIED, lk);
      j = &jobs.at(t);
      lk.unlock();
      std::this_thread::sleep_for(std::chrono::duration<double>(delay_s));
      std::string d;
      host_digests((const uint8_t*)j->copy.data(), j->len, j->piece_len, &d);
      lk.lock();
      j->digests.swap(d);
      j->done = true;
      wcv.notify_all();
      if (j->abandoned)
        jobs.erase(t);
      else
        tell(t, GPU_PART_DONE, lk);
    }
  }
};

CpuPartHasher::CpuPartHasher(double delay_s, int fail_copy_every, int fail_done_every)
    : impl_(new Impl) {
  Impl* m = impl_.get();
  m->delay_s = delay_s;
  m->fail_copy_every = fail_copy_every;
  m->fail_done_every = fail_done_every;
  m->api.abi = GPU_PART_API_ABI;
  m->api.ctx = m;
  m->api.reg = [](void* c, void*, size_t) {
    Impl* i = (Impl*)c;
    std::lock_guard<std::mutex> g(i->mu);
    i->registered++;
    return 0;
  };
  m->api.unreg = [](void*, void*) {};
  m->api.submit = [](void* c, const uint8_t* d, int64_t len, int64_t pl) -> uint64_t {
    Impl* i = (Impl*)c;
    std::lock_guard<std::mutex> g(i->mu);
    if (i->stop || len <= 0 || pl <= 0) return 0;
    uint64_t t = ++i->seq;
    CpuJob& j = i->jobs[t];
    j.host = d;
    j.len = len;
    j.piece_len = pl;
    j.fail_copy = i->fail_copy_every > 0 && t % (uint64_t)i->fail_copy_every == 0;
    j.fail_done = i->fail_done_every > 0 && t % (uint64_t)i->fail_done_every == 0;
    i->queue.push_back(t);
    i->cv.notify_all();
    return t;
  };
  m->api.wait = [](void* c, uint64_t t, int phase, uint8_t* out, size_t ol, char* err,
                   size_t el) -> int {
    Impl* i = (Impl*)c;
    std::unique_lock<std::mutex> lk(i->mu);
    auto it = i->jobs.find(t);
    if (it == i->jobs.end()) {
      snprintf(err, el, "unknown ticket");
      return -1;
    }
    CpuJob* j = &it->second;
    i->wcv.wait(lk, [&] { return phase == GPU_PART_COPIED ? j->copied : j->done; });
    if ((phase == GPU_PART_COPIED && j->fail_copy) || (phase == GPU_PART_DONE && j->fail_done)) {
      snprintf(err, el, "injected device failure (%s)", phase == GPU_PART_COPIED ? "copy" : "hash");
      if (phase == GPU_PART_DONE)
        i->jobs.erase(t);         // the worker thread is done with it (by key: `it` may be
                                  // stale after the wait)
      else
        j->abandoned = true;      // erased by the worker thread once it is done with it
      return -1;
    }
    if (phase == GPU_PART_DONE) {
      if (ol < j->digests.size()) {
        snprintf(err, el, "digest buffer too small");
        return -1;
      }
      memcpy(out, j->digests.data(), j->digests.size());
      i->jobs.erase(t);
    }
    return 0;
  };
  m->api.set_notify = [](void* c, gpu_part_notify_fn fn, void* arg) {
    Impl* i = (Impl*)c;
    std::lock_guard<std::mutex> g(i->mu);
    i->notify = fn;
    i->notify_arg = arg;
  };
  m->th = std::thread([m] { m->run(); });
}

CpuPartHasher::~CpuPartHasher() {
  {
    std::lock_guard<std::mutex> g(impl_->mu);
    impl_->stop = true;
  }
  impl_->cv.notify_all();
  impl_->th.join();
}

const void* CpuPartHasher::api() const { return &impl_->api; }

uint64_t CpuPartHasher::registered() const {
  std::lock_guard<std::mutex> g(impl_->mu);
  return impl_->registered;
}

GpuPartStats gpu_part_stats() {
  size_t pending;
  {
    std::lock_guard<std::mutex> g(g_gpu_mu);
    pending = g_gpu_parts.size();
  }
  return GpuPartStats{g_gpu_submitted.load(), g_gpu_fallbacks.load(), g_gpu_refused.load(),
                      pending};
}

// Iterators into g_gpu_parts do not survive a wait: relays insert (and may rehash) while the
// lock is released, so every wake looks the part up again.
std::string gpu_part_wait(uint64_t id) {
  std::unique_lock<std::mutex> lk(g_gpu_mu);
  auto w = g_gpu_parts.find(id);
  if (w == g_gpu_parts.end()) throw IoError("gpu_part_wait: unknown part");
  w->second.waited = true;           // from here on gpu_part_poll does not collect it
  g_gpu_cv.wait(lk, [&] {
    auto f = g_gpu_parts.find(id);
    return f == g_gpu_parts.end() || f->second.finished;
  });
  auto it = g_gpu_parts.find(id);
  if (it == g_gpu_parts.end()) throw IoError("gpu_part_wait: part already collected");
  GpuPending p = std::move(it->second);
  g_gpu_parts.erase(it);
  if (p.failed) throw IoError(p.result);
  return p.result;
}

void gpu_part_forget(uint64_t id) {
  std::unique_lock<std::mutex> lk(g_gpu_mu);
  auto it = g_gpu_parts.find(id);
  if (it == g_gpu_parts.end()) return;
  it->second.forgotten = true;
  // the caller's buffer lease ends when this returns, as for a part hashed on the host
  g_gpu_cv.wait(lk, [&] {
    auto f = g_gpu_parts.find(id);
    return f == g_gpu_parts.end() || f->second.copied;
  });
  it = g_gpu_parts.find(id);
  if (it != g_gpu_parts.end() && it->second.finished) g_gpu_parts.erase(it);
}

int gpu_part_eventfd() { return gpu_efd(); }

std::vector<GpuPartEvent> gpu_part_poll() {
  uint64_t cnt;
  ssize_t r = read(gpu_efd(), &cnt, sizeof cnt);   // reset the counter before draining
  (void)r;
  std::vector<GpuPartEvent> out;
  std::lock_guard<std::mutex> g(g_gpu_mu);
  while (!g_gpu_news.empty()) {
    const uint64_t id = g_gpu_news.front();
    g_gpu_news.pop_front();
    auto it = g_gpu_parts.find(id);
    if (it == g_gpu_parts.end() || it->second.forgotten || it->second.waited) continue;
    GpuPending& p = it->second;
    if (p.copied && !p.copied_reported) {
      p.copied_reported = true;
      out.push_back(GpuPartEvent{id, 1, std::string()});
    }
    if (p.finished) {
      out.push_back(GpuPartEvent{id, p.failed ? 3 : 2, std::move(p.result)});
      g_gpu_parts.erase(it);
    }
  }
  return out;
}

void set_relay_dup(const std::string& mode) {
  if (mode != "peek" && mode != "tee") throw std::invalid_argument("relay dup mode: peek or tee");
  g_relay_peek.store(mode == "peek" ? 1 : 0);
}
std::string relay_dup_mode() { return relay_peek_on() ? "peek" : "tee"; }

size_t relay_pool_trim(size_t keep_bytes) { return part_pool().trim(keep_bytes); }
PipeStats pipe_stats() { return pipe_pool().stats(); }

RelayCounters relay_counters() {
  RelayCounters c{};
  for (int i = 0; i < 4; ++i) {
    c.relays[i] = g_rc.relays[i].load();
    c.bytes[i] = g_rc.bytes[i].load();
    c.cpu_ns[i] = g_rc.cpu_ns[i].load();
  }
  c.splice_in_calls = g_rc.splice_in.load();
  c.splice_out_calls = g_rc.splice_out.load();
  c.dup_calls = g_rc.dup_calls.load();
  c.dup_bytes = g_rc.dup_bytes.load();
  c.crc_ns = g_rc.crc_ns.load();
  c.crc_bytes = g_rc.crc_bytes.load();
  c.sha1_ns = g_rc.sha1_ns.load();
  c.nt_bytes = g_rc.nt_bytes.load();
  return c;
}
void set_pipes_refused(bool on) { g_pipes_refused.store(on); }
void set_pipe_sizes(size_t main, size_t tee) {
  if (main) g_pipe_main.store(main);
  if (tee) g_pipe_tee.store(tee);
  pipe_pool().drop_idle();
}
void relay_pool_set_max_idle(size_t n) { part_pool().set_max_idle(n); }
void relay_pool_set_budget(size_t bytes) { part_pool().set_budget(bytes); }
void relay_pool_reset_peak() { part_pool().reset_peak(); }
RelayPoolStats relay_pool_stats() { return part_pool().stats(); }

// STAGER_PART_NT: how a hashed relay fills its part buffer. 0: the peek lands in the part
// buffer itself (a cold 64 MiB buffer: the kernel's copy reads each line for ownership before
// writing it back - three DRAM passes per byte once the DMA or the host's SHA-1 reads it
// again); 1 (parts bound for the gfx950 PartHasher) / 2 (every hashed part): the peek lands in
// an L2-sized buffer, is CRC'd there and streamed into the part buffer with non-temporal
// stores - two passes, for one user-space copy out of L2. Pinned torrent A/B (config 4, 20 GB,
// 5 alternating runs x 4 pairs each, profiles/r6/nt/): the device arm 33.7 - 34.0 GB/s with 1
// vs 32.0 - 33.7 with 0 (ratio to the host arm 1.20 - 1.22 vs 1.13 - 1.20), worker 0.239 vs
// 0.246 CPU-s/GB; 2 did not speed the host arm up (30.6 / 28.2 vs 31.9 / 29.9 GB/s with 0).
static int part_nt_mode() {
  static const int m = [] {
    const char* e = getenv("STAGER_PART_NT");
    return e ? std::max(0, std::min(2, atoi(e))) : 1;
  }();
  return m;
}

__attribute__((target("avx2"))) static void stream_copy_avx2(uint8_t* d, const uint8_t* s,
                                                              size_t n) {
  size_t head = std::min(n, (size_t)(-(uintptr_t)d & 31));
  memcpy(d, s, head);
  d += head, s += head, n -= head;
  for (; n >= 128; n -= 128, d += 128, s += 128) {
    const __m256i a = _mm256_loadu_si256((const __m256i*)s);
    const __m256i b = _mm256_loadu_si256((const __m256i*)(s + 32));
    const __m256i c = _mm256_loadu_si256((const __m256i*)(s + 64));
    const __m256i e = _mm256_loadu_si256((const __m256i*)(s + 96));
    _mm256_stream_si256((__m256i*)d, a);
    _mm256_stream_si256((__m256i*)(d + 32), b);
    _mm256_stream_si256((__m256i*)(d + 64), c);
    _mm256_stream_si256((__m256i*)(d + 96), e);
  }
  for (; n >= 32; n -= 32, d += 32, s += 32)
    _mm256_stream_si256((__m256i*)d, _mm256_loadu_si256((const __m256i*)s));
  memcpy(d, s, n);
  _mm_sfence();                        // ordered before the part is handed to the DMA / hash
}

static void stream_copy(uint8_t* d, const uint8_t* s, size_t n) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2)
    stream_copy_avx2(d, s, n);
  else
    memcpy(d, s, n);
}

int64_t HttpConn::relay_body_hashed_mb(HttpConn& dst, int64_t n, int64_t skip,
                                       int64_t full_len, int64_t piece_len, Progress* prog,
                                       std::string* digests, std::string* head,
                                       std::string* tail, uint32_t* crc,
                                       uint64_t* gpu_ticket) {
  // The whole part lands in a pooled buffer on its way to `dst` (plain sockets: a tee()d
  // copy of the spliced pages; TLS or no pipes: recv into it, send from it), then its pieces
  // are hashed 16 at a time in the lanes of the AVX-512 multi-buffer SHA-1 - 3-5x the
  // per-core rate of a single SHA-NI chain, which bounds the chunked path once many parts
  // are in flight.
  PartLease lease((size_t)n);
  uint8_t* b = lease.b->data;
  int64_t pos = 0;
  const int64_t np = (full_len + piece_len - 1) / piece_len;
  const GpuPartHashApi* api = gpu_ticket ? g_gpu_api.load() : nullptr;
  const int nt = part_nt_mode();
  if (!ssl_ && !dst.ssl_ && relay_tee_on() &&
      (nt == 2 || (nt == 1 && api && np >= g_gpu_min_pieces.load()))) {
    thread_local std::vector<uint8_t> sbuf(peek_stage_bytes());
    relay_dup(
        dst, n, 0, prog,
        [&](size_t& len) {
          len = std::min({len, sbuf.size(), (size_t)(n - pos)});
          return sbuf.data();
        },
        [&](const uint8_t* p, size_t k) {
          if (crc) {
            uint64_t t0 = mono_ns();
            *crc = stager::crc32c(p, k, *crc);
            t_tally.crc_ns += mono_ns() - t0;
          }
          stream_copy(b + pos, p, k);
          pos += (int64_t)k;
        });
    g_rc.nt_bytes.fetch_add((uint64_t)pos, std::memory_order_relaxed);
  } else if (!ssl_ && !dst.ssl_ && relay_tee_on()) {
    relay_dup(
        dst, n, 0, prog,
        [&](size_t& len) {
          len = std::min<size_t>(len, (size_t)(n - pos));
          return b + pos;
        },
        [&](const uint8_t* p, size_t k) {
          if (crc) {
            uint64_t t0 = mono_ns();
            *crc = stager::crc32c(p, k, *crc);
            t_tally.crc_ns += mono_ns() - t0;
          }
          pos += (int64_t)k;
        });
  }
  while (pos < n) {
    if (prog && prog->cancelled.load(std::memory_order_relaxed)) {
      reusable_ = false;
      dst.reusable_ = false;
      throw IoError("cancelled");
    }
    const int64_t want = std::min<int64_t>(n - pos, 1 << 20);
    int64_t k = take_buffered(b + pos, want);
    if (k == 0) {
      size_t r;
      try {
        r = recv_some(b + pos, (size_t)want);
      } catch (...) {
        dst.reusable_ = false;
        throw;
      }
      if (r == 0) {
        reusable_ = false;
        dst.reusable_ = false;
        throw IoError("source closed mid-body");
      }
      k = (int64_t)r;
    }
    if (crc) *crc = stager::crc32c(b + pos, (size_t)k, *crc);
    try {
      dst.send_all(b + pos, (size_t)k);
    } catch (...) {
      reusable_ = false;
      throw;
    }
    pos += k;
    if (prog) prog->bytes.fetch_add(k, std::memory_order_relaxed);
  }
  head->assign((const char*)b, (size_t)skip);
  tail->assign((const char*)b + skip + full_len, (size_t)(n - skip - full_len));
  if (api && np >= g_gpu_min_pieces.load()) {
    PartBuffer* pb = lease.b.get();
    if (!pb->reg_api && api->reg(api->ctx, pb->data, pb->cap) == 0)
      pb->reg_api = api;
    if (pb->reg_api == api) {
      // held across submit: the hasher's COPIED for this ticket cannot overtake the record
      std::lock_guard<std::mutex> g(g_gpu_mu);
      const uint64_t t = api->submit(api->ctx, b + skip, full_len, piece_len);
      if (t) {
        const uint64_t id = ++g_gpu_next_id;
        GpuPending& pend = g_gpu_parts[id];
        pend.buf = std::move(lease.b);            // leased until the DMA is done
        pend.api = api;
        pend.ticket = t;
        pend.skip = skip;
        pend.full_len = full_len;
        pend.piece_len = piece_len;
        const bool fresh = g_gpu_ids.emplace(std::make_pair(api, t), id).second;
        if (!fresh) throw std::logic_error("gpu part hasher reused a pending ticket");
        g_gpu_submitted++;
        digests->clear();
        *gpu_ticket = id;
        return pos;
      }
    }
    g_gpu_refused++;
  }
  host_digests(b + skip, full_len, piece_len, digests);
  return pos;
}

void HttpConn::discard_body(const ResponseHead& h) {
  if (h.chunked || h.content_length > 0) {
    read_body(h, (int64_t)1 << 40);
  } else if (h.content_length < 0 && h.status != 204 && h.status != 304) {
    reusable_ = false;
  }
}

}  // namespace stager
