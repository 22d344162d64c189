// blobd - native benchmark peer for the staging daemon.
//
// One multi-threaded HTTP/1.1 server that plays both external systems of the reference's
// hot path: the HTTP origin (`request(url)`, lib/download.js:160) and the
// S3/MinIO staging endpoint (`fPutObject`, lib/upload.js:45). Python servers would cap the
// bench far below what one worker can move, so the peers are native too.
//
//   origin:  GET|HEAD /media/<name>?size=N&seed=S   deterministic random bytes, Range support
//   s3:      HEAD|PUT /<bucket>, GET /<bucket>?list-type=2, GET /<bucket>?uploads,
//            PUT|GET|HEAD|DELETE /<bucket>/<key>, multipart (POST ?uploads, PUT ?partNumber,
//            POST ?uploadId, DELETE ?uploadId)
//   stats:   GET /_stats  (JSON: bytes received/served, objects, requests)
//   pool:    GET /_pool   (the pool every synthetic byte is taken from: 64 MiB + 4 KiB, see kPool)
//   crc:     GET /_crc_selected?key=K&part=N  ("1" when --crc-check recomputes that body's CRC)
//   --synth-files FILE ("<path> <size> <seed>" lines): BEP-19 webseed files under
//            /files/<path> made of pool bytes (a 20 GB torrent without 20 GB on disk)
//   --synth-bucket NAME --synth-manifest FILE ("<key> <size>" lines): a read-only source
//            bucket of synthetic objects (List v2, HEAD, GET with Range) for bucket:// jobs;
//            query-string auth (presigned URLs) is accepted, signatures are not checked
//
// --tls-cert/--tls-key: serve https (OpenSSL, one session per connection thread) for the TLS
// staging bench; bodies then pass through user space both ways (no sendfile / splice).
//
// Uploaded bodies are received into a per-connection buffer and folded into a 64-bit
// checksum (so every byte crosses memory like a real store); objects <= --keep-bytes are
// kept in memory (done markers, tests), larger ones keep only size + checksum.
// SigV4 is NOT verified here (the Python FakeS3 does that in the test-suite).
//
// --sink picks what happens to large S3 bodies:
//   checksum  every byte folded into the checksum (default)
//   discard   dropped in the kernel (recv MSG_TRUNC), no user-space copy
//   sample    dropped like discard, but a window of --sample-len bytes every --sample-stride
//             bytes (plus the body's last window) is read and kept, then compared with the
//             bytes the origin generator produced for that object once its offset is known
//   verify    every byte CRC32C'd on arrival, compared at completion with the CRC32C of the
//             generator's bytes for the same range
// An S3 object is matched to its origin object through the key the staging service writes,
// `<id>/original/<base64(basename)>`, and the /media/<basename> requests this process served
// (size, seed). Multipart parts are checked at CompleteMultipartUpload, when their offsets are
// known. Counters: verify_objects / verify_bytes / verify_mismatches / verify_unknown.
//
// Payload checksums are verified whatever the sink: `x-amz-checksum-crc32c` as a header or as
// an aws-chunked trailer (`x-amz-trailer`, `Content-Encoding: aws-chunked`), and `Content-MD5`;
// a mismatch is answered 400 BadDigest and nothing is stored. --s3-corrupt-rate P flips one
// byte of that share of checksummed bodies on arrival (transit corruption, fault injection).
// --crc-check N recomputes the CRC32C of a deterministic 1-in-N subset of the checksummed
// bodies (selected by a salted hash of key + part number the sender cannot predict,
// --crc-salt); the others must still carry a well-formed CRC but are dropped in the kernel
// like the sample sink's bytes. The bench's S3 then stops costing the worker's CPU slice a
// full second read of every byte while any wrong CRC the worker sends is still caught with
// probability 1/N per body (counters crc_checked_puts / crc_unchecked_puts / bad_digests).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <fcntl.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/ssl.h>

#include "crc32c.h"

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

struct Object {
  std::string data;  // kept only when small
  uint64_t size = 0;
  uint64_t sum = 0;
  std::string etag;
};

// Sampled window of a body: bytes [pos, pos + bytes.size()) of the PUT payload.
struct Sample {
  uint64_t pos;
  std::string bytes;
};

// What the sample / verify sinks keep of one PUT body until its object offset is known.
struct BodyCheck {
  uint64_t len = 0;
  uint64_t sum = 0;              // verify: CRC32C of every byte
  std::vector<Sample> windows;   // sample
};

struct Upload {
  std::string bucket, key;
  std::map<int, Object> parts;
  std::map<int, BodyCheck> checks;
};

std::mutex g_mu;
std::unordered_map<std::string, std::map<std::string, Object>> g_buckets;
std::unordered_map<std::string, Upload> g_uploads;
std::unordered_map<std::string, int> g_fail_counts;
std::atomic<uint64_t> g_rx{0}, g_tx{0}, g_reqs{0}, g_objects{0}, g_upload_seq{1};
std::vector<uint8_t> g_pool;  // random pool the origin serves from
size_t g_keep_bytes = 1 << 20;
enum SinkMode { kSinkChecksum, kSinkDiscard, kSinkSample, kSinkVerify };
SinkMode g_sink = kSinkChecksum;
bool g_discard = false;     // large bodies dropped in the kernel (--sink discard | sample)
uint64_t g_sample_stride = 1 << 20, g_sample_len = 4096;
double g_s3_corrupt_rate = 0;
std::mutex g_media_mu;
std::unordered_map<std::string, std::pair<uint64_t, uint64_t>> g_media;  // basename -> size, seed
std::atomic<uint64_t> g_verify_objects{0}, g_verify_bytes{0}, g_verify_mismatch{0},
    g_verify_unknown{0}, g_bad_digest{0}, g_checksummed{0}, g_corrupted{0}, g_parts{0},
    g_mp_objects{0}, g_mp_parts{0};
int g_pool_fd = -1;         // memfd holding the origin pool (sendfile source)
std::string g_files_root;  // --files-root: GET|HEAD /files/<path> served with sendfile (webseeds)
uint64_t g_default_size = 100ull << 20;
SSL_CTX* g_tls = nullptr;  // --tls-cert / --tls-key
std::string g_synth_bucket;                       // --synth-bucket
// --synth-files FILE ("<path> <size> <seed>" lines): webseed files under /files/<path> whose
// bytes are the origin pool's (no disk, sendfile from the pool's memfd)
std::unordered_map<std::string, std::pair<uint64_t, uint64_t>> g_synth_files;
std::map<std::string, uint64_t> g_synth_objects;  // key -> size (--synth-manifest)
uint64_t g_synth_shift = 0;  // --synth-shift B: webseed files served B bytes off (fault tests)
double g_s3_fail_rate = 0;  // --s3-fail-rate: this share of object/part PUTs answer 503 SlowDown
std::atomic<uint64_t> g_s3_faults{0};
uint64_t g_crc_check = 1;        // --crc-check N: recompute 1 in N checksummed bodies
int g_rcvlowat = 0;              // --rcvlowat KB: SO_RCVLOWAT of the sink's kernel drops
uint64_t g_crc_salt = 0;         // --crc-salt S (default: random per run)
std::atomic<uint64_t> g_crc_checked{0}, g_crc_unchecked{0}, g_media_puts{0}, g_media_puts_crc{0};

// Pool period: 64 MiB + one 4 KiB page. A period that divided the multipart part size (64 MiB)
// or the torrent piece length (4 MiB) would make a part fetched with another part's Range, or
// a webseed read shifted by whole parts, carry the very bytes it should: with 16385 pages
// (odd, so coprime with every power of two) an offset error of k x 4 MiB aliases only when
// k is a multiple of 16385 (64 GiB). Every rule below (origin, webseeds, sink compare,
// bench/synth_torrent.py) uses this one constant.
#ifndef BLOBD_POOL_BYTES      // (-D only to rebuild the round-5 generator for the A/B test)
#define BLOBD_POOL_BYTES ((64ull << 20) + 4096)
#endif
constexpr size_t kPool = BLOBD_POOL_BYTES;

uint64_t mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  return h * 0xff51afd7ed558ccdull;
}

// Order-dependent 64-bit checksum of a byte stream fed in arbitrary chunk sizes:
// processes whole 8-byte words; carries a partial word between calls.
struct Summer {
  uint64_t h = 0x12345678ull, carry = 0;
  int nc = 0;
  void feed(const uint8_t* p, size_t n) {
    while (n && nc) {
      carry |= (uint64_t)*p++ << (8 * nc);
      --n;
      if (++nc == 8) {
        h = mix(h, carry);
        carry = 0;
        nc = 0;
      }
    }
    size_t w = n / 8;
    for (size_t i = 0; i < w; ++i) {
      uint64_t v;
      memcpy(&v, p + 8 * i, 8);
      h = mix(h, v);
    }
    p += 8 * w;
    n -= 8 * w;
    while (n--) carry |= (uint64_t)*p++ << (8 * nc++);
  }
  uint64_t final() const { return nc ? mix(h, carry ^ ((uint64_t)nc << 56)) : h; }
};

// Is the CRC32C of this body (`key`, multipart part number or 0) recomputed? A salted hash,
// so the subset is fixed for a run but not known to the sender.
bool crc_selected(const std::string& key, int part) {
  if (g_crc_check <= 1) return true;
  uint64_t h = 0xcbf29ce484222325ull;
  for (unsigned char ch : key) h = (h ^ ch) * 0x100000001b3ull;
  h = mix(mix(g_crc_salt, h), (uint64_t)(uint32_t)part);
  return (h >> 17) % g_crc_check == 0;
}

std::string hex64(uint64_t a, uint64_t b) {
  char buf[40];
  snprintf(buf, sizeof buf, "%016" PRIx64 "%016" PRIx64, a, b);
  return buf;
}

std::string url_decode(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size()) {
      o.push_back((char)strtol(s.substr(i + 1, 2).c_str(), nullptr, 16));
      i += 2;
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

std::string xml_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '&') o += "&amp;";
    else if (c == '<') o += "&lt;";
    else if (c == '>') o += "&gt;";
    else o.push_back(c);
  }
  return o;
}

bool b64_decode(const std::string& in, std::string& out) {
  static int8_t T[256];
  static bool init = [] {
    memset(T, -1, sizeof T);
    const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) T[(uint8_t)A[i]] = (int8_t)i;
    return true;
  }();
  (void)init;
  out.clear();
  uint32_t acc = 0;
  int bits = 0;
  for (char ch : in) {
    if (ch == '=') break;
    int v = T[(uint8_t)ch];
    if (v < 0) return false;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((char)((acc >> bits) & 0xff));
    }
  }
  return true;
}

// Origin object behind a staged key `<id>/original/<base64(basename)>` (the key layout of
// lib/upload.js:43-45): false for keys of another shape and for the done marker.
bool media_of_key(const std::string& key, uint64_t& size, uint64_t& seed, bool& media_like) {
  media_like = false;
  size_t p = key.find("/original/");
  if (p == std::string::npos) return false;
  std::string enc = key.substr(p + 10), name;
  if (enc == "done" || enc.empty()) return false;
  media_like = true;
  if (!b64_decode(enc, name)) return false;
  std::lock_guard<std::mutex> lk(g_media_mu);
  auto it = g_media.find(name);
  if (it == g_media.end()) return false;
  size = it->second.first;
  seed = it->second.second;
  return true;
}

inline const uint8_t* pool_at(uint64_t o, uint64_t seed, uint64_t& avail) {
  uint64_t po = (o + seed * 7919ull) % kPool;
  avail = kPool - po;
  return g_pool.data() + po;
}

// Does `chk` (a body received for bytes [off, off + chk.len) of the object with `seed`) match
// what the origin generated for that range?
bool check_range(const BodyCheck& chk, uint64_t off, uint64_t seed) {
  if (g_sink == kSinkVerify) {    // CRC32C of the generated range vs of the received body
    uint32_t c = 0;
    uint64_t o = off, left = chk.len;
    while (left) {
      uint64_t avail;
      const uint8_t* p = pool_at(o, seed, avail);
      uint64_t k = std::min(left, avail);
      c = crc32c_update(c, p, (size_t)k);
      o += k;
      left -= k;
    }
    g_verify_bytes += chk.len;
    return c == (uint32_t)chk.sum;
  }
  for (const Sample& w : chk.windows) {
    uint64_t o = off + w.pos, i = 0;
    while (i < w.bytes.size()) {
      uint64_t avail;
      const uint8_t* p = pool_at(o + i, seed, avail);
      uint64_t k = std::min<uint64_t>(w.bytes.size() - i, avail);
      if (memcmp(p, w.bytes.data() + i, (size_t)k) != 0) return false;
      i += k;
    }
    g_verify_bytes += w.bytes.size();
  }
  return true;
}

// Consumer of one request body's payload bytes (after any aws-chunked framing is removed):
// checksum fold, small-body capture, CRC32C / MD5 of payload checksums, sampled windows.
struct Consumer {
  Summer sum;
  bool fold = false;
  std::string* out = nullptr;
  size_t keep = 0;
  bool crc_on = false;
  uint32_t crc = 0;
  EVP_MD_CTX* md5 = nullptr;
  std::vector<Sample>* windows = nullptr;   // sample sink
  bool vcrc_on = false;                     // verify sink: CRC32C of every byte
  uint32_t vcrc = 0;
  uint64_t total = 0;                       // payload length (window layout)
  int64_t corrupt_at = -1;                  // fault injection: flip this payload byte
  ~Consumer() {
    if (md5) EVP_MD_CTX_free(md5);
  }
  bool needs_all() const { return fold || crc_on || vcrc_on || md5 != nullptr || out != nullptr; }
  uint64_t tail_start() const { return total > g_sample_len ? total - g_sample_len : 0; }
  bool in_window(uint64_t pos) const {
    return pos % g_sample_stride < g_sample_len || pos >= tail_start();
  }
  uint64_t window_end(uint64_t pos) const {      // pos in a window
    if (pos >= tail_start()) return total;
    uint64_t e = pos - pos % g_sample_stride + g_sample_len;
    return e >= tail_start() ? total : std::min(e, total);
  }
  uint64_t next_window(uint64_t pos) const {     // pos outside every window
    return std::min({(pos / g_sample_stride + 1) * g_sample_stride, tail_start(), total});
  }
  void sample(uint64_t pos, const uint8_t* p, size_t k) {
    while (k) {
      if (in_window(pos)) {
        size_t t = (size_t)std::min<uint64_t>(k, window_end(pos) - pos);
        if (!windows->empty() && windows->back().pos + windows->back().bytes.size() == pos)
          windows->back().bytes.append((const char*)p, t);
        else
          windows->push_back(Sample{pos, std::string((const char*)p, t)});
        pos += t;
        p += t;
        k -= t;
      } else {
        size_t t = (size_t)std::min<uint64_t>(k, next_window(pos) - pos);
        pos += t;
        p += t;
        k -= t;
      }
    }
  }
  void feed_raw(uint64_t pos, const uint8_t* p, size_t k) {
    if (fold) sum.feed(p, k);
    if (out && out->size() < keep) out->append((const char*)p, std::min(k, keep - out->size()));
    if (crc_on) crc = crc32c_update(crc, p, k);
    if (vcrc_on) vcrc = crc32c_update(vcrc, p, k);
    if (md5) EVP_DigestUpdate(md5, p, k);
    if (windows) sample(pos, p, k);
  }
  void feed(uint64_t pos, const uint8_t* p, size_t k) {
    if (corrupt_at >= 0 && (uint64_t)corrupt_at >= pos && (uint64_t)corrupt_at < pos + k) {
      size_t i = (size_t)((uint64_t)corrupt_at - pos);
      uint8_t flipped = p[i] ^ 0x01;
      feed_raw(pos, p, i);
      feed_raw(pos + i, &flipped, 1);
      feed_raw(pos + i + 1, p + i + 1, k - i - 1);
      corrupt_at = -1;
      g_corrupted++;
      return;
    }
    feed_raw(pos, p, k);
  }
};

// Parts (in part-number order) of one staged object against its origin object.
void verify_object(const std::vector<BodyCheck>& parts, bool known, uint64_t size, uint64_t seed) {
  if (!known) {
    g_verify_unknown++;
    return;
  }
  uint64_t off = 0;
  bool ok = true;
  for (const BodyCheck& c : parts) {
    if (g_sink == kSinkVerify || !c.windows.empty() || c.len == 0) {
      if (!check_range(c, off, seed)) ok = false;
    } else {
      ok = false;   // a part that arrived before the check was set up: unplaceable
    }
    off += c.len;
  }
  if (off != size) ok = false;
  g_verify_objects++;
  if (!ok) g_verify_mismatch++;
}

struct Request {
  std::string method, path, query;
  std::map<std::string, std::string> q;
  std::map<std::string, std::string> h;
  int64_t content_length = 0;
  bool keep_alive = true;
};

class Conn {
 public:
  explicit Conn(int fd) : fd_(fd), buf_(1 << 20) {}
  ~Conn() {
    if (ssl_) SSL_free(ssl_);
    ::close(fd_);
  }

  void serve() {
    if (g_tls) {
      ssl_ = SSL_new(g_tls);
      if (!ssl_) return;
      SSL_set_fd(ssl_, fd_);
      if (SSL_accept(ssl_) != 1) {
        ERR_clear_error();
        return;
      }
      BIO* sock = SSL_get_wbio(ssl_);  // coalesce 16 KiB records into 256 KiB sends
      BIO* b = BIO_new(BIO_f_buffer());
      if (b && BIO_set_write_buffer_size(b, 256 * 1024) == 1) {
        BIO_up_ref(sock);
        SSL_set0_wbio(ssl_, BIO_push(b, sock));
      } else if (b) {
        BIO_free(b);
      }
    }
    for (;;) {
      Request r;
      if (!read_request(r)) return;
      g_reqs++;
      if (!dispatch(r)) return;
      if (!r.keep_alive) return;
    }
  }

 private:
  bool fill() {
    if (pos_ == end_) pos_ = end_ = 0;
    if (end_ == buf_.size()) {
      memmove(buf_.data(), buf_.data() + pos_, end_ - pos_);
      end_ -= pos_;
      pos_ = 0;
    }
    if (ssl_) {
      int r = SSL_read(ssl_, buf_.data() + end_, (int)(buf_.size() - end_));
      if (r <= 0) {
        ERR_clear_error();
        return false;
      }
      end_ += (size_t)r;
      while (end_ < buf_.size() && SSL_has_pending(ssl_)) {
        r = SSL_read(ssl_, buf_.data() + end_, (int)(buf_.size() - end_));
        if (r <= 0) {
          ERR_clear_error();
          break;
        }
        end_ += (size_t)r;
      }
      return true;
    }
    ssize_t r = ::recv(fd_, buf_.data() + end_, buf_.size() - end_, 0);
    if (r <= 0) return false;
    end_ += (size_t)r;
    return true;
  }

  bool read_request(Request& r) {
    std::string head;
    for (;;) {
      const char* b = (const char*)buf_.data() + pos_;
      size_t n = end_ - pos_;
      const char* e = (const char*)memmem(b, n, "\r\n\r\n", 4);
      if (e) {
        head.assign(b, (size_t)(e - b));
        pos_ += (size_t)(e - b) + 4;
        break;
      }
      if (n > 256 * 1024) return false;
      if (!fill()) return false;
    }
    size_t le = head.find("\r\n");
    std::string line = head.substr(0, le);
    size_t s1 = line.find(' '), s2 = line.rfind(' ');
    if (s1 == std::string::npos || s2 == s1) return false;
    r.method = line.substr(0, s1);
    std::string target = line.substr(s1 + 1, s2 - s1 - 1);
    size_t qm = target.find('?');
    r.path = url_decode(target.substr(0, qm));
    if (qm != std::string::npos) {
      r.query = target.substr(qm + 1);
      size_t i = 0;
      while (i <= r.query.size()) {
        size_t amp = r.query.find('&', i);
        if (amp == std::string::npos) amp = r.query.size();
        std::string kv = r.query.substr(i, amp - i);
        size_t eq = kv.find('=');
        if (!kv.empty())
          r.q[url_decode(kv.substr(0, eq))] = eq == std::string::npos ? "" : url_decode(kv.substr(eq + 1));
        i = amp + 1;
      }
    }
    size_t p = le == std::string::npos ? head.size() : le + 2;
    while (p < head.size()) {
      size_t e = head.find("\r\n", p);
      if (e == std::string::npos) e = head.size();
      std::string hl = head.substr(p, e - p);
      size_t c = hl.find(':');
      if (c != std::string::npos) {
        std::string k = hl.substr(0, c);
        for (auto& ch : k) ch = (char)tolower((unsigned char)ch);
        size_t vs = hl.find_first_not_of(' ', c + 1);
        r.h[k] = vs == std::string::npos ? "" : hl.substr(vs);
      }
      p = e + 2;
    }
    auto it = r.h.find("content-length");
    if (it != r.h.end()) r.content_length = atoll(it->second.c_str());
    it = r.h.find("connection");
    if (it != r.h.end() && strcasestr(it->second.c_str(), "close")) r.keep_alive = false;
    return true;
  }

  // Read `n` plain payload bytes into `c` (payload offset `pos` onwards). Spliced socket ->
  // /dev/null when no consumer needs every byte (discard / sample sinks), reading only the
  // sampled windows into user space.
  bool read_plain(int64_t n, Consumer& c, uint64_t pos = 0) {
    if (pos_ < end_ && n > 0) {
      size_t k = (size_t)std::min<int64_t>(n, (int64_t)(end_ - pos_));
      c.feed(pos, buf_.data() + pos_, k);
      pos_ += k;
      pos += k;
      n -= (int64_t)k;
      g_rx += k;
    }
    if (n == 0) return true;
    if (!c.needs_all() && !ssl_) return discard_plain(n, c, pos);
    while (n > 0) {
      if (pos_ == end_ && !fill()) return false;
      size_t k = (size_t)std::min<int64_t>(n, (int64_t)(end_ - pos_));
      c.feed(pos, buf_.data() + pos_, k);
      pos_ += k;
      pos += k;
      n -= (int64_t)k;
      g_rx += k;
    }
    return true;
  }

  // Bytes nobody needs are dropped in the kernel with recv(MSG_TRUNC) (TCP discards them
  // without copying): no pipe, so the sink holds nothing of the user's pipe page budget
  // (fs.pipe-user-pages-soft, shared with the workers' relays on the same box).
  bool discard_plain(int64_t n, Consumer& c, uint64_t pos) {
    uint8_t win[16384];
    bool lowat_set = false;
    struct Reset {
      int fd;
      bool* on;
      ~Reset() {
        if (*on) {
          int one = 1;
          setsockopt(fd, SOL_SOCKET, SO_RCVLOWAT, &one, sizeof one);
        }
      }
    } reset{fd_, &lowat_set};
    // --rcvlowat: wake for at least this much while more than twice that is still to come
    // (TCP wakes a sleeping reader only once sk_rcvlowat bytes are queued, whatever it asked
    // for: before fewer are left the mark goes back to 1). Checked before every recv.
    auto adjust = [&] {
      const bool want = g_rcvlowat && n > 2 * (int64_t)g_rcvlowat;
      if (want != lowat_set) {
        int v = want ? g_rcvlowat : 1;
        setsockopt(fd_, SOL_SOCKET, SO_RCVLOWAT, &v, sizeof v);
        lowat_set = want;
      }
    };
    while (n > 0) {
      if (c.windows && c.in_window(pos)) {   // a sampled window: recv exactly its bytes
        size_t want = (size_t)std::min<uint64_t>((uint64_t)n, c.window_end(pos) - pos);
        want = std::min(want, sizeof win);
        adjust();
        ssize_t r = ::recv(fd_, win, want, 0);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        c.feed(pos, win, (size_t)r);
        pos += (uint64_t)r;
        n -= r;
        g_rx += (uint64_t)r;
        continue;
      }
      uint64_t stop = c.windows ? std::min<uint64_t>(c.next_window(pos), pos + (uint64_t)n)
                                : pos + (uint64_t)n;
      int64_t run = (int64_t)(stop - pos);

      while (run > 0) {
        // no buffer: TCP drops MSG_TRUNC bytes without copying (and a 16 KiB one with a
        // longer length trips _FORTIFY_SOURCE's recv check)
        adjust();
        ssize_t in = ::recv(fd_, nullptr, (size_t)std::min<int64_t>(run, 1 << 20), MSG_TRUNC);
        if (in < 0 && errno == EINTR) continue;
        if (in <= 0) return false;
        run -= in;
        n -= in;
        pos += (uint64_t)in;
        g_rx += (uint64_t)in;
      }
    }
    return true;
  }

  // Control bodies (bucket ops, complete XML, refused PUTs): into user space unless large
  // and the sink discards.
  bool read_body(int64_t n, Summer& s, std::string* out, size_t keep) {
    Consumer c;
    const bool big = g_discard && n > (int64_t)keep;
    c.fold = !big;
    c.out = big ? nullptr : out;
    c.keep = keep;
    if (!read_plain(n, c, 0)) return false;
    s = c.sum;
    return true;
  }

  bool get_line(std::string& line, size_t max = 8192) {
    for (;;) {
      const char* b = (const char*)buf_.data() + pos_;
      size_t n = end_ - pos_;
      const char* e = (const char*)memmem(b, n, "\r\n", 2);
      if (e) {
        line.assign(b, (size_t)(e - b));
        pos_ += (size_t)(e - b) + 2;
        return true;
      }
      if (n > max) return false;
      if (!fill()) return false;
    }
  }

  // aws-chunked payload: `<hex>[;ext]\r\n<data>\r\n` ... `0\r\n<trailer lines>\r\n\r\n`.
  bool read_aws_chunked(Consumer& c, uint64_t& data_len, std::map<std::string, std::string>& trailers) {
    data_len = 0;
    std::string line;
    for (;;) {
      if (!get_line(line)) return false;
      std::string hx = line.substr(0, line.find(';'));
      char* endp = nullptr;
      uint64_t k = strtoull(hx.c_str(), &endp, 16);
      if (hx.empty() || (endp && *endp)) return false;
      if (k == 0) {
        for (;;) {
          if (!get_line(line)) return false;
          if (line.empty()) return true;
          size_t colon = line.find(':');
          if (colon == std::string::npos) continue;
          std::string name = line.substr(0, colon);
          for (auto& ch : name) ch = (char)tolower((unsigned char)ch);
          size_t vs = line.find_first_not_of(' ', colon + 1);
          trailers[name] = vs == std::string::npos ? "" : line.substr(vs);
        }
      }
      // buffered bytes first, then the socket: dropped in the kernel (windows aside) when
      // nothing needs every byte (a body outside the --crc-check subset on a discarding sink)
      if (!read_plain((int64_t)k, c, data_len)) return false;
      data_len += k;
      if (!get_line(line) || !line.empty()) return false;
    }
  }

  static bool aws_chunked(const Request& r) {
    auto it = r.h.find("content-encoding");
    return it != r.h.end() && strcasestr(it->second.c_str(), "aws-chunked") != nullptr;
  }

  static uint64_t payload_len(const Request& r) {
    if (!aws_chunked(r)) return (uint64_t)std::max<int64_t>(0, r.content_length);
    auto it = r.h.find("x-amz-decoded-content-length");
    return it == r.h.end() ? 0 : strtoull(it->second.c_str(), nullptr, 10);
  }

  // Consume a refused PUT's payload, whatever its encoding.
  bool skip_payload(const Request& r) {
    Consumer c;
    if (aws_chunked(r)) {
      uint64_t got;
      std::map<std::string, std::string> tr;
      return read_aws_chunked(c, got, tr);
    }
    return read_plain(r.content_length, c, 0);
  }

  bool send_all(const void* p, size_t n) {
    const char* c = (const char*)p;
    if (ssl_) {
      while (n) {
        int w = SSL_write(ssl_, c, (int)std::min<size_t>(n, (size_t)1 << 30));
        if (w <= 0) {
          ERR_clear_error();
          return false;
        }
        c += w;
        n -= (size_t)w;
      }
      return BIO_flush(SSL_get_wbio(ssl_)) > 0;
    }
    while (n) {
      ssize_t w = ::send(fd_, c, n, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      c += w;
      n -= (size_t)w;
    }
    return true;
  }

  bool respond(int status, const char* reason, const std::string& body,
               const std::string& extra = "", const char* ctype = "application/xml",
               bool head_only = false) {
    char hdr[512];
    int n = snprintf(hdr, sizeof hdr,
                     "HTTP/1.1 %d %s\r\nServer: blobd\r\nContent-Type: %s\r\nContent-Length: %zu\r\n",
                     status, reason, ctype, body.size());
    std::string out(hdr, (size_t)n);
    out += extra;
    out += "\r\n";
    if (!head_only) out += body;
    return send_all(out.data(), out.size());
  }

  bool s3_error(int status, const char* reason, const char* code, const std::string& res) {
    return respond(status, reason,
                   std::string("<?xml version=\"1.0\" encoding=\"UTF-8\"?><Error><Code>") + code +
                       "</Code><Message>" + code + "</Message><Resource>" + xml_escape(res) +
                       "</Resource></Error>");
  }

  bool origin(const Request& r) {
    uint64_t size = g_default_size, seed = 0;
    // ?fail=N : the first N GETs of this exact URL answer 503 (retry-path fault injection)
    auto fit = r.q.find("fail");
    if (fit != r.q.end() && r.method == "GET") {
      std::lock_guard<std::mutex> lk(g_mu);
      int& seen = g_fail_counts[r.path + "?" + r.query];
      if (seen < atoi(fit->second.c_str())) {
        ++seen;
        return respond(503, "Service Unavailable", "injected", "", "text/plain");
      }
    }
    auto it = r.q.find("size");
    if (it != r.q.end()) size = strtoull(it->second.c_str(), nullptr, 10);
    it = r.q.find("seed");
    if (it != r.q.end()) seed = strtoull(it->second.c_str(), nullptr, 10);
    if ((g_sink == kSinkSample || g_sink == kSinkVerify) && r.path.rfind("/media/", 0) == 0) {
      std::lock_guard<std::mutex> lk(g_media_mu);  // what a staged copy of it must contain
      g_media[r.path.substr(7)] = {size, seed};
    }
    return serve_pool(r, size, seed, "Content-Type: video/x-matroska\r\n");
  }

  // GET|HEAD (with Range) of a synthetic object: byte o = pool[(o + seed * 7919) % kPool].
  bool serve_pool(const Request& r, uint64_t size, uint64_t seed, const char* ctype,
                  uint64_t shift = 0) {
    uint64_t start = 0, end = size ? size - 1 : 0;
    bool ranged = false;
    auto it = r.h.find("range");
    if (it != r.h.end() && it->second.rfind("bytes=", 0) == 0) {
      std::string spec = it->second.substr(6);
      size_t dash = spec.find('-');
      std::string a = spec.substr(0, dash), b = spec.substr(dash + 1);
      if (a.empty()) {
        uint64_t suf = strtoull(b.c_str(), nullptr, 10);
        start = size > suf ? size - suf : 0;
      } else {
        start = strtoull(a.c_str(), nullptr, 10);
        if (!b.empty()) end = std::min<uint64_t>(strtoull(b.c_str(), nullptr, 10), size - 1);
      }
      ranged = true;
      if (start > end || start >= size)
        return respond(416, "Range Not Satisfiable", "", "Content-Range: bytes */" + std::to_string(size) + "\r\n");
    }
    uint64_t len = size ? end - start + 1 : 0;
    char hdr[512];
    int n = snprintf(hdr, sizeof hdr,
                     "HTTP/1.1 %d %s\r\nServer: blobd\r\n%s"
                     "Accept-Ranges: bytes\r\nContent-Length: %" PRIu64 "\r\n",
                     ranged ? 206 : 200, ranged ? "Partial Content" : "OK", ctype, len);
    std::string out(hdr, (size_t)n);
    if (ranged)
      out += "Content-Range: bytes " + std::to_string(start) + "-" + std::to_string(end) + "/" +
             std::to_string(size) + "\r\n";
    out += "\r\n";
    if (!send_all(out.data(), out.size())) return false;
    if (r.method == "HEAD") return true;
    // Object byte at offset o = pool[(o + seed * 7919) % kPool]; the pool lives in a memfd so
    // the body goes out with sendfile (page references, no user-space copy).
    uint64_t o = start + shift, left = len;
    while (left) {
      uint64_t po = (o + seed * 7919ull) % kPool;
      size_t k = (size_t)std::min<uint64_t>(left, std::min<uint64_t>(kPool - po, 4ull << 20));
      if (g_pool_fd >= 0 && !ssl_) {
        off_t fo = (off_t)po;
        size_t sent = 0;
        while (sent < k) {
          ssize_t w = ::sendfile(fd_, g_pool_fd, &fo, k - sent);
          if (w < 0 && errno == EINTR) continue;
          if (w <= 0) return false;
          sent += (size_t)w;
        }
      } else if (!send_all(g_pool.data() + po, k)) {
        return false;
      }
      g_tx += k;
      o += k;
      left -= k;
    }
    return true;
  }

  // Static files for BEP-19 webseeds: Range support, zero-copy sendfile from the page cache.
  bool files(const Request& r) {
    std::string rel = r.path.substr(7);
    auto sy = g_synth_files.find(rel);      // a synthetic file (--synth-files): the origin pool
    if (sy != g_synth_files.end())
      return serve_pool(r, sy->second.first, sy->second.second, "", g_synth_shift);
    if (g_files_root.empty() || rel.find("..") != std::string::npos)
      return respond(404, "Not Found", "no such file", "", "text/plain");
    std::string full = g_files_root + "/" + rel;
    int fd = ::open(full.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return respond(404, "Not Found", "no such file", "", "text/plain");
    struct stat st;
    fstat(fd, &st);
    uint64_t size = (uint64_t)st.st_size, start = 0, end = size ? size - 1 : 0;
    bool ranged = false;
    auto it = r.h.find("range");
    if (it != r.h.end() && it->second.rfind("bytes=", 0) == 0) {
      std::string spec = it->second.substr(6);
      size_t dash = spec.find('-');
      std::string a = spec.substr(0, dash), b = spec.substr(dash + 1);
      start = a.empty() ? (size > strtoull(b.c_str(), nullptr, 10) ? size - strtoull(b.c_str(), nullptr, 10) : 0)
                        : strtoull(a.c_str(), nullptr, 10);
      if (!a.empty() && !b.empty()) end = std::min<uint64_t>(strtoull(b.c_str(), nullptr, 10), size - 1);
      ranged = true;
      if (start > end || start >= size) {
        ::close(fd);
        return respond(416, "Range Not Satisfiable", "", "", "text/plain");
      }
    }
    uint64_t len = size ? end - start + 1 : 0;
    char hdr[512];
    int n = snprintf(hdr, sizeof hdr,
                     "HTTP/1.1 %d %s\r\nServer: blobd\r\nAccept-Ranges: bytes\r\nContent-Length: %" PRIu64 "\r\n",
                     ranged ? 206 : 200, ranged ? "Partial Content" : "OK", len);
    std::string out(hdr, (size_t)n);
    if (ranged)
      out += "Content-Range: bytes " + std::to_string(start) + "-" + std::to_string(end) + "/" +
             std::to_string(size) + "\r\n";
    out += "\r\n";
    bool ok = send_all(out.data(), out.size());
    if (ok && r.method != "HEAD") {
      off_t o = (off_t)start;
      uint64_t left = len;
      std::vector<uint8_t> tb(ssl_ ? 256 * 1024 : 0);
      while (ok && left && ssl_) {
        ssize_t k = ::pread(fd, tb.data(), (size_t)std::min<uint64_t>(left, tb.size()), o);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0 || !send_all(tb.data(), (size_t)k)) {
          ok = false;
        } else {
          o += k;
          left -= (uint64_t)k;
          g_tx += (uint64_t)k;
        }
      }
      while (ok && left) {
        ssize_t w = ::sendfile(fd_, fd, &o, (size_t)std::min<uint64_t>(left, 8u << 20));
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) ok = false;
        else {
          left -= (uint64_t)w;
          g_tx += (uint64_t)w;
        }
      }
    }
    ::close(fd);
    return ok;
  }

  // Read-only synthetic source bucket: object bytes are the origin pool at an offset derived
  // from the key, so any Range of any object is reproducible without storing it.
  bool synth(const Request& r, const std::string& key) {
    if (key.empty()) {
      if (r.method == "HEAD") return respond(200, "OK", "", "", "application/xml", true);
      std::string prefix = r.q.count("prefix") ? r.q.at("prefix") : "";
      std::string body = "<?xml version=\"1.0\" encoding=\"UTF-8\"?><ListBucketResult><Name>" +
                         g_synth_bucket + "</Name><IsTruncated>false</IsTruncated>";
      for (auto& kv : g_synth_objects)
        if (kv.first.compare(0, prefix.size(), prefix) == 0)
          body += "<Contents><Key>" + xml_escape(kv.first) + "</Key><Size>" +
                  std::to_string(kv.second) + "</Size></Contents>";
      body += "</ListBucketResult>";
      return respond(200, "OK", body);
    }
    auto it = g_synth_objects.find(key);
    if (it == g_synth_objects.end()) return s3_error(404, "Not Found", "NoSuchKey", key);
    Request o = r;
    o.q["size"] = std::to_string(it->second);
    o.q["seed"] = std::to_string(std::hash<std::string>{}(key) % 100000);
    o.q.erase("fail");
    return origin(o);
  }

  bool s3(const Request& r) {
    std::string p = r.path.substr(1);
    size_t sl = p.find('/');
    std::string bucket = p.substr(0, sl), key = sl == std::string::npos ? "" : p.substr(sl + 1);
    const std::string& m = r.method;
    if (!g_synth_bucket.empty() && bucket == g_synth_bucket && (m == "GET" || m == "HEAD"))
      return synth(r, key);
    if (bucket.empty()) return s3_error(400, "Bad Request", "InvalidBucketName", r.path);
    if (key.empty()) {
      if (r.content_length > 0) {
        Summer s;
        if (!read_body(r.content_length, s, nullptr, 0)) return false;
      }
      std::lock_guard<std::mutex> lk(g_mu);
      bool exists = g_buckets.count(bucket) > 0;
      if (m == "HEAD") return respond(exists ? 200 : 404, exists ? "OK" : "Not Found", "", "", "application/xml", true);
      if (m == "PUT") {
        if (exists) return s3_error(409, "Conflict", "BucketAlreadyOwnedByYou", bucket);
        g_buckets[bucket];
        return respond(200, "OK", "");
      }
      if (!exists) return s3_error(404, "Not Found", "NoSuchBucket", bucket);
      if (m == "GET" && r.q.count("uploads")) {   // ListMultipartUploads (one page)
        std::string prefix = r.q.count("prefix") ? r.q.at("prefix") : "";
        std::string body = "<?xml version=\"1.0\" encoding=\"UTF-8\"?><ListMultipartUploadsResult><Bucket>" +
                           bucket + "</Bucket><IsTruncated>false</IsTruncated>";
        for (auto& kv : g_uploads)
          if (kv.second.bucket == bucket && kv.second.key.compare(0, prefix.size(), prefix) == 0)
            body += "<Upload><Key>" + xml_escape(kv.second.key) + "</Key><UploadId>" + kv.first +
                    "</UploadId></Upload>";
        body += "</ListMultipartUploadsResult>";
        return respond(200, "OK", body);
      }
      if (m == "GET") {
        std::string prefix = r.q.count("prefix") ? r.q.at("prefix") : "";
        std::string body = "<?xml version=\"1.0\" encoding=\"UTF-8\"?><ListBucketResult><Name>" + bucket +
                           "</Name><IsTruncated>false</IsTruncated>";
        for (auto& kv : g_buckets[bucket])
          if (kv.first.compare(0, prefix.size(), prefix) == 0)
            body += "<Contents><Key>" + xml_escape(kv.first) + "</Key><Size>" + std::to_string(kv.second.size) +
                    "</Size><ETag>&quot;" + kv.second.etag + "&quot;</ETag></Contents>";
        body += "</ListBucketResult>";
        return respond(200, "OK", body);
      }
      return s3_error(405, "Method Not Allowed", "MethodNotAllowed", bucket);
    }
    // ---- object level
    if (m == "PUT" && r.h.count("x-amz-copy-source")) {  // no server-side copy here: say so
      if (!skip_payload(r)) return false;
      return s3_error(501, "Not Implemented", "NotImplemented", key);
    }
    thread_local std::mt19937_64 rng(std::random_device{}());
    if (m == "PUT" && g_s3_fail_rate > 0) {
      if (std::uniform_real_distribution<double>(0, 1)(rng) < g_s3_fail_rate) {
        if (!skip_payload(r)) return false;
        g_s3_faults++;
        return s3_error(503, "Slow Down", "SlowDown", key);
      }
    }
    if (m == "PUT") {
      const bool part = r.q.count("uploadId") > 0;
      const uint64_t dlen = payload_len(r);
      const bool chunked = aws_chunked(r);
      Object o;
      BodyCheck chk;
      Consumer c;
      auto hc = r.h.find("x-amz-checksum-crc32c");
      auto tr = r.h.find("x-amz-trailer");
      const bool trailer_crc =
          tr != r.h.end() && strcasestr(tr->second.c_str(), "x-amz-checksum-crc32c") != nullptr;
      auto hm = r.h.find("content-md5");
      const bool has_crc = hc != r.h.end() || trailer_crc;
      const int part_no = part ? atoi(r.q.count("partNumber") ? r.q.at("partNumber").c_str() : "0") : 0;
      c.crc_on = has_crc && crc_selected(key, part_no);
      if (has_crc) (c.crc_on ? g_crc_checked : g_crc_unchecked)++;
      if (hm != r.h.end()) {
        c.md5 = EVP_MD_CTX_new();
        EVP_DigestInit_ex(c.md5, EVP_md5(), nullptr);
      }
      const bool small = dlen <= g_keep_bytes;
      c.fold = small || g_sink == kSinkChecksum;
      if (small) {
        c.out = &o.data;
        c.keep = g_keep_bytes;
      }
      const bool checking = g_sink == kSinkSample || g_sink == kSinkVerify;
      if (key.find("/original/") != std::string::npos &&
          !(key.size() >= 5 && key.compare(key.size() - 5, 5, "/done") == 0)) {
        g_media_puts++;
        if (has_crc) g_media_puts_crc++;
      }
      bool media_like = false, known = false;
      uint64_t msize = 0, mseed = 0;
      if (checking) {
        known = !part && media_of_key(key, msize, mseed, media_like);
        if (part) media_like = key.find("/original/") != std::string::npos;
        if (g_sink == kSinkSample && media_like) {
          c.windows = &chk.windows;
          c.total = dlen;
        }
        if (g_sink == kSinkVerify && media_like) c.vcrc_on = true;
      }
      if ((c.crc_on || c.md5) && g_s3_corrupt_rate > 0 && dlen > 0 &&
          std::uniform_real_distribution<double>(0, 1)(rng) < g_s3_corrupt_rate)
        c.corrupt_at = (int64_t)(dlen / 2);
      uint64_t got = 0;
      std::map<std::string, std::string> trailers;
      if (chunked) {
        if (!read_aws_chunked(c, got, trailers)) return false;
      } else {
        if (!read_plain(r.content_length, c, 0)) return false;
        got = (uint64_t)std::max<int64_t>(0, r.content_length);
      }
      std::string extra;
      if (has_crc || c.md5) g_checksummed++;
      if (chunked && got != dlen) return s3_error(400, "Bad Request", "IncompleteBody", key);
      if (has_crc && !c.crc_on) {     // not recomputed: it must still be there, well-formed
        const std::string& v = hc != r.h.end() ? hc->second : trailers["x-amz-checksum-crc32c"];
        std::string raw;
        if (v.size() != 8 || !b64_decode(v, raw) || raw.size() != 4) {
          g_bad_digest++;
          return s3_error(400, "Bad Request", "InvalidDigest", key);
        }
        extra += "x-amz-checksum-crc32c: " + v + "\r\n";
      }
      if (c.crc_on) {
        char b[9];
        crc32c_b64(c.crc, b);
        const std::string want = hc != r.h.end() ? hc->second : trailers["x-amz-checksum-crc32c"];
        if (want != b) {
          g_bad_digest++;
          return s3_error(400, "Bad Request", "BadDigest", key);
        }
        extra += std::string("x-amz-checksum-crc32c: ") + b + "\r\n";
      }
      if (c.md5) {
        unsigned char d[EVP_MAX_MD_SIZE];
        unsigned int dl = 0;
        EVP_DigestFinal_ex(c.md5, d, &dl);
        unsigned char enc[64];
        int el = EVP_EncodeBlock(enc, d, (int)dl);
        if (hm->second != std::string((const char*)enc, (size_t)el)) {
          g_bad_digest++;
          return s3_error(400, "Bad Request", "BadDigest", key);
        }
      }
      if (!small) o.data.clear();
      o.size = got;
      o.sum = c.vcrc_on && !c.fold ? c.vcrc : c.sum.final();
      o.etag = hex64(o.sum, o.size);
      chk.len = got;
      chk.sum = c.vcrc;
      extra = "ETag: \"" + o.etag + "\"\r\n" + extra;
      if (part) {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_uploads.find(r.q.at("uploadId"));
        if (it == g_uploads.end()) return s3_error(404, "Not Found", "NoSuchUpload", key);
        int num = part_no;
        it->second.parts[num] = std::move(o);
        if (checking && media_like) it->second.checks[num] = std::move(chk);
        g_parts++;
        return respond(200, "OK", "", extra);
      }
      {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_buckets.count(bucket)) return s3_error(404, "Not Found", "NoSuchBucket", bucket);
        g_buckets[bucket][key] = std::move(o);
        g_objects++;
      }
      if (checking && media_like) {
        std::vector<BodyCheck> one;
        one.push_back(std::move(chk));
        verify_object(one, known, msize, mseed);
      }
      return respond(200, "OK", "", extra);
    }
    if (m == "POST") {
      Summer s;
      std::string body;
      if (!read_body(r.content_length, s, &body, 1 << 20)) return false;
      std::string reply;
      std::vector<BodyCheck> checks;
      {
        std::lock_guard<std::mutex> lk(g_mu);
        if (r.q.count("uploads")) {
          std::string id = "up" + std::to_string(g_upload_seq++);
          g_uploads[id] = Upload{bucket, key, {}, {}};
          return respond(200, "OK",
                         "<?xml version=\"1.0\" encoding=\"UTF-8\"?><InitiateMultipartUploadResult><Bucket>" +
                             bucket + "</Bucket><Key>" + xml_escape(key) + "</Key><UploadId>" + id +
                             "</UploadId></InitiateMultipartUploadResult>");
        }
        auto up = r.q.find("uploadId");
        if (up == r.q.end()) return s3_error(400, "Bad Request", "InvalidRequest", key);
        auto it = g_uploads.find(up->second);
        if (it == g_uploads.end()) return s3_error(404, "Not Found", "NoSuchUpload", key);
        Object o;
        uint64_t h = 0x5bd1e995ull;
        for (auto& kv : it->second.parts) {
          o.size += kv.second.size;
          h = mix(h, kv.second.sum);
          if (o.size <= g_keep_bytes) o.data += kv.second.data;
        }
        if (o.size > g_keep_bytes) o.data.clear();
        o.sum = h;
        o.etag = hex64(h, o.size) + "-" + std::to_string(it->second.parts.size());
        g_mp_objects++;
        g_mp_parts += it->second.parts.size();
        for (auto& kv : it->second.parts) {   // a part without a check cannot be placed
          auto ck = it->second.checks.find(kv.first);
          checks.push_back(ck == it->second.checks.end() ? BodyCheck{kv.second.size, 0, {}}
                                                         : std::move(ck->second));
        }
        std::string et = o.etag;
        g_buckets[bucket][key] = std::move(o);
        g_uploads.erase(it);
        g_objects++;
        reply = "<?xml version=\"1.0\" encoding=\"UTF-8\"?><CompleteMultipartUploadResult><Bucket>" +
                bucket + "</Bucket><Key>" + xml_escape(key) + "</Key><ETag>&quot;" + et +
                "&quot;</ETag></CompleteMultipartUploadResult>";
      }
      if (g_sink == kSinkSample || g_sink == kSinkVerify) {   // offsets are known now
        bool media_like = false;
        uint64_t msize = 0, mseed = 0;
        bool known = media_of_key(key, msize, mseed, media_like);
        if (media_like) verify_object(checks, known, msize, mseed);
      }
      return respond(200, "OK", reply);
    }
    if (r.content_length > 0) {
      Summer s;
      if (!read_body(r.content_length, s, nullptr, 0)) return false;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if (m == "DELETE") {
      auto up = r.q.find("uploadId");
      if (up != r.q.end()) g_uploads.erase(up->second);
      else if (g_buckets.count(bucket)) g_buckets[bucket].erase(key);
      return respond(204, "No Content", "");
    }
    auto b = g_buckets.find(bucket);
    if (b == g_buckets.end()) return s3_error(404, "Not Found", "NoSuchBucket", bucket);
    auto o = b->second.find(key);
    if (o == b->second.end()) {
      if (m == "HEAD") return respond(404, "Not Found", "", "", "application/xml", true);
      return s3_error(404, "Not Found", "NoSuchKey", key);
    }
    std::string extra = "ETag: \"" + o->second.etag + "\"\r\nX-Blobd-Sum: " + std::to_string(o->second.sum) + "\r\n";
    if (m == "HEAD") {
      char hdr[256];
      int n = snprintf(hdr, sizeof hdr, "HTTP/1.1 200 OK\r\nContent-Length: %" PRIu64 "\r\n", o->second.size);
      std::string out(hdr, (size_t)n);
      out += extra + "\r\n";
      return send_all(out.data(), out.size());
    }
    if (o->second.data.size() != o->second.size)
      return s3_error(501, "Not Implemented", "NotStored", key);  // large bodies are not retained
    return respond(200, "OK", o->second.data, extra, "application/octet-stream");
  }

  bool stats() {
    char b[2048];
    size_t nup;
    {
      std::lock_guard<std::mutex> lk(g_mu);
      nup = g_uploads.size();
    }
    const char* sink = g_sink == kSinkDiscard ? "discard" : g_sink == kSinkSample ? "sample"
                       : g_sink == kSinkVerify ? "verify" : "checksum";
    snprintf(b, sizeof b,
             "{\"bytes_received\":%" PRIu64 ",\"bytes_served\":%" PRIu64 ",\"requests\":%" PRIu64
             ",\"objects\":%" PRIu64 ",\"open_uploads\":%zu,\"s3_faults\":%" PRIu64
             ",\"sink\":\"%s\",\"verify_objects\":%" PRIu64 ",\"verify_bytes\":%" PRIu64
             ",\"verify_mismatches\":%" PRIu64 ",\"verify_unknown\":%" PRIu64
             ",\"checksummed_puts\":%" PRIu64 ",\"bad_digests\":%" PRIu64 ",\"corrupted\":%" PRIu64
             ",\"parts\":%" PRIu64 ",\"multipart_objects\":%" PRIu64 ",\"multipart_parts\":%" PRIu64
             ",\"crc_check\":%" PRIu64 ",\"crc_checked_puts\":%" PRIu64 ",\"crc_unchecked_puts\":%" PRIu64
             ",\"media_puts\":%" PRIu64 ",\"media_puts_crc\":%" PRIu64 "}",
             g_rx.load(), g_tx.load(), g_reqs.load(), g_objects.load(), nup, g_s3_faults.load(), sink,
             g_verify_objects.load(), g_verify_bytes.load(), g_verify_mismatch.load(),
             g_verify_unknown.load(), g_checksummed.load(), g_bad_digest.load(), g_corrupted.load(),
             g_parts.load(), g_mp_objects.load(), g_mp_parts.load(), g_crc_check, g_crc_checked.load(),
             g_crc_unchecked.load(), g_media_puts.load(), g_media_puts_crc.load());
    return respond(200, "OK", b, "", "application/json");
  }

  bool dispatch(const Request& r) {
    if (r.path == "/_stats") return stats();
    if (r.path == "/_crc_selected") {
      int part = atoi(r.q.count("part") ? r.q.at("part").c_str() : "0");
      return respond(200, "OK", crc_selected(r.q.count("key") ? r.q.at("key") : "", part) ? "1" : "0",
                     "", "text/plain");
    }
    // the origin pool itself: lets a client build metainfo (piece hashes) for --synth-files
    if (r.path == "/_pool" && r.method == "GET") return serve_pool(r, kPool, 0, "");
    if (r.path.rfind("/media/", 0) == 0 && (r.method == "GET" || r.method == "HEAD")) return origin(r);
    if (r.path.rfind("/files/", 0) == 0 && (r.method == "GET" || r.method == "HEAD")) return files(r);
    return s3(r);
  }

  int fd_;
  SSL* ssl_ = nullptr;
  std::vector<uint8_t> buf_;
  size_t pos_ = 0, end_ = 0;
};

}  // namespace

int main(int argc, char** argv) {
  int port = 0;
  std::string host = "127.0.0.1";
  const char* port_file = nullptr;
  std::string tls_cert, tls_key;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&] { return i + 1 < argc ? argv[++i] : (char*)""; };
    if (a == "--port") port = atoi(next());
    else if (a == "--host") host = next();
    else if (a == "--port-file") port_file = next();
    else if (a == "--keep-bytes") g_keep_bytes = strtoull(next(), nullptr, 10);
    else if (a == "--default-size") g_default_size = strtoull(next(), nullptr, 10);
    else if (a == "--files-root") g_files_root = next();
    else if (a == "--sink") {
      std::string v = next();
      g_sink = v == "discard" ? kSinkDiscard : v == "sample" ? kSinkSample
             : v == "verify" ? kSinkVerify : kSinkChecksum;
      g_discard = g_sink == kSinkDiscard || g_sink == kSinkSample;
    }
    else if (a == "--sample-stride") g_sample_stride = std::max<uint64_t>(1, strtoull(next(), nullptr, 10));
    else if (a == "--sample-len") g_sample_len = std::max<uint64_t>(1, strtoull(next(), nullptr, 10));
    else if (a == "--s3-corrupt-rate") g_s3_corrupt_rate = atof(next());
    else if (a == "--crc-check") g_crc_check = std::max<uint64_t>(1, strtoull(next(), nullptr, 10));
    else if (a == "--crc-salt") g_crc_salt = strtoull(next(), nullptr, 10);
    else if (a == "--synth-shift") g_synth_shift = strtoull(next(), nullptr, 10);
    else if (a == "--rcvlowat") g_rcvlowat = atoi(next()) * 1024;
    else if (a == "--tls-cert") tls_cert = next();
    else if (a == "--tls-key") tls_key = next();
    else if (a == "--s3-fail-rate") g_s3_fail_rate = atof(next());
    else if (a == "--synth-bucket") g_synth_bucket = next();
    else if (a == "--synth-files") {
      FILE* f = fopen(next(), "r");
      char line[4096];
      while (f && fgets(line, sizeof line, f)) {
        std::string l(line);
        while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
        size_t b = l.rfind(' ');
        size_t a2 = b == std::string::npos || b == 0 ? std::string::npos : l.rfind(' ', b - 1);
        if (a2 == std::string::npos) continue;
        g_synth_files[l.substr(0, a2)] = {strtoull(l.c_str() + a2 + 1, nullptr, 10),
                                          strtoull(l.c_str() + b + 1, nullptr, 10)};
      }
      if (f) fclose(f);
    }
    else if (a == "--synth-manifest") {
      FILE* f = fopen(next(), "r");
      char line[4096];
      while (f && fgets(line, sizeof line, f)) {
        std::string l(line);
        size_t sp = l.rfind(' ');
        if (sp == std::string::npos) continue;
        g_synth_objects[l.substr(0, sp)] = strtoull(l.c_str() + sp + 1, nullptr, 10);
      }
      if (f) fclose(f);
    }
    else {
      fprintf(stderr, "usage: blobd [--host H] [--port P] [--port-file F] [--keep-bytes N] "
                      "[--default-size N] [--files-root DIR] [--sink checksum|discard|sample|verify] "
                      "[--sample-stride N] [--sample-len N] [--s3-corrupt-rate P] [--crc-check N] [--crc-salt S] "
                      "[--tls-cert PEM --tls-key PEM] [--s3-fail-rate P]\n");
      return 2;
    }
  }
  if (!tls_cert.empty()) {
    g_tls = SSL_CTX_new(TLS_server_method());
    if (!g_tls || SSL_CTX_use_certificate_chain_file(g_tls, tls_cert.c_str()) != 1 ||
        SSL_CTX_use_PrivateKey_file(g_tls, (tls_key.empty() ? tls_cert : tls_key).c_str(),
                                    SSL_FILETYPE_PEM) != 1) {
      fprintf(stderr, "blobd: cannot load TLS certificate / key\n");
      return 1;
    }
    SSL_CTX_set_min_proto_version(g_tls, TLS1_2_VERSION);
    SSL_CTX_set_options(g_tls, SSL_OP_IGNORE_UNEXPECTED_EOF | SSL_OP_NO_COMPRESSION);
    SSL_CTX_set_read_ahead(g_tls, 1);
    SSL_CTX_set_default_read_buffer_len(g_tls, 256 * 1024);
  }
  signal(SIGPIPE, SIG_IGN);
  if (!g_crc_salt) g_crc_salt = std::random_device{}() | ((uint64_t)std::random_device{}() << 32);
  g_pool.resize(kPool);
  std::mt19937_64 rng(0xB10BDull);
  for (size_t i = 0; i < kPool; i += 8) {
    uint64_t v = rng();
    memcpy(g_pool.data() + i, &v, 8);
  }
  g_pool_fd = memfd_create("blobd-pool", MFD_CLOEXEC);
  if (g_pool_fd >= 0) {
    size_t off = 0;
    while (off < kPool) {
      ssize_t w = ::write(g_pool_fd, g_pool.data() + off, kPool - off);
      if (w <= 0) {
        ::close(g_pool_fd);
        g_pool_fd = -1;
        break;
      }
      off += (size_t)w;
    }
  }
  int ls = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  inet_pton(AF_INET, host.c_str(), &sa.sin_addr);
  if (bind(ls, (sockaddr*)&sa, sizeof sa) < 0 || listen(ls, 1024) < 0) {
    perror("bind/listen");
    return 1;
  }
  socklen_t sl = sizeof sa;
  getsockname(ls, (sockaddr*)&sa, &sl);
  int bound = ntohs(sa.sin_port);
  if (port_file) {
    std::string tmp = std::string(port_file) + ".tmp";
    FILE* f = fopen(tmp.c_str(), "w");
    if (f) {
      fprintf(f, "%d\n", bound);
      fclose(f);
      rename(tmp.c_str(), port_file);
    }
  }
  printf("blobd listening on %s:%d\n", host.c_str(), bound);
  fflush(stdout);
  for (;;) {
    int fd = accept4(ls, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR || errno == ECONNABORTED) continue;
      perror("accept");
      continue;
    }
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    int big = 4 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    std::thread([fd] {
      Conn c(fd);
      c.serve();
    }).detach();
  }
}
