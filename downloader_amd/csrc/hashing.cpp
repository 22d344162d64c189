// Native hashing for the staging data path.
//
// Replaces the OpenSSL-in-Node hashing the reference reaches through its libraries
// (SURVEY.md §2.5): SHA-1 torrent piece verification (webtorrent -> simple-sha1 -> Node
// crypto) and SHA-256 / MD5 over S3 payloads (minio-js SigV4 / Content-MD5). Everything runs
// with the GIL released on a pool of std::threads; digests come from OpenSSL EVP, which uses
// SHA-NI / AVX2 on the host CPU.
#include "native.h"
#include "crc32c.h"

#include <openssl/evp.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sched.h>
#include <fcntl.h>
#include <stdexcept>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace stager {

const EVP_MD* md_for(const std::string& algo) {
  if (algo == "sha1") return EVP_sha1();
  if (algo == "sha256") return EVP_sha256();
  if (algo == "md5") return EVP_md5();
  throw std::invalid_argument("unsupported hash algorithm: " + algo);
}

size_t digest_size(const std::string& algo) { return (size_t)EVP_MD_get_size(md_for(algo)); }

void digest_into(const EVP_MD* md, const uint8_t* p, size_t n, uint8_t* out) {
  unsigned int len = 0;
  if (EVP_Digest(p, n, out, &len, md, nullptr) != 1) throw std::runtime_error("EVP_Digest failed");
}

// CPUs this process may actually use: the affinity mask, capped by a cgroup v2 CPU quota
// (cpu.max "quota period"). Containers commonly expose hundreds of CPUs in the mask but grant
// a 16-CPU quota; spawning a thread per visible CPU would only add run-queue contention.
int effective_cpus() {
  static const int cached = [] {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) {
      unsigned hc = std::thread::hardware_concurrency();
      n = hc ? (int)hc : 4;
    }
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char quota[32] = {0};
      long period = 0;
      if (fscanf(f, "%31s %ld", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0) {
        long q = atol(quota);
        int lim = (int)((q + period - 1) / period);
        if (lim > 0 && lim < n) n = lim;
      }
      fclose(f);
    }
    return n;
  }();
  return cached;
}

int resolve_threads(int threads, size_t work_items) {
  if (threads <= 0) threads = effective_cpus();
  if ((size_t)threads > work_items) threads = (int)(work_items ? work_items : 1);
  return threads;
}

// Run fn(i) for i in [0, n) on `threads` workers pulling indices from an atomic counter.
template <class F>
void parallel_for(size_t n, int threads, F&& fn) {
  threads = resolve_threads(threads, n);
  if (threads <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i, 0);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> pool;
  std::vector<std::exception_ptr> errs(threads);
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t] {
      try {
        for (;;) {
          size_t i = next.fetch_add(1, std::memory_order_relaxed);
          if (i >= n) break;
          fn(i, t);
        }
      } catch (...) {
        errs[t] = std::current_exception();
        next.store(n);
      }
    });
  }
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

// ---------------------------------------------------------------------------------------
// Streaming hasher
Hasher::Hasher(const std::string& algo) : algo_(algo), ctx_(EVP_MD_CTX_new()) {
  if (!ctx_ || EVP_DigestInit_ex(ctx_, md_for(algo), nullptr) != 1)
    throw std::runtime_error("EVP_DigestInit failed");
}
Hasher::~Hasher() {
  if (ctx_) EVP_MD_CTX_free(ctx_);
}
void Hasher::update(const uint8_t* p, size_t n) {
  if (EVP_DigestUpdate(ctx_, p, n) != 1) throw std::runtime_error("EVP_DigestUpdate failed");
}
std::string Hasher::digest() const {
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  EVP_MD_CTX_copy_ex(c, ctx_);
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_DigestFinal_ex(c, out, &len);
  EVP_MD_CTX_free(c);
  return std::string((const char*)out, len);
}
std::string Hasher::finish_and_reset() {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  if (EVP_DigestFinal_ex(ctx_, out, &len) != 1 || EVP_DigestInit_ex(ctx_, md_for(algo_), nullptr) != 1)
    throw std::runtime_error("EVP_DigestFinal failed");
  return std::string((const char*)out, len);
}
std::unique_ptr<Hasher> Hasher::copy() const {
  auto h = std::make_unique<Hasher>(algo_);
  EVP_MD_CTX_copy_ex(h->ctx_, ctx_);
  return h;
}
void Hasher::update_fd(int fd, int64_t offset, int64_t length) {
  std::vector<uint8_t> buf(std::min<int64_t>(length > 0 ? length : 1, 8 << 20));
  int64_t done = 0;
  while (done < length) {
    size_t want = (size_t)std::min<int64_t>((int64_t)buf.size(), length - done);
    ssize_t r = pread(fd, buf.data(), want, offset + done);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("pread: ") + strerror(errno));
    }
    if (r == 0) throw std::runtime_error("short file while hashing");
    update(buf.data(), (size_t)r);
    done += r;
  }
}

// ---------------------------------------------------------------------------------------
// One-shot helpers
std::string digest(const std::string& algo, const uint8_t* p, size_t n) {
  unsigned char out[EVP_MAX_MD_SIZE];
  const EVP_MD* md = md_for(algo);
  digest_into(md, p, n, out);
  return std::string((const char*)out, (size_t)EVP_MD_get_size(md));
}

std::string hash_pieces(const std::string& algo, const uint8_t* p, size_t n, size_t piece_len,
                        int threads) {
  if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
  const EVP_MD* md = md_for(algo);
  size_t ds = (size_t)EVP_MD_get_size(md);
  size_t np = (n + piece_len - 1) / piece_len;
  std::string out(np * ds, '\0');
  if (algo == "sha1" && sha1_mb_supported() && np >= 8) {
    // 16 pieces per task in the lanes of one AVX-512 multi-buffer SHA-1
    parallel_for((np + 15) / 16, threads, [&](size_t g, int) {
      const uint8_t* ptrs[16];
      size_t lens[16];
      size_t k = std::min<size_t>(16, np - g * 16);
      for (size_t l = 0; l < k; ++l) {
        size_t off = (g * 16 + l) * piece_len;
        ptrs[l] = p + off;
        lens[l] = std::min(piece_len, n - off);
      }
      sha1_mb(ptrs, lens, k, (uint8_t*)&out[g * 16 * ds]);
    });
    return out;
  }
  parallel_for(np, threads, [&](size_t i, int) {
    size_t off = i * piece_len;
    size_t len = std::min(piece_len, n - off);
    digest_into(md, p + off, len, (uint8_t*)&out[i * ds]);
  });
  return out;
}

namespace {

// SHA-1 of up to 16 storage pieces of equal length `len` (starting at offs[l]) in the lanes of
// one multi-buffer state, reading `chunk` bytes per lane per step into `buf` (16 * chunk).
// present[l] = false for a lane whose bytes are (partly) missing; its digest is not written.
void mb_storage_group(const Storage& st, const int64_t* offs, size_t k, int64_t len,
                      size_t chunk, uint8_t* buf, bool* present, uint8_t* out20) {
  uint32_t state[5][16];
  sha1x16_init(state);
  uint16_t active = (uint16_t)((1u << k) - 1);
  const uint8_t* ptr[16];
  for (int l = 0; l < 16; ++l) ptr[l] = buf + (size_t)l * chunk;
  int64_t off = 0;
  for (;;) {
    const int64_t n = std::min<int64_t>((int64_t)chunk, len - off);
    for (size_t l = 0; l < k; ++l)
      if ((active >> l) & 1 && !st.read(offs[l] + off, n, buf + l * chunk))
        active &= (uint16_t)~(1u << l);
    const size_t whole = (size_t)n / 64;
    if (active && whole) sha1_mb16_blocks(state, ptr, whole, active);
    off += n;
    if (off >= len) {
      const uint8_t* tails[16];
      for (int l = 0; l < 16; ++l) tails[l] = ptr[l] + whole * 64;
      if (active) sha1x16_finish(state, tails, (size_t)n % 64, (uint64_t)len, active, out20);
      break;
    }
  }
  for (size_t l = 0; l < k; ++l) present[l] = (active >> l) & 1;
}

constexpr size_t kMbChunk = 256 * 1024;   // per lane per step: 16 lanes = 4 MiB per thread

}  // namespace

// ---------------------------------------------------------------------------------------
// Torrent storage: a list of files concatenated in order, split into fixed pieces.
Storage::Storage(const std::vector<std::pair<std::string, int64_t>>& files) {
  int64_t off = 0;
  for (auto& f : files) {
    Entry e;
    e.path = f.first;
    e.length = f.second;
    e.offset = off;
    e.fd = -1;
    off += f.second;
    entries.push_back(e);
  }
  total = off;
}
Storage::~Storage() { close_all(); }
void Storage::open_all(bool missing_ok) {
  for (auto& e : entries) {
    if (e.fd >= 0 || e.length == 0) continue;
    e.fd = ::open(e.path.c_str(), O_RDONLY | O_CLOEXEC);
    if (e.fd < 0 && !missing_ok) throw std::runtime_error("open " + e.path + ": " + strerror(errno));
  }
}
void Storage::close_all() {
  for (auto& e : entries)
    if (e.fd >= 0) {
      ::close(e.fd);
      e.fd = -1;
    }
}
// Read [off, off+len) of the concatenated storage into buf; returns false if any byte is
// missing (file absent or short).
bool Storage::read(int64_t off, int64_t len, uint8_t* buf) const {
  int64_t done = 0;
  for (auto& e : entries) {
    if (done >= len) break;
    int64_t pos = off + done;
    if (pos >= e.offset + e.length || e.length == 0) continue;
    if (pos < e.offset) return false;
    int64_t in_file = pos - e.offset;
    int64_t want = std::min(len - done, e.length - in_file);
    if (e.fd < 0) return false;
    int64_t got = 0;
    while (got < want) {
      ssize_t r = pread(e.fd, buf + done + got, (size_t)(want - got), in_file + got);
      if (r < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      if (r == 0) return false;
      got += r;
    }
    done += want;
  }
  return done == len;
}

std::vector<uint8_t> verify_pieces(const std::vector<std::pair<std::string, int64_t>>& files,
                                   int64_t piece_len, const std::string& hashes,
                                   const std::vector<int64_t>& which, int threads) {
  Storage st(files);
  st.open_all(true);
  const EVP_MD* md = EVP_sha1();
  const size_t ds = 20;
  if (piece_len <= 0) throw std::invalid_argument("piece_len must be > 0");
  int64_t np = (st.total + piece_len - 1) / piece_len;
  if ((int64_t)(hashes.size() / ds) != np || hashes.size() % ds)
    throw std::invalid_argument("hash list does not match the piece count");
  std::vector<int64_t> idx = which;
  if (idx.empty()) {
    idx.resize((size_t)np);
    for (int64_t i = 0; i < np; ++i) idx[(size_t)i] = i;
  }
  std::vector<uint8_t> ok(idx.size(), 0);
  if (sha1_mb_supported() && idx.size() >= 8) {
    // Full-length pieces go 16 per task through the multi-buffer SHA-1 (streamed in 256 KiB
    // steps per lane); the torrent's short last piece and out-of-range entries one by one.
    std::vector<size_t> full, odd;
    for (size_t k = 0; k < idx.size(); ++k) {
      const int64_t i = idx[k];
      if (i < 0 || i >= np) continue;
      (std::min<int64_t>(piece_len, st.total - i * piece_len) == piece_len ? full : odd)
          .push_back(k);
    }
    const size_t chunk = std::min<size_t>(kMbChunk, (size_t)piece_len);
    const size_t groups = (full.size() + 15) / 16;
    int nt = resolve_threads(threads, groups + odd.size());
    std::vector<std::vector<uint8_t>> bufs(nt, std::vector<uint8_t>(16 * chunk));
    parallel_for(groups + odd.size(), nt, [&](size_t task, int t) {
      if (task < groups) {
        int64_t offs[16];
        bool present[16];
        uint8_t d[16 * 20];
        const size_t k = std::min<size_t>(16, full.size() - task * 16);
        for (size_t l = 0; l < k; ++l) offs[l] = idx[full[task * 16 + l]] * piece_len;
        mb_storage_group(st, offs, k, piece_len, chunk, bufs[t].data(), present, d);
        for (size_t l = 0; l < k; ++l) {
          const size_t kk = full[task * 16 + l];
          ok[kk] = present[l] &&
                   memcmp(d + 20 * l, hashes.data() + (size_t)idx[kk] * ds, ds) == 0;
        }
        return;
      }
      const size_t kk = odd[task - groups];
      const int64_t i = idx[kk];
      const int64_t off = i * piece_len;
      const int64_t len = st.total - off;
      std::vector<uint8_t> b((size_t)len);
      if (!st.read(off, len, b.data())) return;
      uint8_t d[20];
      digest_into(md, b.data(), (size_t)len, d);
      ok[kk] = memcmp(d, hashes.data() + (size_t)i * ds, ds) == 0;
    });
    return ok;
  }
  int nt = resolve_threads(threads, idx.size());
  std::vector<std::vector<uint8_t>> bufs(nt, std::vector<uint8_t>((size_t)piece_len));
  parallel_for(idx.size(), nt, [&](size_t k, int t) {
    int64_t i = idx[k];
    if (i < 0 || i >= np) return;
    int64_t off = i * piece_len;
    int64_t len = std::min<int64_t>(piece_len, st.total - off);
    uint8_t* b = bufs[t].data();
    if (!st.read(off, len, b)) return;
    uint8_t d[20];
    digest_into(md, b, (size_t)len, d);
    ok[k] = memcmp(d, hashes.data() + (size_t)i * ds, ds) == 0;
  });
  return ok;
}

std::string hash_storage_pieces(const std::vector<std::pair<std::string, int64_t>>& files,
                                int64_t piece_len, const std::string& algo, int threads) {
  Storage st(files);
  st.open_all(false);
  const EVP_MD* md = md_for(algo);
  size_t ds = (size_t)EVP_MD_get_size(md);
  int64_t np = (st.total + piece_len - 1) / piece_len;
  std::string out((size_t)np * ds, '\0');
  const int64_t nfull = st.total / piece_len;   // pieces of full length
  if (algo == "sha1" && sha1_mb_supported() && nfull >= 8) {
    const size_t chunk = std::min<size_t>(kMbChunk, (size_t)piece_len);
    const size_t groups = (size_t)(nfull + 15) / 16;
    const size_t tasks = groups + (size_t)(np - nfull);
    int nt = resolve_threads(threads, tasks);
    std::vector<std::vector<uint8_t>> bufs(nt, std::vector<uint8_t>(16 * chunk));
    parallel_for(tasks, nt, [&](size_t task, int t) {
      if (task < groups) {
        int64_t offs[16];
        bool present[16];
        const size_t k = (size_t)std::min<int64_t>(16, nfull - (int64_t)task * 16);
        for (size_t l = 0; l < k; ++l) offs[l] = ((int64_t)task * 16 + (int64_t)l) * piece_len;
        mb_storage_group(st, offs, k, piece_len, chunk, bufs[t].data(), present,
                         (uint8_t*)&out[task * 16 * ds]);
        for (size_t l = 0; l < k; ++l)
          if (!present[l]) throw std::runtime_error("short read while hashing");
        return;
      }
      const int64_t off = nfull * piece_len;    // the short last piece
      std::vector<uint8_t> b((size_t)(st.total - off));
      if (!st.read(off, (int64_t)b.size(), b.data()))
        throw std::runtime_error("short read while hashing");
      digest_into(md, b.data(), b.size(), (uint8_t*)&out[(size_t)nfull * ds]);
    });
    return out;
  }
  int nt = resolve_threads(threads, (size_t)np);
  std::vector<std::vector<uint8_t>> bufs(nt, std::vector<uint8_t>((size_t)piece_len));
  parallel_for((size_t)np, nt, [&](size_t i, int t) {
    int64_t off = (int64_t)i * piece_len;
    int64_t len = std::min<int64_t>(piece_len, st.total - off);
    if (!st.read(off, len, bufs[t].data())) throw std::runtime_error("short read while hashing");
    digest_into(md, bufs[t].data(), (size_t)len, (uint8_t*)&out[i * ds]);
  });
  return out;
}

std::vector<std::string> hash_file_ranges(const std::string& path,
                                          const std::vector<std::pair<int64_t, int64_t>>& ranges,
                                          const std::string& algo, int threads) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) throw std::runtime_error("open " + path + ": " + strerror(errno));
  std::vector<std::string> out(ranges.size());
  try {
    parallel_for(ranges.size(), threads, [&](size_t i, int) {
      Hasher h(algo);
      h.update_fd(fd, ranges[i].first, ranges[i].second);
      out[i] = h.digest();
    });
  } catch (...) {
    ::close(fd);
    throw;
  }
  ::close(fd);
  return out;
}

// ---- CRC32C (S3 flexible payload checksums, csrc/crc32c.h) ------------------------------
uint32_t crc32c(const uint8_t* p, size_t n, uint32_t crc) { return crc32c_update(crc, p, n); }

uint32_t crc32c_fd(int fd, int64_t off, int64_t len) {
  // 256 KiB reads stay in L2 between the page-cache copy and the CRC pass.
  thread_local std::vector<uint8_t> buf(256 * 1024);
  uint32_t c = 0;
  while (len > 0) {
    ssize_t r = ::pread(fd, buf.data(), (size_t)std::min<int64_t>(len, (int64_t)buf.size()), off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) throw std::runtime_error("crc32c_fd: short read");
    c = crc32c_update(c, buf.data(), (size_t)r);
    off += r;
    len -= r;
  }
  return c;
}

std::string crc32c_base64(uint32_t crc) {
  char b[9];
  crc32c_b64(crc, b);
  return std::string(b, 8);
}

const char* crc32c_impl() {
  return crc32c_detail::have_vpclmul() ? "avx512-vpclmulqdq" : "sse4.2-3way";
}

}  // namespace stager
