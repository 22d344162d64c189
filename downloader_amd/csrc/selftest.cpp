// Standalone self-test of the host native code, built under sanitizers (SURVEY.md §5.2:
// "an ASan/UBSan build of the C++ module in CI; TSan for the threaded hashing pool").
//
//   g++ -fsanitize=address,undefined selftest.cpp hashing.cpp sha1_mb.cpp transfer.cpp tls.cpp
//       -lssl -lcrypto -lpthread                      (python -m downloader_amd.ops.build does it)
//   g++ -fsanitize=thread            (same sources)
//
// Covers: digests vs known vectors, the threaded piece hasher/verifier (threads race on a
// shared atomic work counter and per-thread buffers), and the HTTP transport against
// in-process loopback servers: Content-Length body spliced to a file, chunked body, a
// sendfile request body, the socket->socket relay, the hashed relay, and the same transfers
// over TLS (throwaway in-memory certificate; handshake, verification failure, TLS relay).
// Then the GPU part hasher's completion machinery end to end on a CPU: PartDispatcher
// (part_dispatch.h, the state machine gfx950's PartHasher runs) over a fake device of host
// threads, behind the relay module's part ids / notify / wait / forget / poll, with 64 relays
// at once, hashers replaced mid-flight, the part budget oscillating and injected device faults.
// A run that would hang (a part nobody is told about) is ended by a watchdog and fails.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>

#include <poll.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "native.h"
#include "part_dispatch.h"
#include "part_fake_device.h"

using namespace stager;

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

static std::string hex(const std::string& s) {
  static const char* h = "0123456789abcdef";
  std::string o;
  for (unsigned char c : s) {
    o.push_back(h[c >> 4]);
    o.push_back(h[c & 15]);
  }
  return o;
}

static uint32_t rd32(const char* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return ntohl(v);
}

static std::vector<uint8_t> rnd(size_t n, uint32_t seed) {
  std::mt19937 g(seed);
  std::vector<uint8_t> v(n);
  for (auto& b : v) b = (uint8_t)g();
  return v;
}

static std::string tmpfile_with(const std::vector<uint8_t>& d, const char* tag) {
  char path[] = "/tmp/stager-selftest-XXXXXX";
  int fd = mkstemp(path);
  size_t off = 0;
  while (off < d.size()) {
    ssize_t w = write(fd, d.data() + off, d.size() - off);
    if (w <= 0) break;
    off += (size_t)w;
  }
  close(fd);
  (void)tag;
  return path;
}

// One-shot loopback server: accepts one connection and runs `fn(fd)`.
struct Server {
  int ls = -1, port = 0;
  std::thread th;
  explicit Server(std::function<void(int)> fn) {
    ls = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    bind(ls, (sockaddr*)&a, sizeof a);
    listen(ls, 4);
    socklen_t sl = sizeof a;
    getsockname(ls, (sockaddr*)&a, &sl);
    port = ntohs(a.sin_port);
    th = std::thread([this, fn] {
      int c = accept(ls, nullptr, nullptr);
      if (c >= 0) {
        fn(c);
        close(c);
      }
    });
  }
  ~Server() {
    th.join();
    close(ls);
  }
};

static std::string read_head(int fd) {
  std::string h;
  char c;
  while (h.size() < 65536 && recv(fd, &c, 1, 0) == 1) {
    h.push_back(c);
    if (h.size() >= 4 && h.compare(h.size() - 4, 4, "\r\n\r\n") == 0) break;
  }
  return h;
}

static void send_str(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t w = send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (w <= 0) return;
    off += (size_t)w;
  }
}

static int64_t drain_body(int fd, int64_t n) {
  std::vector<char> b(1 << 16);
  int64_t got = 0;
  while (got < n) {
    ssize_t r = recv(fd, b.data(), (size_t)std::min<int64_t>(n - got, (int64_t)b.size()), 0);
    if (r <= 0) break;
    got += r;
  }
  return got;
}

// ---- TLS fixtures: self-signed P-256 certificate for 127.0.0.1, made in memory
struct TestCert {
  EVP_PKEY* key = nullptr;
  X509* crt = nullptr;
  std::string pem_path;
  TestCert() {
    key = EVP_EC_gen("P-256");
    crt = X509_new();
    X509_set_version(crt, 2);
    ASN1_INTEGER_set(X509_get_serialNumber(crt), 1);
    X509_gmtime_adj(X509_getm_notBefore(crt), -60);
    X509_gmtime_adj(X509_getm_notAfter(crt), 3600);
    X509_set_pubkey(crt, key);
    X509_NAME* nm = X509_get_subject_name(crt);
    X509_NAME_add_entry_by_txt(nm, "CN", MBSTRING_ASC, (const unsigned char*)"127.0.0.1", -1, -1, 0);
    X509_set_issuer_name(crt, nm);
    X509V3_CTX v3;
    X509V3_set_ctx_nodb(&v3);
    X509V3_set_ctx(&v3, crt, crt, nullptr, nullptr, 0);
    for (auto [nid, val] : {std::pair<int, const char*>{NID_subject_alt_name, "IP:127.0.0.1"},
                            {NID_basic_constraints, "critical,CA:TRUE"}}) {
      X509_EXTENSION* ext = X509V3_EXT_conf_nid(nullptr, &v3, nid, val);
      X509_add_ext(crt, ext, -1);
      X509_EXTENSION_free(ext);
    }
    X509_sign(crt, key, EVP_sha256());
    char path[] = "/tmp/stager-selftest-ca-XXXXXX";
    int fd = mkstemp(path);
    FILE* f = fdopen(fd, "w");
    PEM_write_X509(f, crt);
    fclose(f);
    pem_path = path;
  }
  ~TestCert() {
    unlink(pem_path.c_str());
    X509_free(crt);
    EVP_PKEY_free(key);
  }
};

// Server side of a TLS test connection: handshake on fd, then plain byte helpers.
struct TlsServerConn {
  SSL_CTX* ctx;
  SSL* s;
  TlsServerConn(const TestCert& c, int fd) {
    ctx = SSL_CTX_new(TLS_server_method());
    SSL_CTX_use_certificate(ctx, c.crt);
    SSL_CTX_use_PrivateKey(ctx, c.key);
    s = SSL_new(ctx);
    SSL_set_fd(s, fd);
    if (SSL_accept(s) != 1) {
      ERR_clear_error();
      SSL_free(s);
      s = nullptr;
    }
  }
  ~TlsServerConn() {
    if (s) SSL_free(s);
    SSL_CTX_free(ctx);
  }
  std::string head() {
    std::string h;
    char ch;
    while (s && h.size() < 65536 && SSL_read(s, &ch, 1) == 1) {
      h.push_back(ch);
      if (h.size() >= 4 && h.compare(h.size() - 4, 4, "\r\n\r\n") == 0) break;
    }
    return h;
  }
  void send(const std::string& d) {
    size_t off = 0;
    while (s && off < d.size()) {
      int w = SSL_write(s, d.data() + off, (int)(d.size() - off));
      if (w <= 0) return;
      off += (size_t)w;
    }
  }
  int64_t drain(int64_t n) {
    std::vector<char> b(1 << 16);
    int64_t got = 0;
    while (s && got < n) {
      int r = SSL_read(s, b.data(), (int)std::min<int64_t>(n - got, (int64_t)b.size()));
      if (r <= 0) break;
      got += r;
    }
    return got;
  }
};

// Keep-alive loopback peer for the part-hashing stress: on one connection, answers
// `GET /p?off=O&len=N` with data[O, O + N) and drains PUT bodies (200, empty body), until the
// client closes.
struct KeepAlivePeer {
  int ls = -1, port = 0;
  std::thread th;
  explicit KeepAlivePeer(const std::vector<uint8_t>& data) {
    ls = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    bind(ls, (sockaddr*)&a, sizeof a);
    listen(ls, 4);
    socklen_t sl = sizeof a;
    getsockname(ls, (sockaddr*)&a, &sl);
    port = ntohs(a.sin_port);
    th = std::thread([this, &data] {
      int c = accept(ls, nullptr, nullptr);
      if (c < 0) return;
      for (;;) {
        std::string h = read_head(c);
        if (h.empty()) break;
        long long off = 0, len = 0;
        if (h.compare(0, 4, "GET ") == 0 &&
            sscanf(h.c_str(), "GET /p?off=%lld&len=%lld", &off, &len) == 2) {
          send_str(c, "HTTP/1.1 200 OK\r\nContent-Length: " + std::to_string(len) + "\r\n\r\n");
          send_str(c, std::string((const char*)data.data() + off, (size_t)len));
        } else {
          const char* cl = strcasestr(h.c_str(), "content-length:");
          drain_body(c, cl ? atoll(cl + 15) : 0);
          send_str(c, "HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n");
        }
      }
      close(c);
    });
  }
  ~KeepAlivePeer() {
    th.join();
    close(ls);
  }
};

using FakeHasher = PartDispatcher<FakePartDevice>;

static std::unique_ptr<FakeHasher> fake_hasher(FakeDeviceKnobs k) {
  const int64_t slot_bytes = 4 << 20;
  const int max_lanes = 256;
  return std::unique_ptr<FakeHasher>(
      new FakeHasher(slot_bytes, max_lanes, slot_bytes, /*slots*/ 4, /*compute*/ 2, /*copy*/ 2,
                     max_lanes, k));
}

// Ends the process (failing) if a section does not finish in time: a part whose phase nobody
// reports leaves its waiter blocked for good, which is exactly what must be caught.
// Where each stress relay thread is (for the watchdog's report): phase and part id.
static std::atomic<int> g_stress_phase[64];
static std::atomic<uint64_t> g_stress_id[64];

struct Watchdog {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  std::thread th;
  Watchdog(const char* what, int seconds) {
    th = std::thread([this, what, seconds] {
      std::unique_lock<std::mutex> lk(mu);
      // system_clock: see the wait in part_dispatch.h (steady waits are invisible to TSan)
      if (!cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::seconds(seconds),
                         [&] { return done; })) {
        fprintf(stderr, "selftest: %s did not finish in %d s (a part was never reported)\n",
                what, seconds);
        static const char* names[] = {"idle", "relay", "forget", "wait", "poll", "done"};
        for (int i = 0; i < 64; ++i)
          if (g_stress_phase[i].load() != 0 && g_stress_phase[i].load() != 5)
            fprintf(stderr, "  relay %d: %s, part %llu\n", i, names[g_stress_phase[i].load()],
                    (unsigned long long)g_stress_id[i].load());
        GpuPartStats st = gpu_part_stats();
        fprintf(stderr, "  parts: %llu submitted, %llu pending\n",
                (unsigned long long)st.submitted, (unsigned long long)st.pending);
        _exit(3);
      }
    });
  }
  ~Watchdog() {
    {
      std::lock_guard<std::mutex> g(mu);
      done = true;
    }
    cv.notify_all();
    th.join();
  }
};

struct PartStress {
  int threads = 64, parts = 32;          // relays at once x parts each
  int64_t piece = 16 << 10;
  int pieces = 8;                        // the relay module hands parts of >= 8 pieces over
  int replace_every_ms = 5;              // a fresh hasher installed while tickets are pending
  FakeDeviceKnobs knobs;
  FakeDeviceKnobs first;                 // the knobs of the first hasher (a faulty one)
  bool oscillate_budget = true;
};

struct PartStressResult {
  int good = 0, failed = 0, forgotten = 0, polled = 0, hashers = 0;
  bool digests_ok = true;
};

// 64 relays (one keep-alive origin + S3 peer pair each) stage parts through the hashed relay;
// each part is then waited for (gpu_part_wait), left to a poller thread (gpu_part_poll on the
// eventfd) or forgotten as if its job was cancelled (gpu_part_forget), a third each.
static PartStressResult part_stress(const PartStress& cfg) {
  PartStressResult res;
  const int64_t part = cfg.piece * cfg.pieces;
  auto data = rnd(8 << 20, 77);
  std::vector<std::unique_ptr<FakeHasher>> hashers;
  std::mutex hmu;
  hashers.push_back(fake_hasher(cfg.first));
  set_gpu_part_hasher(hashers.back()->api(), cfg.pieces);
  std::atomic<bool> stop{false};
  // the poller: what the asyncio side does (eventfd readable -> gpu_part_poll)
  std::mutex pmu;
  std::condition_variable pcv;
  std::map<uint64_t, std::pair<bool, std::string>> polled;   // id -> (ok, digests / error)
  std::thread poller([&] {
    pollfd pf{gpu_part_eventfd(), POLLIN, 0};
    while (!stop.load()) {
      poll(&pf, 1, 5);
      for (auto& ev : gpu_part_poll()) {
        if (ev.kind == 1) continue;
        std::lock_guard<std::mutex> g(pmu);
        polled[ev.id] = {ev.kind == 2, ev.data};
        pcv.notify_all();
      }
    }
  });
  std::thread replacer([&] {
    uint32_t seed = 100;
    for (int n = 0; n < 200 && !stop.load(); ++n) {   // bounded: a hang must not eat memory
      std::this_thread::sleep_for(std::chrono::milliseconds(cfg.replace_every_ms));
      FakeDeviceKnobs k = cfg.knobs;
      k.seed = ++seed;
      auto h = fake_hasher(k);
      set_gpu_part_hasher(h->api(), cfg.pieces);   // the old one keeps serving its tickets
      std::lock_guard<std::mutex> g(hmu);
      hashers.push_back(std::move(h));
    }
  });
  std::thread budget([&] {
    std::mt19937 g(5);
    while (!stop.load() && cfg.oscillate_budget) {
      relay_pool_set_budget((size_t)(1 + g() % 16) << 20);
      std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
  });
  std::atomic<int> good{0}, failed{0}, forgotten{0}, by_poll{0};
  std::atomic<bool> digests_ok{true};
  std::vector<std::thread> ths;
  for (int t = 0; t < cfg.threads; ++t) {
    ths.emplace_back([&, t] {
      g_stress_phase[t] = 1;
      KeepAlivePeer origin(data), sink(data);
      std::mt19937 g(1000 + t);
      try {
        HttpConn src("127.0.0.1", origin.port, 30, 30), dst("127.0.0.1", sink.port, 30, 30);
        for (int i = 0; i < cfg.parts; ++i) {
          const int64_t off = (int64_t)(g() % (uint32_t)(data.size() - part)) & ~(int64_t)63;
          g_stress_phase[t] = 1;
          src.send_request("GET /p?off=" + std::to_string(off) + "&len=" + std::to_string(part) +
                               " HTTP/1.1\r\nHost: x\r\n\r\n", nullptr, 0);
          ResponseHead gh = src.read_head();
          dst.send_raw("PUT /s HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(part) +
                       "\r\n\r\n");
          std::string digests, head, tail;
          uint64_t id = 0;
          src.relay_body_hashed(dst, gh.content_length, 0, part, cfg.piece, nullptr, &digests,
                                &head, &tail, nullptr, &id);
          ResponseHead ph = dst.read_head();
          dst.read_body(ph, 16);
          const std::string want =
              hash_pieces("sha1", data.data() + off, (size_t)part, (size_t)cfg.piece, 1);
          const int mode = (int)(g() % 3);
          g_stress_id[t] = id;
          if (id && mode == 0) {                       // cancelled job: nobody asks
            g_stress_phase[t] = 2;
            gpu_part_forget(id);
            forgotten++;
            continue;
          }
          std::string got = digests;
          bool err = false;
          auto from_poll = [&] {
            g_stress_phase[t] = 4;
            std::unique_lock<std::mutex> lk(pmu);
            if (!pcv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::seconds(60),
                                [&] { return polled.count(id) > 0; })) {
              fprintf(stderr, "part stress: part %llu never reported\n", (unsigned long long)id);
              err = true;
              return;
            }
            err = !polled[id].first;
            got = polled[id].second;
            polled.erase(id);
            by_poll++;
          };
          if (id && mode == 1) {
            try {
              g_stress_phase[t] = 3;
              got = gpu_part_wait(id);
            } catch (const std::exception& e) {
              // the poller collected it first (before this wait claimed it / while it waited)
              if (strstr(e.what(), "already collected") || strstr(e.what(), "unknown part"))
                from_poll();
              else
                err = true;
            }
          } else if (id) {
            from_poll();
          }
          if (err && getenv("SELFTEST_VERBOSE")) fprintf(stderr, "failed: %s\n", got.c_str());
          if (err) {
            failed++;
          } else if (got == want) {
            good++;
          } else {
            digests_ok = false;
          }
        }
      } catch (const std::exception& e) {
        fprintf(stderr, "part stress relay %d: %s\n", t, e.what());
        digests_ok = false;
      }
      g_stress_phase[t] = 5;
    });
  }
  for (auto& th : ths) th.join();
  stop = true;
  replacer.join();
  budget.join();
  poller.join();
  relay_pool_set_budget(0);
  set_gpu_part_hasher(nullptr, 0);
  res.hashers = (int)hashers.size();
  hashers.clear();                 // each drains what it still holds before its thread ends
  res.good = good;
  res.failed = failed;
  res.forgotten = forgotten;
  res.polled = by_poll;
  res.digests_ok = digests_ok;
  return res;
}

// ---- the native peer wire (peerwire.cpp): 4 connections (socketpairs) feed PIECE messages
// for the same 24 pieces in random order, split at random points, with duplicates, a bogus
// block, control messages in between and one corrupt copy of a piece on one connection;
// every piece must be verified once, written to the two storage files, and reported.
static void wire_section(bool gpu) {
  const int64_t plen = 65536, total = 24 * plen - 1000;      // short last piece
  // gpu: pieces verified on a GPU part hasher - PartDispatcher over the fake device, the
  // state machine of the gfx950 PartHasher - from page-locked pooled buffers
  std::unique_ptr<FakeHasher> hasher;
  if (gpu) {
    FakeDeviceKnobs k;
    k.seed = 3;
    hasher = fake_hasher(k);
    set_gpu_part_hasher(hasher->api(), 8);
  }
  auto data = rnd((size_t)total, 99);
  std::string hashes;
  for (int64_t off = 0; off < total; off += plen)
    hashes += digest("sha1", data.data() + off, (size_t)std::min(plen, total - off));
  char p1[] = "/tmp/stager-selftest-wire-XXXXXX", p2[] = "/tmp/stager-selftest-wire-XXXXXX";
  int f1 = mkstemp(p1), f2 = mkstemp(p2);
  const int64_t n1 = 500000, n2 = total - n1;                 // pieces straddle the files
  SwarmWire w(2);
  w.set_gpu(gpu);
  w.set_storage(plen, total, hashes, {{f1, n1}, {f2, n2}});
  const int npieces = (int)((total + plen - 1) / plen);
  for (int i = 0; i < npieces; ++i) w.begin_piece((uint32_t)i);
  std::vector<std::thread> feeders;
  std::vector<int> ours;
  for (int c = 0; c < 4; ++c) {
    int sv[2];
    socketpair(AF_UNIX, SOCK_STREAM, 0, sv);
    w.attach(sv[0], (uint64_t)(c + 1), c == 0 ? std::string("\0\0\0\0", 4) : "");
    ours.push_back(sv[1]);
    feeders.emplace_back([&, c, fd = sv[1]] {
      std::mt19937 g(7 + c);
      std::string out;
      auto msg = [&](uint8_t id, const std::string& pl) {
        uint32_t n = htonl((uint32_t)(pl.size() + 1));
        out.append((const char*)&n, 4);
        out.push_back((char)id);
        out += pl;
      };
      std::vector<int> order(npieces);
      for (int i = 0; i < npieces; ++i) order[i] = i;
      std::shuffle(order.begin(), order.end(), g);
      for (int i : order) {
        for (int64_t b = 0; b < plen; b += 16384) {
          const int64_t off = (int64_t)i * plen + b;
          if (off >= total) break;
          const int64_t len = std::min<int64_t>(16384, total - off);
          std::string pl(8, '\0');
          uint32_t be[2] = {htonl((uint32_t)i), htonl((uint32_t)b)};
          memcpy(&pl[0], be, 8);
          std::string blk((const char*)data.data() + off, (size_t)len);
          if (c == 0 && i == 5 && b == 0) blk[7] ^= 0x5A;      // a corrupt copy
          msg(7, pl + blk);
        }
        if (g() % 4 == 0) msg(4, std::string("\0\0\0\x01", 4));   // HAVE in between
      }
      msg(7, std::string("\0\0\0\x63\0\0\0\0xyz", 11));       // no such piece
      for (size_t off = 0; off < out.size();) {                   // random split points
        size_t k = std::min(out.size() - off, (size_t)(1 + g() % 70000));
        ssize_t wr = send(fd, out.data() + off, k, MSG_NOSIGNAL);
        if (wr <= 0) break;
        off += (size_t)wr;
      }
    });
    if (c == 0) feeders.back().join();   // connection 0 first: its corrupt piece 5 arrives first
  }
  for (auto& t : feeders)
    if (t.joinable()) t.join();
  // collect until every piece is verified (a corrupt first copy is re-begun and fed again)
  std::vector<int> verified(npieces, 0);
  int bad = 0, msgs = 0, done = 0;
  uint64_t blocks_taken = 0;
  const auto t0 = std::chrono::steady_clock::now();
  while (done < npieces && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(60)) {
    pollfd pf{w.eventfd(), POLLIN, 0};
    ::poll(&pf, 1, 100);
    for (auto& e : w.poll()) {
      if (e.kind == SwarmWire::kEvMsg) msgs++;
      if (e.kind == SwarmWire::kEvBlocks)
        for (size_t k = 0; k + 16 <= e.data.size(); k += 16)
          blocks_taken += e.data[k + 15] != 0;
      if (e.kind == SwarmWire::kEvPiece) {
        const uint32_t idx = ntohl(*(const uint32_t*)e.data.data());
        if (e.data[4] == 1) {
          verified[idx]++;
          done++;
        } else {
          bad++;
          w.begin_piece(idx);                 // wanted again: the next copy fills it
          int fd = ours[0];
          std::string out;
          for (int64_t b = 0; b < plen; b += 16384) {
            const int64_t off = (int64_t)idx * plen + b;
            const int64_t len = std::min<int64_t>(16384, total - off);
            uint32_t hdr[3] = {htonl((uint32_t)(len + 9)), htonl(idx), htonl((uint32_t)b)};
            out.append((const char*)hdr, 4);
            out.push_back(7);
            out.append((const char*)&hdr[1], 8);
            out.append((const char*)data.data() + off, (size_t)len);
          }
          send(fd, out.data(), out.size(), MSG_NOSIGNAL);
        }
      }
    }
  }
  CHECK(done == npieces);
  for (int i = 0; i < npieces; ++i) CHECK(verified[i] == 1);
  CHECK(msgs > 0 && blocks_taken >= (uint64_t)(npieces * 4));
  SwarmWireStats st = w.stats();
  CHECK(bad == 1 && st.verified == (uint64_t)npieces && st.hash_fails == 1);
  if (gpu) CHECK(st.gpu_pieces == (uint64_t)npieces + 1 && st.gpu_errors == 0);
  w.close();
  CHECK(w.stats().pool_in_use == 0);   // every piece buffer back in the process-wide pool
  if (gpu) {
    set_gpu_part_hasher(nullptr, 0);
    swarm_piece_pool_forget(hasher->api());   // idle buffers page-locked for it go first
    hasher.reset();
  }
  std::vector<uint8_t> back((size_t)total);
  CHECK(pread(f1, back.data(), (size_t)n1, 0) == n1);
  CHECK(pread(f2, back.data() + n1, (size_t)n2, 0) == n2);
  CHECK(back == data);
  for (int fd : ours) close(fd);
  close(f1);
  close(f2);
  unlink(p1);
  unlink(p2);
  fprintf(stderr, "wire%s: %d pieces verified, %d corrupt copies refused\n",
          gpu ? " (gpu hasher)" : "", done, bad);
}

// ---- owned pieces: the wire requests the blocks itself. Two seeders answer every REQUEST
// (the first copy of piece 7 served is corrupt; seeder 2 adds a block of a piece nobody asked
// it for); the driver assigns pieces while a connection's queue is low, re-assigns the failed
// piece to connection 1, and half-way releases connection 2's pieces (as on a CHOKE) and
// hands them to connection 1, while seeder 2 still answers the requests it had. Every piece
// must be verified once and written, no block reported one by one, and the late answers
// refused.
static void wire_owned_section() {
  const int64_t plen = 65536, total = 40 * plen - 5000;
  const int npieces = (int)((total + plen - 1) / plen);
  auto data = rnd((size_t)total, 17);
  std::string hashes;
  for (int64_t off = 0; off < total; off += plen)
    hashes += digest("sha1", data.data() + off, (size_t)std::min(plen, total - off));
  char p1[] = "/tmp/stager-selftest-owned-XXXXXX";
  int f1 = mkstemp(p1);
  SwarmWire w(2);
  w.set_storage(plen, total, hashes, {{f1, total}});
  w.set_pipeline(6);
  std::vector<std::thread> seeders;
  std::vector<int> theirs;
  std::atomic<int> requests{0};
  std::atomic<bool> corrupted{false};
  for (int c = 0; c < 2; ++c) {
    int sv[2];
    socketpair(AF_UNIX, SOCK_STREAM, 0, sv);
    w.attach(sv[0], (uint64_t)(c + 1), "");
    theirs.push_back(sv[1]);
    seeders.emplace_back([&, c, fd = sv[1]] {
      std::string in;
      bool stray = false;
      char buf[65536];
      for (;;) {
        ssize_t r = recv(fd, buf, sizeof buf, 0);
        if (r <= 0) return;
        in.append(buf, (size_t)r);
        std::string out;
        size_t pos = 0;
        while (in.size() - pos >= 4) {
          const uint32_t n = rd32(in.data() + pos);
          if (in.size() - pos < 4 + (size_t)n) break;
          const char* m = in.data() + pos + 4;
          if (n == 13 && m[0] == 6) {
            requests++;
            const uint32_t idx = rd32(m + 1), begin = rd32(m + 5), len = rd32(m + 9);
            uint32_t hdr[3] = {htonl(len + 9), htonl(idx), htonl(begin)};
            out.append((const char*)hdr, 4);
            out.push_back(7);
            out.append((const char*)&hdr[1], 8);
            std::string blk((const char*)data.data() + (int64_t)idx * plen + begin, len);
            if (idx == 7 && !corrupted.exchange(true)) blk[3] ^= 0x21;   // the first copy
            out += blk;
            if (c == 1 && !stray) {               // unrequested: piece 1 is not ours
              stray = true;
              uint32_t h2[3] = {htonl(9 + 16384), htonl(1), htonl(16384)};
              out.append((const char*)h2, 4);
              out.push_back(7);
              out.append((const char*)&h2[1], 8);
              out.append(16384, 'x');
            }
          }
          pos += 4 + n;
        }
        in.erase(0, pos);
        for (size_t off = 0; off < out.size();) {
          ssize_t wr = send(fd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
          if (wr <= 0) return;
          off += (size_t)wr;
        }
      }
    });
  }
  // (between release and re-assignment a released piece is an ordinary one: a late answer
  // from seeder 2 may land in it and be reported block by block)
  int next = 0, done = 0, bad = 0, block_records = 0, records_before = -1, needs = 0;
  bool released = false;
  std::vector<int> verified(npieces, 0);
  auto top_up = [&](uint64_t conn) {
    size_t t = w.todo(conn);
    while (t < 12 && next < npieces) {
      w.begin_piece((uint32_t)next);
      t = w.assign(conn, (uint32_t)next++);
    }
  };
  top_up(1);
  top_up(2);
  const auto t0 = std::chrono::steady_clock::now();
  while (done < npieces && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(60)) {
    pollfd pf{w.eventfd(), POLLIN, 0};
    ::poll(&pf, 1, 100);
    for (auto& e : w.poll()) {
      if (e.kind == SwarmWire::kEvBlocks)       // blocks taken one by one (stray junk is
        for (size_t k = 0; k + 16 <= e.data.size(); k += 16)   // reported as not taken)
          block_records += e.data[k + 15] != 0;
      if (e.kind == SwarmWire::kEvNeed) {
        needs++;
        top_up(e.conn);
      }
      if (e.kind == SwarmWire::kEvPiece) {
        const uint32_t idx = rd32(e.data.data());
        if (e.data[4] == 1) {
          verified[idx]++;
          done++;
        } else {
          bad++;
          w.begin_piece(idx);
          w.assign(1, idx);                  // fetched again, a fresh copy
        }
        if (!released && done >= npieces / 2) {
          released = true;                   // connection 2 "choked": its pieces go to 1
          records_before = block_records;
          for (auto& r : w.release(2)) {
            CHECK(r.second.size() == (size_t)((std::min<int64_t>(plen, total - (int64_t)r.first * plen) + 16383) / 16384));
            w.assign(1, r.first);
          }
        }
      }
    }
  }
  CHECK(done == npieces);
  for (int i = 0; i < npieces; ++i) CHECK(verified[i] == 1);
  SwarmWireStats st = w.stats();
  CHECK(bad == 1 && st.hash_fails == 1 && st.verified == (uint64_t)npieces);
  CHECK(released && records_before == 0);
  CHECK(needs > 0);
  CHECK(st.blocks_ignored >= 1);            // the stray block at least
  w.close();
  for (auto& t : seeders) t.join();          // close() shut their peers' sockets down
  std::vector<uint8_t> back((size_t)total);
  CHECK(pread(f1, back.data(), (size_t)total, 0) == total);
  CHECK(back == data);
  for (int fd : theirs) close(fd);
  close(f1);
  unlink(p1);
  fprintf(stderr, "wire (owned): %d pieces, %d requests, %d NEED events, %llu blocks refused\n",
          done, requests.load(), needs, (unsigned long long)st.blocks_ignored);
}

// Multi-slot launches: with kernels slower than the parts arrive, slots
// close while both compute streams are busy, and the next launch must take every closed slot
// at once - lanes of several slots in one kernel, digests handed back to the right parts.
static void multislot_section() {
  Watchdog wd("multi-slot launches", 60);
  FakeDeviceKnobs k;
  k.kernel_us_max = 30000;                // 0 - 30 ms per launch: slots pile up behind them
  k.copy_us_max = 100;
  k.lag = 0.3;
  k.seed = 7;
  auto h = fake_hasher(k);                // 4 slots of 4 MiB / 256 lanes, 2 compute streams
  const GpuPartHashApi* api = h->api();
  const int64_t piece = 16 << 10;
  const int parts = 160, pieces = 8;      // 8 pieces a part: 32 parts fill a slot
  auto data = rnd((size_t)parts * pieces * piece, 91);
  std::vector<uint64_t> tickets;
  for (int i = 0; i < parts; ++i) {
    const uint8_t* p = data.data() + (size_t)i * pieces * piece;
    uint64_t t = 0;
    while (!(t = api->submit(api->ctx, p, pieces * piece, piece)))
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    tickets.push_back(t);
  }
  bool ok = true;
  for (int i = 0; i < parts; ++i) {
    uint8_t dig[pieces * 20];
    char err[256] = {0};
    if (api->wait(api->ctx, tickets[(size_t)i], GPU_PART_DONE, dig, sizeof dig, err, sizeof err) != 0) {
      fprintf(stderr, "multi-slot: part %d failed: %s\n", i, err);
      ok = false;
      continue;
    }
    for (int q = 0; q < pieces; ++q) {
      const uint8_t* pc = data.data() + ((size_t)i * pieces + q) * piece;
      if (digest("sha1", pc, (size_t)piece) != std::string((const char*)dig + q * 20, 20)) ok = false;
    }
  }
  const PartDispatchStats st = h->stats();
  fprintf(stderr, "multi-slot: %llu launches, %llu spanning >= 2 slots, up to %llu slots / %llu lanes\n",
          (unsigned long long)st.launches, (unsigned long long)st.multi_slot_launches,
          (unsigned long long)st.max_launch_slots, (unsigned long long)st.max_batch_lanes);
  CHECK(ok);
  CHECK(st.multi_slot_launches > 0 && st.max_launch_slots >= 2);
  CHECK(st.max_batch_lanes > 256);        // more than one slot's lanes in one kernel
  CHECK(st.lanes == (uint64_t)parts * pieces && st.pending == 0);
}

static void stress_sections() {
  multislot_section();
  // ---- the completion machinery under load: 64 relays x 32 parts (2,048) through
  // PartDispatcher<FakePartDevice>, copies that complete before they are seen, hashers
  // replaced every few ms, the part budget oscillating, a third of the parts forgotten
  {
    Watchdog wd("part stress", 90);
    PartStress cfg;
    GpuPartStats before = gpu_part_stats();
    PartStressResult r = part_stress(cfg);
    GpuPartStats after = gpu_part_stats();
    fprintf(stderr, "part stress: %d good, %d forgotten, %d via poll, %d failed, %d hashers\n",
            r.good, r.forgotten, r.polled, r.failed, r.hashers);
    CHECK(r.digests_ok && r.failed == 0);
    CHECK(r.good + r.forgotten == cfg.threads * cfg.parts);
    CHECK(r.forgotten > 0 && r.hashers > 2);
    // every part went to a hasher, or was hashed on the host because its pooled buffer was
    // page-locked for a hasher replaced meanwhile (refused)
    CHECK(after.submitted - before.submitted + after.refused - before.refused ==
          (uint64_t)(cfg.threads * cfg.parts));
    CHECK(after.submitted - before.submitted > (uint64_t)(cfg.threads * cfg.parts) / 2);
    CHECK(after.pending == 0);     // every part collected, or forgotten and dropped
  }
  // ---- device faults: every hasher fails at its 3rd / 4th launch (parts it had finished in
  // the same pass must still be reported) or at its 400th event query
  {
    Watchdog wd("part stress with device faults", 90);
    PartStress cfg;
    cfg.threads = 16;
    cfg.parts = 24;
    cfg.replace_every_ms = 20;
    cfg.first.fail_launch_at = 3;
    cfg.knobs.fail_launch_at = 4;      // every replacement fails too, at its 4th launch
    cfg.knobs.fail_query_at = 400;
    GpuPartStats before = gpu_part_stats();
    PartStressResult r = part_stress(cfg);
    GpuPartStats after = gpu_part_stats();
    fprintf(stderr, "part stress (faults): %d good, %d forgotten, %d failed, %d host fallbacks\n",
            r.good, r.forgotten, r.failed, (int)(after.host_fallbacks - before.host_fallbacks));
    CHECK(r.digests_ok);
    CHECK(r.good + r.forgotten + r.failed == cfg.threads * cfg.parts);
    CHECK(r.failed + (int)(after.host_fallbacks - before.host_fallbacks) > 0);
    CHECK(after.pending == 0);
  }
}

int main() {
  signal(SIGPIPE, SIG_IGN);
  if (getenv("SELFTEST_ONLY") && strcmp(getenv("SELFTEST_ONLY"), "wire") == 0) {
    wire_section(false);
    wire_section(true);
    wire_owned_section();
    printf(g_fail ? "selftest: failures\n" : "selftest ok\n");
    return g_fail ? 1 : 0;
  }
  if (getenv("SELFTEST_ONLY") && strcmp(getenv("SELFTEST_ONLY"), "stress") == 0) {
    stress_sections();                 // the part-hasher sections alone (quick iteration)
    printf(g_fail ? "selftest: failures\n" : "selftest ok\n");
    return g_fail ? 1 : 0;
  }  // SSL_write on a reset socket (Python does the same at start)
  // ---- digests
  const uint8_t* abc = (const uint8_t*)"abc";
  CHECK(hex(digest("sha1", abc, 3)) == "a9993e364706816aba3e25717850c26c9cd0d89d");
  CHECK(hex(digest("md5", abc, 3)) == "900150983cd24fb0d6963f7d28e17f72");
  CHECK(hex(digest("sha256", abc, 3)) ==
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad");

  // ---- threaded piece hashing: 8 threads == 1 thread
  auto data = rnd(8 << 20, 1);
  std::string p1 = hash_pieces("sha1", data.data(), data.size(), 65536, 1);
  std::string p8 = hash_pieces("sha1", data.data(), data.size(), 65536, 8);
  CHECK(p1 == p8);

  // ---- storage verification across file boundaries, threaded
  auto a = rnd(3000001, 2), b = rnd(777777, 3);
  std::string fa = tmpfile_with(a, "a"), fb = tmpfile_with(b, "b");
  std::vector<std::pair<std::string, int64_t>> files = {{fa, (int64_t)a.size()}, {fb, (int64_t)b.size()}};
  std::string hashes = hash_storage_pieces(files, 262144, "sha1", 8);
  auto ok = verify_pieces(files, 262144, hashes, {}, 8);
  bool all = true;
  for (auto v : ok) all = all && v;
  CHECK(all);
  {
    int fd = open(fb.c_str(), O_WRONLY);
    uint8_t x = b[5] ^ 0xFF;
    pwrite(fd, &x, 1, 5);
    close(fd);
  }
  ok = verify_pieces(files, 262144, hashes, {}, 8);
  int bad = 0;
  for (auto v : ok) bad += !v;
  CHECK(bad == 1);

  // ---- transfer: Content-Length body spliced into a file
  auto body = rnd(1 << 20, 4);
  {
    Server s([&](int fd) {
      read_head(fd);
      send_str(fd, "HTTP/1.1 200 OK\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n");
      send_str(fd, std::string((const char*)body.data(), body.size()));
    });
    HttpConn c("127.0.0.1", s.port, 5, 5);
    c.send_request("GET /x HTTP/1.1\r\nHost: x\r\n\r\n", nullptr, 0);
    ResponseHead h = c.read_head();
    char path[] = "/tmp/stager-selftest-dl-XXXXXX";
    int out = mkstemp(path);
    Progress prog;
    int64_t n = c.read_body_to_fd(h, out, 0, (int64_t)1 << 40, &prog);
    CHECK(h.status == 200 && n == (int64_t)body.size() && prog.bytes.load() == n);
    std::vector<uint8_t> back(body.size());
    pread(out, back.data(), back.size(), 0);
    CHECK(back == body);
    close(out);
    unlink(path);
  }
  // ---- chunked body into memory
  {
    Server s([&](int fd) {
      read_head(fd);
      send_str(fd, "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n6\r\n world\r\n0\r\n\r\n");
    });
    HttpConn c("127.0.0.1", s.port, 5, 5);
    c.send_request("GET /c HTTP/1.1\r\nHost: x\r\n\r\n", nullptr, 0);
    ResponseHead h = c.read_head();
    CHECK(h.chunked && c.read_body(h, 1 << 20) == "hello world");
  }
  // ---- sendfile request body
  {
    int64_t got = 0;
    Server s([&](int fd) {
      read_head(fd);
      got = drain_body(fd, (int64_t)a.size());
      send_str(fd, "HTTP/1.1 200 OK\r\nETag: \"e\"\r\nContent-Length: 0\r\n\r\n");
    });
    HttpConn c("127.0.0.1", s.port, 5, 5);
    int fd = open(fa.c_str(), O_RDONLY);
    c.send_request_fd("PUT /p HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(a.size()) + "\r\n\r\n",
                      fd, 0, (int64_t)a.size(), nullptr);
    ResponseHead h = c.read_head();
    close(fd);
    CHECK(h.status == 200);
    c.read_body(h, 1024);
    CHECK(got == (int64_t)a.size());
  }
  // ---- relay: origin socket -> pipe -> sink socket
  {
    int64_t sunk = 0;
    Server origin([&](int fd) {
      read_head(fd);
      send_str(fd, "HTTP/1.1 206 Partial Content\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n");
      send_str(fd, std::string((const char*)body.data(), body.size()));
    });
    Server sink([&](int fd) {
      read_head(fd);
      sunk = drain_body(fd, (int64_t)body.size());
      send_str(fd, "HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n");
    });
    HttpConn src("127.0.0.1", origin.port, 5, 5), dst("127.0.0.1", sink.port, 5, 5);
    src.send_request("GET /r HTTP/1.1\r\nHost: x\r\nRange: bytes=0-\r\n\r\n", nullptr, 0);
    ResponseHead g = src.read_head();
    dst.send_raw("PUT /s HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n");
    int64_t moved = src.relay_body_to(dst, g.content_length, nullptr);
    ResponseHead p = dst.read_head();
    CHECK(moved == (int64_t)body.size() && p.status == 200);
    dst.read_body(p, 16);
    CHECK(sunk == (int64_t)body.size());
  }
  // ---- hashed relay, 4 threads at once: the chunked single-chain path (< 8 pieces) and the
  // pooled multi-buffer path (>= 8 pieces; buffers shared through the process-wide pool)
  for (int64_t plen : {(int64_t)1 << 18, (int64_t)1 << 16}) {
    const int64_t skip = 1000, n = (int64_t)body.size();
    const int64_t full = ((n - skip) / plen) * plen;   // whole pieces, then a tail fragment
    std::string want = hash_pieces("sha1", body.data() + skip, (size_t)full, (size_t)plen, 1);
    std::vector<std::thread> ths;
    std::atomic<int> good{0};
    for (int t = 0; t < 4; ++t) {
      ths.emplace_back([&] {
        Server origin([&](int fd) {
          read_head(fd);
          send_str(fd, "HTTP/1.1 206 Partial Content\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n");
          send_str(fd, std::string((const char*)body.data(), body.size()));
        });
        int64_t sunk = 0;
        Server sink([&](int fd) {
          read_head(fd);
          sunk = drain_body(fd, n);
          send_str(fd, "HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n");
        });
        HttpConn src("127.0.0.1", origin.port, 5, 5), dst("127.0.0.1", sink.port, 5, 5);
        src.send_request("GET /h HTTP/1.1\r\nHost: x\r\n\r\n", nullptr, 0);
        ResponseHead g = src.read_head();
        dst.send_raw("PUT /h HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n");
        std::string digests, head, tail;
        int64_t moved = src.relay_body_hashed(dst, g.content_length, skip, full, plen, nullptr,
                                              &digests, &head, &tail);
        ResponseHead p = dst.read_head();
        dst.read_body(p, 16);
        bool ok = moved == n && p.status == 200 && digests == want &&
                  head == std::string((const char*)body.data(), (size_t)skip) &&
                  tail == std::string((const char*)body.data() + skip + full, (size_t)(n - skip - full));
        if (ok) good.fetch_add(1);
        (void)sunk;
      });
    }
    for (auto& th : ths) th.join();
    CHECK(good.load() == 4);
  }
  // ---- TLS: upload from a file (pread + SSL_write), TLS -> TLS hashed relay on 2 threads
  // (multi-buffer path through a pooled buffer), and a failed verification
  {
    TestCert cert;
    auto ctx = std::make_shared<TlsContext>(true, cert.pem_path);
    int64_t got = 0;
    {
      Server s([&](int fd) {
        TlsServerConn t(cert, fd);
        t.head();
        got = t.drain((int64_t)a.size());
        t.send("HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nok");
      });
      HttpConn c("127.0.0.1", s.port, 5, 5, ctx);
      CHECK(c.is_tls());
      int fd = open(fa.c_str(), O_RDONLY);
      Progress prog;
      c.send_request_fd("PUT /p HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(a.size()) +
                            "\r\n\r\n", fd, 0, (int64_t)a.size(), &prog);
      ResponseHead h = c.read_head();
      close(fd);
      CHECK(h.status == 200 && c.read_body(h, 16) == "ok" && prog.bytes.load() == (int64_t)a.size());
      CHECK(got == (int64_t)a.size());
    }
    const int64_t plen = 1 << 16, skip = 1000, n = (int64_t)body.size();
    const int64_t full = ((n - skip) / plen) * plen;
    std::string want = hash_pieces("sha1", body.data() + skip, (size_t)full, (size_t)plen, 1);
    std::atomic<int> good{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < 2; ++t) {
      ths.emplace_back([&] {
        Server origin([&](int fd) {
          TlsServerConn s(cert, fd);
          s.head();
          s.send("HTTP/1.1 200 OK\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n");
          s.send(std::string((const char*)body.data(), body.size()));
        });
        int64_t sunk = 0;
        Server sink([&](int fd) {
          TlsServerConn s(cert, fd);
          s.head();
          sunk = s.drain(n);
          s.send("HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n");
        });
        try {
          HttpConn src("127.0.0.1", origin.port, 5, 5, ctx), dst("127.0.0.1", sink.port, 5, 5, ctx);
          src.send_request("GET /h HTTP/1.1\r\nHost: x\r\n\r\n", nullptr, 0);
          ResponseHead g = src.read_head();
          dst.send_raw("PUT /h HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n");
          std::string digests, head, tail;
          int64_t moved = src.relay_body_hashed(dst, g.content_length, skip, full, plen, nullptr,
                                                &digests, &head, &tail);
          ResponseHead p = dst.read_head();
          dst.read_body(p, 16);
          if (moved == n && p.status == 200 && digests == want && sunk == n) good.fetch_add(1);
        } catch (const std::exception& e) {
          fprintf(stderr, "tls relay: %s\n", e.what());
        }
      });
    }
    for (auto& th : ths) th.join();
    CHECK(good.load() == 2);
    // no trust for the throwaway CA: the handshake fails with the verification reason
    auto strict = std::make_shared<TlsContext>(true, "");
    Server s([&](int fd) { TlsServerConn t(cert, fd); });
    std::string err;
    try {
      HttpConn c("127.0.0.1", s.port, 5, 5, strict);
    } catch (const std::exception& e) {
      err = e.what();
    }
    CHECK(err.find("certificate verify failed") != std::string::npos);
  }
  // ---- CRC32C: check value, the VPCLMULQDQ fold (>= 1 KiB) and the crc32 chains agree with
  // a bitwise reference at odd lengths / offsets, and a CRC'd relay reports the body's CRC
  {
    CHECK(crc32c((const uint8_t*)"123456789", 9) == 0xE3069283u);
    auto bitwise = [](const uint8_t* p, size_t n) {
      uint32_t c = ~0u;
      for (size_t i = 0; i < n; ++i) {
        c ^= p[i];
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1)));
      }
      return ~c;
    };
    for (size_t n : {(size_t)1, (size_t)1023, (size_t)1024, (size_t)4099, (size_t)77777, (size_t)300000})
      for (size_t off : {(size_t)0, (size_t)3}) {
        const uint8_t* p = body.data() + off;
        uint32_t split = crc32c(p + n / 3, n - n / 3, crc32c(p, n / 3));
        CHECK(crc32c(p, n) == bitwise(p, n) && split == bitwise(p, n));
      }
    CHECK(crc32c_base64(0xE3069283u) == "4waSgw==");
    Server origin([&](int fd) {
      read_head(fd);
      send_str(fd, "HTTP/1.1 206 Partial Content\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n");
      send_str(fd, std::string((const char*)body.data(), body.size()));
    });
    Server sink([&](int fd) {
      read_head(fd);
      drain_body(fd, (int64_t)body.size());
      send_str(fd, "HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n");
    });
    HttpConn src("127.0.0.1", origin.port, 5, 5), dst("127.0.0.1", sink.port, 5, 5);
    src.send_request("GET /r HTTP/1.1\r\nHost: x\r\n\r\n", nullptr, 0);
    ResponseHead g = src.read_head();
    dst.send_raw("PUT /s HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n");
    uint32_t crc = 0;
    int64_t moved = src.relay_body_to(dst, g.content_length, nullptr, &crc);
    ResponseHead p = dst.read_head();
    dst.read_body(p, 16);
    CHECK(moved == (int64_t)body.size() && crc == crc32c(body.data(), body.size()));
  }
  // ---- asynchronous part hashing (gpu_part_api.h) served by the host double: 4 relays hand
  // their parts over at once, the waits return the digests and the buffers come back to the
  // pool; then the hasher is replaced (registered buffers of the old one are dropped)
  {
    CpuPartHasher cph(0.002);
    set_gpu_part_hasher(cph.api(), 8);
    const int64_t plen = 1 << 16, skip = 1000, n = (int64_t)body.size();
    const int64_t full = ((n - skip) / plen) * plen;
    std::string want = hash_pieces("sha1", body.data() + skip, (size_t)full, (size_t)plen, 1);
    std::atomic<int> good{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < 4; ++t) {
      ths.emplace_back([&] {
        Server origin([&](int fd) {
          read_head(fd);
          send_str(fd, "HTTP/1.1 206 Partial Content\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n");
          send_str(fd, std::string((const char*)body.data(), body.size()));
        });
        Server sink([&](int fd) {
          read_head(fd);
          drain_body(fd, n);
          send_str(fd, "HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n");
        });
        HttpConn src("127.0.0.1", origin.port, 5, 5), dst("127.0.0.1", sink.port, 5, 5);
        src.send_request("GET /g HTTP/1.1\r\nHost: x\r\n\r\n", nullptr, 0);
        ResponseHead g = src.read_head();
        dst.send_raw("PUT /g HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n");
        std::string digests, head, tail;
        uint64_t ticket = 0;
        int64_t moved = src.relay_body_hashed(dst, g.content_length, skip, full, plen, nullptr,
                                              &digests, &head, &tail, nullptr, &ticket);
        ResponseHead p = dst.read_head();
        dst.read_body(p, 16);
        if (ticket) digests = gpu_part_wait(ticket);
        if (moved == n && p.status == 200 && ticket != 0 && digests == want) good.fetch_add(1);
      });
    }
    for (auto& th : ths) th.join();
    CHECK(good.load() == 4);
    GpuPartStats gs = gpu_part_stats();
    CHECK(gs.submitted >= 4 && cph.registered() >= 1);
    set_gpu_part_hasher(nullptr, 0);
  }
  // ---- the same with a failing device: every 2nd copy fails (host fallback, the job is
  // abandoned to the hasher thread), every 3rd hash fails (gpu_part_wait throws)
  {
    CpuPartHasher bad(0.001, 2, 3);
    set_gpu_part_hasher(bad.api(), 8);
    const int64_t plen = 1 << 16, skip = 0, n = (int64_t)body.size();
    const int64_t full = (n / plen) * plen;
    std::string want = hash_pieces("sha1", body.data(), (size_t)full, (size_t)plen, 1);
    std::atomic<int> good{0}, failed{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < 6; ++t) {
      ths.emplace_back([&] {
        Server origin([&](int fd) {
          read_head(fd);
          send_str(fd, "HTTP/1.1 200 OK\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n");
          send_str(fd, std::string((const char*)body.data(), body.size()));
        });
        Server sink([&](int fd) {
          read_head(fd);
          drain_body(fd, n);
          send_str(fd, "HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n");
        });
        HttpConn src("127.0.0.1", origin.port, 5, 5), dst("127.0.0.1", sink.port, 5, 5);
        src.send_request("GET /f HTTP/1.1\r\nHost: x\r\n\r\n", nullptr, 0);
        ResponseHead g = src.read_head();
        dst.send_raw("PUT /f HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(n) + "\r\n\r\n");
        std::string digests, head, tail;
        uint64_t ticket = 0;
        src.relay_body_hashed(dst, g.content_length, skip, full, plen, nullptr, &digests, &head,
                              &tail, nullptr, &ticket);
        ResponseHead p = dst.read_head();
        dst.read_body(p, 16);
        try {
          if (ticket) digests = gpu_part_wait(ticket);
          if (digests == want) good.fetch_add(1);
        } catch (const std::exception&) {
          failed.fetch_add(1);
        }
      });
    }
    for (auto& th : ths) th.join();
    CHECK(good.load() + failed.load() == 6 && good.load() >= 3 && failed.load() >= 1);
    set_gpu_part_hasher(nullptr, 0);
  }
  stress_sections();
  wire_section(false);
  wire_section(true);
  wire_owned_section();
  {
    RelayPoolStats st = relay_pool_stats();
    CHECK(st.in_use == 0 && st.idle_buffers <= st.max_idle);
    PipeStats ps = pipe_stats();   // every splice transfer returned its leased pipes
    CHECK(ps.created > 0 && ps.in_use == 0 && ps.idle <= 32);
    relay_pool_trim();
    CHECK(relay_pool_stats().idle_bytes == 0);
  }
  unlink(fa.c_str());
  unlink(fb.c_str());
  if (g_fail) {
    fprintf(stderr, "selftest: %d failure(s)\n", g_fail);
    return 1;
  }
  printf("selftest ok\n");
  return 0;
}
