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

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "native.h"

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

int main() {
  signal(SIGPIPE, SIG_IGN);  // SSL_write on a reset socket (Python does the same at start)
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
