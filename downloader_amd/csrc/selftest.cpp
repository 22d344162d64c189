// Standalone self-test of the host native code, built under sanitizers (SURVEY.md §5.2:
// "an ASan/UBSan build of the C++ module in CI; TSan for the threaded hashing pool").
//
//   g++ -fsanitize=address,undefined selftest.cpp hashing.cpp transfer.cpp -lcrypto -lpthread
//   g++ -fsanitize=thread            selftest.cpp hashing.cpp transfer.cpp -lcrypto -lpthread
//
// Covers: digests vs known vectors, the threaded piece hasher/verifier (threads race on a
// shared atomic work counter and per-thread buffers), and the HTTP transport against
// in-process loopback servers: Content-Length body spliced to a file, chunked body, a
// sendfile request body, and the socket->socket relay.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

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

int main() {
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
  {
    RelayPoolStats st = relay_pool_stats();
    CHECK(st.in_use == 0 && st.idle_buffers <= st.max_idle);
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
