// relaybench: per-byte CPU cost of the ways a relay can move (and CRC) a body socket -> socket.
//
// The headline relay splices origin -> pipe -> S3 without the bytes entering user space; a
// payload checksum needs every byte read once by the CPU. This isolates that cost from HTTP,
// the event loop and the bench peers: T relay threads, each between its own loopback TCP
// producer (send() from a resident buffer) and consumer (recv(MSG_TRUNC): the kernel drops the
// bytes without copying them out), move --gb GB each in one of these modes:
//   splice    socket -> pipe -> socket (page references only; the headline path)
//   tee       splice + tee() into a 2nd pipe + read() of the duplicate into an L2 buffer
//   teecrc    tee + CRC32C of the copied bytes (s3.checksum: always, csrc/transfer.cpp)
//   peekcrc   recv(MSG_PEEK) into the L2 buffer + CRC32C, then splice the same bytes
//   copycrc   recv() into the L2 buffer + CRC32C + send() (two copies; TLS-style relay)
// and reports GB/s and relay-thread CPU seconds per GB (CLOCK_THREAD_CPUTIME_ID), so the
// difference between modes is the copy / CRC cost per GB on this CPU.
#include "crc32c.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

double now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}
double thread_cpu() {
  timespec t;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

void die(const char* what) {
  fprintf(stderr, "relaybench: %s: %s\n", what, strerror(errno));
  exit(2);
}

int listener(int* port) {
  int s = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (s < 0) die("socket");
  int one = 1;
  setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (bind(s, (sockaddr*)&a, sizeof a) < 0 || listen(s, 8) < 0) die("bind/listen");
  socklen_t l = sizeof a;
  getsockname(s, (sockaddr*)&a, &l);
  *port = ntohs(a.sin_port);
  return s;
}

int connect_to(int port) {
  int s = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons((uint16_t)port);
  if (connect(s, (sockaddr*)&a, sizeof a) < 0) die("connect");
  return s;
}

struct Pipe {
  int r = -1, w = -1;
  explicit Pipe(size_t cap) {
    int p[2];
    if (pipe2(p, O_CLOEXEC) < 0) die("pipe");
    r = p[0];
    w = p[1];
    fcntl(w, F_SETPIPE_SZ, (int)cap);
  }
  ~Pipe() {
    close(r);
    close(w);
  }
};

void splice_all(int from, int to, ssize_t n) {
  while (n > 0) {
    ssize_t k = splice(from, nullptr, to, nullptr, (size_t)n, SPLICE_F_MOVE | SPLICE_F_MORE);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) die("splice");
    n -= k;
  }
}

void send_all(int fd, const uint8_t* p, size_t n) {
  while (n > 0) {
    ssize_t k = send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) die("send");
    p += k;
    n -= (size_t)k;
  }
}

struct Result {
  double wall = 0, cpu = 0;
  uint32_t crc = 0;
};

// Relay exactly `total` bytes src -> dst in `mode`; the relay thread's CPU and wall time.
Result relay(int src, int dst, int64_t total, const std::string& mode, size_t pipe_cap,
             size_t buf_cap) {
  std::vector<uint8_t> buf(buf_cap);
  Pipe main(pipe_cap), dup(pipe_cap);
  Result r;
  const double c0 = thread_cpu(), w0 = now();
  int64_t moved = 0;
  while (moved < total) {
    const size_t want = (size_t)std::min<int64_t>(total - moved, (int64_t)pipe_cap);
    if (mode == "copycrc") {
      ssize_t k = recv(src, buf.data(), std::min(want, buf_cap), 0);
      if (k <= 0) die("recv");
      r.crc = crc32c_update(r.crc, buf.data(), (size_t)k);
      send_all(dst, buf.data(), (size_t)k);
      moved += k;
      continue;
    }
    if (mode == "peekcrc") {
      ssize_t k = recv(src, buf.data(), std::min(want, buf_cap), MSG_PEEK);
      if (k <= 0) die("recv(peek)");
      r.crc = crc32c_update(r.crc, buf.data(), (size_t)k);
      // exactly the peeked bytes: socket -> pipe -> socket
      for (ssize_t left = k; left > 0;) {
        ssize_t in = splice(src, nullptr, main.w, nullptr, (size_t)left, SPLICE_F_MOVE | SPLICE_F_MORE);
        if (in < 0 && errno == EINTR) continue;
        if (in <= 0) die("splice(src)");
        splice_all(main.r, dst, in);
        left -= in;
      }
      moved += k;
      continue;
    }
    ssize_t in = splice(src, nullptr, main.w, nullptr, want, SPLICE_F_MOVE | SPLICE_F_MORE);
    if (in < 0 && errno == EINTR) continue;
    if (in <= 0) die("splice(src)");
    if (mode == "splice") {
      splice_all(main.r, dst, in);
    } else {
      for (ssize_t left = in; left > 0;) {
        ssize_t t = tee(main.r, dup.w, (size_t)left, 0);
        if (t < 0 && errno == EINTR) continue;
        if (t <= 0) die("tee");
        for (ssize_t seen = 0; seen < t;) {
          ssize_t k = read(dup.r, buf.data(), std::min((size_t)(t - seen), buf_cap));
          if (k < 0 && errno == EINTR) continue;
          if (k <= 0) die("read(tee)");
          if (mode == "teecrc") r.crc = crc32c_update(r.crc, buf.data(), (size_t)k);
          seen += k;
        }
        splice_all(main.r, dst, t);
        left -= t;
      }
    }
    moved += in;
  }
  r.cpu = thread_cpu() - c0;
  r.wall = now() - w0;
  return r;
}

}  // namespace

int main(int argc, char** argv) {
  std::string mode = "splice";
  double gb = 4.0;
  int threads = 1;
  size_t pipe_kb = 1024, buf_kb = 256;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i], v = argv[i + 1];
    if (k == "--mode") mode = v;
    else if (k == "--gb") gb = atof(v.c_str());
    else if (k == "--threads") threads = atoi(v.c_str());
    else if (k == "--pipe-kb") pipe_kb = (size_t)atol(v.c_str());
    else if (k == "--buf-kb") buf_kb = (size_t)atol(v.c_str());
    else {
      fprintf(stderr, "relaybench: unknown option %s\n", k.c_str());
      return 2;
    }
  }
  if (mode != "splice" && mode != "tee" && mode != "teecrc" && mode != "peekcrc" &&
      mode != "copycrc") {
    fprintf(stderr, "relaybench: bad mode %s\n", mode.c_str());
    return 2;
  }
  const int64_t total = (int64_t)(gb * 1e9);
  // the producer's body: 4 MiB of pseudo-random bytes sent over and over
  std::vector<uint8_t> body(4 << 20);
  uint64_t x = 0x9e3779b97f4a7c15ull;
  for (auto& b : body) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    b = (uint8_t)x;
  }
  uint32_t want_crc = 0;
  for (int64_t off = 0; off < total;) {
    size_t k = (size_t)std::min<int64_t>(total - off, (int64_t)body.size());
    want_crc = crc32c_update(want_crc, body.data(), k);
    off += (int64_t)k;
  }
  std::vector<Result> res((size_t)threads);
  std::vector<std::thread> ths;
  std::atomic<int> bad{0};
  for (int t = 0; t < threads; ++t) {
    ths.emplace_back([&, t] {
      int pa, pb;
      int la = listener(&pa), lb = listener(&pb);
      std::thread producer([&] {
        int s = connect_to(pa);
        for (int64_t off = 0; off < total;) {
          size_t k = (size_t)std::min<int64_t>(total - off, (int64_t)body.size());
          send_all(s, body.data(), k);
          off += (int64_t)k;
        }
        close(s);
      });
      int src = accept4(la, nullptr, nullptr, SOCK_CLOEXEC);
      int dst = connect_to(pb);
      int sink = accept4(lb, nullptr, nullptr, SOCK_CLOEXEC);
      std::thread consumer([&] {
        std::vector<uint8_t> scratch(1 << 20);
        int64_t got = 0;
        while (got < total) {
          ssize_t k = recv(sink, scratch.data(), scratch.size(), MSG_TRUNC);
          if (k < 0 && errno == EINTR) continue;
          if (k <= 0) die("recv(sink)");
          got += k;
        }
      });
      res[(size_t)t] = relay(src, dst, total, mode, pipe_kb << 10, buf_kb << 10);
      producer.join();
      consumer.join();
      if ((mode == "teecrc" || mode == "peekcrc" || mode == "copycrc") &&
          res[(size_t)t].crc != want_crc)
        bad.fetch_add(1);
      close(src);
      close(dst);
      close(sink);
      close(la);
      close(lb);
    });
  }
  for (auto& th : ths) th.join();
  double wall = 0, cpu = 0;
  for (auto& r : res) {
    wall = std::max(wall, r.wall);
    cpu += r.cpu;
  }
  const double all_gb = total * threads / 1e9;
  printf("{\"mode\": \"%s\", \"threads\": %d, \"gb_per_thread\": %.2f, \"pipe_kb\": %zu, "
         "\"buf_kb\": %zu, \"GBps\": %.2f, \"relay_cpu_s_per_GB\": %.4f, \"crc_ok\": %s, "
         "\"crc_impl\": \"%s\"}\n",
         mode.c_str(), threads, total / 1e9, pipe_kb, buf_kb, all_gb / wall, cpu / all_gb,
         bad.load() ? "false" : "true", crc32c_detail::have_vpclmul() ? "avx512-vpclmulqdq" : "sse4.2-3way");
  return bad.load() ? 1 : 0;
}
