// swarmd - heterogeneous fake BitTorrent seeders for the swarm bench and tests.
//
// The reference's main torrent path is a public magnet through webtorrent
// (/root/reference/lib/download.js:64-121): up to 55 peers a torrent (webtorrent's default),
// over links of very different speed and latency, some of which stall or disappear. The
// loopback seeders of config 6 are 1 - 4 fast, zero-RTT peers; this process plays a realistic
// swarm instead. Each line of --peers is one seeder on its own 127.0.0.1 port:
//
//   <rate bytes/s> <delay ms> <stall after bytes> <hang up after bytes>
//
//   rate    token bucket on the PIECE payload it sends (burst: 64 KiB or 50 ms of rate)
//   delay   every REQUEST is answered no earlier than this after it arrived (one-way
//           latency of the link, as seen by the leecher's request pipeline)
//   stall   after this many payload bytes the peer stops answering - mid-piece - but keeps
//           the connection open and reads (0: never)
//   hangup  after this many payload bytes the peer closes the connection (0: never)
//
// Protocol: BEP-3 handshake (no extensions), a full BITFIELD, UNCHOKE, then REQUEST / CANCEL;
// blocks are read from --file (the torrent's single data file) with pread. One thread reads
// and one sends per connection: this is a test peer, not production code.
//
//   swarmd --file DATA --info-hash HEX40 --pieces N --peers SPEC --port-file OUT
// The port file gets one port per spec line, in order. /stats is not served: the seeders'
// counters go to stderr when the process is told to stop (SIGTERM).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

struct Spec {
  double rate = 0;        // bytes/s (0: unlimited)
  int delay_ms = 0;
  uint64_t stall = 0, hangup = 0;
};

struct Counters {
  std::atomic<uint64_t> sent{0}, requests{0}, cancels{0}, conns{0};
};

int g_file = -1;
uint64_t g_file_size = 0;
uint8_t g_info_hash[20];
uint32_t g_pieces = 0, g_piece_len = 0;
std::vector<Spec> g_specs;
std::vector<std::unique_ptr<Counters>> g_counters;

uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
void put32(std::string& s, uint32_t v) {
  char b[4] = {(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
  s.append(b, 4);
}

bool read_n(int fd, void* p, size_t n) {
  uint8_t* c = (uint8_t*)p;
  while (n) {
    ssize_t r = ::recv(fd, c, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    c += r;
    n -= (size_t)r;
  }
  return true;
}

bool send_n(int fd, const void* p, size_t n, int flags = 0) {
  const uint8_t* c = (const uint8_t*)p;
  while (n) {
    ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL | flags);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    c += w;
    n -= (size_t)w;
  }
  return true;
}

struct Request {
  uint32_t idx, begin, len;
  Clock::time_point ready;
};

// One leecher connection to seeder `k`.
void serve_conn(int fd, int k) {
  const Spec sp = g_specs[(size_t)k];
  Counters& ct = *g_counters[(size_t)k];
  ct.conns++;
  uint8_t hs[68];
  if (!read_n(fd, hs, 68) || hs[0] != 19 || memcmp(hs + 1, "BitTorrent protocol", 19) != 0 ||
      memcmp(hs + 28, g_info_hash, 20) != 0) {
    ::close(fd);
    return;
  }
  std::string out;
  out.push_back((char)19);
  out += "BitTorrent protocol";
  out.append(8, '\0');
  out.append((const char*)g_info_hash, 20);
  char pid[21];
  snprintf(pid, sizeof pid, "-SD0001-%012d", k);
  out.append(pid, 20);
  const uint32_t nb = (g_pieces + 7) / 8;
  put32(out, nb + 1);
  out.push_back((char)5);
  std::string bits(nb, (char)0xff);
  if (g_pieces % 8) bits.back() = (char)(0xff << (8 - g_pieces % 8));
  out += bits;
  put32(out, 1);
  out.push_back((char)1);   // UNCHOKE
  if (!send_n(fd, out.data(), out.size())) {
    ::close(fd);
    return;
  }
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Request> q;
  bool closed = false;
  std::thread sender([&] {
    double tokens = 0;
    const double cap = std::max(65536.0, sp.rate * 0.05);
    Clock::time_point last = Clock::now();
    uint64_t sent = 0;
    bool stalled = false;
    std::vector<uint8_t> buf;
    for (;;) {
      Request r;
      {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
          if (closed) return;
          if (!q.empty() && !stalled) {
            const auto now = Clock::now();
            if (q.front().ready <= now) break;
            cv.wait_until(lk, q.front().ready);
            continue;
          }
          cv.wait(lk);
        }
        r = q.front();
        q.pop_front();
      }
      if (sp.rate > 0) {
        for (;;) {
          const auto now = Clock::now();
          tokens = std::min(cap, tokens + sp.rate * std::chrono::duration<double>(now - last).count());
          last = now;
          if (tokens >= r.len) break;
          std::this_thread::sleep_for(std::chrono::duration<double>((r.len - tokens) / sp.rate));
        }
        tokens -= r.len;
      }
      buf.resize(13 + r.len);
      std::string hdr;
      put32(hdr, r.len + 9);
      hdr.push_back((char)7);
      put32(hdr, r.idx);
      put32(hdr, r.begin);
      memcpy(buf.data(), hdr.data(), 13);
      const uint64_t off = (uint64_t)r.idx * g_piece_len + r.begin;
      if (::pread(g_file, buf.data() + 13, r.len, (off_t)off) != (ssize_t)r.len) break;
      if (!send_n(fd, buf.data(), buf.size())) break;
      sent += r.len;
      ct.sent += r.len;
      if (sp.hangup && sent >= sp.hangup) {
        ::shutdown(fd, SHUT_RDWR);
        break;
      }
      if (sp.stall && sent >= sp.stall) stalled = true;     // mid-piece: never answers again
    }
    std::lock_guard<std::mutex> g(mu);
    closed = true;
  });
  // reader: REQUEST / CANCEL; everything else is ignored
  std::vector<uint8_t> m;
  for (;;) {
    uint8_t lb[4];
    if (!read_n(fd, lb, 4)) break;
    const uint32_t n = be32(lb);
    if (n > (1u << 20)) break;
    m.resize(n);
    if (n && !read_n(fd, m.data(), n)) break;
    if (n == 13 && (m[0] == 6 || m[0] == 8)) {
      const uint32_t idx = be32(&m[1]), begin = be32(&m[5]), len = be32(&m[9]);
      if (idx >= g_pieces || len == 0 || len > 131072 ||
          (uint64_t)idx * g_piece_len + begin + len > g_file_size)
        continue;
      std::lock_guard<std::mutex> g(mu);
      if (m[0] == 6) {
        ct.requests++;
        q.push_back(Request{idx, begin, len, Clock::now() + std::chrono::milliseconds(sp.delay_ms)});
      } else {
        ct.cancels++;
        for (auto it = q.begin(); it != q.end(); ++it)
          if (it->idx == idx && it->begin == begin && it->len == len) {
            q.erase(it);
            break;
          }
      }
      cv.notify_all();
    }
  }
  {
    std::lock_guard<std::mutex> g(mu);
    closed = true;
  }
  cv.notify_all();
  sender.join();
  ::close(fd);
}

std::atomic<bool> g_stop{false};

void on_term(int) { g_stop.store(true); }

}  // namespace

int main(int argc, char** argv) {
  std::string file, ih, peers, port_file;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&] { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (a == "--file") file = next();
    else if (a == "--info-hash") ih = next();
    else if (a == "--pieces") g_pieces = (uint32_t)strtoul(next().c_str(), nullptr, 10);
    else if (a == "--piece-length") g_piece_len = (uint32_t)strtoul(next().c_str(), nullptr, 10);
    else if (a == "--peers") peers = next();
    else if (a == "--port-file") port_file = next();
    else {
      fprintf(stderr, "usage: swarmd --file F --info-hash HEX --pieces N --piece-length L "
                      "--peers SPEC --port-file OUT\n");
      return 2;
    }
  }
  if (ih.size() != 40 || !g_pieces || !g_piece_len) {
    fprintf(stderr, "swarmd: --info-hash (40 hex), --pieces and --piece-length are required\n");
    return 2;
  }
  for (int i = 0; i < 20; ++i) g_info_hash[i] = (uint8_t)strtoul(ih.substr(2 * i, 2).c_str(), nullptr, 16);
  g_file = ::open(file.c_str(), O_RDONLY | O_CLOEXEC);
  if (g_file < 0) {
    perror("swarmd: open");
    return 1;
  }
  g_file_size = (uint64_t)::lseek(g_file, 0, SEEK_END);
  FILE* f = fopen(peers.c_str(), "r");
  if (!f) {
    perror("swarmd: peers");
    return 1;
  }
  char line[256];
  while (fgets(line, sizeof line, f)) {
    Spec s;
    unsigned long long st = 0, hu = 0;
    if (sscanf(line, "%lf %d %llu %llu", &s.rate, &s.delay_ms, &st, &hu) >= 2) {
      s.stall = st;
      s.hangup = hu;
      g_specs.push_back(s);
    }
  }
  fclose(f);
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa {};
  sa.sa_handler = on_term;
  sigaction(SIGTERM, &sa, nullptr);
  std::vector<int> ls;
  std::string ports;
  for (size_t k = 0; k < g_specs.size(); ++k) {
    g_counters.emplace_back(new Counters());
    int s = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(s, (sockaddr*)&a, sizeof a) < 0 || listen(s, 16) < 0) {
      perror("swarmd: bind");
      return 1;
    }
    socklen_t l = sizeof a;
    getsockname(s, (sockaddr*)&a, &l);
    ports += std::to_string(ntohs(a.sin_port)) + "\n";
    ls.push_back(s);
  }
  for (size_t k = 0; k < ls.size(); ++k) {
    std::thread([k, s = ls[k]] {
      for (;;) {
        int c = accept4(s, nullptr, nullptr, SOCK_CLOEXEC);
        if (c < 0) {
          if (errno == EINTR) continue;
          return;
        }
        int one = 1;
        setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        std::thread(serve_conn, c, (int)k).detach();
      }
    }).detach();
  }
  {
    std::string tmp = port_file + ".tmp";
    FILE* pf = fopen(tmp.c_str(), "w");
    if (!pf) return 1;
    fputs(ports.c_str(), pf);
    fclose(pf);
    rename(tmp.c_str(), port_file.c_str());
  }
  while (!g_stop.load()) pause();
  for (size_t k = 0; k < g_specs.size(); ++k)
    fprintf(stderr, "seeder %zu: %llu B sent, %llu requests, %llu cancels, %llu conns\n", k,
            (unsigned long long)g_counters[k]->sent.load(),
            (unsigned long long)g_counters[k]->requests.load(),
            (unsigned long long)g_counters[k]->cancels.load(),
            (unsigned long long)g_counters[k]->conns.load());
  return 0;
}
