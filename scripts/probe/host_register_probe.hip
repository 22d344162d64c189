// Probe: can the MI355X DMA straight out of the page cache? hipHostRegister a read-only
// MAP_SHARED mapping of a file, then time H2D copies from it (1D and 2D strided) vs the
// pinned-staging path (pread into hipHostMalloc memory + copy).
//   hipcc --offload-arch=gfx950 -O2 host_register_probe.hip -o host_register_probe
//   ./host_register_probe FILE
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <atomic>
#include <thread>
#include <unistd.h>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"step\": \"%s\", \"error\": \"%s\"}\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  int fd = open(argv[1], O_RDONLY);
  struct stat st;
  fstat(fd, &st);
  size_t n = (size_t)st.st_size & ~(size_t)4095;
  void* p = mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) { printf("{\"error\": \"mmap\"}\n"); return 1; }
  madvise(p, n, MADV_WILLNEED);
  uint8_t* d = nullptr;
  CK(hipMalloc((void**)&d, n));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  unsigned flags[] = {hipHostRegisterReadOnly, hipHostRegisterDefault};
  const char* names[] = {"readonly", "default"};
  for (int f = 0; f < 2; ++f) {
    double t0 = now();
    hipError_t e = hipHostRegister(p, n, flags[f]);
    double t1 = now();
    printf("{\"register\": \"%s\", \"ok\": %s, \"err\": \"%s\", \"s\": %.4f, \"bytes\": %zu}\n", names[f],
           e == hipSuccess ? "true" : "false", hipGetErrorString(e), t1 - t0, n);
    fflush(stdout);
    if (e != hipSuccess) { (void)hipGetLastError(); continue; }
    for (int rep = 0; rep < 3; ++rep) {
      double a = now();
      CK(hipMemcpyAsync(d, p, n, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      double b = now();
      // 2D: 64 KiB rows at a 4 MiB pitch (chunk c of every 4 MiB piece)
      const size_t pitch = 4 << 20, w = 64 << 10, h = n / pitch;
      double c0 = now();
      for (size_t c = 0; c < pitch / w; ++c)
        CK(hipMemcpy2DAsync(d + c * w, pitch, (uint8_t*)p + c * w, pitch, w, h, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      double c1 = now();
      printf("{\"flags\": \"%s\", \"rep\": %d, \"h2d_1d_GBps\": %.1f, \"h2d_2d_64k_rows_GBps\": %.1f}\n",
             names[f], rep, n / (b - a) / 1e9, (h * pitch) / (c1 - c0) / 1e9);
      fflush(stdout);
    }
    double u0 = now();
    CK(hipHostUnregister(p));
    printf("{\"unregister_s\": %.4f}\n", now() - u0);
    break;
  }
  // parallel registration: T threads each register n/T bytes (page aligned)
  for (int T : {1, 2, 4, 8, 16}) {
    size_t per = (n / T) & ~(size_t)4095;
    std::vector<std::thread> th;
    std::vector<hipError_t> errs(T, hipSuccess);
    double r0 = now();
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] { errs[t] = hipHostRegister((uint8_t*)p + t * per, per, hipHostRegisterReadOnly); });
    for (auto& x : th) x.join();
    double r1 = now();
    int bad = 0;
    for (auto e : errs) bad += e != hipSuccess;
    for (int t = 0; t < T; ++t) if (errs[t] == hipSuccess) (void)hipHostUnregister((uint8_t*)p + t * per);
    printf("{\"register_threads\": %d, \"s\": %.4f, \"GBps\": %.1f, \"failed\": %d}\n", T, r1 - r0,
           (double)per * T / (r1 - r0) / 1e9, bad);
    fflush(stdout);
  }
  // register + DMA pipelined in 256 MiB segments (registration on 4 threads ahead of the copy)
  {
    const size_t seg = 256 << 20;
    size_t nseg = n / seg;
    std::vector<std::atomic<int>> ready(nseg);
    for (auto& r : ready) r = 0;
    std::atomic<size_t> next{0};
    double a0 = now();
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t)
      th.emplace_back([&] {
        for (size_t i; (i = next.fetch_add(1)) < nseg;) {
          hipError_t e = hipHostRegister((uint8_t*)p + i * seg, seg, hipHostRegisterReadOnly);
          ready[i] = e == hipSuccess ? 1 : -1;
        }
      });
    int bad = 0;
    for (size_t i = 0; i < nseg; ++i) {
      while (ready[i] == 0) std::this_thread::yield();
      if (ready[i] < 0) { bad++; continue; }
      CK(hipMemcpyAsync(d + i * seg, (uint8_t*)p + i * seg, seg, hipMemcpyHostToDevice, s));
    }
    CK(hipStreamSynchronize(s));
    double a1 = now();
    for (auto& x : th) x.join();
    for (size_t i = 0; i < nseg; ++i) if (ready[i] > 0) (void)hipHostUnregister((uint8_t*)p + i * seg);
    printf("{\"pipelined_register_dma_GBps\": %.1f, \"failed\": %d}\n", nseg * seg / (a1 - a0) / 1e9, bad);
    fflush(stdout);
  }
  // baseline: pread into pinned staging (8 threads) + copy, 256 MiB slots
  const size_t slot = 256 << 20;
  uint8_t* h = nullptr;
  CK(hipHostMalloc((void**)&h, slot, hipHostMallocDefault));
  double a = now();
  for (size_t off = 0; off < n; off += slot) {
    size_t len = std::min(slot, n - off);
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t)
      th.emplace_back([&, t] {
        size_t per = len / 8, o = t * per, l = t == 7 ? len - o : per;
        size_t got = 0;
        while (got < l) { ssize_t r = pread(fd, h + o + got, l - got, off + o + got); if (r <= 0) break; got += r; }
      });
    for (auto& x : th) x.join();
    CK(hipMemcpy(d + off, h, len, hipMemcpyHostToDevice));
  }
  printf("{\"pread_pinned_serial_GBps\": %.1f}\n", n / (now() - a) / 1e9);
  return 0;
}
