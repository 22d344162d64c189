// Probe 2: first-time cost of DMA straight out of the page cache. For each registration
// thread count T, map the file afresh (no PTEs yet), register 256 MiB segments on T threads
// and DMA each segment to the device as soon as it is registered.
//   hipcc --offload-arch=gfx950 -O2 host_register_probe2.hip -o host_register_probe2
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/resource.h>
#include <thread>
#include <unistd.h>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double cpu() {
  rusage r;
  getrusage(RUSAGE_SELF, &r);
  return r.ru_utime.tv_sec + r.ru_stime.tv_sec + 1e-6 * (r.ru_utime.tv_usec + r.ru_stime.tv_usec);
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"step\": \"%s\", \"error\": \"%s\"}\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  int fd = open(argv[1], O_RDONLY);
  struct stat st;
  fstat(fd, &st);
  const size_t seg = 256 << 20;
  size_t n = ((size_t)st.st_size / seg) * seg, nseg = n / seg;
  uint8_t* d = nullptr;
  CK(hipMalloc((void**)&d, n));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (int T : {1, 4, 8, 1}) {
    void* p = mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
    std::vector<std::atomic<int>> ready(nseg);
    for (auto& r : ready) r = 0;
    std::atomic<size_t> next{0};
    double a0 = now(), c0 = cpu();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
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
    double a1 = now(), c1 = cpu();
    for (auto& x : th) x.join();
    double u0 = now();
    for (size_t i = 0; i < nseg; ++i) if (ready[i] > 0) CK(hipHostUnregister((uint8_t*)p + i * seg));
    double u1 = now();
    munmap(p, n);
    printf("{\"threads\": %d, \"fresh_register_dma_GBps\": %.1f, \"cpu_s\": %.3f, \"unregister_s\": %.4f, \"failed\": %d}\n",
           T, n / (a1 - a0) / 1e9, c1 - c0, u1 - u0, bad);
    fflush(stdout);
  }
  return 0;
}
