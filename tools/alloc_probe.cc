// Times hipMalloc of CHUNK_GIB blocks until TOTAL_GIB are held (none freed),
// printing the host time of each call: where the allocator starts to wait
// after another process freed HBM (tools/gpu_alloc_stall_probe.sh).
// Build: hipcc --offload-arch=gfx950 -O2 tools/alloc_probe.cc -o tools/bin/alloc_probe
// Usage: alloc_probe TOTAL_GIB CHUNK_GIB
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char **argv) {
  const int total = argc > 1 ? atoi(argv[1]) : 64, chunk = argc > 2 ? atoi(argv[2]) : 4;
  const auto t0 = std::chrono::steady_clock::now();
  auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  if (hipSetDevice(0) != hipSuccess) return 1;
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  printf("t=%.1f ms init, free %.1f of %.1f GiB\n", ms(), fr / 1073741824.0, tot / 1073741824.0);
  std::vector<void *> held;
  for (int have = 0; have + chunk <= total; have += chunk) {
    void *p = nullptr;
    const double a = ms();
    const hipError_t e = hipMalloc(&p, static_cast<size_t>(chunk) << 30);
    const double b = ms();
    (void)hipMemGetInfo(&fr, &tot);
    printf("t=%.1f ms: hold %d GiB, call %.1f ms, rc %d, free %.1f GiB\n", b, have + chunk, b - a, static_cast<int>(e),
           fr / 1073741824.0);
    if (e != hipSuccess) break;
    held.push_back(p);
  }
  for (void *p : held) (void)hipFree(p);
  return 0;
}
