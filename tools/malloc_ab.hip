// hipMalloc cost on the box: per-byte or per-call, and does GPU work queued
// before a large hipMalloc keep running while the host is inside it?
// Build: hipcc -O2 --offload-arch=gfx950 tools/malloc_ab.hip -o /tmp/malloc_ab
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void spin(uint64_t *p, uint64_t n) {
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t x = i;
  for (int k = 0; k < 20000; ++k) x = x * 6364136223846793005ull + 1442695040888963407ull;
  if (i < n) p[i] = x;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const uint64_t GB = 1ull << 30;
  for (uint64_t sz : {1 * GB, 4 * GB, 16 * GB, 32 * GB}) {
    void *p = nullptr;
    double t0 = now_ms();
    if (hipMalloc(&p, sz) != hipSuccess) { printf("alloc %llu failed\n", (unsigned long long)sz); return 1; }
    double t1 = now_ms();
    hipFree(p);
    double t2 = now_ms();
    printf("hipMalloc %3llu GB: %8.2f ms   hipFree %8.2f ms\n", (unsigned long long)(sz / GB), t1 - t0, t2 - t1);
  }
  // 8 x 4 GB vs 1 x 32 GB
  {
    std::vector<void *> v(8);
    double t0 = now_ms();
    for (auto &p : v) hipMalloc(&p, 4 * GB);
    double t1 = now_ms();
    for (auto p : v) hipFree(p);
    printf("8 x 4 GB: %8.2f ms\n", t1 - t0);
  }
  // Overlap: queue ~200 ms of GPU work, then hipMalloc 32 GB; sync.
  uint64_t *d;
  hipMalloc(&d, 1 << 26);
  hipStream_t st;
  hipStreamCreate(&st);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int pass = 0; pass < 2; ++pass) {
    double t0 = now_ms();
    hipEventRecord(e0, st);
    spin<<<8192, 256, 0, st>>>(d, 1 << 23);
    hipEventRecord(e1, st);
    void *p = nullptr;
    double ta = now_ms();
    if (pass) hipMalloc(&p, 32 * GB);
    double tb = now_ms();
    hipStreamSynchronize(st);
    double t1 = now_ms();
    float k = 0;
    hipEventElapsedTime(&k, e0, e1);
    printf("spin kernel %.2f ms; %s: host malloc %.2f ms, wall %.2f ms\n", k, pass ? "with 32 GB malloc" : "alone", tb - ta,
           t1 - t0);
    if (p) hipFree(p);
  }
  // hipMallocAsync from the default pool, then again after a free (reuse).
  for (int r = 0; r < 2; ++r) {
    void *p = nullptr;
    double t0 = now_ms();
    hipMallocAsync(&p, 16 * GB, st);
    hipStreamSynchronize(st);
    double t1 = now_ms();
    hipFreeAsync(p, st);
    hipStreamSynchronize(st);
    printf("hipMallocAsync 16 GB (round %d): %.2f ms\n", r, t1 - t0);
  }
  return 0;
}
