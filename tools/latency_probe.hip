// Per-call latency building blocks on the box: what a
// small-batch encode round trip can cost.  Prints one line per variant:
// mean microseconds over N calls.
//   hipcc --offload-arch=gfx950 -O2 tools/latency_probe.hip -o tools/bin/latency_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

__global__ void empty_kernel(int *p) {
  if (threadIdx.x == 0 && p) p[0] += 0;
}

// Copies `n` bytes host -> device (dwords), 256 threads.
__global__ void stage_kernel(const uint32_t *src, uint32_t *dst, uint32_t nw) {
  for (uint32_t k = threadIdx.x; k < nw; k += blockDim.x) dst[k] = src[k];
}

__global__ void publish_kernel(const uint32_t *src, uint32_t *host_dst, uint32_t nw, uint32_t *flag, uint32_t seq) {
  for (uint32_t k = threadIdx.x; k < nw; k += blockDim.x) host_dst[k] = src[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int Spin(hipStream_t st) {
  for (;;) {
    const hipError_t e = hipStreamQuery(st);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotReady) return 1;
  }
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 2000;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int *d = nullptr;
  uint32_t *h = nullptr, *dd = nullptr;
  CK(hipMalloc(&d, 1 << 20));
  CK(hipMalloc(&dd, 1 << 20));
  CK(hipHostMalloc(&h, 1 << 20));
  std::memset(h, 1, 1 << 20);
  auto bench = [&](const char *name, auto &&body) -> int {
    for (int k = 0; k < 50; ++k)
      if (body(k)) return 1;
    const double t0 = Now();
    for (int k = 0; k < N; ++k)
      if (body(k)) return 1;
    std::printf("%-44s %8.2f us\n", name, (Now() - t0) * 1e6 / N);
    return 0;
  };
  int rc = 0;
  rc |= bench("launch + hipStreamSynchronize", [&](int) {
    empty_kernel<<<1, 64, 0, st>>>(d);
    return hipStreamSynchronize(st) != hipSuccess;
  });
  rc |= bench("launch + spin hipStreamQuery", [&](int) {
    empty_kernel<<<1, 64, 0, st>>>(d);
    return Spin(st);
  });
  rc |= bench("3 launches + spin", [&](int) {
    for (int j = 0; j < 3; ++j) empty_kernel<<<1, 64, 0, st>>>(d);
    return Spin(st);
  });
  rc |= bench("6 launches + spin", [&](int) {
    for (int j = 0; j < 6; ++j) empty_kernel<<<1, 64, 0, st>>>(d);
    return Spin(st);
  });
  rc |= bench("H2D 256 B memcpyAsync + sync", [&](int) {
    return hipMemcpyAsync(dd, h, 256, hipMemcpyHostToDevice, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess;
  });
  rc |= bench("H2D 256 B + D2H 256 B memcpyAsync + spin", [&](int) {
    return hipMemcpyAsync(dd, h, 256, hipMemcpyHostToDevice, st) != hipSuccess ||
           hipMemcpyAsync(h + 1024, dd, 256, hipMemcpyDeviceToHost, st) != hipSuccess || Spin(st);
  });
  rc |= bench("stage kernel 256 B from pinned + spin", [&](int) {
    stage_kernel<<<1, 256, 0, st>>>(h, dd, 64);
    return Spin(st);
  });
  rc |= bench("stage 4 KB + empty + publish 256 B + spin", [&](int) {
    stage_kernel<<<1, 256, 0, st>>>(h, dd, 1024);
    empty_kernel<<<1, 64, 0, st>>>(d);
    publish_kernel<<<1, 256, 0, st>>>(dd, h + 4096, 64, h + 8192, 1);
    return Spin(st);
  });
  volatile uint32_t *flag = h + 8192;
  rc |= bench("stage + empty + publish + poll host flag", [&](int k) {
    const uint32_t seq = 1000 + k;
    stage_kernel<<<1, 256, 0, st>>>(h, dd, 1024);
    empty_kernel<<<1, 64, 0, st>>>(d);
    publish_kernel<<<1, 256, 0, st>>>(dd, h + 4096, 64, h + 8192, seq);
    const double t0 = Now();
    while (*flag != seq)
      if (Now() - t0 > 1.0) return 1;
    return 0;
  });
  (void)hipStreamSynchronize(st);
  std::printf("%s\n", rc ? "FAILED" : "DONE");
  return rc;
}
