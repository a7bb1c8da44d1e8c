// scratch_cache_selftest — checks the trainer's scratch cache
// (scratch_cache.h) on a GPU: carving, best fit, coalescing, disjoint
// ranges, release at scope end and at the last free after it.  Prints "ok"
// and exits 0, or names the failed check and exits 1.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "scratch_cache.h"

using namespace spm_amd;

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "scratch_cache_selftest: %s (line %d)\n", #c, __LINE__); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

int main() {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess);
  const uint64_t MB = 1 << 20;
  void *held = nullptr;
  {
    ScratchCacheScope scope;
    void *a, *b;
    CHECK(ScratchAlloc(&a, MB) == hipSuccess);
    CHECK(ScratchAlloc(&b, 4 * MB) == hipSuccess);
    CHECK(hipMemsetAsync(a, 1, MB, st) == hipSuccess);
    CHECK(hipMemsetAsync(b, 2, 4 * MB, st) == hipSuccess);
    ScratchFree(a, st);
    ScratchFree(b, st);
    ScratchCacheStats s = ScratchCacheGetStats();
    CHECK(s.bases == 2 && s.ranges == 2 && s.free_bytes == 5 * MB && s.used_bytes == 0 && s.mallocs == 2);
    // A 4-byte counter is carved from the 1 MB base (best fit), not the 4 MB.
    void *c, *d, *e, *f;
    CHECK(ScratchAlloc(&c, 4) == hipSuccess);
    CHECK(c == a);
    CHECK(ScratchAlloc(&d, 4 * MB) == hipSuccess);
    CHECK(d == b);
    CHECK(ScratchAlloc(&e, MB - 256) == hipSuccess);
    CHECK(static_cast<char *>(e) == static_cast<char *>(a) + 256);
    s = ScratchCacheGetStats();
    CHECK(s.mallocs == 2 && s.ranges == 0 && s.used_bytes == 5 * MB);
    // Nothing left: a fresh base.
    CHECK(ScratchAlloc(&f, 100) == hipSuccess);
    CHECK(ScratchCacheGetStats().mallocs == 3);
    // Disjoint ranges: distinct fills survive.
    CHECK(hipMemsetAsync(c, 7, 256, st) == hipSuccess);
    CHECK(hipMemsetAsync(e, 9, MB - 256, st) == hipSuccess);
    std::vector<unsigned char> h(MB);
    CHECK(hipMemcpyAsync(h.data(), a, MB, hipMemcpyDeviceToHost, st) == hipSuccess);
    CHECK(hipStreamSynchronize(st) == hipSuccess);
    CHECK(h[0] == 7 && h[255] == 7 && h[256] == 9 && h[MB - 1] == 9);
    // Frees in any order coalesce back to one range per base.
    ScratchFree(e, st);
    ScratchFree(d, st);
    ScratchFree(c, st);
    ScratchFree(f, st);
    s = ScratchCacheGetStats();
    CHECK(s.bases == 3 && s.ranges == 3 && s.free_bytes == s.base_bytes && s.used_bytes == 0);
    // A range in use when the scope ends is freed by its last ScratchFree.
    CHECK(ScratchAlloc(&held, 2 * MB) == hipSuccess);
    CHECK(held == b);
  }
  ScratchCacheStats s = ScratchCacheGetStats();
  CHECK(s.bases == 1 && s.used_bytes == 2 * MB);
  ScratchFree(held, st);
  s = ScratchCacheGetStats();
  CHECK(s.bases == 0 && s.ranges == 0 && s.used_bytes == 0);
  // Outside a scope: plain hipMalloc / hipFree.
  CHECK(ScratchAlloc(&held, 1000) == hipSuccess);
  CHECK(ScratchCacheGetStats().bases == 0);
  ScratchFree(held, st);
  CHECK(hipStreamSynchronize(st) == hipSuccess);
  std::puts("ok");
  return 0;
}
