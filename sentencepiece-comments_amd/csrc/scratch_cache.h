// scratch_cache.h — reuse of the trainer's large device scratch across stages.
//
// Seed mining holds ~35 B per corpus char of sort/rank/LCP scratch (~87 GB at
// BASELINE config 5's 100 M lines) and frees it before the whitespace split
// and the E-steps allocate theirs.  A fresh hipMalloc of memory that another
// process (or an earlier stage) used is paid again on the host when the
// driver hands the pages out: on a box that had just run the GPU tests, c5
// spent 3.7 s of seed mining and 4.0 s of the split inside hipMalloc
// (profiles/r03zb_bench.json), against 4 ms in a fresh process.
//
// While a CacheScope is open, the blocks these stages free are kept as free
// ranges of their hipMalloc'd base blocks: a request is carved best-fit out
// of the smallest free range that holds it (256-byte granules), so a small
// counter takes 256 bytes of a large range, not the whole range; freed
// ranges coalesce with free neighbours of the same base.  ScratchFree
// records an event on the stream the block was used on; the next carve from
// that range waits for the event (not for the whole device).  The scope's end
// frees every base.  Outside a scope the calls are plain hipMalloc / hipFree.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace spm_amd {

// Device-memory accounting.  Every device block the library allocates (the
// scratch cache's bases, the encoder's and E-step's workspaces, the trainer's
// corpus and scratch) goes through DevMalloc / DevFree, which keep the live
// byte count and its high-water mark for the process: spm_train reports the
// peak of a training run (peak_device_bytes) and bench.py the peak per rank.
hipError_t DevMallocRaw(void **p, uint64_t bytes);
hipError_t DevFree(void *p);
template <class T>
hipError_t DevMalloc(T **p, uint64_t bytes) {
  return DevMallocRaw(reinterpret_cast<void **>(p), bytes);
}
uint64_t DevLiveBytes();
uint64_t DevPeakBytes();
void DevPeakReset();  // high-water mark := live bytes

// Defined in scratch_cache.cc (one instance in libspm_hip.so).
hipError_t ScratchAlloc(void **p, uint64_t bytes);
void ScratchFree(void *p, hipStream_t st = nullptr);
void ScratchCacheBegin();
void ScratchCacheEnd();  // frees every cached block

// Introspection for tests: bases held and their bytes, free ranges and their
// bytes, bytes handed out, hipMalloc calls made inside scopes.
struct ScratchCacheStats {
  uint64_t bases, base_bytes, ranges, free_bytes, used_bytes, mallocs;
};
ScratchCacheStats ScratchCacheGetStats();

struct ScratchCacheScope {
  ScratchCacheScope() { ScratchCacheBegin(); }
  ~ScratchCacheScope() { ScratchCacheEnd(); }
  ScratchCacheScope(const ScratchCacheScope &) = delete;
  ScratchCacheScope &operator=(const ScratchCacheScope &) = delete;
};

}  // namespace spm_amd
