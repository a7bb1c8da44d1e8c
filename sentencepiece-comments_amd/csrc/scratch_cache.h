// scratch_cache.h — reuse of the trainer's large device scratch across stages.
//
// Seed mining holds ~35 B per corpus char of sort/rank/LCP scratch (~87 GB at
// BASELINE config 5's 100 M lines) and frees it before the whitespace split
// and the E-steps allocate theirs.  A fresh hipMalloc of memory that another
// process (or an earlier stage) used is paid again on the host when the
// driver hands the pages out: on a box that had just run the GPU tests, c5
// spent 3.7 s of seed mining and 4.0 s of the split inside hipMalloc
// (profiles/r03zb_bench.json), against 4 ms in a fresh process.  While a
// CacheScope is open, blocks the seed and split stages free are kept and
// handed back best-fit to later requests of these stages; the scope's end
// frees them.  Outside a scope the calls are plain hipMalloc / hipFree.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace spm_amd {

// Defined in seed_kernels.hip (one instance in libspm_hip.so).
hipError_t ScratchAlloc(void **p, uint64_t bytes);
void ScratchFree(void *p);
void ScratchCacheBegin();
void ScratchCacheEnd();  // frees every cached block

struct ScratchCacheScope {
  ScratchCacheScope() { ScratchCacheBegin(); }
  ~ScratchCacheScope() { ScratchCacheEnd(); }
  ScratchCacheScope(const ScratchCacheScope &) = delete;
  ScratchCacheScope &operator=(const ScratchCacheScope &) = delete;
};

}  // namespace spm_amd
