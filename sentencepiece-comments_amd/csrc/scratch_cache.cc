// scratch_cache.cc — the trainer's device scratch cache (scratch_cache.h).
//
// Bases are hipMalloc'd blocks; inside a scope every request is a range of
// some base.  Free ranges are indexed by address (to coalesce neighbours of
// the same base) and by size (best fit).  Each free range carries the events
// of the frees that produced it; carving from it waits for them first, so a
// block released on one stream is not reused on another before its last
// kernels finish.
#include "scratch_cache.h"

#include <algorithm>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace spm_amd {
namespace {

constexpr uint64_t kGranule = 256;

struct FreeRange {
  uint64_t size;
  char *base;
  std::vector<hipEvent_t> pending;
};

struct Used {
  uint64_t size;
  char *base;
};

struct CacheState {
  std::mutex mu;
  int depth = 0;
  std::map<char *, FreeRange> free_by_addr;
  std::multimap<uint64_t, char *> free_by_size;
  std::unordered_map<char *, Used> used;       // ranges handed out
  std::map<char *, uint64_t> base_size;        // live bases
  std::unordered_map<char *, uint64_t> base_used;  // handed-out ranges per base
  uint64_t mallocs = 0;
};

CacheState &Cache() {
  static CacheState c;
  return c;
}

void EraseSizeIndex(CacheState &c, uint64_t size, char *addr) {
  auto r = c.free_by_size.equal_range(size);
  for (auto it = r.first; it != r.second; ++it)
    if (it->second == addr) {
      c.free_by_size.erase(it);
      return;
    }
}

void WaitAll(std::vector<hipEvent_t> *ev) {
  for (hipEvent_t e : *ev) {
    (void)hipEventSynchronize(e);
    (void)hipEventDestroy(e);
  }
  ev->clear();
}

void InsertFree(CacheState &c, char *addr, FreeRange r) {
  // Coalesce with the next range of the same base.
  auto nx = c.free_by_addr.find(addr + r.size);
  if (nx != c.free_by_addr.end() && nx->second.base == r.base) {
    EraseSizeIndex(c, nx->second.size, nx->first);
    r.size += nx->second.size;
    r.pending.insert(r.pending.end(), nx->second.pending.begin(), nx->second.pending.end());
    c.free_by_addr.erase(nx);
  }
  // And with the previous one.
  auto pv = c.free_by_addr.lower_bound(addr);
  if (pv != c.free_by_addr.begin()) {
    --pv;
    if (pv->second.base == r.base && pv->first + pv->second.size == addr) {
      EraseSizeIndex(c, pv->second.size, pv->first);
      pv->second.size += r.size;
      pv->second.pending.insert(pv->second.pending.end(), r.pending.begin(), r.pending.end());
      c.free_by_size.emplace(pv->second.size, pv->first);
      return;
    }
  }
  c.free_by_size.emplace(r.size, addr);
  c.free_by_addr.emplace(addr, std::move(r));
}

// Frees a base whose ranges are all free (one coalesced range).
void ReleaseBase(CacheState &c, char *base) {
  auto it = c.free_by_addr.find(base);
  if (it != c.free_by_addr.end()) {
    EraseSizeIndex(c, it->second.size, base);
    for (hipEvent_t e : it->second.pending) (void)hipEventDestroy(e);
    c.free_by_addr.erase(it);
  }
  c.base_size.erase(base);
  c.base_used.erase(base);
  (void)DevFree(base);  // synchronizes the device
}

void ReleaseIdleBases(CacheState &c) {
  std::vector<char *> idle;
  for (auto &b : c.base_size)
    if (c.base_used[b.first] == 0) idle.push_back(b.first);
  for (char *b : idle) ReleaseBase(c, b);
}

struct DevAccount {
  std::mutex mu;
  std::unordered_map<void *, uint64_t> size;
  uint64_t live = 0, peak = 0;
};

DevAccount &Account() {
  static DevAccount a;
  return a;
}

}  // namespace

hipError_t DevMallocRaw(void **p, uint64_t bytes) {
  const hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return e;
  DevAccount &a = Account();
  std::lock_guard<std::mutex> lock(a.mu);
  a.size[*p] = bytes;
  a.live += bytes;
  a.peak = std::max(a.peak, a.live);
  return e;
}

hipError_t DevFree(void *p) {
  if (!p) return hipSuccess;
  {
    DevAccount &a = Account();
    std::lock_guard<std::mutex> lock(a.mu);
    auto it = a.size.find(p);
    if (it != a.size.end()) {
      a.live -= it->second;
      a.size.erase(it);
    }
  }
  return hipFree(p);
}

uint64_t DevLiveBytes() {
  DevAccount &a = Account();
  std::lock_guard<std::mutex> lock(a.mu);
  return a.live;
}

uint64_t DevPeakBytes() {
  DevAccount &a = Account();
  std::lock_guard<std::mutex> lock(a.mu);
  return a.peak;
}

void DevPeakReset() {
  DevAccount &a = Account();
  std::lock_guard<std::mutex> lock(a.mu);
  a.peak = a.live;
}

hipError_t ScratchAlloc(void **p, uint64_t bytes) {
  CacheState &c = Cache();
  std::lock_guard<std::mutex> lock(c.mu);
  if (c.depth == 0) return DevMallocRaw(p, bytes);
  const uint64_t need = (std::max<uint64_t>(bytes, 1) + kGranule - 1) / kGranule * kGranule;
  auto fit = c.free_by_size.lower_bound(need);
  if (fit != c.free_by_size.end()) {
    char *addr = fit->second;
    c.free_by_size.erase(fit);
    auto node = c.free_by_addr.extract(addr);
    FreeRange r = std::move(node.mapped());
    WaitAll(&r.pending);
    if (r.size > need) {
      c.free_by_addr.emplace(addr + need, FreeRange{r.size - need, r.base, {}});
      c.free_by_size.emplace(r.size - need, addr + need);
    }
    c.used[addr] = Used{need, r.base};
    ++c.base_used[r.base];
    *p = addr;
    return hipSuccess;
  }
  hipError_t e = DevMallocRaw(p, need);
  if (e == hipErrorOutOfMemory && !c.free_by_addr.empty()) {
    (void)hipGetLastError();
    ReleaseIdleBases(c);
    e = DevMallocRaw(p, need);
  }
  if (e != hipSuccess) return e;
  char *b = static_cast<char *>(*p);
  ++c.mallocs;
  c.base_size[b] = need;
  c.base_used[b] = 1;
  c.used[b] = Used{need, b};
  return hipSuccess;
}

void ScratchFree(void *p, hipStream_t st) {
  if (!p) return;
  CacheState &c = Cache();
  std::lock_guard<std::mutex> lock(c.mu);
  char *addr = static_cast<char *>(p);
  auto it = c.used.find(addr);
  if (it == c.used.end()) {
    (void)DevFree(p);  // allocated outside a scope
    return;
  }
  const Used u = it->second;
  c.used.erase(it);
  FreeRange r{u.size, u.base, {}};
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess && hipEventRecord(ev, st) == hipSuccess) {
    r.pending.push_back(ev);
  } else {
    (void)hipGetLastError();
    if (ev) (void)hipEventDestroy(ev);
    (void)hipStreamSynchronize(st);
  }
  InsertFree(c, addr, std::move(r));
  if (--c.base_used[u.base] == 0 && c.depth == 0) ReleaseBase(c, u.base);
}

void ScratchCacheBegin() {
  CacheState &c = Cache();
  std::lock_guard<std::mutex> lock(c.mu);
  ++c.depth;
}

void ScratchCacheEnd() {
  CacheState &c = Cache();
  std::lock_guard<std::mutex> lock(c.mu);
  if (c.depth > 0 && --c.depth == 0) ReleaseIdleBases(c);  // bases still in use go at their last free
}

ScratchCacheStats ScratchCacheGetStats() {
  CacheState &c = Cache();
  std::lock_guard<std::mutex> lock(c.mu);
  ScratchCacheStats s{c.base_size.size(), 0, c.free_by_addr.size(), 0, 0, c.mallocs};
  for (auto &b : c.base_size) s.base_bytes += b.second;
  for (auto &f : c.free_by_addr) s.free_bytes += f.second.size;
  for (auto &u : c.used) s.used_bytes += u.second.size;
  return s;
}

}  // namespace spm_amd
