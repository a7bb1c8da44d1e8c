// Single-pass prefix sums across workgroups (decoupled look-back).  Device
// code only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace spm_amd {

// Descriptor of one tile: 2 flag bits + a 62-bit value.
constexpr uint64_t kLbAggregate = 1ull << 62;
constexpr uint64_t kLbPrefix = 2ull << 62;
constexpr uint64_t kLbValue = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t WaveSum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor(static_cast<uint32_t>(v), o);
    const uint32_t hi = __shfl_xor(static_cast<uint32_t>(v >> 32), o);
    v += (static_cast<uint64_t>(hi) << 32) | lo;
  }
  return v;
}

// Coherent (L2) read of a descriptor: a relaxed agent-scope atomic load,
// which bypasses the non-coherent L1.
__device__ __forceinline__ uint64_t LoadDesc(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by all 64 lanes of ONE wavefront of the workgroup holding tile
// `t` (tiles are handed out in launch order by a ticket counter, so every
// predecessor is resident or finished and publishes its aggregate without
// waiting on anyone: the spin below always ends).  Publishes the tile's
// aggregate, sums predecessors back to the nearest published prefix,
// publishes the inclusive prefix and returns the exclusive one (uniform).
// While a predecessor is unpublished only lane 0 polls it, with plain
// coherent loads and a sleep between polls: a spinning tile must not load
// L2 (the running tiles' trie walks live there).
__device__ inline uint64_t LookbackExclusive(uint64_t *desc, uint64_t t, uint64_t total, int lane) {
  if (t == 0) {
    if (lane == 0) __hip_atomic_store(desc, kLbPrefix | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0) __hip_atomic_store(desc + t, kLbAggregate | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t excl = 0;
  int64_t j = static_cast<int64_t>(t) - 1;
  for (;;) {
    if (lane == 0)
      while ((LoadDesc(desc + j) >> 62) == 0) __builtin_amdgcn_s_sleep(8);
    const int64_t q = j - lane;
    const uint64_t v = q >= 0 ? LoadDesc(desc + q) : kLbPrefix;
    const uint64_t pm = __builtin_amdgcn_ballot_w64((v >> 62) == 2);
    const uint64_t zm = __builtin_amdgcn_ballot_w64((v >> 62) == 0);
    const int fp = pm ? __builtin_ctzll(pm) : 64;  // nearest predecessor with a prefix
    const uint64_t upto = fp >= 63 ? ~0ull : (2ull << fp) - 1;
    if (zm & upto) {  // a predecessor nearer than that prefix has not published
      __builtin_amdgcn_s_sleep(8);
      continue;
    }
    excl += WaveSum64(lane <= fp ? (v & kLbValue) : 0);
    if (fp < 64) break;
    j -= 64;
  }
  if (lane == 0)
    __hip_atomic_store(desc + t, kLbPrefix | (excl + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

}  // namespace spm_amd
