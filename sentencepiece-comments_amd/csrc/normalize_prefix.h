// Device helpers of Normalizer::NormalizePrefix (normalizer.cc:231-300):
// UTF-8 validity, the precompiled charsmap's longest match (darts-clone
// units, normalizer.h:169) and the user-defined symbols' longest match.
// Shared by normalize_kernels.hip (one sentence per lane) and
// coop_encode.hip (one line per wave, small raw-line calls).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "normalize_device.h"

namespace spm_amd {
namespace {

__device__ __forceinline__ bool DTrail(uint8_t c) { return (c & 0xC0u) == 0x80u; }
__device__ __forceinline__ bool DValidCp(uint32_t c) { return c < 0xD800u || (c >= 0xE000u && c <= 0x10FFFFu); }

// IsValidDecodeUTF8 length (util.h:459-462): 0 = invalid.
__device__ uint32_t DValidCharLen(const uint8_t *in, uint64_t n) {
  const uint32_t c0 = in[0];
  if (c0 < 0x80u) return 1;
  if (n >= 2 && (c0 & 0xE0u) == 0xC0u) {
    const uint32_t cp = ((c0 & 0x1Fu) << 6) | (in[1] & 0x3Fu);
    if (DTrail(in[1]) && cp >= 0x80u && DValidCp(cp)) return 2;
  } else if (n >= 3 && (c0 & 0xF0u) == 0xE0u) {
    const uint32_t cp = ((c0 & 0x0Fu) << 12) | ((in[1] & 0x3Fu) << 6) | (in[2] & 0x3Fu);
    if (DTrail(in[1]) && DTrail(in[2]) && cp >= 0x800u && DValidCp(cp)) return 3;
  } else if (n >= 4 && (c0 & 0xF8u) == 0xF0u) {
    const uint32_t cp = ((c0 & 0x07u) << 18) | ((in[1] & 0x3Fu) << 12) | ((in[2] & 0x3Fu) << 6) |
                        (in[3] & 0x3Fu);
    if (DTrail(in[1]) && DTrail(in[2]) && DTrail(in[3]) && cp >= 0x10000u && DValidCp(cp)) return 4;
  }
  return 0;
}

// darts-clone unit accessors (darts.h:50-80)
__device__ __forceinline__ uint32_t DOff(uint32_t u) { return (u >> 10) << ((u & (1u << 9)) >> 6); }

// Longest charsmap key prefixing in[0:n) (first 32 matches, normalizer.h:169).
__device__ uint32_t CharsmapLongest(const NormTables &t, const uint8_t *in, uint64_t n,
                                    uint32_t *value) {
  if (!t.units) return 0;
  uint32_t best = 0, found = 0;
  uint32_t pos = DOff(t.units[0]);
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t c = in[i];
    pos ^= c;
    if (pos >= t.num_units) break;
    const uint32_t u = t.units[pos];
    if ((u & 0x800000FFu) != c) break;
    pos ^= DOff(u);
    if ((u >> 8) & 1u) {
      if (found++ >= 32) break;
      // Out-of-range value unit / pool offset (a corrupted blob): no match,
      // as the host Normalizer (normalizer.cc); no read leaves the blob.
      if (pos >= t.num_units) continue;
      const uint32_t v = t.units[pos] & 0x7FFFFFFFu;
      if (v >= t.pool_size) continue;
      best = static_cast<uint32_t>(i + 1);
      *value = v;
    }
  }
  return best;
}

// Longest key of a DoubleArray (double_array.h layout) prefixing in[0:n).
__device__ uint32_t TrieLongest(const uint32_t *units, uint32_t num_units, const uint8_t *in,
                                uint64_t n) {
  uint32_t node = 0, best = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t c = in[i];
    if (c == 0) break;
    const uint32_t next = (units[node] >> 9) ^ c;
    if (next >= num_units || (units[next] & 0xFFu) != c) break;
    node = next;
    if ((units[node] >> 8) & 1u) best = static_cast<uint32_t>(i + 1);
  }
  return best;
}

}  // namespace
}  // namespace spm_amd
