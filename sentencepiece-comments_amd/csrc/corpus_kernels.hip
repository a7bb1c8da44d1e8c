// Trainer corpus passes on gfx950 (LoadSentences, trainer_interface.cc:
// 401-455): char histogram, rare-char replacement, CSR gather.  One sentence
// per lane; the histogram keeps code points < kLdsChars (plus U+2581) in an
// LDS table of 64-bit counters flushed once per block, the rest go to global
// 64-bit atomics.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "normalize_device.h"

namespace spm_amd {
namespace {

constexpr int kLdsChars = 8191;  // slot kLdsChars holds U+2581

__device__ __forceinline__ uint32_t Decode(const uint8_t *b, uint64_t len, uint32_t *mblen) {
  const uint32_t c0 = b[0];
  auto trail = [](uint32_t x) { return (x & 0xC0u) == 0x80u; };
  auto valid = [](uint32_t c) { return c < 0xD800u || (c >= 0xE000u && c <= 0x10FFFFu); };
  if (c0 < 0x80u) {
    *mblen = 1;
    return c0;
  } else if (len >= 2 && (c0 & 0xE0u) == 0xC0u) {
    const uint32_t cp = ((c0 & 0x1Fu) << 6) | (b[1] & 0x3Fu);
    if (trail(b[1]) && cp >= 0x80u && valid(cp)) {
      *mblen = 2;
      return cp;
    }
  } else if (len >= 3 && (c0 & 0xF0u) == 0xE0u) {
    const uint32_t cp = ((c0 & 0x0Fu) << 12) | ((b[1] & 0x3Fu) << 6) | (b[2] & 0x3Fu);
    if (trail(b[1]) && trail(b[2]) && cp >= 0x800u && valid(cp)) {
      *mblen = 3;
      return cp;
    }
  } else if (len >= 4 && (c0 & 0xF8u) == 0xF0u) {
    const uint32_t cp = ((c0 & 0x07u) << 18) | ((b[1] & 0x3Fu) << 12) | ((b[2] & 0x3Fu) << 6) |
                        (b[3] & 0x3Fu);
    if (trail(b[1]) && trail(b[2]) && trail(b[3]) && cp >= 0x10000u && valid(cp)) {
      *mblen = 4;
      return cp;
    }
  }
  *mblen = 1;
  return 0xFFFDu;
}

__global__ __launch_bounds__(256) void hist_kernel(const uint8_t *bytes, const uint64_t *off,
                                                   const int64_t *freq, uint64_t n,
                                                   unsigned long long *counts, uint32_t *flags) {
  __shared__ unsigned long long tab[kLdsChars + 1];
  for (int k = threadIdx.x; k <= kLdsChars; k += 256) tab[k] = 0;
  __syncthreads();
  uint32_t fl = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    const uint8_t *s = bytes + off[i];
    const uint64_t len = off[i + 1] - off[i];
    const unsigned long long f = static_cast<unsigned long long>(freq[i]);
    if (len == 0) fl |= 4u;
    uint64_t p = 0;
    while (p < len) {
      uint32_t m;
      const uint32_t c = Decode(s + p, len - p, &m);
      p += m;
      if (c == 0) {
        fl |= 2u;
        continue;
      }
      if (c == 0x20u) {
        fl |= 1u;
        continue;
      }
      if (c < kLdsChars) atomicAdd(&tab[c], f);
      else if (c == 0x2581u) atomicAdd(&tab[kLdsChars], f);
      else atomicAdd(&counts[c], f);
    }
  }
  if (fl) atomicOr(flags, fl);
  __syncthreads();
  for (int k = threadIdx.x; k <= kLdsChars; k += 256) {
    const unsigned long long v = tab[k];
    if (v) atomicAdd(&counts[k == kLdsChars ? 0x2581u : static_cast<uint32_t>(k)], v);
  }
}

template <bool WRITE>
__global__ void replace_kernel(const uint8_t *bytes, const uint64_t *off, uint64_t n,
                               const uint32_t *req, uint64_t *len_out, uint8_t *out,
                               const uint64_t *out_off) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *s = bytes + off[i];
  const uint64_t len = off[i + 1] - off[i];
  uint8_t *o = WRITE ? out + out_off[i] : nullptr;
  uint64_t p = 0, w = 0;
  while (p < len) {
    uint32_t m;
    uint32_t c = Decode(s + p, len - p, &m);
    p += m;
    if (!((req[c >> 5] >> (c & 31)) & 1u)) c = 0x2585u;
    // EncodeUTF8 (util.cc:250-286); c is a valid code point here.
    if (c <= 0x7Fu) {
      if (WRITE) o[w] = static_cast<uint8_t>(c);
      w += 1;
    } else if (c <= 0x7FFu) {
      if (WRITE) {
        o[w] = static_cast<uint8_t>(0xC0u | (c >> 6));
        o[w + 1] = static_cast<uint8_t>(0x80u | (c & 0x3Fu));
      }
      w += 2;
    } else if (c <= 0xFFFFu) {
      if (WRITE) {
        o[w] = static_cast<uint8_t>(0xE0u | (c >> 12));
        o[w + 1] = static_cast<uint8_t>(0x80u | ((c >> 6) & 0x3Fu));
        o[w + 2] = static_cast<uint8_t>(0x80u | (c & 0x3Fu));
      }
      w += 3;
    } else {
      if (WRITE) {
        o[w] = static_cast<uint8_t>(0xF0u | (c >> 18));
        o[w + 1] = static_cast<uint8_t>(0x80u | ((c >> 12) & 0x3Fu));
        o[w + 2] = static_cast<uint8_t>(0x80u | ((c >> 6) & 0x3Fu));
        o[w + 3] = static_cast<uint8_t>(0x80u | (c & 0x3Fu));
      }
      w += 4;
    }
  }
  if (!WRITE) len_out[i] = w;
}

__global__ void gather_len_kernel(const uint64_t *off, const uint64_t *idx, uint64_t m, uint64_t *len) {
  const uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= m) return;
  const uint64_t i = idx[k];
  len[k] = off[i + 1] - off[i];
}

// One wave per sentence copies its bytes (coalesced).
__global__ void gather_write_kernel(const uint8_t *bytes, const uint64_t *off, const int64_t *freq,
                                    const uint64_t *idx, uint64_t m, uint8_t *out,
                                    const uint64_t *out_off, int64_t *out_freq) {
  const uint64_t k = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= m) return;
  const uint64_t i = idx[k];
  const uint64_t b = off[i], len = off[i + 1] - b, o = out_off[k];
  for (uint64_t x = lane; x < len; x += 64) out[o + x] = bytes[b + x];
  if (lane == 0) out_freq[k] = freq[i];
}

inline unsigned Blocks(uint64_t n, unsigned t = 256) { return static_cast<unsigned>((n + t - 1) / t); }

}  // namespace

hipError_t CorpusCharHistogram(const uint8_t *d_bytes, const uint64_t *d_off, const int64_t *d_freq,
                               uint64_t n, unsigned long long *d_counts, uint32_t *d_flags,
                               hipStream_t st) {
  if (n == 0) return hipSuccess;
  const unsigned blocks = Blocks(n) < 4096u ? Blocks(n) : 4096u;  // grid-stride: one LDS flush per block
  hist_kernel<<<blocks, 256, 0, st>>>(d_bytes, d_off, d_freq, n, d_counts, d_flags);
  return hipGetLastError();
}

hipError_t CorpusReplaceLengths(const uint8_t *d_bytes, const uint64_t *d_off, uint64_t n,
                                const uint32_t *d_req, uint64_t *d_len, hipStream_t st) {
  if (n == 0) return hipSuccess;
  replace_kernel<false><<<Blocks(n), 256, 0, st>>>(d_bytes, d_off, n, d_req, d_len, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t CorpusReplaceWrite(const uint8_t *d_bytes, const uint64_t *d_off, uint64_t n,
                              const uint32_t *d_req, uint8_t *d_out, const uint64_t *d_out_off,
                              hipStream_t st) {
  if (n == 0) return hipSuccess;
  replace_kernel<true><<<Blocks(n), 256, 0, st>>>(d_bytes, d_off, n, d_req, nullptr, d_out, d_out_off);
  return hipGetLastError();
}

hipError_t CorpusGatherLengths(const uint64_t *d_off, const uint64_t *d_idx, uint64_t m,
                               uint64_t *d_len, hipStream_t st) {
  if (m == 0) return hipSuccess;
  gather_len_kernel<<<Blocks(m), 256, 0, st>>>(d_off, d_idx, m, d_len);
  return hipGetLastError();
}

hipError_t CorpusGatherWrite(const uint8_t *d_bytes, const uint64_t *d_off, const int64_t *d_freq,
                             const uint64_t *d_idx, uint64_t m, uint8_t *d_out,
                             const uint64_t *d_out_off, int64_t *d_out_freq, hipStream_t st) {
  if (m == 0) return hipSuccess;
  gather_write_kernel<<<Blocks(m, 4), 256, 0, st>>>(d_bytes, d_off, d_freq, d_idx, m, d_out, d_out_off,
                                                    d_out_freq);
  return hipGetLastError();
}

}  // namespace spm_amd
