// Trainer corpus passes on gfx950 (LoadSentences, trainer_interface.cc:
// 401-455): char histogram, rare-char replacement, CSR gather.  One sentence
// per lane; the histogram keeps code points < kLdsChars (plus U+2581) in an
// LDS table of 64-bit counters flushed once per block, the rest go to global
// 64-bit atomics.
#include <hip/hip_runtime.h>

#include "scratch_cache.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <vector>

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

// One wave per sentence copies its bytes (coalesced); waves stride over the
// sentences (the launch's total work-items must stay below 2^32).
__global__ void gather_write_kernel(const uint8_t *bytes, const uint64_t *off, const int64_t *freq,
                                    const uint64_t *idx, uint64_t m, uint8_t *out,
                                    const uint64_t *out_off, int64_t *out_freq) {
  const int lane = threadIdx.x & 63;
  for (uint64_t k = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); k < m; k += uint64_t(gridDim.x) * 4) {
    const uint64_t i = idx[k];
    const uint64_t b = off[i], len = off[i + 1] - b, o = out_off[k];
    for (uint64_t x = lane; x < len; x += 64) out[o + x] = bytes[b + x];
    if (lane == 0) out_freq[k] = freq[i];
  }
}

inline unsigned Blocks(uint64_t n, unsigned t = 256) { return static_cast<unsigned>((n + t - 1) / t); }
// Wave-per-item kernels: at most this many 256-thread blocks (a launch's
// blocks x threads must stay below 2^32 work-items), striding over the items.
constexpr unsigned kWaveGrid = 1u << 20;

// ---- Text-file lines (CorpusParseLines) -------------------------------------
// A tile of kLineTile file bytes per block, 64 consecutive bytes per thread.
constexpr uint32_t kLineTile = 256 * 64;

// Newlines per tile.
__global__ __launch_bounds__(256) void nl_count_kernel(const uint8_t *__restrict__ f, uint64_t size,
                                                       uint32_t *__restrict__ tile_cnt) {
  __shared__ uint32_t red[4];
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kLineTile + threadIdx.x * 64ull;
  uint32_t c = 0;
  if (b + 64 <= size) {
    const uint4 *q = reinterpret_cast<const uint4 *>(f + b);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 v = q[k];
      for (uint32_t w : {v.x, v.y, v.z, v.w}) {
        const uint32_t y = w ^ 0x0A0A0A0Au;  // zero bytes where w has '\n'
        // High bit of each byte: set iff the byte is non-zero (exact; the
        // borrow trick would also flag a 0x01 byte after a zero byte).
        const uint32_t nz = (((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
        c += 4u - static_cast<uint32_t>(__popc(nz));
      }
    }
  } else {
    for (uint64_t x = b; x < size && x < b + 64; ++x) c += f[x] == '\n';
  }
  for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Newline positions in file order: pos[tile_base[t] + rank] = byte index.
__global__ __launch_bounds__(256) void nl_write_kernel(const uint8_t *__restrict__ f, uint64_t size,
                                                       const uint64_t *__restrict__ tile_base,
                                                       uint64_t *__restrict__ pos) {
  __shared__ uint32_t scan[256];
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * kLineTile + threadIdx.x * 64ull;
  const uint64_t e = b + 64 < size ? b + 64 : size;
  uint32_t c = 0;
  for (uint64_t x = b; x < e; ++x) c += f[x] == '\n';
  scan[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t v = threadIdx.x >= static_cast<unsigned>(o) ? scan[threadIdx.x - o] : 0u;
    __syncthreads();
    scan[threadIdx.x] += v;
    __syncthreads();
  }
  uint64_t w = tile_base[blockIdx.x] + scan[threadIdx.x] - c;
  for (uint64_t x = b; x < e; ++x)
    if (f[x] == '\n') pos[w++] = x;
}

// Line i = [start, end): start = 0 or pos[i-1] + 1, end = pos[i] or size (the
// last line when the file does not end with a newline).  keep: 0 < len <=
// max_len and no kUNKStr (U+2585, E2 96 85) in the line
// (trainer_interface.cc:287-316); kept lines' lengths in klen (0 otherwise),
// their flags in kflag; too-long lines counted.
__global__ __launch_bounds__(256) void line_verdict_kernel(const uint8_t *__restrict__ f, uint64_t size,
                                                           const uint64_t *__restrict__ pos, uint64_t nl,
                                                           uint64_t lines, int64_t max_len,
                                                           uint64_t *__restrict__ klen, uint32_t *__restrict__ kflag,
                                                           unsigned long long *__restrict__ too_long) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  uint32_t tl = 0;
  if (i < lines) {
    const uint64_t start = i == 0 ? 0 : pos[i - 1] + 1;
    const uint64_t end = i < nl ? pos[i] : size;
    const uint64_t len = end - start;
    bool keep = len > 0;
    if (keep && static_cast<int64_t>(len) > max_len) {
      keep = false;
      tl = 1;
    }
    if (keep) {
      for (uint64_t x = start; x + 2 < end; ++x)
        if (f[x] == 0xE2u && f[x + 1] == 0x96u && f[x + 2] == 0x85u) {
          keep = false;
          break;
        }
    }
    klen[i] = keep ? len : 0;
    kflag[i] = keep ? 1u : 0u;
  }
  const uint64_t m = __ballot(tl != 0);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(too_long, static_cast<unsigned long long>(__popcll(m)));
}

// One wave per line: kept line i goes to slot kidx[i] at byte offset koff[i].
__global__ __launch_bounds__(256) void line_copy_kernel(const uint8_t *__restrict__ f, uint64_t size,
                                                        const uint64_t *__restrict__ pos, uint64_t nl,
                                                        uint64_t lines, const uint32_t *__restrict__ kflag,
                                                        const uint64_t *__restrict__ kidx,
                                                        const uint64_t *__restrict__ koff,
                                                        uint8_t *__restrict__ out, uint64_t *__restrict__ out_off) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); i < lines;
       i += static_cast<uint64_t>(gridDim.x) * 4) {
    if (!kflag[i]) continue;
    const uint64_t start = i == 0 ? 0 : pos[i - 1] + 1;
    const uint64_t end = i < nl ? pos[i] : size;
    const uint64_t o = koff[i];
    for (uint64_t x = lane; x < end - start; x += 64) out[o + x] = f[start + x];
    if (lane == 0) out_off[kidx[i] + 1] = o + (end - start);
  }
}

__global__ void fill_i64_kernel(int64_t *p, uint64_t n, int64_t v) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) p[i] = v;
}

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
  gather_write_kernel<<<std::min(Blocks(m, 4), kWaveGrid), 256, 0, st>>>(d_bytes, d_off, d_freq, d_idx, m, d_out, d_out_off,
                                                    d_out_freq);
  return hipGetLastError();
}

namespace {
struct DevBlocks {
  std::vector<void *> p;
  ~DevBlocks() {
    for (void *x : p) (void)DevFree(x);
  }
  template <class T>
  hipError_t Get(T **out, uint64_t count) {
    void *v = nullptr;
    hipError_t e = DevMalloc(&v, (count ? count : 1) * sizeof(T));
    if (e == hipSuccess) {
      p.push_back(v);
      *out = static_cast<T *>(v);
    }
    return e;
  }
};
#define PARSE_TRY(x)                  \
  do {                                \
    hipError_t e_ = (x);              \
    if (e_ != hipSuccess) return e_;  \
  } while (0)
}  // namespace

hipError_t CorpusParseLines(const uint8_t *d_file, uint64_t size, int64_t max_len, ParsedLines *out,
                            hipStream_t st) {
  *out = ParsedLines();
  DevBlocks S;
  const uint64_t tiles = (size + kLineTile - 1) / kLineTile;
  // hipCUB item counts are int and the tile scan runs over tiles + 1 items.
  if (tiles == 0 || tiles + 1 > static_cast<uint64_t>(INT32_MAX)) return hipErrorInvalidValue;
  uint32_t *tile_cnt;
  uint64_t *tile_base;
  PARSE_TRY(S.Get(&tile_cnt, tiles));
  PARSE_TRY(S.Get(&tile_base, tiles + 1));
  nl_count_kernel<<<static_cast<unsigned>(tiles), 256, 0, st>>>(d_file, size, tile_cnt);
  PARSE_TRY(hipGetLastError());
  size_t tb = 0;
  const int ti = static_cast<int>(tiles);
  PARSE_TRY(hipcub::DeviceScan::ExclusiveScan(nullptr, tb, tile_cnt, tile_base, hipcub::Sum(), uint64_t(0), ti + 1, st));
  void *tmp;
  uint8_t *tmpb;
  PARSE_TRY(S.Get(&tmpb, tb));
  tmp = tmpb;
  // (tile_cnt[tiles] is read by the scan of tiles + 1 items: one extra zero.)
  uint32_t *tile_cnt1;
  PARSE_TRY(S.Get(&tile_cnt1, tiles + 1));
  PARSE_TRY(hipMemcpyAsync(tile_cnt1, tile_cnt, tiles * 4, hipMemcpyDeviceToDevice, st));
  PARSE_TRY(hipMemsetAsync(tile_cnt1 + tiles, 0, 4, st));
  PARSE_TRY(hipcub::DeviceScan::ExclusiveScan(tmp, tb, tile_cnt1, tile_base, hipcub::Sum(), uint64_t(0), ti + 1, st));
  uint64_t nl = 0;
  uint8_t last = 0;
  PARSE_TRY(hipMemcpyAsync(&nl, tile_base + tiles, 8, hipMemcpyDeviceToHost, st));
  PARSE_TRY(hipMemcpyAsync(&last, d_file + size - 1, 1, hipMemcpyDeviceToHost, st));
  PARSE_TRY(hipStreamSynchronize(st));
  const uint64_t lines = nl + (last != '\n' ? 1 : 0);  // std::getline: no empty line after a final newline
  // hipCUB item counts are int and the line scans run over lines + 1 items.
  if (lines + 1 > static_cast<uint64_t>(INT32_MAX)) return hipErrorInvalidValue;
  uint64_t *pos, *klen, *kidx, *koff;
  uint32_t *kflag;
  unsigned long long *d_tl;
  PARSE_TRY(S.Get(&pos, nl));
  PARSE_TRY(S.Get(&klen, lines + 1));
  PARSE_TRY(S.Get(&kflag, lines + 1));
  PARSE_TRY(S.Get(&kidx, lines + 1));
  PARSE_TRY(S.Get(&koff, lines + 1));
  PARSE_TRY(S.Get(&d_tl, 1));
  nl_write_kernel<<<static_cast<unsigned>(tiles), 256, 0, st>>>(d_file, size, tile_base, pos);
  PARSE_TRY(hipGetLastError());
  PARSE_TRY(hipMemsetAsync(d_tl, 0, 8, st));
  PARSE_TRY(hipMemsetAsync(klen + lines, 0, 8, st));
  PARSE_TRY(hipMemsetAsync(kflag + lines, 0, 4, st));
  line_verdict_kernel<<<Blocks(lines), 256, 0, st>>>(d_file, size, pos, nl, lines, max_len, klen, kflag, d_tl);
  PARSE_TRY(hipGetLastError());
  const int li = static_cast<int>(lines);
  size_t tb2 = 0, tb3 = 0;
  PARSE_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, klen, koff, li + 1, st));
  PARSE_TRY(hipcub::DeviceScan::ExclusiveScan(nullptr, tb3, kflag, kidx, hipcub::Sum(), uint64_t(0), li + 1, st));
  uint8_t *tmp2;
  PARSE_TRY(S.Get(&tmp2, tb2 > tb3 ? tb2 : tb3));
  PARSE_TRY(hipcub::DeviceScan::ExclusiveSum(tmp2, tb2, klen, koff, li + 1, st));
  PARSE_TRY(hipcub::DeviceScan::ExclusiveScan(tmp2, tb3, kflag, kidx, hipcub::Sum(), uint64_t(0), li + 1, st));
  uint64_t kept = 0, bytes = 0;
  unsigned long long tl = 0;
  PARSE_TRY(hipMemcpyAsync(&kept, kidx + lines, 8, hipMemcpyDeviceToHost, st));
  PARSE_TRY(hipMemcpyAsync(&bytes, koff + lines, 8, hipMemcpyDeviceToHost, st));
  PARSE_TRY(hipMemcpyAsync(&tl, d_tl, 8, hipMemcpyDeviceToHost, st));
  PARSE_TRY(hipStreamSynchronize(st));
  out->lines = lines;
  out->too_long = tl;
  out->n = kept;
  out->total = bytes;
  DevBlocks O;
  PARSE_TRY(O.Get(&out->bytes, bytes));
  PARSE_TRY(O.Get(&out->off, kept + 1));
  PARSE_TRY(O.Get(&out->freq, kept));
  PARSE_TRY(hipMemsetAsync(out->off, 0, 8, st));
  line_copy_kernel<<<std::min(Blocks(lines, 4), kWaveGrid), 256, 0, st>>>(d_file, size, pos, nl, lines, kflag, kidx, koff, out->bytes,
                                                     out->off);
  PARSE_TRY(hipGetLastError());
  if (kept) fill_i64_kernel<<<Blocks(kept), 256, 0, st>>>(out->freq, kept, 1);
  PARSE_TRY(hipGetLastError());
  PARSE_TRY(hipStreamSynchronize(st));
  O.p.clear();  // the caller owns the outputs now
  return hipSuccess;
}

}  // namespace spm_amd
