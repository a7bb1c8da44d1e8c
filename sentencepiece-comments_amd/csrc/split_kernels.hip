// SplitSentencesByWhitespace on gfx950 (trainer_interface.cc:465-477 over
// SplitIntoWords, model_interface.cc:155-190): the unique words of the
// normalized corpus with their summed sentence freqs.  The reference counts
// words in a std::unordered_map and then Sorted()s them (freq desc, string
// asc), so the result does not depend on the map's order; here:
//   count pass   — words per sentence (one sentence per lane);
//   emit pass    — per word occurrence: a 64-bit hash of its bytes (key), its
//                  start, length and the sentence freq;
//   radix sort   — occurrences grouped by hash;
//   heads        — a run of equal hashes is one word: every occurrence is
//                  compared byte for byte with its predecessor in the run, so
//                  a hash collision between different words is detected (the
//                  caller then runs the host split) instead of merging them;
//   reduce       — summed freq per run, the run's first occurrence as the
//                  word; the unique words (60 k for the c5 corpus) go to the
//                  host, which applies the reference's Sorted order.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <vector>

#include "device_common.h"
#include "normalize_device.h"
#include "scratch_cache.h"

namespace spm_amd {
namespace {

// U+2581 (kWSStr): the only whitespace SplitIntoWords knows.
__device__ __forceinline__ bool IsWs(const uint8_t *s, uint64_t b, uint32_t mblen) {
  return mblen == 3 && s[b] == 0xE2u && s[b + 1] == 0x96u && s[b + 2] == 0x81u;
}

__device__ __forceinline__ uint64_t WordHash(const uint8_t *s, uint64_t len) {
  uint64_t h = 0xcbf29ce484222325ull ^ (len * 0x9E3779B97F4A7C15ull);  // FNV-1a, length-seeded
  for (uint64_t k = 0; k < len; ++k) h = (h ^ s[k]) * 0x100000001b3ull;
  h ^= h >> 33;  // splitmix64 finalizer
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  return h ^ (h >> 33);
}

// The host split's loop (trainer.cc SplitSentencesByWhitespace), per lane.
// kEmit false: cnt[i] = words of sentence i; true: the word records at woff[i].
template <bool kEmit>
__global__ __launch_bounds__(256) void split_kernel(const uint8_t *__restrict__ text, const uint64_t *__restrict__ off,
                                                    const int64_t *__restrict__ freq, uint64_t n, bool suffix,
                                                    uint64_t *__restrict__ cnt, const uint64_t *__restrict__ woff,
                                                    uint64_t *__restrict__ key, uint32_t *__restrict__ idx,
                                                    uint64_t *__restrict__ wstart, uint32_t *__restrict__ wlen,
                                                    int64_t *__restrict__ wfreq) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = off[i];
  const uint8_t *__restrict__ s = text + o;
  const uint64_t len = off[i + 1] - o;
  uint64_t k = 0;
  auto word = [&](uint64_t a, uint64_t b) {
    if constexpr (kEmit) {
      const uint64_t j = woff[i] + k;
      key[j] = WordHash(s + a, b - a);
      idx[j] = static_cast<uint32_t>(j);
      wstart[j] = o + a;
      wlen[j] = static_cast<uint32_t>(b - a);
      wfreq[j] = freq[i];
    }
    ++k;
  };
  uint64_t b = 0, start = 0;
  bool open = false;
  while (b < len) {
    uint32_t mblen = OneCharLenDev(s[b]);
    if (mblen > len - b) mblen = static_cast<uint32_t>(len - b);
    const bool ws = IsWs(s, b, mblen);
    if (suffix) {
      if (!open) {
        open = true;
        start = b;
      }
      b += mblen;
      if (b < len && ws) {
        word(start, b);
        open = false;
      }
    } else {
      if (b == 0 || ws) {
        if (open) word(start, b);
        open = true;
        start = b;
      }
      b += mblen;
    }
  }
  if (open) word(start, len);
  if constexpr (!kEmit) cnt[i] = k;
}

// Sorted order: run heads, the freq of each occurrence, and a byte compare of
// every occurrence with its predecessor inside a run (*collide = 1 when two
// different words share a hash).
__global__ __launch_bounds__(256) void split_heads_kernel(const uint8_t *__restrict__ text,
                                                          const uint64_t *__restrict__ skey,
                                                          const uint32_t *__restrict__ sidx,
                                                          const uint64_t *__restrict__ wstart,
                                                          const uint32_t *__restrict__ wlen,
                                                          const int64_t *__restrict__ wfreq, uint64_t m,
                                                          uint8_t *__restrict__ head, int64_t *__restrict__ sfreq,
                                                          uint32_t *__restrict__ collide) {
  const uint64_t j = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool in = j < m;
  const uint32_t w = in ? sidx[j] : 0u;
  const uint32_t lw = in ? wlen[w] : 0u;
  const uint64_t sw = in ? wstart[w] : 0u;
  // The predecessor's (start, length): lane l - 1's own, by shuffle (the
  // first lane of a wave gathers them).
  const int lane = threadIdx.x & 63;
  uint32_t lp = __shfl_up(lw, 1);
  uint64_t sp = __shfl_up(sw, 1);
  if (!in) return;
  sfreq[j] = wfreq[w];
  const bool h = j == 0 || skey[j] != skey[j - 1];
  head[j] = h ? 1 : 0;
  if (!h) {
    if (lane == 0) {
      const uint32_t p = sidx[j - 1];
      lp = wlen[p];
      sp = wstart[p];
    }
    bool same = lw == lp;
    // Four bytes per step, the eight loads issued together.
    for (uint32_t k = 0; same && k < lw; k += 4) {
      uint32_t x[4], y[4];
#pragma unroll
      for (uint32_t t = 0; t < 4; ++t) {
        x[t] = k + t < lw ? text[sw + k + t] : 0u;
        y[t] = k + t < lw ? text[sp + k + t] : 0u;
      }
#pragma unroll
      for (uint32_t t = 0; t < 4; ++t) same = same && x[t] == y[t];
    }
    if (!same) atomicOr(collide, 1u);
  }
}

__global__ __launch_bounds__(256) void split_rep_len_kernel(const uint32_t *__restrict__ rep,
                                                            const uint32_t *__restrict__ wlen, uint64_t u,
                                                            uint64_t *__restrict__ len) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k < u) len[k] = wlen[rep[k]];
}

__global__ __launch_bounds__(256) void split_rep_copy_kernel(const uint8_t *__restrict__ text,
                                                             const uint32_t *__restrict__ rep,
                                                             const uint64_t *__restrict__ wstart,
                                                             const uint64_t *__restrict__ roff, uint64_t u,
                                                             uint8_t *__restrict__ out) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= u) return;
  const uint8_t *s = text + wstart[rep[k]];
  const uint64_t o = roff[k], l = roff[k + 1] - o;
  for (uint64_t q = 0; q < l; ++q) out[o + q] = s[q];
}

unsigned Blocks(uint64_t n) { return static_cast<unsigned>((n + 255) / 256); }

struct Scratch {
  std::vector<void *> ptrs;
  hipStream_t st = nullptr;  // the stream the blocks are used on
  ~Scratch() {
    for (void *p : ptrs) ScratchFree(p, st);  // scratch_cache.h
  }
  template <class T>
  hipError_t Get(T **p, uint64_t count) {
    void *q = nullptr;
    hipError_t e = ScratchAlloc(&q, std::max<uint64_t>(count, 1) * sizeof(T));
    if (e != hipSuccess) return e;
    ptrs.push_back(q);
    *p = static_cast<T *>(q);
    return hipSuccess;
  }
};

#define SPLIT_TRY(x)                   \
  do {                                 \
    hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return e_;   \
  } while (0)

}  // namespace

hipError_t CorpusSplitWords(const uint8_t *d_text, const uint64_t *d_off, const int64_t *d_freq, uint64_t n,
                            bool suffix, SplitWords *out, hipStream_t st) {
  *out = SplitWords();
  if (n == 0) {
    out->off.assign(1, 0);
    return hipSuccess;
  }
  Scratch S;
  S.st = st;
  uint64_t *cnt, *woff;
  SPLIT_TRY(S.Get(&cnt, n));
  SPLIT_TRY(S.Get(&woff, n + 1));
  split_kernel<false><<<Blocks(n), 256, 0, st>>>(d_text, d_off, d_freq, n, suffix, cnt, nullptr, nullptr, nullptr,
                                                  nullptr, nullptr, nullptr);
  SPLIT_TRY(hipGetLastError());
  size_t tb = 0;
  SPLIT_TRY(LengthsToOffsets(cnt, n, woff, nullptr, &tb, st));
  void *tmp = nullptr;
  SPLIT_TRY(S.Get(reinterpret_cast<uint8_t **>(&tmp), tb));
  SPLIT_TRY(LengthsToOffsets(cnt, n, woff, tmp, &tb, st));
  uint64_t m = 0;
  SPLIT_TRY(hipMemcpyAsync(&m, woff + n, 8, hipMemcpyDeviceToHost, st));
  SPLIT_TRY(hipStreamSynchronize(st));
  out->occurrences = m;
  // hipCUB's item counts are int: a larger corpus takes the host split.
  if (m >= 0x7FFFFFFFull) {
    out->fallback = true;
    return hipSuccess;
  }
  if (m == 0) {
    out->off.assign(1, 0);
    return hipSuccess;
  }
  uint64_t *key, *skey, *wstart;
  uint32_t *idx, *sidx, *wlen, *collide;
  int64_t *wfreq, *sfreq;
  SPLIT_TRY(S.Get(&key, m));
  SPLIT_TRY(S.Get(&skey, m));
  SPLIT_TRY(S.Get(&idx, m));
  SPLIT_TRY(S.Get(&sidx, m));
  SPLIT_TRY(S.Get(&wstart, m));
  SPLIT_TRY(S.Get(&wlen, m));
  SPLIT_TRY(S.Get(&wfreq, m));
  SPLIT_TRY(S.Get(&sfreq, m));
  SPLIT_TRY(S.Get(&collide, 2));
  split_kernel<true><<<Blocks(n), 256, 0, st>>>(d_text, d_off, d_freq, n, suffix, nullptr, woff, key, idx, wstart,
                                                 wlen, wfreq);
  SPLIT_TRY(hipGetLastError());
  const int mi = static_cast<int>(m);
  tb = 0;
  SPLIT_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, skey, idx, sidx, mi, 0, 64, st));
  uint8_t *t2;
  SPLIT_TRY(S.Get(&t2, tb));
  SPLIT_TRY(hipcub::DeviceRadixSort::SortPairs(t2, tb, key, skey, idx, sidx, mi, 0, 64, st));
  // key / idx / wfreq storage is free now: head flags and the run outputs.
  uint8_t *head = reinterpret_cast<uint8_t *>(key);
  uint32_t *rep = idx;
  SPLIT_TRY(hipMemsetAsync(collide, 0, 8, st));
  split_heads_kernel<<<Blocks(m), 256, 0, st>>>(d_text, skey, sidx, wstart, wlen, wfreq, m, head, sfreq, collide);
  SPLIT_TRY(hipGetLastError());
  // Runs: summed freqs (aggregates in wfreq's storage — every wfreq read is
  // done by the heads kernel above) and the run heads' word ids.
  int64_t *agg = wfreq;
  uint64_t *ukeys;
  SPLIT_TRY(S.Get(&ukeys, m));
  int *d_runs = reinterpret_cast<int *>(collide + 1);
  tb = 0;
  SPLIT_TRY(hipcub::DeviceReduce::ReduceByKey(nullptr, tb, skey, ukeys, sfreq, agg, d_runs, hipcub::Sum(), mi, st));
  uint8_t *t3;
  SPLIT_TRY(S.Get(&t3, tb));
  SPLIT_TRY(hipcub::DeviceReduce::ReduceByKey(t3, tb, skey, ukeys, sfreq, agg, d_runs, hipcub::Sum(), mi, st));
  int *d_sel;
  SPLIT_TRY(S.Get(&d_sel, 1));
  tb = 0;
  SPLIT_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, sidx, head, rep, d_sel, mi, st));
  uint8_t *t4;
  SPLIT_TRY(S.Get(&t4, tb));
  SPLIT_TRY(hipcub::DeviceSelect::Flagged(t4, tb, sidx, head, rep, d_sel, mi, st));
  uint32_t hc[2] = {0, 0};
  int hsel = 0;
  SPLIT_TRY(hipMemcpyAsync(hc, collide, 8, hipMemcpyDeviceToHost, st));
  SPLIT_TRY(hipMemcpyAsync(&hsel, d_sel, 4, hipMemcpyDeviceToHost, st));
  SPLIT_TRY(hipStreamSynchronize(st));
  const uint64_t u = static_cast<uint64_t>(static_cast<int>(hc[1]));
  // SPM_HIP_SPLIT_FORCE_FALLBACK (debug): take the collision exit after all
  // of the device work, so tests cover the host split that follows it.
  static const bool force_fallback = std::getenv("SPM_HIP_SPLIT_FORCE_FALLBACK") != nullptr;
  if (hc[0] != 0 || static_cast<uint64_t>(hsel) != u || force_fallback) {
    out->fallback = true;  // a 64-bit hash collision between different words
    return hipSuccess;
  }
  uint64_t *rlen, *roff;
  SPLIT_TRY(S.Get(&rlen, u));
  SPLIT_TRY(S.Get(&roff, u + 1));
  split_rep_len_kernel<<<Blocks(u), 256, 0, st>>>(rep, wlen, u, rlen);
  SPLIT_TRY(hipGetLastError());
  tb = 0;
  SPLIT_TRY(LengthsToOffsets(rlen, u, roff, nullptr, &tb, st));
  uint8_t *t5;
  SPLIT_TRY(S.Get(&t5, tb));
  SPLIT_TRY(LengthsToOffsets(rlen, u, roff, t5, &tb, st));
  out->off.resize(u + 1);
  out->freq.resize(u);
  SPLIT_TRY(hipMemcpyAsync(out->off.data(), roff, (u + 1) * 8, hipMemcpyDeviceToHost, st));
  SPLIT_TRY(hipMemcpyAsync(out->freq.data(), agg, u * 8, hipMemcpyDeviceToHost, st));
  SPLIT_TRY(hipStreamSynchronize(st));
  uint8_t *wbytes;
  SPLIT_TRY(S.Get(&wbytes, out->off[u]));
  split_rep_copy_kernel<<<Blocks(u), 256, 0, st>>>(d_text, rep, wstart, roff, u, wbytes);
  SPLIT_TRY(hipGetLastError());
  out->bytes.resize(out->off[u]);
  if (out->off[u]) SPLIT_TRY(hipMemcpyAsync(out->bytes.data(), wbytes, out->off[u], hipMemcpyDeviceToHost, st));
  SPLIT_TRY(hipStreamSynchronize(st));
  return hipSuccess;
}

}  // namespace spm_amd
