// Seed-piece mining for the unigram trainer on gfx950 (MI355X).
//
// Reference: unigram::Trainer::MakeSeedSentencePieces
// (unigram_model_trainer.cc:124-225) over esaxx (esa.hxx:37-122): all
// sentences concatenated as char32 with a 0 after each, suffix array, PLCP,
// internal nodes (L, R, D) enumerated by a stack in suffixtree(); each node
// with D > 1, no boundary inside and IsValidSentencePiece
// (trainer_interface.cc:178-267) scores (R-L)*D; seeds = every char by
// frequency, then substrings Sorted by (score desc, node index asc).
//
// Device restatement (no stack, no global suffix order past a boundary):
//  * A node whose D-prefix has no boundary is the interval of one 0-free
//    string w; its members, its R and its D depend only on how suffixes
//    compare up to and including their first 0.  So suffixes are sorted by
//    their TRUNCATED strings (ties in any order) and the LCP array is capped
//    at "common prefix including the shared 0" — the set of 0-free nodes and
//    their (L, R, D) are exactly the reference's.
//  * suffixtree() emits a node when the scan reaches its right end R, deepest
//    first, so "node index ascending" == (R ascending, D descending): that is
//    the tie order used here.
//  * Only D <= max_sentencepiece_length can pass IsValidSentencePiece, so the
//    LCP is clamped at max_len + 1 and stored as uint8 (uint16 when max_len
//    > 254, up to the TrainerSpec limit 512); a node of depth d is
//    found at its leftmost boundary j (H[j] == d, the nearest H <= d on the
//    left is < d); L and R come from nearest-smaller-value searches over a
//    64-ary min pyramid of H.
// Pipeline (one call, one stream): decode → suffix order by LSD radix passes
// over packed-symbol chunk keys (prefix doubling for long pieces / large
// alphabets; corpora of >= 2^28 chars split first into 4 parts by first
// symbol, each part sorted alone into its segment of SA) → capped LCP →
// pyramid → candidate nodes → two stable radix sorts → top K gathered.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/spm_hip.h"
#include "device_model.h"
#include "scratch_cache.h"
#include "trace.h"
#include "unicode_script_table.h"

struct spm_hip_seeds {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> offsets{0};
  std::vector<float> scores;
  std::vector<int64_t> raw;  // freq-weighted char counts / (R-L)*D before ToLogProb
  uint64_t num_chars = 0;    // seeds [0, num_chars) are single chars
  uint64_t candidates = 0;   // valid substring nodes found on the device
  float device_ms = 0.f;     // device time of the substring pipeline
  float stages[7] = {};      // spm_hip_seeds_stage_times (include/spm_hip.h)
};

namespace spm_amd {
namespace {

thread_local std::string g_seed_error;

constexpr uint32_t kFlagInvalid = 1u << 16;  // UNK char, NUL, tab, space, bad code point
constexpr uint32_t kFlagWS = 1u << 17;       // U+2581
constexpr uint32_t kFlagNumber = 1u << 18;   // 0-9
constexpr uint32_t kScriptMask = 0xFFFFu;
constexpr int kMaxLevels = 7;
// LSD suffix order while it takes at most this many 32-bit key chunks
// (max_sentencepiece_length 16: alphabets up to 2^10 symbols); beyond, the
// prefix doubling (log2 rounds) is cheaper.
constexpr int kMaxLsdChunks = 9;
constexpr int kDepthBits = 10;  // key1 depth field: max_sentencepiece_length <= 512
constexpr uint64_t kDepthMask = (1u << kDepthBits) - 1;

struct SeedOpts {
  int max_len;
  bool by_script, by_number, by_ws, ws_suffix;
};

// HT: uint8_t for max_sentencepiece_length <= 254, uint16_t up to 512.
template <typename HT>
struct Pyramid {
  const HT *lv[kMaxLevels];
  uint64_t size[kMaxLevels];
  int levels;
};

// util.cc:187-227 DecodeUTF8
__device__ __forceinline__ uint32_t DecodeUTF8Dev(const uint8_t *b, uint64_t len, uint32_t *mblen) {
  const uint32_t c0 = b[0];
  auto trail = [](uint32_t x) { return (x & 0xC0) == 0x80; };
  auto valid = [](uint32_t c) { return c < 0xD800 || (c >= 0xE000 && c <= 0x10FFFF); };
  if (c0 < 0x80) {
    *mblen = 1;
    return c0;
  } else if (len >= 2 && (c0 & 0xE0) == 0xC0) {
    const uint32_t cp = ((c0 & 0x1F) << 6) | (b[1] & 0x3F);
    if (trail(b[1]) && cp >= 0x80 && valid(cp)) {
      *mblen = 2;
      return cp;
    }
  } else if (len >= 3 && (c0 & 0xF0) == 0xE0) {
    const uint32_t cp = ((c0 & 0x0F) << 12) | ((b[1] & 0x3F) << 6) | (b[2] & 0x3F);
    if (trail(b[1]) && trail(b[2]) && cp >= 0x800 && valid(cp)) {
      *mblen = 3;
      return cp;
    }
  } else if (len >= 4 && (c0 & 0xF8) == 0xF0) {
    const uint32_t cp = ((c0 & 0x07) << 18) | ((b[1] & 0x3F) << 12) | ((b[2] & 0x3F) << 6) |
                        (b[3] & 0x3F);
    if (trail(b[1]) && trail(b[2]) && trail(b[3]) && cp >= 0x10000 && valid(cp)) {
      *mblen = 4;
      return cp;
    }
  }
  *mblen = 1;
  return 0xFFFD;
}

// chars per sentence + 1 (the boundary)
__global__ void seed_count_kernel(const uint8_t *bytes, const uint64_t *off, uint64_t n,
                                  uint64_t *cnt) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *b = bytes + off[i];
  const uint64_t len = off[i + 1] - off[i];
  uint64_t p = 0, c = 0;
  while (p < len) {
    uint32_t m;
    DecodeUTF8Dev(b + p, len - p, &m);
    p += m;
    ++c;
  }
  cnt[i] = c + 1;
}

// T = alphabet rank of each char (0 = boundary), dist = chars before the
// next boundary (saturating at 0xFFFF).
__global__ void seed_decode_kernel(const uint8_t *bytes, const uint64_t *off, uint64_t n,
                                   const uint64_t *coff, const uint32_t *lut, uint32_t *T,
                                   uint16_t *dist, uint32_t *err) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *b = bytes + off[i];
  const uint64_t len = off[i + 1] - off[i];
  const uint64_t base = coff[i];
  const uint64_t nc = coff[i + 1] - base - 1;
  if (nc >= 0xFFFF) atomicOr(err, 2u);
  uint64_t p = 0, c = 0;
  while (p < len) {
    uint32_t m;
    const uint32_t cp = DecodeUTF8Dev(b + p, len - p, &m);
    const uint32_t r = lut[cp];
    if (r == 0) atomicOr(err, 1u);
    T[base + c] = r;
    dist[base + c] = static_cast<uint16_t>(min<uint64_t>(nc - c, 0xFFFF));
    p += m;
    ++c;
  }
  T[base + nc] = 0;
  dist[base + nc] = 0;
}

// First key: k0 chars of bits b each, zero after the boundary.
__global__ void seed_key0_kernel(const uint32_t *T, const uint16_t *dist, uint64_t n, int bits,
                                 int k0, uint64_t *keys, uint32_t *vals) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int m = min<int>(k0, dist[i]);
  uint64_t key = 0;
  for (int c = 0; c < m; ++c) key |= uint64_t(T[i + c]) << (bits * (k0 - 1 - c));
  keys[i] = key;
  vals[i] = static_cast<uint32_t>(i);
}

// LSD suffix-order sorts: rocPRIM onesweep, 10 bits per pass (the E-step's
// record sort configuration, estep_kernels.hip).
using SeedSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 6>, 10,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

// T carries kTPad zero words past its end for the LCP kernel's 4-symbol
// steps.  (Unrolled, predicated chunk-key loads measured slower: 70.7 -> 81.2
// ms per pass at c5.)
constexpr uint64_t kTPad = 64;

// LSD prefix sort, one 32-bit key per chunk of kc chars starting c0 chars
// into the suffix (zero after the boundary).  The suffix of slot j is
// vals_in[j] (nullptr: j itself, and vals_out[j] = j).
__global__ void seed_chunkkey_kernel(const uint32_t *T, const uint16_t *dist, uint64_t n, int bits, int c0, int kc,
                                     const uint32_t *vals_in, uint32_t *keys, uint32_t *vals_out) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t i = vals_in ? vals_in[j] : j;
  const int m = min<int>(kc, max<int>(0, int(dist[i]) - c0));
  uint32_t key = 0;
  for (int c = 0; c < m; ++c) key |= T[i + c0 + c] << (bits * (kc - 1 - c));
  keys[j] = key;
  if (!vals_in) vals_out[j] = static_cast<uint32_t>(j);
}

// ---- MSD split of the suffix order for large corpora: part q holds the
// suffixes whose first symbol is in [b[q], b[q + 1]); the parts are sorted
// one after another, each by the LSD passes over its own suffixes, straight
// into its segment of SA (the first symbol is the most significant digit, so
// the segments in part order are the whole order, ties still by ascending
// suffix: the split is stable).  The sort buffers then hold one part.
constexpr int kMaxParts = 8;
constexpr int kPartTile = 4096;  // suffixes per block of the split (256 threads x 16)
constexpr int kHistBins = 8192;  // first-symbol histogram bins (LDS counters)
struct PartBounds {
  uint32_t b[kMaxParts + 1];
  int parts;
};

__device__ __forceinline__ int PartOf(const PartBounds &pb, uint32_t t) {
  int q = 0;
  for (int k = 1; k < pb.parts; ++k) q += t >= pb.b[k];
  return q;
}

// hist[t >> shift] += 1 over the suffixes' first symbols T[0, n).
__global__ __launch_bounds__(256) void seed_hist_kernel(const uint32_t *T, uint64_t n, int shift, uint32_t bins,
                                                        unsigned long long *hist) {
  __shared__ uint32_t lh[kHistBins];
  for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x) lh[k] = 0;
  __syncthreads();
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    atomicAdd(&lh[T[i] >> shift], 1u);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < bins; k += blockDim.x)
    if (lh[k]) atomicAdd(&hist[k], static_cast<unsigned long long>(lh[k]));
}

// counts[q * tiles + tile] = suffixes of part q in the tile.
__global__ __launch_bounds__(256) void seed_part_count_kernel(const uint32_t *T, uint64_t n, PartBounds pb,
                                                              uint64_t tiles, uint64_t *counts) {
  __shared__ uint32_t c[kMaxParts];
  if (threadIdx.x < kMaxParts) c[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = uint64_t(blockIdx.x) * kPartTile;
  for (uint32_t k = threadIdx.x; k < kPartTile; k += blockDim.x) {
    const uint64_t i = t0 + k;
    if (i < n) atomicAdd(&c[PartOf(pb, T[i])], 1u);
  }
  __syncthreads();
  if (threadIdx.x < static_cast<unsigned>(pb.parts)) counts[uint64_t(threadIdx.x) * tiles + blockIdx.x] = c[threadIdx.x];
}

// out[base[q * tiles + tile] + (rank of suffix i among the tile's part-q
// suffixes)] = i: ascending i within each part (stable).
__global__ __launch_bounds__(256) void seed_part_scatter_kernel(const uint32_t *T, uint64_t n, PartBounds pb,
                                                                uint64_t tiles, const uint64_t *base,
                                                                uint32_t *out) {
  __shared__ uint32_t run[kMaxParts];           // the tile's part-q suffixes placed so far
  __shared__ uint32_t wcnt[4][kMaxParts];       // this round's per-wave counts
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (tid < kMaxParts) run[tid] = 0;
  const uint64_t t0 = uint64_t(blockIdx.x) * kPartTile;
  const uint64_t lanes_below = (lane ? ~0ull >> (64 - lane) : 0ull);
  for (int r = 0; r < kPartTile / 256; ++r) {
    const uint64_t i = t0 + uint64_t(r) * 256 + tid;
    const int q = i < n ? PartOf(pb, T[i]) : -1;
    uint32_t below = 0;
    for (int p = 0; p < pb.parts; ++p) {
      const uint64_t m = __ballot(q == p);
      if (q == p) below = __popcll(m & lanes_below);
      if (lane == 0) wcnt[wave][p] = __popcll(m);
    }
    __syncthreads();
    if (q >= 0) {
      uint32_t at = run[q] + below;
      for (int w = 0; w < wave; ++w) at += wcnt[w][q];
      out[base[uint64_t(q) * tiles + blockIdx.x] + at] = static_cast<uint32_t>(i);
    }
    __syncthreads();
    if (tid < pb.parts) run[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
    __syncthreads();
  }
}

// g[j] = j if sorted key j starts a group else 0 (inclusive max-scan → group start).
__global__ void seed_heads_kernel(const uint64_t *keys, uint64_t n, uint32_t *g) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  g[j] = (j == 0 || keys[j] != keys[j - 1]) ? static_cast<uint32_t>(j) : 0u;
}

// rank[suffix] = its group start; flag unfinished groups (size > 1 and the
// truncated strings longer than h).
__global__ void seed_rank_kernel(const uint64_t *keys, const uint32_t *vals, const uint32_t *gs,
                                 const uint16_t *dist, uint64_t n, uint32_t h, uint32_t *rank,
                                 uint32_t *unfinished) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t i = vals[j];
  rank[i] = gs[j];
  if (j > 0 && keys[j] == keys[j - 1] && dist[i] >= h) *unfinished = 1u;
}

// Doubling key in current order: (rank[i], rank[i+h] + 1 or 0 if the
// truncated string ends within h chars).
__global__ void seed_pairkey_kernel(const uint32_t *vals, const uint32_t *rank,
                                    const uint16_t *dist, uint64_t n, uint32_t h, uint64_t *keys) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t i = vals[j];
  const uint64_t second = dist[i] >= h ? uint64_t(rank[i + h]) + 1 : 0;
  keys[j] = (uint64_t(rank[i]) << 32) | second;
}

// H[j] = min(clamp, common prefix of suffixes SA[j-1], SA[j] counting a
// shared boundary); H[0] = 0.
template <typename HT>
__global__ void seed_lcp_kernel(const uint32_t *T, const uint32_t *SA, uint64_t n, int clamp,
                                HT *H) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  if (j == 0) {
    H[0] = 0;
    return;
  }
  const uint32_t *a = T + SA[j - 1];
  const uint32_t *b = T + SA[j];
  int c = 0;
  // Four symbols of each suffix per step, their loads issued together (T
  // is padded past its end): a quarter of the dependent steps of a
  // compare-as-you-load loop, at most three symbols read past the answer.
  // (Loading all clamp symbols at once read too much: 514 -> 744 ms at c5.)
  while (c < clamp) {
    uint32_t x[4], y[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[k] = a[c + k];
      y[k] = b[c + k];
    }
    int stop = -1;
#pragma unroll
    for (int k = 3; k >= 0; --k) {  // the first position that ends the prefix
      if (x[k] != y[k]) stop = k;
      else if (x[k] == 0) stop = k + 1 + 8;  // (tag: a shared boundary counts)
    }
    if (stop >= 0) {
      c += stop >= 8 ? stop - 8 : stop;
      break;
    }
    c += 4;
  }
  if (c > clamp) c = clamp;
  H[j] = static_cast<HT>(c);
}

template <typename HT>
__global__ void seed_pyr_kernel(const HT *in, uint64_t n_in, HT *out, uint64_t n_out) {
  const uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= n_out) return;
  const uint64_t b = k * 64, e = min<uint64_t>(b + 64, n_in);
  HT m = static_cast<HT>(~HT(0));
  for (uint64_t x = b; x < e; ++x) m = in[x] < m ? in[x] : m;
  out[k] = m;
}

// First k > j with H[k] < d, or n.
template <typename HT>
__device__ uint64_t NextLess(const Pyramid<HT> &P, uint64_t j, int d) {
  uint64_t k = j + 1;
  int L = 0;
  while (true) {
    if (k >= P.size[L]) return P.size[0];
    const uint64_t end = min<uint64_t>((k | 63) + 1, P.size[L]);
    for (; k < end; ++k)
      if (P.lv[L][k] < d) goto descend;
    if (end == P.size[L] || L + 1 == P.levels) return P.size[0];
    k = end >> 6;
    ++L;
  }
descend:
  while (L > 0) {
    --L;
    k *= 64;
    const uint64_t end = min<uint64_t>(k + 64, P.size[L]);
    while (k < end && P.lv[L][k] >= d) ++k;
  }
  return k;
}

// Last k < j with H[k] <= d (exists: H[0] = 0).
template <typename HT>
__device__ uint64_t PrevLeq(const Pyramid<HT> &P, uint64_t j, int d) {
  int64_t k = int64_t(j) - 1;
  int L = 0;
  while (true) {
    const int64_t beg = k & ~int64_t(63);
    for (; k >= beg; --k)
      if (P.lv[L][k] <= d) goto descend;
    if (beg == 0) return 0;
    k = (beg >> 6) - 1;
    ++L;
  }
descend:
  while (L > 0) {
    --L;
    k = k * 64 + 63;
    if (k >= int64_t(P.size[L])) k = int64_t(P.size[L]) - 1;
    while (P.lv[L][k] > d) --k;
  }
  return uint64_t(k);
}

// trainer_interface.cc:178-267 over alphabet-rank flags.
__device__ bool ValidPiece(const uint32_t *s, int d, const uint32_t *rtab, const SeedOpts &o) {
  int prev = -1;
  for (int pos = 0; pos < d; ++pos) {
    const uint32_t f = rtab[s[pos]];
    if (f & kFlagInvalid) return false;
    if (f & kFlagWS) {
      if (o.ws_suffix) {
        if ((o.by_ws && pos < d - 1) || (!o.by_ws && pos < d - 1 && pos == 0)) return false;
      } else {
        if ((o.by_ws && pos > 0) || (!o.by_ws && pos > 0 && pos == d - 1)) return false;
      }
    } else {
      int sc = int(f & kScriptMask);
      if (!o.by_number && (f & kFlagNumber)) sc = -1;
      if (o.by_script && sc != -1 && prev != -1 && prev != sc) return false;
      prev = sc;
    }
  }
  return true;
}

// One candidate per valid 0-free node of depth 2..max_len, at its leftmost
// boundary j.  key1 = R << 10 | (1023 - D) (node index order), score = (R-L)*D.
template <typename HT>
__global__ void seed_nodes_kernel(const uint32_t *T, const uint32_t *SA, Pyramid<HT> P,
                                  const uint32_t *rtab, SeedOpts o, uint64_t *key1,
                                  uint64_t *score, uint32_t *pos_out, uint32_t *idx,
                                  unsigned long long *count, uint64_t cap) {
  const uint64_t n = P.size[0];
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  bool emit = false;
  uint64_t k1 = 0, sc = 0;
  uint32_t pos = 0;
  if (j >= 1 && j < n) {
    const HT *H = P.lv[0];
    const int d = H[j];
    if (d >= 2 && d <= o.max_len) {
      pos = SA[j];
      const uint32_t *s = T + pos;
      const int hp = H[j - 1];
      if (s[d - 1] != 0 && hp != d && ValidPiece(s, d, rtab, o)) {
        uint64_t l = j - 1;
        bool leftmost = true;
        if (hp > d) {
          l = PrevLeq(P, j, d);
          leftmost = H[l] < d;
        }
        if (leftmost) {
          const uint64_t r = (j + 1 < n && H[j + 1] < d) ? j + 1 : NextLess(P, j, d);
          k1 = (r << kDepthBits) | uint64_t(kDepthMask - d);
          sc = (r - l) * uint64_t(d);
          emit = true;
        }
      }
    }
  }
  // wave-aggregated append
  const unsigned long long mask = __ballot(emit);
  if (mask == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll(static_cast<long long>(mask)) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(count, static_cast<unsigned long long>(__popcll(mask)));
  base = __shfl(base, leader);
  if (emit) {
    const unsigned long long slot =
        base + __popcll(mask & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
    if (slot >= cap) return;  // counted; the host re-runs with room for all
    key1[slot] = k1;
    score[slot] = sc;
    pos_out[slot] = pos;
    idx[slot] = static_cast<uint32_t>(slot);
  }
}

// key2 (score descending) in key1-sorted order.
__global__ void seed_key2_kernel(const uint32_t *idx, const uint64_t *score, uint64_t m,
                                 uint64_t *key2) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= m) return;
  key2[j] = (uint64_t(1) << 48) - 1 - score[idx[j]];
}

// Top K: depth and score of each selected node, then its chars (alphabet
// ranks) packed at host-scanned offsets.
__global__ void seed_gather_len_kernel(const uint32_t *idx, const uint64_t *key1, const uint64_t *score,
                                       uint64_t K, int64_t *out_score, int32_t *out_len) {
  const uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const uint32_t c = idx[k];
  out_len[k] = int(kDepthMask) - int(key1[c] & kDepthMask);
  out_score[k] = static_cast<int64_t>(score[c]);
}

__global__ void seed_gather_chars_kernel(const uint32_t *idx, const uint32_t *pos, const uint32_t *T,
                                         uint64_t K, const uint64_t *out_off, uint32_t *out_chars) {
  const uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const uint32_t *s = T + pos[idx[k]];
  const uint64_t b = out_off[k], d = out_off[k + 1] - b;
  for (uint64_t x = 0; x < d; ++x) out_chars[b + x] = s[x];
}

struct MaxOp {
  __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const {
    return a > b ? a : b;
  }
};

inline unsigned Blocks(uint64_t n, unsigned t = 256) {
  return static_cast<unsigned>((n + t - 1) / t);
}

int SeedFail(int code, const std::string &msg) {
  g_seed_error = msg;
  return code;
}

#define SEED_TRY(expr)                                                                  \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return SeedFail(SPM_INTERNAL, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

}  // namespace

namespace {

// Scratch owned by one call; released on every return path (into the
// trainer's scratch cache while one is open, scratch_cache.h).
struct Scratch {
  std::vector<void *> ptrs;
  hipStream_t st = nullptr;  // the stream the blocks are used on
  double alloc_ms = 0;       // host wall time inside hipMalloc
  ~Scratch() {
    for (void *p : ptrs) ScratchFree(p, st);
  }
  template <typename T>
  hipError_t Alloc(T **p, uint64_t count) {
    void *v = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = ScratchAlloc(&v, std::max<uint64_t>(count, 1) * sizeof(T));
    alloc_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (e == hipSuccess) {
      ptrs.push_back(v);
      *p = static_cast<T *>(v);
    }
    return e;
  }
};

void AppendUTF8(uint32_t c, std::vector<uint8_t> *out) {
  if (c <= 0x7F) {
    out->push_back(uint8_t(c));
  } else if (c <= 0x7FF) {
    out->push_back(uint8_t(0xC0 | (c >> 6)));
    out->push_back(uint8_t(0x80 | (c & 0x3F)));
  } else if (c <= 0xFFFF) {
    out->push_back(uint8_t(0xE0 | (c >> 12)));
    out->push_back(uint8_t(0x80 | ((c >> 6) & 0x3F)));
    out->push_back(uint8_t(0x80 | (c & 0x3F)));
  } else {
    out->push_back(uint8_t(0xF0 | (c >> 18)));
    out->push_back(uint8_t(0x80 | ((c >> 12) & 0x3F)));
    out->push_back(uint8_t(0x80 | ((c >> 6) & 0x3F)));
    out->push_back(uint8_t(0x80 | (c & 0x3F)));
  }
}

int HostScript(uint32_t c) {
  int lo = 0, hi = kNumScriptRanges - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) / 2;
    if (c < kScriptRanges[mid].lo) hi = mid - 1;
    else if (c > kScriptRanges[mid].hi) lo = mid + 1;
    else return kScriptRanges[mid].script;
  }
  return kScriptCommon;
}

// Substring part on the device.  alphabet: sorted code points (rank = index
// + 1).  Fills (chars, score) of the top K nodes in Sorted order.
int MineSubstrings(const uint8_t *h_bytes, const uint64_t *h_off, uint64_t n, bool on_device,
                   const std::vector<uint32_t> &alphabet, const SeedOpts &o, uint64_t K,
                   std::vector<std::vector<uint32_t>> *out, std::vector<int64_t> *out_score,
                   uint64_t *num_candidates, float *ms, float *stages) {
  spm_amd::TraceRange trace_range_("seed_mine_substrings");
  hipStream_t st = nullptr;
  Scratch S;
  // Stage boundaries (events on the stream): 0 start, 1 decoded, 2 first
  // sort, 3 prefix doubling done, 4 candidate nodes, 5 end.
  hipEvent_t ev[6];
  for (auto &e : ev) SEED_TRY(hipEventCreate(&e));
  struct EvGuard {
    hipEvent_t *v;
    ~EvGuard() {
      for (int k = 0; k < 6; ++k) (void)hipEventDestroy(v[k]);
    }
  } evg{ev};
  hipEvent_t e0 = ev[0], e1 = ev[5];
  int rounds = 0;
  uint64_t nbytes = 0;
  if (on_device) {
    SEED_TRY(hipMemcpy(&nbytes, h_off + n, 8, hipMemcpyDeviceToHost));
  } else {
    nbytes = h_off[n];
  }
  uint8_t *d_bytes;
  uint64_t *d_off, *d_coff;
  uint32_t *d_lut, *d_rtab, *d_err;
  if (on_device) {
    d_bytes = const_cast<uint8_t *>(h_bytes);
    d_off = const_cast<uint64_t *>(h_off);
  } else {
    SEED_TRY(S.Alloc(&d_bytes, nbytes));
    SEED_TRY(S.Alloc(&d_off, n + 1));
  }
  SEED_TRY(S.Alloc(&d_coff, n + 1));
  SEED_TRY(S.Alloc(&d_lut, 0x110000));
  SEED_TRY(S.Alloc(&d_rtab, alphabet.size() + 1));
  SEED_TRY(S.Alloc(&d_err, 2));
  std::vector<uint32_t> lut(0x110000, 0u), rtab(alphabet.size() + 1, 0u);
  rtab[0] = kFlagInvalid;  // the boundary (never inside a counted piece)
  for (size_t r = 0; r < alphabet.size(); ++r) {
    const uint32_t c = alphabet[r];
    lut[c] = uint32_t(r + 1);
    uint32_t f = 0;
    const bool valid_cp = c < 0xD800 || (c >= 0xE000 && c <= 0x10FFFF);
    if (c == 0x2585 || c == 0 || c == 0x09 || c == 0x20 || !valid_cp) f |= kFlagInvalid;
    if (c == 0x2581) f |= kFlagWS;
    if (c >= 0x30 && c <= 0x39) f |= kFlagNumber;
    int s = HostScript(c);
    // Hiragana / Katakana / U+30FC merge into Han (trainer_interface.cc:238-242).
    if (s == kScriptHiragana || s == kScriptKatakana || c == 0x30FC) s = kScriptHan;
    rtab[r + 1] = f | uint32_t(s);
  }
  SEED_TRY(hipEventRecord(e0, st));
  if (!on_device) {
    SEED_TRY(hipMemcpyAsync(d_bytes, h_bytes, nbytes, hipMemcpyHostToDevice, st));
    SEED_TRY(hipMemcpyAsync(d_off, h_off, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  }
  SEED_TRY(hipMemcpyAsync(d_lut, lut.data(), lut.size() * 4, hipMemcpyHostToDevice, st));
  SEED_TRY(hipMemcpyAsync(d_rtab, rtab.data(), rtab.size() * 4, hipMemcpyHostToDevice, st));
  SEED_TRY(hipMemsetAsync(d_err, 0, 8, st));
  // chars per sentence → offsets
  uint64_t *d_cnt;
  SEED_TRY(S.Alloc(&d_cnt, n));
  seed_count_kernel<<<Blocks(n), 256, 0, st>>>(d_bytes, d_off, n, d_cnt);
  SEED_TRY(hipGetLastError());
  SEED_TRY(hipMemsetAsync(d_coff, 0, 8, st));
  size_t tb = 0;
  SEED_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb, d_cnt, d_coff + 1, n, st));
  void *d_tmp = nullptr;
  size_t tmp_cap = tb;
  SEED_TRY(S.Alloc(reinterpret_cast<uint8_t **>(&d_tmp), tb));
  SEED_TRY(hipcub::DeviceScan::InclusiveSum(d_tmp, tb, d_cnt, d_coff + 1, n, st));
  uint64_t N = 0;
  SEED_TRY(hipMemcpyAsync(&N, d_coff + n, 8, hipMemcpyDeviceToHost, st));
  SEED_TRY(hipStreamSynchronize(st));
  if (N >= 0xFFFFFFFFull) return SeedFail(SPM_RESOURCE_EXHAUSTED, "corpus exceeds 2^32-1 chars");
  uint32_t *T;
  uint16_t *dist;
  SEED_TRY(S.Alloc(&T, N + 1 + kTPad));
  SEED_TRY(hipMemsetAsync(T + N + 1, 0, kTPad * 4, st));
  SEED_TRY(S.Alloc(&dist, N + 1));
  seed_decode_kernel<<<Blocks(n), 256, 0, st>>>(d_bytes, d_off, n, d_coff, d_lut, T, dist, d_err);
  SEED_TRY(hipGetLastError());
  uint32_t herr[2] = {0, 0};
  SEED_TRY(hipMemcpyAsync(herr, d_err, 8, hipMemcpyDeviceToHost, st));
  SEED_TRY(hipStreamSynchronize(st));
  if (herr[0] & 1u) return SeedFail(SPM_INVALID_ARGUMENT, "a sentence holds a char outside the alphabet");
  if (herr[0] & 2u) return SeedFail(SPM_UNIMPLEMENTED, "sentence longer than 65534 chars");
  SEED_TRY(hipEventRecord(ev[1], st));
  int bits = 1;
  while ((uint64_t(1) << bits) <= alphabet.size()) ++bits;
  auto ensure_tmp = [&](size_t need) -> hipError_t {
    if (need <= tmp_cap) return hipSuccess;
    tmp_cap = need;
    return S.Alloc(reinterpret_cast<uint8_t **>(&d_tmp), need);
  };
  auto sort_pairs = [&](const uint64_t *ki, uint64_t *ko, const uint32_t *vi, uint32_t *vo,
                        uint64_t m, int end_bit) -> hipError_t {
    size_t need = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, need, ki, ko, vi, vo, m, 0, end_bit, st);
    if (e != hipSuccess) return e;
    if ((e = ensure_tmp(need)) != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairs(d_tmp, need, ki, ko, vi, vo, m, 0, end_bit, st);
  };
  // The nodes only need the suffixes ordered by their first L = max_len + 1
  // (truncated) symbols: every 0-free node of depth <= max_len is a union of
  // whole groups of that order, with the same L, R and D.
  const int Lsym = o.max_len + 1;
  const int kc32 = 32 / bits;  // symbols per 32-bit key
  const int chunks = kc32 > 0 ? (Lsym + kc32 - 1) / kc32 : 0;
  const uint32_t *SA = nullptr;
  // Candidate node arrays and their capacity (the nodes kernel counts past
  // it; the host then re-runs it with exact room).
  uint64_t *key1 = nullptr, *score = nullptr, *key2;
  uint32_t *cpos = nullptr, *idx = nullptr;
  uint8_t *h_borrow = nullptr;  // room for a uint8 LCP array the sort left free
  uint64_t cap = 0;
  if (chunks >= 1 && chunks <= kMaxLsdChunks) {
    // LSD radix order over ceil(L / kc32) chunks of 32-bit keys, the last
    // chunk first, each a stable sort of (chunk key, suffix) in the current
    // order, ping-ponging between two key and two value buffers (no sort
    // temp of N items).  22 B per char (T 4, dist 2, keys 2 x 4, suffixes
    // 2 x 4) instead of the prefix doubling's ~51 B with its rank and group
    // arrays and the 12 B/char sort temp; the key kernels read T in order
    // (first chunk) or gather one short run per suffix, and there are no
    // rank scatters.
    uint32_t *kA, *kB, *vA, *vB;
    // rocPRIM onesweep with 10-bit digits (3 passes for the 30-bit keys of
    // a <= 31-symbol alphabet instead of hipCUB's four 8-bit ones), the two
    // buffers ping-ponging (no N-item temp); stable like every LSD pass needs.
    auto sort32 = [&](hipcub::DoubleBuffer<uint32_t> &dk, hipcub::DoubleBuffer<uint32_t> &dv,
                      int end_bit, uint64_t m) -> hipError_t {
      rocprim::double_buffer<uint32_t> rk(dk.d_buffers[dk.selector], dk.d_buffers[dk.selector ^ 1]);
      rocprim::double_buffer<uint32_t> rv(dv.d_buffers[dv.selector], dv.d_buffers[dv.selector ^ 1]);
      size_t need = 0;
      hipError_t e = rocprim::radix_sort_pairs<SeedSortConfig>(nullptr, need, rk, rv, m, 0u,
                                                              static_cast<unsigned>(end_bit), st);
      if (e != hipSuccess) return e;
      if ((e = ensure_tmp(need)) != hipSuccess) return e;
      e = rocprim::radix_sort_pairs<SeedSortConfig>(d_tmp, need, rk, rv, m, 0u, static_cast<unsigned>(end_bit), st);
      if (e != hipSuccess) return e;
      if (rk.current() != dk.d_buffers[dk.selector]) dk.selector ^= 1;
      if (rv.current() != dv.d_buffers[dv.selector]) dv.selector ^= 1;
      return hipSuccess;
    };
    // Parts (MSD split by first symbol, see seed_part_scatter_kernel): 4 for
    // corpora of >= 2^28 chars, where the 16 B/char of sort buffers set the
    // trainer's peak (70.3 GB at c5); SPM_HIP_SEED_PARTS=1..8 overrides.
    int parts = N >= (1ull << 28) ? 4 : 1;
    if (const char *e = std::getenv("SPM_HIP_SEED_PARTS")) parts = std::max(1, std::min(kMaxParts, std::atoi(e)));
    PartBounds pb{};
    std::vector<uint64_t> part_n;
    uint64_t max_part = N;
    uint32_t *SAbuf = nullptr;
    uint64_t tiles = 0;
    uint64_t *pbase = nullptr;
    if (parts > 1) {
      // First-symbol histogram (bins of 2^shift symbols), then cut points at
      // bin edges near every N / parts suffixes.
      const uint32_t nsym = static_cast<uint32_t>(alphabet.size()) + 1;
      int shift = 0;
      while (((nsym - 1) >> shift) + 1 > static_cast<uint32_t>(kHistBins)) ++shift;
      const uint32_t bins = ((nsym - 1) >> shift) + 1;
      unsigned long long *d_hist;
      SEED_TRY(S.Alloc(&d_hist, bins));
      SEED_TRY(hipMemsetAsync(d_hist, 0, bins * 8, st));
      seed_hist_kernel<<<2048, 256, 0, st>>>(T, N, shift, bins, d_hist);
      SEED_TRY(hipGetLastError());
      std::vector<unsigned long long> hist(bins);
      SEED_TRY(hipMemcpyAsync(hist.data(), d_hist, bins * 8, hipMemcpyDeviceToHost, st));
      SEED_TRY(hipStreamSynchronize(st));
      pb.b[0] = 0;
      int q = 0;
      uint64_t acc = 0, in_part = 0;
      part_n.clear();
      for (uint32_t k = 0; k < bins; ++k) {
        acc += hist[k];
        in_part += hist[k];
        if (q + 1 < parts && acc * parts >= (q + 1) * N && k + 1 < bins) {
          pb.b[++q] = (k + 1) << shift;
          part_n.push_back(in_part);
          in_part = 0;
        }
      }
      part_n.push_back(in_part);
      parts = q + 1;
      pb.b[parts] = 0xFFFFFFFFu;
      pb.parts = parts;
      if (acc != N) return SeedFail(SPM_INTERNAL, "seed split: histogram does not cover the suffixes");
      max_part = *std::max_element(part_n.begin(), part_n.end());
    }
    if (parts > 1) {
      // The stable split into SA's segments (tile counts, an exclusive scan
      // in part-major order, a scatter).
      SEED_TRY(S.Alloc(&SAbuf, N));
      tiles = (N + kPartTile - 1) / kPartTile;
      uint64_t *d_cnt2;
      SEED_TRY(S.Alloc(&d_cnt2, uint64_t(parts) * tiles));
      SEED_TRY(S.Alloc(&pbase, uint64_t(parts) * tiles));
      seed_part_count_kernel<<<static_cast<unsigned>(tiles), 256, 0, st>>>(T, N, pb, tiles, d_cnt2);
      SEED_TRY(hipGetLastError());
      size_t need = 0;
      SEED_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, need, d_cnt2, pbase, static_cast<int>(parts * tiles), st));
      SEED_TRY(ensure_tmp(need));
      SEED_TRY(hipcub::DeviceScan::ExclusiveSum(d_tmp, need, d_cnt2, pbase, static_cast<int>(parts * tiles), st));
      seed_part_scatter_kernel<<<static_cast<unsigned>(tiles), 256, 0, st>>>(T, N, pb, tiles, pbase, SAbuf);
      SEED_TRY(hipGetLastError());
      SEED_TRY(S.Alloc(&kA, max_part));
      SEED_TRY(S.Alloc(&kB, max_part));
      SEED_TRY(S.Alloc(&vB, max_part));
      SEED_TRY(hipEventRecord(ev[2], st));
      uint64_t at = 0;
      for (int p = 0; p < parts; ++p) {
        const uint64_t m = part_n[p];
        uint32_t *seg = SAbuf + at;
        at += m;
        if (m == 0) continue;
        int c = chunks - 1;
        const int kc_last = Lsym - c * kc32;
        seed_chunkkey_kernel<<<Blocks(m), 256, 0, st>>>(T, dist, m, bits, c * kc32, kc_last, seg, kA, nullptr);
        SEED_TRY(hipGetLastError());
        hipcub::DoubleBuffer<uint32_t> dk(kA, kB), dv(seg, vB);
        SEED_TRY(sort32(dk, dv, bits * kc_last, m));
        for (--c; c >= 0; --c) {
          if (p == 0) ++rounds;
          seed_chunkkey_kernel<<<Blocks(m), 256, 0, st>>>(T, dist, m, bits, c * kc32, kc32, dv.Current(),
                                                           dk.Alternate(), nullptr);
          SEED_TRY(hipGetLastError());
          dk.selector ^= 1;
          SEED_TRY(sort32(dk, dv, bits * kc32, m));
        }
        if (dv.Current() != seg) SEED_TRY(hipMemcpyAsync(seg, dv.Current(), m * 4, hipMemcpyDeviceToDevice, st));
      }
      SA = SAbuf;
      // The capped LCP (1 B per suffix) borrows one key buffer (4 B x
      // max_part >= N bytes), the candidate arrays the other one (key1 and
      // score, 8 B x max_part / 4 each), the value buffer and dist.
      if (max_part * 4 >= N) h_borrow = reinterpret_cast<uint8_t *>(kB);  // (<= 4 parts)
      cap = max_part / 4;
      key1 = reinterpret_cast<uint64_t *>(kA);
      score = reinterpret_cast<uint64_t *>(kA) + cap;
      cpos = vB;
      idx = reinterpret_cast<uint32_t *>(dist);
    } else {
    SEED_TRY(S.Alloc(&kA, N));
    SEED_TRY(S.Alloc(&vA, N));
    int c = chunks - 1;
    const int kc_last = Lsym - c * kc32;
    seed_chunkkey_kernel<<<Blocks(N), 256, 0, st>>>(T, dist, N, bits, c * kc32, kc_last, nullptr, kA, vA);
    SEED_TRY(hipGetLastError());
    SEED_TRY(S.Alloc(&kB, N));
    SEED_TRY(S.Alloc(&vB, N));
    hipcub::DoubleBuffer<uint32_t> dk(kA, kB), dv(vA, vB);
    SEED_TRY(sort32(dk, dv, bits * kc_last, N));
    SEED_TRY(hipEventRecord(ev[2], st));
    for (--c; c >= 0; --c) {
      ++rounds;
      seed_chunkkey_kernel<<<Blocks(N), 256, 0, st>>>(T, dist, N, bits, c * kc32, kc32, dv.Current(),
                                                       dk.Alternate(), nullptr);
      SEED_TRY(hipGetLastError());
      dk.selector ^= 1;
      SEED_TRY(sort32(dk, dv, bits * kc32, N));
    }
    SA = dv.Current();
    // The candidate arrays live in buffers the sort no longer needs: the two
    // key buffers (8 B x N/2 each), the other suffix buffer and dist.
    cap = N / 2;
    key1 = reinterpret_cast<uint64_t *>(dk.Current());
    score = reinterpret_cast<uint64_t *>(dk.Alternate());
    cpos = dv.Alternate();
    idx = reinterpret_cast<uint32_t *>(dist);
    }
  } else {
    // Prefix doubling (long max_sentencepiece_length or huge alphabets).
    // Each ~4-8 B/char buffer is allocated just before its first use: with
    // the six allocated together, the host spent 0.73 s inside hipMalloc at
    // c5 (100 M lines, profiles/r03z_bench.json seed_stages_ms[5]).
    uint32_t *rank, *vals_a, *vals_b, *g;
    uint64_t *keys_a, *keys_b;
    SEED_TRY(S.Alloc(&keys_a, N));
    SEED_TRY(S.Alloc(&vals_a, N));
    const int k0 = 64 / bits;
    seed_key0_kernel<<<Blocks(N), 256, 0, st>>>(T, dist, N, bits, k0, keys_a, vals_a);
    SEED_TRY(hipGetLastError());
    SEED_TRY(S.Alloc(&keys_b, N));
    SEED_TRY(S.Alloc(&vals_b, N));
    SEED_TRY(sort_pairs(keys_a, keys_b, vals_a, vals_b, N, bits * k0));
    SEED_TRY(S.Alloc(&rank, N));  // while the first sort runs
    SEED_TRY(S.Alloc(&g, N));
    SEED_TRY(hipEventRecord(ev[2], st));
    uint32_t h = static_cast<uint32_t>(k0);
    while (true) {
      ++rounds;
      // keys_b / vals_b: sorted by the first h chars (truncated).
      seed_heads_kernel<<<Blocks(N), 256, 0, st>>>(keys_b, N, g);
      SEED_TRY(hipGetLastError());
      // group starts (inclusive max-scan) into keys_a's storage, free here
      uint32_t *gs = reinterpret_cast<uint32_t *>(keys_a);
      size_t need = 0;
      SEED_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, need, g, gs, MaxOp(), N, st));
      SEED_TRY(ensure_tmp(need));
      SEED_TRY(hipcub::DeviceScan::InclusiveScan(d_tmp, need, g, gs, MaxOp(), N, st));
      SEED_TRY(hipMemsetAsync(d_err + 1, 0, 4, st));
      seed_rank_kernel<<<Blocks(N), 256, 0, st>>>(keys_b, vals_b, gs, dist, N, h, rank, d_err + 1);
      SEED_TRY(hipGetLastError());
      uint32_t unfinished = 0;
      SEED_TRY(hipMemcpyAsync(&unfinished, d_err + 1, 4, hipMemcpyDeviceToHost, st));
      SEED_TRY(hipStreamSynchronize(st));
      if (!unfinished || h >= static_cast<uint32_t>(Lsym)) break;
      if (h >= 0x8000u) return SeedFail(SPM_INTERNAL, "suffix sort did not converge");
      seed_pairkey_kernel<<<Blocks(N), 256, 0, st>>>(vals_b, rank, dist, N, h, keys_a);
      SEED_TRY(hipGetLastError());
      SEED_TRY(sort_pairs(keys_a, keys_b, vals_b, vals_a, N, 64));
      std::swap(vals_a, vals_b);
      h *= 2;
    }
    SA = vals_b;
    // capped LCP + min pyramid + candidate nodes (re-using the sort buffers)
    cap = N;
    key1 = keys_a;
    score = keys_b;
    cpos = rank;
    idx = g;
  }
  SEED_TRY(hipEventRecord(ev[3], st));
  if (const char *e = std::getenv("SPM_HIP_SEED_NODE_CAP"))  // test knob: force the exact-room re-run
    cap = std::min<uint64_t>(cap, std::strtoull(e, nullptr, 10));
  unsigned long long *d_count;
  SEED_TRY(S.Alloc(&d_count, 1));
  SEED_TRY(hipMemsetAsync(d_count, 0, 8, st));
  unsigned long long m = 0;
  auto nodes = [&](auto tag) -> hipError_t {
    using HT = decltype(tag);
    HT *H = nullptr;
    hipError_t e = hipSuccess;
    if (sizeof(HT) == 1 && h_borrow) H = reinterpret_cast<HT *>(h_borrow);
    else if ((e = S.Alloc(&H, N)) != hipSuccess) return e;
    seed_lcp_kernel<HT><<<Blocks(N), 256, 0, st>>>(T, SA, N, o.max_len + 1, H);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    Pyramid<HT> P{};
    P.lv[0] = H;
    P.size[0] = N;
    P.levels = 1;
    while (P.size[P.levels - 1] > 64 && P.levels < kMaxLevels) {
      const uint64_t in_n = P.size[P.levels - 1];
      const uint64_t out_n = (in_n + 63) / 64;
      HT *lv;
      if ((e = S.Alloc(&lv, out_n)) != hipSuccess) return e;
      seed_pyr_kernel<HT><<<Blocks(out_n), 256, 0, st>>>(P.lv[P.levels - 1], in_n, lv, out_n);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      P.lv[P.levels] = lv;
      P.size[P.levels] = out_n;
      ++P.levels;
    }
    seed_nodes_kernel<HT><<<Blocks(N), 256, 0, st>>>(T, SA, P, d_rtab, o, key1, score, cpos, idx, d_count, cap);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&m, d_count, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    if (m <= cap) return hipSuccess;
    // More candidates than the borrowed buffers hold: exact room, again.
    if ((e = S.Alloc(&key1, m)) != hipSuccess || (e = S.Alloc(&score, m)) != hipSuccess ||
        (e = S.Alloc(&cpos, m)) != hipSuccess || (e = S.Alloc(&idx, m)) != hipSuccess)
      return e;
    cap = m;
    if ((e = hipMemsetAsync(d_count, 0, 8, st)) != hipSuccess) return e;
    seed_nodes_kernel<HT><<<Blocks(N), 256, 0, st>>>(T, SA, P, d_rtab, o, key1, score, cpos, idx, d_count, cap);
    return hipGetLastError();
  };
  if (o.max_len + 1 <= 255) SEED_TRY(nodes(uint8_t{}));
  else SEED_TRY(nodes(uint16_t{}));
  SEED_TRY(hipEventRecord(ev[4], st));
  *num_candidates = m;
  const uint64_t take = std::min<uint64_t>(K, m);
  if (take > 0) {
    uint64_t *key1s;
    uint32_t *idx2;
    SEED_TRY(S.Alloc(&key1s, m));
    SEED_TRY(S.Alloc(&key2, m));
    SEED_TRY(S.Alloc(&idx2, m));
    // node index order (R asc, D desc), then stable by score descending.
    SEED_TRY(sort_pairs(key1, key1s, idx, idx2, m, 32 + kDepthBits));
    seed_key2_kernel<<<Blocks(m), 256, 0, st>>>(idx2, score, m, key1s);
    SEED_TRY(hipGetLastError());
    SEED_TRY(sort_pairs(key1s, key2, idx2, idx, m, 48));
    int64_t *os;
    int32_t *ol;
    SEED_TRY(S.Alloc(&os, take));
    SEED_TRY(S.Alloc(&ol, take));
    seed_gather_len_kernel<<<Blocks(take), 256, 0, st>>>(idx, key1, score, take, os, ol);
    SEED_TRY(hipGetLastError());
    std::vector<int32_t> hl(take);
    out_score->resize(take);
    SEED_TRY(hipMemcpyAsync(hl.data(), ol, hl.size() * 4, hipMemcpyDeviceToHost, st));
    SEED_TRY(hipMemcpyAsync(out_score->data(), os, take * 8, hipMemcpyDeviceToHost, st));
    SEED_TRY(hipStreamSynchronize(st));
    std::vector<uint64_t> hoff(take + 1, 0);
    for (uint64_t k = 0; k < take; ++k) hoff[k + 1] = hoff[k] + static_cast<uint64_t>(hl[k]);
    uint64_t *doff;
    uint32_t *oc;
    SEED_TRY(S.Alloc(&doff, take + 1));
    SEED_TRY(S.Alloc(&oc, hoff[take]));
    SEED_TRY(hipMemcpyAsync(doff, hoff.data(), (take + 1) * 8, hipMemcpyHostToDevice, st));
    seed_gather_chars_kernel<<<Blocks(take), 256, 0, st>>>(idx, cpos, T, take, doff, oc);
    SEED_TRY(hipGetLastError());
    std::vector<uint32_t> hc(hoff[take]);
    SEED_TRY(hipMemcpyAsync(hc.data(), oc, hc.size() * 4, hipMemcpyDeviceToHost, st));
    SEED_TRY(hipEventRecord(e1, st));
    SEED_TRY(hipStreamSynchronize(st));
    out->resize(take);
    for (uint64_t k = 0; k < take; ++k) {
      auto &w = (*out)[k];
      w.resize(hl[k]);
      for (int x = 0; x < hl[k]; ++x) w[x] = alphabet[hc[hoff[k] + x] - 1];
    }
  } else {
    SEED_TRY(hipEventRecord(e1, st));
    SEED_TRY(hipStreamSynchronize(st));
  }
  SEED_TRY(hipEventElapsedTime(ms, e0, e1));
  for (int k = 0; k < 5; ++k) SEED_TRY(hipEventElapsedTime(&stages[k], ev[k], ev[k + 1]));
  stages[5] = static_cast<float>(S.alloc_ms);
  stages[6] = static_cast<float>(rounds);
  return SPM_OK;
}

}  // namespace
}  // namespace spm_amd

extern "C" {

static int SeedMineImpl(const uint8_t *sent_bytes, const uint64_t *sent_offsets, uint64_t n,
                        bool on_device, const uint32_t *chars, const int64_t *char_freq,
                        uint64_t num_chars, const spm_hip_seed_options *opt, spm_hip_seeds **out) {
  using namespace spm_amd;
  if (!out || !opt || !sent_offsets || (n && !sent_bytes) || (num_chars && (!chars || !char_freq)))
    return SeedFail(SPM_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  if (n == 0) return SeedFail(SPM_INVALID_ARGUMENT, "no sentences");
  // TrainerSpec range (trainer_interface.cc:74).
  if (opt->max_sentencepiece_length < 1 || opt->max_sentencepiece_length > 512)
    return SeedFail(SPM_OUT_OF_RANGE, "max_sentencepiece_length must be in [1, 512]");
  // Alphabet: the given chars plus the UNK char (rare chars were replaced by
  // it in LoadSentences), rank = position in code point order.
  std::vector<uint32_t> alphabet(chars, chars + num_chars);
  alphabet.push_back(0x2585);
  std::sort(alphabet.begin(), alphabet.end());
  alphabet.erase(std::unique(alphabet.begin(), alphabet.end()), alphabet.end());
  if (!alphabet.empty() && alphabet[0] == 0)
    return SeedFail(SPM_INVALID_ARGUMENT, "NUL in the alphabet");
  for (uint32_t c : alphabet)
    if (c > 0x10FFFF) return SeedFail(SPM_INVALID_ARGUMENT, "code point out of range");
  auto *res = new spm_hip_seeds();
  // Single chars first: Sorted(all_chars) = (freq desc, UTF-8 asc) (:196-198);
  // all_chars excludes the UNK char (:137).
  std::vector<std::pair<std::vector<uint8_t>, int64_t>> cs;
  for (uint64_t i = 0; i < num_chars; ++i) {
    if (chars[i] == 0x2585) continue;
    std::vector<uint8_t> u;
    AppendUTF8(chars[i], &u);
    cs.emplace_back(std::move(u), char_freq[i]);
  }
  std::sort(cs.begin(), cs.end(), [](const auto &a, const auto &b) {
    return a.second > b.second || (a.second == b.second && a.first < b.first);
  });
  for (auto &c : cs) {
    res->bytes.insert(res->bytes.end(), c.first.begin(), c.first.end());
    res->offsets.push_back(res->bytes.size());
    res->raw.push_back(c.second);
  }
  res->num_chars = cs.size();
  const uint64_t limit = opt->seed_sentencepiece_size < 0 ? 0 : uint64_t(opt->seed_sentencepiece_size);
  const uint64_t K = limit > cs.size() ? limit - cs.size() : 0;
  if (K > 0) {
    SeedOpts o{opt->max_sentencepiece_length, opt->split_by_unicode_script != 0,
               opt->split_by_number != 0, opt->split_by_whitespace != 0,
               opt->treat_whitespace_as_suffix != 0};
    std::vector<std::vector<uint32_t>> subs;
    std::vector<int64_t> sc;
    const int rc = MineSubstrings(sent_bytes, sent_offsets, n, on_device, alphabet, o, K, &subs, &sc,
                                  &res->candidates, &res->device_ms, res->stages);
    if (rc != SPM_OK) {
      delete res;
      return rc;
    }
    for (size_t k = 0; k < subs.size(); ++k) {
      for (uint32_t c : subs[k]) AppendUTF8(c, &res->bytes);
      res->offsets.push_back(res->bytes.size());
      res->raw.push_back(sc[k]);
    }
  }
  // ToLogProb (unigram_model_trainer.cc:65-74): float sum, double log, float store.
  float sum = 0.0f;
  for (int64_t v : res->raw) sum += static_cast<float>(v);
  const float logsum = static_cast<float>(std::log(static_cast<double>(sum)));
  res->scores.resize(res->raw.size());
  for (size_t i = 0; i < res->raw.size(); ++i)
    res->scores[i] = static_cast<float>(std::log(static_cast<double>(static_cast<float>(res->raw[i]))) -
                                        static_cast<double>(logsum));
  *out = res;
  return SPM_OK;
}

int spm_hip_seed_mine(const uint8_t *sent_bytes, const uint64_t *sent_offsets, uint64_t n,
                      const uint32_t *chars, const int64_t *char_freq, uint64_t num_chars,
                      const spm_hip_seed_options *opt, spm_hip_seeds **out) {
  return SeedMineImpl(sent_bytes, sent_offsets, n, false, chars, char_freq, num_chars, opt, out);
}

int spm_hip_seed_mine_device(const uint8_t *d_sent_bytes, const uint64_t *d_sent_offsets, uint64_t n,
                             const uint32_t *chars, const int64_t *char_freq, uint64_t num_chars,
                             const spm_hip_seed_options *opt, spm_hip_seeds **out) {
  return SeedMineImpl(d_sent_bytes, d_sent_offsets, n, true, chars, char_freq, num_chars, opt, out);
}

uint64_t spm_hip_seeds_size(const spm_hip_seeds *s) { return s ? s->scores.size() : 0; }
const uint8_t *spm_hip_seeds_bytes(const spm_hip_seeds *s) { return s ? s->bytes.data() : nullptr; }
const uint64_t *spm_hip_seeds_offsets(const spm_hip_seeds *s) { return s ? s->offsets.data() : nullptr; }
const float *spm_hip_seeds_scores(const spm_hip_seeds *s) { return s ? s->scores.data() : nullptr; }
int spm_hip_seeds_stats(const spm_hip_seeds *s, uint64_t *num_chars, uint64_t *candidates,
                        float *device_ms) {
  if (!s) return SPM_INVALID_ARGUMENT;
  if (num_chars) *num_chars = s->num_chars;
  if (candidates) *candidates = s->candidates;
  if (device_ms) *device_ms = s->device_ms;
  return SPM_OK;
}
int spm_hip_seeds_stage_times(const spm_hip_seeds *s, float *ms, uint32_t capacity, uint32_t *count) {
  if (!s || !count || (capacity && !ms)) return SPM_INVALID_ARGUMENT;
  const uint32_t k = capacity < 7 ? capacity : 7;
  for (uint32_t i = 0; i < k; ++i) ms[i] = s->stages[i];
  *count = k;
  return SPM_OK;
}
void spm_hip_seeds_free(spm_hip_seeds *s) { delete s; }
const char *spm_hip_seed_last_error(void) { return spm_amd::g_seed_error.c_str(); }

}  // extern "C"
