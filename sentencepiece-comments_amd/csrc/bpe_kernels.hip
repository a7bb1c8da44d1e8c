// BPE greedy-merge encode for gfx950 (MI355X).
//
// Reference: bpe::Model::Encode (bpe_model.cc:37-199).  The reference pops a
// priority queue of adjacent symbol pairs ordered by (score desc, left index
// asc), skipping stale entries; that is the same as repeatedly merging the
// arg-max over the currently live adjacent pairs.
//
// bpe_lane_kernel — one sentence per LANE (the default for vocabularies of
//   < 32768 pieces): sentences of <= 32 chars and <= 255 bytes, the tile's
//   sentences sorted by length, symbol state in LDS columns ([char][lane],
//   conflict-free for any per-lane index), the live symbols as a 32-bit mask.
//   Per merge a lane scans its pair keys (<= 31 LDS reads), merges the
//   arg-max (smallest left index on ties) and probes its two new neighbour
//   pairs.  A wave then does 64 sentences' merges with the VALU work of one
//   sequential merge each, where the wave-per-sentence kernels below spend a
//   wave-wide reduction and scalar chain per merge of one or two sentences.
// bpe_fast_kernel — one sentence per wavefront, one byte (= one initial
//   symbol for ASCII, one char start otherwise) per lane, symbol state in
//   VGPRs, the live set as a wave-uniform 64-bit mask.  Per merge: a DPP
//   wave max over order-preserving score keys, a ballot for the lowest lane
//   holding it (smallest left index), then the two new neighbour pairs are
//   looked up in the (left id, right id) hash table by two lanes in one
//   divergent probe.  The kernel is VALU-issue bound (one sentence per
//   wave), so the per-merge instruction count is what matters.
//   Covers sentences of <= 64 bytes on models without USER_DEFINED pieces;
//   pushes of UNUSED pieces (which need the rev_merge resegmentation) and
//   chars outside the vocabulary on "irregular" models flag the sentence.
// bpe_general_kernel — the reference algorithm literally, one sentence per
//   lane: symbol list, binary-heap agenda with the same comparator, stale
//   check by size, string lookups by exact-match walks of the concatenated
//   bytes, rev_merge (last push wins) and the recursive resegment.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <type_traits>

#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "bpe_tables.h"
#include "device_common.h"
#include "kernels.h"
#include "lookback.h"
#include "normalizer.h"

namespace spm_amd {
namespace {

constexpr uint64_t kEmptyKey = ~0ull;
constexpr uint8_t kPieceOther = 0, kPieceUserDefined = 1, kPieceUnused = 2;

__device__ __forceinline__ uint32_t OneCharLenB(uint32_t lead) {
  return (0x4322111111111111ull >> ((lead >> 4) * 4)) & 0xFu;
}

// Hash of a (left id << 32 | right id) pair key: 32-bit multiplies only (the
// fast kernel computes it once per merge; 64-bit multiplies cost ~4x the VALU
// issue).  Linear probing at load factor <= 0.5.
__host__ __device__ __forceinline__ uint32_t PairHash(uint64_t k) {
  uint32_t h = static_cast<uint32_t>(k >> 32) * 0x9E3779B1u ^ static_cast<uint32_t>(k) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

struct BpeArgs {
  const uint8_t *__restrict__ bytes;
  const uint64_t *__restrict__ off;
  uint64_t n;
  const uint32_t *__restrict__ units;
  const int32_t *__restrict__ values;     // entry index
  const int32_t *__restrict__ entry_piece;
  const int32_t *__restrict__ entry_out;
  const float *__restrict__ scores;       // per piece id
  const uint8_t *__restrict__ piece_kind;
  const int32_t *__restrict__ piece_out;
  const uint64_t *__restrict__ pair_keys;
  const int32_t *__restrict__ pair_vals;
  const uint4 *__restrict__ pair_ent;     // fused: key, merged id | unused bit, score
  uint64_t pair_mask;
  uint32_t root_base;
  int32_t unk_id;
  int32_t irregular;
  int32_t *__restrict__ slot_ids;
  uint32_t *__restrict__ slot_len;
  uint32_t *__restrict__ ntok;
  uint32_t *__restrict__ flagged;
  uint32_t *__restrict__ status;
  uint64_t capacity;                      // caller's bound on off[n]
  const uint32_t *__restrict__ chain;     // asynchronous chain status (nullable)
  const int16_t *__restrict__ rank_piece; // unique score ranks: rank -> merged piece (lane kernel)
  int32_t rank_base;                      // >= 0: merged piece = rank_base - rank (BpeDevice::rank_base)
  int32_t pipe_probes;                    // lane kernel: new pairs' probes in flight across the next scan
  // bpe_lane_kernel's tile-dense output (lane_ids[off[tile base] + k] for
  // the tile's k-th token in sentence order; lane_len alongside, nullable).
  int32_t *__restrict__ lane_ids;
  uint32_t *__restrict__ lane_len;
};

// ntok[i] of a sentence bpe_lane_kernel encoded: bit 31 set, bits 8-30 the
// tile-local index of its first token, bits 0-7 its token count (<= 32).
constexpr uint32_t kLaneTok = 0x80000000u;

// Nothing to do when an earlier step of an asynchronous chain failed or the
// batch exceeds the caller's capacity (the slots are sized by it): status
// bit 1 makes the compaction skip too.
__device__ __forceinline__ bool BpeSkip(const BpeArgs &a) {
  if ((a.chain && *a.chain) || a.off[a.n] > a.capacity) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&a.status[kStError], 2u);
    return true;
  }
  return false;
}

// Exact-match walk of s[0:len) in the string trie; returns entry or -1.
__device__ __forceinline__ int32_t ExactEntry(const BpeArgs &a, const uint8_t *s, uint32_t len) {
  uint32_t base = a.root_base, node = 0, u = 0;
  for (uint32_t j = 0; j < len; ++j) {
    const uint32_t c = s[j];
    if (c == 0) return -1;
    node = base ^ c;
    u = a.units[node];
    if ((u & 0xFFu) != c) return -1;
    base = u >> 9;
  }
  return (len && (u & 0x100u)) ? a.values[node] : -1;
}

__device__ __forceinline__ int32_t PairLookup(const BpeArgs &a, int32_t l, int32_t r) {
  if (l < 0 || r < 0) return -1;
  const uint64_t key = (static_cast<uint64_t>(static_cast<uint32_t>(l)) << 32) | static_cast<uint32_t>(r);
  uint64_t h = PairHash(key) & a.pair_mask;
  for (;;) {
    const uint64_t k = a.pair_keys[h];
    if (k == key) return a.pair_vals[h];
    if (k == kEmptyKey) return -1;
    h = (h + 1) & a.pair_mask;
  }
}

// One 16-byte load per probe returns the merged id, its score and whether it
// is UNUSED (the fast kernel's per-merge dependent chain is this load alone).
__device__ __forceinline__ int32_t PairLookupFused(const BpeArgs &a, int32_t l, int32_t r, uint32_t *rank,
                                                   bool *unused) {
  if (l < 0 || r < 0) return -1;
  const uint64_t key = (static_cast<uint64_t>(static_cast<uint32_t>(l)) << 32) | static_cast<uint32_t>(r);
  const uint32_t mask = static_cast<uint32_t>(a.pair_mask);  // table < 2^32 entries
  uint32_t h = PairHash(key) & mask;
  for (;;) {
    const uint4 e = a.pair_ent[h];
    if (e.x == static_cast<uint32_t>(r) && e.y == static_cast<uint32_t>(l)) {
      *rank = e.w;
      *unused = (e.z >> 31) != 0;
      return static_cast<int32_t>(e.z & 0x7FFFFFFFu);
    }
    if (e.x == 0xFFFFFFFFu && e.y == 0xFFFFFFFFu) return -1;
    h = (h + 1) & mask;
  }
}

// Pair keys: the entry's w word is the merged piece's score as a dense rank
// (BpeScoreRanks, host side): equal scores share a rank, a higher score has a
// higher rank, 0 = no pair — the same order as the scores themselves, in 16
// bits for vocabularies under 32768 pieces.
// Wave-wide max of a key (all 64 lanes active): DPP within each 16-lane row
// (quad perms, half-row and row mirrors — VALU, no LDS round trip), then the
// four row maxima through v_readlane.
__device__ __forceinline__ uint32_t WaveMaxU(uint32_t v) {
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), 0xB1, 0xF, 0xF, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), 0x4E, 0xF, 0xF, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), 0x141, 0xF, 0xF, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), 0x140, 0xF, 0xF, false)));
  const uint32_t r0 = __builtin_amdgcn_readlane(static_cast<int>(v), 0);
  const uint32_t r1 = __builtin_amdgcn_readlane(static_cast<int>(v), 16);
  const uint32_t r2 = __builtin_amdgcn_readlane(static_cast<int>(v), 32);
  const uint32_t r3 = __builtin_amdgcn_readlane(static_cast<int>(v), 48);
  return max(max(r0, r1), max(r2, r3));
}

__device__ __forceinline__ int32_t ReadLane(int32_t v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

__device__ __forceinline__ void FlagSentence(const BpeArgs &a, uint64_t i, uint32_t nb) {
  a.ntok[i] = 0xFFFFFFFFu;
  const uint32_t k = atomicAdd(&a.status[0], 1u);
  a.flagged[k] = static_cast<uint32_t>(i);
  atomicMax(&a.status[1], nb);
}

// LDS hand-off between the lanes of ONE wavefront (the half kernel's loop
// trip count is per wave, so a block barrier would not be uniform).
__device__ __forceinline__ void WaveSync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// bpe_half_kernel — two sentences per wavefront (lanes 0-31 and 32-63), one
//   CHAR per lane: the merge loop is latency/issue bound per wave, so two
//   sentences per wave nearly halve the cost per sentence.  A half takes its
//   sentence when it has <= 128 bytes and <= 32 chars and the char split by
//   "non-continuation byte" equals the reference's OneCharLen walk
//   (bpe_model.cc:121-131); other sentences go to `rest` for bpe_fast_kernel.
//   Same merge rule as bpe_fast_kernel, with the wave-uniform scalars (L, R,
//   RR, P) kept per half.
__global__ __launch_bounds__(256) void bpe_half_kernel(BpeArgs a, uint32_t *__restrict__ rest,
                                                       uint32_t *__restrict__ rest_count) {
  __shared__ uint32_t lds_w[4][64];  // per wave: each half's first 128 bytes
  __shared__ uint8_t lds_pos[4][64]; // per wave: char start offsets per half
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int hl = lane >> 5, sl = lane & 31;
  const uint64_t hmask = hl ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull;
  if (BpeSkip(a)) return;
  const uint64_t wave = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 6;
  const uint8_t *lb = reinterpret_cast<const uint8_t *>(&lds_w[wv][hl * 32]);
  for (uint64_t pr = wave; 2 * pr < a.n; pr += nwaves) {
    const uint64_t i = 2 * pr + hl;
    const bool has = i < a.n;
    const uint64_t b0 = has ? a.off[i] : 0;
    const uint32_t nb = has ? static_cast<uint32_t>(a.off[i + 1] - b0) : 0;
    const uint8_t *__restrict__ s = a.bytes + b0;
    // Bytes 4sl .. 4sl+3 of the half's sentence.
    uint32_t bw = 0;
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) {
      const uint32_t q = 4 * sl + t;
      if (q < nb && q < 128) bw |= static_cast<uint32_t>(s[q]) << (8 * t);
    }
    lds_w[wv][lane] = bw;
    WaveSync();
    // Char starts = non-continuation bytes; check each start's OneCharLen
    // span against them (so the split equals the reference's walk).
    uint32_t sm = 0;
    bool incons = false;
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) {
      const uint32_t q = 4 * sl + t;
      if (q >= nb || q >= 128) continue;
      const uint32_t b = (bw >> (8 * t)) & 0xFFu;
      if ((b & 0xC0u) == 0x80u) {
        if (q == 0) incons = true;
        continue;
      }
      sm |= 1u << t;
      uint32_t L = OneCharLenB(b);
      if (L > nb - q) L = nb - q;
      for (uint32_t k = 1; k < L; ++k)
        if (q + k >= 128 || (lb[q + k] & 0xC0u) != 0x80u) incons = true;
      if (q + L < nb && q + L < 128 && (lb[q + L] & 0xC0u) == 0x80u) incons = true;
    }
    // Exclusive prefix count of starts within the half.
    const uint32_t c = __popc(sm);
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 32);
      if (sl >= o) x += y;
    }
    const uint32_t nchars = __shfl(x, 31, 32);
    const bool elig_h = has && nb <= 128 && nchars <= 32 && ((__ballot(incons) & hmask) == 0);
    uint32_t rank = x - c;
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t)
      if (((sm >> t) & 1) && elig_h) lds_pos[wv][hl * 32 + rank++] = static_cast<uint8_t>(4 * sl + t);
    WaveSync();
    const bool mine = elig_h && static_cast<uint32_t>(sl) < nchars;
    uint32_t start = 0, len = 0;
    int32_t sym = -1, out = a.unk_id;
    if (mine) {
      start = lds_pos[wv][lane];
      const uint32_t end = static_cast<uint32_t>(sl) + 1 < nchars ? lds_pos[wv][lane + 1] : nb;
      len = end - start;
      const int32_t e = ExactEntry(a, s + start, len);
      if (e >= 0) {
        sym = a.entry_piece[e];
        out = a.entry_out[e];
      }
    }
    bool bad = a.irregular && mine && sym < 0;
    uint64_t alive = __ballot(mine);
    int32_t pres = -1;
    uint32_t pkey = 0;
    {
      const int32_t rsym = __shfl_down(sym, 1, 32);
      if (mine && static_cast<uint32_t>(sl) + 1 < nchars) {
        uint32_t sc = 0u;
        bool unused = false;
        pres = PairLookupFused(a, sym, rsym, &sc, &unused);
        if (pres >= 0) {
          pkey = sc;
          if (unused) bad = true;
        }
      }
    }
    // A half whose sentence already failed does no merges.
    if ((__ballot(bad) & hmask) != 0) pkey = 0;
    for (;;) {
      uint32_t v = pkey;
      v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), 0xB1, 0xF, 0xF, false)));
      v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), 0x4E, 0xF, 0xF, false)));
      v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), 0x141, 0xF, 0xF, false)));
      v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), 0x140, 0xF, 0xF, false)));
      const uint32_t m0 = max(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 0)),
                              static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 16)));
      const uint32_t m1 = max(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 32)),
                              static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 48)));
      if (m0 == 0 && m1 == 0) break;
      const uint64_t cand = __ballot(pkey != 0 && pkey == (hl ? m1 : m0));
      int L[2] = {-1, -1}, R[2] = {-1, -1}, RR[2] = {-1, -1}, P[2] = {-1, -1};
      int32_t merged[2] = {-1, -1}, rrsym[2] = {-1, -1};
      uint32_t rlen[2] = {0, 0};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if ((h ? m1 : m0) == 0) continue;
        const uint64_t hm = h ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull;
        const uint64_t am = alive & hm;
        const int l = __ffsll(static_cast<long long>(cand & hm)) - 1;
        const uint64_t rmask = am & ~((2ull << l) - 1);
        const int r = __ffsll(static_cast<long long>(rmask)) - 1;
        const uint64_t rrmask = r == 63 ? 0 : (am & ~((2ull << r) - 1));
        const uint64_t lmask = am & ((1ull << l) - 1);
        L[h] = l;
        R[h] = r;
        RR[h] = rrmask ? __ffsll(static_cast<long long>(rrmask)) - 1 : -1;
        P[h] = lmask ? 63 - __clzll(static_cast<long long>(lmask)) : -1;
        merged[h] = ReadLane(pres, l);
        rlen[h] = static_cast<uint32_t>(ReadLane(static_cast<int32_t>(len), r));
        rrsym[h] = ReadLane(sym, RR[h] < 0 ? 0 : RR[h]);
        alive &= ~(1ull << r);
      }
      const int hL = L[hl], hR = R[hl], hRR = RR[hl], hP = P[hl];
      const int32_t hmerged = merged[hl];
      if (lane == hR) {
        len = 0;
        pres = -1;
        pkey = 0;
      }
      if (lane == hL) {
        sym = hmerged;
        len += rlen[hl];
      }
      // New pairs (P, L) and (L, RR) of both halves in one divergent probe.
      const bool isP = lane == hP, isL = lane == hL;
      int32_t q = -1;
      uint32_t qs = 0u;
      bool qu = false;
      if (isP || (isL && hRR >= 0)) q = PairLookupFused(a, sym, isP ? hmerged : rrsym[hl], &qs, &qu);
      if (isP || isL) {
        pres = q;
        pkey = q >= 0 ? qs : 0u;
        if (q >= 0 && qu) bad = true;
      }
    }
    const bool bad_h = (__ballot(bad) & hmask) != 0;
    if (!has) continue;
    if (!elig_h) {
      if (sl == 0) rest[atomicAdd(rest_count, 1u)] = static_cast<uint32_t>(i);
      continue;
    }
    if (bad_h) {
      if (sl == 0) FlagSentence(a, i, nb);
      continue;
    }
    const uint32_t nt = __popcll(alive & hmask);
    if ((alive >> lane) & 1) {
      if (sym >= 0) out = a.piece_out[sym];
      const uint32_t j = __popcll(alive & hmask & ((1ull << lane) - 1));
      const uint64_t slot = b0 + nb - nt + j;
      a.slot_ids[slot] = out;
      if (a.slot_len) a.slot_len[slot] = len;
    }
    if (sl == 0) a.ntok[i] = nt;
  }
}

// Two independent fused probes issued together (the merge's new neighbour
// pairs (P, L) and (L, RR)): a miss on either side costs one more round.
__device__ __forceinline__ void PairLookupFused2(const BpeArgs &a, int32_t l0, int32_t r0, bool en0, int32_t l1,
                                                 int32_t r1, bool en1, int32_t *m0, uint32_t *k0, bool *u0,
                                                 int32_t *m1, uint32_t *k1, bool *u1) {
  const uint32_t mask = static_cast<uint32_t>(a.pair_mask);
  bool go0 = en0 && l0 >= 0 && r0 >= 0, go1 = en1 && l1 >= 0 && r1 >= 0;
  uint32_t h0 = go0 ? PairHash((static_cast<uint64_t>(static_cast<uint32_t>(l0)) << 32) | static_cast<uint32_t>(r0)) & mask : 0u;
  uint32_t h1 = go1 ? PairHash((static_cast<uint64_t>(static_cast<uint32_t>(l1)) << 32) | static_cast<uint32_t>(r1)) & mask : 0u;
  *m0 = *m1 = -1;
  *k0 = *k1 = 0u;
  *u0 = *u1 = false;
  while (go0 || go1) {
    uint4 e0 = make_uint4(0u, 0u, 0u, 0u), e1 = make_uint4(0u, 0u, 0u, 0u);
    if (go0) e0 = a.pair_ent[h0];
    if (go1) e1 = a.pair_ent[h1];
    if (go0) {
      if (e0.x == static_cast<uint32_t>(r0) && e0.y == static_cast<uint32_t>(l0)) {
        *m0 = static_cast<int32_t>(e0.z & 0x7FFFFFFFu);
        *k0 = e0.w;
        *u0 = (e0.z >> 31) != 0;
        go0 = false;
      } else if (e0.x == 0xFFFFFFFFu && e0.y == 0xFFFFFFFFu) {
        go0 = false;
      } else {
        h0 = (h0 + 1) & mask;
      }
    }
    if (go1) {
      if (e1.x == static_cast<uint32_t>(r1) && e1.y == static_cast<uint32_t>(l1)) {
        *m1 = static_cast<int32_t>(e1.z & 0x7FFFFFFFu);
        *k1 = e1.w;
        *u1 = (e1.z >> 31) != 0;
        go1 = false;
      } else if (e1.x == 0xFFFFFFFFu && e1.y == 0xFFFFFFFFu) {
        go1 = false;
      } else {
        h1 = (h1 + 1) & mask;
      }
    }
  }
}

constexpr int kLB = 128;         // lanes (sentences) per tile
// Chars per sentence on the lane path: 34 covers the synthetic ~25-char
// sentences' longest (33 chars with the dummy prefix), at 8 tiles per CU
// (LDS 19.9 KB per tile); live-symbol masks are 64-bit.
constexpr int kLaneChars = 34;
static_assert(kLaneChars <= 64, "64-bit live masks, 6-bit column ranks");
constexpr uint32_t kLaneBytes = 255;

// Symbol word of char k: low 16 bits symx (the pieces_ id, or ~PieceToId of
// an unmerged char outside pieces_), high 16 bits the merged id of the pair
// (k, next live symbol) or -1.
__device__ __forceinline__ int32_t SymOf(uint32_t w) { return static_cast<int16_t>(w & 0xFFFFu); }
__device__ __forceinline__ int32_t PresOf(uint32_t w) { return static_cast<int16_t>(w >> 16); }
__device__ __forceinline__ uint32_t SymWord(int32_t sym, int32_t pres) {
  return (static_cast<uint32_t>(sym) & 0xFFFFu) | (static_cast<uint32_t>(pres) << 16);
}

// bpe_lane_kernel: see the header.  Sentences it does not take (> 32 chars or
// > 255 bytes) go to `rest` (bpe_fast_kernel); sentences that push an UNUSED
// piece or hold a char outside an irregular vocabulary are flagged for the
// general kernel.
// kRankIds (models whose pair-merged pieces have distinct scores, e.g. every
// reference-trained BPE model, score = -merge index): a pair's 16-bit score
// rank identifies its merged piece, so the symbol columns keep only the
// 16-bit symbol and the winner's merged id comes from the rank -> piece
// table (one L1-resident load per merge): 17.5 KB of LDS per tile instead of
// 25.5 KB, 9 tiles per CU instead of 6 (4 waves per SIMD instead of 3).
template <bool kRankIds>
__global__ __launch_bounds__(kLB) void bpe_lane_kernel(BpeArgs a, uint32_t *__restrict__ rest,
                                                       uint32_t *__restrict__ rest_count) {
  // 25.5 KB of LDS per 128-lane tile (6 tiles, 3 waves per SIMD): pair keys
  // are 16-bit score ranks, and the chars' byte offsets are re-derived from
  // the sentence at output instead of being stored.
  using SymT = typename std::conditional<kRankIds, uint16_t, uint32_t>::type;
  __shared__ uint16_t lkey[kLaneChars * kLB];  // [k][lane]: rank key of pair (k, next live symbol), 0 = none
  __shared__ SymT lsp[kLaneChars * kLB];       // [k][lane]: SymWord (kRankIds: the symbol only)
  __shared__ uint32_t lds_sort[2 * kLB + 128]; // histogram (256 bins) + permutation
  // (sym, PieceToId) of every one-byte char and of U+2581 (the escaped
  // space, 3 bytes): the char split reads them instead of walking the string
  // trie (three dependent loads per char on the lane's serial chain).
  // Packed as (sym & 0xFFFF) | PieceToId << 16 (both < 2^15 on this path).
  __shared__ uint32_t lds_c1[256];
  __shared__ uint32_t lds_ws;
  if (BpeSkip(a)) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  {
    // Exact-match walk of the bytes of `w` (low byte first, n of them).
    auto entry_packed = [&](uint32_t w, uint32_t n) -> uint32_t {
      uint32_t base = a.root_base, node = 0, u = 0;
      bool ok = true;
      for (uint32_t j = 0; j < n && ok; ++j) {
        const uint32_t c = (w >> (8 * j)) & 0xFFu;
        node = base ^ c;
        u = c ? a.units[node] : 0u;
        ok = c != 0 && (u & 0xFFu) == c;
        base = u >> 9;
      }
      const int32_t e = ok && (u & 0x100u) ? a.values[node] : -1;
      const int32_t sym = e >= 0 ? a.entry_piece[e] : -1;
      const int32_t out = e >= 0 ? a.entry_out[e] : a.unk_id;
      return (static_cast<uint32_t>(sym) & 0xFFFFu) | (static_cast<uint32_t>(out) << 16);
    };
    for (uint32_t c = static_cast<uint32_t>(tid); c < 256; c += kLB) lds_c1[c] = entry_packed(c, 1);
    if (tid == 0) lds_ws = entry_packed(0x8196E2u, 3);
  }  // (the first tile's sort barriers publish the table)
  for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * kLB; base < a.n;
       base += static_cast<uint64_t>(gridDim.x) * kLB) {
    // Counting sort of the tile's sentences by byte length (each wave's lanes
    // then run similar merge counts).
    uint32_t sid;
    {
      uint32_t *hist = lds_sort, *perm = lds_sort + 256;
      const uint64_t ii = base + tid;
      const uint32_t len = ii < a.n ? static_cast<uint32_t>(a.off[ii + 1] - a.off[ii]) : 0u;
      const uint32_t bucket = len < 255u ? len : 255u;
      hist[tid] = 0;
      hist[tid + kLB] = 0;
      __syncthreads();
      const uint32_t r = atomicAdd(&hist[bucket], 1u);
      __syncthreads();
      if (tid < 64) {  // exclusive scan of 256 bins, 4 per lane
        uint32_t v[4], tot = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = hist[lane * 4 + q];
          tot += v[q];
        }
        uint32_t x = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(x, o);
          if (lane >= o) x += y;
        }
        uint32_t run = x - tot;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t c = v[q];
          hist[lane * 4 + q] = run;
          run += c;
        }
      }
      __syncthreads();
      perm[hist[bucket] + r] = static_cast<uint32_t>(tid);
      __syncthreads();
      sid = perm[tid];
    }
    const uint64_t i = base + sid;
    const bool valid = i < a.n;
    const uint64_t b0 = valid ? a.off[i] : 0;
    const uint32_t nb = valid ? static_cast<uint32_t>(a.off[i + 1] - b0) : 0u;
    const uint8_t *__restrict__ s = a.bytes + b0;
    // Char split by OneCharLen clamped to the sentence (bpe_model.cc:121-131
    // via PrefixMatcher with no user-defined symbols), symbols and the
    // initial pairs (k-1, k).
    bool elig = valid && nb <= kLaneBytes, bad = false;
    // The byte window's buffer resource covers at most 0x7FFFFFF0 bytes from
    // the tile's first (aligned) byte: a sentence reaching past it (a tile
    // behind a > 2 GB sentence) would read zeros, so it takes the rest path.
    if (elig && (b0 - (a.off[base] & ~3ull)) + nb + 8 > 0x7FFFFFF0ull) elig = false;
    uint32_t nch = 0;
    uint64_t clen = 0;  // char k's byte length - 1 in bits 2k, 2k + 1 (for the output's offsets)
    uint32_t clen_hi = 0;  // the same for chars 32.. (bits 2(k - 32), ...)
    if (elig) {
      // Char split and symbols; the pairs' lookups follow in a second pass
      // (independent probes, several in flight).  The bytes come through an
      // 8-byte register window of aligned dwords (a buffer resource over the
      // tile's range: loads past the batch read 0), one load per 4 bytes on
      // the lane's serial chain instead of one per byte.
      const uint64_t tb_al = a.off[base] & ~3ull;
      const uint64_t trem = a.off[a.n] - tb_al;
      const auto brs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.bytes + tb_al), 0,
                                                         static_cast<int>(trem < 0x7FFFFFF0ull ? trem : 0x7FFFFFF0ull),
                                                         0x00020000);
      const uint32_t rel0 = static_cast<uint32_t>(b0 - tb_al);
      // (A dword load that straddles num_records reads as 0: the batch's
      // last partial dword comes byte by byte.)
      auto load32 = [&](uint32_t at) -> uint32_t {
        if (at + 4 <= trem) return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(brs, at, 0, 0));
        uint32_t x = 0;
        for (uint32_t t = 0; t < 4; ++t)
          if (at + t < trem) x |= static_cast<uint32_t>(a.bytes[tb_al + at + t]) << (8 * t);
        return x;
      };
      uint32_t wpos = 1, w0 = 0, w1 = 0;  // (not a dword offset: the first access loads)
      for (uint32_t q = 0; q < nb;) {
        if (nch == kLaneChars) {
          elig = false;
          break;
        }
        const uint32_t o = rel0 + q, al = o & ~3u;
        if (al != wpos) {
          w0 = al == wpos + 4 ? w1 : load32(al);
          w1 = load32(al + 4);
          wpos = al;
        }
        const uint32_t w3 = static_cast<uint32_t>(((static_cast<uint64_t>(w1) << 32) | w0) >> (8 * (o & 3u)));
        const uint32_t c0 = w3 & 0xFFu;  // bytes q, q + 1, q + 2 in w3's low bytes
        uint32_t L = OneCharLenB(c0);
        if (L > nb - q) L = nb - q;
        if (nch < 32) clen |= static_cast<uint64_t>(L - 1) << (2 * nch);
        else clen_hi |= static_cast<uint32_t>(L - 1) << (2 * (nch - 32));
        int32_t sym, out;
        if (L == 1 || (L == 3 && (w3 & 0xFFFFFFu) == 0x8196E2u)) {
          const uint32_t so = L == 1 ? lds_c1[c0] : lds_ws;
          sym = static_cast<int16_t>(so & 0xFFFFu);
          out = static_cast<int32_t>(so >> 16);
        } else {
          const int32_t e = ExactEntry(a, s + q, L);
          sym = e >= 0 ? a.entry_piece[e] : -1;
          out = e >= 0 ? a.entry_out[e] : a.unk_id;
        }
        if (a.irregular && sym < 0) bad = true;
        const int32_t symx = sym >= 0 ? sym : ~out;
        lsp[nch * kLB + tid] = kRankIds ? static_cast<SymT>(symx & 0xFFFF) : static_cast<SymT>(SymWord(symx, -1));
        lkey[nch * kLB + tid] = 0u;
        ++nch;
        q += L;
      }
    }
    if (elig) {
      // Pairs (k, k + 1) of in-vocabulary symbols, kPairBatch probes issued
      // together; a probe that meets another key walks on alone.
      constexpr int kPairBatch = 4;
      const uint32_t mask = static_cast<uint32_t>(a.pair_mask);
      int32_t r_next = nch > 0 ? SymOf(static_cast<uint32_t>(lsp[tid])) : -1;
      for (uint32_t k0 = 0; k0 + 1 < nch; k0 += kPairBatch) {
        int32_t l[kPairBatch], r[kPairBatch];
        uint32_t h[kPairBatch];
        uint4 e[kPairBatch];
        StaticFor<0, kPairBatch>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          const uint32_t k = k0 + j;
          l[j] = r_next;
          r[j] = k + 1 < nch ? SymOf(static_cast<uint32_t>(lsp[(k + 1) * kLB + tid])) : -1;
          r_next = r[j];
          const bool need = l[j] >= 0 && r[j] >= 0;
          const uint64_t key = (static_cast<uint64_t>(static_cast<uint32_t>(l[j])) << 32) | static_cast<uint32_t>(r[j]);
          h[j] = PairHash(key) & mask;
          e[j] = need ? a.pair_ent[h[j]] : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);
        });
        StaticFor<0, kPairBatch>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          const uint32_t k = k0 + j;
          if (l[j] < 0 || r[j] < 0) return;
          uint4 x = e[j];
          uint32_t hh = h[j];
          while (!(x.x == static_cast<uint32_t>(r[j]) && x.y == static_cast<uint32_t>(l[j])) &&
                 !(x.x == 0xFFFFFFFFu && x.y == 0xFFFFFFFFu)) {
            hh = (hh + 1) & mask;
            x = a.pair_ent[hh];
          }
          if (x.x == 0xFFFFFFFFu && x.y == 0xFFFFFFFFu) return;
          lkey[k * kLB + tid] = static_cast<uint16_t>(x.w);
          if constexpr (!kRankIds) lsp[k * kLB + tid] = SymWord(SymOf(static_cast<uint32_t>(lsp[k * kLB + tid])),
                                                                static_cast<int32_t>(x.z & 0x7FFFFFFFu));
          if ((x.z >> 31) != 0) bad = true;
        });
      }
    }
    // Columns past the lane's chars hold an earlier tile's keys: zero them
    // once, so the merge scan reads whole groups of columns unconditionally.
    if (elig)
      for (uint32_t k = nch; k < kLaneChars; ++k) lkey[k * kLB + tid] = 0u;
    uint64_t live = nch >= 64 ? ~0ull : ((1ull << nch) - 1ull);
    bool act = elig && !bad && nch > 1;
    if (kRankIds && a.pipe_probes) {
      // The same merges with the two new pairs' probes in flight across the
      // next arg-max scan: a merge zeroes the columns of (P, L) and (L, RR),
      // issues the first-slot loads of both probes and moves on; the next
      // iteration scans the columns from LDS, then resolves the probes (the
      // rare collision walks on), writes their keys and folds them into the
      // arg-max with their own column ranks — the scan's LDS latency hides
      // the probes'.  An UNUSED push is seen before the next merge, as in the
      // unpipelined loop.
      const uint32_t mask = static_cast<uint32_t>(a.pair_mask);
      bool pend = false;
      int qP = -1, qL = 0;
      int32_t l0 = -1, r0 = -1, l1 = -1, r1 = -1;
      uint32_t h0 = 0, h1 = 0;
      uint4 e0 = make_uint4(0u, 0u, 0u, 0u), e1 = e0;
      while (__ballot(act || pend) != 0) {
        uint32_t bm = 0u;
        if (act) {
          uint32_t v[kLaneChars];
#pragma unroll
          for (int q = 0; q < kLaneChars; ++q) v[q] = lkey[q * kLB + tid];
#pragma unroll
          for (int q = 0; q < kLaneChars; ++q) bm = max(bm, (v[q] << 6) | static_cast<uint32_t>(63 - q));
        }
        if (pend) {
          auto resolve = [&](int32_t l, int32_t r, uint32_t h, uint4 e, uint32_t *key, bool *unused) {
            *key = 0u;
            *unused = false;
            if (l < 0 || r < 0) return;
            while (!(e.x == static_cast<uint32_t>(r) && e.y == static_cast<uint32_t>(l))) {
              if (e.x == 0xFFFFFFFFu && e.y == 0xFFFFFFFFu) return;
              h = (h + 1) & mask;
              e = a.pair_ent[h];
            }
            *key = e.w;
            *unused = (e.z >> 31) != 0;
          };
          uint32_t kP, kL;
          bool uP, uL;
          resolve(l0, r0, h0, e0, &kP, &uP);
          resolve(l1, r1, h1, e1, &kL, &uL);
          if (qP >= 0) {
            lkey[qP * kLB + tid] = static_cast<uint16_t>(kP);
            bm = max(bm, (kP << 6) | static_cast<uint32_t>(63 - qP));
          }
          lkey[qL * kLB + tid] = static_cast<uint16_t>(kL);
          bm = max(bm, (kL << 6) | static_cast<uint32_t>(63 - qL));
          if (uP || uL) {
            bad = true;
            act = false;
          }
          pend = false;
        }
        if (act) {
          const uint32_t best = bm >> 6;
          const int Lk = 63 - static_cast<int>(bm & 63u);
          if (best == 0u) {
            act = false;
          } else {
            const uint64_t above = live & ~((2ull << Lk) - 1ull);
            const int Rk = __builtin_ctzll(above);
            const uint64_t above_r = Rk == 63 ? 0ull : (live & ~((2ull << Rk) - 1ull));
            const int RRk = above_r ? __builtin_ctzll(above_r) : -1;
            const uint64_t below = live & ((1ull << Lk) - 1ull);
            const int Pk = below ? 63 - __builtin_clzll(below) : -1;
            const int32_t merged = a.rank_base >= 0 ? a.rank_base - static_cast<int32_t>(best)
                                                    : static_cast<int32_t>(a.rank_piece[best]);
            live &= ~(1ull << Rk);
            lkey[Rk * kLB + tid] = 0;
            l0 = Pk >= 0 ? SymOf(static_cast<uint32_t>(lsp[Pk * kLB + tid])) : -1;
            r0 = merged;
            l1 = merged;
            r1 = RRk >= 0 ? SymOf(static_cast<uint32_t>(lsp[RRk * kLB + tid])) : -1;
            lsp[Lk * kLB + tid] = static_cast<SymT>(merged & 0xFFFF);
            if (Pk >= 0) lkey[Pk * kLB + tid] = 0;
            lkey[Lk * kLB + tid] = 0;
            h0 = l0 >= 0 ? PairHash((static_cast<uint64_t>(static_cast<uint32_t>(l0)) << 32) | static_cast<uint32_t>(r0)) & mask : 0u;
            h1 = r1 >= 0 ? PairHash((static_cast<uint64_t>(static_cast<uint32_t>(l1)) << 32) | static_cast<uint32_t>(r1)) & mask : 0u;
            e0 = l0 >= 0 ? a.pair_ent[h0] : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);
            e1 = r1 >= 0 ? a.pair_ent[h1] : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);
            qP = Pk;
            qL = Lk;
            pend = true;
          }
        }
      }
    }
    while (!(kRankIds && a.pipe_probes) && __ballot(act) != 0) {
      if (act) {
        // Arg-max of the pair keys, smallest column on ties: one max over
        // (key << 6 | 63 - k), every column's load issued before the first
        // max (columns past a lane's chars are zero).  (Loading only the
        // 8-column groups up to the wave's longest list measured the same.)
        uint32_t bm = 0u;
        {
          uint32_t v[kLaneChars];
#pragma unroll
          for (int q = 0; q < kLaneChars; ++q) v[q] = lkey[q * kLB + tid];
#pragma unroll
          for (int q = 0; q < kLaneChars; ++q) bm = max(bm, (v[q] << 6) | static_cast<uint32_t>(63 - q));
        }
        const uint32_t best = bm >> 6;
        const int bk = 63 - static_cast<int>(bm & 63u);
        if (best == 0u) {
          act = false;
        } else {
          const int Lk = bk;
          const uint64_t above = live & ~((2ull << Lk) - 1ull);
          const int Rk = __builtin_ctzll(above);
          const uint64_t above_r = Rk == 63 ? 0ull : (live & ~((2ull << Rk) - 1ull));
          const int RRk = above_r ? __builtin_ctzll(above_r) : -1;
          const uint64_t below = live & ((1ull << Lk) - 1ull);
          const int Pk = below ? 63 - __builtin_clzll(below) : -1;
          const int32_t merged = !kRankIds        ? PresOf(lsp[Lk * kLB + tid])
                                 : a.rank_base >= 0 ? a.rank_base - static_cast<int32_t>(best)
                                                    : static_cast<int32_t>(a.rank_piece[best]);
          live &= ~(1ull << Rk);
          lkey[Rk * kLB + tid] = 0;
          // New pairs (P, L) and (L, RR) — the reference's push order.
          const uint32_t wP = Pk >= 0 ? static_cast<uint32_t>(lsp[Pk * kLB + tid]) : 0u;
          const int32_t symRR = RRk >= 0 ? SymOf(static_cast<uint32_t>(lsp[RRk * kLB + tid])) : -1;
          int32_t mP, mL;
          uint32_t kP, kL;
          bool uP, uL;
          PairLookupFused2(a, SymOf(wP), merged, Pk >= 0, merged, symRR, RRk >= 0, &mP, &kP, &uP, &mL, &kL, &uL);
          if (Pk >= 0) {
            lkey[Pk * kLB + tid] = static_cast<uint16_t>(mP >= 0 ? kP : 0u);
            if constexpr (!kRankIds) lsp[Pk * kLB + tid] = SymWord(SymOf(wP), mP);
          }
          lkey[Lk * kLB + tid] = static_cast<uint16_t>(mL >= 0 ? kL : 0u);
          lsp[Lk * kLB + tid] = kRankIds ? static_cast<SymT>(merged & 0xFFFF) : static_cast<SymT>(SymWord(merged, mL));
          if ((mP >= 0 && uP) || (mL >= 0 && uL)) {
            bad = true;
            act = false;
          }
        }
      }
    }
    // Output, staged in LDS: the tile's tokens in sentence order, one dense
    // run per tile written with coalesced stores (written straight from each
    // lane, 64 lanes' stores scattered over 64 sentences' slot ranges cost
    // ~4.7x the output bytes in HBM writes, profiles/r04final_prof_pmc_bpe_lane.json).
    // The pair-key columns (dead after the merges) hold the ids, the sort
    // table the piece lengths; tokens past the staging room go straight out.
    const bool mine = valid && elig && !bad;
    const uint32_t nt = mine && nch ? static_cast<uint32_t>(__popcll(live)) : 0u;
    uint32_t *const lcnt = lds_sort;  // [sid]: token count, then tile-local offset
    uint32_t *const stage_id = reinterpret_cast<uint32_t *>(lkey);
    uint8_t *const stage_len = reinterpret_cast<uint8_t *>(lds_sort + kLB + 4);  // (after lcnt[0..kLB])
    const uint32_t stage_cap = a.lane_len ? static_cast<uint32_t>((2 * kLB + 128 - kLB - 4) * 4)
                                          : static_cast<uint32_t>(kLaneChars * kLB / 2);
    __syncthreads();  // every lane's merges done: lkey / lds_sort are free
    lcnt[sid] = nt;
    __syncthreads();
    {
      const uint32_t v = lcnt[tid];
      uint32_t x = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
      }
      __shared__ uint32_t s_w0;
      if (tid == 63) s_w0 = x;
      __syncthreads();
      lcnt[tid] = x - v + (tid >= 64 ? s_w0 : 0u);
      if (tid == kLB - 1) lcnt[kLB] = x + s_w0;  // the tile's token count
    }
    __syncthreads();
    const uint32_t lp = lcnt[sid];
    const uint64_t tile_off = a.off[base];
    if (valid) {
      if (!elig) {
        rest[atomicAdd(rest_count, 1u)] = static_cast<uint32_t>(i);
      } else if (bad) {
        FlagSentence(a, i, nb);
      } else {
        uint32_t j = 0;
        auto emit = [&](int k, uint32_t beg, uint32_t end) {
          const int32_t symx = SymOf(static_cast<uint32_t>(lsp[k * kLB + tid]));
          const int32_t id = symx >= 0 ? a.piece_out[symx] : ~symx;
          const uint32_t li = lp + j;
          if (li < stage_cap) {
            stage_id[li] = static_cast<uint32_t>(id);
            if (a.lane_len) stage_len[li] = static_cast<uint8_t>(end - beg);
          } else {
            a.lane_ids[tile_off + li] = id;
            if (a.lane_len) a.lane_len[tile_off + li] = end - beg;
          }
          ++j;
        };
        // Byte offsets of the live symbols: the char split's lengths.
        int pk = -1;
        uint32_t pbeg = 0, q = 0;
        for (uint32_t k = 0; k < nch; ++k) {
          if ((live >> k) & 1ull) {
            if (pk >= 0) emit(pk, pbeg, q);
            pk = static_cast<int>(k);
            pbeg = q;
          }
          q += static_cast<uint32_t>(k < 32 ? (clen >> (2 * k)) & 3u : (clen_hi >> (2 * (k - 32))) & 3u) + 1u;
        }
        if (pk >= 0) emit(pk, pbeg, nb);
        a.ntok[i] = kLaneTok | lp << 8 | nt;
      }
    }
    __syncthreads();
    {
      const uint32_t tot = lcnt[kLB];
      const uint32_t m = tot < stage_cap ? tot : stage_cap;
      for (uint32_t t = static_cast<uint32_t>(tid); t < m; t += kLB) {
        a.lane_ids[tile_off + t] = static_cast<int32_t>(stage_id[t]);
        if (a.lane_len) a.lane_len[tile_off + t] = stage_len[t];
      }
    }
    __syncthreads();  // the next tile reuses the LDS columns
  }
}

// One sentence per wavefront, over the sentences the half kernel left in
// `list` (or every sentence when list == nullptr).
__global__ __launch_bounds__(256) void bpe_fast_kernel(BpeArgs a, const uint32_t *__restrict__ list,
                                                       const uint32_t *__restrict__ list_count) {
  const int lane = threadIdx.x & 63;
  if (BpeSkip(a)) return;
  const uint64_t wave = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 6;
  const uint64_t count = list ? *list_count : a.n;
  for (uint64_t jl = wave; jl < count; jl += nwaves) {
    const uint64_t i = list ? list[jl] : jl;
    const uint64_t b0 = a.off[i];
    const uint32_t nb = static_cast<uint32_t>(a.off[i + 1] - b0);
    if (nb == 0) {
      if (lane == 0) a.ntok[i] = 0;
      continue;
    }
    if (nb > 64) {
      if (lane == 0) FlagSentence(a, i, nb);
      continue;
    }
    const uint8_t *__restrict__ s = a.bytes + b0;
    const uint32_t byte = lane < static_cast<int>(nb) ? s[lane] : 0u;
    // Char starts: split by OneCharLen (bpe_model.cc:121-131 via
    // PrefixMatcher::PrefixMatch with no user-defined symbols).
    uint64_t starts;
    const uint64_t ascii = __ballot(lane < static_cast<int>(nb) && byte < 0x80u);
    const uint64_t valid = nb == 64 ? ~0ull : ((1ull << nb) - 1);
    if (ascii == valid) {
      starts = valid;
    } else {
      const uint32_t cl = OneCharLenB(byte);
      starts = 0;
      for (uint32_t p = 0; p < nb;) {
        starts |= 1ull << p;
        const uint32_t l = __shfl(cl, static_cast<int>(p));
        p += l < nb - p ? l : nb - p;
      }
    }
    const bool is_start = (starts >> lane) & 1;
    // Byte length of this lane's symbol: distance to the next start.
    const uint64_t above = lane == 63 ? 0 : (starts & ~((2ull << lane) - 1));
    uint32_t len = is_start ? (above ? (__ffsll(static_cast<long long>(above)) - 1 - lane) : (nb - lane)) : 0;
    // Symbol id (pieces_ id) and PieceToId of a single char.
    int32_t sym = -1, out = a.unk_id;
    if (is_start) {
      const int32_t e = ExactEntry(a, s + lane, len);
      if (e >= 0) {
        sym = a.entry_piece[e];
        out = a.entry_out[e];
      }
    }
    bool bad = a.irregular && __any(is_start && sym < 0);
    uint64_t alive = starts;
    // Pair (this symbol, next live symbol).
    int32_t pres = -1;
    uint32_t psc = 0u;
    uint32_t pkey = 0;  // rank key of this lane's pair, 0 = none
    {
      const int nxt = above ? (__ffsll(static_cast<long long>(above)) - 1) : -1;
      const int32_t rsym = __shfl(sym, nxt < 0 ? 0 : nxt);
      if (is_start && nxt >= 0) {
        bool unused = false;
        pres = PairLookupFused(a, sym, rsym, &psc, &unused);
        if (pres >= 0 && unused) bad = true;
        if (pres >= 0) pkey = psc;
      }
    }
    bad = __any(bad);
    // Merges until no adjacent pair is in the vocabulary.  A pushed UNUSED
    // piece only flags the sentence (checked once after the loop: merging on
    // is harmless, the general kernel redoes the sentence).
    // (bad is wave-uniform here; inside the loop it becomes per-lane and must
    // not steer the loop, which has to stay convergent for the DPP max.)
    const bool skip = bad;
    while (!skip) {
      const uint32_t m = WaveMaxU(pkey);
      if (m == 0) break;
      const uint64_t cand = __ballot(pkey == m);
      const int L = __ffsll(static_cast<long long>(cand)) - 1;
      const uint64_t rmask = alive & ~((2ull << L) - 1);
      const int R = __ffsll(static_cast<long long>(rmask)) - 1;
      const uint64_t rrmask = R == 63 ? 0 : (alive & ~((2ull << R) - 1));
      const int RR = rrmask ? __ffsll(static_cast<long long>(rrmask)) - 1 : -1;
      const uint64_t lmask = alive & ((1ull << L) - 1);
      const int P = lmask ? 63 - __clzll(static_cast<long long>(lmask)) : -1;
      // L, R, RR are wave-uniform: v_readlane, not an LDS permute.
      const int32_t merged = ReadLane(pres, L);
      const uint32_t rlen = static_cast<uint32_t>(ReadLane(static_cast<int32_t>(len), R));
      const int32_t rrsym = ReadLane(sym, RR < 0 ? 0 : RR);
      alive &= ~(1ull << R);
      if (lane == R) {
        len = 0;
        pres = -1;
        pkey = 0;
      }
      if (lane == L) {
        sym = merged;
        len += rlen;
      }
      // New pairs: (P, L) then (L, RR) — the reference's push order.  Both
      // probes run in one divergent call (lanes P and L), so the lookup code
      // is issued once per merge.
      int32_t q = -1;
      uint32_t qs = 0u;
      bool qu = false;
      if (lane == P || (lane == L && RR >= 0)) q = PairLookupFused(a, sym, lane == P ? merged : rrsym, &qs, &qu);
      if (lane == P || lane == L) {
        pres = q;
        pkey = q >= 0 ? qs : 0u;
        if (q >= 0 && qu) bad = true;
      }
    }
    bad = __any(bad);
    if (bad) {
      if (lane == 0) FlagSentence(a, i, nb);
      continue;
    }
    const uint32_t nt = __popcll(alive);
    if ((alive >> lane) & 1) {
      // PieceToId of the final symbol (= entry_out of an unmerged char).
      if (sym >= 0) out = a.piece_out[sym];
      const uint32_t j = __popcll(alive & ((1ull << lane) - 1));
      const uint64_t slot = b0 + nb - nt + j;
      a.slot_ids[slot] = out;
      if (a.slot_len) a.slot_len[slot] = len;
    }
    if (lane == 0) a.ntok[i] = nt;
  }
}

// ---------------------------------------------------------------------------
// General kernel: the reference, literally, one sentence per lane.
// ---------------------------------------------------------------------------
struct PairRec {
  int32_t left, right;
  float score;
  uint32_t size;
};

struct GenBpeArgs {
  BpeArgs a;
  const uint32_t *__restrict__ list;
  const uint32_t *__restrict__ count;
  uint64_t list_n;
  uint8_t *__restrict__ scratch;
  uint64_t slab_bytes;
  uint32_t max_nb;
  uint32_t *__restrict__ error;
  int32_t has_user_defined;
  uint32_t *__restrict__ ovf_list;    // sentences longer than max_nb (nullptr: error)
  uint32_t *__restrict__ ovf_count;
  uint32_t lanes;                     // slabs in scratch
};

// comparator of bpe_model.cc:55-61: true if h1 has LOWER priority than h2.
__device__ __forceinline__ bool Lower(const PairRec &h1, const PairRec &h2) {
  return h1.score < h2.score || (h1.score == h2.score && h1.left > h2.left);
}

__global__ __launch_bounds__(64) void bpe_general_kernel(GenBpeArgs g) {
  const BpeArgs &a = g.a;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (tid >= g.lanes || BpeSkip(a)) return;
  const uint64_t nthreads = g.lanes;
  const uint64_t total = g.count ? *g.count : g.list_n;
  for (uint64_t j = tid; j < total; j += nthreads) {
    const uint32_t i = g.list ? g.list[j] : static_cast<uint32_t>(j);
    const uint64_t b0 = a.off[i];
    const uint32_t nb = static_cast<uint32_t>(a.off[i + 1] - b0);
    if (nb == 0) {
      a.ntok[i] = 0;
      continue;
    }
    if (nb > g.max_nb) {
      if (g.ovf_list) {
        g.ovf_list[atomicAdd(g.ovf_count, 1u)] = i;
      } else {
        atomicOr(g.error, 1u);
        a.ntok[i] = 0;
      }
      continue;
    }
    const uint8_t *__restrict__ s = a.bytes + b0;
    uint8_t *slab = g.scratch + tid * g.slab_bytes;
    uint32_t *soff = reinterpret_cast<uint32_t *>(slab);
    uint32_t *slen = soff + nb;
    int32_t *sprev = reinterpret_cast<int32_t *>(slen + nb);
    int32_t *snext = sprev + nb;
    uint32_t *sfrz = reinterpret_cast<uint32_t *>(snext + nb);
    PairRec *pool = reinterpret_cast<PairRec *>(sfrz + nb);
    const uint32_t cap = 3 * nb + 4;
    int32_t *heap = reinterpret_cast<int32_t *>(pool + cap);
    int32_t *rev_piece = heap + cap;
    uint32_t *rev_left = reinterpret_cast<uint32_t *>(rev_piece + cap);
    uint32_t *stk = rev_left + cap;  // (off, len) pairs, 2*nb entries each
    int32_t npool = 0, nheap = 0, nrev = 0;

    auto heap_push = [&](int32_t r) {
      int32_t c = nheap++;
      heap[c] = r;
      while (c > 0) {
        const int32_t p = (c - 1) >> 1;
        if (!Lower(pool[heap[p]], pool[heap[c]])) break;
        const int32_t t = heap[p];
        heap[p] = heap[c];
        heap[c] = t;
        c = p;
      }
    };
    auto heap_pop = [&]() -> int32_t {
      const int32_t top = heap[0];
      heap[0] = heap[--nheap];
      int32_t c = 0;
      for (;;) {
        const int32_t l = 2 * c + 1, r = l + 1;
        int32_t m = c;
        if (l < nheap && Lower(pool[heap[m]], pool[heap[l]])) m = l;
        if (r < nheap && Lower(pool[heap[m]], pool[heap[r]])) m = r;
        if (m == c) break;
        const int32_t t = heap[m];
        heap[m] = heap[c];
        heap[c] = t;
        c = m;
      }
      return top;
    };
    // MaybeAddNewSymbolPair (bpe_model.cc:94-115).
    auto maybe_add = [&](int32_t left, int32_t right) {
      if (left < 0 || right < 0 || sfrz[left] || sfrz[right]) return;
      const uint32_t sz = slen[left] + slen[right];
      const int32_t e = ExactEntry(a, s + soff[left], sz);
      const int32_t pid = e >= 0 ? a.entry_piece[e] : -1;
      if (pid < 0) return;
      const int32_t r = npool++;
      pool[r] = PairRec{left, right, a.scores[pid], sz};
      heap_push(r);
      if (a.piece_kind[pid] == kPieceUnused) {
        rev_piece[nrev] = pid;
        rev_left[nrev] = slen[left];
        ++nrev;
      }
    };
    // Split into symbols (bpe_model.cc:121-131).
    int32_t ns = 0;
    for (uint32_t q = 0; q < nb;) {
      uint32_t mblen = OneCharLenB(s[q]);
      if (mblen > nb - q) mblen = nb - q;
      bool frozen = false;
      if (g.has_user_defined) {
        // PrefixMatcher::PrefixMatch: longest user-defined symbol.
        uint32_t base = a.root_base, best = 0;
        for (uint32_t t = q; t < nb; ++t) {
          const uint32_t c = s[t];
          if (c == 0) break;
          const uint32_t node = base ^ c;
          const uint32_t u = a.units[node];
          if ((u & 0xFFu) != c) break;
          base = u >> 9;
          if (u & 0x100u) {
            const int32_t pid = a.entry_piece[a.values[node]];
            if (pid >= 0 && a.piece_kind[pid] == kPieceUserDefined) best = t + 1 - q;
          }
        }
        if (best) {
          mblen = best;
          frozen = true;
        }
      }
      soff[ns] = q;
      slen[ns] = mblen;
      sfrz[ns] = frozen;
      sprev[ns] = ns - 1;
      q += mblen;
      snext[ns] = q >= nb ? -1 : ns + 1;
      ++ns;
    }
    for (int32_t k = 1; k < ns; ++k) maybe_add(k - 1, k);
    while (nheap > 0) {
      const PairRec top = pool[heap_pop()];
      if (slen[top.left] == 0 || slen[top.right] == 0 ||
          slen[top.left] + slen[top.right] != top.size)
        continue;
      slen[top.left] += slen[top.right];
      snext[top.left] = snext[top.right];
      if (snext[top.right] >= 0) sprev[snext[top.right]] = top.left;
      slen[top.right] = 0;
      maybe_add(sprev[top.left], top.left);
      maybe_add(top.left, snext[top.left]);
    }
    // Resegment (bpe_model.cc:171-196), iterative, writing left-aligned.
    int32_t *__restrict__ out_id = a.slot_ids + b0;
    uint32_t *__restrict__ out_len = a.slot_len ? a.slot_len + b0 : nullptr;
    uint32_t k = 0;
    for (int32_t idx = 0; idx != -1; idx = snext[idx]) {
      int32_t sp = 0;
      stk[0] = soff[idx];
      stk[1] = slen[idx];
      sp = 1;
      while (sp > 0) {
        --sp;
        const uint32_t wo = stk[2 * sp], wl = stk[2 * sp + 1];
        const int32_t e = ExactEntry(a, s + wo, wl);
        const int32_t id = e >= 0 ? a.entry_out[e] : a.unk_id;  // PieceToId
        int32_t split = -1;
        if (id >= 0 && a.piece_kind[id] == kPieceUnused && e >= 0 && a.entry_piece[e] == id) {
          for (int32_t t = nrev - 1; t >= 0; --t)
            if (rev_piece[t] == id) {
              split = static_cast<int32_t>(rev_left[t]);
              break;
            }
        }
        if (split < 0) {
          out_id[k] = id;
          if (out_len) out_len[k] = wl;
          ++k;
        } else {
          // push right then left so left is processed first
          stk[2 * sp] = wo + split;
          stk[2 * sp + 1] = wl - split;
          ++sp;
          stk[2 * sp] = wo;
          stk[2 * sp + 1] = split;
          ++sp;
        }
      }
    }
    // Move to the right-aligned layout the compaction expects.
    if (k < nb) {
      for (int64_t t = static_cast<int64_t>(k) - 1; t >= 0; --t) {
        out_id[nb - k + t] = out_id[t];
        if (out_len) out_len[nb - k + t] = out_len[t];
      }
    }
    a.ntok[i] = k;
  }
}

uint64_t BpeGeneralSlabBytes(uint32_t max_nb) {
  const uint64_t nb = max_nb;
  const uint64_t cap = 3 * nb + 4;
  return nb * 20 + cap * sizeof(PairRec) + cap * 12 + nb * 16 + 64;
}

}  // namespace

int LoadBpe(spm_hip_model *m, std::string *err) {
  const auto &pieces = m->proto.pieces;
  // String entries: pieces_ ∪ reserved_id_map_.
  std::unordered_map<std::string, int32_t> entry_of;
  std::vector<int32_t> entry_piece, entry_out;
  auto entry = [&](const std::string &s) -> int32_t {
    auto it = entry_of.find(s);
    if (it != entry_of.end()) return it->second;
    const int32_t e = static_cast<int32_t>(entry_piece.size());
    entry_of.emplace(s, e);
    entry_piece.push_back(-1);
    entry_out.push_back(m->unk_id);
    return e;
  };
  for (const auto &kv : m->pieces) entry_piece[entry(kv.first)] = kv.second;
  for (const auto &kv : m->reserved) entry(kv.first);
  for (const auto &kv : entry_of) {
    auto r = m->reserved.find(kv.first);
    if (r != m->reserved.end()) entry_out[kv.second] = r->second;
    else entry_out[kv.second] = entry_piece[kv.second];
  }
  std::vector<std::pair<std::string, int32_t>> keys(entry_of.begin(), entry_of.end());
  if (!BuildDoubleArray(std::move(keys), &m->trie, err)) return SPM_RESOURCE_EXHAUSTED;
  // Per piece tables.
  const size_t V = pieces.size();
  std::vector<float> scores(V);
  std::vector<uint8_t> kind(V, kPieceOther);
  std::vector<int32_t> piece_out(V, m->unk_id);
  for (size_t i = 0; i < V; ++i) {
    scores[i] = pieces[i].score;
    if (pieces[i].type == kUserDefined) kind[i] = kPieceUserDefined;
    if (pieces[i].type == kUnused) kind[i] = kPieceUnused;
  }
  for (const auto &kv : m->pieces) {
    auto r = m->reserved.find(kv.first);
    piece_out[kv.second] = r != m->reserved.end() ? r->second : kv.second;
  }
  // Pair table over char-boundary splits P = X · Y with X, Y in pieces_.
  std::vector<std::pair<uint64_t, int32_t>> pairs;
  bool irregular = false;
  for (const auto &kv : m->pieces) {
    const std::string &p = kv.first;
    std::vector<size_t> cuts;
    for (size_t q = 0; q < p.size();) {
      q += std::min<size_t>(OneCharLen(static_cast<uint8_t>(p[q])), p.size() - q);
      if (q < p.size()) cuts.push_back(q);
    }
    for (size_t c : cuts) {
      const std::string x = p.substr(0, c), y = p.substr(c);
      auto ix = m->pieces.find(x), iy = m->pieces.find(y);
      const bool xc = ix == m->pieces.end() &&
                      OneCharLen(static_cast<uint8_t>(x[0])) >= x.size();
      const bool yc = iy == m->pieces.end() &&
                      OneCharLen(static_cast<uint8_t>(y[0])) >= y.size();
      if (ix != m->pieces.end() && iy != m->pieces.end())
        pairs.emplace_back((static_cast<uint64_t>(static_cast<uint32_t>(ix->second)) << 32) |
                               static_cast<uint32_t>(iy->second),
                           kv.second);
      else if ((xc && (iy != m->pieces.end() || yc)) || (yc && ix != m->pieces.end()))
        irregular = true;
    }
  }
  uint64_t cap = 1024;
  while (cap < pairs.size() * 2 + 16) cap <<= 1;
  std::vector<uint64_t> hk(cap, kEmptyKey);
  std::vector<int32_t> hv(cap, -1);
  for (const auto &pr : pairs) {
    uint64_t h = PairHash(pr.first) & (cap - 1);
    while (hk[h] != kEmptyKey && hk[h] != pr.first) h = (h + 1) & (cap - 1);
    hk[h] = pr.first;
    hv[h] = pr.second;
  }
  // Fused entries (kernel probes read one uint4): the w word is the merged
  // piece's dense score rank.  Keys compare as the scores do: the order-
  // preserving bit key of score + 0.0f (-0.0 == +0.0; the all-ones NaN key 0
  // stays 0, "no pair"), then distinct keys numbered from 1 upwards.
  std::vector<uint32_t> rank(V, 0);
  {
    std::vector<uint32_t> bits(V);
    for (size_t v = 0; v < V; ++v) {
      uint32_t b;
      const float x = scores[v] + 0.0f;
      std::memcpy(&b, &x, 4);
      bits[v] = b ^ ((b >> 31) ? 0xFFFFFFFFu : 0x80000000u);
    }
    std::vector<uint32_t> d(bits);
    std::sort(d.begin(), d.end());
    d.erase(std::unique(d.begin(), d.end()), d.end());
    if (!d.empty() && d[0] == 0u) d.erase(d.begin());
    for (size_t v = 0; v < V; ++v)
      rank[v] = bits[v] == 0u ? 0u
                              : static_cast<uint32_t>(std::lower_bound(d.begin(), d.end(), bits[v]) - d.begin()) + 1u;
  }
  // Distinct ranks among the pieces a pair merges into: the rank then names
  // the merged piece (bpe_lane_kernel<true>'s rank -> piece table).
  std::vector<int16_t> rank_piece;
  {
    std::vector<int32_t> rp(V + 2, -1);
    bool unique = V <= 32767;
    for (size_t h = 0; h < cap && unique; ++h) {
      if (hk[h] == kEmptyKey) continue;
      const int32_t v = hv[h];
      const uint32_t r = rank[v];
      if (r == 0 || r > V + 1) unique = false;
      else if (rp[r] == -1) rp[r] = v;
      else if (rp[r] != v) unique = false;
    }
    if (unique) rank_piece.assign(rp.begin(), rp.end());
    m->bpe.rank_base = -1;
    if (unique) {
      int64_t c = -1;
      bool affine = true;
      for (size_t r = 0; r < rp.size() && affine; ++r) {
        if (rp[r] < 0) continue;
        const int64_t cr = static_cast<int64_t>(rp[r]) + static_cast<int64_t>(r);
        if (c < 0) c = cr;
        else if (cr != c) affine = false;
      }
      if (affine && c >= 0 && c < (1 << 30)) m->bpe.rank_base = static_cast<int32_t>(c);
    }
  }
  std::vector<uint32_t> he(cap * 4, 0xFFFFFFFFu);
  for (uint64_t h = 0; h < cap; ++h) {
    if (hk[h] == kEmptyKey) continue;
    he[4 * h + 0] = static_cast<uint32_t>(hk[h]);
    he[4 * h + 1] = static_cast<uint32_t>(hk[h] >> 32);
    const int32_t v = hv[h];
    he[4 * h + 2] = static_cast<uint32_t>(v) | (kind[v] == kPieceUnused ? 0x80000000u : 0u);
    he[4 * h + 3] = rank[v];
  }
  m->bpe.pair_mask = cap - 1;
  m->bpe.irregular = irregular;
  m->bpe.has_user_defined = !m->user_defined.empty();
  // bpe_lane_kernel keeps symbol and merged ids as int16 (PieceToId values
  // and the unk id are < V as well).
  m->bpe.lane_ok = V <= 32767;
  m->bpe.rank_ids = !rank_piece.empty();
  m->max_piece_chars = 0;
  m->up.root_base = DoubleArray::Base(m->trie.units[0]);
  m->up.unk_id = m->unk_id;
  if (m->host_only) return SPM_OK;
  auto up = [&](DevBuf *b, const void *src, size_t bytes) -> bool {
    if (b->Reserve(std::max<size_t>(bytes, 4)) != hipSuccess) return false;
    return hipMemcpy(b->ptr, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up(&m->d_units, m->trie.units.data(), m->trie.units.size() * 4) ||
      !up(&m->d_values, m->trie.values.data(), m->trie.values.size() * 4) ||
      !up(&m->d_scores, scores.data(), V * 4) ||
      !up(&m->bpe.entry_piece, entry_piece.data(), entry_piece.size() * 4) ||
      !up(&m->bpe.entry_out, entry_out.data(), entry_out.size() * 4) ||
      !up(&m->bpe.piece_kind, kind.data(), V) ||
      !up(&m->bpe.piece_out, piece_out.data(), V * 4) ||
      !up(&m->bpe.pair_keys, hk.data(), cap * 8) || !up(&m->bpe.pair_vals, hv.data(), cap * 4) ||
      !up(&m->bpe.pair_ent, he.data(), cap * 16) ||
      (!rank_piece.empty() && !up(&m->bpe.rank_piece, rank_piece.data(), rank_piece.size() * 2))) {
    *err = "device upload failed";
    return SPM_INTERNAL;
  }
  return SPM_OK;
}

// Token count of a sentence from its ntok word (bpe_lane_kernel's packed
// form or a plain count).
struct BpeCount {
  __host__ __device__ uint64_t operator()(uint32_t v) const { return (v & kLaneTok) ? (v & 0xFFu) : v; }
};

// Dense CSR output, one bpe_lane_kernel tile (kLB sentences) per block
// iteration.  A tile whose sentences all came from the lane kernel is one
// tile-dense run in sentence order: it is copied with coalesced loads and
// stores (per-sentence copies by one thread each wrote ~2.4x the ids' bytes,
// profiles/pmc/c3__bpe_compact_kernel.json of round 6).  Any other tile goes
// sentence by sentence: lane-encoded ones from the run, the rest from their
// right-aligned slots.
constexpr int kCompactThreads = 256;
__global__ __launch_bounds__(kCompactThreads) void bpe_compact_kernel(
    const uint64_t *__restrict__ off, uint64_t n, const uint32_t *__restrict__ ntok,
    const int32_t *__restrict__ lane_ids, const uint32_t *__restrict__ lane_len, const int32_t *__restrict__ slot_ids,
    const uint32_t *__restrict__ slot_len, int32_t *__restrict__ ids, uint32_t *__restrict__ piece_len,
    const uint64_t *__restrict__ tok_off, const uint32_t *__restrict__ status, uint32_t *__restrict__ out_status) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && out_status && status && status[kStError])
    atomicCAS(out_status, 0u, 8u);  // SPM_RESOURCE_EXHAUSTED, first error wins
  if (status && (status[kStError] & 2u)) return;
  __shared__ uint32_t s_tot;
  const int tid = threadIdx.x;
  for (uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kLB; t0 < n; t0 += static_cast<uint64_t>(gridDim.x) * kLB) {
    const uint64_t t1 = t0 + kLB < n ? t0 + kLB : n;
    const uint64_t i = t0 + static_cast<uint64_t>(tid);
    const uint32_t v = tid < kLB && i < t1 ? ntok[i] : kLaneTok;
    // The run's source and destination, loaded beside the counts (not after
    // the barrier that tells whether the tile is one run).
    const uint64_t s0 = off[t0], d0 = tok_off[t0];
    if (i + 1 == t1) s_tot = ((v >> 8) & 0x7FFFFFu) + (v & 0xFFu);  // the run's length (if all lane)
    if (__syncthreads_and((v & kLaneTok) != 0)) {
      const uint32_t tot = s_tot;
      const int32_t *__restrict__ src = lane_ids + s0;
      for (uint32_t j = static_cast<uint32_t>(tid); j < tot; j += kCompactThreads) ids[d0 + j] = src[j];
      if (piece_len) {
        const uint32_t *__restrict__ srcl = lane_len + s0;
        for (uint32_t j = static_cast<uint32_t>(tid); j < tot; j += kCompactThreads) piece_len[d0 + j] = srcl[j];
      }
    } else if (tid < kLB && i < t1) {
      const uint64_t o0 = tok_off[i], k = tok_off[i + 1] - o0;
      const int32_t *src;
      const uint32_t *srcl;
      if (v & kLaneTok) {
        const uint64_t r0 = s0 + ((v >> 8) & 0x7FFFFFu);
        src = lane_ids + r0;
        srcl = lane_len ? lane_len + r0 : nullptr;
      } else {
        const uint64_t r0 = off[i + 1] - k;
        src = slot_ids + r0;
        srcl = slot_len ? slot_len + r0 : nullptr;
      }
      for (uint64_t j = 0; j < k; ++j) ids[o0 + j] = src[j];
      if (piece_len)
        for (uint64_t j = 0; j < k; ++j) piece_len[o0 + j] = srcl[j];
    }
    __syncthreads();  // s_tot is rewritten by the next tile
  }
}

hipError_t LaunchBpeCompact(const uint64_t *off, uint64_t n, const uint32_t *ntok, const int32_t *lane_ids,
                            const uint32_t *lane_len, const int32_t *slot_ids, const uint32_t *slot_len,
                            int32_t *ids, uint32_t *piece_len, uint64_t *tok_off, void *scan_tmp,
                            size_t *scan_tmp_bytes, const uint32_t *status, uint32_t *out_status, hipStream_t st) {
  hipcub::TransformInputIterator<uint64_t, BpeCount, const uint32_t *> in(ntok, BpeCount());
  if (scan_tmp == nullptr)
    return hipcub::DeviceScan::InclusiveSum(nullptr, *scan_tmp_bytes, in, tok_off + 1,
                                            static_cast<int>(n > 0 ? n : 1), st);
  hipError_t e = hipMemsetAsync(tok_off, 0, sizeof(uint64_t), st);
  if (e != hipSuccess || n == 0) return e;
  e = hipcub::DeviceScan::InclusiveSum(scan_tmp, *scan_tmp_bytes, in, tok_off + 1, static_cast<int>(n), st);
  if (e != hipSuccess) return e;
  const uint64_t g64 = (n + kLB - 1) / kLB;
  const unsigned grid = static_cast<unsigned>(g64 < 16384 ? g64 : 16384);
  hipLaunchKernelGGL(bpe_compact_kernel, dim3(grid), dim3(kCompactThreads), 0, st, off, n, ntok, lane_ids, lane_len, slot_ids,
                     slot_len, ids, piece_len, tok_off, status, out_status);
  return hipGetLastError();
}

// Encode of one batch: bpe_lane_kernel (one sentence per lane; bpe_half_kernel,
// two sentences per wave, for vocabularies of >= 32768 pieces) + bpe_fast_kernel
// for the rest, then the general kernel on the flagged sentences with a
// device-side count (a fixed pool of lane slabs, one lane with the whole pool
// for longer sentences), scan + compaction.  No host synchronization unless
// c.host_sized (general kernel over every sentence, scratch sized from the
// longest sentence: models with user-defined symbols, force_general).
int EncodeBpe(spm_hip_model *m, EncodeWorkspace *ws, const EncodeCall &c, std::string *err) {
#define BPE_TRY(expr)                                              \
  do {                                                             \
    hipError_t _e = (expr);                                        \
    if (_e != hipSuccess) {                                        \
      *err = std::string(#expr) + ": " + hipGetErrorString(_e);    \
      return SPM_INTERNAL;                                         \
    }                                                              \
  } while (0)
  const uint64_t n = c.n, nn = std::max<uint64_t>(n, 1), cap = std::max<uint64_t>(c.capacity, 1);
  const hipStream_t st = c.st;
  const size_t ctl_bytes = kStWords * 4;
  BPE_TRY(ws->w_ctl.Reserve(ctl_bytes + 8 * (FastTiles(n) + kScanTiles)));
  BPE_TRY(hipMemsetAsync(ws->w_ctl.ptr, 0, ctl_bytes, st));
  uint32_t *status = ws->w_ctl.as<uint32_t>();
  BPE_TRY(ws->w_slot2_ids.Reserve(cap * 4));
  if (c.len) BPE_TRY(ws->w_slot2_len.Reserve(cap * 4));
  BPE_TRY(ws->w_ntok.Reserve(nn * 4));
  BPE_TRY(ws->w_flagged.Reserve(nn * 4));
  BpeArgs a{c.bytes, c.off, n, m->d_units.as<uint32_t>(), m->d_values.as<int32_t>(),
            m->bpe.entry_piece.as<int32_t>(), m->bpe.entry_out.as<int32_t>(),
            m->d_scores.as<float>(), m->bpe.piece_kind.as<uint8_t>(), m->bpe.piece_out.as<int32_t>(),
            m->bpe.pair_keys.as<uint64_t>(), m->bpe.pair_vals.as<int32_t>(),
            m->bpe.pair_ent.as<uint4>(), m->bpe.pair_mask,
            m->up.root_base, m->unk_id, m->bpe.irregular ? 1 : 0, ws->w_slot2_ids.as<int32_t>(),
            c.len ? ws->w_slot2_len.as<uint32_t>() : nullptr, ws->w_ntok.as<uint32_t>(),
            ws->w_flagged.as<uint32_t>(), status, cap, c.out_status,
            m->bpe.rank_ids ? m->bpe.rank_piece.as<int16_t>() : nullptr, m->bpe.rank_base, 1, nullptr, nullptr};
  static const int kPipeProbes = [] {  // A/B knob: SPM_HIP_BPE_PIPE=0 resolves each merge's probes at once
    const char *e = std::getenv("SPM_HIP_BPE_PIPE");
    return e ? std::atoi(e) : 1;
  }();
  a.pipe_probes = kPipeProbes;
  int slot = -1;
  bool timed_fast = false;
  if (m->timing) {
    slot = static_cast<int>(ws->tcount % EncodeWorkspace::kTimingRing);
    for (int k = 0; k < 2; ++k)
      if (!ws->tev[2 * slot + k]) BPE_TRY(hipEventCreate(&ws->tev[2 * slot + k]));
    for (auto &e : ws->ev)
      if (!e) BPE_TRY(hipEventCreate(&e));
    ++ws->tcount;
    ws->last_slot = slot;
  }
  if (c.host_sized) {
    const uint32_t max_nb = std::max<uint32_t>(c.max_nb, 1);
    const uint64_t slab = BpeGeneralSlabBytes(max_nb);
    uint64_t threads = std::min<uint64_t>(nn, 16384);
    while (threads > 64 && threads * slab > (4ull << 30)) threads /= 2;
    if (threads * slab > (16ull << 30)) {
      *err = "sentence too long for the general BPE path";
      return SPM_RESOURCE_EXHAUSTED;
    }
    BPE_TRY(ws->w_scratch.Reserve(threads * slab));
    GenBpeArgs g{a, nullptr, nullptr, n, ws->w_scratch.as<uint8_t>(), slab, max_nb, status + kStError,
                 m->bpe.has_user_defined ? 1 : 0, nullptr, nullptr, static_cast<uint32_t>(threads)};
    if (slot >= 0) BPE_TRY(hipEventRecord(ws->ev[0], st));
    if (n) hipLaunchKernelGGL(bpe_general_kernel, dim3((threads + 63) / 64), dim3(64), 0, st, g);
    BPE_TRY(hipGetLastError());
    if (slot >= 0) BPE_TRY(hipEventRecord(ws->ev[1], st));
  } else if (n) {
    // Two sentences per wave first; the rest (long / non-UTF-8-regular) one
    // per wave from the device-side list.
    BPE_TRY(ws->w_rest.Reserve(nn * 4));
    if (slot >= 0) BPE_TRY(hipEventRecord(ws->tev[2 * slot], st));
    if (m->bpe.lane_ok) {
      BPE_TRY(ws->w_slot_ids.Reserve(cap * 4));
      if (c.len) BPE_TRY(ws->w_slot_len.Reserve(cap * 4));
      a.lane_ids = ws->w_slot_ids.as<int32_t>();
      a.lane_len = c.len ? ws->w_slot_len.as<uint32_t>() : nullptr;
      const uint64_t tiles = (n + kLB - 1) / kLB;
      static const int kRankIdsKnob = [] {  // A/B knob: SPM_HIP_BPE_RANK_IDS=0 keeps the 32-bit symbol words
        const char *e = std::getenv("SPM_HIP_BPE_RANK_IDS");
        return e ? std::atoi(e) : 1;
      }();
      const dim3 grid(static_cast<unsigned>(std::min<uint64_t>(tiles, 1u << 20)));
      if (m->bpe.rank_ids && kRankIdsKnob)
        hipLaunchKernelGGL(bpe_lane_kernel<true>, grid, dim3(kLB), 0, st, a, ws->w_rest.as<uint32_t>(), status + 8);
      else
        hipLaunchKernelGGL(bpe_lane_kernel<false>, grid, dim3(kLB), 0, st, a, ws->w_rest.as<uint32_t>(), status + 8);
    } else {
      const uint64_t hblocks64 = (((n + 1) / 2) * 64 + 255) / 256;
      const unsigned hblocks = static_cast<unsigned>(std::min<uint64_t>(hblocks64, 1u << 20));
      hipLaunchKernelGGL(bpe_half_kernel, dim3(hblocks), dim3(256), 0, st, a, ws->w_rest.as<uint32_t>(), status + 8);
    }
    BPE_TRY(hipGetLastError());
    const uint64_t blocks64 = (n * 64 + 255) / 256;
    hipLaunchKernelGGL(bpe_fast_kernel, dim3(static_cast<unsigned>(std::min<uint64_t>(blocks64, 8192u))), dim3(256),
                       0, st, a, ws->w_rest.as<uint32_t>(), status + 8);
    BPE_TRY(hipGetLastError());
    timed_fast = slot >= 0;  // the timed span ends after the output compaction below
    const GeneralPool gp = PlanGeneralPool(cap, 128, 2048, [](uint32_t nb) { return BpeGeneralSlabBytes(nb); });
    BPE_TRY(ws->w_scratch.Reserve(gp.pool));
    const uint64_t ovf_cap = std::min<uint64_t>(nn, cap / (gp.small_nb + 1ull) + 1);
    BPE_TRY(ws->w_ovf.Reserve(ovf_cap * 4));
    uint32_t *ovf = ws->w_ovf.as<uint32_t>();
    const int32_t ud = m->bpe.has_user_defined ? 1 : 0;
    if (slot >= 0) BPE_TRY(hipEventRecord(ws->ev[0], st));
    GenBpeArgs g1{a, ws->w_flagged.as<uint32_t>(), status + kStFlagged, 0, ws->w_scratch.as<uint8_t>(), gp.slab,
                  gp.small_nb, status + kStError, ud, ovf, status + kStOverflow, gp.lanes};
    hipLaunchKernelGGL(bpe_general_kernel, dim3((gp.lanes + 63) / 64), dim3(64), 0, st, g1);
    BPE_TRY(hipGetLastError());
    GenBpeArgs g2{a, ovf, status + kStOverflow, 0, ws->w_scratch.as<uint8_t>(), gp.pool, gp.big_nb,
                  status + kStError, ud, nullptr, nullptr, 1};
    hipLaunchKernelGGL(bpe_general_kernel, dim3(1), dim3(64), 0, st, g2);
    BPE_TRY(hipGetLastError());
    if (slot >= 0) BPE_TRY(hipEventRecord(ws->ev[1], st));
  }
  size_t tmp_bytes = 0;
  BPE_TRY(LaunchBpeCompact(c.off, n, ws->w_ntok.as<uint32_t>(), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                           c.tok, nullptr, &tmp_bytes, status, c.out_status, st));
  BPE_TRY(ws->w_scan.Reserve(tmp_bytes + 16));
  BPE_TRY(LaunchBpeCompact(c.off, n, ws->w_ntok.as<uint32_t>(), a.lane_ids, a.lane_len, ws->w_slot2_ids.as<int32_t>(),
                           c.len ? ws->w_slot2_len.as<uint32_t>() : nullptr, c.ids, c.len, c.tok, ws->w_scan.ptr,
                           &tmp_bytes, status, c.out_status, st));
  // Timed span of the lane path: lane + fast kernels, the general kernels
  // (no-ops unless a sentence was flagged) and the output compaction.
  if (timed_fast) BPE_TRY(hipEventRecord(ws->tev[2 * slot + 1], st));
  return SPM_OK;
#undef BPE_TRY
}

}  // namespace spm_amd
