// Unigram Viterbi encode kernels for gfx950 (MI355X).
//
// Reference path: unigram::Model::Encode (unigram_model.cc:705-720) =
//   Lattice::SetSentence (:147-187) + Model::PopulateNodes (:535-604, a darts
//   commonPrefixSearch per char position) + Lattice::Viterbi (:222-261).
//
// unigram_fast_kernel — one sentence per lane, lattice never materialised:
//   Viterbi's backtrace score of a node (b,e) with score s is
//     max_l fl(bt_l + s) over lnodes ending at b  ==  fl(T_b + s),
//   T_b = max bt of the nodes ending at b, because float rounding is monotone.
//   So the forward pass keeps only T per pending end position, in a register
//   ring of W slots indexed by the (static, unrolled) char distance d of the
//   trie walk.  The argmax *identity* (the back-pointer) is what float ties
//   can change: the reference takes the FIRST lnode in end_nodes order
//   (= ascending begin) with the maximal fl(bt_l + s).  Only the successive
//   running-max setters of an end position can win; a setter more than a few
//   ulps below the final max never ties.  So per end position the kernel
//   keeps B (first setter of T) and, when the previous setter is within the
//   near-tie bound, an "ambiguity" entry (T, T2, B2) in registers; the
//   backtrace resolves winner = (fl(T2+s) == fl(T+s)) ? B2 : B exactly.  A
//   sentence whose ties chain deeper (3 near setters), overflows the entry
//   list, or meets a trie leaf inside a UTF-8 char is flagged and re-run by
//   unigram_general_kernel, a literal restatement of the reference lattice
//   (node lists + Viterbi over every (rnode, lnode) pair) in global scratch.
//
// Back-pointers: one byte per char position (end byte offset - winner begin
// byte offset), stored at the sentence's own byte offsets in a scratch array
// the size of the input.  Node ids on the best path are re-derived in the
// backtrace by an exact-match walk (or UNK), so the forward pass stores no
// per-node data at all.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "device_common.h"
#include "kernels.h"

namespace spm_amd {
namespace {

struct FastArgs {
  const uint8_t *__restrict__ bytes;
  const uint64_t *__restrict__ off;
  uint64_t n;
  const uint32_t *__restrict__ units;
  const int32_t *__restrict__ values;
  const float *__restrict__ scores;
  UnigramParams p;
  int32_t *__restrict__ slot_ids;   // block-dense token slots
  uint32_t *__restrict__ slot_len;  // nullable
  uint32_t *__restrict__ ntok;
  uint32_t *__restrict__ lo;        // block-local token offset (kNone: general path)
  uint8_t *__restrict__ bp;         // back-pointers of char positions >= kLdsBpPos
  uint32_t *__restrict__ flagged;
  uint32_t *__restrict__ status;    // [0] flagged count, [1] max flagged bytes
  const float *__restrict__ vscore; // per unit: leaf score or NaN tag (kVar & 4)
  uint32_t num_units;
  const uint2 *__restrict__ jump2;  // {unit, score} after two bytes (kVar & 4096)
};

constexpr int kBlock = 256;
constexpr int kLdsBpPos = 64;  // back-pointer bytes kept in LDS per lane

constexpr uint32_t kLdsBytes = 12288;  // staged sentence bytes per block (kVar & 1)
constexpr uint32_t kLdsUnits = 2048;   // cached top of the double array (kVar & 2)

// kVar bit 0: stage the block's sentence bytes in LDS; bit 1: keep the first
// kLdsUnits trie units (BFS layout = top levels) in LDS; bit 2: read the leaf
// score from the per-unit score table (one load instead of value + score);
// bit 5: lanes take the block's sentences in ascending byte length (LDS
// counting sort), so each wave's 64 sentences have similar lengths and the
// per-wave loop trip count (the longest sentence) drops; bit 6: the leaf-score
// loads and inserts of a position stop at the wave's deepest live trie step;
// bit 7: positions are walked in pairs (two independent load chains per lane);
// bit 8 (with 7): all four positions of a group walked together; bit 10 (with
// 3): the byte window advances by one aligned dword buffer load per group
// (spliced by alignbyte) instead of four byte loads; bit 12 (with 7 and 3):
// the walk's depth-2 unit and score come from a 65536-entry table indexed by
// the first two bytes, loaded beside the depth-1 unit, so a walk's chain of
// dependent loads is one shorter; bit 14 (with 7, no 2/12): each position's
// inserts lag its walk by one step (score registers live one step, see the
// pair walk) and the ring's back-pointers are packed distances with 2 near-tie
// entries (register diet, see kPackB); bit 15: occupancy target 5 waves per
// SIMD instead of 4 (96 VGPRs; forcing it on 1272 spills 175 VGPRs to scratch:
// 7.7 vs 6.1 ms); bit 16: target 6 waves (80 VGPRs); bit 17: 7 waves (72);
// bit 18 (with 14): a single near-tie entry.
template <int W, int kVar>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(
    (kVar & 131072) ? 7 : (kVar & 65536) ? 6 : (kVar & 32768) ? 5 : (W == 16 ? 4 : 1)))) void unigram_fast_kernel(FastArgs a) {
  // Back-pointer bytes of byte positions [0, kLdsBpPos) of each lane's
  // sentence: word (pos/4)*kBlock + tid, byte pos%4 (lanes at the same pos
  // hit consecutive words).
  __shared__ uint32_t lds_bp[(kLdsBpPos / 4) * kBlock];
  __shared__ uint32_t lds_wave[kBlock / 64];
  __shared__ uint32_t lds_bytes[(kVar & 1) ? kLdsBytes / 4 : 1];
  // kVar & 2 in the byte-position pass: the first kTop units and their leaf
  // scores (the BFS top of the array: 80 % of the synthetic corpus's walk
  // loads hit units < 512) are staged in LDS; a walk step whose 64 lanes all
  // address the top reads LDS instead of L2.
  constexpr uint32_t kTop = (kVar & 8) ? ((kVar & 2048) ? 4096u : (kVar & 512) ? 2048u : 1024u) : kLdsUnits;
  __shared__ uint32_t lds_units[(kVar & 2) ? kTop : 1];
  __shared__ float lds_vs[((kVar & 2) && (kVar & 8)) ? kTop : 1];
  constexpr bool kPackB = (kVar & 16384) != 0;  // register diet (see the ring below)
  static_assert(!kPackB || (kVar & 8) != 0, "packed back-pointers need the byte-position pass");
  uint8_t *lbp = reinterpret_cast<uint8_t *>(lds_bp);
  const uint8_t *lby = reinterpret_cast<const uint8_t *>(lds_bytes);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  const uint64_t total_bytes = a.off[a.n];
  const auto units_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(a.units), 0,
                                                            static_cast<int>(a.num_units * 4u), 0x00020000);
  const auto vscore_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.vscore), 0,
                                                             static_cast<int>(a.num_units * 4u), 0x00020000);
  if constexpr ((kVar & 2) != 0) {
    for (uint32_t k = tid; k < kTop; k += kBlock) {
      const bool in = k < a.num_units;
      // Beyond the array: label 0xFF never matches a staged byte (the byte
      // pass flags 0xFF input) and the score is NaN (no node).
      lds_units[k] = in ? a.units[k] : ((kVar & 8) ? 0xFFu : 0u);
      if constexpr ((kVar & 8) != 0) lds_vs[k] = in ? a.vscore[k] : __builtin_nanf("");
    }
    __syncthreads();
  }
  __shared__ uint32_t lds_sort[(kVar & 32) ? 2 * kBlock : 1];
  __shared__ uint32_t lds_scan[kBlock];
  for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * kBlock; base < a.n; base += step) {
    uint32_t sid = static_cast<uint32_t>(tid);
    if constexpr ((kVar & 32) != 0) {
      // Counting sort of the block's sentences by length bucket (0..255).
      uint32_t *hist = lds_sort, *perm = lds_sort + kBlock;
      const uint64_t ii = base + tid;
      const uint32_t len = ii < a.n ? static_cast<uint32_t>(a.off[ii + 1] - a.off[ii]) : 0u;
      const uint32_t bucket = len < kBlock - 1 ? len : kBlock - 1;
      hist[tid] = 0;
      __syncthreads();
      const uint32_t r = atomicAdd(&hist[bucket], 1u);
      __syncthreads();
      if (wave == 0) {  // exclusive scan of 256 bins, 4 per lane
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
    const uint32_t nb = valid ? static_cast<uint32_t>(a.off[i + 1] - b0) : 0;
    const uint8_t *__restrict__ s = a.bytes + b0;
    uint8_t *__restrict__ gbp = a.bp + b0;
    // The block's bytes (and back-pointer scratch) from its first aligned
    // byte as buffer resources: lanes address them by a 32-bit offset
    // (kPackB keeps no per-lane 64-bit pointers live).
    const uint64_t blk_al = a.off[base] & ~3ull;
    const uint64_t blk_rem = total_bytes - blk_al;
    const int blk_nrec = static_cast<int>(blk_rem < 0x7FFFFFF0ull ? blk_rem : 0x7FFFFFF0ull);
    const auto bytes_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.bytes + blk_al), 0,
                                                              blk_nrec, 0x00020000);
    // Back-pointer scratch of the block: uniform base + 32-bit lane offset.
    // (A buffer-resource byte store/load pair here hung on sentences longer
    // than the LDS window: the load never saw the store; global accesses do.)
    uint8_t *__restrict__ blk_bp = a.bp + blk_al;
    const uint32_t lrel = static_cast<uint32_t>(b0 - blk_al);  // lane's first byte, block-relative
    uint64_t lds_off = ~0ull;  // lane's first byte in the staged block bytes
    if constexpr ((kVar & 1) != 0) {
      const uint64_t blk0 = a.off[base];
      const uint64_t blk1 = a.off[base + kBlock < a.n ? base + kBlock : a.n];
      const uint64_t al = blk0 & ~3ull;
      uint64_t nw = (blk1 - al + 3) / 4;
      if (nw > kLdsBytes / 4) nw = kLdsBytes / 4;
      for (uint64_t k = tid; k < nw; k += kBlock) {
        const uint64_t g = al + 4 * k;
        uint32_t w;
        if (g + 4 <= total_bytes) {
          w = *reinterpret_cast<const uint32_t *>(a.bytes + g);
        } else {
          w = 0;
          for (uint32_t t = 0; t < 4 && g + t < total_bytes; ++t) w |= uint32_t(a.bytes[g + t]) << (8 * t);
        }
        lds_bytes[k] = w;
      }
      lds_off = b0 - al;
      __syncthreads();
    }
    auto byte_at = [&](uint32_t q) -> uint32_t {
      if constexpr ((kVar & 1) != 0) {
        const uint64_t p = lds_off + q;
        if (p < kLdsBytes) return lby[p];
      }
      if constexpr (kPackB) return __builtin_amdgcn_raw_buffer_load_b8(bytes_rsrc, lrel + q, 0, 0);
      return s[q];
    };
    auto unit_at = [&](uint32_t node) -> uint32_t {
      if constexpr ((kVar & 2) != 0 && (kVar & 8) == 0) {
        if (node < kTop) return lds_units[node];
      }
      return a.units[node];
    };
    auto bp_store = [&](uint32_t pos, uint32_t v) {
      if (pos < kLdsBpPos) lbp[((pos >> 2) * kBlock + tid) * 4 + (pos & 3)] = static_cast<uint8_t>(v);
      else if constexpr (kPackB) blk_bp[lrel + pos] = static_cast<uint8_t>(v);
      else gbp[pos] = static_cast<uint8_t>(v);
    };
    auto bp_load = [&](uint32_t pos) -> uint32_t {
      if (pos < kLdsBpPos) return lbp[((pos >> 2) * kBlock + tid) * 4 + (pos & 3)];
      if constexpr (kPackB) return blk_bp[lrel + pos];
      return gbp[pos];
    };

    // Ring slot d = end position (current byte + d); nodes end only at char
    // boundaries, other slots stay empty.  Slot 0 of the first position is
    // BOS (score 0, backtrace 0: FreeList zero-fill, freelist.h:79).
    // kVar & 16384 (register diet): the back-pointer of slot k is kept as the
    // distance end - begin (<= W - 1, invariant under the ring shift), four
    // slots per register, and only 2 near-tie entries are kept (a sentence
    // that needs a third goes to the general kernel, as an overflow does).
    constexpr int kAmb = kPackB ? ((kVar & 262144) ? 1 : 2) : kAmbEntries;
    float T[W + 3];
    uint32_t B[kPackB ? 1 : W + 3];
    uint32_t Bw[kPackB ? (W + 6) / 4 : 1];
#pragma unroll
    for (int d = 0; d < W + 3; ++d) T[d] = 0.f;
#pragma unroll
    for (int d = 0; d < (kPackB ? 1 : W + 3); ++d) B[d] = 0;
#pragma unroll
    for (int d = 0; d < (kPackB ? (W + 6) / 4 : 1); ++d) Bw[d] = 0;
    // Distance from the setter's begin to `end` (the end position of slot k).
    auto b_dist = [&](auto kc, uint32_t end) -> uint32_t {
      constexpr int k = decltype(kc)::value;
      if constexpr (kPackB) return (Bw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
      else return end - B[k];
    };
    // Slot k's setter := the node [begin, begin + L) when gt.
    auto b_set = [&](auto kc, bool gt, uint32_t begin, auto lc) {
      constexpr int k = decltype(kc)::value;
      if constexpr (kPackB) {
        constexpr uint32_t L = decltype(lc)::value, sh = 8 * (k & 3);
        const uint32_t w = (Bw[k >> 2] & ~(0xFFu << sh)) | (L << sh);
        Bw[k >> 2] = gt ? w : Bw[k >> 2];
      } else {
        B[k] = gt ? begin : B[k];
      }
    };
    uint64_t has = 1;   // bit d: slot d holds a node
    std::conditional_t<kPackB, uint32_t, uint64_t> ambm = 0;  // bit d: slot d has an ambiguity entry
    uint32_t ae[kAmb], aB2[kAmb];
    float aT[kAmb], aT2[kAmb];
#pragma unroll
    for (int k = 0; k < kAmb; ++k) {
      ae[k] = kNone;
      aB2[k] = 0;
      aT[k] = 0.f;
      aT2[k] = 0.f;
    }
    bool bad = false, any_amb = false;
    // Offsets past the block's buffer range (a > 2 GB block) would read 0:
    // such a sentence takes the general kernel.
    if constexpr (kPackB) bad = valid && (b0 - blk_al) + nb > static_cast<uint64_t>(blk_nrec);

    // Rare path of insert: maintain the near-tie entry of end position `end`.
    auto amb_update = [&](auto dc, float bt, bool nr, uint32_t end) {
      constexpr int d = decltype(dc)::value;
      int slot = -1, free_slot = -1;
#pragma unroll
      for (int k = 0; k < kAmb; ++k) {
        if (ae[k] == end) slot = k;
        if (ae[k] == kNone && free_slot < 0) free_slot = k;
      }
      if (slot >= 0) {
#pragma unroll
        for (int k = 0; k < kAmb; ++k)
          if (k == slot) {
            // Older setter (aT2) also near the new max: 3-deep tie chain.
            if (NearTie(aT2[k], bt, a.p.tie_mag)) bad = true;
            if (nr) {
              aT2[k] = T[d];
              aB2[k] = end - b_dist(dc, end);
              aT[k] = bt;
            } else {
              ae[k] = kNone;
              ambm &= ~(1ull << d);
            }
          }
      } else if (nr) {
        if (free_slot < 0) bad = true;
        any_amb = true;
        ambm |= 1ull << d;
#pragma unroll
        for (int k = 0; k < kAmb; ++k)
          if (k == free_slot) {
            ae[k] = end;
            aT2[k] = T[d];
            aB2[k] = end - b_dist(dc, end);
            aT[k] = bt;
          }
      }
    };
    // Insert node [begin, end) with backtrace score bt into ring slot d.
    // Nodes reach a slot in ascending begin order (= end_nodes_ order).
    auto insert = [&](auto dc, float bt, uint32_t begin, uint32_t end) {
      constexpr int d = decltype(dc)::value;
      if (!((has >> d) & 1)) {
        has |= (1ull << d);
        T[d] = bt;
        B[d] = begin;
      } else if (bt > T[d]) {
        bool nr;
        if constexpr ((kVar & 8) != 0) nr = NearTieHi(T[d], bt, a.p.tie_mag);
        else nr = NearTie(T[d], bt, a.p.tie_mag);
        if (nr || ((ambm >> d) & 1)) amb_update(dc, bt, nr, end);
        T[d] = bt;
        B[d] = begin;
      }
    };

    if constexpr ((kVar & 8) != 0) {
      // Byte-position forward pass (units = the 0xFF-padded image, see
      // BuildUnitsFF).  Every byte position p is visited; p is a char start
      // iff the lead-byte chain from 0 reaches it (OneCharLen clamped to the
      // sentence, unigram_model.cc:155-160 / util.h:389), so malformed UTF-8
      // needs no special case.  Pieces split exactly into chars (checked at
      // load), hence a leaf reached from a char start ends at a char start.
      // Positions are processed kU at a time against a ring R[k] = end
      // p0 + k (k < W + kU - 1), shifted by kU registers per group.
      constexpr int kU = 4;
      constexpr int kR = W + kU - 1;
      // Window words: bytes p0 .. p0 + 4*kWin - 1 (the walks read up to byte
      // p0 + kU - 1 + W - 2; kPackB drops the spare word).
      constexpr int kWin = kPackB ? (kR + 3) / 4 : (kR + 3) / 4 + 1;
      static_assert(4 * kWin >= kU + W - 1, "window covers every walk byte");
      static_assert(kR <= W + 3, "ring arrays are sized W + 3");
#pragma unroll
      for (int d = 0; d < W + 3; ++d) T[d] = d == 0 ? 0.f : -__builtin_inff();
      has = ~0ull;
      // Bytes q .. q+3 of the sentence, zero beyond nb; flags 0xFF bytes
      // (the padded trie image matches 0xFF on empty units).
      auto load_rel = [&](uint32_t q) -> uint32_t {
        uint32_t x;
        const uint64_t A = lds_off + q;
        bool staged = false;
        if constexpr ((kVar & 1) != 0) staged = A + 8 <= kLdsBytes;
        if (staged) {
          const uint32_t wi = static_cast<uint32_t>(A >> 2);
          x = __builtin_amdgcn_alignbyte(lds_bytes[wi + 1], lds_bytes[wi], static_cast<uint32_t>(A & 3));
        } else {
          x = 0;
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (q + t < nb) x |= static_cast<uint32_t>(s[q + t]) << (8 * t);
        }
        if (q + 4 > nb) x &= q >= nb ? 0u : (1u << (8 * (nb - q))) - 1u;
        const uint32_t y = ~x;  // 0xFF byte in x <=> zero byte in y
        if (((y - 0x01010101u) & ~y & 0x80808080u) != 0) bad = true;
        return x;
      };
      // kVar & 1024: the window slides 4 bytes per group, so each group needs
      // one new ALIGNED dword (buffer load relative to the block's first byte,
      // out of range → 0) spliced with the previous one by alignbyte, instead
      // of 4 byte gathers.
      const uint32_t sh = lrel & 3u;
      const uint32_t lane_al = lrel & ~3u;
      auto word_at = [&](uint32_t m) -> uint32_t {
        const uint32_t o = lane_al + 4u * m;
        if (o + 4 <= blk_rem) return __builtin_amdgcn_raw_buffer_load_b32(bytes_rsrc, o, 0, 0);
        // The batch's last, partial dword: byte loads (a dword load that
        // straddles num_records would read as 0).
        uint32_t x = 0;
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t)
          if (o + t < blk_rem) x |= static_cast<uint32_t>(a.bytes[blk_al + o + t]) << (8 * t);
        return x;
      };
      auto finish = [&](uint32_t x, uint32_t q) -> uint32_t {
        if (q + 4 > nb) x &= q >= nb ? 0u : (1u << (8 * (nb - q))) - 1u;
        const uint32_t y = ~x;
        if (((y - 0x01010101u) & ~y & 0x80808080u) != 0) bad = true;
        return x;
      };
      uint32_t wprev = 0;
      uint32_t rw[kWin];
      if constexpr ((kVar & 1024) != 0) {
        if (nb > 0) wprev = word_at(0);
#pragma unroll
        for (int k = 0; k < kWin; ++k) {
          const uint32_t q = 4 * k;
          const uint32_t wn = q < nb ? word_at(k + 1) : 0u;
          rw[k] = q < nb ? finish(__builtin_amdgcn_alignbyte(wn, wprev, sh), q) : 0u;
          wprev = wn;
        }
      } else {
#pragma unroll
        for (int k = 0; k < kWin; ++k) rw[k] = nb > 0 ? load_rel(4 * k) : 0u;
      }
      uint32_t next_start = 0;
      for (uint32_t p0 = 0; p0 <= nb; p0 += kU) {
        auto position = [&](auto jc) {
          constexpr int j = decltype(jc)::value;
          const uint32_t p = p0 + j;
          if (p <= nb && p == next_start) {
            if (p > 0) bp_store(p, b_dist(std::integral_constant<int, j>{}, p));
            if (p < nb) {
              const float T0 = T[j];
              const uint32_t c0 = (rw[j >> 2] >> (8 * (j & 3))) & 0xFFu;
              uint32_t clen0 = OneCharLenDev(c0);
              if (clen0 > nb - p) clen0 = nb - p;
              next_start = p + clen0;
              // Phase 1: the walk (unit loads only on the dependent chain).
              uint32_t base_u = a.p.root_base;
              uint32_t leafmask = 0;
              uint32_t lnode[W];
              bool alive = true;
              auto walk = [&](auto dc) {
                constexpr int d = decltype(dc)::value;
                constexpr int t = j + d - 1;
                const uint32_t c = (rw[t >> 2] >> (8 * (t & 3))) & 0xFFu;
                if (alive) {
                  const uint32_t node = base_u ^ c;
                  const uint32_t u = unit_at(node);
                  if ((u & 0xFFu) != c) {
                    alive = false;
                  } else {
                    base_u = u >> 9;
                    lnode[d] = node;
                    if (u & 0x100u) leafmask |= 1u << d;
                  }
                }
              };
              StaticFor<1, W>(walk);
              // Phase 2: leaf scores / kind tags (independent loads).
              auto score = [&](auto dc) {
                constexpr int d = decltype(dc)::value;
                if ((leafmask >> d) & 1) lnode[d] = __float_as_uint(a.vscore[lnode[d]]);
              };
              StaticFor<1, W>(score);
              // Phase 3: nodes in ascending length; the UNK node
              // (unigram_model.cc:597-601) replaces a missing usable
              // single-char node at d == clen0.
              auto ins = [&](auto dc) {
                constexpr int d = decltype(dc)::value;
                bool use = false;
                float s_node = 0.f;
                if ((leafmask >> d) & 1) {
                  const uint32_t sb = lnode[d];
                  const int32_t kind =
                      (sb & 0x7FFFFFFFu) > 0x7F800000u ? static_cast<int32_t>(sb & 3u) : 0;
                  if (kind != kKindUnused) {
                    use = true;
                    s_node = __uint_as_float(sb);
                    if (kind == kKindUserDefined) {
                      int chars = 0;
                      for (uint32_t q = p; q < p + d; q += OneCharLenDev(byte_at(q))) ++chars;
                      s_node = UserDefinedScore(chars, a.p.max_score);
                    }
                  }
                }
                if constexpr (d <= 4) {
                  if (!use && d == static_cast<int>(clen0)) {
                    use = true;
                    s_node = a.p.unk_score;
                  }
                }
                if (use) insert(std::integral_constant<int, j + d>{}, __fadd_rn(T0, s_node), p, p + d);
              };
              StaticFor<1, W>(ins);
            }
          }
        };
        if constexpr ((kVar & 128) != 0) {
          // Pairs of positions: the two trie walks are independent chains,
          // so their unit loads (and each step's leaf-score load) are issued
          // together — two chains in flight per lane instead of one.  The
          // inserts stay in position order: position j1's T0 and back-pointer
          // are read after position j0's nodes (length 1 ends at j1) landed.
          // Node [p, p + d) of position j with raw score sc (NaN: no node).
          auto insert_one = [&](auto jc, auto dc, uint32_t p, float T0, uint32_t clen0, bool st,
                                float sc, int dmax) {
            constexpr int j = decltype(jc)::value;
            constexpr int d = decltype(dc)::value;
            if (d > 4 && d > dmax) return;
            float s_node = sc;
            if constexpr (d <= 4)
              s_node = (d == static_cast<int>(clen0) && __builtin_isnan(s_node)) ? a.p.unk_score : s_node;
            if (!st) s_node = __builtin_nanf("");
            const float bt = __fadd_rn(T0, s_node);
            constexpr int k = j + d;
            const bool gt = bt > T[k];  // false for NaN
            const bool rare = gt && (NearTieHi(T[k], bt, a.p.tie_mag) || ((ambm >> k) & 1));
            if (__builtin_amdgcn_ballot_w64(rare) != 0) {
              if (rare) amb_update(std::integral_constant<int, k>{}, bt, NearTieHi(T[k], bt, a.p.tie_mag), p + d);
            }
            T[k] = gt ? bt : T[k];
            b_set(std::integral_constant<int, k>{}, gt, p, dc);
          };
          auto insert_pos = [&](auto jc, uint32_t p, float T0, uint32_t clen0, bool st,
                                const float *sc, int dmax) {
            StaticFor<1, W>([&](auto dc) {
              insert_one(jc, dc, p, T0, clen0, st, sc[decltype(dc)::value], dmax);
            });
          };
          // kNI positions walked together (bit 8: all kU = 4, else pairs).
          constexpr int kNI = (kVar & 256) ? 4 : 2;
          StaticFor<0, kU / kNI>([&](auto pc) {
            constexpr int jb = kNI * decltype(pc)::value;
            uint32_t pp[kNI], cl[kNI];
            bool at[kNI], st[kNI], any[kNI];
            // Char starts in order (next_start chains through the group).
            StaticFor<0, kNI>([&](auto qc) {
              constexpr int q = decltype(qc)::value, j = jb + q;
              pp[q] = p0 + j;
              at[q] = pp[q] <= nb && pp[q] == next_start;
              if (q == 0 && at[q] && pp[q] > 0) bp_store(pp[q], b_dist(std::integral_constant<int, j>{}, pp[q]));
              st[q] = at[q] && pp[q] < nb;
              cl[q] = OneCharLenDev((rw[j >> 2] >> (8 * (j & 3))) & 0xFFu);
              if (cl[q] > nb - pp[q]) cl[q] = nb - pp[q];
              if (st[q]) next_start = pp[q] + cl[q];
              any[q] = __builtin_amdgcn_ballot_w64(st[q]) != 0;
            });
            bool any_st = false;
            StaticFor<0, kNI>([&](auto qc) { any_st = any_st || any[decltype(qc)::value]; });
            if constexpr ((kVar & 16384) != 0) {
              // Lagged inserts: position q's node of length dd is inserted at
              // step d = dd + 1 + q, right after the walk's loads of step d
              // are issued.  Its score load (issued at step dd) has landed by
              // then, so each score register lives about one step instead of
              // the whole walk (2 x 16 live scores before).  Every insert into
              // slot jb + d - 1 happens at step d, in ascending q = ascending
              // begin, as end_nodes_ order requires; position q's own T0 and
              // back-pointer (slot jb + q, final after step q + 1) are read at
              // step q + 2, before its first insert.
              static_assert((kVar & 2) == 0 && (kVar & 4096) == 0, "plain unit loads only");
              float scl[kNI][W];
              float T0q[kNI];
              int dm[kNI];
              uint32_t bs[kNI];
              bool al[kNI];
              StaticFor<0, kNI>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                dm[q] = 0;
                T0q[q] = 0.f;
                bs[q] = st[q] ? a.p.root_base : 0u;
                al[q] = st[q];
              });
              bool go = any_st;
              // Software pipeline: step d waits for the unit loads of depth d
              // (issued the step before, together with the score loads of
              // depth d - 1), issues the score loads of depth d and the unit
              // loads of depth d + 1, and only then runs the lagged inserts,
              // so their VALU work overlaps the loads in flight.  Scores are
              // consumed through an asm copy taken once they are known to
              // have landed (sok): the copy is what the inserts read, so the
              // join after the walk branch never makes the compiler drain the
              // loads just issued.
              uint32_t nd[kNI], u[kNI], c[kNI];
              float sok[kNI][W];
              if (go) {
                StaticFor<0, kNI>([&](auto qc) {
                  constexpr int q = decltype(qc)::value, t = jb + q;
                  c[q] = (rw[t >> 2] >> (8 * (t & 3))) & 0xFFu;
                  nd[q] = bs[q] ^ c[q];
                  u[q] = __builtin_amdgcn_raw_buffer_load_b32(units_rsrc, nd[q] * 4u, 0, 0);
                });
              }
              auto land = [&](float x) -> float {
                float y;
                __asm__("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
                return y;
              };
              StaticFor<1, W + kNI>([&](auto dc) {
                constexpr int d = decltype(dc)::value;
                if constexpr (d < W) {
                  StaticFor<0, kNI>([&](auto qc) { scl[decltype(qc)::value][d] = __builtin_nanf(""); });
                  if (go) {
                    bool g = false;
                    StaticFor<0, kNI>([&](auto qc) {
                      constexpr int q = decltype(qc)::value;
                      al[q] = al[q] && (u[q] & 0xFFu) == c[q];
                      bs[q] = al[q] ? u[q] >> 9 : 0u;
                      const bool gq = __builtin_amdgcn_ballot_w64(al[q]) != 0;
                      if (gq) dm[q] = d;
                      g = g || gq;
                    });
                    if constexpr (d > 1)
                      StaticFor<0, kNI>([&](auto qc) { sok[decltype(qc)::value][d - 1] = land(scl[decltype(qc)::value][d - 1]); });
                    StaticFor<0, kNI>([&](auto qc) {
                      constexpr int q = decltype(qc)::value;
                      scl[q][d] = __uint_as_float(
                          __builtin_amdgcn_raw_buffer_load_b32(vscore_rsrc, (al[q] ? nd[q] : 0u) * 4u, 0, 0));
                    });
                    go = g;
                    if constexpr (d + 1 < W) {
                      if (go) {
                        StaticFor<0, kNI>([&](auto qc) {
                          constexpr int q = decltype(qc)::value, t = jb + q + d;
                          c[q] = (rw[t >> 2] >> (8 * (t & 3))) & 0xFFu;
                          nd[q] = bs[q] ^ c[q];
                          u[q] = __builtin_amdgcn_raw_buffer_load_b32(units_rsrc, nd[q] * 4u, 0, 0);
                        });
                      }
                    }
                  } else if constexpr (d > 1) {
                    StaticFor<0, kNI>([&](auto qc) { sok[decltype(qc)::value][d - 1] = land(scl[decltype(qc)::value][d - 1]); });
                  }
                } else if constexpr (d == W) {
                  StaticFor<0, kNI>([&](auto qc) { sok[decltype(qc)::value][W - 1] = land(scl[decltype(qc)::value][W - 1]); });
                }
                StaticFor<0, kNI>([&](auto qc) {
                  constexpr int q = decltype(qc)::value, j = jb + q, dd = d - 1 - q;
                  if constexpr (dd == 1) {
                    if (q > 0 && at[q] && pp[q] > 0) bp_store(pp[q], b_dist(std::integral_constant<int, j>{}, pp[q]));
                    T0q[q] = T[j];
                  }
                  if constexpr (dd >= 1 && dd < W) {
                    if (any[q])
                      insert_one(std::integral_constant<int, j>{}, std::integral_constant<int, dd>{}, pp[q],
                                 T0q[q], cl[q], st[q], sok[q][dd], dm[q]);
                  }
                });
              });
              return;
            }
            float sc[kNI][W];
            int dm[kNI];
            StaticFor<0, kNI>([&](auto qc) { dm[decltype(qc)::value] = 0; });
            if (any_st) {
              uint32_t bs[kNI];
              bool al[kNI];
              uint2 j2[kNI];
              StaticFor<0, kNI>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                bs[q] = st[q] ? a.p.root_base : 0u;
                al[q] = st[q];
              });
              bool go = true;
              StaticFor<1, W>([&](auto dc) {
                constexpr int d = decltype(dc)::value;
                StaticFor<0, kNI>([&](auto qc) { sc[decltype(qc)::value][d] = __builtin_nanf(""); });
                if (go) {
                  uint32_t nd[kNI], u[kNI], c[kNI];
                  bool top = false;
                  StaticFor<0, kNI>([&](auto qc) {
                    constexpr int q = decltype(qc)::value, t = jb + q + d - 1;
                    c[q] = (rw[t >> 2] >> (8 * (t & 3))) & 0xFFu;
                    nd[q] = bs[q] ^ c[q];
                  });
                  if constexpr ((kVar & 2) != 0) {
                    bool out = false;
                    StaticFor<0, kNI>([&](auto qc) { out = out || nd[decltype(qc)::value] >= kTop; });
                    top = __builtin_amdgcn_ballot_w64(out) == 0;  // wave-uniform
                  }
                  constexpr bool kJ2 = (kVar & 4096) != 0 && d == 2;
                  if constexpr ((kVar & 4096) != 0 && d == 1) {
                    // Depth 2 from the first two bytes, issued beside depth 1.
                    StaticFor<0, kNI>([&](auto qc) {
                      constexpr int q = decltype(qc)::value, t = jb + q + 1;  // the second byte
                      const uint32_t c2 = (rw[t >> 2] >> (8 * (t & 3))) & 0xFFu;
                      j2[q] = a.jump2[c[q] | c2 << 8];
                    });
                  }
                  if constexpr (kJ2) {
                    StaticFor<0, kNI>([&](auto qc) {
                      constexpr int q = decltype(qc)::value;
                      u[q] = j2[q].x;
                    });
                  } else if (top) {
                    StaticFor<0, kNI>([&](auto qc) {
                      constexpr int q = decltype(qc)::value;
                      u[q] = lds_units[nd[q]];
                    });
                  } else {
                    StaticFor<0, kNI>([&](auto qc) {
                      constexpr int q = decltype(qc)::value;
                      u[q] = __builtin_amdgcn_raw_buffer_load_b32(units_rsrc, nd[q] * 4u, 0, 0);
                    });
                  }
                  bool g = false;
                  StaticFor<0, kNI>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    al[q] = al[q] && (u[q] & 0xFFu) == c[q];
                    bs[q] = al[q] ? u[q] >> 9 : 0u;
                    // (Gating this load on the has_leaf bit of u measured
                    // slower: the address then waits on the unit load.)
                    if (kJ2)
                      sc[q][d] = al[q] ? __uint_as_float(j2[q].y) : __builtin_nanf("");
                    else if (top)
                      sc[q][d] = lds_vs[al[q] ? nd[q] : 0u];
                    else
                      sc[q][d] = __uint_as_float(
                          __builtin_amdgcn_raw_buffer_load_b32(vscore_rsrc, (al[q] ? nd[q] : 0u) * 4u, 0, 0));
                    const bool gq = __builtin_amdgcn_ballot_w64(al[q]) != 0;
                    if (gq) dm[q] = d;
                    g = g || gq;
                  });
                  go = g;
                }
              });
            }
            StaticFor<0, kNI>([&](auto qc) {
              constexpr int q = decltype(qc)::value, j = jb + q;
              if (q > 0 && at[q] && pp[q] > 0) bp_store(pp[q], b_dist(std::integral_constant<int, j>{}, pp[q]));
              if (any[q]) insert_pos(std::integral_constant<int, j>{}, pp[q], T[j], cl[q], st[q], sc[q], dm[q]);
            });
          });
        } else if constexpr ((kVar & 16) != 0) {
          // Branch-free body: units / vscore through buffer loads
          // (out-of-range → 0), vscore = per-unit node score with USER_DEFINED
          // scores folded in and NaN for "no usable node" (BuildVscoreBP).
          StaticFor<0, kU>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            const uint32_t p = p0 + j;
            const bool at = p <= nb && p == next_start;
            if (at && p > 0) bp_store(p, b_dist(std::integral_constant<int, j>{}, p));
            const bool st = at && p < nb;
            const uint32_t c0 = (rw[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            uint32_t clen0 = OneCharLenDev(c0);
            if (clen0 > nb - p) clen0 = nb - p;
            if (st) next_start = p + clen0;
            if (__builtin_amdgcn_ballot_w64(st) == 0) return;
            const float T0 = T[j];
            uint32_t base_u = st ? a.p.root_base : 0u;
            bool alive = st;
            uint32_t nodes[W];
            bool go = true;
            int dmax = 0;  // wave-uniform: deepest step where some lane is alive
            StaticFor<1, W>([&](auto dc) {
              constexpr int d = decltype(dc)::value;
              constexpr int t = j + d - 1;
              nodes[d] = 0;
              if (go) {
                const uint32_t c = (rw[t >> 2] >> (8 * (t & 3))) & 0xFFu;
                const uint32_t node = base_u ^ c;
                const uint32_t u = __builtin_amdgcn_raw_buffer_load_b32(units_rsrc, node * 4u, 0, 0);
                alive = alive && (u & 0xFFu) == c;
                base_u = alive ? u >> 9 : 0u;
                nodes[d] = alive ? node : 0u;
                go = __builtin_amdgcn_ballot_w64(alive) != 0;
                if (go) dmax = d;
              }
            });
            float sc[W];
            StaticFor<1, W>([&](auto dc) {
              constexpr int d = decltype(dc)::value;
              // kVar & 64: no lane has a node deeper than dmax (nodes[d] = 0
              // there, whose vscore is NaN), so those loads are skipped.
              if ((kVar & 64) == 0 || d <= dmax)
                sc[d] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vscore_rsrc, nodes[d] * 4u, 0, 0));
              else
                sc[d] = __builtin_nanf("");
            });
            StaticFor<1, W>([&](auto dc) {
              constexpr int d = decltype(dc)::value;
              // Beyond dmax (and past the UNK lengths 1..4) nothing is inserted.
              if constexpr ((kVar & 64) != 0) {
                if (d > 4 && d > dmax) return;
              }
              float s_node = sc[d];
              // UNK node (unigram_model.cc:597-601): no usable single-char node.
              if constexpr (d <= 4)
                s_node = (d == static_cast<int>(clen0) && __builtin_isnan(s_node)) ? a.p.unk_score : s_node;
              if (!st) s_node = __builtin_nanf("");
              const float bt = __fadd_rn(T0, s_node);
              constexpr int k = j + d;
              const bool gt = bt > T[k];  // false for NaN
              const bool rare = gt && (NearTieHi(T[k], bt, a.p.tie_mag) || ((ambm >> k) & 1));
              if (__builtin_amdgcn_ballot_w64(rare) != 0) {
                if (rare) amb_update(std::integral_constant<int, k>{}, bt, NearTieHi(T[k], bt, a.p.tie_mag), p + d);
              }
              T[k] = gt ? bt : T[k];
              b_set(std::integral_constant<int, k>{}, gt, p, dc);
            });
          });
        } else {
          StaticFor<0, kU>(position);
        }
        // Next group: shift the ring and the byte window by kU.
#pragma unroll
        for (int k = 0; k < kR; ++k) {
          if (k + kU < kR) {
            T[k] = T[k + kU];
            if constexpr (!kPackB) B[k] = B[k + kU];
          } else {
            T[k] = -__builtin_inff();
            if constexpr (!kPackB) B[k] = 0;
          }
        }
        if constexpr (kPackB) {
          static_assert(kU == 4, "one packed word per group");
#pragma unroll
          for (int m = 0; m < (W + 6) / 4; ++m) Bw[m] = m + 1 < (W + 6) / 4 ? Bw[m + 1] : 0u;
        }
        ambm >>= kU;
#pragma unroll
        for (int k = 0; k + 1 < kWin; ++k) rw[k] = rw[k + 1];
        const uint32_t qn = p0 + kU + 4 * (kWin - 1);
        if constexpr ((kVar & 1024) != 0) {
          static_assert(kU == 4, "one aligned word per group");
          const uint32_t wn = qn < nb ? word_at(qn / 4 + 1) : 0u;
          rw[kWin - 1] = qn < nb ? finish(__builtin_amdgcn_alignbyte(wn, wprev, sh), qn) : 0u;
          wprev = wn;
        } else {
          rw[kWin - 1] = qn < nb ? load_rel(qn) : 0u;
        }
      }
    } else {
      uint32_t pos = 0;  // byte offset of the current char position
      while (nb > 0) {
        if (pos > 0) bp_store(pos, pos - B[0]);
        if (pos >= nb) break;
        const float T0 = T[0];
        // Bytes pos .. pos+W-1 of the sentence (packed, little endian).  The
        // trie walk below then depends only on its own unit loads.
        uint32_t win[W / 4];
        {
          const uint64_t lp = lds_off + pos;
          bool from_lds = false;
          if constexpr ((kVar & 1) != 0) from_lds = lp + W + 4 <= kLdsBytes;
          if (from_lds) {
            const uint32_t wi = static_cast<uint32_t>(lp >> 2), sh = static_cast<uint32_t>(lp & 3);
            uint32_t w[W / 4 + 1];
  #pragma unroll
            for (int k = 0; k <= W / 4; ++k) w[k] = lds_bytes[wi + k];
  #pragma unroll
            for (int k = 0; k < W / 4; ++k) win[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
          } else {
  #pragma unroll
            for (int k = 0; k < W / 4; ++k) {
              uint32_t x = 0;
  #pragma unroll
              for (int t = 0; t < 4; ++t) {
                const uint64_t g = b0 + pos + 4 * k + t;
                x |= (g < total_bytes ? static_cast<uint32_t>(a.bytes[g]) : 0u) << (8 * t);
              }
              win[k] = x;
            }
          }
        }
        uint32_t base_u = a.p.root_base;
        uint32_t rem = 0;        // bytes left in the current char (0: next byte starts one)
        uint32_t clen0 = 1;      // byte length of the first char
        uint64_t cbmask = 0;     // bit d: a char ends after byte d
        uint64_t leafmask = 0;   // bit d: a piece ends at a char boundary after byte d
        uint32_t lnode[W];
        bool alive = true, single = false;
        // Phase 1: the walk, one trie edge (one byte) per step; d = byte distance.
        auto walk = [&](auto dc) {
          constexpr int d = decltype(dc)::value;
          const uint32_t c = (win[(d - 1) >> 2] >> (8 * ((d - 1) & 3))) & 0xFFu;
          if (alive) {
            const uint32_t q = pos + d - 1;
            if (q >= nb) {
              alive = false;
            } else {
              if (rem == 0) {
                rem = OneCharLenDev(c);
                if (rem > nb - q) rem = nb - q;
                if (d == 1) clen0 = rem;
              }
              const uint32_t node = base_u ^ c;
              const uint32_t u = c ? unit_at(node) : 0u;
              if ((u & 0xFFu) != c || c == 0) {
                alive = false;
              } else {
                base_u = u >> 9;
                --rem;
                if (rem == 0) cbmask |= 1ull << d;
                if (u & 0x100u) {
                  if (rem != 0) {
                    bad = true;  // leaf inside a UTF-8 char: general path
                  } else {
                    leafmask |= 1ull << d;
                    lnode[d] = node;
                  }
                }
              }
            }
          }
        };
        StaticFor<1, W>(walk);
        // Phase 2: all leaf scores (independent loads), written over lnode[]:
        // a score, or a NaN tag 0x7FC00000|kind for USER_DEFINED / UNUSED.
        auto score = [&](auto dc) {
          constexpr int d = decltype(dc)::value;
          if ((leafmask >> d) & 1) {
            if constexpr ((kVar & 4) != 0) {
              lnode[d] = __float_as_uint(a.vscore[lnode[d]]);
            } else {
              const int32_t v = a.values[lnode[d]];
              const int32_t k = v >> kKindShift;
              lnode[d] = k == 0 ? __float_as_uint(a.scores[v & kIdMask]) : (0x7FC00000u | k);
            }
          }
        };
        StaticFor<1, W>(score);
        // Phase 3: nodes in ascending length, then UNK (begin_nodes_ order).
        auto ins = [&](auto dc) {
          constexpr int d = decltype(dc)::value;
          if ((leafmask >> d) & 1) {
            const uint32_t sb = lnode[d];
            const int32_t kind = (sb & 0x7FFFFFFFu) > 0x7F800000u ? static_cast<int32_t>(sb & 3u) : 0;
            if (kind != kKindUnused) {
              const float s_node =
                  kind == kKindUserDefined
                      ? UserDefinedScore(__popcll(cbmask & ((2ull << d) - 1)), a.p.max_score)
                      : __uint_as_float(sb);
              insert(dc, __fadd_rn(T0, s_node), pos, pos + d);
              if (d == static_cast<int>(clen0)) single = true;
            }
          }
          // UNK node (unigram_model.cc:597-601) at the end of the first char.
          if constexpr (d <= 4) {
            if (d == static_cast<int>(clen0) && !single)
              insert(dc, __fadd_rn(T0, a.p.unk_score), pos, pos + clen0);
          }
        };
        StaticFor<1, W>(ins);
        // Advance one char (clen0 bytes): shift the ring.
        for (uint32_t t = 0; t < clen0; ++t) {
  #pragma unroll
          for (int d = 0; d + 1 < W; ++d) {
            T[d] = T[d + 1];
            B[d] = B[d + 1];
          }
          T[W - 1] = 0.f;
          B[W - 1] = 0;
          has >>= 1;
          ambm >>= 1;
        }
        pos += clen0;
      }
    }

    // Node (b, e) on the best path: exact-match walk, else UNK.
    auto node_of = [&](uint32_t b, uint32_t e, int32_t *id_out, float *sc_out) {
      uint32_t nbase = a.p.root_base, node = 0, u = 0;
      bool found = true;
      for (uint32_t j = b; j < e; ++j) {
        const uint32_t c = byte_at(j);
        node = nbase ^ c;
        u = c ? unit_at(node) : 0u;
        if ((u & 0xFFu) != c || c == 0) {
          found = false;
          break;
        }
        nbase = u >> 9;
      }
      int32_t id = a.p.unk_id;
      float sc = a.p.unk_score;
      if (found && (u & 0x100u)) {
        const int32_t v = a.values[node];
        const int32_t kind = v >> kKindShift;
        if (kind != kKindUnused) {
          id = v & kIdMask;
          if (kind == kKindUserDefined) {
            int chars = 0;
            for (uint32_t j = b; j < e; j += OneCharLenDev(byte_at(j))) ++chars;
            sc = UserDefinedScore(chars, a.p.max_score);
          } else {
            sc = a.scores[id];
          }
        }
      }
      *id_out = id;
      *sc_out = sc;
    };
    // Backtrace from EOS (score 0).  write=false only counts tokens (node
    // scores are needed only to resolve recorded near-ties).
    auto backtrace = [&](bool write, int32_t *out_id, uint32_t *out_len, uint32_t kt) -> uint32_t {
      uint32_t e = nb, k = 0;
      float rs = 0.f;
      while (e > 0) {
        uint32_t b = e - bp_load(e);
#pragma unroll
        for (int t = 0; t < kAmb; ++t)
          if (ae[t] == e && __fadd_rn(aT2[t], rs) == __fadd_rn(aT[t], rs)) b = aB2[t];
        if (write || any_amb) {
          int32_t id;
          float sc;
          node_of(b, e, &id, &sc);
          if (write) {
            out_id[kt - 1 - k] = id;
            if (out_len) out_len[kt - 1 - k] = e - b;
          }
          rs = sc;
        }
        ++k;
        e = b;
      }
      return k;
    };
    uint32_t k = 0;
    if (valid && nb > 0 && !bad) k = backtrace(false, nullptr, nullptr, 0);
    // Group-exclusive scan of the token counts in SENTENCE order (lanes may
    // hold the group's sentences permuted by length): the group's fast-path
    // tokens then form one contiguous range in sentence order, which
    // compact_kernel moves as a block.
    lds_scan[sid] = k;
    __syncthreads();
    const uint32_t kk = lds_scan[tid];
    uint32_t x = kk;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) lds_wave[wave] = x;
    __syncthreads();
    uint32_t ex = x - kk;
    for (int w = 0; w < wave; ++w) ex += lds_wave[w];
    lds_scan[tid] = ex;
    __syncthreads();
    const uint32_t excl = lds_scan[sid];
    __syncthreads();
    if (valid) {
      if (bad) {
        a.ntok[i] = kNone;
        a.lo[i] = kNone;
        const uint32_t fk = atomicAdd(&a.status[0], 1u);
        a.flagged[fk] = static_cast<uint32_t>(i);
        atomicMax(&a.status[1], nb);
      } else {
        const uint64_t dst = a.off[base] + excl;
        if (k) {
          backtrace(true, a.slot_ids + dst, a.slot_len ? a.slot_len + dst : nullptr, k);
        }
        a.ntok[i] = k;
        a.lo[i] = excl;
      }
    }
    if constexpr ((kVar & 1) != 0) __syncthreads();  // staged bytes reused next iteration
  }
}

// ---------------------------------------------------------------------------
// General kernel: the reference Lattice, literally (node lists, Viterbi over
// every (rnode, lnode) pair in end_nodes_ insertion order, strict '>').
// One flagged sentence per lane, scratch slab per lane.
// ---------------------------------------------------------------------------
struct GeneralArgs {
  const uint8_t *__restrict__ bytes;
  const uint64_t *__restrict__ off;
  const uint32_t *__restrict__ units;
  const int32_t *__restrict__ values;
  const float *__restrict__ scores;
  UnigramParams p;
  int32_t *__restrict__ slot_ids;
  uint32_t *__restrict__ slot_len;
  uint32_t *__restrict__ ntok;
  const uint32_t *__restrict__ list;  // sentence indices
  const uint32_t *__restrict__ count; // device count of `list`
  uint64_t list_n;                    // used when count == nullptr
  uint8_t *__restrict__ scratch;
  uint64_t slab_bytes;
  uint32_t max_nb;                    // slab sized for sentences <= max_nb bytes
  uint32_t *__restrict__ error;
};

__global__ __launch_bounds__(64) void unigram_general_kernel(GeneralArgs a) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nthreads = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t total = a.count ? *a.count : a.list_n;
  const int K = a.p.trie_results_size + 1;
  for (uint64_t j = tid; j < total; j += nthreads) {
    const uint32_t i = a.list ? a.list[j] : static_cast<uint32_t>(j);
    const uint64_t b0 = a.off[i];
    const uint32_t nb = static_cast<uint32_t>(a.off[i + 1] - b0);
    if (nb == 0) {
      a.ntok[i] = 0;
      continue;
    }
    if (nb > a.max_nb) {
      atomicOr(a.error, 1u);
      a.ntok[i] = 0;
      continue;
    }
    const uint8_t *__restrict__ s = a.bytes + b0;
    uint8_t *slab = a.scratch + tid * a.slab_bytes;
    const uint32_t cap_nodes = nb * K + 2;
    // Slab carve (all 4-byte arrays).
    uint32_t *cs = reinterpret_cast<uint32_t *>(slab);        // nb + 1
    int32_t *end_head = reinterpret_cast<int32_t *>(cs + nb + 1);
    int32_t *end_tail = end_head + nb + 1;
    int32_t *bfirst = end_tail + nb + 1;
    int32_t *bcount = bfirst + nb + 1;
    float *nscore = reinterpret_cast<float *>(bcount + nb + 1);
    float *nbt = nscore + cap_nodes;
    int32_t *nid = reinterpret_cast<int32_t *>(nbt + cap_nodes);
    int32_t *nprev = nid + cap_nodes;
    int32_t *nnext = nprev + cap_nodes;  // next in end list
    uint32_t *npos = reinterpret_cast<uint32_t *>(nnext + cap_nodes);
    uint32_t *nlen = npos + cap_nodes;

    // SetSentence (:147-187)
    uint32_t nc = 0;
    for (uint32_t q = 0; q < nb;) {
      cs[nc++] = q;
      uint32_t cl = OneCharLenDev(s[q]);
      q += cl < nb - q ? cl : nb - q;
    }
    cs[nc] = nb;
    for (uint32_t p = 0; p <= nc; ++p) {
      end_head[p] = -1;
      end_tail[p] = -1;
      bfirst[p] = 0;
      bcount[p] = 0;
    }
    auto push_end = [&](uint32_t q, int32_t nd) {
      nnext[nd] = -1;
      if (end_tail[q] < 0) end_head[q] = nd;
      else nnext[end_tail[q]] = nd;
      end_tail[q] = nd;
    };
    int32_t nn = 0;
    // BOS
    nscore[0] = 0.f; nbt[0] = 0.f; nid[0] = -1; nprev[0] = -1; npos[0] = 0; nlen[0] = 0;
    push_end(0, 0);
    nn = 1;
    // EOS
    nscore[1] = 0.f; nbt[1] = 0.f; nid[1] = -1; nprev[1] = -1; npos[1] = nc; nlen[1] = 0;
    nn = 2;
    bfirst[nc] = 1;
    bcount[nc] = 1;
    // PopulateNodes (:535-604)
    for (uint32_t p = 0; p < nc; ++p) {
      bfirst[p] = nn;
      bool single = false;
      uint32_t base = a.p.root_base;
      uint32_t cpos = p;  // char index reached by the walk
      for (uint32_t q = cs[p]; q < nb; ++q) {
        const uint32_t c = s[q];
        if (c == 0) break;
        const uint32_t node = base ^ c;
        const uint32_t u = a.units[node];
        if ((u & 0xFFu) != c) break;
        base = u >> 9;
        if (u & 0x100u) {
          const uint32_t e = q + 1;
          while (cs[cpos] < e) ++cpos;  // get_chars_length
          const uint32_t length = cpos - p;
          const int32_t v = a.values[node];
          const int32_t kind = v >> kKindShift;
          if (kind == kKindUnused) continue;
          const int32_t nd = nn++;
          nid[nd] = v & kIdMask;
          nscore[nd] = kind == kKindUserDefined ? UserDefinedScore(length, a.p.max_score)
                                                : a.scores[v & kIdMask];
          npos[nd] = p;
          nlen[nd] = length;
          push_end(p + length, nd);
          if (length == 1) single = true;
        }
      }
      if (!single) {
        const int32_t nd = nn++;
        nid[nd] = a.p.unk_id;
        nscore[nd] = a.p.unk_score;
        npos[nd] = p;
        nlen[nd] = 1;
        push_end(p + 1, nd);
      }
      bcount[p] = nn - bfirst[p];
    }
    // Viterbi (:222-261)
    bool fail = false;
    for (uint32_t p = 0; p <= nc && !fail; ++p) {
      for (int32_t r = bfirst[p]; r < bfirst[p] + bcount[p]; ++r) {
        nprev[r] = -1;
        float best_score = 0.f;
        int32_t best = -1;
        for (int32_t l = end_head[p]; l >= 0; l = nnext[l]) {
          const float sc = __fadd_rn(nbt[l], nscore[r]);
          if (best < 0 || sc > best_score) {
            best = l;
            best_score = sc;
          }
        }
        if (best < 0) {
          fail = true;
          break;
        }
        nprev[r] = best;
        nbt[r] = best_score;
      }
    }
    int32_t *__restrict__ out_id = a.slot_ids + b0 + nb;
    uint32_t *__restrict__ out_len = a.slot_len ? a.slot_len + b0 + nb : nullptr;
    uint32_t k = 0;
    if (!fail) {
      for (int32_t nd = nprev[1]; nd >= 0 && nprev[nd] >= 0; nd = nprev[nd]) {
        ++k;
        out_id[-static_cast<int64_t>(k)] = nid[nd];
        if (out_len) out_len[-static_cast<int64_t>(k)] = cs[npos[nd] + nlen[nd]] - cs[npos[nd]];
      }
    }
    a.ntok[i] = k;
  }
}

}  // namespace

uint64_t UnigramGeneralSlabBytes(uint32_t max_nb, int trie_results_size) {
  const uint64_t nb = max_nb;
  const uint64_t cap_nodes = nb * (trie_results_size + 1) + 2;
  return ((nb + 1) * 5 + cap_nodes * 7) * 4 + 64;
}

hipError_t LaunchUnigramFast(int W, int variant, const UnigramLaunch &l, hipStream_t st) {
  FastArgs a{l.bytes, l.off, l.n, l.units, l.values, l.scores, l.p,
             l.slot_ids, l.slot_len, l.ntok, l.lo, l.bp, l.flagged, l.status, l.vscore, l.num_units, l.jump2};
  const uint64_t blocks64 = (l.n + kBlock - 1) / kBlock;
  const unsigned blocks = static_cast<unsigned>(blocks64 < (1u << 30) ? blocks64 : (1u << 30));
  if (blocks == 0) return hipSuccess;
#define SPM_FAST_CASE(WW, VV) \
  case WW * 524288 + VV:      \
    hipLaunchKernelGGL((unigram_fast_kernel<WW, VV>), dim3(blocks), dim3(kBlock), 0, st, a); break;
  switch (W * 524288 + (variant & 524287)) {
    // 1274 = 1272 + LDS trie top (1024 units): measured 6.39 vs 6.17 ms per
    // 10M sentences (2048 units 6.43, 4096 units 8.34; profiles/r02b_variant_ab.txt).
    SPM_FAST_CASE(16, 0) SPM_FAST_CASE(16, 7) SPM_FAST_CASE(16, 1272) SPM_FAST_CASE(16, 1274)
    SPM_FAST_CASE(16, 5368)
    SPM_FAST_CASE(16, 17656) SPM_FAST_CASE(16, 50424) SPM_FAST_CASE(16, 115960)  // + diet (+ 5 / 6 waves)
    SPM_FAST_CASE(16, 247032) SPM_FAST_CASE(16, 509176)  // + diet, 7 waves (2 / 1 near-tie entries)
    SPM_FAST_CASE(32, 0) SPM_FAST_CASE(32, 7)
    SPM_FAST_CASE(64, 0) SPM_FAST_CASE(64, 7)
    default: return hipErrorInvalidValue;
  }
#undef SPM_FAST_CASE
  return hipGetLastError();
}

hipError_t LaunchUnigramGeneral(const UnigramLaunch &l, const uint32_t *list, const uint32_t *count,
                                uint64_t list_n, uint8_t *scratch, uint64_t slab_bytes,
                                uint32_t max_nb, uint32_t threads, uint32_t *error,
                                hipStream_t st) {
  GeneralArgs a{l.bytes, l.off, l.units, l.values, l.scores, l.p, l.slot2_ids, l.slot2_len,
                l.ntok, list, count, list_n, scratch, slab_bytes, max_nb, error};
  const unsigned blocks = (threads + 63) / 64;
  hipLaunchKernelGGL(unigram_general_kernel, dim3(blocks), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace spm_amd
