// Wave-cooperative unigram encode for gfx950 (MI355X): ONE sentence per
// wavefront, for the sentences the lane-per-sentence fast kernels hand over
// (long lines of real text) and for few-sentence calls at
// the plugin point (ModelInterface::Encode, model_interface.h:117, called once
// per line by spm_encode_main.cc:189-191).
//
// Reference: Lattice::SetSentence / Insert / Viterbi (unigram_model.cc:
// 147-261) and Model::PopulateNodes (:535-604), restated by byte position:
//   * char starts are the lead-byte chain of OneCharLen from 0, clamped to
//     the sentence (util.h:389); the kernel accepts a sentence only when that
//     chain equals "every non-continuation byte" (valid structure), so a
//     char start is a non-continuation byte;
//   * begin_nodes_[p] = the trie's prefix matches at p in ascending length
//     (UNUSED skipped; USER_DEFINED scored length * max_score + 1.0), with an
//     UNK node of one char (min_score - 10) when no one-char node exists —
//     either way the one-char node is the shortest, slot 0;
//   * end_nodes_[e] is in ascending begin order (one node per (begin, end));
//   * Viterbi: per begin position in ascending order, every rnode takes the
//     FIRST lnode with the maximal float backtrace_score + rnode score
//     (strict `>`), BOS has backtrace_score 0, EOS has score 0.
// Sentences with a trie leaf inside a UTF-8 char, more than kCK nodes at one
// position, a 0xFF byte (the walk's 0xFF-padded table) or malformed UTF-8 go
// to the general kernel (the reference lattice literally), so every
// sentence's result is the reference's.
//
// Work per sentence, in windows of 64 CHARS (lane r = the window's r-th char
// start; a window spans at most 192 bytes):
//   1. lattice: every lane walks the trie from its char start through the
//      (unit, node score) table (root level in LDS), keeping its nodes'
//      scores in registers (slot 0 the one-char node, then ascending length)
//      and writing a length bit mask into an LDS ring of 256 byte positions
//      (the window + the 64-byte lookback any node reaches); the nodes are
//      numbered densely in (char, slot) order (a wave prefix sum of the
//      lanes' node counts) and their trie nodes go to global scratch, with
//      each char's first node index;
//   2. Viterbi over the window's char starts in order: lane L-1 reads the
//      mask and backtrace scores of the position L bytes back in one LDS
//      round, the rnodes at e (slot r on lane r, scores broadcast from the
//      walker lane) fold the candidates in ascending begin order with
//      readlane broadcasts; each rnode's chosen lnode (length, slot, chars)
//      goes to global scratch at the rnode's dense index;
//   3. backtrace from EOS through the scratch (64-char blocks staged in LDS
//      from the dense arrays), tokens (dense node index, length) written
//      right-aligned in the sentence's slot range;
//   4. ids from the trie nodes, lanes in parallel.
// Scratch per char: 4 B of first index + 6 B per node (~2.5 nodes per char
// on Japanese text), instead of 8 slots x 6 B (round 5: 37x the algorithmic
// bytes in HBM traffic per Japanese launch).
// A sentence's trie walks run 64 at a time instead of one after the other in
// a single lane, which is what bounds the lane kernels on long lines (one
// lane's chain of dependent trie loads) and on one-sentence calls.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "epilogue.h"
#include "kernels.h"
#include "normalize_prefix.h"

namespace spm_amd {
namespace {

constexpr int kCK = kCoopSlots;  // node slots per char start
constexpr int kCPos = 256;       // LDS ring of byte positions
constexpr int kCWaves = 4;       // waves (independent sentences) per block
constexpr uint32_t kCSpan = 192; // bytes a window may span

struct CoopWave {
  // Per byte position (ring): bit L-1 = a node of L bytes begins here
  // (0: no char start), and the nodes' Viterbi backtrace scores by slot.
  uint64_t lmask[kCPos];
  union {
    float bt[kCPos][kCK];
    struct {                      // backtrace: a 64-char block of
      uint32_t pv[64][kCK];       //   (chosen lnode (length | slot << 7 | chars << 10) | node index
                                  //   - the block's first << 16) by (char, slot), and
      uint16_t dpv[64 * kCK];     //   the dense window of chosen lnodes the rows come from
    } b;
  } u;
  uint8_t ordlo[kCPos];         // per byte position (ring): low 8 bits of its char ordinal
  uint32_t bytes[kCPos / 4];    // sentence bytes [w, w + 256) of the current window
  uint32_t start[64];           // the window's char starts
  float score[64][kCK];         // node scores of the window's k-th char start, by slot
};

__device__ __forceinline__ bool Cont(uint32_t c) { return (c & 0xC0u) == 0x80u; }

// LDS written by some lanes is read by others of the same wave: keep the
// compiler's order (the wave issues LDS operations in order).
__device__ __forceinline__ void WaveSync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float ReadLaneF(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Encodes sentence [b0, b0 + nb) with one wave (wave slab `wid` when
// a.slab_chars != 0).  Tokens are written into slot_ids[b0 + nb - ntok, b0 +
// nb) (and slot_len), in order; returns ntok, or kNone when the sentence needs
// the general kernel.  Wave-uniform result.
// kLdsTrie (the one-block small calls, when the model's whole (unit, score)
// table fits kCoopLdsUnits): the lattice's trie steps read `trie`, the table
// staged in LDS, instead of the L2 — a call is one wave's latency chain, and
// its walks are a chain of dependent loads (r06z: 22 k of a botchan line's
// 122 k cycles).
template <bool kLdsTrie = false>
__device__ uint32_t CoopEncodeSentence(const CoopArgs &a, CoopWave &W, const uint2 *lds_root, uint64_t b0,
                                       uint32_t nb, uint64_t wid, const uint2 *trie = nullptr) {
  const int lane = threadIdx.x & 63;
  // Wave-uniform by contract; made provably so, so that the window / Viterbi /
  // backtrace control (e, L, slot) lives in scalar registers with scalar
  // branches instead of exec-mask branching.
  nb = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(nb)));
  if (nb == 0) return 0;
  const uint8_t *__restrict__ g = a.bytes + b0;
  // Scratch: the sentence's (or the wave slab's) region of kCK entries per
  // char (a sentence has at most nb chars), used DENSELY: a char has at most
  // kCK - 1 nodes, numbered in (char, slot) order; the chosen lnode (pv_g)
  // and trie node (nd_g) of node j at index j, and each char's first node
  // index (nb_g) in the last 1/kCK of the node region.
  const uint64_t row0 = a.slab_chars ? wid * a.slab_chars : b0;
  const uint32_t max_chars = a.slab_chars ? static_cast<uint32_t>(a.slab_chars) : nb;
  uint16_t *__restrict__ pv_g = a.pv_scratch + row0 * kCK;
  uint32_t *__restrict__ nd_g = a.nd_scratch + row0 * kCK;
  uint32_t *__restrict__ nb_g = nd_g + static_cast<uint64_t>(max_chars) * (kCK - 1);
  uint32_t wo = 0, nch = 0;  // char ordinal of the window's first char start; chars of the sentence
  uint32_t node_run = 0;     // nodes of the windows before this one
  uint32_t wbase = 0;        // lane i < 64: the first node index of char 64 i
  const uint2 *__restrict__ uvs = reinterpret_cast<const uint2 *>(a.uvs);
  uint32_t eos_pv = 0;
  bool bad = false;
  uint32_t w = 0;
  // SPM_HIP_COOP_PROF: shader-clock cycles per phase (a.prof[0..4]: window
  // setup, lattice, Viterbi, backtrace, ids), summed by lane 0 of each wave.
  uint64_t t_setup = 0, t_lat = 0, t_vit = 0;
  uint64_t t0 = a.prof ? clock64() : 0;
  for (;;) {
    // Window bytes [w, w + 256), zero past the sentence; char starts.
    const uint32_t q4 = w + 4u * static_cast<uint32_t>(lane);
    uint32_t x = 0;
    if (q4 + 4 <= nb) {
      x = static_cast<uint32_t>(g[q4]) | static_cast<uint32_t>(g[q4 + 1]) << 8 |
          static_cast<uint32_t>(g[q4 + 2]) << 16 | static_cast<uint32_t>(g[q4 + 3]) << 24;
    } else {
      for (uint32_t t = 0; t < 4; ++t)
        if (q4 + t < nb) x |= static_cast<uint32_t>(g[q4 + t]) << (8 * t);
    }
    W.bytes[lane] = x;
    uint32_t nib = 0;
    for (uint32_t t = 0; t < 4; ++t) {
      const uint32_t c = (x >> (8 * t)) & 0xFFu;
      if (q4 + t < nb) {
        if (c == 0xFFu) bad = true;  // matches the walk table's padding: general path
        if (!Cont(c) && q4 + t < w + kCSpan) nib |= 1u << t;
      }
    }
    // Exclusive prefix of the lanes' start counts.
    const uint32_t cnt = __popc(nib);
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    uint32_t r = incl - cnt;
    for (uint32_t t = 0; t < 4; ++t)
      if ((nib >> t) & 1) {
        if (r < 64) W.start[r] = q4 + t;
        ++r;
      }
    const uint32_t total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
    const uint32_t T = total < 64 ? total : 64;
    // The window: char starts [0, T), bytes [w, w_end).
    WaveSync();
    const uint32_t w_end = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(
        T == 64 && total > 64 ? W.start[63] + 1 : (nb + 1 < w + kCSpan ? nb + 1 : w + kCSpan))));
    if (w == 0 && (T == 0 || W.start[0] != 0)) bad = true;  // byte 0 must start a char
    if (wo + T > max_chars) bad = true;                     // outgrows the wave's slab
    // Clear the ring's masks of the window's positions (continuation bytes
    // keep mask 0: the Viterbi's candidate test reads them).
    for (uint32_t q = w + static_cast<uint32_t>(lane); q < w_end; q += 64) W.lmask[q & (kCPos - 1)] = 0;
    WaveSync();
    auto sb = [&](uint32_t q) -> uint32_t {  // byte q of the sentence, q in [w, w + 256)
      const uint32_t rr = q - w;
      return (W.bytes[rr >> 2] >> (8 * (rr & 3))) & 0xFFu;
    };
    uint64_t t1 = a.prof ? clock64() : 0;
    t_setup += t1 - t0;
    // ---- 1. lattice of the window's char starts (lane k: the k-th; its
    // nodes' scores stay in its registers, slot 0 = the one-char node).
    uint32_t p = 0, ncnt = 0;  // char start; its node count
    uint64_t bits = 0;
    float sc[kCK];
    uint32_t ndr[kCK];  // the nodes' trie units by slot (kNone: UNK)
#pragma unroll
    for (int k = 0; k < kCK; ++k) {
      sc[k] = 0.f;
      ndr[k] = 0;
    }
    if (static_cast<uint32_t>(lane) < T && !bad) {
      p = W.start[lane];
      const uint32_t c0 = sb(p);
      uint32_t clen = OneCharLenDev(c0);
      if (clen > nb - p) clen = nb - p;
      // The chain must equal the non-continuation bytes: the char's other
      // bytes are continuation bytes and the next byte starts a char.
      for (uint32_t j = 1; j < clen; ++j)
        if (!Cont(sb(p + j))) bad = true;
      if (p + clen < nb && Cont(sb(p + clen))) bad = true;
      uint32_t base = a.p.root_base, nlong = 0;
      bool single = false;
      for (uint32_t d = 1; d <= a.max_len && !bad; ++d) {
        const uint32_t q = p + d - 1;
        if (q >= nb) break;
        const uint32_t c = sb(q);
        const uint32_t node = base ^ c;
        const uint2 ux = d == 1 ? lds_root[c]
                         : (node < a.num_units ? (kLdsTrie ? trie[node] : uvs[node]) : make_uint2(0xFFu, 0u));
        if ((ux.x & 0xFFu) != c) break;
        base = ux.x >> 9;
        if (ux.x & 0x100u) {
          const uint32_t e = p + d;
          if (e < nb && Cont(sb(e))) {  // a leaf inside a UTF-8 char
            bad = true;
            break;
          }
          const float s_node = __uint_as_float(ux.y);
          if (__builtin_isnan(s_node)) continue;  // no usable node (UNUSED)
          uint32_t slot;
          if (d == clen) {
            single = true;
            slot = 0;
          } else {
            if (nlong + 1 == kCK) {
              bad = true;
              break;
            }
            slot = ++nlong;
          }
#pragma unroll
          for (int k = 0; k < kCK; ++k)
            if (static_cast<uint32_t>(k) == slot) {
              sc[k] = s_node;
              ndr[k] = node;
            }
          bits |= 1ull << (d - 1);
        }
      }
      if (!single) {
        // UNK node of one char (unigram_model.cc:597-601).
        sc[0] = a.p.unk_score;
        ndr[0] = kNone;
        bits |= 1ull << (clen - 1);
      }
      ncnt = nlong + 1;
      W.lmask[p & (kCPos - 1)] = bits;
      W.ordlo[p & (kCPos - 1)] = static_cast<uint8_t>(wo + static_cast<uint32_t>(lane));
      reinterpret_cast<float4 *>(W.score[lane])[0] = make_float4(sc[0], sc[1], sc[2], sc[3]);
      reinterpret_cast<float4 *>(W.score[lane])[1] = make_float4(sc[4], sc[5], sc[6], sc[7]);
    }
    bad = __builtin_amdgcn_ballot_w64(bad) != 0;
    if (bad) break;
    // Dense node numbering: the window's chars' nodes follow the earlier
    // windows', in char order; each lane stores its char's first index and
    // its nodes (one contiguous run over the wave).
    uint32_t nincl = ncnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(nincl, o);
      if (lane >= o) nincl += y;
    }
    const uint32_t nbk = node_run + nincl - ncnt;
    if (static_cast<uint32_t>(lane) < T) {
      nb_g[wo + static_cast<uint32_t>(lane)] = nbk;
#pragma unroll
      for (int k = 0; k < kCK - 1; ++k)
        if (static_cast<uint32_t>(k) < ncnt) nd_g[nbk + k] = ndr[k];
    }
    // (Windows hold <= 64 chars, not always 64: the 64-char blocks' first
    // indices come from the lanes whose char ordinal is a multiple of 64.)
    for (uint64_t m = __builtin_amdgcn_ballot_w64(static_cast<uint32_t>(lane) < T && ((wo + lane) & 63u) == 0);
         m != 0; m &= m - 1) {
      const int j = __builtin_ctzll(m);
      const uint32_t v = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(nbk), j));
      if (static_cast<uint32_t>(lane) == ((wo + static_cast<uint32_t>(j)) >> 6)) wbase = v;
    }
    node_run += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(nincl), 63));
    WaveSync();
    uint64_t t2 = a.prof ? clock64() : 0;
    t_lat += t2 - t1;
    // ---- 2. Viterbi over the window's char starts, then EOS.  Iteration
    // k: e = the k-th start and its nodes' scores (lane k's registers,
    // broadcast); lane L-1 reads the lnode of L bytes ending at e (mask and
    // scores of its begin in one LDS round); the rnodes at e (slot r on lane
    // r) fold the candidates in ascending begin order.
    const bool has_eos = nb < w_end;
    const uint32_t maxl = a.max_len;
    const uint32_t kend = T + (has_eos ? 1u : 0u);
    const uint32_t L = static_cast<uint32_t>(lane) + 1;
    // Lane L-1: the position L bytes back — its mask and all its slots'
    // backtrace scores, and the rnode scores, in ONE LDS round: the reads
    // are unconditional (ring addresses are always in range; score row k & 63
    // is read but unused at EOS).  (Issuing iteration k + 1's round before
    // iteration k's fold, with the one operand it cannot see yet — the
    // one-char node of e_k — forwarded through a readlane, measured slower
    // both in the many-wave list kernel, 48.8 vs 45.2 ms per ja batch, and
    // for one wave alone, 57.8k vs 53.4k Viterbi cycles per botchan line:
    // the loop is bound by its instruction chain, not the LDS round.)
    uint32_t ne = 0, nblo = 0, nbhi = 0, nolo = 0;
    float ns = 0.f;
    uint64_t nlmb = 0;
    float4 nb0v = make_float4(0.f, 0.f, 0.f, 0.f), nb1v = nb0v;
    auto load_ops = [&](uint32_t k) {
      ne = k == T ? nb : static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(p), k));
      nblo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(bits), k));
      nbhi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(bits >> 32), k));
      const uint32_t br = (ne - L) & (kCPos - 1);
      ns = W.score[k & 63u][lane];
      nlmb = W.lmask[br];
      nolo = W.ordlo[br];
      nb0v = reinterpret_cast<const float4 *>(W.u.bt[br])[0];
      nb1v = reinterpret_cast<const float4 *>(W.u.bt[br])[1];
    };
    for (uint32_t k = 0; k < kend; ++k) {
      const bool eos = k == T;
      load_ops(k);
      const uint32_t e = ne, blo = nblo, bhi = nbhi, olo = nolo;
      const float s_all = ns;
      const uint64_t lmb = nlmb;
      const float4 b0v = nb0v, b1v = nb1v;
      // (pinned above the branches, so the compiler cannot sink the score
      // reads behind the mask's wait)
      asm volatile("" ::"v"(s_all), "v"(olo), "v"(b0v.x), "v"(b0v.y), "v"(b0v.z), "v"(b0v.w), "v"(b1v.x),
                   "v"(b1v.y), "v"(b1v.z), "v"(b1v.w));
      const int cnt_e = eos ? 1 : __popc(blo) + __popc(bhi);
      const float s_r = (!eos && lane < cnt_e) ? s_all : 0.f;
      const bool valid = L <= e && L <= maxl && ((lmb >> lane) & 1);
      const uint32_t rank = __popcll(lmb & ((1ull << lane) - 1));
      // Slot `rank` (< kCK = 8 on a valid lane) by a 3-level select tree.
      static_assert(kCK == 8, "select tree over 8 slots");
      const bool r1 = (rank & 1u) != 0, r2 = (rank & 2u) != 0, r4 = (rank & 4u) != 0;
      const float m0 = r1 ? b0v.y : b0v.x, m1 = r1 ? b0v.w : b0v.z;
      const float m2 = r1 ? b1v.y : b1v.x, m3 = r1 ? b1v.w : b1v.z;
      const float n0 = r2 ? m1 : m0, n1 = r2 ? m3 : m2;
      const float btc = r4 ? n1 : n0;
      uint64_t cm = __builtin_amdgcn_ballot_w64(valid);
      float best = 0.f;
      uint32_t best_pv = 0;  // chosen lnode: length | slot << 7 | chars << 10 (0: BOS)
      if (e == 0) {
        best = __fadd_rn(0.f, s_r);  // BOS (backtrace score 0)
      } else {
        if (cm == 0) bad = true;  // no lnode: inconsistent lattice
        // Ascending begin = descending length; the first candidate seeds the
        // running max, later ones replace it only when strictly greater
        // (selects, no exec-mask branch per candidate).
        if (cm) {
          int j = 63 - __builtin_clzll(cm);
          cm &= ~(1ull << j);
          // Each lnode's (length | slot << 7 | chars << 10) code, formed once
          // per lane; chars = ordinal of e (wo + k, also at EOS) - its begin's.
          const uint32_t code = L | rank << 7 | ((wo + k - olo) & 0xFFu) << 10;
          best = __fadd_rn(ReadLaneF(btc, j), s_r);
          best_pv = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(code), j));
          while (cm) {
            j = 63 - __builtin_clzll(cm);
            cm &= ~(1ull << j);
            const float v = __fadd_rn(ReadLaneF(btc, j), s_r);
            const uint32_t cand = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(code), j));
            const bool better = v > best;
            best = better ? v : best;
            best_pv = better ? cand : best_pv;
          }
        }
      }
      if (eos) {
        eos_pv = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(best_pv)));
      } else if (lane < cnt_e) {
        W.u.bt[e & (kCPos - 1)][lane] = best;
        // The char's nodes are dense from its first index (lane k's).
        const uint32_t nbe = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(nbk), k));
        pv_g[nbe + static_cast<uint32_t>(lane)] = static_cast<uint16_t>(best_pv);
      }
      WaveSync();
    }
    if (__builtin_amdgcn_ballot_w64(bad) != 0) return kNone;
    t0 = a.prof ? clock64() : 0;
    t_vit += t0 - t2;
    if (has_eos) {
      nch = wo + T;
      break;
    }
    wo += T;
    w = w_end;
  }
  if (bad) return kNone;
  // The global scratch written above is read below by other lanes.
  __threadfence_block();
  WaveSync();
  const uint64_t t3 = a.prof ? clock64() : 0;
  // ---- 3. backtrace from EOS over the per-char rows: each token is the
  // (begin ordinal, slot) of its lnode; its byte length comes with the code.
  // (e, oe, L, slot, chars are wave-uniform: kept in scalar registers.)
  uint32_t e = nb, oe = nch, L = eos_pv & 0x7Fu, slot = (eos_pv >> 7) & 7u, dch = eos_pv >> 10, ntok = 0;
  uint32_t bw = ~0u, cur_b0 = 0;  // the staged block; its first char's node index
  int32_t *__restrict__ out = a.slot_ids + b0 + nb;
  uint32_t *__restrict__ out_len = a.slot_len ? a.slot_len + b0 + nb : nullptr;
  // The chain moves down one 64-char block at a time (a node spans < 64
  // chars).  A block [wb, wb + 64) is staged from its chars' first node
  // indices and the dense window [lo, hi) of chosen lnodes that holds their
  // nodes (hi: the next block's first index, or the sentence's node count;
  // a block has at most 64 (kCK - 1) nodes), expanded in LDS to rows by
  // (char, slot) of (chosen lnode | node index - the block's first << 16),
  // so a token costs one LDS read, as with per-char scratch rows.  The next
  // lower block is fetched into registers as soon as a block is staged, so
  // crossing into it costs LDS work, not a global round trip.
  uint4 pf_pv = make_uint4(0, 0, 0, 0);
  uint32_t pf_nb = 0, pf_nx = 0, pf_lo = 0, pf_b = ~0u;
  auto fetch = [&](uint32_t wb, uint32_t hi, uint32_t &v_nb, uint32_t &v_nx, uint4 &v_pv, uint32_t &lo) {
    constexpr uint32_t kNeed = 64 * (kCK - 1);
    lo = (hi > kNeed ? hi - kNeed : 0u) & ~static_cast<uint32_t>(kCK - 1);
    const uint32_t q = wb + static_cast<uint32_t>(lane);
    v_nb = q < nch ? nb_g[q] : hi;
    v_nx = q + 1 < nch && lane < 63 ? nb_g[q + 1] : hi;  // the next char's (the block's end: hi)
    const uint32_t j = lo + kCK * static_cast<uint32_t>(lane);
    if (j < hi) v_pv = *reinterpret_cast<const uint4 *>(pv_g + j);
  };
  while (e > 0) {
    if (L == 0 || L > e || dch == 0 || dch > oe) return kNone;  // inconsistent chain: general path
    const uint32_t ob = oe - dch;
    const uint32_t wb = ob & ~63u;
    if (wb != bw) {
      if (bw != ~0u && wb + 64 != bw) return kNone;  // (blocks are visited top down, adjacent)
      // (The first block staged may lie below the sentence's last block:
      // the next one's first index from the windows' register, or loaded.)
      const uint32_t wnext = (wb >> 6) + 1;
      const uint32_t hi = bw != ~0u ? cur_b0
                          : wb + 64 >= nch ? node_run
                          : wnext < 64 ? static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wbase), wnext))
                                       : nb_g[wb + 64];
      WaveSync();
      if (wb != pf_b) fetch(wb, hi, pf_nb, pf_nx, pf_pv, pf_lo);
      reinterpret_cast<uint4 *>(W.u.b.dpv)[lane] = pf_pv;
      const uint32_t mine = pf_nb, lo = pf_lo, cnt_l = pf_nx - pf_nb;  // 0 past the sentence's chars
      cur_b0 = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(pf_nb)));
      if (__builtin_amdgcn_ballot_w64(cnt_l > kCK - 1 || mine < lo || mine + cnt_l > hi) != 0)
        return kNone;  // inconsistent numbering: general path
      WaveSync();
      // Whole rows, no exec-mask branches: slots past a char's nodes (and
      // rows past the sentence) get entries no chain reads.
      static_assert(kCK == 8, "rows of two 16-byte stores");
      uint32_t r[kCK - 1];
#pragma unroll
      for (int s = 0; s < kCK - 1; ++s) r[s] = W.u.b.dpv[min(mine - lo + s, 64u * kCK - 1u)];
      const uint32_t rel = (mine - cur_b0) << 16;
      reinterpret_cast<uint4 *>(W.u.b.pv[lane])[0] =
          make_uint4(r[0] | rel, r[1] | (rel + (1u << 16)), r[2] | (rel + (2u << 16)), r[3] | (rel + (3u << 16)));
      reinterpret_cast<uint4 *>(W.u.b.pv[lane])[1] =
          make_uint4(r[4] | (rel + (4u << 16)), r[5] | (rel + (5u << 16)), r[6] | (rel + (6u << 16)), 0u);
      bw = wb;
      if (wb >= 64) {
        pf_b = wb - 64;
        fetch(pf_b, cur_b0, pf_nb, pf_nx, pf_pv, pf_lo);
      }
      WaveSync();
    }
    const uint32_t px = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(W.u.b.pv[ob - wb][slot])));
    const uint32_t pv = px & 0xFFFFu, node_ix = cur_b0 + (px >> 16);  // (the slot is in the offset)
    ++ntok;
    // Every lane stores the same word (one store, no divergent branch): the
    // lnode's dense node index, resolved to an id below.
    out[-static_cast<int64_t>(ntok)] = static_cast<int32_t>(node_ix);
    if (out_len) out_len[-static_cast<int64_t>(ntok)] = L;
    e -= L;
    oe = ob;
    L = pv & 0x7Fu;
    slot = (pv >> 7) & 7u;
    dch = pv >> 10;
  }
  if (L != 0 || oe != 0) return kNone;  // the chain must end at BOS
  __threadfence_block();
  WaveSync();
  const uint64_t t4 = a.prof ? clock64() : 0;
  // ---- 4. ids from the trie nodes.
  int32_t *__restrict__ tok = out - ntok;
  for (uint32_t t = static_cast<uint32_t>(lane); t < ntok; t += 64) {
    const uint32_t node = nd_g[static_cast<uint32_t>(tok[t])];  // one independent gather per token
    tok[t] = node == kNone ? a.p.unk_id : (a.values[node] & kIdMask);
  }
  if (a.prof && lane == 0) {
    const uint64_t t5 = clock64();
    atomicAdd(reinterpret_cast<unsigned long long *>(a.prof + 0), static_cast<unsigned long long>(t_setup));
    atomicAdd(reinterpret_cast<unsigned long long *>(a.prof + 1), static_cast<unsigned long long>(t_lat));
    atomicAdd(reinterpret_cast<unsigned long long *>(a.prof + 2), static_cast<unsigned long long>(t_vit));
    atomicAdd(reinterpret_cast<unsigned long long *>(a.prof + 3), static_cast<unsigned long long>(t4 - t3));
    atomicAdd(reinterpret_cast<unsigned long long *>(a.prof + 4), static_cast<unsigned long long>(t5 - t4));
    atomicAdd(reinterpret_cast<unsigned long long *>(a.prof + 5), static_cast<unsigned long long>(nb));
    atomicAdd(reinterpret_cast<unsigned long long *>(a.prof + 6), static_cast<unsigned long long>(nch));
    atomicAdd(reinterpret_cast<unsigned long long *>(a.prof + 7), static_cast<unsigned long long>(ntok));
  }
  return ntok;
}

// Sentences of a device list (or all n): ntok[i] + right-aligned slots, or
// the sentence appended to rest (general kernel).
__global__ __launch_bounds__(64 * kCWaves) void coop_list_kernel(CoopArgs a) {
  __shared__ CoopWave lds[kCWaves];
  __shared__ uint2 lds_root[256];  // (unit, score) of the root's children
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (a.chain && *a.chain) return;
  {
    const uint32_t nd = a.p.root_base ^ static_cast<uint32_t>(threadIdx.x);
    lds_root[threadIdx.x] = nd < a.num_units ? reinterpret_cast<const uint2 *>(a.uvs)[nd] : make_uint2(0xFFu, 0u);
  }
  __syncthreads();
  CoopWave &W = lds[wave];
  const uint64_t count = a.list ? static_cast<uint64_t>(*a.count) : a.list_n;
  const uint64_t waves = static_cast<uint64_t>(gridDim.x) * kCWaves;
  const uint64_t n_long = a.part ? *a.part_long : 0;
  uint64_t k = static_cast<uint64_t>(blockIdx.x) * kCWaves + wave;
  for (;;) {
    if (a.queue) {  // dynamic: the next unclaimed entry (long sentences first)
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(a.queue, 1u);
      k = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(t)));
    }
    if (k >= count) break;
    const uint64_t i = a.part ? (k < n_long ? a.part[k] : a.part[a.part_n - 1 - (k - n_long)])
                              : (a.list ? a.list[k] : k);
    if (!a.queue) k += waves;
    const uint64_t b0 = a.off[i];
    const uint32_t nb = static_cast<uint32_t>(a.off[i + 1] - b0);
    const uint32_t nt =
        CoopEncodeSentence(a, W, lds_root, b0, nb, static_cast<uint64_t>(blockIdx.x) * kCWaves + wave);
    if (lane == 0) {
      if (nt == kNone) a.rest[atomicAdd(a.rest_count, 1u)] = static_cast<uint32_t>(i);
      else a.ntok[i] = nt;
    }
  }
}

// Block-shared state of the one-block small calls (one block per CU at
// ~120 KB of LDS: these kernels run one block).
constexpr uint32_t kCoopLdsUnits = 8192;  // 64 KB of (unit, score) pairs
struct CoopShared {
  CoopWave lds[kCWaves];
  uint2 lds_root[256];  // (unit, score) of the root's children
  uint2 trie[kCoopLdsUnits];  // the whole table, when a.num_units <= kCoopLdsUnits
  uint32_t ntok[kCoopSmallMax + 1];
  uint32_t failed;
};

__device__ __forceinline__ bool CoopTrieFits(const CoopArgs &a) { return a.num_units <= kCoopLdsUnits; }

// The model's (unit, score) table into sh.trie when it fits (once per
// launch: the resident server keeps it across requests).
__device__ void CoopStageTrie(const CoopArgs &a, CoopShared &sh) {
  if (!CoopTrieFits(a)) return;
  const uint4 *src = reinterpret_cast<const uint4 *>(a.uvs);  // 16-byte aligned device table
  uint4 *dst = reinterpret_cast<uint4 *>(sh.trie);
  for (uint32_t k = threadIdx.x; 2 * k + 1 < a.num_units; k += 64 * kCWaves) dst[k] = src[k];
  if ((a.num_units & 1u) && threadIdx.x == 0)
    sh.trie[a.num_units - 1] = reinterpret_cast<const uint2 *>(a.uvs)[a.num_units - 1];
}

__device__ void CoopStageAndRoot(const CoopArgs &a, const uint32_t *stage_src, uint32_t *stage_dst, uint32_t words,
                                 CoopShared &sh, bool stage_trie) {
  const int tid = threadIdx.x;
  if (stage_trie) CoopStageTrie(a, sh);
  // System-scope loads: the staging area is host memory the host rewrites
  // between the requests of one resident server launch (no cache may hold it).
  for (uint32_t k = static_cast<uint32_t>(tid); k < words; k += 64 * kCWaves)
    stage_dst[k] = __hip_atomic_load(const_cast<uint32_t *>(stage_src) + k, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
  const uint32_t nd = a.p.root_base ^ static_cast<uint32_t>(tid);
  sh.lds_root[tid] = nd < a.num_units ? reinterpret_cast<const uint2 *>(a.uvs)[nd] : make_uint2(0xFFu, 0u);
  if (tid == 0) sh.failed = 0;
  __threadfence_block();
  __syncthreads();
}

// Publishes a small call's completion: host_pub[1] (0 done / 1 not taken),
// then the sequence word, after a system-scope fence over the outputs.
__device__ void CoopPublish(const CoopCall &c, bool ok) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    c.host_pub[1] = ok ? 0u : 1u;
    __threadfence_system();
    __hip_atomic_store(&c.host_pub[0], c.pub_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// One block, n <= kCoopSmallMax sentences of a host call (EncodeHostSmall):
// the input image (offsets, bytes) comes from pinned host memory (staged at
// s.stage_dst: a.off, the bytes at a.bytes + c.in_at), the waves encode
// sentences w, w + 4, ..., and the block writes the final token offsets, ids
// and piece lengths straight into pinned host memory, then the status word
// and the sequence number the host polls for.  A sentence the cooperative
// kernel does not take sets the status (the host re-runs the call on the
// lane kernels).
__device__ void CoopSmallBody(const CoopSmallArgs &s, const CoopCall &c, CoopShared &sh, bool stage_trie) {
  const CoopArgs &a = s.a;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  CoopStageAndRoot(a, s.stage_src, s.stage_dst, c.stage_words, sh, stage_trie);
  const bool in_lds = CoopTrieFits(a);
  for (uint32_t i = static_cast<uint32_t>(wave); i < c.n; i += kCWaves) {
    const uint64_t b0 = c.in_at + a.off[i];
    const uint32_t nb = static_cast<uint32_t>(a.off[i + 1] - a.off[i]);
    const uint32_t nt = in_lds ? CoopEncodeSentence<true>(a, sh.lds[wave], sh.lds_root, b0, nb,
                                                          static_cast<uint64_t>(wave), sh.trie)
                               : CoopEncodeSentence(a, sh.lds[wave], sh.lds_root, b0, nb, static_cast<uint64_t>(wave));
    if (lane == 0) {
      if (nt == kNone) sh.failed = 1;
      sh.ntok[i] = nt;
    }
  }
  __threadfence_block();
  __syncthreads();
  const bool ok = sh.failed == 0;
  if (ok && tid == 0) {  // token offsets (n <= kCoopSmallMax: one thread)
    uint64_t t = 0;
    c.tok[0] = 0;
    for (uint32_t i = 0; i < c.n; ++i) {
      const uint32_t nt = sh.ntok[i];
      sh.ntok[i] = static_cast<uint32_t>(t);
      t += nt;
      c.tok[i + 1] = t;
    }
    sh.ntok[c.n] = static_cast<uint32_t>(t);
  }
  __syncthreads();
  if (ok) {
    for (uint32_t i = static_cast<uint32_t>(wave); i < c.n; i += kCWaves) {
      const uint32_t t0 = sh.ntok[i], nt = sh.ntok[i + 1] - t0;
      const uint64_t src = c.in_at + a.off[i + 1] - nt;
      for (uint32_t j = static_cast<uint32_t>(lane); j < nt; j += 64) {
        c.ids[t0 + j] = a.slot_ids[src + j];
        if (c.len) c.len[t0 + j] = a.slot_len[src + j];
      }
    }
  }
  CoopPublish(c, ok);
}

__global__ __launch_bounds__(64 * kCWaves) void coop_small_kernel(CoopSmallArgs s, CoopCall c) {
  __shared__ CoopShared sh;
  CoopSmallBody(s, c, sh, true);
}

// ---- Small raw-line calls (SentencePieceProcessor::Encode(line, &ids),
// sentencepiece_processor.cc:319-330, called once per line by
// spm_encode_main.cc:189-191): the device normalizer's state machine
// (normalize_kernels.hip = Normalizer::Normalize, normalizer.cc:88-211) on
// one lane, fed by NormalizePrefix results the wave computes 64 positions at
// a time; then CoopEncodeSentence; then the unknown-run merge of
// PopulateSentencePieceText (:525-529, epilogue.h Emits).

// NormalizePrefix (normalizer.cc:231-300) as (rlen | consumed << 16, source):
// source 0 = the input at p, 1 << 30 | off = the charsmap pool at off,
// 2 << 30 = U+FFFD.
__device__ uint2 NormalizePrefixPacked(const NormTables &t, const uint8_t *in, uint64_t n) {
  if (t.ud_units) {
    const uint32_t m = TrieLongest(t.ud_units, t.ud_num_units, in, n);
    if (m) return make_uint2(m | m << 16, 0u);
  }
  uint32_t value = 0;
  const uint32_t longest = CharsmapLongest(t, in, n, &value);
  if (longest == 0) {
    const uint32_t len = DValidCharLen(in, n);
    if (len == 0) return make_uint2(3u | 1u << 16, 2u << 30);
    return make_uint2(len | len << 16, 0u);
  }
  const uint8_t *r = t.pool + value;
  uint32_t l = 0;
  while (r[l]) ++l;
  return make_uint2(l | longest << 16, 1u << 30 | value);
}

// Raw bytes one call takes per line: the prefix table lives in W.u.bt.
constexpr uint32_t kRawMaxBytes = sizeof(float) * kCPos * kCK / sizeof(uint2);

// Normalizes in[0, n) into out (capacity cap); returns the length, or kNone
// when the line is longer than kRawMaxBytes or its output exceeds cap.
__device__ uint32_t NormalizeLineWave(const NormTables &t, CoopWave &W, const uint8_t *in_g, uint32_t n, uint8_t *out,
                                      uint32_t cap) {
  const int lane = threadIdx.x & 63;
  if (n > kRawMaxBytes) return kNone;
  uint2 *pref = reinterpret_cast<uint2 *>(&W.u.bt[0][0]);
  // The line's bytes in LDS (W.lmask, free until the encode): the state
  // machine's byte reads are on its serial chain.
  static_assert(sizeof(W.lmask) >= kRawMaxBytes, "raw line staging");
  uint8_t *lin = reinterpret_cast<uint8_t *>(W.lmask);
  for (uint32_t q = static_cast<uint32_t>(lane); q < n; q += 64) lin[q] = in_g[q];
  WaveSync();
  const uint8_t *in = lin;
  for (uint32_t base = 0; base < n; base += 64) {
    const uint32_t p = base + static_cast<uint32_t>(lane);
    if (p < n) pref[p] = NormalizePrefixPacked(t, in + p, n - p);
  }
  WaveSync();
  // The state machine, 64 chain positions at a time.  Serially it walks the
  // chain p -> p + consumed(p), skips leading single-space pieces, emits the
  // dummy prefix, drops a piece's leading spaces after a space, escapes
  // spaces, and finally drops the trailing whitespace units.  Here the chain
  // is walked with scalar readlanes over the lanes' consumed lengths; each
  // visited lane then knows its piece's prev_space (ballots: the last
  // earlier non-empty piece ends in a space), counts its output bytes and
  // whitespace units, takes its offset from one wave scan and writes its
  // bytes; the trailing whitespace run is carried from block to block.
  const bool rew = t.remove_extra_whitespaces, esc = t.escape_whitespaces;
  const uint32_t wsl = esc ? 3u : 1u;
  const bool prefix_ws = !t.suffix && t.add_dummy_prefix;
  uint32_t p = 0, olen = 0, run = 0;
  bool started = false, carry_ps = rew;
  for (uint32_t base = 0; base < n; base += 64) {
    const uint32_t q = base + static_cast<uint32_t>(lane);
    const uint2 x = q < n ? pref[q] : make_uint2(1u << 16, 0u);
    const uint32_t rlen = x.x & 0xFFFFu, src = x.y;
    auto rbyte = [&](uint32_t k) -> uint32_t {
      const uint32_t kind = src >> 30;
      if (kind == 0) return in[q + k];
      if (kind == 1) return t.pool[(src & 0x3FFFFFFFu) + k];
      return (0xBDBFEFu >> (8 * k)) & 0xFFu;  // U+FFFD
    };
    // Chain positions in this block (wave-uniform walk over the lanes'
    // consumed lengths; every consumed length is >= 1).
    const uint32_t lim = n < base + 64 ? n : base + 64;
    const uint32_t cons = x.x >> 16;
    uint64_t vis = 0;
    if (__builtin_amdgcn_ballot_w64(q < n && cons != 1u) == 0) {
      // Every position of the block consumes one byte (ASCII text without
      // charsmap rewrites): the chain is every position from p on.
      const uint64_t upto = lim - base == 64 ? ~0ull : (1ull << (lim - base)) - 1ull;
      if (p < lim) vis = upto & ~((1ull << (p - base)) - 1ull);
      p = p < lim ? lim : p;
    } else {
      while (p < lim) {
        vis |= 1ull << (p - base);
        p += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(cons), static_cast<int>(p - base)));
      }
    }
    const bool mine = (vis >> lane) & 1;
    // Leading whitespace (remove_extra_whitespaces): visited single-space
    // pieces before the first other one emit nothing; the dummy prefix goes
    // in front of that first emitting piece.
    int first = -1;
    uint64_t emitm = vis;
    if (!started && vis) {
      uint64_t cand = vis;
      if (rew) {
        const uint64_t sp = __builtin_amdgcn_ballot_w64(mine && rlen == 1 && rbyte(0) == ' ');
        cand = vis & ~sp;
      }
      if (cand) {
        first = __builtin_ctzll(cand);
        emitm = vis & ~((1ull << first) - 1);
        started = true;
      } else {
        emitm = 0;
      }
    }
    const bool emit = (emitm >> lane) & 1;
    // prev_space of this lane's piece (rew only): does the last earlier
    // non-empty emitting piece end in a space?
    const uint64_t ne = __builtin_amdgcn_ballot_w64(emit && rlen > 0);
    const uint64_t ls = __builtin_amdgcn_ballot_w64(emit && rlen > 0 && rbyte(rlen - 1) == ' ');
    bool ps = false;
    if (rew) {
      const uint64_t below = ne & ((1ull << lane) - 1);
      ps = below ? ((ls >> (63 - __builtin_clzll(below))) & 1) != 0 : carry_ps;
    }
    // Output bytes and whitespace units of this lane's piece (count pass,
    // then the same loop writes).
    const bool dummy = prefix_ws && lane == first;
    uint32_t ob = 0, wsu = 0, wtail = 0;
    bool nonws = false;
    uint32_t k0 = 0;
    if (emit) {
      if (dummy) {
        ob = wsl;
        wsu = wtail = 1;
      }
      if (ps)
        while (k0 < rlen && rbyte(k0) == ' ') ++k0;
      for (uint32_t k = k0; k < rlen;) {
        const uint32_t b0 = rbyte(k);
        if (b0 == ' ') {
          ob += wsl;
          ++wsu;
          ++wtail;
          ++k;
          continue;
        }
        const uint32_t cl = min(OneCharLenDev(b0), rlen - k);
        const bool is_ws = esc && cl == 3 && b0 == 0xE2 && rbyte(k + 1) == 0x96 && rbyte(k + 2) == 0x81;
        ob += cl;
        if (is_ws) {
          ++wsu;
          ++wtail;
        } else {
          nonws = true;
          wtail = 0;
        }
        k += cl;
      }
    }
    // Offsets: one inclusive scan of (bytes | ws units << 16).
    const uint32_t packed = ob | wsu << 16;
    uint32_t incl = packed;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    const uint32_t tot = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
    if (emit) {
      uint32_t o = olen + ((incl - packed) & 0xFFFFu);
      auto put = [&](uint32_t v) {
        if (o < cap) out[o] = static_cast<uint8_t>(v);
        ++o;
      };
      auto put_ws = [&]() {
        if (esc) {
          put(0xE2);
          put(0x96);
          put(0x81);
        } else {
          put(' ');
        }
      };
      if (dummy) put_ws();
      for (uint32_t k = k0; k < rlen;) {
        const uint32_t b0 = rbyte(k);
        if (b0 == ' ') {
          put_ws();
          ++k;
          continue;
        }
        const uint32_t cl = min(OneCharLenDev(b0), rlen - k);
        for (uint32_t j = 0; j < cl; ++j) put(rbyte(k + j));
        k += cl;
      }
    }
    olen += tot & 0xFFFFu;
    // The trailing whitespace run: from the last lane with a non-whitespace
    // char, or carried on through a block without one.
    const uint64_t nw = __builtin_amdgcn_ballot_w64(emit && nonws);
    const uint32_t tot_ws = tot >> 16;
    if (nw) {
      const int J = 63 - __builtin_clzll(nw);
      run = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wtail), J)) + tot_ws -
            (static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), J)) >> 16);
    } else {
      run += tot_ws;
    }
    if (ne) carry_ps = ((ls >> (63 - __builtin_clzll(ne))) & 1) != 0;
  }
  uint32_t len = 0;
  if (started) {
    len = olen;
    if (rew && run > 0) len -= run * wsl;  // trailing whitespace (normalizer.cc:191-202)
    if (t.suffix && t.add_dummy_prefix) {
      const uint32_t o = len + static_cast<uint32_t>(lane);
      if (static_cast<uint32_t>(lane) < wsl && o < cap)
        out[o] = static_cast<uint8_t>(esc ? (0x8196E2u >> (8 * lane)) & 0xFFu : ' ');
      len += wsl;
    }
  }
  const bool ok = len <= cap;
  __threadfence_block();
  WaveSync();
  return ok ? len : kNone;
}

__device__ void CoopRawBody(const CoopRawArgs &s, const CoopCall &c, CoopShared &sh, bool stage_trie) {
  CoopWave *lds = sh.lds;
  const uint2 *lds_root = sh.lds_root;
  uint32_t *ntok = sh.ntok;
  uint32_t &failed = sh.failed;
  const CoopArgs &a = s.a;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // a.prof (SPM_HIP_SERVICE_PROF): thread 0's shader-clock cycles per phase
  // into a.prof[8..13] (stage, normalize, encode, unknown merge, outputs +
  // publish, calls) and wall-clock ticks of the whole call into a.prof[14]
  // (the encode's own phases go to a.prof[0..7], CoopEncodeSentence).
  const bool prof = a.prof && tid == 0;
  const uint64_t p0 = prof ? clock64() : 0;
  const long long w0 = prof ? wall_clock64() : 0;
  uint64_t p_norm = 0, p_enc = 0, p_unk = 0;
  CoopStageAndRoot(a, s.stage_src, s.stage_dst, c.stage_words, sh, stage_trie);
  const bool in_lds = CoopTrieFits(a);
  const uint64_t p1 = prof ? clock64() : 0;
  const uint64_t *raw_off = reinterpret_cast<const uint64_t *>(s.stage_dst);
  const uint8_t *raw = reinterpret_cast<const uint8_t *>(s.stage_dst) + c.in_at;
  uint8_t *norm = const_cast<uint8_t *>(a.bytes);
  for (uint32_t i = static_cast<uint32_t>(wave); i < c.n; i += kCWaves) {
    const uint64_t rb0 = raw_off[i];
    const uint32_t rn = static_cast<uint32_t>(raw_off[i + 1] - rb0);
    const uint64_t nb0 = 4 * rb0 + 8ull * i;
    const uint64_t q0 = prof ? clock64() : 0;
    const uint32_t nn = NormalizeLineWave(s.t, lds[wave], raw + rb0, rn, norm + nb0, 4 * rn + 8);
    const uint64_t q1 = prof ? clock64() : 0;
    uint32_t nt = nn == kNone ? kNone
                  : in_lds   ? CoopEncodeSentence<true>(a, lds[wave], lds_root, nb0, nn, static_cast<uint64_t>(wave),
                                                        sh.trie)
                             : CoopEncodeSentence(a, lds[wave], lds_root, nb0, nn, static_cast<uint64_t>(wave));
    const uint64_t q2 = prof ? clock64() : 0;
    p_norm += q1 - q0;
    p_enc += q2 - q1;
    if (nt != kNone) {
      // Unknown runs merge (epilogue.h Emits): tokens [nb0 + nn - nt, nb0 +
      // nn) compacted in order to [nb0, nb0 + m); 64 at a time, the previous
      // token's unknown bit from the ballot (the chunk's first: carried).
      __threadfence_block();
      WaveSync();
      int32_t *tok = a.slot_ids + nb0;
      const int32_t *src = tok + nn - nt;
      uint32_t m = 0;
      bool prev_unk = false;
      for (uint32_t c0 = 0; c0 < nt; c0 += 64) {
        const uint32_t t = c0 + static_cast<uint32_t>(lane);
        const int32_t id = t < nt ? src[t] : 0;
        const uint8_t ty = (t < nt && id >= 0 && id < s.num_types) ? s.types[id] : 0;
        const bool unk = (ty & kPieceUnknown) != 0;
        const uint64_t um = __builtin_amdgcn_ballot_w64(unk && t < nt);
        const bool pu = lane == 0 ? prev_unk : ((um >> (lane - 1)) & 1) != 0;
        const bool emit = t < nt && ((ty & kPieceControl) != 0 || !(pu && unk));
        const uint64_t em = __builtin_amdgcn_ballot_w64(emit);
        WaveSync();  // every lane's load of this chunk before any store
        if (emit) tok[m + __popcll(em & ((1ull << lane) - 1))] = id;
        m += static_cast<uint32_t>(__popcll(em));
        const uint32_t last = (nt - c0 < 64 ? nt - c0 : 64) - 1;
        prev_unk = ((um >> last) & 1) != 0;
      }
      nt = m;
    }
    if (prof) p_unk += clock64() - q2;
    if (lane == 0) {
      if (nt == kNone) failed = 1;
      ntok[i] = nt;
    }
  }
  __threadfence_block();
  __syncthreads();
  const uint64_t p2 = prof ? clock64() : 0;
  if (failed == 0 && tid == 0) {
    uint64_t t = 0;
    c.tok[0] = 0;
    for (uint32_t i = 0; i < c.n; ++i) {
      const uint32_t nt = ntok[i];
      ntok[i] = static_cast<uint32_t>(t);
      t += nt;
      c.tok[i + 1] = t;
    }
    ntok[c.n] = static_cast<uint32_t>(t);
    if (t > c.ids_cap) failed = 1;
  }
  __syncthreads();
  const bool ok = failed == 0;
  if (ok) {
    for (uint32_t i = static_cast<uint32_t>(wave); i < c.n; i += kCWaves) {
      const uint32_t t0 = ntok[i], nt = ntok[i + 1] - t0;
      const int32_t *src = a.slot_ids + 4 * raw_off[i] + 8ull * i;
      for (uint32_t j = static_cast<uint32_t>(lane); j < nt; j += 64) c.ids[t0 + j] = src[j];
    }
  }
  CoopPublish(c, ok);
  if (prof) {
    const uint64_t p3 = clock64();
    unsigned long long *pr = reinterpret_cast<unsigned long long *>(a.prof);
    atomicAdd(pr + 8, static_cast<unsigned long long>(p1 - p0));
    atomicAdd(pr + 9, static_cast<unsigned long long>(p_norm));
    atomicAdd(pr + 10, static_cast<unsigned long long>(p_enc));
    atomicAdd(pr + 11, static_cast<unsigned long long>(p_unk));
    atomicAdd(pr + 12, static_cast<unsigned long long>(p3 - p2));
    atomicAdd(pr + 13, 1ull);
    atomicAdd(pr + 14, static_cast<unsigned long long>(wall_clock64() - w0));
    atomicAdd(pr + 15, static_cast<unsigned long long>(p3 - p0));
  }
}

__global__ __launch_bounds__(64 * kCWaves) void coop_raw_kernel(CoopRawArgs s, CoopCall c) {
  __shared__ CoopShared sh;
  CoopRawBody(s, c, sh, true);
}

// The resident small-call server (CoopServiceBox): thread 0 polls the box's
// sequence word in host memory (s_sleep between reads), the block copies the
// call and serves it, until `stop` or idle_ticks of wall clock without a
// request.  Every wave reaches the exit: the poll's outcome is broadcast
// through LDS and each loop iteration ends at a block barrier.
__global__ __launch_bounds__(64 * kCWaves) void coop_service_kernel(CoopServiceArgs sv) {
  __shared__ CoopShared sh;
  __shared__ uint32_t cmd;
  __shared__ uint64_t callw[sizeof(CoopCall) / 8];
  static_assert(sizeof(CoopCall) % 8 == 0, "call words");
  const int tid = threadIdx.x;
  uint32_t last = sv.last;
  if (tid == 0) __hip_atomic_store(&sv.box->alive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  uint32_t served = 0;
  uint64_t ticks_copy = 0, ticks_busy = 0;
  long long t_seen = 0;
  // The model's table is staged once per launch in practice: a request
  // stages it only when its call kind's table differs from the staged one
  // (a kind never called before this launch has zero arguments), and the
  // body's first barrier publishes it.
  const uint32_t *staged = nullptr;
  for (;;) {
    if (tid == 0) {
      uint32_t k = 0;
      const long long t0 = wall_clock64();
      for (;;) {
        if (__hip_atomic_load(&sv.box->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        const uint32_t q = __hip_atomic_load(&sv.box->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (q != last) {
          last = q;
          k = q >> 30;
          t_seen = wall_clock64();
          break;
        }
        if (static_cast<uint64_t>(wall_clock64() - t0) > sv.idle_ticks) break;
        __builtin_amdgcn_s_sleep(1);
      }
      cmd = k;
    }
    __syncthreads();
    const uint32_t kind = cmd;
    if (kind == 0) break;
    // The call's words, one per thread, from host memory.
    if (tid < static_cast<int>(sizeof(CoopCall) / 8))
      callw[tid] = __hip_atomic_load(reinterpret_cast<const uint64_t *>(&sv.box->call) + tid, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    CoopCall c;
    __builtin_memcpy(&c, callw, sizeof(CoopCall));
    const long long t_copied = wall_clock64();
    const CoopArgs &ka = kind == 1 ? sv.small.a : sv.raw.a;
    const bool stage = ka.uvs != staged;
    staged = ka.uvs;
    if (kind == 1) CoopSmallBody(sv.small, c, sh, stage);
    else CoopRawBody(sv.raw, c, sh, stage);
    ++served;
    if (tid == 0) {
      ticks_copy += static_cast<uint64_t>(t_copied - t_seen);
      ticks_busy += static_cast<uint64_t>(wall_clock64() - t_seen);
    }
    __syncthreads();
  }
  if (tid == 0) {
    __hip_atomic_store(&sv.box->ticks_copy, ticks_copy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&sv.box->ticks_busy, ticks_busy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&sv.box->served, served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&sv.box->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The flagged list split by length: long sentences packed from the front,
// the others from the back of `part` (n entries).
__global__ void coop_partition_kernel(const uint32_t *list, const uint32_t *count, const uint64_t *off, uint64_t n,
                                      uint32_t *part, uint32_t *n_long, uint32_t *n_short) {
  const uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= *count) return;
  const uint32_t i = list[k];
  if (off[i + 1] - off[i] >= kCoopLongNb) part[atomicAdd(n_long, 1u)] = i;
  else part[n - 1 - atomicAdd(n_short, 1u)] = i;
}

}  // namespace

hipError_t LaunchCoopRaw(const CoopRawArgs &s, const CoopCall &c, hipStream_t st) {
  if (c.n == 0 || c.n > kCoopSmallMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(coop_raw_kernel, dim3(1), dim3(64 * kCWaves), 0, st, s, c);
  return hipGetLastError();
}

hipError_t LaunchCoopSmall(const CoopSmallArgs &s, const CoopCall &c, hipStream_t st) {
  if (c.n == 0 || c.n > kCoopSmallMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(coop_small_kernel, dim3(1), dim3(64 * kCWaves), 0, st, s, c);
  return hipGetLastError();
}

hipError_t LaunchCoopService(const CoopServiceArgs &s, hipStream_t st) {
  if (!s.box || s.idle_ticks == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(coop_service_kernel, dim3(1), dim3(64 * kCWaves), 0, st, s);
  return hipGetLastError();
}

hipError_t LaunchCoopPartition(const uint32_t *list, const uint32_t *count, const uint64_t *off, uint64_t n,
                               uint32_t *part, uint32_t *n_long, uint32_t *n_short, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t g = (n + 255) / 256;
  hipLaunchKernelGGL(coop_partition_kernel, dim3(static_cast<unsigned>(g < (1u << 30) ? g : (1u << 30))), dim3(256),
                     0, st, list, count, off, n, part, n_long, n_short);
  return hipGetLastError();
}

hipError_t LaunchCoopEncode(const CoopArgs &a, uint32_t max_blocks, hipStream_t st) {
  if (max_blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(coop_list_kernel, dim3(max_blocks), dim3(64 * kCWaves), 0, st, a);
  return hipGetLastError();
}

}  // namespace spm_amd
