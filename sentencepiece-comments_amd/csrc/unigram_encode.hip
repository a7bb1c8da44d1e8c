// Unigram Viterbi encode kernels for gfx950 (MI355X).
//
// Reference path: unigram::Model::Encode (unigram_model.cc:705-720) =
//   Lattice::SetSentence (:147-187) + Model::PopulateNodes (:535-604, a darts
//   commonPrefixSearch per char position) + Lattice::Viterbi (:222-261).
//
// unigram_fast_kernel — one sentence per lane, the lattice never materialised:
//   Viterbi's backtrace score of a node (b,e) with score s is
//     max_l fl(bt_l + s) over lnodes ending at b  ==  fl(T_b + s),
//   T_b = max bt of the nodes ending at b, because float rounding is monotone.
//   So the forward pass keeps only T per pending end position, in a register
//   ring indexed by the (static, unrolled) distance of the trie walk.  The
//   argmax *identity* (the back-pointer) is what float ties can change: the
//   reference takes the FIRST lnode in end_nodes order (= ascending begin)
//   with the maximal fl(bt_l + s).  Only the successive running-max setters of
//   an end position can win; a setter more than a few ulps below the final
//   max never ties.  So per end position the kernel keeps B (first setter of
//   T) and, when the previous setter is within the near-tie bound, an
//   "ambiguity" entry (T, T2, B2); the backtrace resolves
//   winner = (fl(T2+s) == fl(T+s)) ? B2 : B exactly.  A sentence whose ties
//   chain deeper, overflows the entry list, meets a trie leaf inside a UTF-8
//   char, holds a 0xFF byte (byte kernel) or has an inconsistent back-pointer
//   chain is flagged and re-run by unigram_general_kernel, a literal
//   restatement of the reference lattice.
//
// Two forward passes:
//   kByte (W = 16, models whose pieces are whole chars of < 16 bytes): every
//     byte position is visited, char starts found by the lead-byte chain;
//     positions walked in pairs (two independent trie-load chains per lane),
//     inserts lagged one walk step behind their score loads (software
//     pipeline), back-pointers packed as 8-bit distances, 2 near-tie entries,
//     7 waves/SIMD.  (Round-2 A/B of the alternatives — LDS trie top, jump
//     table, lane-decoupled walk, 4-6 waves — is in DESIGN.md §4.)
//   kChar (W = 16/32/64): one char position at a time, full back-pointers,
//     4 near-tie entries, values + scores tables.
//
// Output: lanes count their tokens with a first backtrace, the block scans
// the counts in sentence order and the second backtrace writes ids / piece
// lengths densely into the tile's slot range (at the tile's first input
// byte); tile_compact_kernel then places every tile (compact.hip).
//
// Back-pointers: one byte per char position (end - winner begin), in LDS for
// byte positions < kLdsBpPos, beyond that in a global scratch array indexed
// like the input bytes (position nb — EOS — included).  The backtrace checks
// every step (begin < end) and flags the sentence otherwise, so a bad
// back-pointer can never spin a wave.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "device_common.h"
#include "kernels.h"
#include "lookback.h"  // status words

namespace spm_amd {
namespace {

struct FastArgs {
  const uint8_t *__restrict__ bytes;
  const uint64_t *__restrict__ off;
  uint64_t n;
  uint64_t capacity;
  const uint32_t *__restrict__ units;
  const int32_t *__restrict__ values;
  const float *__restrict__ scores;
  uint32_t num_units;
  UnigramParams p;
  int32_t *__restrict__ ids;
  uint32_t *__restrict__ len;
  uint64_t *__restrict__ tok_off;
  uint8_t *__restrict__ bp;
  uint32_t *__restrict__ flagged;
  uint32_t *__restrict__ status;
  uint64_t *__restrict__ tile_count;
  uint64_t corrupt_bp;
  const uint32_t *__restrict__ chain;
  int32_t *__restrict__ slot_ids;  // tile-dense token slots (capacity entries)
  uint32_t *__restrict__ slot_len;
  EStepForwardOut e;               // E-step forward pass (kE instantiation only)
  uint32_t *__restrict__ bpn;      // kWide: trie unit of the best node ending at each byte position
  const uint32_t *stage_src;       // single-tile host call: input image in pinned host memory
  uint32_t *stage_dst;
  uint32_t stage_zero;             // leading words zeroed instead of copied (the status block)
  uint32_t stage_words;
  uint32_t *host_pub;              // single-tile host call: status words + sequence to host memory
  uint32_t pub_seq;
  uint32_t coop_min_nb;            // wide / char kernels: longer sentences go to the cooperative kernel
};

constexpr int kBlock = 256;
constexpr int kLdsBpPos = 64;  // back-pointer bytes kept in LDS per lane
constexpr int kEStepWaves = 4;  // E-step forward mode (alpha ring + fp64 LogSumExp)

// kE (byte kernel only): the unigram trainer E-step's forward pass on the same
// walk — besides the Viterbi ring it keeps the alpha ring of PopulateMarginal
// (unigram_model.cc:272-300: alpha of the nodes ending at each byte slot,
// LogSumExp over end_nodes in ascending begin order, which is the order the
// lagged inserts reach a slot), writes alpha at every char start, Z = alpha
// of EOS, the node count and Viterbi().size(), and skips the id output.
template <int W, bool kByte, int kWaves = kByte ? 7 : (W == 16 ? 4 : 1), bool kE = false, bool kWide = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kWaves)))
void unigram_fast_kernel(FastArgs a) {
  static_assert(!kByte || W == 16, "the byte kernel's ring and window are sized for W = 16");
  static_assert(!kE || kByte, "the E-step forward pass is a byte-kernel mode");
  static_assert(!kWide || (!kByte && W == 16), "the wide-char pass rings 16 chars");
  // Back-pointer bytes of byte positions [0, kLdsBpPos) of each lane's
  // sentence: word (pos/4)*kBlock + tid, byte pos%4.
  __shared__ uint32_t lds_bp[(kLdsBpPos / 4) * kBlock];
  __shared__ uint32_t lds_scan[kBlock];
  __shared__ uint32_t lds_wave[kBlock / 64];
  __shared__ uint32_t lds_tile;
  // Byte kernel: (unit, score) of the root's 256 children, the first step of
  // every walk (32 % of the trie gathers), served by LDS instead of the
  // vector-memory address path the walk is bound by: 4.17 -> 4.08 ms per
  // 10 M c2 sentences (profiles/r03k_root_lds_ab.txt).
  constexpr bool kRootLds = kByte || kWide;
  // Byte encode kernel: the length sort's table, the root table and (once
  // both are dead) the tile's output ids share one LDS buffer.  The ids are
  // staged there and written out as one coalesced run per tile: written
  // straight from the backtrace (4 bytes per lane per step, scattered over
  // the tile's range) they were 640 of the kernel's 750 MB of HBM writes and
  // cost 420 MB of reads per 10 M sentences (profiles/r04u_pmc_c2_*.json).
  // The buffer fills what the 7-block occupancy leaves of the CU's LDS
  // (22.5 KB per block after allocation granularity; at 1472 ids the block
  // rounded past it, 6 blocks fit and the kernel ran 7 % slower).
  constexpr bool kStage = kByte && !kE;
  constexpr uint32_t kStageIds = kStage ? 1264u : 2u;
  __shared__ uint2 lds_union[kStageIds / 2];
  __shared__ uint32_t lds_sort_own[kStage ? 1 : 2 * kBlock];
  __shared__ uint2 lds_root_own[(kRootLds && !kStage) ? kBlock : 1];
  uint32_t *const lds_stage = reinterpret_cast<uint32_t *>(lds_union);
  uint32_t *const lds_sort = kStage ? lds_stage : lds_sort_own;
  uint2 *const lds_root = kStage ? lds_union + kBlock : lds_root_own;
  uint8_t *lbp = reinterpret_cast<uint8_t *>(lds_bp);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  if constexpr (!kE) {
    // Single-tile host call: the status block is zeroed here and the rest of
    // the input image (offsets, bytes) comes from pinned host memory in one
    // coalesced pass
    // (no separate copy command on the per-call path).  The fences order
    // these stores before every later read of the same memory.
    if (a.stage_src) {
      for (uint32_t k = static_cast<uint32_t>(tid); k < a.stage_zero; k += kBlock) a.stage_dst[k] = 0u;
      for (uint32_t k = a.stage_zero + static_cast<uint32_t>(tid); k < a.stage_words; k += kBlock)
        a.stage_dst[k] = a.stage_src[k];
      __threadfence_block();
      __syncthreads();
    }
  }
  // An earlier step of an asynchronous chain failed: nothing to do.
  if (a.chain && *a.chain) return;
  const uint64_t total_bytes = a.off[a.n];
  // A batch larger than the caller's capacity (the scratch is sized by it):
  // every tile leaves before touching anything, the error is reported.
  if (total_bytes > a.capacity) {
    if (blockIdx.x == 0 && tid == 0) atomicOr(&a.status[kStError], 2u);
    return;
  }
  // Tiles in launch order (the look-back's progress guarantee).
  if (tid == 0) lds_tile = atomicAdd(&a.status[kStTicket], 1u);
  if constexpr (kRootLds) {
    const uint32_t nd = a.p.root_base ^ static_cast<uint32_t>(tid);
    lds_root[tid] = nd < a.num_units ? reinterpret_cast<const uint2 *>(a.units)[nd] : make_uint2(0u, 0u);
  }
  __syncthreads();
  const uint64_t tile = lds_tile;
  const uint64_t base = tile * kBlock;

  // Counting sort of the tile's sentences by length (0..255): each wave's 64
  // lanes then run similar trip counts.
  uint32_t sid;
  {
    uint32_t *hist = lds_sort, *perm = lds_sort + kBlock;
    const uint64_t ii = base + tid;
    const uint32_t len = ii < a.n ? static_cast<uint32_t>(a.off[ii + 1] - a.off[ii]) : 0u;
    // Exact up to 191 bytes, then 32-byte bins up to 2207 (paragraph-length
    // lines of real text would otherwise share one bin and a wave would run
    // as long as its longest line).
    const uint32_t bucket = len < 192 ? len : len < 2208 ? 192 + (len - 192) / 32 : kBlock - 1;
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
  if constexpr (kE) {
    if (a.e.AT) {
      a.e.lanemap[base + tid] = static_cast<uint8_t>(sid);
      if (valid) a.e.colmap[i] = static_cast<uint16_t>(tid);
    }
  }
  const uint64_t b0 = valid ? a.off[i] : 0;
  const uint32_t nb = valid ? static_cast<uint32_t>(a.off[i + 1] - b0) : 0;

  // Byte kernel: the tile's bytes from its first aligned byte as a buffer
  // resource, lanes address them by a 32-bit offset (no per-lane 64-bit
  // pointers live in the walk).  The back-pointer scratch beyond the LDS
  // window is a second resource over the same offsets (bp + blk_al + lrel +
  // pos == bp + b0 + pos).  Its range is the scratch's own size, capacity +
  // 16 bytes, so it covers position nb of the batch's last sentence, one past
  // the last input byte (the round-2 hang: a back-pointer resource whose
  // num_records ended at the last input byte dropped exactly that store).
  // Buffer accesses also keep the compiler from merging the LDS and global
  // branches of bp_store / bp_load into flat accesses.
  const uint64_t blk_al = a.off[base] & ~3ull;
  const uint64_t blk_rem = total_bytes - blk_al;
  const int blk_nrec = static_cast<int>(blk_rem < 0x7FFFFFF0ull ? blk_rem : 0x7FFFFFF0ull);
  const auto bytes_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.bytes + blk_al), 0, blk_nrec, 0x00020000);
  const uint64_t bp_rem = a.capacity + 16 - blk_al;
  const auto bp_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      a.bp + blk_al, 0, static_cast<int>(bp_rem < 0x7FFFFFFFull ? bp_rem : 0x7FFFFFFFull), 0x00020000);
  const uint32_t lrel = static_cast<uint32_t>(b0 - blk_al);
  const uint8_t *__restrict__ s = a.bytes + b0;

  auto byte_at = [&](uint32_t q) -> uint32_t {
    if constexpr (kByte) return __builtin_amdgcn_raw_buffer_load_b8(bytes_rsrc, lrel + q, 0, 0);
    else return s[q];
  };
  auto bp_store = [&](uint32_t pos, uint32_t v) {
    if (pos < kLdsBpPos) lbp[((pos >> 2) * kBlock + tid) * 4 + (pos & 3)] = static_cast<uint8_t>(v);
    else __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v), bp_rsrc, lrel + pos, 0, 0);
  };
  auto bp_load = [&](uint32_t pos) -> uint32_t {
    if (pos < kLdsBpPos) return lbp[((pos >> 2) * kBlock + tid) * 4 + (pos & 3)];
    return __builtin_amdgcn_raw_buffer_load_b8(bp_rsrc, lrel + pos, 0, 0);
  };

  // Near-tie entries (shared by both passes and the backtrace).
  constexpr int kAmb = kByte ? 2 : kAmbEntries;
  uint32_t ae[kAmb], aB2[kAmb];
  uint32_t aN2[kWide ? kAmb : 1];  // kWide: the second setter's trie unit
  float aT[kAmb], aT2[kAmb];
#pragma unroll
  for (int k = 0; k < kAmb; ++k) {
    ae[k] = kNone;
    aB2[k] = 0;
    aT[k] = 0.f;
    aT2[k] = 0.f;
    if constexpr (kWide) aN2[k] = kNone;
  }
  std::conditional_t<kByte, uint32_t, uint64_t> ambm = 0;  // bit d: ring slot d has an entry
  bool bad = false, any_amb = false;
  uint32_t e_nodes = 0;  // kE: lattice nodes (trie + UNK)
  float e_z = 0.f;       // kE: alpha of EOS
  const float tie_mag = a.p.tie_mag;
  // Maintain the near-tie entry of end position `end` (ring slot d) when a
  // setter replaces (t_old, b_old) by bt (nr: the two are near).
  auto amb_update = [&](auto dc, float bt, bool nr, uint32_t end, float t_old, uint32_t b_old,
                        uint32_t n_old = kNone) {
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
          if (NearTie(aT2[k], bt, tie_mag)) bad = true;  // 3-deep tie chain
          if (nr) {
            aT2[k] = t_old;
            aB2[k] = b_old;
            if constexpr (kWide) aN2[k] = n_old;
            aT[k] = bt;
          } else {
            ae[k] = kNone;
            ambm &= ~(static_cast<decltype(ambm)>(1) << d);
          }
        }
    } else if (nr) {
      if (free_slot < 0) bad = true;
      any_amb = true;
      ambm |= static_cast<decltype(ambm)>(1) << d;
#pragma unroll
      for (int k = 0; k < kAmb; ++k)
        if (k == free_slot) {
          ae[k] = end;
          aT2[k] = t_old;
          aB2[k] = b_old;
          if constexpr (kWide) aN2[k] = n_old;
          aT[k] = bt;
        }
    }
  };

  if constexpr (kByte) {
    // ---- Byte-position pass (units = (unit, score) pairs: the 0xFF-padded
    // image and the usable-node score or NaN per unit).  p is a char start iff the
    // lead-byte chain from 0 reaches it (OneCharLen clamped to the sentence,
    // unigram_model.cc:155-160 / util.h:389), so malformed UTF-8 needs no
    // special case.  Pieces split exactly into chars (checked at load), hence
    // a leaf reached from a char start ends at a char start.  Positions are
    // processed kU at a time against a ring T[k] = best score ending at
    // p0 + k (k < kR), shifted by kU per group.
    constexpr int kU = 4;
    constexpr int kR = W + kU - 1;      // 19 ring slots
    constexpr int kWin = (kR + 3) / 4;  // 5 window words (bytes p0 .. p0 + 19)
    constexpr int kBw = (W + 6) / 4;    // packed back-pointer words (4 slots each)
    constexpr int kNI = 2;              // positions walked together
    // (unit, node score) pairs: a.units is the interleaved table here.
    const auto uvs_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(a.units), 0,
                                                            static_cast<int>(a.num_units * 8u), 0x00020000);
    using UvT = decltype(__builtin_amdgcn_raw_buffer_load_b64(uvs_rsrc, 0u, 0, 0));
    float T[kR];
#pragma unroll
    for (int d = 0; d < kR; ++d) T[d] = d == 0 ? 0.f : -__builtin_inff();  // slot 0: BOS
    // kE: alpha ring.  A slot starts at -inf, so its first LogSumExp returns
    // the node's value exactly as the reference's init_mode does.
    float Ar[kE ? kR : 1];
#pragma unroll
    for (int d = 0; d < (kE ? kR : 1); ++d) Ar[d] = d == 0 ? 0.f : -__builtin_inff();
    // Slot k's back-pointer: distance end - begin (<= W - 1, invariant under
    // the ring shift) as a byte, four slots per register.
    uint32_t Bw[kBw];
#pragma unroll
    for (int m = 0; m < kBw; ++m) Bw[m] = 0;
    auto b_dist = [&](auto kc) -> uint32_t {
      constexpr int k = decltype(kc)::value;
      return (Bw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
    };
    // Offsets past the tile's buffer range (a > 2 GB tile) would read 0:
    // such a sentence takes the general kernel.
    bad = valid && (b0 - blk_al) + nb > static_cast<uint64_t>(blk_nrec);
    // Window: aligned dwords of the lane's bytes, spliced by alignbyte.
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
    // Bytes q .. q+3 with zeros beyond nb; a 0xFF byte (the padded trie image
    // matches 0xFF on empty units) flags the sentence.
    auto finish = [&](uint32_t x, uint32_t q) -> uint32_t {
      if (q + 4 > nb) x &= q >= nb ? 0u : (1u << (8 * (nb - q))) - 1u;
      const uint32_t y = ~x;
      if (((y - 0x01010101u) & ~y & 0x80808080u) != 0) bad = true;
      return x;
    };
    uint32_t wprev = nb > 0 ? word_at(0) : 0u;
    uint32_t rw[kWin];
#pragma unroll
    for (int k = 0; k < kWin; ++k) {
      const uint32_t q = 4 * k;
      const uint32_t wn = q < nb ? word_at(k + 1) : 0u;
      rw[k] = q < nb ? finish(__builtin_amdgcn_alignbyte(wn, wprev, sh), q) : 0u;
      wprev = wn;
    }
    auto byte_of = [&](auto tc) -> uint32_t {
      constexpr int t = decltype(tc)::value;
      return (rw[t >> 2] >> (8 * (t & 3))) & 0xFFu;
    };
    // Node [p, p + d) of position j with raw score sc (NaN: no usable node)
    // into slot j + d.  Nodes reach a slot in ascending begin order.
    auto insert_one = [&](auto jc, auto dc, uint32_t p, float T0, float A0, uint32_t clen0, bool st, float sc,
                          int dmax) {
      constexpr int j = decltype(jc)::value;
      constexpr int d = decltype(dc)::value;
      if (d > 4 && d > dmax) return;
      float s_node = sc;
      // UNK node (unigram_model.cc:597-601): no usable single-char node.
      if constexpr (d <= 4) s_node = (d == static_cast<int>(clen0) && __builtin_isnan(s_node)) ? a.p.unk_score : s_node;
      if (!st) s_node = __builtin_nanf("");
      const float bt = __fadd_rn(T0, s_node);
      constexpr int k = j + d;
      if constexpr (kE) {
        if (!__builtin_isnan(s_node)) {
          Ar[k] = LogSumExpDev(Ar[k], __fadd_rn(s_node, A0), false);
          ++e_nodes;
        }
      }
      const bool gt = bt > T[k];  // false for NaN
      const bool rare = gt && (NearTieHi(T[k], bt, tie_mag) || ((ambm >> k) & 1));
      if (__builtin_amdgcn_ballot_w64(rare) != 0) {
        if (rare)
          amb_update(std::integral_constant<int, k>{}, bt, NearTieHi(T[k], bt, tie_mag), p + d, T[k],
                     p + d - b_dist(std::integral_constant<int, k>{}));
      }
      T[k] = gt ? bt : T[k];
      constexpr uint32_t sh8 = 8 * (k & 3);
      const uint32_t w = (Bw[k >> 2] & ~(0xFFu << sh8)) | (static_cast<uint32_t>(d) << sh8);
      Bw[k >> 2] = gt ? w : Bw[k >> 2];
    };
    uint32_t next_start = 0;
    for (uint32_t p0 = 0; p0 <= nb; p0 += kU) {
      StaticFor<0, kU / kNI>([&](auto pc) {
        constexpr int jb = kNI * decltype(pc)::value;
        uint32_t pp[kNI], cl[kNI];
        bool at[kNI], st[kNI], any[kNI];
        // Char starts in order (next_start chains through the group).
        StaticFor<0, kNI>([&](auto qc) {
          constexpr int q = decltype(qc)::value, j = jb + q;
          pp[q] = p0 + j;
          at[q] = pp[q] <= nb && pp[q] == next_start;
          if (q == 0 && at[q] && pp[q] > 0) bp_store(pp[q], b_dist(std::integral_constant<int, j>{}));
          st[q] = at[q] && pp[q] < nb;
          cl[q] = OneCharLenDev(byte_of(std::integral_constant<int, j>{}));
          if (cl[q] > nb - pp[q]) cl[q] = nb - pp[q];
          if constexpr (kE) {
            // The backward pass finds char starts as non-continuation bytes:
            // a char start must not be one, its tail bytes must all be.
            if (st[q]) {
              const uint32_t lead = byte_of(std::integral_constant<int, j>{});
              bool ok = (lead & 0xC0u) != 0x80u;
              StaticFor<1, 4>([&](auto tc) {
                constexpr int t = decltype(tc)::value;
                if (static_cast<uint32_t>(t) < cl[q] && (byte_of(std::integral_constant<int, j + t>{}) & 0xC0u) != 0x80u)
                  ok = false;
              });
              if (!ok) bad = true;
            }
          }
          if (st[q]) next_start = pp[q] + cl[q];
          any[q] = __builtin_amdgcn_ballot_w64(st[q]) != 0;
        });
        // Lagged inserts: position q's node of length dd is inserted at walk
        // step d = dd + 1 + q, right after the loads of step d are issued.
        // Its score load (issued at step dd) has landed by then, so each
        // score register lives about one step.  Every insert into slot
        // jb + d - 1 happens at step d in ascending q = ascending begin, as
        // end_nodes_ order requires; position q's own T0 and back-pointer
        // (slot jb + q, final after step q + 1) are read at step q + 2,
        // before its first insert.
        float sok[kNI][W];  // node score of depth d (NaN: no usable node)
        float T0q[kNI];
        float A0q[kNI];
        int dm[kNI];
        uint32_t bs[kNI], nd[kNI], c[kNI];
        UvT uv[kNI];
        bool al[kNI];
        StaticFor<0, kNI>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          dm[q] = 0;
          T0q[q] = 0.f;
          bs[q] = st[q] ? a.p.root_base : 0u;
          al[q] = st[q];
        });
        bool go = any[0] || any[1];
        if (go) {
          StaticFor<0, kNI>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            c[q] = byte_of(std::integral_constant<int, jb + q>{});
            if constexpr (kRootLds) {
              const uint2 r = lds_root[c[q]];
              uv[q][0] = r.x;
              uv[q][1] = r.y;
            } else {
              nd[q] = bs[q] ^ c[q];
              uv[q] = __builtin_amdgcn_raw_buffer_load_b64(uvs_rsrc, nd[q] * 8u, 0, 0);
            }
          });
        }
        // Software pipeline: step d waits for the (unit, score) loads of
        // depth d, issues those of depth d + 1, and only then runs the lagged
        // inserts, so their VALU work overlaps the loads in flight.  One
        // 8-byte gather per walk step and lane carries both the unit and its
        // node score: the walk is bound by the vector-memory address path
        // (TA busy 84 % of the kernel with separate unit and score gathers,
        // profiles/r03g_ta_unigram_fast.txt), so a step costs one gather.
        StaticFor<1, W + kNI>([&](auto dc) {
          constexpr int d = decltype(dc)::value;
          if constexpr (d < W) {
            StaticFor<0, kNI>([&](auto qc) { sok[decltype(qc)::value][d] = __builtin_nanf(""); });
            if (go) {
              bool g = false;
              StaticFor<0, kNI>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                const uint32_t u = uv[q][0];
                al[q] = al[q] && (u & 0xFFu) == c[q];
                bs[q] = al[q] ? u >> 9 : 0u;
                sok[q][d] = al[q] ? __uint_as_float(uv[q][1]) : __builtin_nanf("");
                const bool gq = __builtin_amdgcn_ballot_w64(al[q]) != 0;
                if (gq) dm[q] = d;
                g = g || gq;
              });
              go = g;
              if constexpr (d + 1 < W) {
                if (go) {
                  StaticFor<0, kNI>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    c[q] = byte_of(std::integral_constant<int, jb + q + d>{});
                    nd[q] = bs[q] ^ c[q];
                    uv[q] = __builtin_amdgcn_raw_buffer_load_b64(uvs_rsrc, nd[q] * 8u, 0, 0);
                  });
                }
              }
            }
          }
          StaticFor<0, kNI>([&](auto qc) {
            constexpr int q = decltype(qc)::value, j = jb + q, dd = d - 1 - q;
            if constexpr (dd == 1) {
              if (q > 0 && at[q] && pp[q] > 0) bp_store(pp[q], b_dist(std::integral_constant<int, j>{}));
              T0q[q] = T[j];
              if constexpr (kE) {
                // Slot j is final here: alpha of this char start (or Z at EOS).
                A0q[q] = Ar[j];
                if (st[q]) {
                  if (a.e.AT && pp[q] < kATRows)
                    a.e.AT[(tile * kATRows + pp[q]) * kBlock + tid] = Ar[j];
                  else
                    a.e.A[b0 + pp[q]] = Ar[j];
                }
                if (at[q] && pp[q] == nb) e_z = Ar[j];
              }
            }
            if constexpr (dd >= 1 && dd < W) {
              if (any[q])
                insert_one(std::integral_constant<int, j>{}, std::integral_constant<int, dd>{}, pp[q], T0q[q],
                           kE ? A0q[q] : 0.f, cl[q], st[q], sok[q][dd], dm[q]);
            }
          });
        });
      });
      // Next group: shift the ring and the byte window by kU.
#pragma unroll
      for (int k = 0; k < kR; ++k) T[k] = k + kU < kR ? T[k + kU] : -__builtin_inff();
      if constexpr (kE) {
#pragma unroll
        for (int k = 0; k < kR; ++k) Ar[k] = k + kU < kR ? Ar[k + kU] : -__builtin_inff();
      }
#pragma unroll
      for (int m = 0; m < kBw; ++m) Bw[m] = m + 1 < kBw ? Bw[m + 1] : 0u;
      ambm >>= kU;
#pragma unroll
      for (int k = 0; k + 1 < kWin; ++k) rw[k] = rw[k + 1];
      const uint32_t qn = p0 + kU + 4 * (kWin - 1);
      const uint32_t wn = qn < nb ? word_at(qn / 4 + 1) : 0u;
      rw[kWin - 1] = qn < nb ? finish(__builtin_amdgcn_alignbyte(wn, wprev, sh), qn) : 0u;
      wprev = wn;
    }
  } else if constexpr (kWide) {
    // ---- Wide-char pass (models whose pieces are whole chars, < 16 chars,
    // < 64 bytes, some >= 16 bytes: CJK vocabularies).  Ring slot c = the
    // position c CHARS ahead (a 3-byte char costs one slot, not three), so
    // the ring shifts by one slot per char; the walk consumes the sentence
    // from a 32-byte register window (three buffer loads per char position
    // instead of a byte gather per window byte), reads (unit, node score)
    // pairs (the byte kernel's table: one 8-byte gather per trie edge brings
    // the leaf's score), takes the root's children from LDS, inserts each
    // node as soon as its char boundary is reached (ascending length, then
    // UNK: begin_nodes_ order), and each slot keeps the trie unit of its best
    // node, so the backtrace reads the token's id instead of re-walking it.
    constexpr int Wc = W;
    const auto uvs_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(a.units), 0,
                                                            static_cast<int>(a.num_units * 8u), 0x00020000);
    float T[Wc];
    uint32_t B[Wc], Nd[Wc];  // best node's begin byte / trie unit (kNone: UNK) per slot
#pragma unroll
    for (int d = 0; d < Wc; ++d) {
      T[d] = 0.f;
      B[d] = 0;
      Nd[d] = kNone;
    }
    uint32_t has = 1;  // bit c: slot c holds a node
    auto insert = [&](auto dc, float bt, uint32_t begin, uint32_t end, uint32_t node) {
      constexpr int d = decltype(dc)::value;
      if (!((has >> d) & 1)) {
        has |= (1u << d);
        T[d] = bt;
        B[d] = begin;
        Nd[d] = node;
      } else if (bt > T[d]) {
        const bool nr = NearTie(T[d], bt, tie_mag);
        if (nr || ((ambm >> d) & 1)) amb_update(dc, bt, nr, end, T[d], B[d], Nd[d]);
        T[d] = bt;
        B[d] = begin;
        Nd[d] = node;
      }
    };
    // Window: the 32 bytes from byte q of the sentence, zero past its end.
    uint32_t r[8];
    auto load_window = [&](uint32_t q) {
      const uint32_t o = (lrel + q) & ~3u, sh = (lrel + q) & 3u;
      uint32_t w[9];
      if (static_cast<uint64_t>(o) + 36 <= static_cast<uint64_t>(blk_rem)) {
        const auto x0 = __builtin_amdgcn_raw_buffer_load_b128(bytes_rsrc, o, 0, 0);
        const auto x1 = __builtin_amdgcn_raw_buffer_load_b128(bytes_rsrc, o + 16, 0, 0);
        w[0] = x0[0];
        w[1] = x0[1];
        w[2] = x0[2];
        w[3] = x0[3];
        w[4] = x1[0];
        w[5] = x1[1];
        w[6] = x1[2];
        w[7] = x1[3];
        w[8] = __builtin_amdgcn_raw_buffer_load_b32(bytes_rsrc, o + 32, 0, 0);
      } else {  // the batch's last bytes: byte loads (a straddling dword reads 0)
#pragma unroll
        for (uint32_t k = 0; k < 9; ++k) {
          uint32_t x = 0;
#pragma unroll
          for (uint32_t t = 0; t < 4; ++t)
            if (o + 4 * k + t < blk_rem) x |= static_cast<uint32_t>(a.bytes[blk_al + o + 4 * k + t]) << (8 * t);
          w[k] = x;
        }
      }
      const uint32_t left = nb > q ? nb - q : 0u;  // sentence bytes in the window
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        uint32_t x = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
        const uint32_t b = 4u * k;
        if (b + 4 > left) x &= b >= left ? 0u : (1u << (8 * (left - b))) - 1u;
        r[k] = x;
      }
    };
    auto next_byte = [&]() -> uint32_t {  // consume the window's first byte
      const uint32_t c = r[0] & 0xFFu;
#pragma unroll
      for (int k = 0; k < 7; ++k) r[k] = __builtin_amdgcn_alignbyte(r[k + 1], r[k], 1);
      r[7] >>= 8;
      return c;
    };
    // Offsets past the tile's buffer range (a > 2 GB tile) would read 0:
    // such a sentence takes the general kernel.
    bad = valid && (b0 - blk_al) + nb > static_cast<uint64_t>(blk_nrec);
    // Long sentences: the wave-cooperative kernel (flagged without a walk).
    const bool coop = a.coop_min_nb && nb >= a.coop_min_nb;
    if (coop) bad = true;
    uint32_t pos = 0;  // byte offset of the current char position
    while (nb > 0 && !coop) {
      if (pos > 0) {
        bp_store(pos, pos - B[0]);
        a.bpn[b0 + pos] = Nd[0];
      }
      if (pos >= nb) break;
      const float T0 = T[0];
      load_window(pos);
      uint32_t base_u = a.p.root_base;
      uint32_t consumed = 0, woff = 0;  // bytes walked from pos; the window starts at pos + woff
      uint32_t clen0 = 1;
      bool alive = true, single = false;
      // The walk, one char (1-4 trie edges) per step c; a usable leaf at the
      // char boundary is inserted into slot c right away.
      StaticFor<1, Wc>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if (alive && pos + consumed >= nb) alive = false;
        // Refill the window when the next char may not be in it (walks past
        // 28 bytes: pieces of 10+ CJK chars).
        const bool refill = alive && consumed - woff + 4 > 32;
        if (__builtin_amdgcn_ballot_w64(refill) != 0) {
          if (refill) {
            load_window(pos + consumed);
            woff = consumed;
          }
        }
        if (alive) {
          uint32_t L = OneCharLenDev(r[0] & 0xFFu);
          if (L > nb - pos - consumed) L = nb - pos - consumed;
          if (c == 1) clen0 = L;
          uint32_t u = 0, scb = 0, node = 0;
          for (uint32_t t = 0; t < L; ++t) {
            const uint32_t byte = next_byte();
            // 0xFF matches the padded image's empty units: general path.
            if (byte == 0xFFu) bad = true;
            node = base_u ^ byte;
            if (c == 1 && t == 0) {
              const uint2 x = lds_root[byte];
              u = x.x;
              scb = x.y;
            } else {
              const auto x = __builtin_amdgcn_raw_buffer_load_b64(uvs_rsrc, node * 8u, 0, 0);
              u = x[0];
              scb = x[1];
            }
            if ((u & 0xFFu) != byte) {
              alive = false;
              break;
            }
            base_u = u >> 9;
            if ((u & 0x100u) && t + 1 < L) bad = true;  // a leaf inside a UTF-8 char: general path
          }
          if (alive) {
            consumed += L;
            // A usable node (leaf, not UNUSED) is one with a non-NaN score.
            const float s_node = __uint_as_float(scb);
            if ((u & 0x100u) && !__builtin_isnan(s_node)) {
              insert(cc, __fadd_rn(T0, s_node), pos, pos + consumed, node);
              if (c == 1) single = true;
            }
          }
        }
        // UNK node (unigram_model.cc:597-601) after this position's trie nodes.
        if constexpr (c == Wc - 1) {
          if (!single) insert(std::integral_constant<int, 1>{}, __fadd_rn(T0, a.p.unk_score), pos, pos + clen0, kNone);
        }
      });
      // Advance one char: shift the ring by one slot.
#pragma unroll
      for (int d = 0; d + 1 < Wc; ++d) {
        T[d] = T[d + 1];
        B[d] = B[d + 1];
        Nd[d] = Nd[d + 1];
      }
      T[Wc - 1] = 0.f;
      B[Wc - 1] = 0;
      Nd[Wc - 1] = kNone;
      has >>= 1;
      ambm >>= 1;
      pos += clen0;
    }
  } else {
    // ---- Char-position pass: ring slot d = end position (current byte + d);
    // slot 0 of the first position is BOS (score 0, backtrace 0: FreeList
    // zero-fill, freelist.h:79).
    float T[W];
    uint32_t B[W];
#pragma unroll
    for (int d = 0; d < W; ++d) {
      T[d] = 0.f;
      B[d] = 0;
    }
    uint64_t has = 1;  // bit d: slot d holds a node
    // Long sentences: the wave-cooperative kernel (flagged without a walk).
    const bool coop = a.coop_min_nb && nb >= a.coop_min_nb;
    if (coop) bad = true;
    auto insert = [&](auto dc, float bt, uint32_t begin, uint32_t end) {
      constexpr int d = decltype(dc)::value;
      if (!((has >> d) & 1)) {
        has |= (1ull << d);
        T[d] = bt;
        B[d] = begin;
      } else if (bt > T[d]) {
        const bool nr = NearTie(T[d], bt, tie_mag);
        if (nr || ((ambm >> d) & 1)) amb_update(dc, bt, nr, end, T[d], B[d]);
        T[d] = bt;
        B[d] = begin;
      }
    };
    uint32_t pos = 0;  // byte offset of the current char position
    while (nb > 0 && !coop) {
      if (pos > 0) bp_store(pos, pos - B[0]);
      if (pos >= nb) break;
      const float T0 = T[0];
      // Bytes pos .. pos+W-1 (packed, little endian), zero past the batch.
      uint32_t win[W / 4];
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
      uint32_t base_u = a.p.root_base;
      uint32_t rem = 0;        // bytes left in the current char (0: next byte starts one)
      uint32_t clen0 = 1;      // byte length of the first char
      uint64_t cbmask = 0;     // bit d: a char ends after byte d
      uint64_t leafmask = 0;   // bit d: a piece ends at a char boundary after byte d
      uint32_t lnode[W];
      bool alive = true, single = false;
      // Phase 1: the walk, one trie edge (one byte) per step; d = byte distance.
      StaticFor<1, W>([&](auto dc) {
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
            const uint32_t u = c ? a.units[node] : 0u;
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
      });
      // Phase 2: all leaf scores (independent loads), written over lnode[]:
      // a score, or a NaN tag 0x7FC00000|kind for USER_DEFINED / UNUSED.
      StaticFor<1, W>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        if ((leafmask >> d) & 1) {
          const int32_t v = a.values[lnode[d]];
          const int32_t k = v >> kKindShift;
          lnode[d] = k == 0 ? __float_as_uint(a.scores[v & kIdMask]) : (0x7FC00000u | k);
        }
      });
      // Phase 3: nodes in ascending length, then UNK (begin_nodes_ order).
      StaticFor<1, W>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        if ((leafmask >> d) & 1) {
          const uint32_t sb = lnode[d];
          const int32_t kind = (sb & 0x7FFFFFFFu) > 0x7F800000u ? static_cast<int32_t>(sb & 3u) : 0;
          if (kind != kKindUnused) {
            const float s_node = kind == kKindUserDefined
                                     ? UserDefinedScore(__popcll(cbmask & ((2ull << d) - 1)), a.p.max_score)
                                     : __uint_as_float(sb);
            insert(dc, __fadd_rn(T0, s_node), pos, pos + d);
            if (d == static_cast<int>(clen0)) single = true;
          }
        }
        // UNK node (unigram_model.cc:597-601) at the end of the first char.
        if constexpr (d <= 4) {
          if (d == static_cast<int>(clen0) && !single) insert(dc, __fadd_rn(T0, a.p.unk_score), pos, pos + clen0);
        }
      });
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

  // The lane's sentence index again, re-read from the permutation in LDS:
  // keeping the 64-bit index live across the walk cost a scratch spill.
  __asm__ volatile("" ::: "memory");
  const uint32_t sid_e = lds_sort[kBlock + tid];
  const uint64_t ie = base + sid_e;
  const bool valid_e = ie < a.n;
  // Debug knob (spm_hip_model_set_debug_corrupt_bp): zero one sentence's EOS
  // back-pointer after the forward pass, as a corrupted scratch byte would.
  if (a.corrupt_bp != ~0ull && valid_e && ie == a.corrupt_bp && nb > 0) bp_store(nb, 0);

  // Node (b, e) on the best path: exact-match walk, else UNK.
  uint32_t wide_node = kNone;  // kWide: the trie unit of the token the backtrace is at
  auto node_of = [&](uint32_t b, uint32_t e, int32_t *id_out, float *sc_out) {
    if constexpr (kWide) {
      // The forward pass kept the winner's unit (kNone: the UNK node).
      int32_t id = a.p.unk_id;
      float sc = a.p.unk_score;
      if (wide_node != kNone) {
        const int32_t v = a.values[wide_node];
        const int32_t kind = v >> kKindShift;
        id = v & kIdMask;
        if (kind == kKindUserDefined) {
          int chars = 0;
          for (uint32_t j = b; j < e; j += OneCharLenDev(byte_at(j))) ++chars;
          sc = UserDefinedScore(chars, a.p.max_score);
        } else {
          sc = a.scores[id];
        }
      }
      *id_out = id;
      *sc_out = sc;
      return;
    }
    if constexpr (kByte) {
      // The token's bytes (< 16) from one aligned 16-byte load + one dword
      // instead of a byte gather per byte, walked through (unit, score) pairs:
      // the node score comes with the last unit, so only the id is one more
      // gather (the kernel is bound by its gathers' address work).
      const uint32_t o = (lrel + b) & ~3u, sh = (lrel + b) & 3u;
      uint32_t w[5];
      if (static_cast<uint64_t>(o) + 20 <= blk_rem) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(bytes_rsrc, o, 0, 0);
        w[0] = x[0];
        w[1] = x[1];
        w[2] = x[2];
        w[3] = x[3];
        w[4] = __builtin_amdgcn_raw_buffer_load_b32(bytes_rsrc, o + 16, 0, 0);
      } else {  // the batch's last bytes: byte loads (a straddling dword reads 0)
#pragma unroll
        for (uint32_t k = 0; k < 5; ++k) {
          uint32_t x = 0;
#pragma unroll
          for (uint32_t t = 0; t < 4; ++t)
            if (o + 4 * k + t < blk_rem) x |= static_cast<uint32_t>(a.bytes[blk_al + o + 4 * k + t]) << (8 * t);
          w[k] = x;
        }
      }
      uint32_t r0 = __builtin_amdgcn_alignbyte(w[1], w[0], sh), r1 = __builtin_amdgcn_alignbyte(w[2], w[1], sh);
      uint32_t r2 = __builtin_amdgcn_alignbyte(w[3], w[2], sh), r3 = __builtin_amdgcn_alignbyte(w[4], w[3], sh);
      const auto uvs_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(a.units), 0,
                                                              static_cast<int>(a.num_units * 8u), 0x00020000);
      uint32_t nbase = a.p.root_base, node = 0, u = 0, scb = 0;
      bool found = true;
      for (uint32_t j = b; j < e; ++j) {
        const uint32_t c = r0 & 0xFFu;
        r0 = __builtin_amdgcn_alignbyte(r1, r0, 1);
        r1 = __builtin_amdgcn_alignbyte(r2, r1, 1);
        r2 = __builtin_amdgcn_alignbyte(r3, r2, 1);
        r3 >>= 8;
        node = nbase ^ c;
        if (c == 0) {
          found = false;
          break;
        }
        const auto uv = __builtin_amdgcn_raw_buffer_load_b64(uvs_rsrc, node * 8u, 0, 0);
        u = uv[0];
        scb = uv[1];
        if ((u & 0xFFu) != c) {
          found = false;
          break;
        }
        nbase = u >> 9;
      }
      // A usable node (leaf, not UNUSED) is exactly one with a non-NaN score
      // in the pair table (the byte kernel's models have no NaN score).
      const float s_node = __uint_as_float(scb);
      if (found && b < e && !__builtin_isnan(s_node)) {
        *id_out = a.values[node] & kIdMask;
        *sc_out = s_node;
      } else {
        *id_out = a.p.unk_id;
        *sc_out = a.p.unk_score;
      }
      return;
    }
    uint32_t nbase = a.p.root_base, node = 0, u = 0;
    bool found = true;
    for (uint32_t j = b; j < e; ++j) {
      const uint32_t c = byte_at(j);
      node = nbase ^ c;
      u = c ? a.units[node] : 0u;
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
  uint32_t stage_base = 0;  // kStage: the lane's first tile-local token index
  // Backtrace from EOS (score 0).  write=false only counts tokens (node
  // scores are needed only to resolve recorded near-ties).  Every step must
  // move left (begin < end): a zero or out-of-range back-pointer flags the
  // sentence instead of looping.
  auto backtrace = [&](bool write, int32_t *out_id, uint32_t *out_len, uint32_t kt) -> uint32_t {
    uint32_t e = nb, k = 0;
    float rs = 0.f;
    while (e > 0) {
      uint32_t b = e - bp_load(e);
      if constexpr (kWide) wide_node = (write || any_amb) ? a.bpn[b0 + e] : kNone;
#pragma unroll
      for (int t = 0; t < kAmb; ++t)
        if (ae[t] == e && __fadd_rn(aT2[t], rs) == __fadd_rn(aT[t], rs)) {
          b = aB2[t];
          if constexpr (kWide) wide_node = aN2[t];
        }
      if (b >= e || k >= nb) {
        bad = true;
        return 0;
      }
      if (write || any_amb) {
        int32_t id;
        float sc;
        node_of(b, e, &id, &sc);
        if (write) {
          if constexpr (kStage) {
            const uint32_t li = stage_base + (kt - 1 - k);  // tile-local token index
            if (li < kStageIds) lds_stage[li] = id;
            else out_id[kt - 1 - k] = id;
          } else {
            out_id[kt - 1 - k] = id;
          }
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
  if (valid_e && nb > 0 && !bad) k = backtrace(false, nullptr, nullptr, 0);
  if (bad) k = 0;
  if constexpr (kE) {
    // E-step outputs (estep_kernels.hip EArgs: Zlat, N, ntok; a flagged
    // sentence runs estep_general_kernel, which redoes all of it).
    if (valid_e) {
      a.e.Z[ie] = e_z;
      a.e.N[ie] = e_nodes;
      if (bad) {
        a.e.ntok[ie] = kNone;
        const uint32_t fk = atomicAdd(&a.e.fstatus[0], 1u);
        a.e.flagged[fk] = static_cast<uint32_t>(ie);
        atomicMax(&a.e.fstatus[1], nb);
      } else {
        a.e.ntok[ie] = k;
      }
    }
    return;
  }

  // Tile-exclusive scan of the token counts in SENTENCE order (lanes hold
  // the tile's sentences permuted by length), then the tile's global offset.
  lds_scan[sid_e] = k;
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
  // Tile-dense slots at the tile's first input byte (a tile has at most as
  // many tokens as bytes); tile_compact_kernel moves every tile to its final
  // offset once all tile counts are known, so no tile ever waits for
  // another (a decoupled look-back here measured 5.41 vs 4.63 ms per 10 M
  // sentences: finished tiles held their CU slots waiting for slower
  // predecessors, profiles/r03d_c2_output_ab.txt).
  if (tid == 0) a.tile_count[tile] = static_cast<uint64_t>(lds_wave[0]) + lds_wave[1] + lds_wave[2] + lds_wave[3];
  __syncthreads();                       // lds_scan[] complete
  const uint64_t rec = lds_scan[sid_e];  // tile-local exclusive offset
  const uint64_t dst = a.off[base] + rec;
  int32_t *__restrict__ out_ids = a.slot_ids;
  uint32_t *__restrict__ out_len = a.slot_len;
  if (valid_e) {
    if (bad) {
      const uint32_t fk = atomicAdd(&a.status[kStFlagged], 1u);
      a.flagged[fk] = static_cast<uint32_t>(ie);
      atomicMax(&a.status[kStMaxNb], nb);
      a.tok_off[ie + 1] = rec | kTokFlag;
    } else {
      stage_base = static_cast<uint32_t>(rec);
      if (k) backtrace(true, out_ids + dst, out_len ? out_len + dst : nullptr, k);
      a.tok_off[ie + 1] = rec + k;
    }
  }
  if (tile == 0 && tid == 0) a.tok_off[0] = 0;
  if constexpr (kStage) {
    // The staged ids (the tile's first kStageIds tokens) as one coalesced run.
    __syncthreads();
    const uint32_t tot = lds_wave[0] + lds_wave[1] + lds_wave[2] + lds_wave[3];
    const uint32_t m = tot < kStageIds ? tot : kStageIds;
    int32_t *__restrict__ dst0 = out_ids + a.off[base];
    for (uint32_t t = static_cast<uint32_t>(tid); t < m; t += kBlock) dst0[t] = static_cast<int32_t>(lds_stage[t]);
  }
  if (a.host_pub) {
    // Single-tile host call: every wave's output stores (pinned host memory)
    // complete, then the status words and the sequence number the host
    // polls for (EncodeHostSmall) — instead of copy commands and a stream
    // synchronization.
    __threadfence_system();
    __syncthreads();
    if (tid == 0) {
      for (int k = 0; k < kStWords; ++k)
        a.host_pub[1 + k] = __hip_atomic_load(&a.status[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(&a.host_pub[0], a.pub_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------
// General kernel: the reference Lattice, literally (node lists, Viterbi over
// every (rnode, lnode) pair in end_nodes_ insertion order, strict '>').
// One listed sentence per lane, scratch slab per lane.
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
  const uint32_t *__restrict__ list;  // sentence indices (nullptr: identity)
  const uint32_t *__restrict__ count; // device count of `list`
  uint64_t list_n;                    // used when list == nullptr
  uint8_t *__restrict__ scratch;
  uint64_t slab_bytes;
  uint32_t max_nb;                    // slab sized for sentences <= max_nb bytes
  uint32_t *__restrict__ ovf_list;    // longer sentences go here (nullptr: error)
  uint32_t *__restrict__ ovf_count;
  uint32_t *__restrict__ error;
  uint32_t lanes;                     // slabs in scratch (lanes beyond stay idle)
};

__global__ __launch_bounds__(64) void unigram_general_kernel(GeneralArgs a) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (tid >= a.lanes) return;
  const uint64_t nthreads = a.lanes;
  const uint64_t total = a.list ? *a.count : a.list_n;
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
      if (a.ovf_list) {
        a.ovf_list[atomicAdd(a.ovf_count, 1u)] = i;
      } else {
        atomicOr(a.error, 1u);
        a.ntok[i] = 0;
      }
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

hipError_t LaunchUnigramFast(UnigramKernel kind, int W, const UnigramLaunch &l, hipStream_t st) {
  FastArgs a{l.bytes, l.off, l.n, l.capacity, l.units, l.values, l.scores, l.num_units, l.p, l.ids, l.len,
             l.tok_off, l.bp, l.flagged, l.status, l.tile_count, l.corrupt_bp, l.chain, l.slot_ids, l.slot_len,
             EStepForwardOut{}, l.bpn, l.stage_src, l.stage_dst, l.stage_zero, l.stage_words, l.host_pub, l.pub_seq,
             l.coop_min_nb};
  const uint64_t blocks64 = FastTiles(l.n);
  if (blocks64 == 0) return hipSuccess;
  if (blocks64 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  // The staged image and the publication are one block's work.
  if ((l.stage_src || l.host_pub) && blocks64 != 1) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(blocks64));
  // 7 waves/SIMD: 72 VGPRs, no spill.  8 waves (64 VGPRs, 14 spilled)
  // measured 6.78 vs 5.41 ms per 10 M sentences (profiles/r03c_c2_waves_ab.txt).
  if (kind == UnigramKernel::kByte && W == 16) {
    hipLaunchKernelGGL((unigram_fast_kernel<16, true>), grid, dim3(kBlock), 0, st, a);
  } else if (kind == UnigramKernel::kWide && W == 16) {
    hipLaunchKernelGGL((unigram_fast_kernel<16, false, 3, false, true>), grid, dim3(kBlock), 0, st, a);
  } else if (kind == UnigramKernel::kChar && W == 16) {
    hipLaunchKernelGGL((unigram_fast_kernel<16, false>), grid, dim3(kBlock), 0, st, a);
  } else if (kind == UnigramKernel::kChar && W == 32) {
    hipLaunchKernelGGL((unigram_fast_kernel<32, false>), grid, dim3(kBlock), 0, st, a);
  } else if (kind == UnigramKernel::kChar && W == 64) {
    hipLaunchKernelGGL((unigram_fast_kernel<64, false>), grid, dim3(kBlock), 0, st, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t LaunchUnigramEStepForward(const UnigramLaunch &l, const EStepForwardOut &e, hipStream_t st) {
  FastArgs a{l.bytes, l.off, l.n, l.capacity, l.units, l.values, l.scores, l.num_units, l.p, l.ids, l.len,
             l.tok_off, l.bp, l.flagged, l.status, l.tile_count, ~0ull, nullptr, nullptr, nullptr, e};
  const uint64_t blocks64 = FastTiles(l.n);
  if (blocks64 == 0) return hipSuccess;
  if (blocks64 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  // 4 waves/SIMD (128 VGPRs, 14 spilled): c4 FAST 0.272 vs 0.281 s/epoch at
  // 3 waves, PARITY 0.415 vs 0.410 (profiles/r03y_estep_byte_forward_ab.txt).
  hipLaunchKernelGGL((unigram_fast_kernel<16, true, kEStepWaves, true>), dim3(static_cast<unsigned>(blocks64)),
                     dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

hipError_t LaunchUnigramGeneral(const UnigramLaunch &l, const GeneralLaunch &g, hipStream_t st) {
  GeneralArgs a{l.bytes, l.off, l.gen_units, l.values, l.scores, l.p, g.slot_ids, g.slot_len, g.ntok, g.list,
                g.count, g.list_n, g.scratch, g.slab_bytes, g.max_nb, g.ovf_list, g.ovf_count, g.error,
                g.threads};
  const unsigned blocks = (g.threads + 63) / 64;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(unigram_general_kernel, dim3(blocks), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace spm_amd
