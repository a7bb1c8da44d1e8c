// Unigram Viterbi encode, lane-decoupled form (gfx950).
//
// Same result as unigram_fast_kernel's byte-position pass (unigram_kernels.hip;
// reference: unigram::Model::Encode, unigram_model.cc:705-720 = SetSentence
// :147-187 + PopulateNodes :535-604 + Viterbi :222-261), scheduled differently.
//
// The fast kernel walks byte positions in lockstep across the wave: every
// (pair of) position(s) costs the DEEPEST trie walk among the wave's 64 lanes,
// so with the synthetic c2 corpus a wave runs ~176 dependent load rounds for
// ~84 unit loads per sentence (spm_hip_model_trie_stats' wave model), and the
// kernel is issue-bound on that mostly-idle work.  Here every lane runs its
// own sentence as a state machine, ONE trie step per round:
//
//   START  (position p is a char start; all nodes ending at p are in):
//          T0 = ring T[p & 15], back-pointer byte bp[p] = ring D[p & 15],
//          clear the slot (it is end p + 16 next), take the prefetched 16-byte
//          window of the sentence at p, prefetch the window of the next char
//          start;
//   STEP d (d = 1, 2, ...): c = byte p+d-1, node = base ^ c, one unit load and
//          one leaf-score load (both addressed by node, issued together);
//          a usable leaf inserts (end p+d, T0 + score); the UNK node
//          (unigram_model.cc:597-601) is inserted at end p + clen0 when depth
//          clen0 has no usable node; a label mismatch ends the walk and the
//          next round STARTs at p + clen0.
//
// Nodes reach a ring slot in ascending begin order (each lane finishes a walk
// before starting the next), which is the reference's end_nodes_ order, so
// the Viterbi max / first-setter back-pointer and the near-tie ambiguity
// entries are those of the fast kernel (see its header for the identity
// T_b + s).  A wave now takes max over lanes of (unit loads) rounds (~47 per
// two chains, ~100 per chain, vs ~176 lockstep).
//
// State: the 16-slot ring (T float, D = end - begin of the first setter,
// u8) lives in LDS, [slot][lane] so every access is bank-conflict free;
// back-pointer bytes go to a global scratch region per sentence (8-byte
// aligned, written as 8-byte words).  The backtrace, token count, block-dense
// output slots and the general-path flags are the fast kernel's.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_common.h"
#include "kernels.h"

namespace spm_amd {
namespace {

constexpr int kLBlock = 256;
constexpr int kRing = 16;

// kOpt bit 0: one 8-byte {unit, leaf score} entry per trie step (uvs table)
// instead of two 4-byte loads; bit 1: the first kTop entries (the BFS top of
// the array) staged in LDS, lanes whose node is below kTop read LDS.
constexpr uint32_t kTop = 1024;

template <int kOpt>
__global__ __launch_bounds__(kLBlock) void unigram_lane_kernel(UnigramLaunch a, const uint2 *__restrict__ uvs) {
  __shared__ uint2 lds_top[(kOpt & 2) ? kTop : 1];
  __shared__ float ringT[kRing * kLBlock];
  __shared__ uint32_t ringD[(kRing / 4) * kLBlock];
  __shared__ uint32_t lds_sort[2 * kLBlock];
  __shared__ uint32_t lds_wave[kLBlock / 64];
  __shared__ uint32_t lds_scan[kLBlock];
  uint8_t *ringDb = reinterpret_cast<uint8_t *>(ringD);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kLBlock;
  const uint64_t total_bytes = a.off[a.n];
  const UnigramParams P = a.p;
  const auto units_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(a.units), 0,
                                                            static_cast<int>(a.num_units * 4u), 0x00020000);
  const auto vscore_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.vscore), 0,
                                                             static_cast<int>(a.num_units * 4u), 0x00020000);
  const auto uvs_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint2 *>(uvs), 0,
                                                          static_cast<int>(a.num_units * 8u), 0x00020000);
  if constexpr ((kOpt & 2) != 0) {
    for (uint32_t k = threadIdx.x; k < kTop; k += kLBlock)
      lds_top[k] = k < a.num_units ? uvs[k] : make_uint2(0xFFu, 0x7FC00000u);
    __syncthreads();
  }
  auto tslot = [&](uint32_t slot) -> float & { return ringT[slot * kLBlock + tid]; };
  auto dslot = [&](uint32_t slot) -> uint8_t & {
    return ringDb[((slot >> 2) * kLBlock + tid) * 4 + (slot & 3)];
  };

  for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * kLBlock; base < a.n; base += step) {
    // Counting sort of the block's sentences by length: each wave's lanes get
    // similar lengths, so the wave's round count (its longest lane) drops.
    uint32_t sid;
    {
      uint32_t *hist = lds_sort, *perm = lds_sort + kLBlock;
      const uint64_t ii = base + tid;
      const uint32_t len = ii < a.n ? static_cast<uint32_t>(a.off[ii + 1] - a.off[ii]) : 0u;
      const uint32_t bucket = len < kLBlock - 1 ? len : kLBlock - 1;
      hist[tid] = 0;
      __syncthreads();
      const uint32_t r = atomicAdd(&hist[bucket], 1u);
      __syncthreads();
      if (wave == 0) {
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
    // Back-pointer region: 8-byte aligned, disjoint per sentence (scratch of
    // total + 8 n + 16 bytes).
    uint8_t *__restrict__ gbp = a.bp + ((b0 + 8 * i + 7) & ~7ull);

    // Sentence bytes through a buffer resource based at the block's first
    // aligned dword (out of range → 0; the batch's last partial dword by
    // byte loads).
    const uint64_t blk_al = a.off[base] & ~3ull;
    const uint64_t blk_rem64 = total_bytes - blk_al;
    const uint32_t blk_rem = static_cast<uint32_t>(blk_rem64 < 0x7FFFFFF0ull ? blk_rem64 : 0x7FFFFFF0ull);
    const auto bytes_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.bytes + blk_al), 0,
                                                              static_cast<int>(blk_rem), 0x00020000);
    const uint32_t lane_off = static_cast<uint32_t>(b0 - blk_al);
    auto word_at = [&](uint32_t o) -> uint32_t {  // o: block-relative, dword aligned
      if (o + 4 <= blk_rem) return __builtin_amdgcn_raw_buffer_load_b32(bytes_rsrc, o, 0, 0);
      uint32_t x = 0;
#pragma unroll
      for (uint32_t t = 0; t < 4; ++t)
        if (o + t < blk_rem) x |= static_cast<uint32_t>(a.bytes[blk_al + o + t]) << (8 * t);
      return x;
    };
    // Bytes [q, q + 16) of the sentence, zero at and beyond nb.
    auto load_window = [&](uint32_t q, uint32_t *w) {
      const uint32_t o = lane_off + q;
      const uint32_t oa = o & ~3u, sh = o & 3u;
      uint32_t x[5];
      if (oa + 20 <= blk_rem) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(bytes_rsrc, oa, 0, 0);
        x[0] = v[0];
        x[1] = v[1];
        x[2] = v[2];
        x[3] = v[3];
        x[4] = __builtin_amdgcn_raw_buffer_load_b32(bytes_rsrc, oa + 16, 0, 0);
      } else {
#pragma unroll
        for (int k = 0; k < 5; ++k) x[k] = word_at(oa + 4 * k);
      }
      const uint32_t rem = nb - q;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t y = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sh);
        const int lim = static_cast<int>(rem) - 4 * k;
        y = lim >= 4 ? y : lim <= 0 ? 0u : (y & ((1u << (8 * lim)) - 1u));
        w[k] = y;
      }
    };

    // Ring: slot 0 = BOS (score 0, freelist.h:79 zero fill), others empty.
#pragma unroll
    for (int k = 0; k < kRing; ++k) tslot(k) = k == 0 ? 0.f : -__builtin_inff();
#pragma unroll
    for (int k = 0; k < kRing / 4; ++k) ringD[k * kLBlock + tid] = 0;

    uint32_t ambm = 0;  // bit slot: slot has an ambiguity entry
    uint32_t ae[kAmbEntries], aB2[kAmbEntries];
    float aT[kAmbEntries], aT2[kAmbEntries];
#pragma unroll
    for (int k = 0; k < kAmbEntries; ++k) {
      ae[k] = kNone;
      aB2[k] = 0;
      aT[k] = 0.f;
      aT2[k] = 0.f;
    }
    bool bad = false, any_amb = false;
    // Near-tie entry of end e (see unigram_fast_kernel::amb_update); Tc / Bc
    // are the slot's current max and its setter's begin.
    auto amb_update = [&](uint32_t slot, float bt, bool nr, uint32_t e, float Tc, uint32_t Bc) {
      int hit = -1, free_slot = -1;
#pragma unroll
      for (int k = 0; k < kAmbEntries; ++k) {
        if (ae[k] == e) hit = k;
        if (ae[k] == kNone && free_slot < 0) free_slot = k;
      }
      if (hit >= 0) {
#pragma unroll
        for (int k = 0; k < kAmbEntries; ++k)
          if (k == hit) {
            if (NearTie(aT2[k], bt, P.tie_mag)) bad = true;  // 3-deep tie chain
            if (nr) {
              aT2[k] = Tc;
              aB2[k] = Bc;
              aT[k] = bt;
            } else {
              ae[k] = kNone;
              ambm &= ~(1u << slot);
            }
          }
      } else if (nr) {
        if (free_slot < 0) bad = true;
        any_amb = true;
        ambm |= 1u << slot;
#pragma unroll
        for (int k = 0; k < kAmbEntries; ++k)
          if (k == free_slot) {
            ae[k] = e;
            aT2[k] = Tc;
            aB2[k] = Bc;
            aT[k] = bt;
          }
      }
    };

    uint32_t p = 0, d = 0, clen0 = 1, base_u = P.root_base;
    float T0 = 0.f;
    uint32_t win[4] = {0, 0, 0, 0}, nwin[4] = {0, 0, 0, 0};
    bool done = !valid || nb == 0;
    bool walking = false;
    uint64_t bpacc = 0;
    uint32_t bpblk = 0;
    if (!done) load_window(0, nwin);

    while (__builtin_amdgcn_ballot_w64(!done) != 0) {
      if (!done && !walking) {
        // START at char start p: every node ending at p has been inserted.
        const uint32_t slot = p & (kRing - 1);
        T0 = tslot(slot);
        const uint32_t D = dslot(slot);
        tslot(slot) = -__builtin_inff();
        ambm &= ~(1u << slot);
        if (p > 0) {
          const uint32_t blk = p >> 3;
          if (blk != bpblk) {
            *reinterpret_cast<uint64_t *>(gbp + 8 * bpblk) = bpacc;
            bpacc = 0;
            bpblk = blk;
          }
          bpacc |= static_cast<uint64_t>(D) << (8 * (p & 7));
        }
        if (p >= nb) {
          *reinterpret_cast<uint64_t *>(gbp + 8 * bpblk) = bpacc;
          done = true;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) win[k] = nwin[k];
          clen0 = OneCharLenDev(win[0] & 0xFFu);
          if (clen0 > nb - p) clen0 = nb - p;
          const uint32_t pn = p + clen0;
          if (pn < nb) load_window(pn, nwin);
          walking = true;
          d = 0;
          base_u = P.root_base;
        }
      }
      if (walking) {
        const uint32_t c = win[0] & 0xFFu;
        win[0] = __builtin_amdgcn_alignbyte(win[1], win[0], 1);
        win[1] = __builtin_amdgcn_alignbyte(win[2], win[1], 1);
        win[2] = __builtin_amdgcn_alignbyte(win[3], win[2], 1);
        win[3] >>= 8;
        ++d;
        const uint32_t node = base_u ^ c;
        uint32_t u;
        float sc;
        if constexpr ((kOpt & 1) != 0) {
          uint2 x;
          if ((kOpt & 2) != 0 && node < kTop) {
            x = lds_top[node];
          } else {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(uvs_rsrc, node * 8u, 0, 0);
            x = make_uint2(v[0], v[1]);
          }
          u = x.x;
          sc = __uint_as_float(x.y);
        } else {
          u = __builtin_amdgcn_raw_buffer_load_b32(units_rsrc, node * 4u, 0, 0);
          sc = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vscore_rsrc, node * 4u, 0, 0));
        }
        // A 0xFF input byte could match an empty unit of the 0xFF-padded
        // image: such sentences take the general path.
        if (c == 0xFFu) bad = true;
        const bool match = (u & 0xFFu) == c;
        base_u = u >> 9;
        const bool usable = match && !__builtin_isnan(sc);
        // At most one node per round: the piece [p, p + d) or, when depth
        // clen0 has no usable node, the UNK node [p, p + clen0).
        const bool unk = !usable && (d == clen0 || (!match && d < clen0));
        if (usable || unk) {
          const uint32_t len = usable ? d : clen0;
          const uint32_t e = p + len;
          const float bt = __fadd_rn(T0, usable ? sc : P.unk_score);
          const uint32_t slot = e & (kRing - 1);
          const float Tc = tslot(slot);
          const bool gt = bt > Tc;
          const bool rare = gt && (NearTieHi(Tc, bt, P.tie_mag) || ((ambm >> slot) & 1u));
          if (__builtin_amdgcn_ballot_w64(rare) != 0) {
            if (rare) amb_update(slot, bt, NearTieHi(Tc, bt, P.tie_mag), e, Tc, e - dslot(slot));
          }
          if (gt) {
            tslot(slot) = bt;
            dslot(slot) = static_cast<uint8_t>(len);
          }
        }
        if (!match || d >= kRing) {
          walking = false;
          p += clen0;
        }
      }
      if (bad) {
        done = true;
        walking = false;
      }
    }

    // Node (b, e) on the best path: exact-match walk, else UNK.
    auto node_of = [&](uint32_t b, uint32_t e, int32_t *id_out, float *sc_out) {
      uint32_t nbase = P.root_base, node = 0, u = 0;
      bool found = true;
      for (uint32_t j = b; j < e; ++j) {
        const uint32_t c = s[j];
        node = nbase ^ c;
        u = c ? a.units[node] : 0u;
        if ((u & 0xFFu) != c || c == 0) {
          found = false;
          break;
        }
        nbase = u >> 9;
      }
      int32_t id = P.unk_id;
      float sc = P.unk_score;
      if (found && (u & 0x100u)) {
        const int32_t v = a.values[node];
        const int32_t kind = v >> kKindShift;
        if (kind != kKindUnused) {
          id = v & kIdMask;
          if (kind == kKindUserDefined) {
            int chars = 0;
            for (uint32_t j = b; j < e; j += OneCharLenDev(s[j])) ++chars;
            sc = UserDefinedScore(chars, P.max_score);
          } else {
            sc = a.scores[id];
          }
        }
      }
      *id_out = id;
      *sc_out = sc;
    };
    // Backtrace from EOS (score 0); write=false only counts tokens.
    auto backtrace = [&](bool write, int32_t *out_id, uint32_t *out_len, uint32_t kt) -> uint32_t {
      uint32_t e = nb, k = 0;
      float rs = 0.f;
      while (e > 0) {
        uint32_t b = e - gbp[e];
#pragma unroll
        for (int t = 0; t < kAmbEntries; ++t)
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
        if (k) backtrace(true, a.slot_ids + dst, a.slot_len ? a.slot_len + dst : nullptr, k);
        a.ntok[i] = k;
        a.lo[i] = excl;
      }
    }
  }
}

}  // namespace

hipError_t LaunchUnigramLane(int opt, const UnigramLaunch &l, const uint2 *uvs, hipStream_t st) {
  const uint64_t blocks64 = (l.n + kLBlock - 1) / kLBlock;
  const unsigned blocks = static_cast<unsigned>(blocks64 < (1u << 30) ? blocks64 : (1u << 30));
  if (blocks == 0) return hipSuccess;
  switch (opt & 3) {
    case 0: hipLaunchKernelGGL((unigram_lane_kernel<0>), dim3(blocks), dim3(kLBlock), 0, st, l, uvs); break;
    case 1: hipLaunchKernelGGL((unigram_lane_kernel<1>), dim3(blocks), dim3(kLBlock), 0, st, l, uvs); break;
    case 2: hipLaunchKernelGGL((unigram_lane_kernel<2>), dim3(blocks), dim3(kLBlock), 0, st, l, uvs); break;
    default: hipLaunchKernelGGL((unigram_lane_kernel<3>), dim3(blocks), dim3(kLBlock), 0, st, l, uvs); break;
  }
  return hipGetLastError();
}

}  // namespace spm_amd
