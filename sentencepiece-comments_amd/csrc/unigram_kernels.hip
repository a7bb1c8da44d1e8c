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
#include "device_model.h"
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
};

constexpr int kBlock = 256;
constexpr int kLdsBpPos = 64;  // back-pointer bytes kept in LDS per lane

template <int W>
__global__ __launch_bounds__(kBlock) void unigram_fast_kernel(FastArgs a) {
  // Back-pointer bytes of byte positions [0, kLdsBpPos) of each lane's
  // sentence: word (pos/4)*kBlock + tid, byte pos%4 (lanes at the same pos
  // hit consecutive words).
  __shared__ uint32_t lds_bp[(kLdsBpPos / 4) * kBlock];
  __shared__ uint32_t lds_wave[kBlock / 64];
  uint8_t *lbp = reinterpret_cast<uint8_t *>(lds_bp);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * kBlock;
  for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * kBlock; base < a.n; base += step) {
    const uint64_t i = base + tid;
    const bool valid = i < a.n;
    const uint64_t b0 = valid ? a.off[i] : 0;
    const uint32_t nb = valid ? static_cast<uint32_t>(a.off[i + 1] - b0) : 0;
    const uint8_t *__restrict__ s = a.bytes + b0;
    uint8_t *__restrict__ gbp = a.bp + b0;
    auto bp_store = [&](uint32_t pos, uint32_t v) {
      if (pos < kLdsBpPos) lbp[((pos >> 2) * kBlock + tid) * 4 + (pos & 3)] = static_cast<uint8_t>(v);
      else gbp[pos] = static_cast<uint8_t>(v);
    };
    auto bp_load = [&](uint32_t pos) -> uint32_t {
      return pos < kLdsBpPos ? lbp[((pos >> 2) * kBlock + tid) * 4 + (pos & 3)] : gbp[pos];
    };

    // Ring slot d = end position (current char + d).  Slot 0 of the first
    // position is BOS (score 0, backtrace 0: FreeList zero-fill,
    // freelist.h:79).
    float T[W];
    uint32_t B[W];
#pragma unroll
    for (int d = 0; d < W; ++d) {
      T[d] = 0.f;
      B[d] = 0;
    }
    uint64_t has = 1;
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

    // Insert node [begin, end) with backtrace score bt into ring slot d.
    // Nodes reach a slot in ascending begin order (= end_nodes_ order).
    auto insert = [&](auto dc, float bt, uint32_t begin, uint32_t end) {
      constexpr int d = decltype(dc)::value;
      if (!((has >> d) & 1)) {
        has |= (1ull << d);
        T[d] = bt;
        B[d] = begin;
      } else if (bt > T[d]) {
        const bool nr = NearTie(T[d], bt, a.p.tie_mag);
        int slot = -1, free_slot = -1;
#pragma unroll
        for (int k = 0; k < kAmbEntries; ++k) {
          if (ae[k] == end) slot = k;
          if (ae[k] == kNone && free_slot < 0) free_slot = k;
        }
        if (slot >= 0) {
          // Older setter (aT2) also near the new max: 3-deep tie chain.
#pragma unroll
          for (int k = 0; k < kAmbEntries; ++k)
            if (k == slot) {
              if (NearTie(aT2[k], bt, a.p.tie_mag)) bad = true;
              if (nr) {
                aT2[k] = T[d];
                aB2[k] = B[d];
                aT[k] = bt;
              } else {
                ae[k] = kNone;
              }
            }
        } else if (nr) {
          if (free_slot < 0) bad = true;
          any_amb = true;
#pragma unroll
          for (int k = 0; k < kAmbEntries; ++k)
            if (k == free_slot) {
              ae[k] = end;
              aT2[k] = T[d];
              aB2[k] = B[d];
              aT[k] = bt;
            }
        }
        T[d] = bt;
        B[d] = begin;
      }
    };

    uint32_t pos = 0;  // byte offset of the current char position
    while (nb > 0) {
      if (pos > 0) bp_store(pos, pos - B[0]);
      if (pos >= nb) break;
      const float T0 = T[0];
      uint32_t base_u = a.p.root_base;
      uint32_t q = pos;
      uint32_t clen0 = 1;
      bool alive = true, single = false;
      auto stepd = [&](auto dc) {
        constexpr int d = decltype(dc)::value;
        if (alive) {
          if (q >= nb) {
            alive = false;
          } else {
            const uint32_t lead = s[q];
            uint32_t cl = OneCharLenDev(lead);
            if (cl > nb - q) cl = nb - q;
            if (d == 1) clen0 = cl;
            uint32_t u = 0, node = 0;
            for (uint32_t j = 0; j < cl; ++j) {
              const uint32_t c = j == 0 ? lead : static_cast<uint32_t>(s[q + j]);
              node = base_u ^ c;
              u = c ? a.units[node] : 0u;
              if ((u & 0xFFu) != c || c == 0) {
                alive = false;
                break;
              }
              base_u = u >> 9;
              if (j + 1 < cl && (u & 0x100u)) bad = true;  // leaf inside a char
            }
            if (alive) {
              q += cl;
              if (u & 0x100u) {
                const int32_t v = a.values[node];
                const int32_t kind = v >> kKindShift;
                if (kind != kKindUnused) {
                  const float sc = kind == kKindUserDefined ? UserDefinedScore(d, a.p.max_score)
                                                            : a.scores[v & kIdMask];
                  insert(dc, __fadd_rn(T0, sc), pos, q);
                  if (d == 1) single = true;
                }
              }
            }
          }
        }
        if (d == 1 && !single)  // UNK node (unigram_model.cc:597-601)
          insert(dc, __fadd_rn(T0, a.p.unk_score), pos, pos + clen0);
      };
      StaticFor<1, W>(stepd);
      // Advance one char: shift the ring.
#pragma unroll
      for (int d = 0; d + 1 < W; ++d) {
        T[d] = T[d + 1];
        B[d] = B[d + 1];
      }
      T[W - 1] = 0.f;
      B[W - 1] = 0;
      has >>= 1;
      pos += clen0;
    }

    // Node (b, e) on the best path: exact-match walk, else UNK.
    auto node_of = [&](uint32_t b, uint32_t e, int32_t *id_out, float *sc_out) {
      uint32_t nbase = a.p.root_base, node = 0, u = 0;
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
      int32_t id = a.p.unk_id;
      float sc = a.p.unk_score;
      if (found && (u & 0x100u)) {
        const int32_t v = a.values[node];
        const int32_t kind = v >> kKindShift;
        if (kind != kKindUnused) {
          id = v & kIdMask;
          if (kind == kKindUserDefined) {
            int chars = 0;
            for (uint32_t j = b; j < e; j += OneCharLenDev(s[j])) ++chars;
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
    // Block-exclusive scan of the token counts → block-dense output slots.
    uint32_t x = k;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) lds_wave[wave] = x;
    __syncthreads();
    uint32_t excl = x - k;
    for (int w = 0; w < wave; ++w) excl += lds_wave[w];
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

hipError_t LaunchUnigramFast(int W, const UnigramLaunch &l, hipStream_t st) {
  FastArgs a{l.bytes, l.off, l.n, l.units, l.values, l.scores, l.p,
             l.slot_ids, l.slot_len, l.ntok, l.lo, l.bp, l.flagged, l.status};
  const uint64_t blocks64 = (l.n + kBlock - 1) / kBlock;
  const unsigned blocks = static_cast<unsigned>(blocks64 < (1u << 30) ? blocks64 : (1u << 30));
  if (blocks == 0) return hipSuccess;
  switch (W) {
    case 16: hipLaunchKernelGGL(unigram_fast_kernel<16>, dim3(blocks), dim3(256), 0, st, a); break;
    case 32: hipLaunchKernelGGL(unigram_fast_kernel<32>, dim3(blocks), dim3(256), 0, st, a); break;
    case 64: hipLaunchKernelGGL(unigram_fast_kernel<64>, dim3(blocks), dim3(256), 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
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
