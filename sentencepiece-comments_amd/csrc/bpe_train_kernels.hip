// BPE trainer pair census on gfx950 (the bulk "pair-frequency reduction" of
// bpe::Trainer::Train, bpe_model_trainer.cc:200-230 + the first
// UpdateActiveSymbols' ComputeFreq :87-113).
//
// The reference walks every sentence twice on one thread: GetCharSymbol for
// every char (creating char symbols in first-occurrence order), then
// AddNewPair for every adjacent pair (creating the valid pair symbols in
// first-occurrence order and appending EncodePos(sid, l, l+1) to their
// position sets); the first UpdateActiveSymbols then runs ComputeFreq on every
// pair symbol, which erases overlapping positions of (a, a) pairs (in a run of
// identical chars every second pair) and sums the sentence freqs of the rest.
//
// Here: one sentence per lane decodes UTF-8 (util.cc DecodeUTF8 rules) into
// code points and the start of each char's run of identical chars; every
// adjacent pair becomes a record (left << 21 | right, EncodePos); a stable
// radix sort by pair key groups the records in ascending position order; the
// kept flag of a record is "left != right, or an even offset from its run
// start" (exactly ComputeFreq's erase rule on a fresh symbol); segmented
// sums give each pair's freq; the unique pairs are then ordered by their
// first position.  The host creates the symbols in that order, so its
// unordered_map sees the reference's insertion sequence.
#include <hip/hip_runtime.h>

#include "scratch_cache.h"
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/spm_hip.h"
#include "device_types.h"

struct spm_hip_bpe_census {
  std::vector<uint32_t> char_codes;   // decoded text, CSR by sentence
  std::vector<uint64_t> char_off;     // n + 1
  std::vector<uint32_t> uchars;       // unique chars, first-occurrence order
  std::vector<uint64_t> pair_keys;    // left << 21 | right, first-occurrence order
  std::vector<uint64_t> pair_freq;    // sum of sentence freq over kept positions
  std::vector<uint64_t> pos_off;      // num_pairs + 1
  std::vector<uint64_t> positions;    // kept EncodePos, ascending per pair
  float device_ms = 0.f;
};

namespace spm_amd {
namespace {

std::string g_census_error;

__device__ uint32_t DecodeDev(const uint8_t *b, uint64_t len, uint32_t *mblen) {
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

__global__ void census_count_kernel(const uint8_t *bytes, const uint64_t *off, uint64_t n, uint64_t *cnt,
                                    uint32_t *too_long) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *s = bytes + off[i];
  const uint64_t nb = off[i + 1] - off[i];
  uint64_t c = 0;
  for (uint64_t q = 0; q < nb;) {
    uint32_t ml;
    (void)DecodeDev(s + q, nb - q, &ml);
    q += ml;
    ++c;
  }
  cnt[i] = c;
  if (c > 65536) atomicOr(too_long, 1u);  // EncodePos CHECK_LE(l, kuint16max)
}

// codes, run start (offset within the sentence of the run of equal chars),
// and one pair record per char after the first of its sentence (at
// rec_off[i] + k - 1: sentence i contributes max(count - 1, 0) records).
__global__ void census_decode_kernel(const uint8_t *bytes, const uint64_t *off, uint64_t n,
                                     const uint64_t *char_off, const uint64_t *rec_off, uint32_t *codes,
                                     uint32_t *run_start, uint64_t *rec_key, uint64_t *rec_pos) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *s = bytes + off[i];
  const uint64_t nb = off[i + 1] - off[i];
  const uint64_t c0 = char_off[i];
  const uint64_t r0 = rec_off[i];
  uint64_t k = 0;
  uint32_t prev = 0, rs = 0;
  for (uint64_t q = 0; q < nb; ++k) {
    uint32_t ml;
    const uint32_t cp = DecodeDev(s + q, nb - q, &ml);
    q += ml;
    if (k == 0 || cp != prev) rs = static_cast<uint32_t>(k);
    codes[c0 + k] = cp;
    run_start[c0 + k] = rs;
    if (k > 0) {
      rec_key[r0 + k - 1] = static_cast<uint64_t>(prev) << 21 | cp;
      rec_pos[r0 + k - 1] = i << 32 | (k - 1) << 16 | k;
    }
    prev = cp;
  }
}

// Sorted records: segment heads, kept flags (ComputeFreq's erase rule) and
// the sentence freq of every kept record.
__global__ void census_flag_kernel(const uint64_t *key, const uint64_t *pos, uint64_t m,
                                   const uint64_t *char_off, const uint32_t *run_start,
                                   const int64_t *freq, uint32_t *head, uint32_t *kept,
                                   uint64_t *kfreq) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint64_t k = key[j], p = pos[j];
  head[j] = (j == 0 || key[j - 1] != k) ? 1u : 0u;
  const uint32_t l = static_cast<uint32_t>((p >> 16) & 0xFFFFu);
  const uint64_t sid = p >> 32;
  bool keep = true;
  if ((k >> 21) == (k & 0x1FFFFFu)) keep = ((l - run_start[char_off[sid] + l]) & 1u) == 0;
  kept[j] = keep ? 1u : 0u;
  kfreq[j] = keep ? static_cast<uint64_t>(freq[sid]) : 0ull;
}

// One thread per segment (unique pair): key, first position, freq sum and
// the range of its kept positions in the compacted list.
__global__ void census_segment_kernel(const uint32_t *seg_begin, uint64_t nseg, uint64_t m,
                                      const uint64_t *key, const uint64_t *pos,
                                      const uint64_t *freq_incl, const uint64_t *kept_incl,
                                      uint64_t *s_key, uint64_t *s_first, uint64_t *s_freq,
                                      uint64_t *s_kept_lo, uint64_t *s_kept_hi) {
  const uint64_t s = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  const uint64_t b = seg_begin[s], e = s + 1 < nseg ? seg_begin[s + 1] : m;
  s_key[s] = key[b];
  s_first[s] = pos[b];
  s_freq[s] = freq_incl[e - 1] - (b ? freq_incl[b - 1] : 0ull);
  s_kept_lo[s] = b ? kept_incl[b - 1] : 0ull;
  s_kept_hi[s] = kept_incl[e - 1];
}

struct ToU64 {
  __host__ __device__ uint64_t operator()(uint32_t x) const { return x; }
};

#define C_TRY(expr)                                                            \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      g_census_error = std::string(#expr) + ": " + hipGetErrorString(_e);      \
      return SPM_INTERNAL;                                                     \
    }                                                                          \
  } while (0)

struct Scratch {
  std::vector<void *> p;
  template <typename T>
  T *Get(uint64_t count, hipError_t *err) {
    void *v = nullptr;
    const hipError_t e = DevMalloc(&v, std::max<uint64_t>(count, 1) * sizeof(T));
    if (e != hipSuccess) {
      *err = e;
      return nullptr;
    }
    p.push_back(v);
    return static_cast<T *>(v);
  }
  ~Scratch() {
    for (void *x : p) (void)DevFree(x);
  }
};

inline unsigned Blocks(uint64_t n) { return static_cast<unsigned>((n + 255) / 256); }

// ---- The merge loop's pair-frequency refresh (UpdateActiveSymbols,
// bpe_model_trainer.cc:153-183: ComputeFreq :87-113 of every bigram whose
// freq was reset), on device-resident state.
//
// State: the sentences' symbol ids (flat, -1 = merged away), the sentence
// freqs, and every bigram's position set as one array of (symbol, EncodePos)
// entries sorted by (symbol, position) with an alive flag (an erased position
// is a dead entry, which is exactly "not in the set").  The host merge loop
// logs its changes (symbol writes, inserted and erased positions) and hands
// them over at each refresh; the refresh returns the recomputed freqs and the
// positions ComputeFreq erased, which the host removes from its own sets.

struct RefreshEntry {  // sort key (sym, key)
  uint32_t sym;
  uint64_t key;
};

__device__ __forceinline__ bool EntryLess(uint32_t as, uint64_t ak, uint32_t bs, uint64_t bk) {
  return as < bs || (as == bs && ak < bk);
}

// First index in [0, n) whose entry is not less than (s, k) (upper = false),
// or greater than (s, k) (upper = true).
__device__ uint64_t EntryBound(const uint32_t *sym, const uint64_t *key, uint64_t n, uint32_t s, uint64_t k,
                               bool upper) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    const bool go_right = upper ? !EntryLess(s, k, sym[mid], key[mid]) : EntryLess(sym[mid], key[mid], s, k);
    if (go_right) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// One write per position (the host keeps the last of each interval).
__global__ void refresh_write_kernel(int32_t *syms, const uint64_t *writes, uint64_t n) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t w = writes[i];
  syms[w >> 32] = static_cast<int32_t>(static_cast<uint32_t>(w));
}

// Erasures the host made since the last refresh: every entry equal to one
// becomes dead (the position is no longer in the set).
__global__ void refresh_erase_kernel(const uint32_t *a_sym, const uint64_t *a_key, uint8_t *a_alive, uint64_t na,
                                     const uint32_t *d_sym, const uint64_t *d_key, uint64_t nd) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= nd) return;
  const uint32_t s = d_sym[i];
  const uint64_t k = d_key[i];
  for (uint64_t j = EntryBound(a_sym, a_key, na, s, k, false); j < na && a_sym[j] == s && a_key[j] == k; ++j)
    a_alive[j] = 0;
}

// Merge of the sorted inserts b into the sorted entries a (a's equal entries
// first): a's entry i lands at i + #(b < a[i]), b's entry j at j + #(a <= b[j]).
__global__ void refresh_merge_a_kernel(const uint32_t *a_sym, const uint64_t *a_key, const uint8_t *a_alive,
                                       uint64_t na, const uint32_t *b_sym, const uint64_t *b_key, uint64_t nb,
                                       uint32_t *o_sym, uint64_t *o_key, uint8_t *o_alive) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= na) return;
  const uint64_t d = i + EntryBound(b_sym, b_key, nb, a_sym[i], a_key[i], false);
  o_sym[d] = a_sym[i];
  o_key[d] = a_key[i];
  o_alive[d] = a_alive[i];
}

__global__ void refresh_merge_b_kernel(const uint32_t *a_sym, const uint64_t *a_key, uint64_t na,
                                       const uint32_t *b_sym, const uint64_t *b_key, uint64_t nb, uint32_t *o_sym,
                                       uint64_t *o_key, uint8_t *o_alive) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= nb) return;
  const uint64_t d = j + EntryBound(a_sym, a_key, na, b_sym[j], b_key[j], true);
  o_sym[d] = b_sym[j];
  o_key[d] = b_key[j];
  o_alive[d] = 1;
}

// ComputeFreq of one symbol per wave over its alive entries in position
// order.  The reference erases a position when it no longer holds (left,
// right), or when it starts where the previous KEPT position of the same
// sentence ended (the second of two overlapping (a, a) pairs), and resets
// that chain after an erased one:
//   kept_j = valid_j && !(kept_p && link_j)   (p = the previous alive entry)
// so kept alternates along a chain of valid, linked entries and restarts
// (kept) at every valid entry that is not linked to a valid predecessor.  A
// wave takes 64 entries at a time: ballots give each lane its chain start
// (or the carried state of the previous chunk) and its parity.
__global__ __launch_bounds__(256) void refresh_freq_kernel(
    const uint32_t *a_sym, const uint64_t *a_key, uint8_t *a_alive, uint64_t na, const int32_t *syms,
    const uint64_t *sent_off, const int64_t *sent_freq, const uint32_t *todo, uint64_t ntodo, uint64_t *out_freq,
    uint32_t *er_sym, uint64_t *er_key, unsigned long long *er_count) {
  const int lane = threadIdx.x & 63;
  const uint64_t w = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  if (w >= ntodo) return;
  const uint32_t s = todo[3 * w], left = todo[3 * w + 1], right = todo[3 * w + 2];
  const uint64_t lo = EntryBound(a_sym, a_key, na, s, 0, false);
  const uint64_t hi = EntryBound(a_sym, a_key, na, s, ~0ull, true);
  uint64_t freq = 0;
  bool c_has = false, c_valid = false, c_kept = false;  // carried: the previous alive entry
  uint64_t c_sid = 0, c_r = 0;
  for (uint64_t base = lo; base < hi; base += 64) {
    const uint64_t j = base + static_cast<uint64_t>(lane);
    const bool alive = j < hi && a_alive[j] != 0;
    const uint64_t key = alive ? a_key[j] : 0;
    const uint64_t sid = key >> 32, l = (key >> 16) & 0xFFFFu, r = key & 0xFFFFu;
    bool valid = false;
    if (alive) {
      const uint64_t b = sent_off[sid];
      valid = syms[b + l] == static_cast<int32_t>(left) && syms[b + r] == static_cast<int32_t>(right);
    }
    const uint64_t am = __builtin_amdgcn_ballot_w64(alive);
    const uint64_t below = am & ((1ull << lane) - 1);
    // The previous alive entry: in this chunk, or the carried one.
    const int p = below ? 63 - __builtin_clzll(below) : 0;
    const uint64_t p_sid = __shfl(sid, p), p_r = __shfl(r, p);
    const bool p_valid = __shfl(static_cast<int>(valid), p) != 0;
    const bool has_p = below ? true : c_has;
    const uint64_t q_sid = below ? p_sid : c_sid, q_r = below ? p_r : c_r;
    const bool q_valid = below ? p_valid : c_valid;
    const bool cont = alive && valid && has_p && q_valid && q_sid == sid && q_r == l;
    // Chain starts: alive entries that do not continue a chain.
    const uint64_t sm = __builtin_amdgcn_ballot_w64(alive && !cont);
    const uint64_t upto = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1);
    const uint64_t st = sm & upto;
    bool kept;
    if (st) {
      // kept at the start (when valid), then alternating over alive entries.
      const int s0 = 63 - __builtin_clzll(st);
      const uint64_t span = am & upto & ~((1ull << s0) - 1);  // alive entries s0..lane
      kept = valid && ((__popcll(span) - 1) & 1) == 0;
    } else {
      kept = valid && (c_kept ^ ((__popcll(am & upto) & 1) != 0));
    }
    if (kept) freq += static_cast<uint64_t>(sent_freq[sid]);
    const bool erase = alive && !kept;
    const uint64_t em = __builtin_amdgcn_ballot_w64(erase);
    if (em) {
      unsigned long long b0 = 0;
      if (lane == 0) b0 = atomicAdd(er_count, static_cast<unsigned long long>(__popcll(em)));
      b0 = __shfl(b0, 0);
      if (erase) {
        const uint64_t o = b0 + __popcll(em & ((1ull << lane) - 1));
        er_sym[o] = s;
        er_key[o] = key;
        a_alive[j] = 0;
      }
    }
    if (am) {  // carry the last alive entry of the chunk
      const int t = 63 - __builtin_clzll(am);
      c_has = true;
      c_sid = __shfl(sid, t);
      c_r = __shfl(r, t);
      c_valid = __shfl(static_cast<int>(valid), t) != 0;
      c_kept = __shfl(static_cast<int>(kept), t) != 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) freq += __shfl_xor(freq, o);
  if (lane == 0) out_freq[w] = freq;
}

}  // namespace
}  // namespace spm_amd

struct spm_hip_bpe_refresh {
  hipStream_t st = nullptr;
  uint64_t nchars = 0, nsent = 0;
  int32_t *syms = nullptr;
  uint64_t *sent_off = nullptr;
  int64_t *sent_freq = nullptr;
  // entries (double-buffered for the merge)
  uint32_t *a_sym[2] = {nullptr, nullptr};
  uint64_t *a_key[2] = {nullptr, nullptr};
  uint8_t *a_alive[2] = {nullptr, nullptr};
  uint64_t na = 0, cap = 0;
  int cur = 0;
  // per-call inputs / outputs
  uint8_t *in = nullptr;   // device staging of the call's inputs
  uint64_t in_cap = 0;
  uint8_t *pin = nullptr;  // pinned host staging (inputs up, outputs down)
  uint64_t pin_cap = 0;
  uint64_t *out_freq = nullptr;
  uint32_t *er_sym = nullptr;
  uint64_t *er_key = nullptr;
  unsigned long long *er_count = nullptr;
  uint64_t out_cap = 0, er_cap = 0;
  std::vector<uint32_t> h_er_sym;
  std::vector<uint64_t> h_er_key;
  std::vector<uint64_t> h_freq;
  float device_ms = 0.f;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  ~spm_hip_bpe_refresh() {
    for (void *p : {static_cast<void *>(syms), static_cast<void *>(sent_off), static_cast<void *>(sent_freq),
                    static_cast<void *>(a_sym[0]), static_cast<void *>(a_sym[1]), static_cast<void *>(a_key[0]),
                    static_cast<void *>(a_key[1]), static_cast<void *>(a_alive[0]), static_cast<void *>(a_alive[1]),
                    static_cast<void *>(in), static_cast<void *>(out_freq), static_cast<void *>(er_sym),
                    static_cast<void *>(er_key), static_cast<void *>(er_count)})
      if (p) (void)spm_amd::DevFree(p);
    if (pin) (void)hipHostFree(pin);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }
};

extern "C" {

int spm_hip_bpe_pair_census(const uint8_t *d_bytes, const uint64_t *d_off, const int64_t *d_freq,
                            uint64_t n, spm_hip_bpe_census **out, void *stream) {
  using namespace spm_amd;
  if (!out || (n && (!d_bytes || !d_off || !d_freq))) return SPM_INVALID_ARGUMENT;
  *out = nullptr;
  if (n >= (1ull << 31)) return SPM_OUT_OF_RANGE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto res = std::make_unique<spm_hip_bpe_census>();
  res->char_off.assign(n + 1, 0);
  res->pos_off.assign(1, 0);
  if (n == 0) {
    *out = res.release();
    return SPM_OK;
  }
  hipEvent_t e0, e1;
  C_TRY(hipEventCreate(&e0));
  C_TRY(hipEventCreate(&e1));
  C_TRY(hipEventRecord(e0, st));
  Scratch sc;
  hipError_t err = hipSuccess;
  uint64_t *cnt = sc.Get<uint64_t>(n, &err);
  uint64_t *coff = sc.Get<uint64_t>(n + 1, &err);
  uint32_t *flag = sc.Get<uint32_t>(1, &err);
  if (err != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
  C_TRY(hipMemsetAsync(flag, 0, 4, st));
  hipLaunchKernelGGL(census_count_kernel, dim3(Blocks(n)), dim3(256), 0, st, d_bytes, d_off, n, cnt, flag);
  C_TRY(hipGetLastError());
  size_t tb = 0;
  C_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tb, cnt, coff + 1, static_cast<int>(n), st));
  void *tmp = sc.Get<uint8_t>(tb, &err);
  if (err != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
  C_TRY(hipMemsetAsync(coff, 0, 8, st));
  C_TRY(hipcub::DeviceScan::InclusiveSum(tmp, tb, cnt, coff + 1, static_cast<int>(n), st));
  uint32_t too_long = 0;
  C_TRY(hipMemcpyAsync(res->char_off.data(), coff, (n + 1) * 8, hipMemcpyDeviceToHost, st));
  C_TRY(hipMemcpyAsync(&too_long, flag, 4, hipMemcpyDeviceToHost, st));
  C_TRY(hipStreamSynchronize(st));
  if (too_long) {
    g_census_error = "a sentence has more than 65536 chars (EncodePos limit)";
    return SPM_OUT_OF_RANGE;
  }
  const uint64_t total = res->char_off[n];
  uint64_t nonempty = 0;
  for (uint64_t i = 0; i < n; ++i) nonempty += res->char_off[i + 1] > res->char_off[i];
  const uint64_t m = total - nonempty;  // pair records
  if (m >= (1ull << 31) || total >= (1ull << 32)) return SPM_OUT_OF_RANGE;
  uint32_t *codes = sc.Get<uint32_t>(total, &err);
  uint32_t *runs = sc.Get<uint32_t>(total, &err);
  uint64_t *rkey = sc.Get<uint64_t>(m, &err), *rpos = sc.Get<uint64_t>(m, &err);
  uint64_t *skey = sc.Get<uint64_t>(m, &err), *spos = sc.Get<uint64_t>(m, &err);
  uint64_t *d_roff = sc.Get<uint64_t>(n + 1, &err);
  if (err != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
  std::vector<uint64_t> roff(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t c = res->char_off[i + 1] - res->char_off[i];
    roff[i + 1] = roff[i] + (c ? c - 1 : 0);
  }
  C_TRY(hipMemcpyAsync(d_roff, roff.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(census_decode_kernel, dim3(Blocks(n)), dim3(256), 0, st, d_bytes, d_off, n, coff, d_roff,
                     codes, runs, rkey, rpos);
  C_TRY(hipGetLastError());
  res->char_codes.resize(total);
  C_TRY(hipMemcpyAsync(res->char_codes.data(), codes, total * 4, hipMemcpyDeviceToHost, st));
  // Unique chars in first-occurrence order: sort (code, index) by code.
  {
    uint32_t *ckey2 = sc.Get<uint32_t>(total, &err);
    uint32_t *idx = sc.Get<uint32_t>(total, &err), *idx2 = sc.Get<uint32_t>(total, &err);
    if (err != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
    std::vector<uint32_t> iota(total);
    for (uint64_t k = 0; k < total; ++k) iota[k] = static_cast<uint32_t>(k);
    C_TRY(hipMemcpyAsync(idx, iota.data(), total * 4, hipMemcpyHostToDevice, st));
    tb = 0;
    C_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, codes, ckey2, idx, idx2, static_cast<int>(total), 0, 21,
                                             st));
    void *t2 = sc.Get<uint8_t>(tb, &err);
    if (err != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
    C_TRY(hipcub::DeviceRadixSort::SortPairs(t2, tb, codes, ckey2, idx, idx2, static_cast<int>(total), 0, 21, st));
    std::vector<uint32_t> hk(total), hi(total);
    C_TRY(hipMemcpyAsync(hk.data(), ckey2, total * 4, hipMemcpyDeviceToHost, st));
    C_TRY(hipMemcpyAsync(hi.data(), idx2, total * 4, hipMemcpyDeviceToHost, st));
    C_TRY(hipStreamSynchronize(st));
    std::vector<std::pair<uint32_t, uint32_t>> first;  // (first index, code)
    for (uint64_t k = 0; k < total; ++k)
      if (k == 0 || hk[k] != hk[k - 1]) first.emplace_back(hi[k], hk[k]);
    std::sort(first.begin(), first.end());
    for (auto &f : first) res->uchars.push_back(f.second);
  }
  if (m > 0) {
    tb = 0;
    C_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, rkey, skey, rpos, spos, static_cast<int>(m), 0, 42, st));
    void *t3 = sc.Get<uint8_t>(tb, &err);
    uint32_t *head = sc.Get<uint32_t>(m, &err), *kept = sc.Get<uint32_t>(m, &err);
    uint64_t *kfreq = sc.Get<uint64_t>(m, &err), *fincl = sc.Get<uint64_t>(m, &err);
    uint64_t *kincl = sc.Get<uint64_t>(m, &err), *kpos = sc.Get<uint64_t>(m, &err);
    uint32_t *sbeg = sc.Get<uint32_t>(m, &err);
    uint64_t *nsel = sc.Get<uint64_t>(2, &err);
    if (err != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
    C_TRY(hipcub::DeviceRadixSort::SortPairs(t3, tb, rkey, skey, rpos, spos, static_cast<int>(m), 0, 42, st));
    hipLaunchKernelGGL(census_flag_kernel, dim3(Blocks(m)), dim3(256), 0, st, skey, spos, m, coff, runs, d_freq,
                       head, kept, kfreq);
    C_TRY(hipGetLastError());
    // freq and kept-count inclusive scans; segment heads and kept positions
    // compacted.
    hipcub::CountingInputIterator<uint32_t> count_it(0);
    hipcub::TransformInputIterator<uint64_t, ToU64, const uint32_t *> kept64(kept, ToU64());
    size_t t_a = 0, t_b = 0, t_c = 0, t_d = 0;
    C_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, t_a, kfreq, fincl, static_cast<int>(m), st));
    C_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, t_b, kept64, kincl, static_cast<int>(m), st));
    C_TRY(hipcub::DeviceSelect::Flagged(nullptr, t_c, count_it, head, sbeg, nsel, static_cast<int>(m), st));
    C_TRY(hipcub::DeviceSelect::Flagged(nullptr, t_d, spos, kept, kpos, nsel + 1, static_cast<int>(m), st));
    void *t4 = sc.Get<uint8_t>(std::max(std::max(t_a, t_b), std::max(t_c, t_d)), &err);
    if (err != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
    C_TRY(hipcub::DeviceScan::InclusiveSum(t4, t_a, kfreq, fincl, static_cast<int>(m), st));
    C_TRY(hipcub::DeviceScan::InclusiveSum(t4, t_b, kept64, kincl, static_cast<int>(m), st));
    C_TRY(hipcub::DeviceSelect::Flagged(t4, t_c, count_it, head, sbeg, nsel, static_cast<int>(m), st));
    C_TRY(hipcub::DeviceSelect::Flagged(t4, t_d, spos, kept, kpos, nsel + 1, static_cast<int>(m), st));
    uint64_t counts[2] = {0, 0};
    C_TRY(hipMemcpyAsync(counts, nsel, 16, hipMemcpyDeviceToHost, st));
    C_TRY(hipStreamSynchronize(st));
    const uint64_t nseg = counts[0], nkept = counts[1];
    uint64_t *s_key = sc.Get<uint64_t>(nseg, &err), *s_first = sc.Get<uint64_t>(nseg, &err);
    uint64_t *s_freq = sc.Get<uint64_t>(nseg, &err), *s_lo = sc.Get<uint64_t>(nseg, &err);
    uint64_t *s_hi = sc.Get<uint64_t>(nseg, &err);
    if (err != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
    hipLaunchKernelGGL(census_segment_kernel, dim3(Blocks(nseg)), dim3(256), 0, st, sbeg, nseg, m, skey, spos,
                       fincl, kincl, s_key, s_first, s_freq, s_lo, s_hi);
    C_TRY(hipGetLastError());
    std::vector<uint64_t> hkey(nseg), hfirst(nseg), hfreq(nseg), hlo(nseg), hhi(nseg), hkpos(nkept);
    C_TRY(hipMemcpyAsync(hkey.data(), s_key, nseg * 8, hipMemcpyDeviceToHost, st));
    C_TRY(hipMemcpyAsync(hfirst.data(), s_first, nseg * 8, hipMemcpyDeviceToHost, st));
    C_TRY(hipMemcpyAsync(hfreq.data(), s_freq, nseg * 8, hipMemcpyDeviceToHost, st));
    C_TRY(hipMemcpyAsync(hlo.data(), s_lo, nseg * 8, hipMemcpyDeviceToHost, st));
    C_TRY(hipMemcpyAsync(hhi.data(), s_hi, nseg * 8, hipMemcpyDeviceToHost, st));
    C_TRY(hipMemcpyAsync(hkpos.data(), kpos, nkept * 8, hipMemcpyDeviceToHost, st));
    C_TRY(hipStreamSynchronize(st));
    // Unique pairs in first-occurrence order (the reference's creation order).
    std::vector<uint64_t> order(nseg);
    for (uint64_t k = 0; k < nseg; ++k) order[k] = k;
    std::sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return hfirst[a] < hfirst[b]; });
    res->pair_keys.reserve(nseg);
    res->pair_freq.reserve(nseg);
    res->pos_off.reserve(nseg + 1);
    res->positions.reserve(nkept);
    for (uint64_t k : order) {
      res->positions.insert(res->positions.end(), hkpos.begin() + hlo[k], hkpos.begin() + hhi[k]);
      res->pair_keys.push_back(hkey[k]);
      res->pair_freq.push_back(hfreq[k]);
      res->pos_off.push_back(res->positions.size());
    }
  }
  C_TRY(hipEventRecord(e1, st));
  C_TRY(hipEventSynchronize(e1));
  (void)hipEventElapsedTime(&res->device_ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *out = res.release();
  return SPM_OK;
}

void spm_hip_bpe_census_free(spm_hip_bpe_census *c) { delete c; }

int spm_hip_bpe_census_view(const spm_hip_bpe_census *c, const uint32_t **char_codes,
                            const uint64_t **char_offsets, const uint32_t **unique_chars,
                            uint64_t *num_unique_chars, const uint64_t **pair_keys,
                            const uint64_t **pair_freq, const uint64_t **pair_pos_offsets,
                            const uint64_t **pair_positions, uint64_t *num_pairs, float *device_ms) {
  if (!c) return SPM_INVALID_ARGUMENT;
  if (char_codes) *char_codes = c->char_codes.data();
  if (char_offsets) *char_offsets = c->char_off.data();
  if (unique_chars) *unique_chars = c->uchars.data();
  if (num_unique_chars) *num_unique_chars = c->uchars.size();
  if (pair_keys) *pair_keys = c->pair_keys.data();
  if (pair_freq) *pair_freq = c->pair_freq.data();
  if (pair_pos_offsets) *pair_pos_offsets = c->pos_off.data();
  if (pair_positions) *pair_positions = c->positions.data();
  if (num_pairs) *num_pairs = c->pair_keys.size();
  if (device_ms) *device_ms = c->device_ms;
  return SPM_OK;
}
const char *spm_hip_bpe_census_last_error(void) { return spm_amd::g_census_error.c_str(); }

int spm_hip_bpe_refresh_create(const int32_t *syms, const uint64_t *sent_offsets, const int64_t *sent_freq,
                               uint64_t num_sentences, const uint32_t *pos_sym, const uint64_t *pos_key,
                               uint64_t num_positions, void *stream, spm_hip_bpe_refresh **out) {
  using namespace spm_amd;
  if (!out || !sent_offsets || (num_sentences && !sent_freq) || (num_positions && (!pos_sym || !pos_key)))
    return SPM_INVALID_ARGUMENT;
  *out = nullptr;
  auto r = std::make_unique<spm_hip_bpe_refresh>();
  r->st = static_cast<hipStream_t>(stream);
  r->nsent = num_sentences;
  r->nchars = sent_offsets[num_sentences];
  if (r->nchars && !syms) return SPM_INVALID_ARGUMENT;
  for (uint64_t k = 1; k < num_positions; ++k)
    if (pos_sym[k] < pos_sym[k - 1] || (pos_sym[k] == pos_sym[k - 1] && pos_key[k] < pos_key[k - 1])) {
      g_census_error = "bpe refresh: positions are not sorted by (symbol, position)";
      return SPM_INVALID_ARGUMENT;
    }
  r->cap = std::max<uint64_t>(num_positions * 2, 1 << 16);
  if (DevMalloc(&r->syms, std::max<uint64_t>(r->nchars, 1) * 4) != hipSuccess ||
      DevMalloc(&r->sent_off, (num_sentences + 1) * 8) != hipSuccess ||
      DevMalloc(&r->sent_freq, std::max<uint64_t>(num_sentences, 1) * 8) != hipSuccess ||
      DevMalloc(&r->er_count, 8) != hipSuccess)
    return SPM_RESOURCE_EXHAUSTED;
  for (int b = 0; b < 2; ++b)
    if (DevMalloc(&r->a_sym[b], r->cap * 4) != hipSuccess || DevMalloc(&r->a_key[b], r->cap * 8) != hipSuccess ||
        DevMalloc(&r->a_alive[b], r->cap) != hipSuccess)
      return SPM_RESOURCE_EXHAUSTED;
  hipStream_t st = r->st;
  C_TRY(hipEventCreate(&r->e0));
  C_TRY(hipEventCreate(&r->e1));
  if (r->nchars) C_TRY(hipMemcpyAsync(r->syms, syms, r->nchars * 4, hipMemcpyHostToDevice, st));
  C_TRY(hipMemcpyAsync(r->sent_off, sent_offsets, (num_sentences + 1) * 8, hipMemcpyHostToDevice, st));
  if (num_sentences) C_TRY(hipMemcpyAsync(r->sent_freq, sent_freq, num_sentences * 8, hipMemcpyHostToDevice, st));
  if (num_positions) {
    C_TRY(hipMemcpyAsync(r->a_sym[0], pos_sym, num_positions * 4, hipMemcpyHostToDevice, st));
    C_TRY(hipMemcpyAsync(r->a_key[0], pos_key, num_positions * 8, hipMemcpyHostToDevice, st));
    C_TRY(hipMemsetAsync(r->a_alive[0], 1, num_positions, st));
  }
  C_TRY(hipStreamSynchronize(st));
  r->na = num_positions;
  *out = r.release();
  return SPM_OK;
}

void spm_hip_bpe_refresh_free(spm_hip_bpe_refresh *r) { delete r; }

int spm_hip_bpe_refresh_run(spm_hip_bpe_refresh *r, const uint64_t *sym_writes, uint64_t num_writes,
                            const uint32_t *ins_sym, const uint64_t *ins_key, uint64_t num_inserts,
                            const uint32_t *del_sym, const uint64_t *del_key, uint64_t num_erases,
                            const uint32_t *todo, uint64_t num_todo, uint64_t *freq_out,
                            const uint32_t **erased_sym, const uint64_t **erased_key, uint64_t *num_erased) {
  using namespace spm_amd;
  if (!r || (num_writes && !sym_writes) || (num_inserts && (!ins_sym || !ins_key)) ||
      (num_erases && (!del_sym || !del_key)) || (num_todo && (!todo || !freq_out)) || !erased_sym ||
      !erased_key || !num_erased)
    return SPM_INVALID_ARGUMENT;
  hipStream_t st = r->st;
  C_TRY(hipEventRecord(r->e0, st));
  // One upload of the call's inputs through pinned staging:
  // [writes | ins_key | del_key | ins_sym | del_sym | todo].
  const uint64_t o_ik = num_writes * 8, o_dk = o_ik + num_inserts * 8, o_is = o_dk + num_erases * 8;
  const uint64_t o_ds = o_is + num_inserts * 4, o_td = o_ds + num_erases * 4, in_bytes = o_td + num_todo * 12;
  if (in_bytes > r->in_cap) {
    if (r->in) (void)DevFree(r->in);
    r->in = nullptr;
    r->in_cap = std::max<uint64_t>(in_bytes * 2, 1 << 20);
    if (DevMalloc(&r->in, r->in_cap) != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
  }
  const uint64_t pin_bytes = std::max<uint64_t>(in_bytes, num_todo * 8 + 8);
  if (pin_bytes > r->pin_cap) {
    if (r->pin) (void)hipHostFree(r->pin);
    r->pin = nullptr;
    r->pin_cap = std::max<uint64_t>(pin_bytes * 2, 1 << 20);
    C_TRY(hipHostMalloc(reinterpret_cast<void **>(&r->pin), r->pin_cap, hipHostMallocDefault));
  }
  uint8_t *h = r->pin;
  if (num_writes) std::memcpy(h, sym_writes, num_writes * 8);
  if (num_inserts) {
    std::memcpy(h + o_ik, ins_key, num_inserts * 8);
    std::memcpy(h + o_is, ins_sym, num_inserts * 4);
  }
  if (num_erases) {
    std::memcpy(h + o_dk, del_key, num_erases * 8);
    std::memcpy(h + o_ds, del_sym, num_erases * 4);
  }
  if (num_todo) std::memcpy(h + o_td, todo, num_todo * 12);
  if (in_bytes) C_TRY(hipMemcpyAsync(r->in, h, in_bytes, hipMemcpyHostToDevice, st));
  const uint64_t *d_writes = reinterpret_cast<const uint64_t *>(r->in);
  const uint64_t *d_ik = reinterpret_cast<const uint64_t *>(r->in + o_ik);
  const uint64_t *d_dk = reinterpret_cast<const uint64_t *>(r->in + o_dk);
  const uint32_t *d_is = reinterpret_cast<const uint32_t *>(r->in + o_is);
  const uint32_t *d_ds = reinterpret_cast<const uint32_t *>(r->in + o_ds);
  const uint32_t *d_todo = reinterpret_cast<const uint32_t *>(r->in + o_td);
  if (num_writes) {
    hipLaunchKernelGGL(refresh_write_kernel, dim3(Blocks(num_writes)), dim3(256), 0, st, r->syms, d_writes,
                       num_writes);
    C_TRY(hipGetLastError());
  }
  int c = r->cur;
  if (num_erases && r->na) {
    hipLaunchKernelGGL(refresh_erase_kernel, dim3(Blocks(num_erases)), dim3(256), 0, st, r->a_sym[c], r->a_key[c],
                       r->a_alive[c], r->na, d_ds, d_dk, num_erases);
    C_TRY(hipGetLastError());
  }
  if (num_inserts) {
    const uint64_t need = r->na + num_inserts;
    if (need > r->cap) {  // grow both buffers (the current one keeps its entries)
      const uint64_t ncap = need * 2;
      for (int b = 0; b < 2; ++b) {
        uint32_t *ns = nullptr;
        uint64_t *nk = nullptr;
        uint8_t *nl = nullptr;
        if (DevMalloc(&ns, ncap * 4) != hipSuccess || DevMalloc(&nk, ncap * 8) != hipSuccess ||
            DevMalloc(&nl, ncap) != hipSuccess)
          return SPM_RESOURCE_EXHAUSTED;
        if (b == c && r->na) {
          C_TRY(hipMemcpyAsync(ns, r->a_sym[b], r->na * 4, hipMemcpyDeviceToDevice, st));
          C_TRY(hipMemcpyAsync(nk, r->a_key[b], r->na * 8, hipMemcpyDeviceToDevice, st));
          C_TRY(hipMemcpyAsync(nl, r->a_alive[b], r->na, hipMemcpyDeviceToDevice, st));
        }
        C_TRY(hipStreamSynchronize(st));
        (void)DevFree(r->a_sym[b]);
        (void)DevFree(r->a_key[b]);
        (void)DevFree(r->a_alive[b]);
        r->a_sym[b] = ns;
        r->a_key[b] = nk;
        r->a_alive[b] = nl;
      }
      r->cap = ncap;
    }
    const int o = 1 - c;
    if (r->na) {
      hipLaunchKernelGGL(refresh_merge_a_kernel, dim3(Blocks(r->na)), dim3(256), 0, st, r->a_sym[c], r->a_key[c],
                         r->a_alive[c], r->na, d_is, d_ik, num_inserts, r->a_sym[o], r->a_key[o], r->a_alive[o]);
      C_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(refresh_merge_b_kernel, dim3(Blocks(num_inserts)), dim3(256), 0, st, r->a_sym[c],
                       r->a_key[c], r->na, d_is, d_ik, num_inserts, r->a_sym[o], r->a_key[o], r->a_alive[o]);
    C_TRY(hipGetLastError());
    r->na += num_inserts;
    r->cur = c = o;
  }
  *num_erased = 0;
  if (num_todo) {
    if (num_todo > r->out_cap) {
      if (r->out_freq) (void)DevFree(r->out_freq);
      r->out_freq = nullptr;
      r->out_cap = num_todo * 2;
      if (DevMalloc(&r->out_freq, r->out_cap * 8) != hipSuccess) return SPM_RESOURCE_EXHAUSTED;
    }
    if (r->na > r->er_cap) {  // every alive entry could be erased
      if (r->er_sym) (void)DevFree(r->er_sym);
      if (r->er_key) (void)DevFree(r->er_key);
      r->er_sym = nullptr;
      r->er_key = nullptr;
      r->er_cap = r->cap;
      if (DevMalloc(&r->er_sym, r->er_cap * 4) != hipSuccess || DevMalloc(&r->er_key, r->er_cap * 8) != hipSuccess)
        return SPM_RESOURCE_EXHAUSTED;
    }
    C_TRY(hipMemsetAsync(r->er_count, 0, 8, st));
    const uint64_t threads = num_todo * 64;
    hipLaunchKernelGGL(refresh_freq_kernel, dim3(static_cast<unsigned>((threads + 255) / 256)), dim3(256), 0, st,
                       r->a_sym[c], r->a_key[c], r->a_alive[c], r->na, r->syms, r->sent_off, r->sent_freq, d_todo,
                       num_todo, r->out_freq, r->er_sym, r->er_key, r->er_count);
    C_TRY(hipGetLastError());
    C_TRY(hipMemcpyAsync(h, r->out_freq, num_todo * 8, hipMemcpyDeviceToHost, st));
    C_TRY(hipMemcpyAsync(h + num_todo * 8, r->er_count, 8, hipMemcpyDeviceToHost, st));
    C_TRY(hipStreamSynchronize(st));
    std::memcpy(freq_out, h, num_todo * 8);
    uint64_t ne = 0;
    std::memcpy(&ne, h + num_todo * 8, 8);
    r->h_er_sym.resize(ne);
    r->h_er_key.resize(ne);
    if (ne) {
      C_TRY(hipMemcpyAsync(r->h_er_sym.data(), r->er_sym, ne * 4, hipMemcpyDeviceToHost, st));
      C_TRY(hipMemcpyAsync(r->h_er_key.data(), r->er_key, ne * 8, hipMemcpyDeviceToHost, st));
    }
    *num_erased = ne;
  }
  C_TRY(hipEventRecord(r->e1, st));
  C_TRY(hipEventSynchronize(r->e1));
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, r->e0, r->e1);
  r->device_ms += ms;
  *erased_sym = r->h_er_sym.data();
  *erased_key = r->h_er_key.data();
  return SPM_OK;
}

int spm_hip_bpe_refresh_stats(const spm_hip_bpe_refresh *r, uint64_t *num_entries, float *device_ms) {
  if (!r) return SPM_INVALID_ARGUMENT;
  if (num_entries) *num_entries = r->na;
  if (device_ms) *device_ms = r->device_ms;
  return SPM_OK;
}

}  // extern "C"
