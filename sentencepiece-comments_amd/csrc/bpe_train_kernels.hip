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

}  // namespace
}  // namespace spm_amd

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

}  // extern "C"
