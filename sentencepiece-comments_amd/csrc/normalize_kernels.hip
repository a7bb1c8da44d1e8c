// Normalizer on gfx950: Normalizer::Normalize (reference normalizer.cc:88-211)
// with NormalizePrefix (:231-300) over the precompiled charsmap (darts-clone
// units + NUL-terminated targets, :305-337), the user-defined PrefixMatcher
// (:339-384) and, for the trainer, PrefixMatcher::GlobalReplace of the meta
// pieces (:391-405, trainer_interface.cc:370-378).
//
// One sentence per lane, two passes over the same state machine: COUNT gives
// each sentence's normalized length (trailing whitespace stripped in closed
// form: the output is valid UTF-8, so the stripped suffix is the run of
// whitespace chars emitted last), a hipCUB scan turns lengths into CSR
// offsets, WRITE emits the bytes.  The charsmap trie (≈230 KB) and its target
// pool stay L2-resident.  WRITE optionally also emits norm_to_orig (the
// input byte offset, relative to the sentence, of the NormalizePrefix chunk
// each output byte came from, plus one final entry: normalizer.cc:132-208),
// len + 1 uint32 entries per sentence at n2o[out_off[i] + i].
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <string>

#include "normalize_device.h"
#include "normalize_prefix.h"

namespace spm_amd {
namespace {

// NormalizePrefix: returns the replacement (pointer, length) and consumed bytes.

// U+FFFD in global memory: a string literal would live in the constant
// address space, and a pointer that may point to either turns every read
// of the chunk into a flat load.
__device__ uint8_t kReplacementChar[4] = {0xEF, 0xBF, 0xBD, 0};  // (not const: const globals go to the constant space too)

__device__ const uint8_t *NormalizePrefix(const NormTables &t, const uint8_t *in, uint64_t n,
                                          uint32_t *rlen, uint32_t *consumed) {
  if (t.ud_units) {
    const uint32_t m = TrieLongest(t.ud_units, t.ud_num_units, in, n);
    if (m) {
      *rlen = *consumed = m;
      return in;
    }
  }
  uint32_t value = 0;
  const uint32_t longest = CharsmapLongest(t, in, n, &value);
  if (longest == 0) {
    const uint32_t len = DValidCharLen(in, n);
    if (len == 0) {
      *rlen = 3;
      *consumed = 1;
      return kReplacementChar;
    }
    *rlen = *consumed = len;
    return in;
  }
  *consumed = longest;
  const uint8_t *r = t.pool + value;
  uint32_t l = 0;
  while (r[l]) ++l;  // ends at the latest at the NUL appended after the blob (EnsureNormTables)
  *rlen = l;
  return r;
}

constexpr uint32_t kNormLds = 24576;  // WRITE: a block's output staged in LDS when it fits

template <bool WRITE>
__global__ __launch_bounds__(256) void normalize_kernel(NormTables t, const uint8_t *in_bytes,
                                                        const uint64_t *in_off, uint64_t n, uint8_t *out,
                                                        const uint64_t *out_off, uint64_t *len_out,
                                                        uint32_t *n2o_base, uint64_t cap_limit, uint32_t *chain) {
  __shared__ uint8_t lds_out[WRITE ? kNormLds : 1];
  // Asynchronous chains: nothing runs once an earlier step failed, and a
  // result larger than the caller's capacity is reported, not written.
  if (chain && *chain) return;
  if (WRITE && out_off[n] > cap_limit) {
    if (chain && blockIdx.x == 0 && threadIdx.x == 0) atomicCAS(chain, 0u, 8u);  // SPM_RESOURCE_EXHAUSTED
    return;
  }
  const uint64_t base = uint64_t(blockIdx.x) * blockDim.x;
  const uint64_t i = base + threadIdx.x;
  // WRITE: the block's sentences are consecutive, so its output is one
  // contiguous range [B0, B1); lanes write their bytes into LDS and the block
  // stores the range with coalesced dword writes (instead of one scattered
  // byte store per output byte per lane).
  uint64_t B0 = 0, B1 = 0;
  bool use_lds = false;
  if (WRITE) {
    B0 = out_off[base];
    B1 = out_off[base + blockDim.x < n ? base + blockDim.x : n];
    use_lds = B1 - B0 <= kNormLds;
  }
  [&]() {
    if (i >= n) return;
    const uint8_t *in = in_bytes + in_off[i];
    uint64_t left = in_off[i + 1] - in_off[i];
    uint8_t *o = WRITE ? out + out_off[i] : nullptr;
    const uint32_t lo = WRITE && use_lds ? static_cast<uint32_t>(out_off[i] - B0) : 0u;
    auto store = [&](uint64_t at, uint8_t v) {
      if (use_lds) lds_out[lo + at] = v;
      else o[at] = v;
    };
    const uint64_t cap = WRITE ? out_off[i + 1] - out_off[i] : 0;
    const bool rew = t.remove_extra_whitespaces, esc = t.escape_whitespaces;
    const uint32_t wsl = esc ? 3u : 1u;
    uint64_t len = 0;      // bytes emitted so far
    uint64_t ws_run = 0;   // trailing whitespace chars emitted last
    uint32_t rlen, rcons;
    // norm_to_orig: `cons` = input bytes consumed before the current
    // NormalizePrefix chunk; ws_cons = that value for the first char of the
    // trailing whitespace run (what the strip loop leaves in `consumed`).
    uint32_t *n2o = WRITE && n2o_base ? n2o_base + out_off[i] + i : nullptr;
    uint32_t cons = 0, ws_cons = 0;
    if (left == 0) {
      if (!WRITE) len_out[i] = 0;
      if (n2o) n2o[0] = 0;  // the reference returns an empty norm_to_orig here
      return;
    }
    if (rew) {
      while (left > 0) {
        const uint8_t *r = NormalizePrefix(t, in, left, &rlen, &rcons);
        if (!(rlen == 1 && r[0] == ' ')) break;
        in += rcons;
        left -= rcons;
        cons += rcons;
      }
    }
    if (left == 0) {
      if (!WRITE) len_out[i] = 0;
      if (n2o) n2o[0] = cons;  // the reference returns an empty norm_to_orig here
      return;
    }
    // In WRITE mode `cap` is the final length: the stripped trailing
    // whitespace and a suffix dummy land beyond it / at its end (see below).
    uint64_t body_cap = cap;
    if (WRITE && t.suffix && t.add_dummy_prefix) body_cap = cap - wsl;
    auto put_body = [&](uint8_t v) {
      if (WRITE && len < body_cap) {
        store(len, v);
        if (n2o) n2o[len] = cons;
      }
      ++len;
    };
    if (!t.suffix && t.add_dummy_prefix) {
      ws_cons = cons;
      if (esc) {
        put_body(0xE2);
        put_body(0x96);
        put_body(0x81);
      } else {
        put_body(' ');
      }
      ws_run = 1;
    }
    bool prev_space = rew;
    while (left > 0) {
      const uint8_t *r = NormalizePrefix(t, in, left, &rlen, &rcons);
      uint32_t k = 0;
      if (prev_space)
        while (k < rlen && r[k] == ' ') ++k;
      if (k < rlen) {
        // emit r[k:rlen) char by char (valid UTF-8), tracking the trailing
        // whitespace run (' ' → escaped, or a literal U+2581 / ' ').
        while (k < rlen) {
          const uint8_t b0 = r[k];
          if (b0 == ' ') {
            if (ws_run == 0) ws_cons = cons;
            if (esc) {
              put_body(0xE2);
              put_body(0x96);
              put_body(0x81);
            } else {
              put_body(' ');
            }
            ++ws_run;
            ++k;
            continue;
          }
          const uint32_t cl = min<uint32_t>((0x4322111111111111ull >> ((b0 >> 4) * 4)) & 0xFu, rlen - k);
          const bool is_ws = esc ? (cl == 3 && b0 == 0xE2 && r[k + 1] == 0x96 && r[k + 2] == 0x81) : false;
          if (is_ws && ws_run == 0) ws_cons = cons;
          for (uint32_t x = 0; x < cl; ++x) put_body(r[k + x]);
          ws_run = is_ws ? ws_run + 1 : 0;
          k += cl;
        }
        prev_space = r[rlen - 1] == ' ';
      }
      in += rcons;
      left -= rcons;
      cons += rcons;
      if (!rew) prev_space = false;
    }
    // strip trailing whitespace (normalizer.cc:191-202); `consumed` becomes
    // norm_to_orig of the first stripped byte.
    if (rew && ws_run > 0) {
      len -= ws_run * wsl;
      cons = ws_cons;
    }
    if (t.suffix && t.add_dummy_prefix) {
      if (WRITE) {
        if (esc) {
          store(len, 0xE2);
          store(len + 1, 0x96);
          store(len + 2, 0x81);
        } else {
          store(len, ' ');
        }
        if (n2o)
          for (uint32_t x = 0; x < wsl; ++x) n2o[len + x] = cons;
      }
      len += wsl;
    }
    if (n2o) n2o[len] = cons;
    if (!WRITE) len_out[i] = len;
  }();
  if (WRITE && use_lds) {
    __syncthreads();
    const uint32_t total = static_cast<uint32_t>(B1 - B0);
    uint8_t *dst = out + B0;
    const uint32_t head = min<uint32_t>(static_cast<uint32_t>((4u - (B0 & 3u)) & 3u), total);
    for (uint32_t k = threadIdx.x; k < head; k += blockDim.x) dst[k] = lds_out[k];
    const uint32_t nd = (total - head) / 4;
    uint32_t *dw = reinterpret_cast<uint32_t *>(dst + head);
    for (uint32_t w = threadIdx.x; w < nd; w += blockDim.x) {
      const uint32_t q = head + 4 * w;
      dw[w] = static_cast<uint32_t>(lds_out[q]) | (static_cast<uint32_t>(lds_out[q + 1]) << 8) |
              (static_cast<uint32_t>(lds_out[q + 2]) << 16) | (static_cast<uint32_t>(lds_out[q + 3]) << 24);
    }
    for (uint32_t k = head + 4 * nd + threadIdx.x; k < total; k += blockDim.x) dst[k] = lds_out[k];
  }
}

// GlobalReplace of the meta pieces by "\t" (trainer).  COUNT: new length and
// a flag when anything matched; WRITE: the replaced bytes.
template <bool WRITE>
__global__ void meta_replace_kernel(const uint32_t *units, uint32_t num_units, const uint8_t *in_bytes,
                                    const uint64_t *in_off, uint64_t n, uint8_t *out,
                                    const uint64_t *out_off, uint64_t *len_out, uint32_t *any) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *s = in_bytes + in_off[i];
  const uint64_t sl = in_off[i + 1] - in_off[i];
  uint8_t *o = WRITE ? out + out_off[i] : nullptr;
  uint64_t p = 0, len = 0;
  bool hit = false;
  while (p < sl) {
    const uint32_t m = TrieLongest(units, num_units, s + p, sl - p);
    if (m) {
      if (WRITE) o[len] = '\t';
      ++len;
      p += m;
      hit = true;
    } else {
      const uint32_t cl =
          min<uint64_t>((0x4322111111111111ull >> ((s[p] >> 4) * 4)) & 0xFu, sl - p);
      if (WRITE)
        for (uint32_t x = 0; x < cl; ++x) o[len + x] = s[p + x];
      len += cl;
      p += cl;
    }
  }
  if (!WRITE) {
    len_out[i] = len;
    if (hit) *any = 1u;
  }
}

inline unsigned Blocks(uint64_t n) { return static_cast<unsigned>((n + 255) / 256); }

}  // namespace

hipError_t NormalizeLengths(const NormTables &t, const uint8_t *d_in, const uint64_t *d_in_off,
                            uint64_t n, uint64_t *d_len, hipStream_t st, uint32_t *chain) {
  if (n == 0) return hipSuccess;
  normalize_kernel<false><<<Blocks(n), 256, 0, st>>>(t, d_in, d_in_off, n, nullptr, nullptr, d_len, nullptr,
                                                     ~0ull, chain);
  return hipGetLastError();
}

hipError_t NormalizeWrite(const NormTables &t, const uint8_t *d_in, const uint64_t *d_in_off,
                          uint64_t n, uint8_t *d_out, const uint64_t *d_out_off, hipStream_t st,
                          uint32_t *d_n2o, uint64_t cap_limit, uint32_t *chain) {
  if (n == 0) return hipSuccess;
  normalize_kernel<true><<<Blocks(n), 256, 0, st>>>(t, d_in, d_in_off, n, d_out, d_out_off, nullptr, d_n2o,
                                                    cap_limit, chain);
  return hipGetLastError();
}

hipError_t MetaReplaceLengths(const uint32_t *units, uint32_t num_units, const uint8_t *d_in,
                              const uint64_t *d_in_off, uint64_t n, uint64_t *d_len, uint32_t *d_any,
                              hipStream_t st) {
  if (n == 0) return hipSuccess;
  meta_replace_kernel<false><<<Blocks(n), 256, 0, st>>>(units, num_units, d_in, d_in_off, n, nullptr,
                                                        nullptr, d_len, d_any);
  return hipGetLastError();
}

hipError_t MetaReplaceWrite(const uint32_t *units, uint32_t num_units, const uint8_t *d_in,
                            const uint64_t *d_in_off, uint64_t n, uint8_t *d_out,
                            const uint64_t *d_out_off, hipStream_t st) {
  if (n == 0) return hipSuccess;
  meta_replace_kernel<true><<<Blocks(n), 256, 0, st>>>(units, num_units, d_in, d_in_off, n, d_out,
                                                       d_out_off, nullptr, nullptr);
  return hipGetLastError();
}

// Exclusive scan of lengths into CSR offsets (off[0] = 0, off[n] = total).
hipError_t LengthsToOffsets(const uint64_t *d_len, uint64_t n, uint64_t *d_off, void *tmp,
                            size_t *tmp_bytes, hipStream_t st) {
  if (!tmp) {
    return hipcub::DeviceScan::InclusiveSum(nullptr, *tmp_bytes, d_len, d_off + 1, n, st);
  }
  hipError_t e = hipMemsetAsync(d_off, 0, sizeof(uint64_t), st);
  if (e != hipSuccess || n == 0) return e;
  return hipcub::DeviceScan::InclusiveSum(tmp, *tmp_bytes, d_len, d_off + 1, n, st);
}

}  // namespace spm_amd
