// Id epilogue of SentencePieceProcessor::Encode(ids) on the device.
//
// Reference: PopulateSentencePieceText (sentencepiece_processor.cc:488-551)
//   — consecutive UNKNOWN pieces merge into one piece with one id (:525-529),
//     CONTROL pieces pass through (:502-508) and the run flag follows every
//     piece (:540) —
// then ApplyExtraOptions (:945-979) — bos / eos / reverse in option order —
// and Encode(ids) (:319-330) keeps only the ids.
//
// The extra options do not depend on the sentence, so the host folds the
// option list into (pre ids, reversed flag, post ids); every sentence's output
// is  pre · (merged tokens, reversed if flagged) · post.  Two passes, one
// sentence per lane: COUNT (merged tokens + extras) → scan → WRITE.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "epilogue.h"

namespace spm_amd {
namespace {

__device__ __forceinline__ bool Emits(uint8_t type, bool *prev_unk) {
  const bool unk = (type & kPieceUnknown) != 0;
  const bool emit = (type & kPieceControl) != 0 || !(*prev_unk && unk);
  *prev_unk = unk;
  return emit;
}

__global__ __launch_bounds__(256) void epilogue_count_kernel(const int32_t *__restrict__ ids,
                                                             const uint64_t *__restrict__ tok_off,
                                                             uint64_t n, const uint8_t *__restrict__ types,
                                                             int32_t num_types, uint32_t extras,
                                                             uint64_t *__restrict__ count,
                                                             const uint32_t *__restrict__ chain) {
  if (chain && *chain) return;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t b = tok_off[i], e = tok_off[i + 1];
    uint64_t c = 0;
    bool prev_unk = false;
    for (uint64_t k = b; k < e; ++k) {
      const int32_t id = ids[k];
      const uint8_t t = (id >= 0 && id < num_types) ? types[id] : 0;
      c += Emits(t, &prev_unk);
    }
    count[i] = c + extras;
  }
}

__global__ __launch_bounds__(256) void epilogue_write_kernel(const int32_t *__restrict__ ids,
                                                             const uint64_t *__restrict__ tok_off,
                                                             uint64_t n, const uint8_t *__restrict__ types,
                                                             int32_t num_types, EpilogueExtras x,
                                                             const uint64_t *__restrict__ out_off,
                                                             int32_t *__restrict__ out, uint64_t cap_limit,
                                                             uint32_t *__restrict__ chain) {
  if (chain && *chain) return;
  if (out_off[n] > cap_limit) {
    if (chain && blockIdx.x == 0 && threadIdx.x == 0) atomicCAS(chain, 0u, 8u);  // SPM_RESOURCE_EXHAUSTED
    return;
  }
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t b = tok_off[i], e = tok_off[i + 1];
    const uint64_t o0 = out_off[i], o1 = out_off[i + 1];
    for (uint32_t k = 0; k < x.num_pre; ++k) out[o0 + k] = x.ids[k];
    for (uint32_t k = 0; k < x.num_post; ++k) out[o1 - x.num_post + k] = x.ids[kMaxExtras + k];
    // Merged tokens fill [o0 + num_pre, o1 - num_post), forward or reversed.
    const uint64_t m0 = o0 + x.num_pre, m1 = o1 - x.num_post;
    uint64_t j = 0;
    bool prev_unk = false;
    for (uint64_t k = b; k < e; ++k) {
      const int32_t id = ids[k];
      const uint8_t t = (id >= 0 && id < num_types) ? types[id] : 0;
      if (Emits(t, &prev_unk)) {
        out[x.reversed ? m1 - 1 - j : m0 + j] = id;
        ++j;
      }
    }
  }
}

// PopulateSentencePieceText (sentencepiece_processor.cc:488-551) with the
// surfaces as offsets: a non-control piece of normalized bytes [c, c + len)
// gets begin = norm_to_orig[c], end = norm_to_orig[c + len]; an UNKNOWN piece
// after an UNKNOWN piece extends the previous one (piece and surface
// concatenated, end updated, :525-529); a control piece gets begin = end =
// norm_to_orig[c] and does not advance c (:502-508).  Then the folded extra
// options (bos/eos pieces carry zero offsets, :954-972).
__global__ __launch_bounds__(256) void spt_write_kernel(const int32_t *__restrict__ ids,
                                                        const uint32_t *__restrict__ lens,
                                                        const uint64_t *__restrict__ tok_off, uint64_t n,
                                                        const uint8_t *__restrict__ types, int32_t num_types,
                                                        EpilogueExtras x, const uint32_t *__restrict__ n2o,
                                                        const uint64_t *__restrict__ norm_off,
                                                        const uint64_t *__restrict__ out_off,
                                                        spm_hip_piece *__restrict__ out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t b = tok_off[i], e = tok_off[i + 1];
    const uint64_t o0 = out_off[i], o1 = out_off[i + 1];
    const uint32_t *a = n2o + norm_off[i] + i;
    for (uint32_t k = 0; k < x.num_pre; ++k) out[o0 + k] = spm_hip_piece{x.ids[k], 0, 0, 0, 0};
    for (uint32_t k = 0; k < x.num_post; ++k)
      out[o1 - x.num_post + k] = spm_hip_piece{x.ids[kMaxExtras + k], 0, 0, 0, 0};
    const uint64_t m0 = o0 + x.num_pre, m1 = o1 - x.num_post;
    uint64_t j = 0;
    uint32_t c = 0;
    bool prev_unk = false;
    for (uint64_t k = b; k < e; ++k) {
      const int32_t id = ids[k];
      const uint32_t len = lens[k];
      const uint8_t t = (id >= 0 && id < num_types) ? types[id] : 0;
      const bool control = (t & kPieceControl) != 0;
      const bool merge = !control && prev_unk && (t & kPieceUnknown);
      Emits(t, &prev_unk);
      if (control) {
        out[x.reversed ? m1 - 1 - j : m0 + j] = spm_hip_piece{id, a[c], a[c], c, c + len};
        ++j;
      } else if (merge) {
        spm_hip_piece &p = out[x.reversed ? m1 - j : m0 + j - 1];
        p.end = a[c + len];
        p.norm_end = c + len;
        c += len;
      } else {
        out[x.reversed ? m1 - 1 - j : m0 + j] = spm_hip_piece{id, a[c], a[c + len], c, c + len};
        ++j;
        c += len;
      }
    }
  }
}

unsigned Blocks(uint64_t n) {
  const uint64_t b = (n + 255) / 256;
  return static_cast<unsigned>(b < (1u << 20) ? b : (1u << 20));
}

}  // namespace

hipError_t LaunchEpilogueCount(const int32_t *ids, const uint64_t *tok_off, uint64_t n, const uint8_t *types,
                               int32_t num_types, uint32_t extras, uint64_t *count, hipStream_t st,
                               const uint32_t *chain) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(epilogue_count_kernel, dim3(Blocks(n)), dim3(256), 0, st, ids, tok_off, n, types,
                     num_types, extras, count, chain);
  return hipGetLastError();
}

hipError_t LaunchEpilogueWrite(const int32_t *ids, const uint64_t *tok_off, uint64_t n, const uint8_t *types,
                               int32_t num_types, const EpilogueExtras &x, const uint64_t *out_off,
                               int32_t *out, hipStream_t st, uint64_t cap_limit, uint32_t *chain) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(epilogue_write_kernel, dim3(Blocks(n)), dim3(256), 0, st, ids, tok_off, n, types,
                     num_types, x, out_off, out, cap_limit, chain);
  return hipGetLastError();
}

hipError_t LaunchSptWrite(const int32_t *ids, const uint32_t *lens, const uint64_t *tok_off, uint64_t n,
                          const uint8_t *types, int32_t num_types, const EpilogueExtras &x,
                          const uint32_t *n2o, const uint64_t *norm_off, const uint64_t *out_off,
                          spm_hip_piece *out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(spt_write_kernel, dim3(Blocks(n)), dim3(256), 0, st, ids, lens, tok_off, n, types,
                     num_types, x, n2o, norm_off, out_off, out);
  return hipGetLastError();
}

}  // namespace spm_amd
