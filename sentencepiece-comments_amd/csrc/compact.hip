// Output compaction: per-sentence token slots → dense CSR (see kernels.h).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "kernels.h"

namespace spm_amd {
namespace {

struct ToU64 {
  __host__ __device__ uint64_t operator()(uint32_t x) const { return x; }
};

// One block per group of 256 sentences (the fast kernel's block: its tokens
// sit densely, in sentence order, at slot_ids + off[first sentence]).  A
// group whose sentences all took the fast path is one contiguous range in the
// output too, copied with coalesced loads/stores; a group with a
// general-path sentence (tokens in slot2) is copied per sentence.
__global__ __launch_bounds__(256) void compact_kernel(const uint64_t *__restrict__ off, uint64_t n,
                                                       const uint32_t *__restrict__ ntok,
                                                       const uint32_t *__restrict__ lo,
                                                       const int32_t *__restrict__ slot_ids,
                                                       const uint32_t *__restrict__ slot_len,
                                                       const int32_t *__restrict__ slot2_ids,
                                                       const uint32_t *__restrict__ slot2_len,
                                                       int32_t *__restrict__ ids,
                                                       uint32_t *__restrict__ piece_len,
                                                       uint64_t *__restrict__ tok_off) {
  __shared__ uint32_t any_general;
  const uint64_t ngroups = (n + 255) / 256;
  for (uint64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const uint64_t g0 = g * 256, g1 = g0 + 256 < n ? g0 + 256 : n;
    const uint64_t i = g0 + threadIdx.x;
    if (threadIdx.x == 0) any_general = 0;
    __syncthreads();
    if (i < g1 && lo[i] == 0xFFFFFFFFu) any_general = 1;
    if (i == 0) tok_off[0] = 0;
    __syncthreads();
    if (!any_general) {
      const uint64_t d0 = g0 ? tok_off[g0] : 0, d1 = tok_off[g1];
      const int32_t *src = slot_ids + off[g0];
      const uint32_t *srcl = slot_len ? slot_len + off[g0] : nullptr;
      for (uint64_t k = threadIdx.x; k < d1 - d0; k += 256) {
        ids[d0 + k] = src[k];
        if (piece_len) piece_len[d0 + k] = srcl[k];
      }
    } else if (i < g1) {
      const uint32_t k = ntok[i];
      const uint32_t l = lo[i];
      const int32_t *sid;
      const uint32_t *slen;
      if (l == 0xFFFFFFFFu) {
        sid = slot2_ids + off[i + 1] - k;
        slen = slot2_len ? slot2_len + off[i + 1] - k : nullptr;
      } else {
        sid = slot_ids + off[g0] + l;
        slen = slot_len ? slot_len + off[g0] + l : nullptr;
      }
      const uint64_t dst = tok_off[i + 1] - k;
      for (uint32_t j = 0; j < k; ++j) ids[dst + j] = sid[j];
      if (piece_len)
        for (uint32_t j = 0; j < k; ++j) piece_len[dst + j] = slen[j];
    }
    __syncthreads();
  }
}

}  // namespace

hipError_t LaunchCompact(const uint64_t *off, uint64_t n, const uint32_t *ntok, const uint32_t *lo,
                         const int32_t *slot_ids, const uint32_t *slot_len,
                         const int32_t *slot2_ids, const uint32_t *slot2_len, int32_t *ids,
                         uint32_t *piece_len, uint64_t *tok_off, void *scan_tmp,
                         size_t *scan_tmp_bytes, hipStream_t st) {
  hipcub::TransformInputIterator<uint64_t, ToU64, const uint32_t *> in(ntok, ToU64());
  if (scan_tmp == nullptr) {
    return hipcub::DeviceScan::InclusiveSum(nullptr, *scan_tmp_bytes, in, tok_off + 1,
                                            static_cast<int>(n > 0 ? n : 1), st);
  }
  if (n == 0) {
    return hipMemsetAsync(tok_off, 0, sizeof(uint64_t), st);
  }
  hipError_t e = hipcub::DeviceScan::InclusiveSum(scan_tmp, *scan_tmp_bytes, in, tok_off + 1,
                                                  static_cast<int>(n), st);
  if (e != hipSuccess) return e;
  const uint64_t blocks64 = (n + 255) / 256;  // one block per group of 256 sentences
  const unsigned blocks = static_cast<unsigned>(blocks64 < (1u << 30) ? blocks64 : (1u << 30));
  hipLaunchKernelGGL(compact_kernel, dim3(blocks), dim3(256), 0, st, off, n, ntok, lo, slot_ids,
                     slot_len, slot2_ids, slot2_len, ids, piece_len, tok_off);
  return hipGetLastError();
}

}  // namespace spm_amd
