// Output compaction: per-sentence token slots → dense CSR (see kernels.h).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "kernels.h"

namespace spm_amd {
namespace {

struct ToU64 {
  __host__ __device__ uint64_t operator()(uint32_t x) const { return x; }
};

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
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += stride) {
    if (i == 0) tok_off[0] = 0;
    const uint32_t k = ntok[i];
    const uint32_t l = lo[i];
    const int32_t *sid;
    const uint32_t *slen;
    if (l == 0xFFFFFFFFu) {
      sid = slot2_ids + off[i + 1] - k;
      slen = slot2_len ? slot2_len + off[i + 1] - k : nullptr;
    } else {
      sid = slot_ids + off[i & ~static_cast<uint64_t>(255)] + l;
      slen = slot_len ? slot_len + off[i & ~static_cast<uint64_t>(255)] + l : nullptr;
    }
    const uint64_t dst = tok_off[i + 1] - k;
    for (uint32_t j = 0; j < k; ++j) ids[dst + j] = sid[j];
    if (piece_len)
      for (uint32_t j = 0; j < k; ++j) piece_len[dst + j] = slen[j];
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
  const uint64_t blocks64 = (n + 255) / 256;
  const unsigned blocks = static_cast<unsigned>(blocks64 < (1u << 30) ? blocks64 : (1u << 30));
  hipLaunchKernelGGL(compact_kernel, dim3(blocks), dim3(256), 0, st, off, n, ntok, lo, slot_ids,
                     slot_len, slot2_ids, slot2_len, ids, piece_len, tok_off);
  return hipGetLastError();
}

}  // namespace spm_amd
