// Output assembly kernels: right-aligned slots → dense CSR (BPE and
// general-only paths), and the unigram fix-up chain that splices general-path
// sentences into the fast kernel's dense output (see kernels.h).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "kernels.h"
#include "lookback.h"

namespace spm_amd {
namespace {

constexpr uint32_t kStatusOk = 0;                  // SPM_OK
constexpr uint32_t kStatusResourceExhausted = 8;   // SPM_RESOURCE_EXHAUSTED

struct ToU64 {
  __host__ __device__ uint64_t operator()(uint32_t x) const { return x; }
};

__device__ __forceinline__ uint64_t ReadLane64(uint64_t v, uint32_t lane) {
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(lane)));
  const uint32_t hi =
      static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v >> 32), static_cast<int>(lane)));
  return static_cast<uint64_t>(hi) << 32 | lo;
}

// Sentence i's tokens: slot[off[i+1] - k .. off[i+1]) → ids[tok_off[i] ..),
// k = tok_off[i+1] - tok_off[i].  kGuarded: the unigram fix-up (no-op unless
// the fast kernel flagged a sentence); also publishes the call's status.
template <bool kGuarded>
__global__ __launch_bounds__(256) void compact_kernel(const uint64_t *__restrict__ off, uint64_t n,
                                                       const int32_t *__restrict__ slot_ids,
                                                       const uint32_t *__restrict__ slot_len,
                                                       int32_t *__restrict__ ids, uint32_t *__restrict__ piece_len,
                                                       const uint64_t *__restrict__ tok_off,
                                                       const uint32_t *__restrict__ status,
                                                       uint32_t *__restrict__ out_status) {
  if constexpr (kGuarded) {
    // First error wins: the caller zeroes its status word before a chain.
    if (blockIdx.x == 0 && threadIdx.x == 0 && out_status && status[kStError])
      atomicCAS(out_status, kStatusOk, kStatusResourceExhausted);
    if (status[kStFlagged] == 0) return;
  } else {
    if (blockIdx.x == 0 && threadIdx.x == 0 && out_status && status && status[kStError])
      atomicCAS(out_status, kStatusOk, kStatusResourceExhausted);
    if (status && (status[kStError] & 2u)) return;
  }
  // One wave per 64 sentences: the lanes read the 64 sentences' (d0, k,
  // src) together, then the wave copies one sentence at a time with
  // consecutive lanes on consecutive tokens (a lane per sentence copied its
  // run alone: ~100-token runs of real-text lines became strided, partly
  // written lines; 1.26 ms per 1 M Japanese lines, profiles/r06bb trace).
  const int lane = threadIdx.x & 63;
  const uint64_t waves = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
  for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); g * 64 < n;
       g += waves) {
    const uint64_t i = g * 64 + static_cast<uint64_t>(lane);
    uint64_t d0 = 0, k = 0, src = 0;
    if (i < n) {
      d0 = tok_off[i];
      k = tok_off[i + 1] - d0;
      src = off[i + 1] - k;
    }
    const uint32_t m = n - g * 64 < 64 ? static_cast<uint32_t>(n - g * 64) : 64u;
    for (uint32_t s = 0; s < m; ++s) {
      const uint64_t sd0 = ReadLane64(d0, s), sk = ReadLane64(k, s), ssrc = ReadLane64(src, s);
      for (uint64_t j = static_cast<uint64_t>(lane); j < sk; j += 64) ids[sd0 + j] = slot_ids[ssrc + j];
      if (piece_len)
        for (uint64_t j = static_cast<uint64_t>(lane); j < sk; j += 64) piece_len[sd0 + j] = slot_len[ssrc + j];
    }
  }
}

// Fix-up step 1: every fast-path sentence's tokens move from the dense output
// to its right-aligned slot (disjoint per sentence); counts of all sentences
// (flagged ones from the general kernel) go to cnt.
__global__ __launch_bounds__(256) void fixup_gather_kernel(FixupLaunch f) {
  if (f.status[kStFlagged] == 0) return;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < f.n; i += stride) {
    const uint64_t t0 = f.tok_off[i] & ~kTokFlag;
    const uint64_t t1 = f.tok_off[i + 1];
    if (t1 & kTokFlag) {
      f.cnt[i] = f.ntok[i];
      continue;
    }
    const uint32_t k = static_cast<uint32_t>(t1 - t0);
    const uint64_t dst = f.off[i + 1] - k;
    for (uint32_t j = 0; j < k; ++j) f.slot_ids[dst + j] = f.ids[t0 + j];
    if (f.len)
      for (uint32_t j = 0; j < k; ++j) f.slot_len[dst + j] = f.len[t0 + j];
    f.cnt[i] = k;
  }
}

// Fix-up step 2: tok_off[i + 1] = inclusive prefix of cnt.  One contiguous
// chunk per workgroup; chunk offsets by a decoupled look-back.
__global__ __launch_bounds__(256) void fixup_scan_kernel(FixupLaunch f, uint64_t chunk) {
  if (f.status[kStFlagged] == 0) return;
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_w[4];
  __shared__ uint64_t s_carry;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(&f.status[kStScanTicket], 1u);
  __syncthreads();
  const uint64_t tile = s_tile;
  const uint64_t lo = tile * chunk;
  const uint64_t hi = lo + chunk < f.n ? lo + chunk : f.n;
  uint64_t sum = 0;
  for (uint64_t i = lo + tid; i < hi; i += 256) sum += f.cnt[i];
  sum = WaveSum64(sum);
  if (lane == 0) s_w[wave] = sum;
  __syncthreads();
  if (wave == 0) {
    const uint64_t pre = LookbackExclusive(f.scan_desc, tile, s_w[0] + s_w[1] + s_w[2] + s_w[3], lane);
    if (lane == 0) s_carry = pre;
  }
  __syncthreads();
  uint64_t carry = s_carry;
  for (uint64_t r = lo; r < hi; r += 256) {
    const uint64_t i = r + tid;
    const uint64_t v = i < hi ? f.cnt[i] : 0;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t ylo = __shfl_up(static_cast<uint32_t>(x), o);
      const uint32_t yhi = __shfl_up(static_cast<uint32_t>(x >> 32), o);
      if (lane >= o) x += (static_cast<uint64_t>(yhi) << 32) | ylo;
    }
    __syncthreads();  // s_w of the previous round consumed
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    uint64_t wpre = 0;
    for (int w = 0; w < wave; ++w) wpre += s_w[w];
    if (i < hi) f.tok_off[i + 1] = carry + wpre + x;
    carry += s_w[0] + s_w[1] + s_w[2] + s_w[3];
  }
}

// One tile per block: its dense slot range moves to its final offset.
__global__ __launch_bounds__(256) void tile_compact_kernel(const uint64_t *__restrict__ off, uint64_t n,
                                                           const uint64_t *__restrict__ prefix,
                                                           const int32_t *__restrict__ slot_ids,
                                                           const uint32_t *__restrict__ slot_len,
                                                           int32_t *__restrict__ ids, uint32_t *__restrict__ len,
                                                           uint64_t *__restrict__ tok_off,
                                                           const uint32_t *__restrict__ status) {
  if (status[kStError] & 2u) return;  // the fast kernel did not run
  const uint64_t t = blockIdx.x, base = t * 256;
  const uint64_t p0 = prefix[t], cnt = prefix[t + 1] - p0, src = off[base];
  for (uint64_t k = threadIdx.x; k < cnt; k += 256) ids[p0 + k] = slot_ids[src + k];
  if (len)
    for (uint64_t k = threadIdx.x; k < cnt; k += 256) len[p0 + k] = slot_len[src + k];
  const uint64_t i = base + threadIdx.x;
  if (i < n) {
    const uint64_t v = tok_off[i + 1];
    tok_off[i + 1] = (v & kTokFlag) | (p0 + (v & ~kTokFlag));
  }
}

// First error wins: the caller's status word takes `code` only if it is 0.
__global__ void status_set_first_kernel(uint32_t *__restrict__ status, uint32_t code) {
  if (threadIdx.x == 0) atomicCAS(status, 0u, code);
}

}  // namespace

hipError_t LaunchStatusSetFirst(uint32_t *status, uint32_t code, hipStream_t st) {
  hipLaunchKernelGGL(status_set_first_kernel, dim3(1), dim3(64), 0, st, status, code);
  return hipGetLastError();
}

hipError_t LaunchTileCompact(const uint64_t *off, uint64_t n, const uint64_t *tile_count, uint64_t *tile_prefix,
                             const int32_t *slot_ids, const uint32_t *slot_len, int32_t *ids, uint32_t *len,
                             uint64_t *tok_off, void *scan_tmp, size_t *scan_tmp_bytes, const uint32_t *status,
                             hipStream_t st) {
  const uint64_t tiles = FastTiles(n);
  if (scan_tmp == nullptr)
    return hipcub::DeviceScan::InclusiveSum(nullptr, *scan_tmp_bytes, tile_count, tile_prefix + 1,
                                            static_cast<int>(tiles > 0 ? tiles : 1), st);
  if (tiles == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(tile_prefix, 0, sizeof(uint64_t), st);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::InclusiveSum(scan_tmp, *scan_tmp_bytes, tile_count, tile_prefix + 1,
                                       static_cast<int>(tiles), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tile_compact_kernel, dim3(static_cast<unsigned>(tiles)), dim3(256), 0, st, off, n, tile_prefix,
                     slot_ids, slot_len, ids, len, tok_off, status);
  return hipGetLastError();
}

hipError_t LaunchEncodeFixup(const FixupLaunch &f, hipStream_t st) {
  if (f.n == 0) {
    if (f.out_status) return hipMemsetAsync(f.out_status, 0, sizeof(uint32_t), st);
    return hipSuccess;
  }
  const uint64_t g64 = (f.n + 255) / 256;
  const unsigned grid = static_cast<unsigned>(g64 < 1024 ? g64 : 1024);
  hipLaunchKernelGGL(fixup_gather_kernel, dim3(grid), dim3(256), 0, st, f);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  uint64_t tiles = (f.n + 1023) / 1024;
  if (tiles > kScanTiles) tiles = kScanTiles;
  const uint64_t chunk = (f.n + tiles - 1) / tiles;
  tiles = (f.n + chunk - 1) / chunk;
  hipLaunchKernelGGL(fixup_scan_kernel, dim3(static_cast<unsigned>(tiles)), dim3(256), 0, st, f, chunk);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t cg64 = (f.n + 255) / 256;  // (one wave per 64 sentences)
  hipLaunchKernelGGL(compact_kernel<true>, dim3(static_cast<unsigned>(cg64 < 4096 ? cg64 : 4096)), dim3(256), 0, st,
                     f.off, f.n, f.slot_ids, f.slot_len, f.ids, f.len, f.tok_off, f.status, f.out_status);
  return hipGetLastError();
}

hipError_t LaunchCompact(const uint64_t *off, uint64_t n, const uint32_t *ntok, const int32_t *slot_ids,
                         const uint32_t *slot_len, int32_t *ids, uint32_t *piece_len, uint64_t *tok_off,
                         void *scan_tmp, size_t *scan_tmp_bytes, const uint32_t *status, uint32_t *out_status,
                         hipStream_t st) {
  hipcub::TransformInputIterator<uint64_t, ToU64, const uint32_t *> in(ntok, ToU64());
  if (scan_tmp == nullptr) {
    return hipcub::DeviceScan::InclusiveSum(nullptr, *scan_tmp_bytes, in, tok_off + 1,
                                            static_cast<int>(n > 0 ? n : 1), st);
  }
  hipError_t e = hipMemsetAsync(tok_off, 0, sizeof(uint64_t), st);
  if (e != hipSuccess || n == 0) return e;
  e = hipcub::DeviceScan::InclusiveSum(scan_tmp, *scan_tmp_bytes, in, tok_off + 1, static_cast<int>(n), st);
  if (e != hipSuccess) return e;
  const uint64_t g64 = (n + 255) / 256;
  const unsigned grid = static_cast<unsigned>(g64 < 8192 ? g64 : 8192);
  hipLaunchKernelGGL(compact_kernel<false>, dim3(grid), dim3(256), 0, st, off, n, slot_ids, slot_len, ids,
                     piece_len, tok_off, status, out_status);
  return hipGetLastError();
}

}  // namespace spm_amd
