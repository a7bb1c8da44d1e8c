// E-step / pruning shard plan of a multi-GPU spm_train (one rank per GPU).
//
// The reference fans RunEStep out over num_threads = T threads: sentence i
// goes to thread i mod T, each thread accumulates its float vectors in
// sentence order, and the per-thread vectors are summed in thread order
// (unigram_model_trainer.cc:237-287; the pruning Viterbi does the same at
// :383-421).  A rank here owns whole buckets, so every bucket is still
// accumulated on one device in ascending sentence order and the cross-rank
// SUM of zero-padded bucket rows is exact:
//   PARITY, T % W == 0 : rank r takes the sentences r, r+W, r+2W, ... (its
//                        buckets r, r+W, ... interleaved), one strided segment;
//   PARITY, otherwise  : rank r takes buckets b = r, r+W, ... < T, one segment
//                        (b, b+T, b+2T, ...) per bucket;
//   FAST               : a contiguous range (fp64 sums, no bucket order).
// A segment is (index_base, index_stride, count): its k-th sentence has global
// index index_base + k * index_stride -- exactly the contract of
// spm_hip_estep_accumulate.  A rank's local sentences are its segments
// concatenated in plan order.
#ifndef SPM_AMD_SHARD_PLAN_H_
#define SPM_AMD_SHARD_PLAN_H_

#include <cstdint>
#include <vector>

namespace spm_amd {

struct ShardSegment {
  uint64_t index_base = 0, index_stride = 1, count = 0;
};

// Number of i in [0, n) with i = base (mod stride).
inline uint64_t StridedCount(uint64_t n, uint64_t base, uint64_t stride) {
  return base < n ? (n - base + stride - 1) / stride : 0;
}

// parity: bucket-ordered (PARITY) plan, else contiguous (FAST).
inline std::vector<ShardSegment> EStepShardPlan(uint64_t n, bool parity, int T, int W, int r) {
  std::vector<ShardSegment> out;
  if (W < 1 || r < 0 || r >= W) return out;
  if (W == 1) {
    out.push_back({0, 1, n});
    return out;
  }
  if (!parity) {
    const uint64_t lo = n * r / W, hi = n * (r + 1) / W;
    out.push_back({lo, 1, hi - lo});
    return out;
  }
  if (T < 1) T = 1;
  if (T % W == 0) {
    out.push_back({static_cast<uint64_t>(r), static_cast<uint64_t>(W), StridedCount(n, r, W)});
    return out;
  }
  for (int b = r; b < T; b += W)
    out.push_back({static_cast<uint64_t>(b), static_cast<uint64_t>(T), StridedCount(n, b, T)});
  return out;
}

// The rank that accumulates PARITY bucket b in EStepShardPlan (both of its
// PARITY branches give b % W; W > T leaves ranks >= T without buckets).
// ReduceToRank0 gathers row b from this rank.
inline int EStepBucketOwner(int b, int W) { return W < 1 || b < 0 ? -1 : b % W; }

}  // namespace spm_amd

#endif  // SPM_AMD_SHARD_PLAN_H_
