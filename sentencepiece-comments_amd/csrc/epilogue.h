// Device id epilogue (PopulateSentencePieceText unk merge + ApplyExtraOptions),
// see epilogue_kernels.hip.  Internal; the public entry is spm_hip_finalize_ids.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/spm_hip.h"

namespace spm_amd {

// Per-piece type bits (ModelProto::SentencePiece::Type, sentencepiece_model.proto).
constexpr uint8_t kPieceUnknown = 1;
constexpr uint8_t kPieceControl = 2;

constexpr int kMaxExtras = 32;

// Extra options folded on the host: out = pre · mid (reversed?) · post.
struct EpilogueExtras {
  int32_t ids[2 * kMaxExtras];  // [0, num_pre): pre; [kMaxExtras, kMaxExtras + num_post): post
  uint32_t num_pre;
  uint32_t num_post;
  uint32_t reversed;
};

// chain (nullable): an asynchronous call's status word; the kernels do
// nothing once it is non-zero, and an output larger than cap_limit is not
// written (chain := RESOURCE_EXHAUSTED).
hipError_t LaunchEpilogueCount(const int32_t *ids, const uint64_t *tok_off, uint64_t n, const uint8_t *types,
                               int32_t num_types, uint32_t extras, uint64_t *count, hipStream_t st,
                               const uint32_t *chain = nullptr);
hipError_t LaunchEpilogueWrite(const int32_t *ids, const uint64_t *tok_off, uint64_t n, const uint8_t *types,
                               int32_t num_types, const EpilogueExtras &x, const uint64_t *out_off,
                               int32_t *out, hipStream_t st, uint64_t cap_limit = ~0ull,
                               uint32_t *chain = nullptr);

// SentencePieceText epilogue: the merged pieces with begin/end through
// norm_to_orig (layout of spm_hip_normalize_batch_device_align).
hipError_t LaunchSptWrite(const int32_t *ids, const uint32_t *lens, const uint64_t *tok_off, uint64_t n,
                          const uint8_t *types, int32_t num_types, const EpilogueExtras &x,
                          const uint32_t *n2o, const uint64_t *norm_off, const uint64_t *out_off,
                          spm_hip_piece *out, hipStream_t st);

}  // namespace spm_amd
