// Device-side types shared by the kernels and the C-ABI implementation
// (kept apart from device_model.h so kernel objects do not depend on the
// spm_hip_model handle or the public header).
#pragma once

#include <hip/hip_runtime.h>

#include "scratch_cache.h"

#include <cstdint>

namespace spm_amd {

// Grow-only device buffer: encode never allocates after warm-up.
struct DevBuf {
  void *ptr = nullptr;
  size_t cap = 0;
  hipError_t Reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (ptr) (void)DevFree(ptr);
    ptr = nullptr;
    cap = 0;
    size_t c = bytes + bytes / 4 + 256;
    hipError_t e = DevMalloc(&ptr, c);
    if (e == hipSuccess) cap = c;
    return e;
  }
  void Release() {
    if (ptr) (void)DevFree(ptr);
    ptr = nullptr;
    cap = 0;
  }
  template <typename T>
  T *as() const {
    return static_cast<T *>(ptr);
  }
};

// Piece payload stored in the device trie value slot (unigram):
//   bits 0..27 piece id, bits 28..29 kind (0 normal, 1 user-defined, 2 unused).
constexpr int32_t kKindShift = 28;
constexpr int32_t kIdMask = (1 << kKindShift) - 1;
constexpr int32_t kKindUserDefined = 1;
constexpr int32_t kKindUnused = 2;

// Scalars the unigram kernels need (mirrors unigram::Model members:
// unigram_model.cc:677-695 and PopulateNodes :535-604).
struct UnigramParams {
  uint32_t root_base;
  int32_t unk_id;
  float unk_score;     // min_score_ - kUnkPenalty (float arithmetic)
  float max_score;     // starts at FLT_MIN (unigram_model.cc:683)
  float tie_mag;       // bound on |node score| + 1, for the near-tie test
  int32_t trie_results_size;
};

// BPE tables (bpe_model.cc:37-199 restated for the device, see bpe kernels).
// The string trie (m->trie) holds every pieces_ and reserved_id_map_ string;
// its value is an entry index:
//   entry_piece[e] = pieces_ id of the string or -1   (pieces_.find)
//   entry_out[e]   = PieceToId(string)                 (model_interface.cc:87-97)
// Symbols are pieces_ ids (-1 = a char outside pieces_).  pair table: key
// (left id << 32 | right id) → id of the concatenation in pieces_.
struct BpeDevice {
  DevBuf pair_keys;     // uint64, empty = ~0
  DevBuf pair_vals;     // int32 merged pieces_ id
  DevBuf pair_ent;      // uint4 {right id, left id, merged id | unused<<31, score bits}
  DevBuf entry_piece;   // int32
  DevBuf entry_out;     // int32
  DevBuf piece_kind;    // uint8 per piece id: 0 other, 1 user-defined, 2 unused
  DevBuf piece_out;     // int32 PieceToId(piece string) per pieces_ id
  DevBuf rank_piece;    // int16 per score rank: the merged piece (rank_ids only)
  uint64_t pair_mask = 0;
  bool has_user_defined = false;
  bool irregular = false;  // some piece = (char outside pieces_) · (piece) or ·char
  bool lane_ok = false;    // ids fit int16: bpe_lane_kernel (one sentence per lane)
  bool rank_ids = false;   // merged pieces have distinct score ranks: bpe_lane_kernel<true>
  // rank -> merged piece is piece = rank_base - rank on every pair's rank
  // (pieces in descending-score order with distinct scores, as trained BPE
  // models are): the lane kernel skips the table load.  -1: use the table.
  int32_t rank_base = -1;
};

}  // namespace spm_amd
