// Host-side state behind the spm_hip_model handle (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/spm_hip.h"
#include "double_array.h"
#include "model_proto.h"

namespace spm_amd {

// Grow-only device buffer: encode never allocates after warm-up.
struct DevBuf {
  void *ptr = nullptr;
  size_t cap = 0;
  hipError_t Reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    size_t c = bytes + bytes / 4 + 256;
    hipError_t e = hipMalloc(&ptr, c);
    if (e == hipSuccess) cap = c;
    return e;
  }
  void Release() {
    if (ptr) (void)hipFree(ptr);
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
  DevBuf entry_piece;   // int32
  DevBuf entry_out;     // int32
  DevBuf piece_kind;    // uint8 per piece id: 0 other, 1 user-defined, 2 unused
  DevBuf piece_out;     // int32 PieceToId(piece string) per pieces_ id
  uint64_t pair_mask = 0;
  bool has_user_defined = false;
  bool irregular = false;  // some piece = (char outside pieces_) · (piece) or ·char
};

}  // namespace spm_amd

struct spm_hip_model {
  spm_amd::ModelProtoView proto;
  int32_t model_type = 1;
  int32_t unk_id = -1;
  int32_t max_piece_chars = 0;
  float min_score = 0.f, max_score = 0.f;
  std::unordered_map<std::string, int32_t> pieces;    // NORMAL/USER_DEFINED/UNUSED
  std::unordered_map<std::string, int32_t> reserved;  // CONTROL/UNKNOWN
  std::vector<std::string> user_defined;
  spm_amd::DoubleArray trie;  // unigram: vocab trie; bpe: symbol trie
  spm_amd::UnigramParams up{};
  int ring_width = 0;         // 16/32/64, 0 → general kernel only
  bool force_general = false;
  bool host_only = false;     // parsed + tables built, nothing on the device
  // device-resident model tables
  spm_amd::DevBuf d_units, d_values, d_scores, d_vscore;
  spm_amd::DevBuf d_units_ff;  // d_units with empty units = label 0xFF (kVar & 8)
  spm_amd::DevBuf d_vscore_bp; // per-unit usable-node score or NaN (kVar & 16)
  int variant = 7;            // unigram fast-kernel variant bits (kernels.h)
  spm_amd::BpeDevice bpe;
  // device normalizer tables (uploaded on first use): charsmap blob, user-defined trie
  spm_amd::DevBuf d_charsmap, d_ud_units;
  bool norm_ready = false;
  uint32_t ud_units_n = 0;
  spm_amd::DevBuf w_nlen, w_nscan;
  // pooled work buffers
  spm_amd::DevBuf w_slot_ids, w_slot_len, w_slot2_ids, w_slot2_len, w_ntok, w_lo, w_bp, w_flagged,
      w_status, w_scan, w_scratch;
  spm_amd::DevBuf h_in, h_off, h_ids, h_len, h_tok;  // staging for the host API
  uint32_t *pinned_status = nullptr;
  bool timing = false;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // fast begin/end, general begin/end
  spm_hip_encode_stats stats{};
  int device = 0;
};
