// Host-side state behind the spm_hip_model handle (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/spm_hip.h"
#include "device_types.h"
#include "double_array.h"
#include "model_proto.h"



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
  // device id epilogue (spm_hip_finalize_ids): per-piece type bits, counts, scan temp
  spm_amd::DevBuf d_types, w_ecount, w_escan;
  spm_amd::DevBuf w_rest;  // BPE: sentences the two-per-wave kernel left for the one-per-wave kernel
  bool types_ready = false;
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
