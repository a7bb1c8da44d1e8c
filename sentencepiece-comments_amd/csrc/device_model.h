// Host-side state behind the spm_hip_model handle (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/spm_hip.h"
#include "device_types.h"
#include "double_array.h"
#include "model_proto.h"



namespace spm_amd {

// Per-stream encode workspace.  The model tables of a handle are immutable
// after load; everything a call writes lives here, so concurrent calls on one
// handle with different streams never share a buffer (the reference's
// unigram::Model::Encode is const with a stack-local Lattice,
// unigram_model.cc:705-720).  A workspace is bound to one stream (device API)
// or owns a private stream (host-buffer API); `mu` is held for a whole call.
struct EncodeWorkspace {
  std::mutex mu;
  hipStream_t own_stream = nullptr;  // host API: private non-blocking stream
  bool busy = false;                 // host API pool: leased
  DevBuf w_slot_ids, w_slot_len, w_slot2_ids, w_slot2_len, w_ntok, w_lo, w_bp, w_flagged,
      w_status, w_scan, w_scratch, w_rest;
  DevBuf w_nlen, w_nscan;    // device normalizer: lengths, scan temp
  DevBuf w_ecount, w_escan;  // id epilogue: counts, scan temp
  DevBuf w_tids, w_tlen, w_ttok;  // SentencePieceText path: raw ids, piece lengths, token offsets
  DevBuf h_in, h_off, h_ids, h_len, h_tok;  // staging for the host API
  uint32_t *pinned = nullptr;               // 64 B pinned read-back slots
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // fast/general begin/end
  spm_hip_encode_stats stats{};
  void Release();
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
  std::atomic<bool> force_general{false};
  std::atomic<bool> timing{false};
  bool host_only = false;     // parsed + tables built, nothing on the device
  // device-resident model tables
  spm_amd::DevBuf d_units, d_values, d_scores, d_vscore;
  spm_amd::DevBuf d_units_ff;  // d_units with empty units = label 0xFF (kVar & 8)
  spm_amd::DevBuf d_vscore_bp; // per-unit usable-node score or NaN (kVar & 16)
  spm_amd::DevBuf d_uvs;       // per unit {d_units_ff, d_vscore_bp} (lane kernel)
  spm_amd::DevBuf d_jump2;     // uint2[65536]: {unit, score} after the first two bytes (kVar & 4096)
  int variant = 7;            // unigram fast-kernel variant bits (kernels.h)
  spm_amd::BpeDevice bpe;
  // Lazily uploaded tables (under init_mu): device normalizer charsmap blob +
  // user-defined trie; id-epilogue piece type bits.
  std::mutex init_mu;
  spm_amd::DevBuf d_charsmap, d_ud_units;
  std::atomic<bool> norm_ready{false};
  uint32_t ud_units_n = 0;
  spm_amd::DevBuf d_types;
  std::atomic<bool> types_ready{false};
  // Workspaces (under pool_mu): one per caller stream, a pool for the host API.
  std::mutex pool_mu;
  std::unordered_map<hipStream_t, std::unique_ptr<spm_amd::EncodeWorkspace>> by_stream;
  std::vector<std::unique_ptr<spm_amd::EncodeWorkspace>> host_pool;
  spm_hip_encode_stats last_stats{};  // of the last completed encode call (pool_mu)
  int device = 0;
};

namespace spm_amd {

// RAII lease of a workspace: the device API keys it by the caller's stream
// (calls on one stream serialize on its mutex, as the stream itself would);
// the host API takes a free workspace with a private stream.
class WorkspaceLease {
 public:
  WorkspaceLease() = default;
  WorkspaceLease(const WorkspaceLease &) = delete;
  WorkspaceLease &operator=(const WorkspaceLease &) = delete;
  ~WorkspaceLease();
  // Returns hipSuccess or the allocation error.
  hipError_t ForStream(spm_hip_model *m, hipStream_t st);
  hipError_t ForHost(spm_hip_model *m);
  EncodeWorkspace *operator->() const { return ws_; }
  EncodeWorkspace *get() const { return ws_; }
  hipStream_t stream() const { return st_; }

 private:
  spm_hip_model *m_ = nullptr;
  EncodeWorkspace *ws_ = nullptr;
  hipStream_t st_ = nullptr;
  bool host_ = false;
  std::unique_lock<std::mutex> lock_;
};

// Records a call's stats as the handle's last_stats.
void PublishStats(spm_hip_model *m, const spm_hip_encode_stats &s);

}  // namespace spm_amd
