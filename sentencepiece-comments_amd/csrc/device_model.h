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
#include "kernels.h"
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
  uint64_t last_use = 0;             // LRU stamp (by_stream pool)
  uint32_t leases = 0;               // by_stream pool: live leases (pool_mu); never evicted while > 0
  // Encode: w_ctl = status words + tile counts + the fix-up scan's
  // look-back descriptors (zeroed per call); w_slot_* = the fast kernel's
  // tile-dense token slots, w_tprefix their scanned offsets; w_slot2_* =
  // general-path tokens right-aligned in each sentence's byte range; w_bp =
  // back-pointer bytes beyond the LDS window.
  DevBuf w_slot_ids, w_slot_len, w_tprefix;
  DevBuf w_ctl, w_slot2_ids, w_slot2_len, w_ntok, w_cnt, w_bp, w_flagged, w_ovf, w_scan, w_scratch,
      w_rest;
  DevBuf w_bpn;  // wide-char kernel: trie unit of the best node ending at each byte position
  // Wave-cooperative kernel (coop_encode.hip): per-byte length masks and
  // chosen lnode lengths, and its list of sentences left to the general kernel.
  DevBuf w_cpv, w_cnd, w_crest, w_cpart;
  DevBuf w_nlen, w_nscan;    // device normalizer: lengths, scan temp
  DevBuf w_ecount, w_escan;  // id epilogue: counts, scan temp
  DevBuf w_tids, w_tlen, w_ttok;  // SentencePieceText path: raw ids, piece lengths, token offsets
  DevBuf h_in, h_off, h_ids, h_len, h_tok;  // staging for the host API
  // Host API small batches (EncodeHostSmall): one device block [control |
  // offsets | bytes | tok | ids | len] and its pinned host mirror.
  DevBuf w_small;
  uint8_t *pin_small = nullptr;
  size_t pin_small_cap = 0;
  uint32_t pub_seq = 0;  // EncodeHostSmall's publication sequence
  // Resident small-call server (coop_service_kernel) on its own stream: its
  // box in pinned coherent memory, the arguments it was launched with.
  hipStream_t svc_stream = nullptr;
  CoopServiceBox *svc_box = nullptr;
  uint64_t *svc_prof = nullptr;  // SPM_HIP_SERVICE_PROF: raw-call phase cycles (device, 16 words)
  bool svc_running = false;
  CoopServiceArgs svc_args{};
  const void *svc_key[2][6] = {};  // per call kind: the buffers svc_args' tables point into
  void StopService();
  uint32_t *pinned = nullptr;               // 64 B pinned read-back slots
  hipEvent_t ev[2] = {nullptr, nullptr};    // general-path begin/end (timing)
  // Fast-kernel begin/end events of the last kTimingRing timed calls.
  static constexpr int kTimingRing = 64;
  hipEvent_t tev[2 * kTimingRing] = {};
  uint32_t tcount = 0;   // timed calls since the last drain
  int last_slot = -1;    // ring slot of the last timed call
  spm_hip_encode_stats stats{};
  void Release();
};

// One encode call (device pointers, all enqueued on st).  capacity: the
// caller's bound on offsets[n] (every workspace buffer is sized from it).
struct EncodeCall {
  const uint8_t *bytes;
  const uint64_t *off;
  uint64_t n;
  uint64_t capacity;
  int32_t *ids;
  uint32_t *len;
  uint64_t *tok;
  uint32_t *out_status;  // caller's device status word (nullable; first error wins)
  hipStream_t st;
  bool host_sized;       // general kernel over every sentence, scratch sized on the host
  uint32_t max_nb;       // host_sized: longest sentence
};

// Scratch plan of the device-count general path: `lanes` slabs for sentences
// of <= small_nb bytes, then one lane with the whole pool for the longer
// ones (<= big_nb bytes); longer still sets kStError (the blocking entry
// points then re-run the batch with host-sized scratch).
struct GeneralPool {
  uint32_t lanes, small_nb, big_nb;
  uint64_t slab, pool;
};
template <typename SlabFn>
GeneralPool PlanGeneralPool(uint64_t capacity, uint32_t lanes, uint32_t small_cap, SlabFn slab_bytes) {
  GeneralPool g;
  g.lanes = lanes;
  g.small_nb = static_cast<uint32_t>(capacity < small_cap ? (capacity ? capacity : 1) : small_cap);
  g.slab = slab_bytes(g.small_nb);
  g.pool = g.slab * lanes;
  uint64_t lo = g.small_nb, hi = capacity > g.small_nb ? capacity : g.small_nb;
  if (hi > 0xFFFFFFFFull) hi = 0xFFFFFFFFull;
  while (lo < hi) {  // largest nb whose slab fits the pool
    const uint64_t mid = lo + (hi - lo + 1) / 2;
    if (slab_bytes(static_cast<uint32_t>(mid)) <= g.pool) lo = mid;
    else hi = mid - 1;
  }
  g.big_nb = static_cast<uint32_t>(lo);
  return g;
}

}  // namespace spm_amd

struct spm_hip_model {
  spm_amd::ModelProtoView proto;
  int32_t model_type = 1;
  int32_t unk_id = -1;
  int32_t max_piece_chars = 0;
  int32_t max_piece_bytes = 0;  // longest non-UNUSED piece (C-string bytes)
  float min_score = 0.f, max_score = 0.f;
  std::unordered_map<std::string, int32_t> pieces;    // NORMAL/USER_DEFINED/UNUSED
  std::unordered_map<std::string, int32_t> reserved;  // CONTROL/UNKNOWN
  std::vector<std::string> user_defined;
  spm_amd::DoubleArray trie;  // unigram: vocab trie; bpe: symbol trie
  spm_amd::UnigramParams up{};
  int ring_width = 0;         // 16/32/64, 0 → general kernel only
  spm_amd::UnigramKernel kernel = spm_amd::UnigramKernel::kGeneralOnly;
  std::atomic<bool> force_general{false};
  std::atomic<bool> timing{false};
  std::atomic<uint64_t> corrupt_bp{~0ull};  // debug knob (spm_hip_model_set_debug_corrupt_bp)
  std::atomic<uint32_t> coop_min_nb{0};     // wide / char kernels: sentences handed to the cooperative kernel
  std::atomic<int> coop_slab_mode{0};       // spm_hip_model_set_coop_slab
  std::atomic<uint32_t> coop_small_rejects{0};  // consecutive small host calls the cooperative kernel handed back
  std::atomic<uint32_t> coop_slab_chars{static_cast<uint32_t>(spm_amd::kCoopSlabChars)};
  bool host_only = false;     // parsed + tables built, nothing on the device
  // device-resident model tables
  spm_amd::DevBuf d_units, d_values, d_scores;
  // byte kernel: per unit (d_units with empty units = label 0xFF, usable-node
  // score or NaN) interleaved
  spm_amd::DevBuf d_uvs;
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
  uint64_t use_clock = 0;  // LRU stamps of by_stream
  std::vector<std::unique_ptr<spm_amd::EncodeWorkspace>> host_pool;
  spm_hip_encode_stats last_stats{};  // of the last completed encode call (pool_mu)
  int device = 0;
};

namespace spm_amd {

// Workspaces kept per model handle for caller streams (least recently used
// idle ones are released beyond this; spm_hip_model_release_stream drops one
// explicitly).
constexpr size_t kMaxStreamWorkspaces = 16;

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
