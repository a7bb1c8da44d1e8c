// C-ABI implementation (include/spm_hip.h): model load (ModelFactory::Create +
// InitializePieces + unigram::Model / bpe::Model constructors) and the batched
// encode entry points.
#include <hip/hip_runtime.h>

#include "scratch_cache.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "../../include/spm_hip.h"
#include "bpe_tables.h"
#include "device_model.h"
#include "epilogue.h"
#include "kernels.h"
#include "normalize_device.h"
#include "normalizer.h"
#include "shard_plan.h"
#include "trace.h"

namespace {

thread_local std::string g_last_error;
uint32_t DefaultCoopMinNb();  // (below, with the encode plan)

int Fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

#define SPM_HIP_TRY(expr)                                                              \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return Fail(SPM_INTERNAL, std::string(#expr) + ": " + hipGetErrorString(_e));   \
  } while (0)

int CountChars(const std::string &s) {
  int n = 0;
  for (size_t i = 0; i < s.size();) {
    i += std::min<size_t>(spm_amd::OneCharLen(static_cast<uint8_t>(s[i])), s.size() - i);
    ++n;
  }
  return n;
}

template <typename T>
hipError_t Upload(spm_amd::DevBuf *buf, const std::vector<T> &v) {
  hipError_t e = buf->Reserve(std::max<size_t>(v.size(), 1) * sizeof(T));
  if (e != hipSuccess) return e;
  if (v.empty()) return hipSuccess;
  return hipMemcpy(buf->ptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}

// ModelInterface::InitializePieces (model_interface.cc:101-144).
int InitializePieces(spm_hip_model *m) {
  m->unk_id = -1;
  for (size_t i = 0; i < m->proto.pieces.size(); ++i) {
    const auto &sp = m->proto.pieces[i];
    if (sp.piece.empty()) return Fail(SPM_INTERNAL, "piece must not be empty.");
    const bool normal = sp.type == spm_amd::kNormal || sp.type == spm_amd::kUserDefined ||
                        sp.type == spm_amd::kUnused;
    auto &dst = normal ? m->pieces : m->reserved;
    if (!dst.emplace(sp.piece, static_cast<int32_t>(i)).second)
      return Fail(SPM_INTERNAL, sp.piece + " is already defined.");
    if (sp.type == spm_amd::kUserDefined) m->user_defined.push_back(sp.piece);
    if (sp.type == spm_amd::kUnknown) {
      if (m->unk_id >= 0) return Fail(SPM_INTERNAL, "unk is already defined.");
      m->unk_id = static_cast<int32_t>(i);
    }
  }
  if (m->unk_id == -1) return Fail(SPM_INTERNAL, "unk is not defined.");
  std::sort(m->user_defined.begin(), m->user_defined.end());
  return SPM_OK;
}

// unigram::Model::Model (unigram_model.cc:677-695) + BuildTrie (:624-673).
int LoadUnigram(spm_hip_model *m) {
  m->min_score = FLT_MAX;
  m->max_score = FLT_MIN;
  for (const auto &sp : m->proto.pieces)
    if (sp.type == spm_amd::kNormal) {
      m->min_score = std::min(m->min_score, sp.score);
      m->max_score = std::max(m->max_score, sp.score);
    }
  if (m->proto.pieces.size() >= static_cast<size_t>(spm_amd::kIdMask))
    return Fail(SPM_RESOURCE_EXHAUSTED, "too many pieces for the device trie");
  std::vector<std::pair<std::string, int32_t>> keys;
  keys.reserve(m->pieces.size());
  int max_chars = 0;
  size_t max_bytes = 0;
  bool split_ok = true;
  float tie_mag = 0.f;
  for (const auto &kv : m->pieces) {
    const int32_t id = kv.second;
    const int32_t type = m->proto.pieces[id].type;
    int32_t kind = 0;
    if (type == spm_amd::kUserDefined) kind = spm_amd::kKindUserDefined;
    if (type == spm_amd::kUnused) kind = spm_amd::kKindUnused;
    keys.emplace_back(kv.first, id | (kind << spm_amd::kKindShift));
    if (type != spm_amd::kUnused) {
      // C-string key semantics: count chars up to the first NUL.
      std::string k = kv.first.substr(0, kv.first.find('\0'));
      // Byte-position kernel precondition: the lead-byte chain ends exactly
      // at the end of the piece (no char cut by the piece boundary).
      size_t q = 0;
      while (q < k.size()) q += spm_amd::OneCharLen(static_cast<uint8_t>(k[q]));
      if (q != k.size()) split_ok = false;
      max_chars = std::max(max_chars, CountChars(k));
      max_bytes = std::max(max_bytes, k.size());
    }
    if (type == spm_amd::kNormal) tie_mag = std::max(tie_mag, std::fabs(m->proto.pieces[id].score));
  }
  if (keys.empty()) return Fail(SPM_INTERNAL, "no pieces are loaded.");
  std::string err;
  if (!spm_amd::BuildDoubleArray(std::move(keys), &m->trie, &err)) return Fail(SPM_RESOURCE_EXHAUSTED, err);
  if (m->trie.max_prefix_matches == 0) return Fail(SPM_INTERNAL, "no entry is found in the trie.");
  m->max_piece_chars = max_chars;
  m->max_piece_bytes = static_cast<int32_t>(max_bytes);
  const float unk_score = m->min_score - 10.0f;  // kUnkPenalty (unigram_model.cc:563)
  tie_mag = std::max(tie_mag, std::fabs(unk_score));
  tie_mag = std::max(tie_mag, std::fabs(static_cast<float>(max_chars) * m->max_score) + 1.0f);
  m->up.root_base = spm_amd::DoubleArray::Base(m->trie.units[0]);
  m->up.unk_id = m->unk_id;
  m->up.unk_score = unk_score;
  m->up.max_score = m->max_score;
  m->up.tie_mag = tie_mag + 1.0f;
  m->up.trie_results_size = m->trie.max_prefix_matches;
  // The fast kernel's ring is indexed by byte distance: W > longest piece in bytes.
  m->ring_width = max_bytes < 16 ? 16 : max_bytes < 32 ? 32 : max_bytes < 64 ? 64 : 0;
  std::vector<float> scores(m->proto.pieces.size());
  for (size_t i = 0; i < scores.size(); ++i) scores[i] = m->proto.pieces[i].score;
  bool nan_score = false;
  for (size_t u = 0; u < m->trie.units.size(); ++u) {
    if (!spm_amd::DoubleArray::Leaf(m->trie.units[u])) continue;
    const int32_t v = m->trie.values[u];
    if ((v >> spm_amd::kKindShift) == 0) nan_score |= std::isnan(scores[v & spm_amd::kIdMask]);
  }
  // The byte kernel (W = 16 byte-position pass, unigram_encode.hip) needs
  // pieces of < 16 bytes made of whole chars and no NaN score (NaN tags the
  // per-unit score table); other models with pieces of < 64 bytes run the
  // char kernel (values + scores tables), longer ones the general kernel.
  const bool byte_ok = m->ring_width == 16 && !nan_score && split_ok;
  // Wide-char pass: pieces of whole chars, < 16 chars and < 64 bytes (CJK
  // vocabularies, whose pieces outgrow the byte kernel's 16-byte ring); its
  // ring is indexed by chars (W = 16 chars).
  const bool wide_ok = !byte_ok && split_ok && !nan_score && max_chars < 16 && max_bytes < 64 &&
                       std::getenv("SPM_HIP_NO_WIDE") == nullptr;  // A/B knob
  m->kernel = byte_ok   ? spm_amd::UnigramKernel::kByte
              : wide_ok ? spm_amd::UnigramKernel::kWide
              : m->ring_width ? spm_amd::UnigramKernel::kChar : spm_amd::UnigramKernel::kGeneralOnly;
  if (wide_ok) m->ring_width = 16;
  // The wave-cooperative kernel walks the (unit, score) table, whose NaN
  // marks units without a usable node: models with a NaN score keep the
  // lane kernels' path.
  m->coop_min_nb = (nan_score || max_bytes > 56) ? 0u : DefaultCoopMinNb();
  if (m->host_only) return SPM_OK;
  SPM_HIP_TRY(Upload(&m->d_units, m->trie.units));
  SPM_HIP_TRY(Upload(&m->d_values, m->trie.values));
  SPM_HIP_TRY(Upload(&m->d_scores, scores));
  if (byte_ok || wide_ok || (m->kernel == spm_amd::UnigramKernel::kChar && !nan_score)) {
    // Empty units get label 0xFF so a walk needs no NUL test: real labels
    // are never 0 (keys stop at NUL) and a 0xFF input byte flags the sentence.
    // The root (unit 0, label 0) gets 0xFF too: a childless node has base 0,
    // so an input NUL after it would otherwise step onto the root and match.
    std::vector<uint32_t> ff = m->trie.units;
    for (size_t u = 1; u < ff.size(); ++u)
      if (ff[u] == 0) ff[u] = 0xFFu;
    if (!ff.empty()) ff[0] |= 0xFFu;
    // Byte-pass score table: the node score (USER_DEFINED: length * max_score
    // + 1.0, unigram_model.cc:589-591, length = the piece's char count), NaN
    // for units that are no usable node (inner, empty, UNUSED).
    std::vector<float> vbp(m->trie.units.size(), std::numeric_limits<float>::quiet_NaN());
    for (size_t u = 0; u < m->trie.units.size(); ++u) {
      if (!spm_amd::DoubleArray::Leaf(m->trie.units[u])) continue;
      const int32_t v = m->trie.values[u];
      const int32_t kind = v >> spm_amd::kKindShift;
      const int32_t id = v & spm_amd::kIdMask;
      if (kind == 0) {
        vbp[u] = scores[id];
      } else if (kind == spm_amd::kKindUserDefined) {
        const std::string &pc = m->proto.pieces[id].piece;
        const int chars = CountChars(pc.substr(0, pc.find('\0')));
        const float prod = static_cast<float>(chars) * m->max_score;
        vbp[u] = static_cast<float>(static_cast<double>(prod) + 1.0);
      }
    }
    // One (unit, score) pair per unit: the walk reads both with one 8-byte
    // gather per step.
    std::vector<uint32_t> uvs(2 * ff.size());
    for (size_t u = 0; u < ff.size(); ++u) {
      uvs[2 * u] = ff[u];
      std::memcpy(&uvs[2 * u + 1], &vbp[u], 4);
    }
    SPM_HIP_TRY(Upload(&m->d_uvs, uvs));
  }
  return SPM_OK;
}

// Fast-kernel timing: begin/end events of the workspace ring (created on
// first use); -1 when timing is off.
int TimedSlot(spm_hip_model *m, spm_amd::EncodeWorkspace *ws) {
  if (!m->timing) return -1;
  const int slot = static_cast<int>(ws->tcount % spm_amd::EncodeWorkspace::kTimingRing);
  for (int k = 0; k < 2; ++k)
    if (!ws->tev[2 * slot + k] && hipEventCreate(&ws->tev[2 * slot + k]) != hipSuccess) return -1;
  for (auto &e : ws->ev)
    if (!e && hipEventCreate(&e) != hipSuccess) return -1;
  ++ws->tcount;
  ws->last_slot = slot;
  return slot;
}

// Status words + look-back descriptors of one encode call, zeroed on the
// stream.  Returns the status pointer.
int PrepareControl(spm_amd::EncodeWorkspace *ws, uint64_t n, hipStream_t st, uint32_t **status) {
  const size_t bytes = spm_amd::kStWords * 4 + 8 * (spm_amd::FastTiles(n) + spm_amd::kScanTiles);
  SPM_HIP_TRY(ws->w_ctl.Reserve(bytes));
  SPM_HIP_TRY(hipMemsetAsync(ws->w_ctl.ptr, 0, bytes, st));
  *status = ws->w_ctl.as<uint32_t>();
  return SPM_OK;
}

constexpr uint32_t kGeneralLanes = 128;     // general-path lanes of the device-count pass
constexpr uint32_t kGeneralSmallNb = 2048;  // per-lane slab: sentences up to this many bytes

spm_amd::UnigramLaunch UnigramTables(spm_hip_model *m, const spm_amd::EncodeCall &c, uint32_t *status) {
  const bool byte_k = m->kernel == spm_amd::UnigramKernel::kByte || m->kernel == spm_amd::UnigramKernel::kWide;
  spm_amd::UnigramLaunch l{};
  l.bytes = c.bytes;
  l.off = c.off;
  l.n = c.n;
  l.capacity = c.capacity;
  l.units = byte_k ? m->d_uvs.as<uint32_t>() : m->d_units.as<uint32_t>();
  l.gen_units = m->d_units.as<uint32_t>();
  l.values = m->d_values.as<int32_t>();
  l.scores = m->d_scores.as<float>();
  l.num_units = static_cast<uint32_t>(m->trie.units.size());
  l.p = m->up;
  l.ids = c.ids;
  l.len = c.len;
  l.tok_off = c.tok;
  l.status = status;
  l.corrupt_bp = m->corrupt_bp.load();
  l.chain = c.out_status;
  return l;
}


// Unigram fast path: no host synchronization.  Fast kernel (dense output),
// then the device-count general passes and the fix-up chain, which do
// nothing unless the fast kernel flagged a sentence.
// One fast-path unigram encode, in two parts: A = the fast kernel (+ the
// tile compaction), B = the general kernel over the flagged sentences + the
// fix-up chain (device no-ops when nothing was flagged).
struct FastPlan {
  spm_amd::UnigramLaunch l;
  spm_amd::GeneralPool gp;
  uint32_t *status = nullptr;
  uint64_t *desc = nullptr;
  int slot = -1;
  bool coop = false;  // long sentences: the wave-cooperative kernel before the general one
  uint64_t slab_chars = 0;  // CoopArgs::slab_chars
  uint32_t coop_blocks = 0;
};

// The wave-cooperative kernel takes the wide / char kernels' sentences of at
// least kCoopMinNb bytes (SPM_HIP_COOP=0 turns it off, SPM_HIP_COOP_MIN_NB
// moves the threshold; A/B knobs).  The byte kernel (short-piece models, the
// c2 path) keeps every sentence.
uint32_t DefaultCoopMinNb() {
  static const bool on = [] {
    const char *e = std::getenv("SPM_HIP_COOP");
    return !(e && std::atoi(e) == 0);
  }();
  static const uint32_t min_nb = [] {
    const char *e = std::getenv("SPM_HIP_COOP_MIN_NB");
    return e ? static_cast<uint32_t>(std::max(1, std::atoi(e))) : 128u;
  }();
  return on ? min_nb : 0u;
}

// Grid cap of the list kernel (SPM_HIP_COOP_BLOCKS: A/B knob, read per call).
uint32_t CoopMaxBlocks() {
  const char *e = std::getenv("SPM_HIP_COOP_BLOCKS");
  const int v = e ? std::atoi(e) : 0;
  return v > 0 ? static_cast<uint32_t>(v) : spm_amd::kCoopMaxBlocks;
}

// The list kernel takes its sentences from a work queue, long ones first
// (SPM_HIP_COOP_QUEUE=0: static grid stride over the flagged list; A/B knob).
bool CoopQueue() {
  static const bool on = [] {
    const char *e = std::getenv("SPM_HIP_COOP_QUEUE");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

uint32_t CoopMinNb(const spm_hip_model *m) {
  if (m->kernel != spm_amd::UnigramKernel::kWide && m->kernel != spm_amd::UnigramKernel::kChar) return 0;
  return m->coop_min_nb.load();
}

// Work buffers and launch tables; `status` = a zeroed control block of
// PrepareControl's size (nullptr: PrepareControl zeroes the workspace's).
int FastSetup(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const spm_amd::EncodeCall &c, uint32_t *status,
              FastPlan *fp) {
  const uint64_t n = c.n, cap = std::max<uint64_t>(c.capacity, 1), nn = std::max<uint64_t>(n, 1);
  const hipStream_t st = c.st;
  if (!status) {
    int rc = PrepareControl(ws, n, st, &status);
    if (rc != SPM_OK) return rc;
  }
  fp->status = status;
  fp->desc = reinterpret_cast<uint64_t *>(status + spm_amd::kStWords);
  SPM_HIP_TRY(ws->w_bp.Reserve(cap + 16));
  SPM_HIP_TRY(ws->w_flagged.Reserve(nn * 4));
  SPM_HIP_TRY(ws->w_ntok.Reserve(nn * 4));
  SPM_HIP_TRY(ws->w_cnt.Reserve(nn * 4));
  SPM_HIP_TRY(ws->w_slot2_ids.Reserve(cap * 4));
  if (c.len) SPM_HIP_TRY(ws->w_slot2_len.Reserve(cap * 4));
  const int K = m->up.trie_results_size;
  fp->gp = spm_amd::PlanGeneralPool(cap, kGeneralLanes, kGeneralSmallNb,
                                    [&](uint32_t nb) { return spm_amd::UnigramGeneralSlabBytes(nb, K); });
  SPM_HIP_TRY(ws->w_scratch.Reserve(fp->gp.pool));
  const uint64_t ovf_cap = std::min<uint64_t>(nn, cap / (fp->gp.small_nb + 1ull) + 1);
  SPM_HIP_TRY(ws->w_ovf.Reserve(ovf_cap * 4));
  fp->l = UnigramTables(m, c, status);
  fp->l.bp = ws->w_bp.as<uint8_t>();
  if (m->kernel == spm_amd::UnigramKernel::kWide) {
    SPM_HIP_TRY(ws->w_bpn.Reserve((cap + 16) * 4));
    fp->l.bpn = ws->w_bpn.as<uint32_t>();
  }
  fp->l.flagged = ws->w_flagged.as<uint32_t>();
  fp->l.tile_count = fp->desc;
  SPM_HIP_TRY(ws->w_slot_ids.Reserve(cap * 4));
  if (c.len) SPM_HIP_TRY(ws->w_slot_len.Reserve(cap * 4));
  SPM_HIP_TRY(ws->w_tprefix.Reserve((spm_amd::FastTiles(n) + 1) * 8));
  fp->l.slot_ids = ws->w_slot_ids.as<int32_t>();
  fp->l.slot_len = c.len ? ws->w_slot_len.as<uint32_t>() : nullptr;
  fp->l.coop_min_nb = CoopMinNb(m);
  fp->coop = fp->l.coop_min_nb != 0;
  if (fp->coop) {
    // Cooperative-kernel rows (kCoopSlots x 6 B per char): by byte offset
    // when the call is small, else one slab per wave of the list kernel's
    // grid (bounded whatever the call's size).
    const uint64_t slab = m->coop_slab_chars.load();
    fp->coop_blocks = spm_amd::CoopBlocks(n, CoopMaxBlocks());
    const uint64_t slab_rows = uint64_t{fp->coop_blocks} * 4 * slab;
    const int mode = m->coop_slab_mode.load();
    fp->slab_chars = mode == 1 || (mode == 0 && slab_rows < cap + 64) ? slab : 0;
    const uint64_t rows = fp->slab_chars ? slab_rows : cap + 64;
    SPM_HIP_TRY(ws->w_cpv.Reserve(rows * spm_amd::kCoopSlots * 2));
    SPM_HIP_TRY(ws->w_cnd.Reserve(rows * spm_amd::kCoopSlots * 4));
    SPM_HIP_TRY(ws->w_crest.Reserve(nn * 4));
    if (CoopQueue()) SPM_HIP_TRY(ws->w_cpart.Reserve(nn * 4));
  }
  return SPM_OK;
}

// Part A.  compact = false: one tile whose slots start at byte 0
// (FastTiles(n) == 1 and off[0] == 0) writes the final ids / lengths /
// token offsets itself (slots = the outputs, see EncodeHostSmall).
int FastPartA(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const spm_amd::EncodeCall &c, FastPlan *fp,
              bool compact) {
  const hipStream_t st = c.st;
  if (!compact) {
    fp->l.slot_ids = c.ids;
    fp->l.slot_len = c.len;
  }
  fp->slot = TimedSlot(m, ws);
  if (fp->slot >= 0) SPM_HIP_TRY(hipEventRecord(ws->tev[2 * fp->slot], st));
  SPM_HIP_TRY(spm_amd::LaunchUnigramFast(m->kernel, m->ring_width, fp->l, st));
  if (fp->slot >= 0) SPM_HIP_TRY(hipEventRecord(ws->tev[2 * fp->slot + 1], st));
  if (compact) {
    size_t tb = 0;
    SPM_HIP_TRY(spm_amd::LaunchTileCompact(c.off, c.n, fp->desc, ws->w_tprefix.as<uint64_t>(), fp->l.slot_ids,
                                           fp->l.slot_len, c.ids, c.len, c.tok, nullptr, &tb, fp->status, st));
    SPM_HIP_TRY(ws->w_scan.Reserve(tb + 16));
    SPM_HIP_TRY(spm_amd::LaunchTileCompact(c.off, c.n, fp->desc, ws->w_tprefix.as<uint64_t>(), fp->l.slot_ids,
                                           fp->l.slot_len, c.ids, c.len, c.tok, ws->w_scan.ptr, &tb, fp->status,
                                           st));
  }
  return SPM_OK;
}

// Part B.
int FastPartB(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const spm_amd::EncodeCall &c, FastPlan *fp) {
  const hipStream_t st = c.st;
  const uint64_t n = c.n;
  uint32_t *status = fp->status;
  const auto &gp = fp->gp;
  int32_t *s2 = ws->w_slot2_ids.as<int32_t>();
  uint32_t *s2l = c.len ? ws->w_slot2_len.as<uint32_t>() : nullptr;
  uint32_t *ovf = ws->w_ovf.as<uint32_t>();
  if (fp->slot >= 0) SPM_HIP_TRY(hipEventRecord(ws->ev[0], st));
  // Flagged sentences first go through the wave-cooperative kernel (the long
  // ones the wide / char kernels routed there, and any other it can take);
  // the general kernel gets what it leaves.
  const uint32_t *glist = fp->l.flagged, *gcount = status + spm_amd::kStFlagged;
  if (fp->coop) {
    spm_amd::CoopArgs ca{c.bytes, c.off, m->d_uvs.as<uint32_t>(), m->d_values.as<int32_t>(),
                         static_cast<uint32_t>(m->trie.units.size()), m->up,
                         fp->l.flagged, status + spm_amd::kStFlagged, 0, s2, s2l, ws->w_ntok.as<uint32_t>(),
                         ws->w_crest.as<uint32_t>(), status + spm_amd::kStCoopRest, ws->w_cpv.as<uint16_t>(),
                         ws->w_cnd.as<uint32_t>(), static_cast<uint32_t>(std::max(m->max_piece_bytes, 4)),
                         fp->l.chain, nullptr, fp->slab_chars};
    if (CoopQueue()) {
      ca.queue = status + spm_amd::kStCoopQueue;
      ca.part = ws->w_cpart.as<uint32_t>();
      ca.part_long = status + spm_amd::kStCoopLong;
      ca.part_n = n;
      SPM_HIP_TRY(spm_amd::LaunchCoopPartition(fp->l.flagged, status + spm_amd::kStFlagged, c.off, n,
                                               ws->w_cpart.as<uint32_t>(), status + spm_amd::kStCoopLong,
                                               status + spm_amd::kStCoopShort, st));
    }
    const uint64_t blocks = fp->coop_blocks;
    static const bool kProf = std::getenv("SPM_HIP_COOP_PROF") != nullptr;  // debug: phase cycles to stderr
    uint64_t *prof = nullptr;
    if (kProf) {
      SPM_HIP_TRY(spm_amd::DevMalloc(&prof, 64));
      SPM_HIP_TRY(hipMemsetAsync(prof, 0, 64, st));
      ca.prof = prof;
    }
    SPM_HIP_TRY(spm_amd::LaunchCoopEncode(ca, static_cast<uint32_t>(blocks), st));
    if (prof) {
      uint64_t h[8];
      SPM_HIP_TRY(hipMemcpyAsync(h, prof, 64, hipMemcpyDeviceToHost, st));
      SPM_HIP_TRY(hipStreamSynchronize(st));
      (void)spm_amd::DevFree(prof);
      std::fprintf(stderr, "coop prof: setup %llu lattice %llu viterbi %llu backtrace %llu ids %llu cycles; "
                   "bytes %llu chars %llu tokens %llu\n", (unsigned long long)h[0], (unsigned long long)h[1],
                   (unsigned long long)h[2], (unsigned long long)h[3], (unsigned long long)h[4],
                   (unsigned long long)h[5], (unsigned long long)h[6], (unsigned long long)h[7]);
    }
    glist = ws->w_crest.as<uint32_t>();
    gcount = status + spm_amd::kStCoopRest;
  }
  spm_amd::GeneralLaunch g1{glist, gcount, 0, ws->w_scratch.as<uint8_t>(), gp.slab,
                            gp.small_nb, gp.lanes, ovf, status + spm_amd::kStOverflow,
                            status + spm_amd::kStError, s2, s2l, ws->w_ntok.as<uint32_t>()};
  SPM_HIP_TRY(spm_amd::LaunchUnigramGeneral(fp->l, g1, st));
  spm_amd::GeneralLaunch g2{ovf, status + spm_amd::kStOverflow, 0, ws->w_scratch.as<uint8_t>(), gp.pool,
                            gp.big_nb, 1, nullptr, nullptr, status + spm_amd::kStError, s2, s2l,
                            ws->w_ntok.as<uint32_t>()};
  SPM_HIP_TRY(spm_amd::LaunchUnigramGeneral(fp->l, g2, st));
  if (fp->slot >= 0) SPM_HIP_TRY(hipEventRecord(ws->ev[1], st));
  spm_amd::FixupLaunch f{c.off, n, c.ids, c.len, c.tok, s2, s2l, ws->w_ntok.as<uint32_t>(),
                         ws->w_cnt.as<uint32_t>(), status, fp->desc + spm_amd::FastTiles(n), c.out_status};
  SPM_HIP_TRY(spm_amd::LaunchEncodeFixup(f, st));
  return SPM_OK;
}

int EncodeUnigramFast(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const spm_amd::EncodeCall &c) {
  if (c.n == 0) {
    SPM_HIP_TRY(hipMemsetAsync(c.tok, 0, sizeof(uint64_t), c.st));
    return SPM_OK;
  }
  FastPlan fp;
  int rc = FastSetup(m, ws, c, nullptr, &fp);
  if (rc == SPM_OK) rc = FastPartA(m, ws, c, &fp, true);
  if (rc == SPM_OK) rc = FastPartB(m, ws, c, &fp);
  return rc;
}

// General kernel over every sentence with host-sized scratch (models with
// pieces of >= 64 bytes, force_general, and the re-run after a device-path
// overflow): the reference lattice literally, then scan + compaction.
int EncodeUnigramAll(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const spm_amd::EncodeCall &c) {
  const uint64_t n = c.n, cap = std::max<uint64_t>(c.capacity, 1), nn = std::max<uint64_t>(n, 1);
  const hipStream_t st = c.st;
  uint32_t *status = nullptr;
  int rc = PrepareControl(ws, n, st, &status);
  if (rc != SPM_OK) return rc;
  const uint32_t max_nb = std::max<uint32_t>(c.max_nb, 1);
  const uint64_t slab = spm_amd::UnigramGeneralSlabBytes(max_nb, m->up.trie_results_size);
  uint64_t threads = std::min<uint64_t>(nn, 16384);
  while (threads > 64 && threads * slab > (4ull << 30)) threads /= 2;
  if (threads * slab > (16ull << 30)) return Fail(SPM_RESOURCE_EXHAUSTED, "sentence too long for the general encode path");
  SPM_HIP_TRY(ws->w_scratch.Reserve(threads * slab));
  SPM_HIP_TRY(ws->w_slot2_ids.Reserve(cap * 4));
  if (c.len) SPM_HIP_TRY(ws->w_slot2_len.Reserve(cap * 4));
  SPM_HIP_TRY(ws->w_ntok.Reserve(nn * 4));
  spm_amd::UnigramLaunch l = UnigramTables(m, c, status);
  int32_t *s2 = ws->w_slot2_ids.as<int32_t>();
  uint32_t *s2l = c.len ? ws->w_slot2_len.as<uint32_t>() : nullptr;
  const bool timing = TimedSlot(m, ws) >= 0;
  if (timing) SPM_HIP_TRY(hipEventRecord(ws->ev[0], st));
  spm_amd::GeneralLaunch g{nullptr, nullptr, n, ws->w_scratch.as<uint8_t>(), slab, max_nb,
                           static_cast<uint32_t>(threads), nullptr, nullptr, status + spm_amd::kStError, s2, s2l,
                           ws->w_ntok.as<uint32_t>()};
  SPM_HIP_TRY(spm_amd::LaunchUnigramGeneral(l, g, st));
  if (timing) SPM_HIP_TRY(hipEventRecord(ws->ev[1], st));
  size_t tmp = 0;
  SPM_HIP_TRY(spm_amd::LaunchCompact(c.off, n, ws->w_ntok.as<uint32_t>(), s2, s2l, c.ids, c.len, c.tok, nullptr,
                                     &tmp, status, c.out_status, st));
  SPM_HIP_TRY(ws->w_scan.Reserve(tmp + 16));
  SPM_HIP_TRY(spm_amd::LaunchCompact(c.off, n, ws->w_ntok.as<uint32_t>(), s2, s2l, c.ids, c.len, c.tok,
                                     ws->w_scan.ptr, &tmp, status, c.out_status, st));
  return SPM_OK;
}

bool NeedsHostSized(const spm_hip_model *m) {
  if (m->force_general) return true;
  if (m->model_type == spm_amd::kUnigram) return m->kernel == spm_amd::UnigramKernel::kGeneralOnly;
  return m->bpe.has_user_defined;
}

// Enqueues one encode (no synchronization unless c.host_sized).
int EncodeEnqueue(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const spm_amd::EncodeCall &c) {
  if (m->model_type == spm_amd::kUnigram)
    return c.host_sized ? EncodeUnigramAll(m, ws, c) : EncodeUnigramFast(m, ws, c);
  return spm_amd::EncodeBpe(m, ws, c, &g_last_error);
}

int LongestSentence(const uint64_t *d_off, uint64_t n, hipStream_t st, uint32_t *max_nb) {
  *max_nb = 0;
  if (n == 0) return SPM_OK;
  std::vector<uint64_t> off(n + 1);
  SPM_HIP_TRY(hipMemcpyAsync(off.data(), d_off, (n + 1) * 8, hipMemcpyDeviceToHost, st));
  SPM_HIP_TRY(hipStreamSynchronize(st));
  for (uint64_t i = 0; i < n; ++i) *max_nb = std::max<uint32_t>(*max_nb, static_cast<uint32_t>(off[i + 1] - off[i]));
  return SPM_OK;
}

// Blocking encode on a leased workspace (spm_hip_encode_batch and the host
// and SentencePieceText entry points): reads offsets[n], enqueues the
// encode, waits, and reports the status the reference's Encode would return.
// A flagged sentence too long for the device general pass (kStError) makes
// it re-run the batch with host-sized scratch.
int EncodeBlocking(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const uint8_t *d_bytes, const uint64_t *d_off,
                   uint64_t n, int32_t *d_ids, uint32_t *d_len, uint64_t *d_tok, hipStream_t st) {
  uint64_t total = 0;
  SPM_HIP_TRY(hipMemcpyAsync(ws->pinned + 8, d_off + n, 8, hipMemcpyDeviceToHost, st));
  SPM_HIP_TRY(hipStreamSynchronize(st));
  std::memcpy(&total, ws->pinned + 8, 8);
  if (total > 0xFFFFFFFFull * 4) return Fail(SPM_OUT_OF_RANGE, "batch too large");
  spm_amd::EncodeCall c{d_bytes, d_off, n, total, d_ids, d_len, d_tok, nullptr, st, NeedsHostSized(m), 0};
  if (c.host_sized) {
    int rc = LongestSentence(d_off, n, st, &c.max_nb);
    if (rc != SPM_OK) return rc;
  }
  ws->stats = spm_hip_encode_stats{};
  int rc = EncodeEnqueue(m, ws, c);
  if (rc != SPM_OK) return rc;
  SPM_HIP_TRY(hipMemcpyAsync(ws->pinned, ws->w_ctl.ptr, 4 * (spm_amd::kStCoopRest + 1), hipMemcpyDeviceToHost, st));
  SPM_HIP_TRY(hipStreamSynchronize(st));
  uint32_t flagged = ws->pinned[spm_amd::kStFlagged], err = ws->pinned[spm_amd::kStError];
  if (err && !c.host_sized) {
    c.host_sized = true;
    rc = LongestSentence(d_off, n, st, &c.max_nb);
    if (rc == SPM_OK) rc = EncodeEnqueue(m, ws, c);
    if (rc != SPM_OK) return rc;
    SPM_HIP_TRY(hipMemcpyAsync(ws->pinned, ws->w_ctl.ptr, 4 * (spm_amd::kStCoopRest + 1), hipMemcpyDeviceToHost,
                               st));
    SPM_HIP_TRY(hipStreamSynchronize(st));
    err = ws->pinned[spm_amd::kStError];
  }
  if (err) return Fail(SPM_INTERNAL, "general encode path: scratch overflow");
  ws->stats.sentences = n;
  ws->stats.general_path = c.host_sized ? n : flagged;
  ws->stats.coop_rest = c.host_sized ? 0 : ws->pinned[spm_amd::kStCoopRest];
  if (m->timing && ws->last_slot >= 0) {
    const int s = ws->last_slot;
    if (!c.host_sized) SPM_HIP_TRY(hipEventElapsedTime(&ws->stats.fast_kernel_ms, ws->tev[2 * s], ws->tev[2 * s + 1]));
    if (ws->stats.general_path) SPM_HIP_TRY(hipEventElapsedTime(&ws->stats.general_kernel_ms, ws->ev[0], ws->ev[1]));
    ws->tcount = 0;  // consumed here; the ring is for the asynchronous entry point
  }
  spm_amd::PublishStats(m, ws->stats);
  return SPM_OK;
}

// Lazy device tables of the normalizer (charsmap blob, user-defined trie).
int EnsureNormTables(spm_hip_model *m) {
  if (m->norm_ready) return SPM_OK;
  std::lock_guard<std::mutex> g(m->init_mu);
  if (m->norm_ready) return SPM_OK;
  const std::string &blob = m->proto.normalizer_spec.precompiled_charsmap;
  if (!blob.empty()) {
    uint32_t tsize = 0;
    if (blob.size() <= 4) return Fail(SPM_INTERNAL, "Blob for normalization rule is broken.");
    std::memcpy(&tsize, blob.data(), 4);
    if (tsize >= blob.size() || tsize < 4) return Fail(SPM_INTERNAL, "Blob for normalization rule is broken.");
    // The blob plus one NUL: a replacement string the blob leaves
    // unterminated ends there (NormalizePrefix's scan never leaves the copy).
    SPM_HIP_TRY(m->d_charsmap.Reserve(blob.size() + 1));
    SPM_HIP_TRY(hipMemcpy(m->d_charsmap.ptr, blob.data(), blob.size(), hipMemcpyHostToDevice));
    SPM_HIP_TRY(hipMemset(m->d_charsmap.as<uint8_t>() + blob.size(), 0, 1));
  }
  if (!m->user_defined.empty()) {
    std::vector<std::pair<std::string, int32_t>> keys;
    for (const auto &u : m->user_defined) keys.emplace_back(u, 1);
    spm_amd::DoubleArray da;
    std::string err;
    if (!spm_amd::BuildDoubleArray(keys, &da, &err)) return Fail(SPM_INTERNAL, err);
    SPM_HIP_TRY(Upload(&m->d_ud_units, da.units));
    m->ud_units_n = static_cast<uint32_t>(da.units.size());
  }
  m->norm_ready = true;
  return SPM_OK;
}

// Lazy per-piece type bits of the id epilogue.
int EnsureTypes(spm_hip_model *m) {
  if (m->types_ready) return SPM_OK;
  std::lock_guard<std::mutex> g(m->init_mu);
  if (m->types_ready) return SPM_OK;
  std::vector<uint8_t> types(m->proto.pieces.size());
  for (size_t i = 0; i < types.size(); ++i) {
    const int32_t t = m->proto.pieces[i].type;
    types[i] = (t == spm_amd::kUnknown ? spm_amd::kPieceUnknown : 0) |
               (t == spm_amd::kControl ? spm_amd::kPieceControl : 0);
  }
  SPM_HIP_TRY(Upload(&m->d_types, types));
  m->types_ready = true;
  return SPM_OK;
}

#define SPM_LEASE(lease, call)                                                          \
  do {                                                                                  \
    hipError_t _e = (call);                                                             \
    if (_e != hipSuccess)                                                               \
      return Fail(SPM_INTERNAL, std::string("workspace: ") + hipGetErrorString(_e));   \
  } while (0)

// The device normalizer's tables and switches of a model (after
// EnsureNormTables).
spm_amd::NormTables DeviceNormTables(const spm_hip_model *m) {
  const auto &ns = m->proto.normalizer_spec;
  spm_amd::NormTables t;
  if (!ns.precompiled_charsmap.empty()) {
    uint32_t tsize = 0;
    std::memcpy(&tsize, ns.precompiled_charsmap.data(), 4);
    t.units = reinterpret_cast<const uint32_t *>(m->d_charsmap.as<uint8_t>() + 4);
    t.num_units = tsize / 4;
    t.pool = m->d_charsmap.as<uint8_t>() + 4 + tsize;
    t.pool_size = static_cast<uint32_t>(ns.precompiled_charsmap.size() - 4 - tsize);
  }
  if (!m->user_defined.empty()) {
    t.ud_units = m->d_ud_units.as<uint32_t>();
    t.ud_num_units = m->ud_units_n;
  }
  t.add_dummy_prefix = ns.add_dummy_prefix;
  t.remove_extra_whitespaces = ns.remove_extra_whitespaces;
  t.escape_whitespaces = ns.escape_whitespaces;
  t.suffix = m->proto.trainer_spec.treat_whitespace_as_suffix;
  return t;
}

}  // namespace

namespace spm_amd {
// The unigram trainer E-step's forward pass through the byte kernel of a
// TrainerModel (spm_hip_model_from_pieces): see EStepForwardOut (kernels.h).
// ctl: kStWords zeroed status words (tile tickets); bp: back-pointer scratch
// of bytes_end + 16 bytes, indexed like the input.
bool EStepByteForwardOk(const spm_hip_model *m) {
  return m && m->kernel == UnigramKernel::kByte && m->ring_width == 16;
}
int EStepByteForward(spm_hip_model *m, const uint8_t *bytes, const uint64_t *off, uint64_t n, uint64_t bytes_end,
                     uint8_t *bp, uint32_t *ctl, const EStepForwardOut &e, hipStream_t st) {
  if (!EStepByteForwardOk(m)) return SPM_UNIMPLEMENTED;
  UnigramLaunch l{};
  l.bytes = bytes;
  l.off = off;
  l.n = n;
  l.capacity = bytes_end;
  l.units = m->d_uvs.as<uint32_t>();
  l.gen_units = m->d_units.as<uint32_t>();
  l.values = m->d_values.as<int32_t>();
  l.scores = m->d_scores.as<float>();
  l.num_units = static_cast<uint32_t>(m->trie.units.size());
  l.p = m->up;
  l.bp = bp;
  l.status = ctl;
  return LaunchUnigramEStepForward(l, e, st) == hipSuccess ? SPM_OK : SPM_INTERNAL;
}
}  // namespace spm_amd

namespace spm_amd {

// Ends the resident server (stop flag, then its stream drains: it sees the
// flag within one poll).
void EncodeWorkspace::StopService() {
  if (!svc_running) return;
  __atomic_store_n(&svc_box->stop, 1u, __ATOMIC_RELEASE);
  (void)hipStreamSynchronize(svc_stream);
  __atomic_store_n(&svc_box->stop, 0u, __ATOMIC_RELEASE);
  svc_running = false;
  static const bool kProf = std::getenv("SPM_HIP_SERVICE_PROF") != nullptr;  // debug
  if (kProf && svc_box->served) {
    int khz = 100000, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    const double us = 1000.0 / khz;
    std::fprintf(stderr, "service prof: %u requests, seen->copied %.2f us, seen->published %.2f us per request\n",
                 svc_box->served, svc_box->ticks_copy * us / svc_box->served, svc_box->ticks_busy * us / svc_box->served);
  }
  if (kProf && svc_prof) {
    uint64_t h[16];
    if (hipMemcpy(h, svc_prof, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess && h[13]) {
      int khz = 100000, dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
      const double n = static_cast<double>(h[13]), us = h[14] * (1000.0 / khz) / n;
      std::fprintf(stderr,
                   "raw call prof: %llu calls, %.2f us and %.0f shader cycles per call (%.0f MHz); cycles per call: "
                   "stage %.0f normalize %.0f encode %.0f (setup %.0f lattice %.0f viterbi %.0f backtrace %.0f ids "
                   "%.0f) unknown-merge %.0f outputs+publish %.0f; per call %.1f bytes %.1f chars %.1f tokens\n",
                   (unsigned long long)h[13], us, h[15] / n, h[15] / n / us, h[8] / n, h[9] / n, h[10] / n, h[0] / n,
                   h[1] / n, h[2] / n, h[3] / n, h[4] / n, h[11] / n, h[12] / n, h[5] / n, h[6] / n, h[7] / n);
    }
    (void)hipMemset(svc_prof, 0, 16 * 8);
  }
}

void EncodeWorkspace::Release() {
  StopService();
  if (svc_stream) (void)hipStreamDestroy(svc_stream);
  svc_stream = nullptr;
  if (svc_box) (void)hipHostFree(svc_box);
  svc_box = nullptr;
  if (svc_prof) (void)spm_amd::DevFree(svc_prof);
  svc_prof = nullptr;
  for (DevBuf *b : {&w_ctl, &w_slot_ids, &w_slot_len, &w_tprefix, &w_slot2_ids, &w_slot2_len, &w_ntok, &w_cnt, &w_bp, &w_flagged, &w_ovf, &w_scan,
                    &w_scratch, &w_rest, &w_nlen, &w_nscan, &w_ecount, &w_escan, &w_tids, &w_tlen, &w_ttok,
                    &h_in, &h_off, &h_ids, &h_len, &h_tok, &w_small, &w_bpn, &w_cpv, &w_cnd, &w_crest, &w_cpart})
    b->Release();
  if (pinned) (void)hipHostFree(pinned);
  pinned = nullptr;
  if (pin_small) (void)hipHostFree(pin_small);
  pin_small = nullptr;
  pin_small_cap = 0;
  for (auto &e : ev)
    if (e) (void)hipEventDestroy(e);
  for (auto &e : tev)
    if (e) (void)hipEventDestroy(e);
  if (own_stream) (void)hipStreamDestroy(own_stream);
  own_stream = nullptr;
}

static hipError_t NewWorkspace(bool own_stream, std::unique_ptr<EncodeWorkspace> *out) {
  auto ws = std::make_unique<EncodeWorkspace>();
  hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&ws->pinned), 64);
  if (e == hipSuccess && own_stream) e = hipStreamCreateWithFlags(&ws->own_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    ws->Release();
    return e;
  }
  *out = std::move(ws);
  return hipSuccess;
}

hipError_t WorkspaceLease::ForStream(spm_hip_model *m, hipStream_t st) {
  m_ = m;
  st_ = st;
  std::unique_ptr<EncodeWorkspace> evicted;
  {
    std::lock_guard<std::mutex> g(m->pool_mu);
    auto &slot = m->by_stream[st];
    if (!slot) {
      hipError_t e = NewWorkspace(false, &slot);
      if (e != hipSuccess) {
        m->by_stream.erase(st);
        return e;
      }
    }
    ws_ = slot.get();
    ws_->last_use = ++m->use_clock;
    // Leased under pool_mu: from here until this lease ends the workspace
    // is never an eviction victim, even before its mutex is taken below.
    ++ws_->leases;
    // Bound the pool: callers that create short-lived streams would
    // otherwise grow device memory without limit.  The least recently used
    // unleased workspace goes; its buffers are freed after pool_mu is
    // dropped (hipFree waits for the device work that still uses them, and
    // other threads' leases must not queue behind that).
    if (m->by_stream.size() > kMaxStreamWorkspaces) {
      auto victim = m->by_stream.end();
      for (auto it = m->by_stream.begin(); it != m->by_stream.end(); ++it) {
        if (it->second.get() == ws_ || it->second->leases != 0) continue;
        if (victim == m->by_stream.end() || it->second->last_use < victim->second->last_use) victim = it;
      }
      if (victim != m->by_stream.end()) {
        evicted = std::move(victim->second);
        m->by_stream.erase(victim);
      }
    }
  }
  if (evicted) evicted->Release();
  lock_ = std::unique_lock<std::mutex>(ws_->mu);
  return hipSuccess;
}

hipError_t WorkspaceLease::ForHost(spm_hip_model *m) {
  m_ = m;
  host_ = true;
  std::lock_guard<std::mutex> g(m->pool_mu);
  for (auto &w : m->host_pool)
    if (!w->busy) {
      ws_ = w.get();
      break;
    }
  if (!ws_) {
    std::unique_ptr<EncodeWorkspace> w;
    hipError_t e = NewWorkspace(true, &w);
    if (e != hipSuccess) return e;
    ws_ = w.get();
    m->host_pool.push_back(std::move(w));
  }
  ws_->busy = true;
  st_ = ws_->own_stream;
  return hipSuccess;
}

WorkspaceLease::~WorkspaceLease() {
  if (!ws_) return;
  if (lock_.owns_lock()) lock_.unlock();
  std::lock_guard<std::mutex> g(m_->pool_mu);
  if (host_) ws_->busy = false;
  else --ws_->leases;
}

void PublishStats(spm_hip_model *m, const spm_hip_encode_stats &s) {
  std::lock_guard<std::mutex> g(m->pool_mu);
  m->last_stats = s;
}

}  // namespace spm_amd

// list == nullptr in the general kernel means identity (all sentences).

extern "C" {

const char *spm_hip_last_error(void) { return g_last_error.c_str(); }

int spm_hip_device_bytes(uint64_t *live, uint64_t *peak) {
  if (!live && !peak) return SPM_INVALID_ARGUMENT;
  if (live) *live = spm_amd::DevLiveBytes();
  if (peak) *peak = spm_amd::DevPeakBytes();
  return SPM_OK;
}

void spm_hip_device_peak_reset(void) { spm_amd::DevPeakReset(); }

int spm_hip_estep_shard_plan(uint64_t n, int mode, int num_threads, int world, int rank,
                             uint64_t *segs, uint64_t capacity, uint64_t *num_segments) {
  if (!num_segments || (capacity && !segs) || world < 1 || rank < 0 || rank >= world ||
      (mode != SPM_ESTEP_FAST && mode != SPM_ESTEP_PARITY) || num_threads < 1)
    return SPM_INVALID_ARGUMENT;
  const auto plan = spm_amd::EStepShardPlan(n, mode == SPM_ESTEP_PARITY, num_threads, world, rank);
  *num_segments = plan.size();
  for (uint64_t k = 0; k < plan.size() && k < capacity; ++k) {
    segs[3 * k] = plan[k].index_base;
    segs[3 * k + 1] = plan[k].index_stride;
    segs[3 * k + 2] = plan[k].count;
  }
  return SPM_OK;
}

int spm_hip_estep_bucket_owner(int bucket, int num_threads, int world) {
  if (world < 1 || num_threads < 1 || bucket < 0 || bucket >= num_threads) return -1;
  return spm_amd::EStepBucketOwner(bucket, world);
}

static int LoadImpl(const void *model_proto, size_t len, spm_hip_model **out, bool host_only) {
  if (!out) return Fail(SPM_INVALID_ARGUMENT, "out is null");
  *out = nullptr;
  if (!model_proto && len) return Fail(SPM_INVALID_ARGUMENT, "model_proto is null");
  auto *m = new spm_hip_model();
  m->host_only = host_only;
  std::string err;
  if (!spm_amd::ParseModelProto(static_cast<const uint8_t *>(model_proto), len, &m->proto, &err)) {
    delete m;
    return Fail(SPM_INTERNAL, err);
  }
  m->model_type = m->proto.trainer_spec.model_type;
  int rc = InitializePieces(m);
  if (rc == SPM_OK && !host_only) {
    hipError_t e = hipGetDevice(&m->device);
    if (e != hipSuccess) rc = Fail(SPM_INTERNAL, std::string("hipGetDevice: ") + hipGetErrorString(e));
  }
  if (rc == SPM_OK) {
    if (m->model_type == spm_amd::kUnigram) rc = LoadUnigram(m);
    else if (m->model_type == spm_amd::kBpe) rc = spm_amd::LoadBpe(m, &g_last_error);
    else rc = Fail(SPM_UNIMPLEMENTED, "only unigram and bpe models run on the device");
  }
  if (rc != SPM_OK) {
    spm_hip_model_free(m);
    return rc;
  }
  *out = m;
  return SPM_OK;
}

int spm_hip_model_load(const void *model_proto, size_t len, spm_hip_model **out) {
  return LoadImpl(model_proto, len, out, false);
}

// TrainerModel::SetSentencePieces (unigram_model_trainer.cc:97-119): a unigram
// model over a bare piece list — every piece NORMAL with value = list index,
// no InitializePieces, so unk_id_ keeps its default 0 (model_interface.h:336)
// and UNK nodes carry id 0 with score min_score - 10.
int spm_hip_model_from_pieces(const uint8_t *piece_bytes, const uint64_t *piece_offsets,
                              const float *scores, uint64_t num_pieces, spm_hip_model **out) {
  if (!out) return Fail(SPM_INVALID_ARGUMENT, "out is null");
  *out = nullptr;
  if (!piece_offsets || !scores || (num_pieces && !piece_bytes) || num_pieces == 0)
    return Fail(SPM_INVALID_ARGUMENT, "empty piece list");
  auto *m = new spm_hip_model();
  m->model_type = spm_amd::kUnigram;
  m->proto.trainer_spec.model_type = spm_amd::kUnigram;
  m->proto.pieces.resize(num_pieces);
  int rc = SPM_OK;
  for (uint64_t i = 0; i < num_pieces && rc == SPM_OK; ++i) {
    auto &p = m->proto.pieces[i];
    p.piece.assign(reinterpret_cast<const char *>(piece_bytes) + piece_offsets[i],
                   piece_offsets[i + 1] - piece_offsets[i]);
    p.score = scores[i];
    p.type = spm_amd::kNormal;
    if (p.piece.empty() || !m->pieces.emplace(p.piece, static_cast<int32_t>(i)).second)
      rc = Fail(SPM_INTERNAL, "empty or duplicate piece");
  }
  m->unk_id = 0;
  if (rc == SPM_OK) {
    hipError_t e = hipGetDevice(&m->device);
    if (e != hipSuccess) rc = Fail(SPM_INTERNAL, std::string("HIP: ") + hipGetErrorString(e));
  }
  if (rc == SPM_OK) rc = LoadUnigram(m);
  if (rc != SPM_OK) {
    spm_hip_model_free(m);
    return rc;
  }
  *out = m;
  return SPM_OK;
}

int spm_hip_model_load_host_only(const void *model_proto, size_t len, spm_hip_model **out) {
  return LoadImpl(model_proto, len, out, true);
}

void spm_hip_model_free(spm_hip_model *m) {
  if (!m) return;
  for (spm_amd::DevBuf *b : {&m->d_units, &m->d_uvs, &m->d_values, &m->d_scores,
                             &m->bpe.pair_keys, &m->bpe.pair_vals, &m->bpe.pair_ent, &m->bpe.rank_piece, &m->bpe.entry_piece,
                             &m->bpe.entry_out, &m->bpe.piece_kind, &m->bpe.piece_out,
                             &m->d_charsmap, &m->d_ud_units, &m->d_types})
    b->Release();
  for (auto &kv : m->by_stream) kv.second->Release();
  for (auto &w : m->host_pool) w->Release();
  delete m;
}

int spm_hip_model_get_info(const spm_hip_model *m, spm_hip_model_info *info) {
  if (!m || !info) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  info->model_type = m->model_type;
  info->piece_size = static_cast<int32_t>(m->proto.pieces.size());
  info->unk_id = m->unk_id;
  info->max_piece_chars = m->max_piece_chars;
  info->trie_results_size = m->trie.max_prefix_matches;
  info->trie_units = static_cast<int32_t>(m->trie.units.size());
  info->min_score = m->min_score;
  info->max_score = m->max_score;
  info->ring_width = m->model_type == spm_amd::kUnigram ? m->ring_width : 0;
  info->fast_variant = m->model_type == spm_amd::kUnigram ? static_cast<int32_t>(m->kernel) : 0;
  return SPM_OK;
}

int spm_hip_model_trie_stats(const spm_hip_model *m, const uint8_t *bytes, const uint64_t *off,
                             uint64_t n, int num_threads, spm_hip_trie_stats *out) {
  if (!m || !off || !out || (n && !bytes)) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  if (m->model_type != spm_amd::kUnigram) return Fail(SPM_UNIMPLEMENTED, "unigram models only");
  const int T = num_threads > 0 ? num_threads : std::max(1u, std::thread::hardware_concurrency());
  std::vector<spm_hip_trie_stats> part(T);
  const std::vector<uint32_t> &units = m->trie.units;
  const uint32_t root = spm_amd::DoubleArray::Base(units[0]);
  // Walk depth (unit loads) of every byte position of sentence i; 0 where no
  // char starts.
  auto walk = [&](uint64_t i, spm_hip_trie_stats *s, std::vector<uint32_t> *dep) {
    const uint8_t *x = bytes + off[i];
    const uint64_t nb = off[i + 1] - off[i];
    dep->assign(nb + 1, 0);
    for (uint64_t p = 0; p < nb;) {
      ++s->char_starts;
      uint32_t base = root;
      uint32_t depth = 0;
      for (uint64_t q = p; q < nb; ++q) {
        const uint32_t c = x[q];
        const uint32_t node = base ^ c;
        ++s->unit_loads;
        ++depth;
        for (int k = 0; k < 8; ++k)
          if (node < (512u << k)) ++s->units_below[k];
        const uint32_t u = node < units.size() ? units[node] : 0u;
        if (c == 0 || spm_amd::DoubleArray::Label(u) != c) break;
        base = spm_amd::DoubleArray::Base(u);
        if (spm_amd::DoubleArray::Leaf(u)) ++s->leaf_loads;
      }
      (*dep)[p] = depth;
      s->max_depth = std::max<uint64_t>(s->max_depth, depth);
      p += std::min<uint64_t>(spm_amd::OneCharLen(x[p]), nb - p);
    }
  };
  const uint64_t nblocks = (n + 255) / 256;
  auto work = [&](int t) {
    spm_hip_trie_stats s{};
    std::vector<std::vector<uint32_t>> dep(256);
    std::vector<uint32_t> order(256);
    for (uint64_t blk = t; blk < nblocks; blk += T) {
      const uint64_t i0 = blk * 256, cnt = std::min<uint64_t>(256, n - i0);
      for (uint64_t k = 0; k < cnt; ++k) {
        walk(i0 + k, &s, &dep[k]);
        order[k] = static_cast<uint32_t>(k);
      }
      std::stable_sort(order.begin(), order.begin() + cnt, [&](uint32_t a, uint32_t b) {
        return std::min<uint64_t>(dep[a].size() - 1, 255) < std::min<uint64_t>(dep[b].size() - 1, 255);
      });
      for (uint64_t w0 = 0; w0 < cnt; w0 += 64) {
        const uint64_t w1 = std::min<uint64_t>(cnt, w0 + 64);
        ++s.waves;
        uint64_t maxlen = 0, dec = 0;
        for (uint64_t k = w0; k < w1; ++k) {
          const auto &d = dep[order[k]];
          maxlen = std::max<uint64_t>(maxlen, d.size() - 1);
          uint64_t tot = 0;
          for (uint32_t v : d) tot += v;
          dec = std::max(dec, (tot + 1) / 2);
        }
        s.decoupled_rounds += dec;
        for (uint64_t p = 0; p < maxlen; p += 2) {
          uint32_t r = 0;
          for (uint64_t k = w0; k < w1; ++k) {
            const auto &d = dep[order[k]];
            for (uint64_t q = p; q < p + 2 && q < d.size(); ++q) r = std::max(r, d[q]);
          }
          s.lockstep_rounds += r;
        }
      }
    }
    part[t] = s;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(work, t);
  for (auto &x : th) x.join();
  spm_hip_trie_stats r{};
  for (const auto &s : part) {
    r.char_starts += s.char_starts;
    r.unit_loads += s.unit_loads;
    r.leaf_loads += s.leaf_loads;
    r.max_depth = std::max(r.max_depth, s.max_depth);
    for (int k = 0; k < 8; ++k) r.units_below[k] += s.units_below[k];
    r.lockstep_rounds += s.lockstep_rounds;
    r.decoupled_rounds += s.decoupled_rounds;
    r.waves += s.waves;
  }
  *out = r;
  return SPM_OK;
}

int spm_hip_normalize_batch(const spm_hip_model *m, const uint8_t *in, const uint64_t *in_off,
                            uint64_t n, uint8_t *out, uint64_t *out_off, int num_threads) {
  if (!m || !in_off || !out_off || (n && (!in || !out))) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  spm_amd::PrefixMatcher matcher(m->user_defined);
  spm_amd::Normalizer norm(m->proto.normalizer_spec, m->proto.trainer_spec.treat_whitespace_as_suffix);
  if (!norm.ok()) return Fail(SPM_INTERNAL, norm.error());
  norm.SetPrefixMatcher(&matcher);
  int T = num_threads > 0 ? num_threads : static_cast<int>(std::thread::hardware_concurrency());
  T = std::max(1, std::min<int>(T, static_cast<int>(std::max<uint64_t>(n / 256, 1))));
  // Each thread normalizes a contiguous chunk into its own buffer.
  std::vector<std::string> bufs(T);
  std::vector<std::vector<uint64_t>> lens(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t]() {
      const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
      std::string s;
      std::vector<size_t> n2o;
      for (uint64_t i = lo; i < hi; ++i) {
        norm.Normalize(reinterpret_cast<const char *>(in) + in_off[i], in_off[i + 1] - in_off[i], &s, &n2o);
        bufs[t] += s;
        lens[t].push_back(s.size());
      }
    });
  for (auto &x : th) x.join();
  uint64_t w = 0;
  out_off[0] = 0;
  uint64_t i = 0;
  for (int t = 0; t < T; ++t) {
    std::memcpy(out + w, bufs[t].data(), bufs[t].size());
    for (uint64_t l : lens[t]) {
      w += l;
      out_off[++i] = w;
    }
  }
  return SPM_OK;
}

// Normalizer::Normalize on the device (normalize_kernels.hip).
namespace {

// Device Normalizer::Normalize on a leased workspace; d_n2o (optional)
// receives norm_to_orig (len + 1 entries per sentence at d_out_off[i] + i).
int NormalizeImpl(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const uint8_t *d_in,
                  const uint64_t *d_in_off, uint64_t n, uint8_t *d_out, uint64_t out_capacity,
                  uint64_t *d_out_off, uint64_t *total, uint32_t *d_n2o, hipStream_t st,
                  uint32_t *chain = nullptr) {
  int rc = EnsureNormTables(m);
  if (rc != SPM_OK) return rc;
  const spm_amd::NormTables t = DeviceNormTables(m);
  SPM_HIP_TRY(ws->w_nlen.Reserve(std::max<uint64_t>(n, 1) * sizeof(uint64_t)));
  SPM_HIP_TRY(spm_amd::NormalizeLengths(t, d_in, d_in_off, n, ws->w_nlen.as<uint64_t>(), st, chain));
  size_t tb = 0;
  SPM_HIP_TRY(spm_amd::LengthsToOffsets(ws->w_nlen.as<uint64_t>(), n, d_out_off, nullptr, &tb, st));
  SPM_HIP_TRY(ws->w_nscan.Reserve(std::max<size_t>(tb, 16)));
  SPM_HIP_TRY(spm_amd::LengthsToOffsets(ws->w_nlen.as<uint64_t>(), n, d_out_off, ws->w_nscan.ptr, &tb, st));
  if (chain) {  // asynchronous: the write pass checks the capacity itself
    if (!d_out && out_capacity) return Fail(SPM_INVALID_ARGUMENT, "null output");
    SPM_HIP_TRY(spm_amd::NormalizeWrite(t, d_in, d_in_off, n, d_out, d_out_off, st, d_n2o, out_capacity, chain));
    return SPM_OK;
  }
  SPM_HIP_TRY(hipMemcpyAsync(ws->pinned + 2, d_out_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  SPM_HIP_TRY(hipStreamSynchronize(st));
  uint64_t tot = 0;
  std::memcpy(&tot, ws->pinned + 2, sizeof(uint64_t));
  *total = tot;
  if (tot > out_capacity) return Fail(SPM_RESOURCE_EXHAUSTED, "normalized output exceeds out_capacity");
  if (tot > 0 && !d_out) return Fail(SPM_INVALID_ARGUMENT, "null output");
  SPM_HIP_TRY(spm_amd::NormalizeWrite(t, d_in, d_in_off, n, d_out, d_out_off, st, d_n2o));
  return SPM_OK;
}

}  // namespace

int spm_hip_normalize_batch_device(spm_hip_model *m, const uint8_t *d_in, const uint64_t *d_in_off,
                                   uint64_t n, uint8_t *d_out, uint64_t out_capacity,
                                   uint64_t *d_out_off, uint64_t *total, void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_normalize_batch_device");
  return spm_hip_normalize_batch_device_align(m, d_in, d_in_off, n, d_out, out_capacity, d_out_off,
                                              nullptr, total, stream);
}

int spm_hip_normalize_batch_device_align(spm_hip_model *m, const uint8_t *d_in, const uint64_t *d_in_off,
                                         uint64_t n, uint8_t *d_out, uint64_t out_capacity,
                                         uint64_t *d_out_off, uint32_t *d_norm_to_orig, uint64_t *total,
                                         void *stream) {
  if (!m || !d_in_off || !d_out_off || !total || (n && !d_in)) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  if (m->host_only) return Fail(SPM_FAILED_PRECONDITION, "host-only model handle");
  hipStream_t st = static_cast<hipStream_t>(stream);
  spm_amd::WorkspaceLease ws;
  SPM_LEASE(ws, ws.ForStream(m, st));
  return NormalizeImpl(m, ws.get(), d_in, d_in_off, n, d_out, out_capacity, d_out_off, total,
                       d_norm_to_orig, st);
}

int spm_hip_normalize_batch_device_async(spm_hip_model *m, const uint8_t *d_in, const uint64_t *d_in_off,
                                         uint64_t n, uint8_t *d_out, uint64_t out_capacity, uint64_t *d_out_off,
                                         uint32_t *d_norm_to_orig, uint32_t *d_status, void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_normalize_batch_device_async");
  if (!m || !d_in_off || !d_out_off || !d_status || (n && !d_in)) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  if (m->host_only) return Fail(SPM_FAILED_PRECONDITION, "host-only model handle");
  hipStream_t st = static_cast<hipStream_t>(stream);
  spm_amd::WorkspaceLease ws;
  SPM_LEASE(ws, ws.ForStream(m, st));
  return NormalizeImpl(m, ws.get(), d_in, d_in_off, n, d_out, out_capacity, d_out_off, nullptr, d_norm_to_orig,
                       st, d_status);
}

int spm_hip_model_set_force_general(spm_hip_model *m, int force) {
  if (!m) return Fail(SPM_INVALID_ARGUMENT, "null model");
  m->force_general = force != 0;
  return SPM_OK;
}

int spm_hip_model_set_timing(spm_hip_model *m, int enable) {
  if (!m) return Fail(SPM_INVALID_ARGUMENT, "null model");
  m->timing = enable != 0 && !m->host_only;  // events are created per workspace on first use
  return SPM_OK;
}

int spm_hip_model_last_stats(const spm_hip_model *m, spm_hip_encode_stats *s) {
  if (!m || !s) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  auto *mm = const_cast<spm_hip_model *>(m);
  std::lock_guard<std::mutex> g(mm->pool_mu);
  *s = m->last_stats;
  return SPM_OK;
}

int spm_hip_encode_batch(spm_hip_model *m, const uint8_t *d_bytes, const uint64_t *d_off,
                         uint64_t n, int32_t *d_ids, uint32_t *d_len, uint64_t *d_tok,
                         void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_encode_batch");
  if (!m || (!d_off) || (!d_tok) || (n && !d_ids))
    return Fail(SPM_INVALID_ARGUMENT, "null argument");
  if (m->host_only) return Fail(SPM_FAILED_PRECONDITION, "model was loaded host-only");
  if (n >= 0x7FFFFFFFull) return Fail(SPM_OUT_OF_RANGE, "too many sentences in one batch");
  hipStream_t st = static_cast<hipStream_t>(stream);
  spm_amd::WorkspaceLease ws;
  SPM_LEASE(ws, ws.ForStream(m, st));
  return EncodeBlocking(m, ws.get(), d_bytes, d_off, n, d_ids, d_len, d_tok, st);
}

int spm_hip_encode_batch_async(spm_hip_model *m, const uint8_t *d_bytes, const uint64_t *d_off, uint64_t n,
                               uint64_t capacity, int32_t *d_ids, uint32_t *d_len, uint64_t *d_tok,
                               uint32_t *d_status, void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_encode_batch_async");
  if (!m || (!d_off) || (!d_tok) || (n && !d_ids) || !d_status)
    return Fail(SPM_INVALID_ARGUMENT, "null argument");
  if (m->host_only) return Fail(SPM_FAILED_PRECONDITION, "model was loaded host-only");
  if (n >= 0x7FFFFFFFull) return Fail(SPM_OUT_OF_RANGE, "too many sentences in one batch");
  if (capacity > 0xFFFFFFFFull * 4) return Fail(SPM_OUT_OF_RANGE, "batch too large");
  hipStream_t st = static_cast<hipStream_t>(stream);
  spm_amd::WorkspaceLease ws;
  SPM_LEASE(ws, ws.ForStream(m, st));
  if (NeedsHostSized(m)) {
    // General kernel over every sentence: its scratch is sized from the
    // longest sentence, which needs the offsets on the host.  A chain that
    // already failed (e.g. a normalize that overflowed its capacity, whose
    // offsets then point past the caller's buffer) launches nothing: the
    // status word keeps its first error, as every kernel of the pure stream
    // path does.
    SPM_HIP_TRY(hipMemcpyAsync(ws->pinned, d_status, 4, hipMemcpyDeviceToHost, st));
    SPM_HIP_TRY(hipStreamSynchronize(st));
    if (ws->pinned[0] != 0) return SPM_OK;
    const int rc = EncodeBlocking(m, ws.get(), d_bytes, d_off, n, d_ids, d_len, d_tok, st);
    if (rc != SPM_OK) SPM_HIP_TRY(spm_amd::LaunchStatusSetFirst(d_status, static_cast<uint32_t>(rc), st));
    return rc;
  }
  spm_amd::EncodeCall c{d_bytes, d_off, n, capacity, d_ids, d_len, d_tok, d_status, st, false, 0};
  return EncodeEnqueue(m, ws.get(), c);
}

int spm_hip_model_drain_kernel_times(spm_hip_model *m, void *stream, float *ms, uint32_t capacity,
                                     uint32_t *count) {
  if (!m || !count || (capacity && !ms)) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  hipStream_t st = static_cast<hipStream_t>(stream);
  spm_amd::WorkspaceLease ws;
  SPM_LEASE(ws, ws.ForStream(m, st));
  SPM_HIP_TRY(hipStreamSynchronize(st));
  const uint32_t ring = spm_amd::EncodeWorkspace::kTimingRing;
  const uint32_t have = ws->tcount < ring ? ws->tcount : ring;
  const uint32_t first = ws->tcount - have;
  uint32_t k = 0;
  for (uint32_t j = 0; j < have && k < capacity; ++j) {
    const uint32_t slot = (first + j) % ring;
    SPM_HIP_TRY(hipEventElapsedTime(&ms[k], ws->tev[2 * slot], ws->tev[2 * slot + 1]));
    ++k;
  }
  *count = k;
  ws->tcount = 0;
  return SPM_OK;
}

int spm_hip_model_set_coop_min_nb(spm_hip_model *m, uint32_t min_nb) {
  if (!m) return Fail(SPM_INVALID_ARGUMENT, "null model");
  if (min_nb && (!m->d_uvs.ptr || m->max_piece_bytes > 56))
    return Fail(SPM_FAILED_PRECONDITION, "model has no cooperative-kernel tables or pieces over 56 bytes");
  m->coop_min_nb = min_nb;
  return SPM_OK;
}

int spm_hip_model_set_coop_slab(spm_hip_model *m, int mode, uint32_t slab_chars) {
  if (!m) return Fail(SPM_INVALID_ARGUMENT, "null model");
  if (mode < 0 || mode > 2) return Fail(SPM_INVALID_ARGUMENT, "coop slab mode must be 0, 1 or 2");
  m->coop_slab_mode = mode;
  m->coop_slab_chars = slab_chars ? slab_chars : static_cast<uint32_t>(spm_amd::kCoopSlabChars);
  return SPM_OK;
}

int spm_hip_model_set_debug_corrupt_bp(spm_hip_model *m, int64_t sentence) {
  if (!m) return Fail(SPM_INVALID_ARGUMENT, "null model");
  m->corrupt_bp = sentence < 0 ? ~0ull : static_cast<uint64_t>(sentence);
  return SPM_OK;
}

int spm_hip_model_release_stream(spm_hip_model *m, void *stream) {
  if (!m) return Fail(SPM_INVALID_ARGUMENT, "null model");
  std::unique_ptr<spm_amd::EncodeWorkspace> w;
  // A call still holding a lease on that stream's workspace finishes first
  // (it may not have taken the workspace mutex yet, so wait on the count).
  for (;;) {
    {
      std::lock_guard<std::mutex> g(m->pool_mu);
      auto it = m->by_stream.find(static_cast<hipStream_t>(stream));
      if (it == m->by_stream.end()) return SPM_OK;
      if (it->second->leases == 0) {
        w = std::move(it->second);
        m->by_stream.erase(it);
        break;
      }
    }
    std::this_thread::yield();
  }
  SPM_HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  w->Release();
  return SPM_OK;
}

int spm_hip_abi_version(void) { return SPM_HIP_ABI_VERSION; }

namespace {

// ParseExtraOptions (sentencepiece_processor.cc:981-1010) folded for the
// device epilogues: out = pre · (merged pieces, reversed?) · post.
int FoldExtras(spm_hip_model *m, const char *extra_options, spm_amd::EpilogueExtras *xo) {
  auto piece_to_id = [&](const std::string &s) -> int32_t {
    auto r = m->reserved.find(s);
    if (r != m->reserved.end()) return r->second;
    auto p = m->pieces.find(s);
    if (p != m->pieces.end()) return p->second;
    return m->unk_id;
  };
  // Fold the option list: out = pre · (mid, reversed?) · post.
  std::vector<int32_t> pre, post;
  bool reversed = false;
  const std::string opts = extra_options ? extra_options : "";
  size_t s0 = 0;
  while (s0 <= opts.size()) {
    const size_t e = std::min(opts.find(':', s0), opts.size());
    const std::string o = opts.substr(s0, e - s0);
    s0 = e + 1;
    if (o.empty()) continue;  // SplitPiece drops empty fields
    if (o == "bos" || o == "eos") {
      const std::string &piece = o == "bos" ? m->proto.trainer_spec.bos_piece : m->proto.trainer_spec.eos_piece;
      const int32_t id = piece_to_id(piece);
      if (id == m->unk_id) return Fail(SPM_INTERNAL, "id for `" + piece + "` is not defined.");
      if (o == "bos") pre.insert(pre.begin(), id);
      else post.push_back(id);
    } else if (o == "reverse") {
      std::vector<int32_t> np(post.rbegin(), post.rend()), nq(pre.rbegin(), pre.rend());
      pre.swap(np);
      post.swap(nq);
      reversed = !reversed;
    } else {
      return Fail(SPM_INTERNAL, "option \"" + o + "\" is not available.");
    }
  }
  if (pre.size() > static_cast<size_t>(spm_amd::kMaxExtras) || post.size() > static_cast<size_t>(spm_amd::kMaxExtras))
    return Fail(SPM_OUT_OF_RANGE, "too many bos/eos extra options");
  spm_amd::EpilogueExtras &x = *xo;
  x = spm_amd::EpilogueExtras{};
  for (size_t k = 0; k < pre.size(); ++k) x.ids[k] = pre[k];
  for (size_t k = 0; k < post.size(); ++k) x.ids[spm_amd::kMaxExtras + k] = post[k];
  x.num_pre = static_cast<uint32_t>(pre.size());
  x.num_post = static_cast<uint32_t>(post.size());
  x.reversed = reversed ? 1u : 0u;
  return SPM_OK;
}

}  // namespace

// PopulateSentencePieceText's id part + ApplyExtraOptions on the device
// (epilogue_kernels.hip).  Option parsing follows ParseExtraOptions
// (sentencepiece_processor.cc:981-1010).
static int FinalizeImpl(spm_hip_model *m, const char *extra_options, const int32_t *d_ids,
                        const uint64_t *d_tok_off, uint64_t n, int32_t *d_out_ids, uint64_t out_capacity,
                        uint64_t *d_out_off, uint64_t *total, uint32_t *chain, hipStream_t st) {
  if (m->host_only) return Fail(SPM_FAILED_PRECONDITION, "model was loaded host-only");
  spm_amd::EpilogueExtras x{};
  {
    const int rc0 = FoldExtras(m, extra_options, &x);
    if (rc0 != SPM_OK) return rc0;
  }
  int rc = EnsureTypes(m);
  if (rc != SPM_OK) return rc;
  const int32_t num_types = static_cast<int32_t>(m->proto.pieces.size());
  if (n == 0) {
    SPM_HIP_TRY(hipMemsetAsync(d_out_off, 0, sizeof(uint64_t), st));
    if (total) *total = 0;
    return SPM_OK;
  }
  if (!d_ids) return Fail(SPM_INVALID_ARGUMENT, "null ids");
  spm_amd::WorkspaceLease ws;
  SPM_LEASE(ws, ws.ForStream(m, st));
  SPM_HIP_TRY(ws->w_ecount.Reserve(n * sizeof(uint64_t)));
  SPM_HIP_TRY(spm_amd::LaunchEpilogueCount(d_ids, d_tok_off, n, m->d_types.as<uint8_t>(), num_types,
                                            x.num_pre + x.num_post, ws->w_ecount.as<uint64_t>(), st, chain));
  size_t tb = 0;
  SPM_HIP_TRY(spm_amd::LengthsToOffsets(ws->w_ecount.as<uint64_t>(), n, d_out_off, nullptr, &tb, st));
  SPM_HIP_TRY(ws->w_escan.Reserve(std::max<size_t>(tb, 16)));
  SPM_HIP_TRY(spm_amd::LengthsToOffsets(ws->w_ecount.as<uint64_t>(), n, d_out_off, ws->w_escan.ptr, &tb, st));
  if (chain) {  // asynchronous: the write pass checks the capacity itself
    if (!d_out_ids && out_capacity) return Fail(SPM_INVALID_ARGUMENT, "null output");
    SPM_HIP_TRY(spm_amd::LaunchEpilogueWrite(d_ids, d_tok_off, n, m->d_types.as<uint8_t>(), num_types, x,
                                              d_out_off, d_out_ids, st, out_capacity, chain));
    return SPM_OK;
  }
  SPM_HIP_TRY(hipMemcpyAsync(ws->pinned + 12, d_out_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  SPM_HIP_TRY(hipStreamSynchronize(st));
  uint64_t tot = 0;
  std::memcpy(&tot, ws->pinned + 12, sizeof(uint64_t));
  if (total) *total = tot;
  if (tot > out_capacity) return Fail(SPM_RESOURCE_EXHAUSTED, "finalized ids exceed out_capacity");
  if (tot > 0 && !d_out_ids) return Fail(SPM_INVALID_ARGUMENT, "null output");
  SPM_HIP_TRY(spm_amd::LaunchEpilogueWrite(d_ids, d_tok_off, n, m->d_types.as<uint8_t>(), num_types, x,
                                            d_out_off, d_out_ids, st));
  return SPM_OK;
}

// PopulateSentencePieceText's id part + ApplyExtraOptions on the device
// (epilogue_kernels.hip).  Option parsing follows ParseExtraOptions
// (sentencepiece_processor.cc:981-1010).
int spm_hip_finalize_ids(spm_hip_model *m, const char *extra_options, const int32_t *d_ids,
                         const uint64_t *d_tok_off, uint64_t n, int32_t *d_out_ids,
                         uint64_t out_capacity, uint64_t *d_out_off, uint64_t *total, void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_finalize_ids");
  if (!m || !d_tok_off || !d_out_off) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  return FinalizeImpl(m, extra_options, d_ids, d_tok_off, n, d_out_ids, out_capacity, d_out_off, total, nullptr,
                      static_cast<hipStream_t>(stream));
}

int spm_hip_finalize_ids_async(spm_hip_model *m, const char *extra_options, const int32_t *d_ids,
                               const uint64_t *d_tok_off, uint64_t n, int32_t *d_out_ids, uint64_t out_capacity,
                               uint64_t *d_out_off, uint32_t *d_status, void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_finalize_ids_async");
  if (!m || !d_tok_off || !d_out_off || !d_status) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  return FinalizeImpl(m, extra_options, d_ids, d_tok_off, n, d_out_ids, out_capacity, d_out_off, nullptr, d_status,
                      static_cast<hipStream_t>(stream));
}

// Host buffers: a pooled workspace with a private stream, so concurrent host
// calls on one handle run side by side.
// SentencePieceProcessor::Encode(input, SentencePieceText*) (sentencepiece_
// processor.cc:553-575) on the device: one workspace lease for the whole
// pipeline (normalize + norm_to_orig, Encode, SentencePieceText epilogue).
int spm_hip_encode_spt(spm_hip_model *m, const char *extra_options, const uint8_t *d_raw,
                       const uint64_t *d_raw_off, uint64_t n, uint8_t *d_norm, uint64_t norm_capacity,
                       uint64_t *d_norm_off, uint32_t *d_n2o, spm_hip_piece *d_pieces,
                       uint64_t piece_capacity, uint64_t *d_piece_off, uint64_t *total_norm,
                       uint64_t *total_pieces, void *stream) {
  spm_amd::TraceRange trace_range_("spm_hip_encode_spt");
  if (!m || !d_raw_off || !d_norm_off || !d_piece_off || !total_norm || !total_pieces || (n && !d_raw))
    return Fail(SPM_INVALID_ARGUMENT, "null argument");
  if (m->host_only) return Fail(SPM_FAILED_PRECONDITION, "model was loaded host-only");
  if (n >= 0x7FFFFFFFull) return Fail(SPM_OUT_OF_RANGE, "too many sentences in one batch");
  *total_norm = *total_pieces = 0;
  spm_amd::EpilogueExtras x{};
  int rc = FoldExtras(m, extra_options, &x);
  if (rc != SPM_OK) return rc;
  rc = EnsureTypes(m);
  if (rc != SPM_OK) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  spm_amd::WorkspaceLease ws;
  SPM_LEASE(ws, ws.ForStream(m, st));
  if (n == 0) {
    SPM_HIP_TRY(hipMemsetAsync(d_norm_off, 0, sizeof(uint64_t), st));
    SPM_HIP_TRY(hipMemsetAsync(d_piece_off, 0, sizeof(uint64_t), st));
    return SPM_OK;
  }
  if (!d_n2o) return Fail(SPM_INVALID_ARGUMENT, "null norm_to_orig");
  rc = NormalizeImpl(m, ws.get(), d_raw, d_raw_off, n, d_norm, norm_capacity, d_norm_off, total_norm, d_n2o, st);
  if (rc != SPM_OK) return rc;
  const uint64_t tn = *total_norm;
  SPM_HIP_TRY(ws->w_tids.Reserve(std::max<uint64_t>(tn, 1) * 4));
  SPM_HIP_TRY(ws->w_tlen.Reserve(std::max<uint64_t>(tn, 1) * 4));
  SPM_HIP_TRY(ws->w_ttok.Reserve((n + 1) * 8));
  rc = EncodeBlocking(m, ws.get(), d_norm, d_norm_off, n, ws->w_tids.as<int32_t>(), ws->w_tlen.as<uint32_t>(),
                  ws->w_ttok.as<uint64_t>(), st);
  if (rc != SPM_OK) return rc;
  const int32_t num_types = static_cast<int32_t>(m->proto.pieces.size());
  SPM_HIP_TRY(ws->w_ecount.Reserve(n * sizeof(uint64_t)));
  SPM_HIP_TRY(spm_amd::LaunchEpilogueCount(ws->w_tids.as<int32_t>(), ws->w_ttok.as<uint64_t>(), n,
                                            m->d_types.as<uint8_t>(), num_types, x.num_pre + x.num_post,
                                            ws->w_ecount.as<uint64_t>(), st));
  size_t tb = 0;
  SPM_HIP_TRY(spm_amd::LengthsToOffsets(ws->w_ecount.as<uint64_t>(), n, d_piece_off, nullptr, &tb, st));
  SPM_HIP_TRY(ws->w_escan.Reserve(std::max<size_t>(tb, 16)));
  SPM_HIP_TRY(spm_amd::LengthsToOffsets(ws->w_ecount.as<uint64_t>(), n, d_piece_off, ws->w_escan.ptr, &tb, st));
  SPM_HIP_TRY(hipMemcpyAsync(ws->pinned + 12, d_piece_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  SPM_HIP_TRY(hipStreamSynchronize(st));
  uint64_t tot = 0;
  std::memcpy(&tot, ws->pinned + 12, sizeof(uint64_t));
  *total_pieces = tot;
  if (tot > piece_capacity) return Fail(SPM_RESOURCE_EXHAUSTED, "pieces exceed piece_capacity");
  if (tot > 0 && !d_pieces) return Fail(SPM_INVALID_ARGUMENT, "null pieces output");
  SPM_HIP_TRY(spm_amd::LaunchSptWrite(ws->w_tids.as<int32_t>(), ws->w_tlen.as<uint32_t>(),
                                       ws->w_ttok.as<uint64_t>(), n, m->d_types.as<uint8_t>(), num_types, x,
                                       d_n2o, d_norm_off, d_piece_off, d_pieces, st));
  return SPM_OK;
}

namespace {

constexpr uint64_t kSmallMaxSentences = 256;    // one fast-kernel tile
constexpr uint64_t kSmallMaxBytes = 1ull << 20;  // pinned staging bound

inline uint64_t Align256(uint64_t x) { return (x + 255) & ~255ull; }

// Host API, small batches (one fast-kernel tile: n <= 256; unigram fast
// kernels; offsets start at 0).  The reference calls Encode once per line
// (spm_encode_main.cc:189-191, model_interface.h:117); the blocking path
// costs that four synchronizations, pageable copies and a dozen launches.
// Here the zeroed control block, the offsets and the bytes go up in ONE copy
// from pinned staging; the fast kernel's single tile starts at byte 0, so
// its slots are the final ids / lengths / token offsets (no tile
// compaction); the status words and the outputs come back with one
// synchronization.  Only a batch the fast kernel flagged runs the general
// kernel and the fix-up chain, with a second round trip.  *done = false:
// the caller takes the general blocking path (a device-path overflow).
// Host API, very small batches (n <= kCoopSmallMax, unigram models with the
// cooperative kernel's tables): ONE launch of coop_small_kernel, one block
// whose waves encode a sentence each (its trie walks 64 at a time, the
// latency a one-sentence call is made of), with the input read from and the
// outputs written to pinned host memory and completion polled on a host
// word.  *done = false: the caller takes the lane-kernel small path.
// Raw lines -> final ids of Encode(line, &ids) without extra options, in one
// launch (coop_raw_kernel): the raw image goes up through pinned coherent
// memory, ids and offsets come back there, the host polls the completion
// word.  *done = false: a line the fused path does not take (general-kernel
// lattice, a line past kRawMaxBytes, an output past its capacity).
// The resident small-call server (coop_service_kernel, CoopServiceBox):
// on by default; SPM_HIP_SERVICE=0 launches one kernel per call instead.
// SPM_HIP_SERVICE_IDLE_US: wall-clock microseconds without a request after
// which the server exits (default 2000; the next call relaunches it).  While
// it runs it holds one CU and its stream's hardware queue.
bool ServiceOn() {
  static const bool on = [] {
    const char *e = std::getenv("SPM_HIP_SERVICE");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

uint64_t ServiceIdleTicks() {
  static const uint64_t ticks = [] {
    int khz = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) !=
                                                  hipSuccess || khz <= 0)
      khz = 100000;  // 100 MHz
    const char *e = std::getenv("SPM_HIP_SERVICE_IDLE_US");
    const uint64_t us = e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : 2000;
    return static_cast<uint64_t>(khz) * us / 1000;
  }();
  return ticks;
}

// One small call through the server (kind 1: normalized batch with `sa`,
// 2: raw lines with `ra`), or, with the server off, one launch on `st`; then
// the poll of host_pub[0] == c.pub_seq.  A server that has exited meanwhile
// (idle timeout before it saw the request) is relaunched to serve it.
int RunSmallCall(spm_amd::EncodeWorkspace *ws, int kind, const spm_amd::CoopSmallArgs *sa,
                 const spm_amd::CoopRawArgs *ra, const spm_amd::CoopCall &c, hipStream_t st, const char *what) {
  volatile uint32_t *pub = c.host_pub;
  const bool svc = ServiceOn();
  hipStream_t wait_st = st;
  uint32_t prev = 0;
  auto launch = [&](uint32_t last) -> hipError_t {
    ws->svc_args.box = ws->svc_box;
    ws->svc_args.last = last;
    ws->svc_args.idle_ticks = ServiceIdleTicks();
    hipError_t e = spm_amd::LaunchCoopService(ws->svc_args, ws->svc_stream);
    if (e == hipSuccess) ws->svc_running = true;
    return e;
  };
  if (svc) {
    if (!ws->svc_stream) SPM_HIP_TRY(hipStreamCreateWithFlags(&ws->svc_stream, hipStreamNonBlocking));
    if (!ws->svc_box) {
      SPM_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&ws->svc_box), sizeof(spm_amd::CoopServiceBox),
                                hipHostMallocCoherent));
      std::memset(ws->svc_box, 0, sizeof(spm_amd::CoopServiceBox));
    }
    if (ws->svc_running && hipStreamQuery(ws->svc_stream) == hipSuccess) ws->svc_running = false;  // idled out
    // The call's tables are a function of the workspace buffers (and the
    // model): a server launched with other buffers is restarted.
    const void *key[6] = {ws->w_small.ptr, ws->w_slot2_ids.ptr, ws->w_slot2_len.ptr, ws->w_cpv.ptr, ws->w_cnd.ptr,
                          ws->pin_small};
    const bool same = std::memcmp(ws->svc_key[kind - 1], key, sizeof(key)) == 0;
    if (ws->svc_running && !same) ws->StopService();
    std::memcpy(ws->svc_key[kind - 1], key, sizeof(key));
    if (kind == 1) ws->svc_args.small = *sa;
    else ws->svc_args.raw = *ra;
    prev = __atomic_load_n(&ws->svc_box->seq, __ATOMIC_ACQUIRE);
    if (!ws->svc_running) SPM_HIP_TRY(launch(prev));
    std::memcpy(const_cast<spm_amd::CoopCall *>(&ws->svc_box->call), &c, sizeof(c));
    __atomic_store_n(&ws->svc_box->seq, (c.pub_seq & 0x3FFFFFFFu) | static_cast<uint32_t>(kind) << 30,
                     __ATOMIC_RELEASE);
    wait_st = ws->svc_stream;
  } else if (kind == 1) {
    SPM_HIP_TRY(spm_amd::LaunchCoopSmall(*sa, c, st));
  } else {
    SPM_HIP_TRY(spm_amd::LaunchCoopRaw(*ra, c, st));
  }
  bool published = false, relaunched = false;
  for (uint32_t spin = 1;; ++spin) {
    if (pub[0] == c.pub_seq) {
      published = true;
      break;
    }
    if ((spin & 1023) == 0) {
      const hipError_t q = hipStreamQuery(wait_st);
      if (q == hipSuccess) {
        if (pub[0] == c.pub_seq) {
          published = true;
          break;
        }
        if (!svc || relaunched) break;
        // The server exited (idle) before it saw this request: serve it.
        ws->svc_running = false;
        relaunched = true;
        SPM_HIP_TRY(launch(prev));
        continue;
      }
      if (q != hipErrorNotReady) {
        (void)hipStreamSynchronize(wait_st);
        ws->svc_running = false;
        return Fail(SPM_INTERNAL, std::string("HIP: ") + hipGetErrorString(q));
      }
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  if (!published) return Fail(SPM_INTERNAL, std::string(what) + " ended without publishing");
  return SPM_OK;
}

int EncodeRawCoop(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const uint8_t *raw, const uint64_t *raw_off,
                  uint64_t n, int32_t *ids, uint64_t ids_cap, uint64_t *out_off, hipStream_t st, bool *done) {
  *done = false;
  const uint64_t total = raw_off[n];
  const uint64_t ncap = 4 * total + 8 * n + 64;
  const uint64_t o_raw = Align256((n + 1) * 8), in_end = o_raw + total;
  const uint64_t o_out = Align256(in_end + 16), o_ids = Align256(o_out + (n + 1) * 8);
  const uint64_t o_pub = Align256(o_ids + ncap * 4), pin_end = o_pub + 256;
  // Buffers that grow are reallocated: not under a running server.
  if (ws->w_small.cap < in_end + 16 || ws->w_slot2_len.cap < ncap || ws->w_slot2_ids.cap < ncap * 4 ||
      ws->w_cpv.cap < (ncap + 64) * spm_amd::kCoopSlots * 2 || ws->w_cnd.cap < (ncap + 64) * spm_amd::kCoopSlots * 4 ||
      ws->pin_small_cap < pin_end)
    ws->StopService();
  SPM_HIP_TRY(ws->w_small.Reserve(in_end + 16));
  SPM_HIP_TRY(ws->w_slot2_len.Reserve(ncap));  // normalized bytes
  SPM_HIP_TRY(ws->w_slot2_ids.Reserve(ncap * 4));
  SPM_HIP_TRY(ws->w_cpv.Reserve((ncap + 64) * spm_amd::kCoopSlots * 2));
  SPM_HIP_TRY(ws->w_cnd.Reserve((ncap + 64) * spm_amd::kCoopSlots * 4));
  if (ws->pin_small_cap < pin_end) {
    if (ws->pin_small) SPM_HIP_TRY(hipHostFree(ws->pin_small));
    ws->pin_small = nullptr;
    ws->pin_small_cap = 0;
    const size_t want = std::max<uint64_t>(pin_end, 64 << 10);
    SPM_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&ws->pin_small), want, hipHostMallocCoherent));
    ws->pin_small_cap = want;
  }
  uint8_t *h = ws->pin_small;
  uint8_t *d = ws->w_small.as<uint8_t>();
  std::memcpy(h, raw_off, (n + 1) * 8);
  if (total) std::memcpy(h + o_raw, raw, total);
  volatile uint32_t *pub = reinterpret_cast<volatile uint32_t *>(h + o_pub);
  pub[0] = 0;
  if ((++ws->pub_seq & 0x3FFFFFFFu) == 0) ++ws->pub_seq;
  const uint32_t seq = ws->pub_seq & 0x3FFFFFFFu;
  spm_amd::CoopArgs a{ws->w_slot2_len.as<uint8_t>(), nullptr, m->d_uvs.as<uint32_t>(),
                      m->d_values.as<int32_t>(), static_cast<uint32_t>(m->trie.units.size()), m->up,
                      nullptr, nullptr, 0, ws->w_slot2_ids.as<int32_t>(), nullptr, nullptr, nullptr, nullptr,
                      ws->w_cpv.as<uint16_t>(), ws->w_cnd.as<uint32_t>(),
                      static_cast<uint32_t>(std::max(m->max_piece_bytes, 4)), nullptr};
  static const bool kSvcProf = std::getenv("SPM_HIP_SERVICE_PROF") != nullptr;  // debug: phase cycles at stop
  if (kSvcProf) {
    if (!ws->svc_prof) {
      SPM_HIP_TRY(spm_amd::DevMalloc(&ws->svc_prof, 16 * 8));
      SPM_HIP_TRY(hipMemset(ws->svc_prof, 0, 16 * 8));
    }
    a.prof = ws->svc_prof;
  }
  spm_amd::CoopRawArgs ra{a,
                          DeviceNormTables(m),
                          reinterpret_cast<const uint32_t *>(h),
                          reinterpret_cast<uint32_t *>(d),
                          m->d_types.as<uint8_t>(),
                          static_cast<int32_t>(m->proto.pieces.size())};
  spm_amd::CoopCall c{};
  c.n = static_cast<uint32_t>(n);
  c.stage_words = static_cast<uint32_t>((in_end + 3) / 4);
  c.pub_seq = seq;
  c.in_at = o_raw;
  c.ids_cap = ncap;
  c.tok = reinterpret_cast<uint64_t *>(h + o_out);
  c.ids = reinterpret_cast<int32_t *>(h + o_ids);
  c.host_pub = reinterpret_cast<uint32_t *>(h + o_pub);
  const int rc = RunSmallCall(ws, 2, nullptr, &ra, c, st, "raw-line encode");
  if (rc != SPM_OK) return rc;
  if (pub[1] != 0) {  // not taken
    ws->StopService();  // the caller's fallback may share the server's hardware queue
    return SPM_OK;
  }
  std::memcpy(out_off, h + o_out, (n + 1) * 8);
  const uint64_t nt = out_off[n];
  if (nt > ids_cap) return Fail(SPM_RESOURCE_EXHAUSTED, "ids exceed ids_cap");
  if (nt) std::memcpy(ids, h + o_ids, nt * 4);
  *done = true;
  return SPM_OK;
}

int EncodeHostCoop(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const uint8_t *bytes, const uint64_t *off,
                   uint64_t n, int32_t *ids, uint32_t *len, uint64_t *tok, hipStream_t st, bool *done) {
  *done = false;
  const uint64_t total = off[n], cap = std::max<uint64_t>(total, 1);
  const uint64_t o_in = Align256((n + 1) * 8), in_end = o_in + total;
  const uint64_t o_tok = Align256(in_end + 16), o_ids = Align256(o_tok + (n + 1) * 8);
  const uint64_t o_len = Align256(o_ids + cap * 4);
  const uint64_t o_pub = Align256(o_len + cap * 4), pin_end = o_pub + 256;
  // Slots, lengths and scratch rows are indexed by the staged byte offset
  // (o_in + off[i]); buffers that grow are reallocated: not under a server.
  const uint64_t slots = in_end + 16;
  if (ws->w_small.cap < in_end + 16 || ws->w_slot2_ids.cap < slots * 4 || ws->w_slot2_len.cap < slots * 4 ||
      ws->w_cpv.cap < (slots + 64) * spm_amd::kCoopSlots * 2 ||
      ws->w_cnd.cap < (slots + 64) * spm_amd::kCoopSlots * 4 || ws->pin_small_cap < pin_end)
    ws->StopService();
  SPM_HIP_TRY(ws->w_small.Reserve(in_end + 16));
  SPM_HIP_TRY(ws->w_slot2_ids.Reserve(slots * 4));
  SPM_HIP_TRY(ws->w_slot2_len.Reserve(slots * 4));
  SPM_HIP_TRY(ws->w_cpv.Reserve((slots + 64) * spm_amd::kCoopSlots * 2));
  SPM_HIP_TRY(ws->w_cnd.Reserve((slots + 64) * spm_amd::kCoopSlots * 4));
  if (ws->pin_small_cap < pin_end) {
    if (ws->pin_small) SPM_HIP_TRY(hipHostFree(ws->pin_small));
    ws->pin_small = nullptr;
    ws->pin_small_cap = 0;
    const size_t want = std::max<uint64_t>(pin_end, 64 << 10);
    SPM_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&ws->pin_small), want, hipHostMallocCoherent));
    ws->pin_small_cap = want;
  }
  uint8_t *h = ws->pin_small;
  uint8_t *d = ws->w_small.as<uint8_t>();
  std::memcpy(h, off, (n + 1) * 8);
  if (total) std::memcpy(h + o_in, bytes, total);
  volatile uint32_t *pub = reinterpret_cast<volatile uint32_t *>(h + o_pub);
  pub[0] = 0;
  if ((++ws->pub_seq & 0x3FFFFFFFu) == 0) ++ws->pub_seq;
  const uint32_t seq = ws->pub_seq & 0x3FFFFFFFu;
  spm_amd::CoopArgs a{d, reinterpret_cast<const uint64_t *>(d), m->d_uvs.as<uint32_t>(),
                      m->d_values.as<int32_t>(), static_cast<uint32_t>(m->trie.units.size()), m->up,
                      nullptr, nullptr, 0, ws->w_slot2_ids.as<int32_t>(), ws->w_slot2_len.as<uint32_t>(),
                      nullptr, nullptr, nullptr, ws->w_cpv.as<uint16_t>(), ws->w_cnd.as<uint32_t>(),
                      static_cast<uint32_t>(std::max(m->max_piece_bytes, 4)), nullptr};
  spm_amd::CoopSmallArgs sa{a, reinterpret_cast<const uint32_t *>(h), reinterpret_cast<uint32_t *>(d)};
  spm_amd::CoopCall c{};
  c.n = static_cast<uint32_t>(n);
  c.stage_words = static_cast<uint32_t>((in_end + 3) / 4);
  c.pub_seq = seq;
  c.in_at = o_in;
  c.tok = reinterpret_cast<uint64_t *>(h + o_tok);
  c.ids = reinterpret_cast<int32_t *>(h + o_ids);
  c.len = len ? reinterpret_cast<uint32_t *>(h + o_len) : nullptr;
  c.host_pub = reinterpret_cast<uint32_t *>(h + o_pub);
  // SPM_HIP_COOP_PROF (debug): phase cycles of this call to stderr (one
  // launch on `st`, not through the server).
  static const bool kProf = std::getenv("SPM_HIP_COOP_PROF") != nullptr;
  if (kProf) {
    uint64_t *prof = nullptr;
    SPM_HIP_TRY(spm_amd::DevMalloc(&prof, 64));
    SPM_HIP_TRY(hipMemsetAsync(prof, 0, 64, st));
    spm_amd::CoopSmallArgs sp = sa;
    sp.a.prof = prof;
    SPM_HIP_TRY(spm_amd::LaunchCoopSmall(sp, c, st));
    uint64_t hp[8];
    SPM_HIP_TRY(hipMemcpyAsync(hp, prof, 64, hipMemcpyDeviceToHost, st));
    SPM_HIP_TRY(hipStreamSynchronize(st));
    (void)spm_amd::DevFree(prof);
    std::fprintf(stderr, "coop prof: setup %llu lattice %llu viterbi %llu backtrace %llu ids %llu cycles; "
                 "bytes %llu chars %llu tokens %llu\n", (unsigned long long)hp[0], (unsigned long long)hp[1],
                 (unsigned long long)hp[2], (unsigned long long)hp[3], (unsigned long long)hp[4],
                 (unsigned long long)hp[5], (unsigned long long)hp[6], (unsigned long long)hp[7]);
    if (pub[0] != seq) return Fail(SPM_INTERNAL, "cooperative encode ended without publishing");
  } else {
    const int rc = RunSmallCall(ws, 1, &sa, nullptr, c, st, "cooperative encode");
    if (rc != SPM_OK) return rc;
  }
  if (pub[1] != 0) {  // a sentence it does not take: not done
    ws->StopService();  // the lane-kernel re-run may share the server's hardware queue
    return SPM_OK;
  }
  std::memcpy(tok, h + o_tok, (n + 1) * 8);
  const uint64_t ntok = tok[n];
  if (ntok) {
    std::memcpy(ids, h + o_ids, ntok * 4);
    if (len) std::memcpy(len, h + o_len, ntok * 4);
  }
  ws->stats = spm_hip_encode_stats{};
  ws->stats.sentences = n;
  ws->stats.tokens = ntok;
  spm_amd::PublishStats(m, ws->stats);
  *done = true;
  return SPM_OK;
}

// The round-4 small path (one pinned upload, outputs copied back, stream
// synchronization): SPM_HIP_SMALL_ZEROCOPY=0 (A/B knob).
int EncodeHostSmallCopy(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const uint8_t *bytes, const uint64_t *off,
                    uint64_t n, int32_t *ids, uint32_t *len, uint64_t *tok, hipStream_t st, bool *done) {
  *done = false;
  const uint64_t total = off[n];
  const uint64_t ctl_bytes = spm_amd::kStWords * 4 + 8 * (spm_amd::FastTiles(n) + spm_amd::kScanTiles);
  const uint64_t o_off = Align256(ctl_bytes), o_in = Align256(o_off + (n + 1) * 8);
  const uint64_t in_end = o_in + total;
  const uint64_t o_tok = Align256(in_end + 16), o_ids = Align256(o_tok + (n + 1) * 8);
  const uint64_t o_len = Align256(o_ids + std::max<uint64_t>(total, 1) * 4);
  const uint64_t out_end = len ? o_len + std::max<uint64_t>(total, 1) * 4 : o_ids + std::max<uint64_t>(total, 1) * 4;
  SPM_HIP_TRY(ws->w_small.Reserve(out_end));
  if (ws->pin_small_cap < out_end) {
    if (ws->pin_small) SPM_HIP_TRY(hipHostFree(ws->pin_small));
    ws->pin_small = nullptr;
    ws->pin_small_cap = 0;
    const size_t want = std::max<uint64_t>(out_end, 64 << 10);
    SPM_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&ws->pin_small), want));
    ws->pin_small_cap = want;
  }
  uint8_t *h = ws->pin_small;
  uint8_t *d = ws->w_small.as<uint8_t>();
  std::memset(h, 0, ctl_bytes);
  std::memcpy(h + o_off, off, (n + 1) * 8);
  if (total) std::memcpy(h + o_in, bytes, total);
  SPM_HIP_TRY(hipMemcpyAsync(d, h, in_end, hipMemcpyHostToDevice, st));
  spm_amd::EncodeCall c{d + o_in, reinterpret_cast<uint64_t *>(d + o_off), n, total,
                        reinterpret_cast<int32_t *>(d + o_ids), len ? reinterpret_cast<uint32_t *>(d + o_len) : nullptr,
                        reinterpret_cast<uint64_t *>(d + o_tok), nullptr, st, false, 0};
  ws->stats = spm_hip_encode_stats{};
  FastPlan fp;
  int rc = FastSetup(m, ws, c, reinterpret_cast<uint32_t *>(d), &fp);
  if (rc == SPM_OK) rc = FastPartA(m, ws, c, &fp, false);
  if (rc != SPM_OK) return rc;
  auto fetch = [&]() -> hipError_t {
    hipError_t e = hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(h + o_tok, d + o_tok, out_end - o_tok, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
  };
  SPM_HIP_TRY(fetch());
  const uint32_t *hs = reinterpret_cast<const uint32_t *>(h);
  const uint32_t flagged = hs[spm_amd::kStFlagged];
  if (hs[spm_amd::kStError]) return SPM_OK;  // not done: the blocking path
  if (flagged) {
    if ((rc = FastPartB(m, ws, c, &fp)) != SPM_OK) return rc;
    SPM_HIP_TRY(fetch());
    if (hs[spm_amd::kStError]) return SPM_OK;
  }
  std::memcpy(tok, h + o_tok, (n + 1) * 8);
  const uint64_t ntok = tok[n];
  if (ntok) {
    std::memcpy(ids, h + o_ids, ntok * 4);
    if (len) std::memcpy(len, h + o_len, ntok * 4);
  }
  ws->stats.sentences = n;
  ws->stats.general_path = flagged;
  ws->stats.tokens = ntok;
  if (m->timing && fp.slot >= 0) {
    SPM_HIP_TRY(hipEventElapsedTime(&ws->stats.fast_kernel_ms, ws->tev[2 * fp.slot], ws->tev[2 * fp.slot + 1]));
    if (flagged) SPM_HIP_TRY(hipEventElapsedTime(&ws->stats.general_kernel_ms, ws->ev[0], ws->ev[1]));
    ws->tcount = 0;
  }
  spm_amd::PublishStats(m, ws->stats);
  *done = true;
  return SPM_OK;
}

int EncodeHostSmall(spm_hip_model *m, spm_amd::EncodeWorkspace *ws, const uint8_t *bytes, const uint64_t *off,
                    uint64_t n, int32_t *ids, uint32_t *len, uint64_t *tok, hipStream_t st, bool *done) {
  *done = false;
  const uint64_t total = off[n];
  const uint64_t ctl_bytes = spm_amd::kStWords * 4 + 8 * (spm_amd::FastTiles(n) + spm_amd::kScanTiles);
  const uint64_t o_off = Align256(ctl_bytes), o_in = Align256(o_off + (n + 1) * 8);
  const uint64_t in_end = o_in + total;
  const uint64_t o_tok = Align256(in_end + 16), o_ids = Align256(o_tok + (n + 1) * 8);
  const uint64_t o_len = Align256(o_ids + std::max<uint64_t>(total, 1) * 4);
  const uint64_t out_end = len ? o_len + std::max<uint64_t>(total, 1) * 4 : o_ids + std::max<uint64_t>(total, 1) * 4;
  const uint64_t o_pub = Align256(out_end), pin_end = o_pub + 256;
  SPM_HIP_TRY(ws->w_small.Reserve(out_end));
  if (ws->pin_small_cap < pin_end) {
    if (ws->pin_small) SPM_HIP_TRY(hipHostFree(ws->pin_small));
    ws->pin_small = nullptr;
    ws->pin_small_cap = 0;
    const size_t want = std::max<uint64_t>(pin_end, 64 << 10);
    // Coherent (fine-grained): the kernel reads the input image from it and
    // writes the outputs and the publication word into it directly.
    SPM_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&ws->pin_small), want, hipHostMallocCoherent));
    ws->pin_small_cap = want;
  }
  uint8_t *h = ws->pin_small;
  uint8_t *d = ws->w_small.as<uint8_t>();
  std::memcpy(h + o_off, off, (n + 1) * 8);
  if (total) std::memcpy(h + o_in, bytes, total);
  volatile uint32_t *pub = reinterpret_cast<volatile uint32_t *>(h + o_pub);
  pub[0] = 0;
  const uint32_t seq = ++ws->pub_seq == 0 ? ++ws->pub_seq : ws->pub_seq;
  // The fast kernel's single tile reads the image straight from h and writes
  // the final ids / lengths / token offsets into h (its slots are the outputs:
  // one tile whose slots start at byte 0).
  spm_amd::EncodeCall c{d + o_in, reinterpret_cast<uint64_t *>(d + o_off), n, total,
                        reinterpret_cast<int32_t *>(h + o_ids), len ? reinterpret_cast<uint32_t *>(h + o_len) : nullptr,
                        reinterpret_cast<uint64_t *>(h + o_tok), nullptr, st, false, 0};
  ws->stats = spm_hip_encode_stats{};
  FastPlan fp;
  int rc = FastSetup(m, ws, c, reinterpret_cast<uint32_t *>(d), &fp);
  if (rc != SPM_OK) return rc;
  fp.l.stage_src = reinterpret_cast<const uint32_t *>(h);
  fp.l.stage_dst = reinterpret_cast<uint32_t *>(d);
  fp.l.stage_zero = static_cast<uint32_t>(o_off / 4);  // the status block (ctl_bytes <= o_off)
  fp.l.stage_words = static_cast<uint32_t>((in_end + 3) / 4);
  fp.l.host_pub = reinterpret_cast<uint32_t *>(h + o_pub);
  fp.l.pub_seq = seq;
  rc = FastPartA(m, ws, c, &fp, false);
  if (rc != SPM_OK) {
    (void)hipStreamSynchronize(st);  // nothing may still read h when it is reused
    return rc;
  }
  // Completion: the kernel's publication word, polled; the stream is
  // queried now and then so that a kernel that ended without publishing (an
  // early exit) or failed is noticed.
  bool published = false;
  for (uint32_t spin = 1;; ++spin) {
    if (pub[0] == seq) {
      published = true;
      break;
    }
    if ((spin & 1023) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) {
        published = pub[0] == seq;
        break;
      }
      if (q != hipErrorNotReady) {
        (void)hipStreamSynchronize(st);
        return Fail(SPM_INTERNAL, std::string("HIP: ") + hipGetErrorString(q));
      }
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  uint32_t sw[spm_amd::kStWords];
  if (published) {
    for (int k = 0; k < spm_amd::kStWords; ++k) sw[k] = pub[1 + k];
  } else {
    SPM_HIP_TRY(hipMemcpy(sw, d, sizeof(sw), hipMemcpyDeviceToHost));
  }
  uint32_t flagged = sw[spm_amd::kStFlagged];
  if (sw[spm_amd::kStError]) {
    SPM_HIP_TRY(hipStreamSynchronize(st));
    return SPM_OK;  // not done: the blocking path
  }
  if (flagged) {
    // Rare: the general kernel and the fix-up chain over the flagged
    // sentences (they update the outputs in h), then one synchronization.
    if ((rc = FastPartB(m, ws, c, &fp)) != SPM_OK) {
      (void)hipStreamSynchronize(st);
      return rc;
    }
    SPM_HIP_TRY(hipMemcpyAsync(h + o_pub + 128, d, 16, hipMemcpyDeviceToHost, st));
    SPM_HIP_TRY(hipStreamSynchronize(st));
    if (reinterpret_cast<const uint32_t *>(h + o_pub + 128)[spm_amd::kStError]) return SPM_OK;
  }
  std::memcpy(tok, h + o_tok, (n + 1) * 8);
  const uint64_t ntok = tok[n];
  if (ntok) {
    std::memcpy(ids, h + o_ids, ntok * 4);
    if (len) std::memcpy(len, h + o_len, ntok * 4);
  }
  ws->stats.sentences = n;
  ws->stats.general_path = flagged;
  ws->stats.tokens = ntok;
  if (m->timing && fp.slot >= 0) {
    SPM_HIP_TRY(hipEventSynchronize(ws->tev[2 * fp.slot + 1]));
    SPM_HIP_TRY(hipEventElapsedTime(&ws->stats.fast_kernel_ms, ws->tev[2 * fp.slot], ws->tev[2 * fp.slot + 1]));
    if (flagged) SPM_HIP_TRY(hipEventElapsedTime(&ws->stats.general_kernel_ms, ws->ev[0], ws->ev[1]));
    ws->tcount = 0;
  }
  spm_amd::PublishStats(m, ws->stats);
  *done = true;
  return SPM_OK;
}

}  // namespace

int spm_hip_encode_raw_small_host(spm_hip_model *m, const uint8_t *raw, const uint64_t *raw_off, uint64_t n,
                                  int32_t *ids, uint64_t ids_cap, uint64_t *out_off) {
  spm_amd::TraceRange trace_range_("spm_hip_encode_raw_small_host");
  if (!m || !raw_off || !out_off || (n && !raw && raw_off[n])) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  if (m->host_only) return Fail(SPM_FAILED_PRECONDITION, "model was loaded host-only");
  if (n == 0 || n > spm_amd::kCoopSmallMax || raw_off[0] != 0 || raw_off[n] > kSmallMaxBytes / 8 ||
      m->model_type != spm_amd::kUnigram || m->kernel == spm_amd::UnigramKernel::kGeneralOnly ||
      NeedsHostSized(m) || !m->d_uvs.ptr || m->max_piece_bytes > 56)
    return SPM_UNIMPLEMENTED;
  for (uint64_t i = 0; i < n; ++i)
    if (raw_off[i + 1] < raw_off[i]) return Fail(SPM_INVALID_ARGUMENT, "offsets must not decrease");
  int rc = EnsureNormTables(m);
  if (rc == SPM_OK) rc = EnsureTypes(m);
  if (rc != SPM_OK) return rc;
  spm_amd::WorkspaceLease ws;
  SPM_LEASE(ws, ws.ForHost(m));
  bool done = false;
  rc = EncodeRawCoop(m, ws.get(), raw, raw_off, n, ids, ids_cap, out_off, ws.stream(), &done);
  if (rc != SPM_OK) return rc;
  return done ? SPM_OK : SPM_UNIMPLEMENTED;
}

int spm_hip_encode_batch_host(spm_hip_model *m, const uint8_t *bytes, const uint64_t *off,
                              uint64_t n, int32_t *ids, uint32_t *len, uint64_t *tok) {
  spm_amd::TraceRange trace_range_("spm_hip_encode_batch_host");
  if (!m || !off || !tok) return Fail(SPM_INVALID_ARGUMENT, "null argument");
  if (m->host_only) return Fail(SPM_FAILED_PRECONDITION, "model was loaded host-only");
  if (n >= 0x7FFFFFFFull) return Fail(SPM_OUT_OF_RANGE, "too many sentences in one batch");
  const uint64_t total = off[n] - off[0];
  if (off[0] != 0) return Fail(SPM_INVALID_ARGUMENT, "offsets must start at 0");
  spm_amd::WorkspaceLease ws;
  SPM_LEASE(ws, ws.ForHost(m));
  hipStream_t st = ws.stream();
  if (n >= 1 && n <= kSmallMaxSentences && total <= kSmallMaxBytes && m->model_type == spm_amd::kUnigram &&
      m->kernel != spm_amd::UnigramKernel::kGeneralOnly && !NeedsHostSized(m)) {
    bool done = false;
    static const bool kZeroCopy = [] {
      const char *e = std::getenv("SPM_HIP_SMALL_ZEROCOPY");
      return !(e && std::atoi(e) == 0);
    }();
    // SPM_HIP_COOP_SMALL=0: one-sentence calls on the lane kernels too (A/B knob).
    static const bool kCoopSmall = [] {
      const char *e = std::getenv("SPM_HIP_COOP_SMALL");
      return !(e && std::atoi(e) == 0);
    }();
    // A model whose small calls the cooperative kernel keeps handing back
    // (broken UTF-8, > 8 nodes at a position: each costs a second round
    // trip) skips it after 8 rejections in a row, trying again every 64th
    // call; a call it takes resets the count.
    const uint32_t rejects = m->coop_small_rejects.load(std::memory_order_relaxed);
    const bool try_coop = rejects < 8 || rejects % 64 == 0;
    if (!try_coop) m->coop_small_rejects.fetch_add(1, std::memory_order_relaxed);
    if (kCoopSmall && try_coop && n <= spm_amd::kCoopSmallMax && m->d_uvs.ptr && m->max_piece_bytes <= 56 &&
        !m->force_general) {
      const int rc = EncodeHostCoop(m, ws.get(), bytes, off, n, ids, len, tok, st, &done);
      if (rc != SPM_OK) return rc;
      if (done) {
        m->coop_small_rejects.store(0, std::memory_order_relaxed);
        return rc;
      }
      m->coop_small_rejects.fetch_add(1, std::memory_order_relaxed);
    }
    const int rc = kZeroCopy ? EncodeHostSmall(m, ws.get(), bytes, off, n, ids, len, tok, st, &done)
                             : EncodeHostSmallCopy(m, ws.get(), bytes, off, n, ids, len, tok, st, &done);
    if (rc != SPM_OK || done) return rc;
  }
  SPM_HIP_TRY(ws->h_in.Reserve(std::max<uint64_t>(total, 1)));
  SPM_HIP_TRY(ws->h_off.Reserve((n + 1) * 8));
  SPM_HIP_TRY(ws->h_ids.Reserve(std::max<uint64_t>(total, 1) * 4));
  if (len) SPM_HIP_TRY(ws->h_len.Reserve(std::max<uint64_t>(total, 1) * 4));
  SPM_HIP_TRY(ws->h_tok.Reserve((n + 1) * 8));
  if (total) SPM_HIP_TRY(hipMemcpyAsync(ws->h_in.ptr, bytes, total, hipMemcpyHostToDevice, st));
  SPM_HIP_TRY(hipMemcpyAsync(ws->h_off.ptr, off, (n + 1) * 8, hipMemcpyHostToDevice, st));
  int rc = EncodeBlocking(m, ws.get(), ws->h_in.as<uint8_t>(), ws->h_off.as<uint64_t>(), n,
                      ws->h_ids.as<int32_t>(), len ? ws->h_len.as<uint32_t>() : nullptr,
                      ws->h_tok.as<uint64_t>(), st);
  if (rc != SPM_OK) return rc;
  SPM_HIP_TRY(hipMemcpyAsync(tok, ws->h_tok.ptr, (n + 1) * 8, hipMemcpyDeviceToHost, st));
  SPM_HIP_TRY(hipStreamSynchronize(st));
  const uint64_t ntok = tok[n];
  if (ntok) {
    SPM_HIP_TRY(hipMemcpyAsync(ids, ws->h_ids.ptr, ntok * 4, hipMemcpyDeviceToHost, st));
    if (len) SPM_HIP_TRY(hipMemcpyAsync(len, ws->h_len.ptr, ntok * 4, hipMemcpyDeviceToHost, st));
    SPM_HIP_TRY(hipStreamSynchronize(st));
  }
  ws->stats.tokens = ntok;
  spm_amd::PublishStats(m, ws->stats);
  return SPM_OK;
}

}  // extern "C"
