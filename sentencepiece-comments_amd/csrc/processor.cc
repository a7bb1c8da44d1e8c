// SentencePieceProcessor mirror (see processor.h).
#include "processor.h"

#include <hip/hip_runtime.h>

#include "scratch_cache.h"

#include <algorithm>
#include <cstring>
#include <fstream>
#include <iterator>
#include <sstream>

namespace spm_amd {
namespace {

Status Err(int code, const std::string &msg) { return Status{code, msg}; }

Status FromC(int rc) {
  if (rc == SPM_OK) return Status::Ok();
  return Err(rc, spm_hip_last_error());
}

}  // namespace

SentencePieceProcessor::~SentencePieceProcessor() { spm_hip_model_free(model_); }

void *SentencePieceProcessor::Staging::Get(int k, size_t bytes) {
  bytes = std::max<size_t>(bytes, 16);
  if (bytes > cap[k]) {
    if (ptr[k]) (void)DevFree(ptr[k]);
    ptr[k] = nullptr;
    cap[k] = 0;
    const size_t c = bytes + bytes / 4;
    if (DevMalloc(&ptr[k], c) != hipSuccess) return nullptr;
    cap[k] = c;
  }
  return ptr[k];
}

SentencePieceProcessor::Staging::~Staging() {
  for (void *p : ptr)
    if (p) (void)DevFree(p);
}

SentencePieceProcessor::SmallPath::~SmallPath() {
  if (stream) (void)hipStreamDestroy(static_cast<hipStream_t>(stream));
  if (pin) (void)hipHostFree(pin);
}

Status SentencePieceProcessor::Load(const std::string &filename) {
  std::ifstream in(filename, std::ios::binary);
  if (!in) return Err(SPM_NOT_FOUND, "\"" + filename + "\": No such file or directory");
  std::string proto((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  return LoadFromSerializedProto(proto);
}

Status SentencePieceProcessor::LoadFromSerializedProto(const std::string &serialized) {
  spm_hip_model_free(model_);
  model_ = nullptr;
  proto_ = ModelProtoView();
  pieces_.clear();
  reserved_.clear();
  std::string err;
  if (!ParseModelProto(reinterpret_cast<const uint8_t *>(serialized.data()), serialized.size(),
                       &proto_, &err))
    return status_ = Err(SPM_INTERNAL, err);
  Status st = FromC(spm_hip_model_load(serialized.data(), serialized.size(), &model_));
  if (!st.ok()) return status_ = st;
  for (size_t i = 0; i < proto_.pieces.size(); ++i) {
    const auto &p = proto_.pieces[i];
    const bool normal = p.type == kNormal || p.type == kUserDefined || p.type == kUnused;
    (normal ? pieces_ : reserved_).emplace(p.piece, static_cast<int>(i));
  }
  status_ = Status::Ok();
  // Self-test samples (sentencepiece_processor.cc:135-153).
  std::vector<std::string> inputs;
  for (const auto &s : proto_.self_test) inputs.push_back(s.first);
  if (!inputs.empty()) {
    std::vector<std::vector<std::string>> got;
    Status e = EncodeBatch(inputs, nullptr, &got);
    if (!e.ok()) return status_ = e;
    int fails = 0;
    for (size_t i = 0; i < inputs.size(); ++i) {
      std::string joined;
      for (size_t k = 0; k < got[i].size(); ++k) joined += (k ? " " : "") + got[i][k];
      if (joined != proto_.self_test[i].second) ++fails;
    }
    if (fails) return status_ = Err(SPM_INTERNAL, "Self-test failures. See LOG(INFO).");
  }
  return status_;
}

Status SentencePieceProcessor::status() const { return status_; }

int SentencePieceProcessor::GetPieceSize() const { return static_cast<int>(proto_.pieces.size()); }

// ModelInterface::PieceToId (model_interface.cc:87-97).
int SentencePieceProcessor::PieceToId(const std::string &piece) const {
  auto r = reserved_.find(piece);
  if (r != reserved_.end()) return r->second;
  auto p = pieces_.find(piece);
  if (p != pieces_.end()) return p->second;
  return unk_id();
}

const std::string &SentencePieceProcessor::IdToPiece(int id) const {
  static const std::string kEmpty;
  if (id < 0 || id >= GetPieceSize()) return kEmpty;
  return proto_.pieces[id].piece;
}
float SentencePieceProcessor::GetScore(int id) const { return proto_.pieces[id].score; }
bool SentencePieceProcessor::IsUnknown(int id) const {
  return id >= 0 && id < GetPieceSize() && proto_.pieces[id].type == kUnknown;
}
bool SentencePieceProcessor::IsControl(int id) const {
  return id >= 0 && id < GetPieceSize() && proto_.pieces[id].type == kControl;
}
bool SentencePieceProcessor::IsUnused(int id) const {
  return id >= 0 && id < GetPieceSize() && proto_.pieces[id].type == kUnused;
}
int SentencePieceProcessor::unk_id() const {
  for (size_t i = 0; i < proto_.pieces.size(); ++i)
    if (proto_.pieces[i].type == kUnknown) return static_cast<int>(i);
  return -1;
}
int SentencePieceProcessor::bos_id() const {
  const int id = PieceToId(proto_.trainer_spec.bos_piece);
  return IsControl(id) ? id : -1;
}
int SentencePieceProcessor::eos_id() const {
  const int id = PieceToId(proto_.trainer_spec.eos_piece);
  return IsControl(id) ? id : -1;
}
int SentencePieceProcessor::pad_id() const {
  const int id = PieceToId(proto_.trainer_spec.pad_piece);
  return IsControl(id) ? id : -1;
}

// ParseExtraOptions (sentencepiece_processor.cc:981-1010).
Status SentencePieceProcessor::SetEncodeExtraOptions(const std::string &opts) {
  extra_.clear();
  extra_str_.clear();
  if (opts.empty()) return Status::Ok();
  if (!status_.ok()) return status_;
  std::stringstream ss(opts);
  std::string tok;
  std::vector<std::string> parts;
  size_t st = 0;
  while (true) {
    const size_t e = opts.find(':', st);
    parts.push_back(opts.substr(st, e == std::string::npos ? std::string::npos : e - st));
    if (e == std::string::npos) break;
    st = e + 1;
  }
  for (const auto &s : parts) {
    if (s.empty()) continue;  // SplitPiece drops empty fields
    if (s == "bos") {
      if (IsUnknown(PieceToId(proto_.trainer_spec.bos_piece)))
        return Err(SPM_INTERNAL, "id for `" + proto_.trainer_spec.bos_piece + "` is not defined.");
      extra_.push_back(BOS);
    } else if (s == "eos") {
      if (IsUnknown(PieceToId(proto_.trainer_spec.eos_piece)))
        return Err(SPM_INTERNAL, "id for `" + proto_.trainer_spec.eos_piece + "` is not defined.");
      extra_.push_back(EOS);
    } else if (s == "reverse") {
      extra_.push_back(REVERSE);
    } else {
      return Err(SPM_INTERNAL, "option \"" + s + "\" is not available.");
    }
  }
  extra_str_ = opts;
  return Status::Ok();
}

namespace {
constexpr uint64_t kSmallLines = 4096;
constexpr uint64_t kSmallBytes = 64 << 10;
inline uint64_t Al256(uint64_t x) { return (x + 255) & ~255ull; }
}  // namespace

// Encode(ids) of a small batch — the reference's per-line plugin point
// (sentencepiece_processor.cc:319-330) — as ONE stream-ordered chain: the
// zeroed status word, offsets and raw bytes go up in one copy from pinned
// memory, spm_hip_normalize_batch_device_async -> spm_hip_encode_batch_async
// -> spm_hip_finalize_ids_async run back to back on a private stream, and
// the status word and the final ids come back with one synchronization.
// The normalized size is bounded by a guess (4 bytes per raw byte + 8 per
// line); a batch that exceeds it reports RESOURCE_EXHAUSTED in the status
// word and takes the general path.
Status SentencePieceProcessor::EncodeIdsSmall(const std::vector<std::string> &inputs,
                                              std::vector<std::vector<int>> *ids, bool *done) const {
  *done = false;
  const uint64_t n = inputs.size();
  uint64_t raw = 0;
  for (const auto &s : inputs) raw += s.size();
  if (extra_.empty() && n <= 16) {
    // One launch: normalize + encode + unknown-run merge (coop_raw_kernel).
    std::vector<uint64_t> roff(n + 1, 0);
    std::string rb;
    rb.reserve(raw);
    for (uint64_t i = 0; i < n; ++i) {
      rb += inputs[i];
      roff[i + 1] = rb.size();
    }
    std::vector<int32_t> out(4 * raw + 8 * n + 64);
    std::vector<uint64_t> ooff(n + 1);
    const int rc = spm_hip_encode_raw_small_host(model_, reinterpret_cast<const uint8_t *>(rb.data()), roff.data(),
                                                 n, out.data(), out.size(), ooff.data());
    if (rc == SPM_OK) {
      ids->assign(n, {});
      for (uint64_t i = 0; i < n; ++i) (*ids)[i].assign(out.begin() + ooff[i], out.begin() + ooff[i + 1]);
      *done = true;
      return Status::Ok();
    }
    if (rc != SPM_UNIMPLEMENTED) return FromC(rc);
  }
  uint64_t n_extra = 0;
  for (ExtraOption opt : extra_) n_extra += opt != REVERSE;
  const uint64_t cap_norm = 4 * raw + 8 * n + 64, cap_out = cap_norm + n * n_extra;
  // Device block: [status | in_off | in bytes] (uploaded) [norm | norm_off |
  // ids | tok] (device only) [out_off | out ids] (downloaded).
  const uint64_t o_inoff = 256, o_in = Al256(o_inoff + (n + 1) * 8), up_end = o_in + raw;
  const uint64_t o_norm = Al256(up_end + 16), o_noff = Al256(o_norm + cap_norm);
  const uint64_t o_ids = Al256(o_noff + (n + 1) * 8), o_tok = Al256(o_ids + cap_norm * 4);
  const uint64_t o_oo = Al256(o_tok + (n + 1) * 8), o_out = Al256(o_oo + (n + 1) * 8);
  const uint64_t end = o_out + cap_out * 4;
  enum { kSmallBlock = 9 };
  uint8_t *d = static_cast<uint8_t *>(dev_.Get(kSmallBlock, end));
  if (!d) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
  auto fail_hip = [](hipError_t e) { return Err(SPM_INTERNAL, hipGetErrorString(e)); };
  hipError_t he;
  if (!small_.stream) {
    hipStream_t s;
    if ((he = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) return fail_hip(he);
    small_.stream = s;
  }
  if (small_.pin_cap < end) {
    if (small_.pin) (void)hipHostFree(small_.pin);
    small_.pin = nullptr;
    small_.pin_cap = 0;
    const size_t want = std::max<uint64_t>(end + end / 4, 1 << 20);
    if ((he = hipHostMalloc(reinterpret_cast<void **>(&small_.pin), want)) != hipSuccess) return fail_hip(he);
    small_.pin_cap = want;
  }
  hipStream_t st = static_cast<hipStream_t>(small_.stream);
  uint8_t *h = small_.pin;
  std::memset(h, 0, 256);
  uint64_t *in_off = reinterpret_cast<uint64_t *>(h + o_inoff);
  in_off[0] = 0;
  for (uint64_t i = 0; i < n; ++i) {
    std::memcpy(h + o_in + in_off[i], inputs[i].data(), inputs[i].size());
    in_off[i + 1] = in_off[i] + inputs[i].size();
  }
  if ((he = hipMemcpyAsync(d, h, up_end, hipMemcpyHostToDevice, st)) != hipSuccess) return fail_hip(he);
  uint32_t *d_status = reinterpret_cast<uint32_t *>(d);
  int rc = spm_hip_normalize_batch_device_async(model_, d + o_in, reinterpret_cast<uint64_t *>(d + o_inoff), n,
                                                d + o_norm, cap_norm, reinterpret_cast<uint64_t *>(d + o_noff),
                                                nullptr, d_status, st);
  if (rc == SPM_OK)
    rc = spm_hip_encode_batch_async(model_, d + o_norm, reinterpret_cast<uint64_t *>(d + o_noff), n, cap_norm,
                                    reinterpret_cast<int32_t *>(d + o_ids), nullptr,
                                    reinterpret_cast<uint64_t *>(d + o_tok), d_status, st);
  if (rc == SPM_OK)
    rc = spm_hip_finalize_ids_async(model_, extra_str_.c_str(), reinterpret_cast<int32_t *>(d + o_ids),
                                    reinterpret_cast<uint64_t *>(d + o_tok), n, reinterpret_cast<int32_t *>(d + o_out),
                                    cap_out, reinterpret_cast<uint64_t *>(d + o_oo), d_status, st);
  if (rc != SPM_OK) return FromC(rc);
  if ((he = hipMemcpyAsync(h, d, 4, hipMemcpyDeviceToHost, st)) != hipSuccess ||
      (he = hipMemcpyAsync(h + o_oo, d + o_oo, end - o_oo, hipMemcpyDeviceToHost, st)) != hipSuccess ||
      (he = hipStreamSynchronize(st)) != hipSuccess)
    return fail_hip(he);
  uint32_t code;
  std::memcpy(&code, h, 4);
  if (code == SPM_RESOURCE_EXHAUSTED) return Status::Ok();  // not done: the general path
  if (code != SPM_OK) return Err(static_cast<int>(code), "device encode failed");
  const uint64_t *oo = reinterpret_cast<const uint64_t *>(h + o_oo);
  const int32_t *out = reinterpret_cast<const int32_t *>(h + o_out);
  ids->resize(n);
  for (uint64_t i = 0; i < n; ++i) (*ids)[i].assign(out + oo[i], out + oo[i + 1]);
  *done = true;
  return Status::Ok();
}

Status SentencePieceProcessor::EncodeBatch(const std::vector<std::string> &inputs,
                                           std::vector<std::vector<int>> *ids,
                                           std::vector<std::vector<std::string>> *pieces) const {
  if (!status_.ok()) return status_;
  const uint64_t n = inputs.size();
  if (!pieces && ids && n >= 1 && n <= kSmallLines) {
    uint64_t raw = 0;
    for (const auto &s : inputs) raw += s.size();
    if (raw <= kSmallBytes) {
      bool done = false;
      Status st = EncodeIdsSmall(inputs, ids, &done);
      if (!st.ok() || done) return st;
    }
  }
  std::vector<uint64_t> in_off(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) in_off[i + 1] = in_off[i] + inputs[i].size();
  std::string in_bytes;
  in_bytes.reserve(in_off[n]);
  for (const auto &s : inputs) in_bytes += s;
  // Raw lines → device; Normalizer::Normalize and ModelInterface::Encode run
  // on the device over the whole batch; ids, piece lengths and (for piece
  // output) the normalized bytes come back for the per-line epilogue.
  enum { kIn, kInOff, kNorm, kNormOff, kIds, kLen, kTok };
  auto fail_hip = [](hipError_t e) { return Err(SPM_INTERNAL, hipGetErrorString(e)); };
  uint8_t *d_in = static_cast<uint8_t *>(dev_.Get(kIn, in_off[n]));
  uint64_t *d_in_off = static_cast<uint64_t *>(dev_.Get(kInOff, (n + 1) * 8));
  uint64_t *d_norm_off = static_cast<uint64_t *>(dev_.Get(kNormOff, (n + 1) * 8));
  uint64_t *d_tok = static_cast<uint64_t *>(dev_.Get(kTok, (n + 1) * 8));
  if (!d_in || !d_in_off || !d_norm_off || !d_tok) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
  hipError_t he;
  if ((he = hipMemcpy(d_in, in_bytes.data(), in_off[n], hipMemcpyHostToDevice)) != hipSuccess ||
      (he = hipMemcpy(d_in_off, in_off.data(), (n + 1) * 8, hipMemcpyHostToDevice)) != hipSuccess)
    return fail_hip(he);
  uint64_t total = 0;
  uint64_t ncap = dev_.cap[kNorm];
  uint8_t *d_norm = static_cast<uint8_t *>(dev_.Get(kNorm, std::max<uint64_t>(ncap, 1)));
  int rc = spm_hip_normalize_batch_device(model_, d_in, d_in_off, n, d_norm, dev_.cap[kNorm],
                                          d_norm_off, &total, nullptr);
  if (rc == SPM_RESOURCE_EXHAUSTED) {
    d_norm = static_cast<uint8_t *>(dev_.Get(kNorm, total));
    if (!d_norm) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    rc = spm_hip_normalize_batch_device(model_, d_in, d_in_off, n, d_norm, dev_.cap[kNorm], d_norm_off,
                                        &total, nullptr);
  }
  Status st = FromC(rc);
  if (!st.ok()) return st;
  int32_t *d_ids = static_cast<int32_t *>(dev_.Get(kIds, std::max<uint64_t>(total, 1) * 4));
  uint32_t *d_len = static_cast<uint32_t *>(dev_.Get(kLen, std::max<uint64_t>(total, 1) * 4));
  if (!d_ids || !d_len) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
  st = FromC(spm_hip_encode_batch(model_, d_norm, d_norm_off, n, d_ids, d_len, d_tok, nullptr));
  if (!st.ok()) return st;
  if (!pieces) {
    // Encode(ids): the id epilogue (unk-run merge + extra options) runs on the
    // device as well (spm_hip_finalize_ids); only the final ids come back.
    enum { kOut = 7, kOutOff = 8 };
    uint64_t n_extra = 0;
    for (ExtraOption opt : extra_) n_extra += opt != REVERSE;
    const uint64_t cap = total + n * n_extra;
    uint64_t *d_out_off = static_cast<uint64_t *>(dev_.Get(kOutOff, (n + 1) * 8));
    int32_t *d_out = static_cast<int32_t *>(dev_.Get(kOut, std::max<uint64_t>(cap, 1) * 4));
    if (!d_out_off || !d_out) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    uint64_t fin = 0;
    st = FromC(spm_hip_finalize_ids(model_, extra_str_.c_str(), d_ids, d_tok, n, d_out, cap, d_out_off, &fin,
                                    nullptr));
    if (!st.ok()) return st;
    std::vector<uint64_t> out_off(n + 1);
    std::vector<int32_t> out(std::max<uint64_t>(fin, 1));
    if ((he = hipMemcpy(out_off.data(), d_out_off, (n + 1) * 8, hipMemcpyDeviceToHost)) != hipSuccess ||
        (fin && (he = hipMemcpy(out.data(), d_out, fin * 4, hipMemcpyDeviceToHost)) != hipSuccess))
      return fail_hip(he);
    if (ids) {
      ids->resize(n);
      for (uint64_t i = 0; i < n; ++i) (*ids)[i].assign(out.begin() + out_off[i], out.begin() + out_off[i + 1]);
    }
    return Status::Ok();
  }
  std::vector<uint64_t> norm_off(n + 1), tok_off(n + 1);
  if ((he = hipMemcpy(norm_off.data(), d_norm_off, (n + 1) * 8, hipMemcpyDeviceToHost)) != hipSuccess ||
      (he = hipMemcpy(tok_off.data(), d_tok, (n + 1) * 8, hipMemcpyDeviceToHost)) != hipSuccess)
    return fail_hip(he);
  const uint64_t ntok = tok_off[n];
  std::vector<int32_t> tok_ids(std::max<uint64_t>(ntok, 1));
  std::vector<uint32_t> tok_len(std::max<uint64_t>(ntok, 1));
  std::vector<uint8_t> norm(pieces ? std::max<uint64_t>(total, 1) : 0);
  if ((he = hipMemcpy(tok_ids.data(), d_ids, ntok * 4, hipMemcpyDeviceToHost)) != hipSuccess ||
      (he = hipMemcpy(tok_len.data(), d_len, ntok * 4, hipMemcpyDeviceToHost)) != hipSuccess ||
      (pieces && (he = hipMemcpy(norm.data(), d_norm, total, hipMemcpyDeviceToHost)) != hipSuccess))
    return fail_hip(he);
  if (ids) ids->assign(n, {});
  if (pieces) pieces->assign(n, {});
  const std::string &bos = proto_.trainer_spec.bos_piece, &eos = proto_.trainer_spec.eos_piece;
  std::vector<std::pair<std::string, int>> spt;
  for (uint64_t i = 0; i < n; ++i) {
    // PopulateSentencePieceText (sentencepiece_processor.cc:488-551).
    spt.clear();
    const char *normalized = pieces ? reinterpret_cast<const char *>(norm.data()) + norm_off[i] : nullptr;
    const uint64_t nlen = norm_off[i + 1] - norm_off[i];
    uint64_t consumed = 0;
    bool prev_unk = false;
    for (uint64_t k = tok_off[i]; k < tok_off[i + 1]; ++k) {
      const int id = tok_ids[k];
      const uint32_t len = tok_len[k];
      if (len == 0) return Err(SPM_INTERNAL, "Empty piece is not allowed.");
      std::string w = normalized ? std::string(normalized + consumed, len) : std::string();
      const bool is_unk = IsUnknown(id);
      if (IsControl(id)) {
        spt.emplace_back(std::move(w), id);
      } else {
        if (prev_unk && is_unk) spt.back().first += w;
        else spt.emplace_back(std::move(w), id);
        consumed += len;
      }
      prev_unk = is_unk;
    }
    if (consumed != nlen) return Err(SPM_INTERNAL, "all normalized characters are not consumed.");
    // ApplyExtraOptions (sentencepiece_processor.cc:945-979).
    for (ExtraOption opt : extra_) {
      if (opt == REVERSE) std::reverse(spt.begin(), spt.end());
      else if (opt == EOS) spt.emplace_back(eos, PieceToId(eos));
      else spt.insert(spt.begin(), {bos, PieceToId(bos)});
    }
    if (ids)
      for (auto &p : spt) (*ids)[i].push_back(p.second);
    if (pieces)
      for (auto &p : spt) (*pieces)[i].push_back(std::move(p.first));
  }
  return Status::Ok();
}

Status SentencePieceProcessor::Encode(const std::string &input, std::vector<int> *ids) const {
  if (!ids) return Err(SPM_INTERNAL, "output container is null");
  std::vector<std::vector<int>> out;
  Status st = EncodeBatch({input}, &out, nullptr);
  if (st.ok()) *ids = std::move(out[0]);
  return st;
}

Status SentencePieceProcessor::Encode(const std::string &input,
                                      std::vector<std::string> *pieces) const {
  if (!pieces) return Err(SPM_INTERNAL, "output container is null");
  std::vector<std::vector<std::string>> out;
  Status st = EncodeBatch({input}, nullptr, &out);
  if (st.ok()) *pieces = std::move(out[0]);
  return st;
}

}  // namespace spm_amd
