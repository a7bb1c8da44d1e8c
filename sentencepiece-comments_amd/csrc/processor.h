// C++ mirror of sentencepiece::SentencePieceProcessor's encode surface
// (reference src/sentencepiece_processor.h:176-470) on top of the C-ABI.
//
// Same names, argument meaning and error behaviour as the reference for the
// calls on the hot path: Load / LoadFromSerializedProto, SetEncodeExtraOptions,
// Encode(ids), Encode(pieces), PieceToId / IdToPiece / GetPieceSize /
// IsUnknown / IsControl / unk_id / bos_id / eos_id / pad_id.  Encode is
// batched: EncodeBatch runs the device normalizer and the device encode over
// the whole batch; Encode(ids) also runs the id epilogue of
// PopulateSentencePieceText (unk merge, control pieces) + ApplyExtraOptions
// on the device, Encode(pieces) applies it per line on the host.  Small
// Encode(ids) batches (one line included) go through the pure stream calls
// with one upload and one synchronization (EncodeIdsSmall).  Like the
// reference's processor, one instance is not for concurrent Encode calls.
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/spm_hip.h"
#include "model_proto.h"

namespace spm_amd {

struct Status {
  int code = SPM_OK;  // util::error::Code
  std::string message;
  bool ok() const { return code == SPM_OK; }
  static Status Ok() { return Status(); }
};

class SentencePieceProcessor {
 public:
  SentencePieceProcessor() = default;
  ~SentencePieceProcessor();
  SentencePieceProcessor(const SentencePieceProcessor &) = delete;
  SentencePieceProcessor &operator=(const SentencePieceProcessor &) = delete;

  Status Load(const std::string &filename);
  Status LoadFromSerializedProto(const std::string &serialized);
  Status status() const;

  // "bos", "eos", "reverse" separated by ':' (sentencepiece_processor.cc:981-1010).
  Status SetEncodeExtraOptions(const std::string &extra_options);

  Status Encode(const std::string &input, std::vector<int> *ids) const;
  Status Encode(const std::string &input, std::vector<std::string> *pieces) const;
  // Batched encode: ids and/or pieces (either may be null).
  Status EncodeBatch(const std::vector<std::string> &inputs, std::vector<std::vector<int>> *ids,
                     std::vector<std::vector<std::string>> *pieces) const;

  int GetPieceSize() const;
  int PieceToId(const std::string &piece) const;
  const std::string &IdToPiece(int id) const;
  float GetScore(int id) const;
  bool IsUnknown(int id) const;
  bool IsControl(int id) const;
  bool IsUnused(int id) const;
  int unk_id() const;
  int bos_id() const;
  int eos_id() const;
  int pad_id() const;

 private:
  enum ExtraOption { REVERSE, BOS, EOS };
  spm_hip_model *model_ = nullptr;
  ModelProtoView proto_;
  std::unordered_map<std::string, int> pieces_, reserved_;
  std::vector<ExtraOption> extra_;
  std::string extra_str_;  // the accepted option string, for the device epilogue
  Status status_{SPM_INTERNAL, "Model is not initialized."};
  // Grow-only device staging for EncodeBatch (raw lines → normalized → ids).
  struct Staging {
    void *ptr[10] = {};
    size_t cap[10] = {};
    void *Get(int k, size_t bytes);
    ~Staging();
  };
  mutable Staging dev_;
  // Small Encode(ids) batches (EncodeIdsSmall): a private stream and a
  // grow-only pinned host block.
  struct SmallPath {
    void *stream = nullptr;
    uint8_t *pin = nullptr;
    size_t pin_cap = 0;
    ~SmallPath();
  };
  mutable SmallPath small_;
  // true: *ids filled; false: take the general path (capacity guess exceeded).
  Status EncodeIdsSmall(const std::vector<std::string> &inputs, std::vector<std::vector<int>> *ids,
                        bool *done) const;
};

}  // namespace spm_amd
