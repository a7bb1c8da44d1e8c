// Minimal protobuf (proto2 wire format) reader for the ModelProto on-disk
// format: reference src/sentencepiece_model.proto:21-275.  There is no protoc
// in this image and the product needs only the fields below; unknown fields
// are skipped, unknown enum values keep the field default (protobuf-lite
// behaviour for proto2 enums).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace spm_amd {

enum PieceType : int32_t {
  kNormal = 1,       // ModelProto.SentencePiece.NORMAL
  kUnknown = 2,      // UNKNOWN
  kControl = 3,      // CONTROL
  kUserDefined = 4,  // USER_DEFINED
  kUnused = 5,       // UNUSED
};

enum ModelTypeId : int32_t { kUnigram = 1, kBpe = 2, kWord = 3, kChar = 4 };

struct PieceRec {
  std::string piece;
  float score = 0.0f;
  int32_t type = kNormal;
};

struct TrainerSpecView {
  int32_t model_type = kUnigram;
  bool treat_whitespace_as_suffix = false;
  std::string unk_piece = "<unk>";
  std::string bos_piece = "<s>";
  std::string eos_piece = "</s>";
  std::string pad_piece = "<pad>";
  bool has_unk_surface = false;
  std::string unk_surface = " \xE2\x81\x87 ";
};

struct NormalizerSpecView {
  std::string name;
  std::string precompiled_charsmap;
  bool add_dummy_prefix = true;
  bool remove_extra_whitespaces = true;
  bool escape_whitespaces = true;
};

struct ModelProtoView {
  std::vector<PieceRec> pieces;
  TrainerSpecView trainer_spec;
  NormalizerSpecView normalizer_spec;
  std::vector<std::pair<std::string, std::string>> self_test;  // (input, expected)
};

// Returns false (and fills *err) when the buffer is not a valid ModelProto.
bool ParseModelProto(const uint8_t *data, size_t len, ModelProtoView *out, std::string *err);

}  // namespace spm_amd
