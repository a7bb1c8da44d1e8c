// Host normalizer: Normalizer::Normalize / NormalizePrefix
// (reference src/normalizer.cc:88-300) over the precompiled charsmap blob
// (uint32 trie size | darts-clone units | NUL-separated targets,
// normalizer.cc:305-337), plus PrefixMatcher for user-defined symbols
// (normalizer.cc:339-384).  Host threads (spm_hip_normalize_batch); the
// device version is normalize_kernels.hip.  Walks are bounds-checked against
// the blob, so corrupted .model bytes cannot steer a read outside it.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "double_array.h"
#include "model_proto.h"

namespace spm_amd {

// Longest-match over a set of strings (PrefixMatcher).
class PrefixMatcher {
 public:
  PrefixMatcher() = default;
  explicit PrefixMatcher(const std::vector<std::string> &symbols);
  bool empty() const { return empty_; }
  // Byte length of the longest symbol prefixing w; *found false → one char.
  int Match(const char *w, size_t n, bool *found) const;

 private:
  bool empty_ = true;
  DoubleArray trie_;
};

class Normalizer {
 public:
  Normalizer(const NormalizerSpecView &spec, bool treat_whitespace_as_suffix);
  bool ok() const { return ok_; }
  const std::string &error() const { return error_; }
  void SetPrefixMatcher(const PrefixMatcher *m) { matcher_ = m; }

  // normalized bytes + norm_to_orig (size normalized+1), as the reference.
  void Normalize(const char *in, size_t n, std::string *normalized,
                 std::vector<size_t> *norm_to_orig) const;

 private:
  // Returns the replacement for the longest rule prefixing `in` and sets
  // *consumed to the number of input bytes it covers.
  const char *NormalizePrefix(const char *in, size_t n, size_t *out_len, size_t *consumed) const;
  size_t CharsmapLongest(const char *in, size_t n, uint32_t *value) const;

  NormalizerSpecView spec_;
  bool suffix_;
  const uint32_t *units_ = nullptr;
  size_t num_units_ = 0;
  const char *pool_ = nullptr;
  size_t pool_size_ = 0;
  const PrefixMatcher *matcher_ = nullptr;
  bool ok_ = true;
  std::string error_;
};

// UTF-8 helpers shared by host code (util.h:389, util.cc:187-227).
inline int OneCharLen(uint8_t lead) {
  static const uint8_t kTab[16] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 3, 4};
  return kTab[lead >> 4];
}
// Number of bytes of the valid UTF-8 char at `in`, or 0 if invalid (a
// literal U+FFFD counts as valid, util.h:459-462).
size_t ValidUTF8CharLen(const char *in, size_t n);

}  // namespace spm_amd
