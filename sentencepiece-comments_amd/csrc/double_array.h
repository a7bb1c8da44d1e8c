// Byte-wise double-array trie laid out for the GPU walk.
//
// The reference builds a darts-clone DoubleArray over the NORMAL /
// USER_DEFINED / UNUSED pieces (unigram_model.cc:624-673) and walks it with
// commonPrefixSearch (third_party/darts_clone/darts.h:469-512).  Encode parity
// needs only the same (prefix length, value) match set, so the device trie is
// our own layout, built breadth-first so that the hot top levels sit in the
// first few KB of the array:
//
//   unit (uint32) = base << 9 | leaf << 8 | label        child = base ^ byte
//   value[unit]   = piece payload when leaf (see spm_hip.hip), else -1
//
// A slot is a child of parent P only if its label matches the byte and
// base(P) is used by no other parent, so one 4-byte load per input byte is
// enough to follow an edge.  Keys have C-string semantics (a NUL byte ends a
// key, as in darts.h build()), and an input NUL never matches.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace spm_amd {

struct DoubleArray {
  std::vector<uint32_t> units;
  std::vector<int32_t> values;
  int32_t max_prefix_matches = 0;  // == unigram trie_results_size_
  static constexpr uint32_t kBaseLimit = 1u << 23;

  static uint32_t Label(uint32_t u) { return u & 0xFFu; }
  static bool Leaf(uint32_t u) { return (u >> 8) & 1u; }
  static uint32_t Base(uint32_t u) { return u >> 9; }

  // Host-side walk (used for validation and by host-only helpers).
  // Returns the value of `key` or -1.
  int32_t ExactMatch(const char *key, size_t len) const;
  // (value, byte length) of every key that prefixes key[0:len), shortest first.
  void CommonPrefixSearch(const char *key, size_t len,
                          std::vector<std::pair<int32_t, size_t>> *out) const;
};

// keys: (bytes, value).  Duplicate keys (after NUL truncation) keep the first
// value.  Returns false if the array would exceed kBaseLimit units.
bool BuildDoubleArray(std::vector<std::pair<std::string, int32_t>> keys, DoubleArray *out,
                      std::string *err);

}  // namespace spm_amd
