// Host normalizer (see normalizer.h).
#include "normalizer.h"

#include <cstring>

namespace spm_amd {
namespace {

constexpr char kSpaceSymbol[] = "\xe2\x96\x81";  // U+2581
constexpr size_t kSpaceSymbolLen = 3;
constexpr char kReplacementChar[] = "\xEF\xBF\xBD";

inline bool Trail(char c) { return (static_cast<uint8_t>(c) & 0xC0u) == 0x80u; }
inline bool ValidCp(uint32_t c) { return c < 0xD800u || (c >= 0xE000u && c <= 0x10FFFFu); }

// darts-clone unit accessors (third_party/darts_clone/darts.h:50-80): the
// charsmap blob is serialised in that format, so these are an on-disk contract.
inline bool DLeaf(uint32_t u) { return (u >> 8) & 1u; }
inline uint32_t DValue(uint32_t u) { return u & 0x7FFFFFFFu; }
inline uint32_t DLabel(uint32_t u) { return u & 0x800000FFu; }
inline uint32_t DOffset(uint32_t u) { return (u >> 10) << ((u & (1u << 9)) >> 6); }

}  // namespace

size_t ValidUTF8CharLen(const char *in, size_t n) {
  const uint8_t c0 = static_cast<uint8_t>(in[0]);
  uint32_t cp = 0;
  size_t len = 0;
  if (c0 < 0x80u) return 1;
  if (n >= 2 && (c0 & 0xE0u) == 0xC0u) {
    cp = ((c0 & 0x1Fu) << 6) | (in[1] & 0x3F);
    if (Trail(in[1]) && cp >= 0x80u && ValidCp(cp)) len = 2;
  } else if (n >= 3 && (c0 & 0xF0u) == 0xE0u) {
    cp = ((c0 & 0x0Fu) << 12) | ((in[1] & 0x3F) << 6) | (in[2] & 0x3F);
    if (Trail(in[1]) && Trail(in[2]) && cp >= 0x800u && ValidCp(cp)) len = 3;
  } else if (n >= 4 && (c0 & 0xF8u) == 0xF0u) {
    cp = ((c0 & 0x07u) << 18) | ((in[1] & 0x3F) << 12) | ((in[2] & 0x3F) << 6) | (in[3] & 0x3F);
    if (Trail(in[1]) && Trail(in[2]) && Trail(in[3]) && cp >= 0x10000u && ValidCp(cp)) len = 4;
  }
  return len;  // 0: invalid.  (A decoded U+FFFD has len 3 and is accepted.)
}

PrefixMatcher::PrefixMatcher(const std::vector<std::string> &symbols) {
  if (symbols.empty()) return;
  std::vector<std::pair<std::string, int32_t>> keys;
  for (const auto &s : symbols) keys.emplace_back(s, 1);
  std::string err;
  if (BuildDoubleArray(keys, &trie_, &err)) empty_ = false;
}

int PrefixMatcher::Match(const char *w, size_t n, bool *found) const {
  const int one = static_cast<int>(std::min<size_t>(n, OneCharLen(static_cast<uint8_t>(w[0]))));
  if (empty_) {
    if (found) *found = false;
    return one;
  }
  std::vector<std::pair<int32_t, size_t>> res;
  trie_.CommonPrefixSearch(w, n, &res);
  if (found) *found = !res.empty();
  if (res.empty()) return one;
  return static_cast<int>(res.back().second);  // longest
}

Normalizer::Normalizer(const NormalizerSpecView &spec, bool treat_whitespace_as_suffix)
    : spec_(spec), suffix_(treat_whitespace_as_suffix) {
  const std::string &blob = spec_.precompiled_charsmap;
  if (blob.empty()) return;  // identity normalization
  uint32_t trie_size = 0;
  if (blob.size() <= 4) {
    ok_ = false;
  } else {
    std::memcpy(&trie_size, blob.data(), 4);
    // (The reference checks only trie_size < blob size, normalizer.cc:
    // 305-337; a trie of no whole unit cannot even hold its root.)
    if (trie_size >= blob.size() || trie_size < 4) ok_ = false;
  }
  if (!ok_) {
    error_ = "Blob for normalization rule is broken.";
    return;
  }
  units_ = reinterpret_cast<const uint32_t *>(spec_.precompiled_charsmap.data() + 4);
  num_units_ = trie_size / 4;
  pool_ = spec_.precompiled_charsmap.data() + 4 + trie_size;
  pool_size_ = blob.size() - 4 - trie_size;
}

size_t Normalizer::CharsmapLongest(const char *in, size_t n, uint32_t *value) const {
  if (!units_) return 0;
  size_t best = 0, found = 0;
  size_t pos = DOffset(units_[0]);
  for (size_t i = 0; i < n; ++i) {
    const uint32_t c = static_cast<uint8_t>(in[i]);
    pos ^= c;
    if (pos >= num_units_) break;
    const uint32_t u = units_[pos];
    if (DLabel(u) != c) break;
    pos ^= DOffset(u);
    if (DLeaf(u)) {
      // kMaxTrieResultsSize = 32 (normalizer.h:169): only the first 32
      // matches are considered.
      if (found++ >= 32) break;
      // A value unit outside the trie or a value outside the pool (only in a
      // corrupted blob) is no match: untrusted .model bytes never steer a
      // read out of the blob (the device walk does the same).
      if (pos >= num_units_ || DValue(units_[pos]) >= pool_size_) continue;
      best = i + 1;
      *value = DValue(units_[pos]);
    }
  }
  return best;
}

const char *Normalizer::NormalizePrefix(const char *in, size_t n, size_t *out_len,
                                        size_t *consumed) const {
  if (matcher_ && !matcher_->empty()) {
    bool found = false;
    const int mblen = matcher_->Match(in, n, &found);
    if (found) {
      *out_len = *consumed = static_cast<size_t>(mblen);
      return in;
    }
  }
  uint32_t value = 0;
  const size_t longest = CharsmapLongest(in, n, &value);
  if (longest == 0) {
    const size_t len = ValidUTF8CharLen(in, n);
    if (len == 0) {
      *out_len = 3;
      *consumed = 1;
      return kReplacementChar;
    }
    *out_len = *consumed = len;
    return in;
  }
  *consumed = longest;
  const char *r = pool_ + value;
  *out_len = strnlen(r, pool_size_ - value);  // a pool without its final NUL ends at the blob's end
  return r;
}

void Normalizer::Normalize(const char *in, size_t n, std::string *normalized,
                           std::vector<size_t> *n2o) const {
  normalized->clear();
  n2o->clear();
  if (n == 0) return;
  size_t consumed = 0;
  const bool rew = spec_.remove_extra_whitespaces;
  const bool esc = spec_.escape_whitespaces;
  size_t rlen, rcons;
  if (rew) {
    while (n > 0) {
      const char *r = NormalizePrefix(in, n, &rlen, &rcons);
      if (!(rlen == 1 && r[0] == ' ')) break;
      in += rcons;
      n -= rcons;
      consumed += rcons;
    }
  }
  if (n == 0) return;
  normalized->reserve(n * 3);
  n2o->reserve(n * 3);
  auto add_ws = [&]() {
    if (esc) {
      normalized->append(kSpaceSymbol, kSpaceSymbolLen);
      n2o->insert(n2o->end(), kSpaceSymbolLen, consumed);
    } else {
      normalized->push_back(' ');
      n2o->push_back(consumed);
    }
  };
  if (!suffix_ && spec_.add_dummy_prefix) add_ws();
  bool prev_space = rew;
  while (n > 0) {
    const char *r = NormalizePrefix(in, n, &rlen, &rcons);
    size_t k = 0;
    if (prev_space)
      while (k < rlen && r[k] == ' ') ++k;
    if (k < rlen) {
      for (; k < rlen; ++k) {
        if (esc && r[k] == ' ') {
          normalized->append(kSpaceSymbol, kSpaceSymbolLen);
          n2o->insert(n2o->end(), kSpaceSymbolLen, consumed);
        } else {
          normalized->push_back(r[k]);
          n2o->push_back(consumed);
        }
      }
      prev_space = r[rlen - 1] == ' ';
    }
    consumed += rcons;
    in += rcons;
    n -= rcons;
    if (!rew) prev_space = false;
  }
  if (rew) {
    const char *sp = esc ? kSpaceSymbol : " ";
    const size_t sl = esc ? kSpaceSymbolLen : 1;
    while (normalized->size() >= sl &&
           std::memcmp(normalized->data() + normalized->size() - sl, sp, sl) == 0) {
      const size_t length = normalized->size() - sl;
      consumed = (*n2o)[length];
      normalized->resize(length);
      n2o->resize(length);
    }
  }
  if (suffix_ && spec_.add_dummy_prefix) add_ws();
  n2o->push_back(consumed);
}

}  // namespace spm_amd
