// Trie build check under the host sanitizers (ASan+UBSan build and a TSan
// build, tools/sanitize/Makefile): BuildDoubleArray over key sets large
// enough for the threaded subtree placement (double_array.cc Place) and small
// ones placed by one thread, with long shared prefixes, high bytes, NULs,
// duplicates and empty keys.  Every key is looked up (ExactMatch) and random
// queries' CommonPrefixSearch results are compared with a std::map of the
// canonical keys (NUL-truncated, first value of equal keys, empty dropped).
// Prints one JSON line; exits 1 on the first mismatch.
#include <cstdio>
#include <map>
#include <random>
#include <string>
#include <utility>
#include <vector>

#include "double_array.h"

using spm_amd::BuildDoubleArray;
using spm_amd::DoubleArray;
using Keys = std::vector<std::pair<std::string, int32_t>>;

namespace {

int Fail(const char *what, const std::string &key) {
  std::fprintf(stderr, "trie_check: %s (key of %zu bytes)\n", what, key.size());
  return 1;
}

int Check(const Keys &keys, std::mt19937 *rng, size_t *queries) {
  std::map<std::string, int32_t> want;
  for (const auto &k : keys) {
    std::string s = k.first.substr(0, k.first.find('\0'));
    if (!s.empty()) want.emplace(s, k.second);
  }
  DoubleArray da;
  std::string err;
  if (!BuildDoubleArray(keys, &da, &err)) return Fail("build failed", err);
  int32_t maxpm = 0;
  for (const auto &kv : want) {
    if (da.ExactMatch(kv.first.data(), kv.first.size()) != kv.second) return Fail("ExactMatch", kv.first);
    int32_t m = 0;
    for (size_t l = 1; l <= kv.first.size(); ++l) m += want.count(kv.first.substr(0, l)) ? 1 : 0;
    maxpm = std::max(maxpm, m);
  }
  if (da.max_prefix_matches != maxpm) return Fail("max_prefix_matches", "");
  std::vector<std::pair<int32_t, size_t>> got;
  for (size_t q = 0; q < 4000 && !keys.empty(); ++q) {
    std::string s = keys[(*rng)() % keys.size()].first;
    const size_t tail = (*rng)() % 4;
    for (size_t t = 0; t < tail; ++t) s.push_back(static_cast<char>((*rng)() % 256));
    if (!s.empty() && (*rng)() % 3 == 0) s.resize((*rng)() % s.size());
    da.CommonPrefixSearch(s.data(), s.size(), &got);
    std::vector<std::pair<int32_t, size_t>> ref;
    for (size_t l = 1; l <= s.size() && s[l - 1] != '\0'; ++l) {
      auto it = want.find(s.substr(0, l));
      if (it != want.end()) ref.emplace_back(it->second, l);
    }
    if (got != ref) return Fail("CommonPrefixSearch", s);
    if (da.ExactMatch(s.data(), s.size()) != (want.count(s) ? want[s] : -1)) return Fail("ExactMatch miss", s);
    ++*queries;
  }
  return 0;
}

std::string Word(std::mt19937 *rng, int alphabet, int maxlen) {
  std::string w;
  if ((*rng)() % 3) w = "\xE2\x96\x81";
  const int len = 1 + static_cast<int>((*rng)() % maxlen);
  for (int i = 0; i < len; ++i) w.push_back(static_cast<char>('a' + (*rng)() % alphabet));
  return w;
}

}  // namespace

int main() {
  std::mt19937 rng(20261017);
  size_t sets = 0, keys_total = 0, queries = 0;
  auto run = [&](const Keys &k) {
    ++sets;
    keys_total += k.size();
    return Check(k, &rng, &queries);
  };
  // Word-like pieces, threaded placement.
  for (size_t n : {size_t(40000), size_t(90000)}) {
    Keys k;
    for (size_t i = 0; i < n; ++i) k.emplace_back(Word(&rng, 26, 10), static_cast<int32_t>(i));
    if (run(k)) return 1;
  }
  // Long shared prefixes: a few stems, each with many long continuations.
  {
    Keys k;
    std::vector<std::string> stems;
    for (int s = 0; s < 6; ++s) stems.push_back(std::string(20 + s * 7, static_cast<char>('A' + s)));
    for (int i = 0; i < 60000; ++i) {
      std::string w = stems[rng() % stems.size()] + Word(&rng, 4, 24);
      k.emplace_back(w, i);
    }
    if (run(k)) return 1;
  }
  // Arbitrary bytes with NULs, duplicates (first value wins) and empty keys.
  {
    Keys k;
    for (int i = 0; i < 50000; ++i) {
      std::string w;
      const int len = static_cast<int>(rng() % 7);
      for (int j = 0; j < len; ++j) w.push_back(static_cast<char>(rng() % 8 == 0 ? 0 : 128 + rng() % 128));
      k.emplace_back(w, i);
      if (i % 7 == 0) k.emplace_back(w, -5 - i);
    }
    k.emplace_back("", 1);
    if (run(k)) return 1;
  }
  // Small sets (one placement thread).
  for (int r = 0; r < 20; ++r) {
    Keys k;
    const int n = static_cast<int>(rng() % 3000);
    for (int i = 0; i < n; ++i) k.emplace_back(Word(&rng, 3 + r, 8), i);
    if (run(k)) return 1;
  }
  std::printf("{\"sets\": %zu, \"keys\": %zu, \"queries\": %zu}\n", sets, keys_total, queries);
  return 0;
}
