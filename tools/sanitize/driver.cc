// Host sanitizer driver (SURVEY §5 race/failure detection).
// Built with -fsanitize=address,undefined over the product's host sources
// that parse or walk untrusted data: model_proto.cc (.model bytes),
// double_array.cc (trie build + walks) and normalizer.cc (the precompiled
// charsmap blob, PrefixMatcher).  For every .model file given:
//   * the intact file, every truncation on a stride, and seeded bit flips
//     go through ParseModelProto; whatever parses is then exercised:
//   * BuildDoubleArray over its pieces, each piece looked up (ExactMatch,
//     CommonPrefixSearch) and checked against the piece table;
//   * a Normalizer over its NormalizerSpec (with the charsmap blob as
//     parsed, so corrupted blobs too) + a PrefixMatcher of its user-defined
//     pieces normalizes the lines of the given text file.
// Any sanitizer report aborts the process (halt_on_error); the exit code and
// a summary line tell tests/test_sanitize_cpu.py the result.
//
//   driver TEXT_FILE MODEL...
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "double_array.h"
#include "model_proto.h"
#include "normalizer.h"

using namespace spm_amd;

static std::string ReadAll(const char *p) {
  std::ifstream f(p, std::ios::binary);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static int g_flip_cases = 160, g_cut_cases = 160, g_charsmap_cases = 400;
static uint64_t g_parsed = 0, g_rejected = 0, g_norm_bytes = 0, g_lookups = 0;

static int Exercise(const ModelProtoView &mp, const std::vector<std::string> &lines, bool intact,
                    bool trie = true) {
  std::vector<std::pair<std::string, int32_t>> keys;
  std::vector<std::string> user;
  for (size_t i = 0; i < mp.pieces.size(); ++i) {
    const auto &p = mp.pieces[i];
    if (p.type == kNormal || p.type == kUserDefined || p.type == kUnused)
      keys.emplace_back(p.piece, static_cast<int32_t>(i));
    if (p.type == kUserDefined) user.push_back(p.piece);
  }
  DoubleArray da;
  std::string err;
  if (trie && BuildDoubleArray(keys, &da, &err)) {
    // First value of every NUL-truncated key, as the build keeps it.
    std::map<std::string, int32_t> first;
    for (const auto &k : keys) first.emplace(k.first.substr(0, k.first.find('\0')), k.second);
    std::vector<std::pair<int32_t, size_t>> hits;
    for (const auto &k : first) {
      if (k.first.empty()) continue;
      const int32_t v = da.ExactMatch(k.first.data(), k.first.size());
      ++g_lookups;
      if (intact && v != k.second) {
        std::fprintf(stderr, "ExactMatch mismatch for a piece: %d vs %d\n", v, k.second);
        return 1;
      }
      da.CommonPrefixSearch(k.first.data(), k.first.size(), &hits);
      if (intact && (hits.empty() || hits.back().second != k.first.size())) {
        std::fprintf(stderr, "CommonPrefixSearch misses a piece\n");
        return 1;
      }
    }
  }
  PrefixMatcher pm(user);
  Normalizer nz(mp.normalizer_spec, mp.trainer_spec.treat_whitespace_as_suffix);
  if (!nz.ok()) return 0;
  nz.SetPrefixMatcher(&pm);
  std::string out;
  std::vector<size_t> n2o;
  for (const auto &l : lines) {
    nz.Normalize(l.data(), l.size(), &out, &n2o);
    g_norm_bytes += out.size();
    if (n2o.size() != out.size() + 1 && !(out.empty() && n2o.empty())) {
      std::fprintf(stderr, "norm_to_orig size %zu for %zu bytes\n", n2o.size(), out.size());
      return 1;
    }
  }
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  if (const char *e = std::getenv("SANITIZE_CASES")) {  // flips,cuts,charsmap
    std::sscanf(e, "%d,%d,%d", &g_flip_cases, &g_cut_cases, &g_charsmap_cases);
  }
  std::vector<std::string> lines;
  {
    std::ifstream f(argv[1], std::ios::binary);
    for (std::string l; std::getline(f, l) && lines.size() < 400;) lines.push_back(l);
  }
  // Edge inputs: empty, spaces only, broken UTF-8, NUL, long runs.
  lines.push_back("");
  lines.push_back("   ");
  lines.push_back(std::string("\xff\xfe\xe3\x81", 4));
  lines.push_back(std::string("a\0b", 3));
  lines.push_back(std::string(3000, 'x'));
  std::mt19937_64 rng(12345);
  for (int a = 2; a < argc; ++a) {
    const std::string blob = ReadAll(argv[a]);
    std::vector<std::string> cases;
    cases.push_back(blob);
    const size_t stride = std::max<size_t>(1, blob.size() / g_cut_cases);
    for (size_t cut = 0; cut < blob.size(); cut += stride) cases.push_back(blob.substr(0, cut));
    for (int k = 0; k < g_flip_cases; ++k) {
      std::string b = blob;
      const int flips = 1 + static_cast<int>(rng() % 4);
      for (int f = 0; f < flips; ++f) b[rng() % b.size()] ^= static_cast<char>(1u << (rng() % 8));
      cases.push_back(b);
    }
    // Targeted: the intact model with its charsmap blob corrupted (header,
    // trie units, pool), so the normalizer's walks see arbitrary units.
    {
      ModelProtoView mp;
      std::string err;
      if (ParseModelProto(reinterpret_cast<const uint8_t *>(blob.data()), blob.size(), &mp, &err) &&
          mp.normalizer_spec.precompiled_charsmap.size() > 8) {
        const std::string cm = mp.normalizer_spec.precompiled_charsmap;
        for (int k = 0; k < g_charsmap_cases; ++k) {
          std::string b = cm;
          if (k % 8 == 0) {
            const uint32_t ts = static_cast<uint32_t>(rng() % (b.size() + 16));
            std::memcpy(&b[0], &ts, 4);
          }
          const int flips = 1 + static_cast<int>(rng() % 64);
          for (int f = 0; f < flips; ++f) b[rng() % b.size()] ^= static_cast<char>(1u << (rng() % 8));
          if (k % 5 == 0) b.resize(4 + rng() % (b.size() - 4));
          ModelProtoView m2 = mp;
          m2.normalizer_spec.precompiled_charsmap = b;
          ++g_parsed;
          if (Exercise(m2, lines, false, false)) return 1;
        }
      }
    }
    for (size_t c = 0; c < cases.size(); ++c) {
      ModelProtoView mp;
      std::string err;
      if (!ParseModelProto(reinterpret_cast<const uint8_t *>(cases[c].data()), cases[c].size(), &mp, &err)) {
        ++g_rejected;
        continue;
      }
      ++g_parsed;
      if (Exercise(mp, lines, c == 0)) {
        std::fprintf(stderr, "check failed: %s case %zu\n", argv[a], c);
        return 1;
      }
    }
  }
  std::printf("{\"parsed\": %llu, \"rejected\": %llu, \"lookups\": %llu, \"normalized_bytes\": %llu}\n",
              (unsigned long long)g_parsed, (unsigned long long)g_rejected, (unsigned long long)g_lookups,
              (unsigned long long)g_norm_bytes);
  return 0;
}
