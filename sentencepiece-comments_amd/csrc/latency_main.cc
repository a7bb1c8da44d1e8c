// spm_latency — per-call latency of the drop-in's small-batch entry points.
//
// The reference's plugin point is ModelInterface::Encode(normalized), called
// once per line by spm_encode (spm_encode_main.cc:189-191) and by
// SentencePieceProcessor::Encode (sentencepiece_processor.cc:319-330); one
// CPU core does ~9.2 us per ~25-char sentence.  This tool times,
// on lines read from a file:
//   * SentencePieceProcessor::Encode(line, &ids) — one line per call (raw
//     text → device normalize → encode → id epilogue → host ids);
//   * spm_hip_encode_batch_host over B normalized sentences per call, for a
//     range of B — the batch size at which the device adapter beats the
//     reference's per-sentence cost.
// Prints one JSON object.
//
//   spm_latency MODEL LINES_FILE [calls]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "processor.h"

namespace {

double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

[[noreturn]] void Die(const std::string &m) {
  std::fprintf(stderr, "spm_latency: %s\n", m.c_str());
  std::exit(1);
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 3) Die("usage: spm_latency MODEL LINES_FILE [calls]");
  const int calls = argc > 3 ? std::atoi(argv[3]) : 2000;
  std::ifstream in(argv[2], std::ios::binary);
  if (!in) Die("cannot read lines");
  std::vector<std::string> lines;
  for (std::string l; std::getline(in, l);) lines.push_back(l);
  if (lines.empty()) Die("no lines");

  spm_amd::SentencePieceProcessor sp;
  auto st = sp.Load(argv[1]);
  if (!st.ok()) Die(st.message);
  std::vector<int> ids;
  // Warm-up: device tables, staging buffers, workspaces.
  for (int k = 0; k < 20; ++k)
    if (!(st = sp.Encode(lines[k % lines.size()], &ids)).ok()) Die(st.message);
  double t0 = Now();
  uint64_t toks = 0;
  for (int k = 0; k < calls; ++k) {
    st = sp.Encode(lines[k % lines.size()], &ids);
    if (!st.ok()) Die(st.message);
    toks += ids.size();
  }
  const double proc_us = (Now() - t0) * 1e6 / calls;
  // The whole file as one EncodeBatch(ids) call (raw lines -> device
  // normalize, encode and id epilogue -> host ids), best of a few.
  std::vector<std::vector<int>> all;
  double best = 1e30;
  for (int k = 0; k < 6; ++k) {
    const double b0 = Now();
    st = sp.EncodeBatch(lines, &all, nullptr);
    if (!st.ok()) Die(st.message);
    if (k > 0) best = std::min(best, Now() - b0);
  }

  // Normalized sentences for the C-ABI batches (host normalizer, untimed).
  std::string mb;
  {
    std::ifstream f(argv[1], std::ios::binary);
    mb.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  }
  spm_hip_model *m = nullptr;
  if (spm_hip_model_load(mb.data(), mb.size(), &m) != SPM_OK) Die(spm_hip_last_error());
  const uint64_t n = lines.size();
  std::vector<uint64_t> in_off(n + 1, 0);
  std::string raw;
  for (uint64_t i = 0; i < n; ++i) {
    raw += lines[i];
    in_off[i + 1] = raw.size();
  }
  std::vector<uint8_t> norm(raw.size() * 3 + 4 * n + 16);
  std::vector<uint64_t> norm_off(n + 1);
  if (spm_hip_normalize_batch(m, reinterpret_cast<const uint8_t *>(raw.data()), in_off.data(), n, norm.data(),
                              norm_off.data(), 0) != SPM_OK)
    Die(spm_hip_last_error());
  std::printf("{\"calls\": %d, \"encode_single_us\": %.3f, \"encode_single_tokens\": %llu, \"lines\": %llu, "
              "\"encode_file_s\": %.6f, \"encode_file_sentences_per_s\": %.1f, \"batches\": [",
              calls, proc_us, static_cast<unsigned long long>(toks), static_cast<unsigned long long>(n), best,
              n / best);
  bool first = true;
  for (uint64_t B : {1ull, 2ull, 4ull, 8ull, 16ull, 64ull, 256ull, 1024ull, 4096ull, 16384ull, 65536ull}) {
    if (B > n) break;
    const int reps = static_cast<int>(std::max<uint64_t>(8, std::min<uint64_t>(calls, 2000000 / B)));
    std::vector<int32_t> out_ids;
    std::vector<uint32_t> out_len;
    std::vector<uint64_t> tok(B + 1), off(B + 1);
    auto run = [&](uint64_t start) {
      const uint64_t base = norm_off[start];
      for (uint64_t i = 0; i <= B; ++i) off[i] = norm_off[start + i] - base;
      out_ids.resize(std::max<uint64_t>(off[B], 1));
      out_len.resize(std::max<uint64_t>(off[B], 1));
      if (spm_hip_encode_batch_host(m, norm.data() + base, off.data(), B, out_ids.data(), out_len.data(),
                                    tok.data()) != SPM_OK)
        Die(spm_hip_last_error());
    };
    for (int k = 0; k < 5; ++k) run((k * B) % (n - B + 1));
    const double b0 = Now();
    for (int k = 0; k < reps; ++k) run((k * B) % (n - B + 1));
    const double us = (Now() - b0) * 1e6 / reps;
    std::printf("%s{\"batch\": %llu, \"us_per_call\": %.3f, \"us_per_sentence\": %.4f, \"reps\": %d}",
                first ? "" : ", ", static_cast<unsigned long long>(B), us, us / B, reps);
    first = false;
  }
  std::printf("]}\n");
  spm_hip_model_free(m);
  return 0;
}
