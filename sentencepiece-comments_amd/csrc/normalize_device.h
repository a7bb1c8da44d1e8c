// Device normalizer tables and launchers (normalize_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace spm_amd {

struct NormTables {
  const uint32_t *units = nullptr;   // charsmap darts-clone units (null: identity)
  uint32_t num_units = 0;
  const uint8_t *pool = nullptr;     // NUL-terminated replacement strings (+ a NUL after the blob)
  uint32_t pool_size = 0;            // pool bytes (values must be below)
  const uint32_t *ud_units = nullptr;  // user-defined symbols (DoubleArray), or null
  uint32_t ud_num_units = 0;
  bool add_dummy_prefix = true, remove_extra_whitespaces = true, escape_whitespaces = true;
  bool suffix = false;               // treat_whitespace_as_suffix
};

// COUNT pass: normalized byte length of every sentence.  chain (nullable):
// an asynchronous call's status word; the kernels do nothing once it is
// non-zero.
hipError_t NormalizeLengths(const NormTables &t, const uint8_t *d_in, const uint64_t *d_in_off,
                            uint64_t n, uint64_t *d_len, hipStream_t st, uint32_t *chain = nullptr);
// WRITE pass into CSR offsets computed from the lengths; d_n2o (optional):
// norm_to_orig, len + 1 uint32 entries per sentence at d_n2o[out_off[i] + i].
// An output larger than cap_limit is not written (chain := RESOURCE_EXHAUSTED).
hipError_t NormalizeWrite(const NormTables &t, const uint8_t *d_in, const uint64_t *d_in_off,
                          uint64_t n, uint8_t *d_out, const uint64_t *d_out_off, hipStream_t st,
                          uint32_t *d_n2o = nullptr, uint64_t cap_limit = ~0ull, uint32_t *chain = nullptr);
// PrefixMatcher::GlobalReplace(meta pieces → "\t"), two passes; *d_any = 1
// when any sentence changes.
hipError_t MetaReplaceLengths(const uint32_t *units, uint32_t num_units, const uint8_t *d_in,
                              const uint64_t *d_in_off, uint64_t n, uint64_t *d_len, uint32_t *d_any,
                              hipStream_t st);
hipError_t MetaReplaceWrite(const uint32_t *units, uint32_t num_units, const uint8_t *d_in,
                            const uint64_t *d_in_off, uint64_t n, uint8_t *d_out,
                            const uint64_t *d_out_off, hipStream_t st);
// lengths → CSR offsets (call with tmp = null first to size the scratch).
hipError_t LengthsToOffsets(const uint64_t *d_len, uint64_t n, uint64_t *d_off, void *tmp,
                            size_t *tmp_bytes, hipStream_t st);

}  // namespace spm_amd

namespace spm_amd {

// Trainer corpus passes (corpus_kernels.hip), one sentence per lane.
// Char histogram of LoadSentences (trainer_interface.cc:401-420): counts[cp]
// += freq for every valid code point except NUL and U+0020; flags bit 0: a
// U+0020 was seen, bit 1: a NUL, bit 2: an empty sentence.
hipError_t CorpusCharHistogram(const uint8_t *d_bytes, const uint64_t *d_off, const int64_t *d_freq,
                               uint64_t n, unsigned long long *d_counts /*0x110000*/,
                               uint32_t *d_flags, hipStream_t st);
// Rare chars → U+2585 (:444-455): required = bitmap over code points.
hipError_t CorpusReplaceLengths(const uint8_t *d_bytes, const uint64_t *d_off, uint64_t n,
                                const uint32_t *d_required_bits, uint64_t *d_len, hipStream_t st);
hipError_t CorpusReplaceWrite(const uint8_t *d_bytes, const uint64_t *d_off, uint64_t n,
                              const uint32_t *d_required_bits, uint8_t *d_out,
                              const uint64_t *d_out_off, hipStream_t st);
// out sentence k = in sentence idx[k] (CSR gather; d_len = lengths in new order).
hipError_t CorpusGatherLengths(const uint64_t *d_off, const uint64_t *d_idx, uint64_t m,
                               uint64_t *d_len, hipStream_t st);
hipError_t CorpusGatherWrite(const uint8_t *d_bytes, const uint64_t *d_off, const int64_t *d_freq,
                             const uint64_t *d_idx, uint64_t m, uint8_t *d_out,
                             const uint64_t *d_out_off, int64_t *d_out_freq, hipStream_t st);

// The lines of a text file already in device memory, as LoadSentences reads
// them (trainer_interface.cc:269-331 without a sentence selector): std::getline
// semantics (filesystem.cc:42-44), empty lines and lines holding kUNKStr
// dropped, lines longer than max_len bytes dropped and counted.  The kept
// lines become a device CSR with freq 1; the caller owns (hipFree) bytes,
// off and freq.  hipErrorInvalidValue: an empty file or >= 2^31 lines (the
// caller takes the host path).
struct ParsedLines {
  uint8_t *bytes = nullptr;
  uint64_t *off = nullptr;
  int64_t *freq = nullptr;
  uint64_t n = 0, total = 0, lines = 0, too_long = 0;
};
hipError_t CorpusParseLines(const uint8_t *d_file, uint64_t size, int64_t max_len, ParsedLines *out,
                            hipStream_t st);

// SplitSentencesByWhitespace (trainer_interface.cc:465-477, SplitIntoWords
// model_interface.cc:155-190) on the device (split_kernels.hip): the unique
// words (any order; the caller applies Sorted) with summed freqs, on the host.
// fallback: the device could not decide (a 64-bit hash collision between two
// different words, or >= 2^31 word occurrences): run the host split.
struct SplitWords {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off;
  std::vector<int64_t> freq;
  uint64_t occurrences = 0;
  bool fallback = false;
};
hipError_t CorpusSplitWords(const uint8_t *d_text, const uint64_t *d_off, const int64_t *d_freq, uint64_t n,
                            bool suffix, SplitWords *out, hipStream_t st);

}  // namespace spm_amd
