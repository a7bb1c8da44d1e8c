// Kernel launch interfaces (internal; the public boundary is include/spm_hip.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_types.h"

namespace spm_amd {

struct UnigramLaunch {
  const uint8_t *bytes;
  const uint64_t *off;
  uint64_t n;
  const uint32_t *units;
  const int32_t *values;
  const float *scores;
  UnigramParams p;
  int32_t *slot_ids;    // fast kernel: block-dense slots (group of 256 sentences)
  uint32_t *slot_len;
  int32_t *slot2_ids;   // general kernel: right-aligned in the sentence's own range
  uint32_t *slot2_len;
  uint32_t *ntok;
  uint32_t *lo;         // per sentence: offset in its group's dense slots, or ~0 → slot2
  uint8_t *bp;
  uint32_t *flagged;
  uint32_t *status;
  const float *vscore;  // per-unit leaf score / NaN kind tag
  uint32_t num_units;
  const uint2 *jump2 = nullptr;  // {unit, score} after two bytes (kVar & 4096)
};

// variant bits: 1 LDS-staged bytes, 2 LDS trie top, 4 per-unit score table
// (W = 32/64 support variants 0 and 7 only).
hipError_t LaunchUnigramFast(int ring_width, int variant, const UnigramLaunch &l, hipStream_t st);
// Lane-decoupled byte-position pass (unigram_lane_kernel.hip): units = the
// 0xFF-padded image, vscore = the per-unit usable-node scores, bp = scratch of
// total + 8 n + 16 bytes.  Same outputs and flags as LaunchUnigramFast.
// uvs: per unit {0xFF-padded unit, usable-node score bits} (opt & 1); opt & 2
// stages the top of it in LDS.  Variant = kLaneVariant | opt.
constexpr int kLaneVariant = 8192;
hipError_t LaunchUnigramLane(int opt, const UnigramLaunch &l, const uint2 *uvs, hipStream_t st);
hipError_t LaunchUnigramGeneral(const UnigramLaunch &l, const uint32_t *list, const uint32_t *count,
                                uint64_t list_n, uint8_t *scratch, uint64_t slab_bytes,
                                uint32_t max_nb, uint32_t threads, uint32_t *error,
                                hipStream_t st);
uint64_t UnigramGeneralSlabBytes(uint32_t max_nb, int trie_results_size);

// Dense CSR output: tok_off = exclusive scan of ntok; sentence i's tokens
// come from slot[off[i & ~255] + lo[i]] (fast unigram path: dense per group
// of 256 sentences) or, when lo[i] == ~0, from slot2[off[i+1]-ntok[i]]
// (right-aligned in the sentence's own byte range).
hipError_t LaunchCompact(const uint64_t *off, uint64_t n, const uint32_t *ntok, const uint32_t *lo,
                         const int32_t *slot_ids, const uint32_t *slot_len,
                         const int32_t *slot2_ids, const uint32_t *slot2_len, int32_t *ids,
                         uint32_t *piece_len, uint64_t *tok_off, void *scan_tmp,
                         size_t *scan_tmp_bytes, hipStream_t st);

}  // namespace spm_amd
