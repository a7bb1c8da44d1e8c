// Kernel launch interfaces (internal; the public boundary is include/spm_hip.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_model.h"

namespace spm_amd {

struct UnigramLaunch {
  const uint8_t *bytes;
  const uint64_t *off;
  uint64_t n;
  const uint32_t *units;
  const int32_t *values;
  const float *scores;
  UnigramParams p;
  int32_t *slot_ids;
  uint32_t *slot_len;
  uint32_t *ntok;
  uint8_t *bp;
  uint32_t *flagged;
  uint32_t *status;
};

hipError_t LaunchUnigramFast(int ring_width, const UnigramLaunch &l, hipStream_t st);
hipError_t LaunchUnigramGeneral(const UnigramLaunch &l, const uint32_t *list, const uint32_t *count,
                                uint64_t list_n, uint8_t *scratch, uint64_t slab_bytes,
                                uint32_t max_nb, uint32_t threads, uint32_t *error,
                                hipStream_t st);
uint64_t UnigramGeneralSlabBytes(uint32_t max_nb, int trie_results_size);

// Dense CSR output from right-aligned slots: tok_off = exclusive scan of
// ntok; ids/len copied out of [off[i+1]-ntok[i], off[i+1]).
hipError_t LaunchCompact(const uint64_t *off, uint64_t n, const uint32_t *ntok,
                         const int32_t *slot_ids, const uint32_t *slot_len, int32_t *ids,
                         uint32_t *piece_len, uint64_t *tok_off, void *scan_tmp,
                         size_t *scan_tmp_bytes, hipStream_t st);

}  // namespace spm_amd
