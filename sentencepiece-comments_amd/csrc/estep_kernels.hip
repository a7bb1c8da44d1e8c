// Unigram trainer E-step (placeholder until the kernel lands).
#include <hip/hip_runtime.h>

#include "../../include/spm_hip.h"

extern "C" {
int spm_hip_pieces_create(const uint8_t *, const uint64_t *, const float *, uint64_t,
                          spm_hip_pieces **out) {
  if (out) *out = nullptr;
  return SPM_UNIMPLEMENTED;
}
void spm_hip_pieces_free(spm_hip_pieces *) {}
int spm_hip_estep(spm_hip_pieces *, const uint8_t *, const uint64_t *, const int64_t *, uint64_t,
                  int64_t, int, int, float *, float *, int64_t *, void *) {
  return SPM_UNIMPLEMENTED;
}
}
