// BPE model on the device: tables (host build) + encode launch.
// Reference: bpe::Model::Encode (bpe_model.cc:37-199).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "device_model.h"

namespace spm_amd {

// Builds the string trie (pieces_ ∪ reserved_id_map_ strings), the per-string
// entry table and the (left piece, right piece) → merged piece hash table.
int LoadBpe(spm_hip_model *m, std::string *err);

int EncodeBpe(spm_hip_model *m, EncodeWorkspace *ws, const uint8_t *d_bytes, const uint64_t *d_off, uint64_t n,
              uint64_t total, uint32_t max_nb_hint, int32_t *d_ids, uint32_t *d_len,
              uint64_t *d_tok, hipStream_t st, std::string *err);

}  // namespace spm_amd
