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

// Enqueues one batch (see bpe_kernels.hip); no host synchronization unless
// c.host_sized.
int EncodeBpe(spm_hip_model *m, EncodeWorkspace *ws, const EncodeCall &c, std::string *err);

}  // namespace spm_amd
