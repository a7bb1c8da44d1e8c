// C++ mirror of sentencepiece::SentencePieceTrainer / unigram::Trainer
// (reference src/sentencepiece_trainer.{h,cc}, src/trainer_interface.{h,cc},
// src/unigram_model_trainer.{h,cc}) on top of the C-ABI.
//
// Host side: spec parsing (MergeSpecsFromArgs / SetProtoField), LoadSentences
// (threaded normalization and char counting), the whitespace split, the
// M-step, the pruning loss, FinalizeSentencePieces and the .model / .vocab
// writers.  Device side, through include/spm_hip.h: seed mining
// (spm_hip_seed_mine), every E-step (spm_hip_estep, PARITY mode with
// T = num_threads ordered buckets, so results are bit-identical to the
// reference at that thread count) and the pruning Viterbi over all sentences
// (spm_hip_encode_batch on a TrainerModel built by spm_hip_model_from_pieces).
#pragma once

#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "../../include/spm_hip.h"
#include "processor.h"

namespace spm_amd {

// TrainerSpec (sentencepiece_model.proto:26-200) with proto2 presence bits:
// only fields that were set are serialized into the .model, as protobuf does.
struct TrainerSpec {
  std::vector<std::string> input;
  std::string input_format;
  std::string model_prefix;
  int32_t model_type = 1;  // UNIGRAM
  int32_t vocab_size = 8000;
  std::vector<std::string> accept_language;
  int32_t self_test_sample_size = 0;
  float character_coverage = 0.9995f;
  int32_t input_sentence_size = 0;
  bool shuffle_input_sentence = true;
  int32_t seed_sentencepiece_size = 1000000;
  float shrinking_factor = 0.75f;
  int32_t max_sentence_length = 4192;
  int32_t num_threads = 16;
  int32_t num_sub_iterations = 2;
  int32_t max_sentencepiece_length = 16;
  bool split_by_unicode_script = true;
  bool split_by_number = true;
  bool split_by_whitespace = true;
  bool treat_whitespace_as_suffix = false;
  std::vector<std::string> control_symbols;
  std::vector<std::string> user_defined_symbols;
  bool hard_vocab_limit = true;
  bool use_all_vocab = false;
  int32_t unk_id = 0, bos_id = 1, eos_id = 2, pad_id = -1;
  std::string unk_surface = " \xE2\x81\x87 ";
  std::string unk_piece = "<unk>", bos_piece = "<s>", eos_piece = "</s>", pad_piece = "<pad>";
  std::set<int> has;  // field numbers explicitly set
};

// NormalizerSpec (sentencepiece_model.proto:202-232).
struct NormalizerSpec {
  std::string name;
  std::string precompiled_charsmap;
  bool add_dummy_prefix = true;
  bool remove_extra_whitespaces = true;
  bool escape_whitespaces = true;
  std::string normalization_rule_tsv;
  std::set<int> has;
};

// SetProtoField (spec_parser.h) for one "--key=value".  NOT_FOUND if the key
// is not a field of the spec.
Status SetTrainerField(const std::string &key, const std::string &value, TrainerSpec *spec);
Status SetNormalizerField(const std::string &key, const std::string &value, NormalizerSpec *spec);

struct TrainerOptions {
  std::string rules_dir;      // where <rule name>.bin charsmap blobs live
  std::string dump_seeds;     // if set, seed pieces are written here (piece\tscore)
  bool verbose = true;        // LOG(INFO)-style progress on stderr
  int host_threads = 0;       // 0 = hardware concurrency
  int estep_mode = SPM_ESTEP_PARITY;
  // E-step and pruning-Viterbi ranks, one per GPU of this process (RCCL
  // reduce onto rank 0); more ranks than GPUs share devices (host reduce).
  int num_gpus = 1;
  // Test/debug: run SplitSentencesByWhitespace on the host (the device
  // split's fallback path) even when the corpus is resident on the device.
  bool host_split = false;
};

// Timings of the last Train() (seconds, host wall clock).
struct TrainerTimings {
  double load = 0, seed = 0, split = 0, estep = 0, mstep = 0, prune = 0, finalize = 0, total = 0;
  double seed_device_ms = 0;
  // Host time inside load's file read + line parse, and in the trie builds
  // (piece sets for the E-steps and pruning: spm_hip_pieces_create,
  // spm_hip_model_from_pieces, the NBest trie).
  double read = 0, trie_build = 0;
  float seed_stages[7] = {};  // spm_hip_seeds_stage_times
  uint64_t sentences = 0, seed_candidates = 0, em_sentences = 0;
  int em_iterations = 0;
  // BPE merge loop breakdown (model_type=bpe): UpdateActiveSymbols (every
  // 100 merges; its ComputeFreq over all bigrams separately), the dirty
  // symbols' ComputeFreq before each selection, and applying each merge to
  // its positions.
  double bpe_update = 0, bpe_update_freq = 0, bpe_update_scan = 0, bpe_update_sort = 0, bpe_dirty = 0, bpe_apply = 0;
  uint64_t bpe_positions = 0, bpe_refreshed = 0, bpe_updates = 0, bpe_update_replays = 0;
  uint64_t bpe_refresh_checked = 0;  // refreshes cross-checked on the host (SPM_HIP_BPE_REFRESH_CHECK=1)
  float bpe_refresh_device_ms = 0;   // device time of the refreshes (spm_hip_bpe_refresh_stats)
  // host side of the device refresh: logs -> inputs, the call, erasures applied to the host sets
  double bpe_refresh_prep = 0, bpe_refresh_call = 0, bpe_refresh_post = 0;
  uint64_t bpe_refresh_erased = 0;
  // Device bytes live at the high-water mark of the whole run and of each
  // stage: load, seed mining, whitespace split + rank setup, EM + pruning +
  // finalize (the BPE merge loop for model_type=bpe).
  uint64_t peak_device_bytes = 0, stage_peak_bytes[4] = {};
};

class SentencePieceTrainer {
 public:
  // SentencePieceTrainer::Train(args) (sentencepiece_trainer.cc:53-107).
  static Status Train(const std::string &args, const TrainerOptions &opt = TrainerOptions(),
                      TrainerTimings *timings = nullptr);
  // SentencePieceTrainer::Train(trainer_spec, normalizer_spec).
  static Status Train(const TrainerSpec &trainer_spec, const NormalizerSpec &normalizer_spec,
                      const TrainerOptions &opt = TrainerOptions(),
                      TrainerTimings *timings = nullptr);
  static Status MergeSpecsFromArgs(const std::string &args, TrainerSpec *trainer_spec,
                                   NormalizerSpec *normalizer_spec);
  // PopulateNormalizerSpec (:109-136) with rule blobs read from rules_dir.
  static Status PopulateNormalizerSpec(NormalizerSpec *spec, const std::string &rules_dir);
};

// ModelProto serialization of a finished vocabulary (trainer_interface.cc:
// Serialize :479-530).  pieces: (piece, score, type).
std::string SerializeModelProto(const std::vector<PieceRec> &pieces, const TrainerSpec &ts,
                                const NormalizerSpec &ns);

}  // namespace spm_amd
