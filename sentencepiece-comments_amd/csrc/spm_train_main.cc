// spm_train — drop-in for the reference CLI (src/spm_train_main.cc:26-221),
// --model_type=unigram, with seed mining, every E-step and the pruning
// Viterbi on the GPU.  Flags and defaults are the reference's; every flag is
// set into the TrainerSpec / NormalizerSpec as the reference's main() does
// (so the .model's serialized specs carry the same fields).
//
// Extension flags (not in the reference): --rules_dir (directory of
// <rule>.bin precompiled charsmaps, default <exe>/../../data/normalization),
// --dump_seeds (write the seed list: piece \t float bits), --estep_mode
// (parity|fast), --timings (print a JSON line of stage timings on stdout),
// --num_gpus (E-step / pruning-Viterbi ranks, one per GPU, RCCL reduce),
// --host_split (test/debug: the whitespace split on host threads, the device
// split's fallback), --em_checkpoint (write the piece list at the top of every
// EM round to this file) and --resume_from (continue from such a file; the
// same corpus and flags give the model of an uninterrupted run).
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "trainer.h"

namespace {

[[noreturn]] void Die(const std::string &msg) {
  std::cerr << msg << std::endl;
  std::exit(1);
}

std::string ExeDir() {
  char buf[4096];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return ".";
  std::string p(buf, n);
  return p.substr(0, p.rfind('/'));
}

}  // namespace

int main(int argc, char **argv) {
  using namespace spm_amd;
  // Flag defaults (spm_train_main.cc:26-93).
  std::map<std::string, std::string> f = {
      {"input", ""}, {"input_format", ""}, {"model_prefix", ""}, {"model_type", "unigram"},
      {"vocab_size", "8000"}, {"accept_language", ""}, {"self_test_sample_size", "0"},
      {"character_coverage", "0.9995"}, {"input_sentence_size", "0"},
      {"shuffle_input_sentence", "true"}, {"seed_sentencepiece_size", "1000000"},
      {"shrinking_factor", "0.75"}, {"num_threads", "16"}, {"num_sub_iterations", "2"},
      {"max_sentencepiece_length", "16"}, {"max_sentence_length", "4192"},
      {"split_by_unicode_script", "true"}, {"split_by_number", "true"},
      {"split_by_whitespace", "true"}, {"treat_whitespace_as_suffix", "false"},
      {"control_symbols", ""}, {"user_defined_symbols", ""},
      {"normalization_rule_name", "nmt_nfkc"}, {"normalization_rule_tsv", ""},
      {"add_dummy_prefix", "true"}, {"remove_extra_whitespaces", "true"},
      {"hard_vocab_limit", "true"}, {"use_all_vocab", "false"}, {"unk_id", "0"},
      {"bos_id", "1"}, {"eos_id", "2"}, {"pad_id", "-1"}, {"unk_piece", "<unk>"},
      {"bos_piece", "<s>"}, {"eos_piece", "</s>"}, {"pad_piece", "<pad>"},
      {"unk_surface", " \xE2\x81\x87 "},
      // extensions
      {"rules_dir", ExeDir() + "/../../data/normalization"}, {"dump_seeds", ""},
      {"estep_mode", "parity"}, {"timings", "false"}, {"host_threads", "0"}, {"num_gpus", "1"},
      {"host_split", "false"}, {"em_checkpoint", ""}, {"resume_from", ""}};
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.size() < 2 || a[0] != '-') Die("unknown argument: " + a);
    a = a.substr(a[1] == '-' ? 2 : 1);
    std::string k = a, v = "true";
    const size_t eq = a.find('=');
    if (eq != std::string::npos) {
      k = a.substr(0, eq);
      v = a.substr(eq + 1);
    } else if (i + 1 < argc && argv[i + 1][0] != '-') {
      v = argv[++i];
    }
    if (k == "help") {
      std::cout << "Usage: " << argv[0] << " [options]\n";
      for (auto &kv : f) std::cout << "   --" << kv.first << "  default: " << kv.second << "\n";
      return 0;
    }
    if (k == "version") {
      std::cout << "sentencepiece-mi355x 0.1.82" << std::endl;
      return 0;
    }
    if (!f.count(k)) Die("Unknown flag: " + k);
    f[k] = v;
  }
  if (f["input"].empty()) Die("--input must not be empty");
  if (f["model_prefix"].empty()) Die("--model_prefix must not be empty");

  TrainerSpec ts;
  NormalizerSpec ns;
  // SetTrainerSpecFromFlag for every flag (spm_train_main.cc:117-153).
  const char *kTrainerFlags[] = {
      "input_format", "model_prefix", "vocab_size", "self_test_sample_size", "character_coverage",
      "input_sentence_size", "shuffle_input_sentence", "seed_sentencepiece_size",
      "shrinking_factor", "num_threads", "num_sub_iterations", "max_sentencepiece_length",
      "max_sentence_length", "split_by_unicode_script", "split_by_whitespace", "split_by_number",
      "treat_whitespace_as_suffix", "hard_vocab_limit", "use_all_vocab", "unk_id", "bos_id",
      "eos_id", "pad_id", "unk_piece", "bos_piece", "eos_piece", "pad_piece", "unk_surface"};
  for (const char *k : kTrainerFlags) {
    Status s = SetTrainerField(k, f[k], &ts);
    if (!s.ok()) Die(s.message);
  }
  for (const char *k : {"input", "accept_language", "control_symbols", "user_defined_symbols"})
    if (!f[k].empty()) {
      Status s = SetTrainerField(k, f[k], &ts);
      if (!s.ok()) Die(s.message);
    }
  ns.name = f["normalization_rule_name"];
  ns.has.insert(1);
  for (const char *k : {"normalization_rule_tsv", "add_dummy_prefix", "remove_extra_whitespaces"}) {
    Status s = SetNormalizerField(k, f[k], &ns);
    if (!s.ok()) Die(s.message);
  }
  {
    Status s = SetTrainerField("model_type", f["model_type"], &ts);
    if (!s.ok()) Die(s.message);
  }
  // (read by the trainer from its environment, trainer.cc Train)
  if (!f["em_checkpoint"].empty()) setenv("SPM_HIP_EM_CHECKPOINT", f["em_checkpoint"].c_str(), 1);
  if (!f["resume_from"].empty()) setenv("SPM_HIP_EM_RESUME", f["resume_from"].c_str(), 1);
  TrainerOptions opt;
  opt.rules_dir = f["rules_dir"];
  opt.dump_seeds = f["dump_seeds"];
  opt.estep_mode = f["estep_mode"] == "fast" ? SPM_ESTEP_FAST : SPM_ESTEP_PARITY;
  opt.host_threads = std::atoi(f["host_threads"].c_str());
  opt.num_gpus = std::atoi(f["num_gpus"].c_str());
  opt.host_split = f["host_split"] == "true";
  if (opt.num_gpus < 1 || opt.num_gpus > 64) Die("--num_gpus must be in [1, 64]");
  TrainerTimings tm;
  Status s = SentencePieceTrainer::Train(ts, ns, opt, &tm);
  if (!s.ok()) Die(s.message);
  if (f["timings"] == "true") {
    std::printf(
        "{\"load_s\": %.4f, \"seed_s\": %.4f, \"seed_device_ms\": %.3f, \"seed_candidates\": %llu, "
        "\"split_s\": %.4f, \"estep_s\": %.4f, \"mstep_s\": %.4f, \"prune_s\": %.4f, "
        "\"finalize_s\": %.4f, \"total_s\": %.4f, \"sentences\": %llu, \"em_sentences\": %llu, "
        "\"em_iterations\": %d, \"bpe_update_s\": %.4f, \"bpe_update_freq_s\": %.4f, "
        "\"bpe_update_scan_s\": %.4f, \"bpe_update_sort_s\": %.4f, "
        "\"bpe_dirty_s\": %.4f, \"bpe_apply_s\": %.4f, \"bpe_positions\": %llu, \"bpe_refreshed\": %llu, "
        "\"bpe_updates\": %llu, \"bpe_update_replays\": %llu, \"bpe_refresh_device_ms\": %.3f, "
        "\"bpe_refresh_checked\": %llu, \"bpe_refresh_prep_s\": %.4f, \"bpe_refresh_call_s\": %.4f, "
        "\"bpe_refresh_post_s\": %.4f, \"bpe_refresh_erased\": %llu, "
        "\"read_s\": %.4f, \"trie_build_s\": %.4f, "
        "\"peak_device_bytes\": %llu, \"stage_peak_bytes\": [%llu, %llu, %llu, %llu], "
        "\"seed_stages_ms\": [%.2f, %.2f, %.2f, %.2f, %.2f, %.2f, %.0f]}\n",
        tm.load, tm.seed, tm.seed_device_ms, static_cast<unsigned long long>(tm.seed_candidates),
        tm.split, tm.estep, tm.mstep, tm.prune, tm.finalize, tm.total,
        static_cast<unsigned long long>(tm.sentences),
        static_cast<unsigned long long>(tm.em_sentences), tm.em_iterations, tm.bpe_update, tm.bpe_update_freq,
        tm.bpe_update_scan, tm.bpe_update_sort, tm.bpe_dirty, tm.bpe_apply, static_cast<unsigned long long>(tm.bpe_positions),
        static_cast<unsigned long long>(tm.bpe_refreshed), static_cast<unsigned long long>(tm.bpe_updates),
        static_cast<unsigned long long>(tm.bpe_update_replays), tm.bpe_refresh_device_ms,
        static_cast<unsigned long long>(tm.bpe_refresh_checked), tm.bpe_refresh_prep, tm.bpe_refresh_call,
        tm.bpe_refresh_post, static_cast<unsigned long long>(tm.bpe_refresh_erased), tm.read, tm.trie_build,
        static_cast<unsigned long long>(tm.peak_device_bytes),
        static_cast<unsigned long long>(tm.stage_peak_bytes[0]), static_cast<unsigned long long>(tm.stage_peak_bytes[1]),
        static_cast<unsigned long long>(tm.stage_peak_bytes[2]), static_cast<unsigned long long>(tm.stage_peak_bytes[3]),
        tm.seed_stages[0],
        tm.seed_stages[1],
        tm.seed_stages[2], tm.seed_stages[3], tm.seed_stages[4], tm.seed_stages[5], tm.seed_stages[6]);
  }
  return 0;
}
