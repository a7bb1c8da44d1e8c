// Unigram trainer host code (see trainer.h).  Reference citations are to
// /root/reference/src/*.cc of SentencePiece v0.1.82.
#include "trainer.h"
#include "trace.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <functional>
#include <iostream>
#include <memory>
#include <queue>
#include <random>
#include <sstream>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "double_array.h"
#include "heap_select.h"
#include "normalize_device.h"
#include "normalizer.h"
#include "scratch_cache.h"
#include "shard_plan.h"
#include "unicode_script_table.h"

namespace spm_amd {
namespace {

constexpr uint32_t kUNKChar = 0x2585, kUPPBoundaryChar = 0x09;
const char kUNKStr[] = "\xe2\x96\x85";
const char kWSStr[] = "\xe2\x96\x81";

Status Err(int code, const std::string &msg) {
  Status s;
  s.code = code;
  s.message = msg;
  return s;
}

#define RETURN_IF_ERROR(expr)   \
  do {                          \
    Status _s = (expr);         \
    if (!_s.ok()) return _s;    \
  } while (0)

double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Host worker count: the request, else OMP_NUM_THREADS (the GPU box sets it
// to the job's CPU share), else hardware concurrency; at most 64.
int HostThreads(int req) {
  int t = req;
  if (t <= 0) {
    const char *e = std::getenv("OMP_NUM_THREADS");
    t = e ? std::atoi(e) : 0;
  }
  if (t <= 0) t = static_cast<int>(std::thread::hardware_concurrency());
  return std::max(1, std::min(t, 64));
}

// Runs f(t, lo, hi) over [0, n) split in contiguous chunks.
void ParallelChunks(uint64_t n, int threads, const std::function<void(int, uint64_t, uint64_t)> &f) {
  const int T = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(threads, n / 1024 + 1)));
  if (T == 1) {
    f(0, 0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back([&, t]() { f(t, n * t / T, n * (t + 1) / T); });
  for (auto &x : th) x.join();
}

// ---- UTF-8 (util.cc:187-331) ----------------------------------------------
uint32_t DecodeUTF8(const char *b, const char *e, size_t *mblen) {
  const size_t len = e - b;
  const unsigned char c0 = b[0];
  auto trail = [](char x) { return (static_cast<unsigned char>(x) & 0xC0) == 0x80; };
  auto valid = [](uint32_t c) { return c < 0xD800 || (c >= 0xE000 && c <= 0x10FFFF); };
  if (c0 < 0x80) {
    *mblen = 1;
    return c0;
  } else if (len >= 2 && (c0 & 0xE0) == 0xC0) {
    const uint32_t cp = ((c0 & 0x1F) << 6) | (b[1] & 0x3F);
    if (trail(b[1]) && cp >= 0x80 && valid(cp)) {
      *mblen = 2;
      return cp;
    }
  } else if (len >= 3 && (c0 & 0xF0) == 0xE0) {
    const uint32_t cp = ((c0 & 0x0F) << 12) | ((b[1] & 0x3F) << 6) | (b[2] & 0x3F);
    if (trail(b[1]) && trail(b[2]) && cp >= 0x800 && valid(cp)) {
      *mblen = 3;
      return cp;
    }
  } else if (len >= 4 && (c0 & 0xF8) == 0xF0) {
    const uint32_t cp = ((c0 & 0x07) << 18) | ((b[1] & 0x3F) << 12) | ((b[2] & 0x3F) << 6) |
                        (b[3] & 0x3F);
    if (trail(b[1]) && trail(b[2]) && trail(b[3]) && cp >= 0x10000 && valid(cp)) {
      *mblen = 4;
      return cp;
    }
  }
  *mblen = 1;
  return 0xFFFD;
}
bool IsValidCodepoint(uint32_t c) { return c < 0xD800 || (c >= 0xE000 && c <= 0x10FFFF); }
void AppendUTF8(uint32_t c, std::string *out) {
  if (c <= 0x7F) {
    out->push_back(char(c));
  } else if (c <= 0x7FF) {
    out->push_back(char(0xC0 | (c >> 6)));
    out->push_back(char(0x80 | (c & 0x3F)));
  } else {
    if (c > 0x10FFFF) c = 0xFFFD;
    if (c <= 0xFFFF) {
      out->push_back(char(0xE0 | (c >> 12)));
      out->push_back(char(0x80 | ((c >> 6) & 0x3F)));
      out->push_back(char(0x80 | (c & 0x3F)));
    } else {
      out->push_back(char(0xF0 | (c >> 18)));
      out->push_back(char(0x80 | ((c >> 12) & 0x3F)));
      out->push_back(char(0x80 | ((c >> 6) & 0x3F)));
      out->push_back(char(0x80 | (c & 0x3F)));
    }
  }
}

// string_util::Split(str, delim) with allow_empty = false (util.cc:33-49).
std::vector<std::string> Split(const std::string &v, char delim) {
  std::vector<std::string> r;
  size_t cur = 0, found;
  while ((found = v.find(delim, cur)) != std::string::npos) {
    if (found > cur) r.push_back(v.substr(cur, found - cur));
    cur = found + 1;
  }
  if (v.size() > cur) r.push_back(v.substr(cur));
  return r;
}

// trainer_interface.h:35-43
template <typename K, typename V>
std::vector<std::pair<K, V>> Sorted(std::vector<std::pair<K, V>> v) {
  std::sort(v.begin(), v.end(), [](const std::pair<K, V> &a, const std::pair<K, V> &b) {
    return a.second > b.second || (a.second == b.second && a.first < b.first);
  });
  return v;
}

// ---- spec parsing (spec_parser.h, util.h lexical_cast) ---------------------
template <typename T>
bool LexicalCast(const std::string &arg, T *out) {
  std::stringstream ss;
  return static_cast<bool>(ss << arg) && static_cast<bool>(ss >> *out);
}
bool LexicalCastBool(const std::string &arg, bool *out) {
  std::string v = arg;
  std::transform(v.begin(), v.end(), v.begin(), ::tolower);
  static const char *kT[] = {"1", "t", "true", "y", "yes"};
  static const char *kF[] = {"0", "f", "false", "n", "no"};
  for (int i = 0; i < 5; ++i) {
    if (v == kT[i]) return *out = true, true;
    if (v == kF[i]) return *out = false, true;
  }
  return false;
}

// ---- protobuf wire writer --------------------------------------------------
void PutVarint(uint64_t v, std::string *o) {
  while (v >= 0x80) {
    o->push_back(char((v & 0x7F) | 0x80));
    v >>= 7;
  }
  o->push_back(char(v));
}
void PutKey(int field, int wt, std::string *o) { PutVarint(uint64_t(field) << 3 | wt, o); }
void PutBytes(int field, const std::string &s, std::string *o) {
  PutKey(field, 2, o);
  PutVarint(s.size(), o);
  o->append(s);
}
void PutInt32(int field, int32_t v, std::string *o) {
  PutKey(field, 0, o);
  PutVarint(static_cast<uint64_t>(static_cast<int64_t>(v)), o);  // negative: 10 bytes
}
void PutBool(int field, bool v, std::string *o) {
  PutKey(field, 0, o);
  PutVarint(v ? 1 : 0, o);
}
void PutFloat(int field, float v, std::string *o) {
  PutKey(field, 5, o);
  char b[4];
  std::memcpy(b, &v, 4);
  o->append(b, 4);
}

// ---- host lattice for NBest(2) of the pruning step -------------------------
// Lattice (unigram_model.cc:147-261, NBest :339-477) + PopulateNodes
// (:535-604) with the TrainerModel quirks (unk_id 0, every piece NORMAL).
struct HostLattice {
  struct Node {
    int pos, length, id;
    float score, bt;
    int prev;
  };
  std::vector<Node> nodes;
  std::vector<std::vector<int>> begin_nodes, end_nodes;
  int len = 0;

  void Build(const std::string &s, const DoubleArray &trie, const std::vector<float> &score,
             float min_score, std::vector<std::pair<int32_t, size_t>> *res) {
    std::vector<size_t> surface;
    for (size_t i = 0; i < s.size();) {
      surface.push_back(i);
      i += std::min<size_t>(OneCharLen(static_cast<uint8_t>(s[i])), s.size() - i);
    }
    surface.push_back(s.size());
    len = static_cast<int>(surface.size()) - 1;
    nodes.clear();
    begin_nodes.assign(len + 1, {});
    end_nodes.assign(len + 1, {});
    nodes.push_back({0, 0, -1, 0.f, 0.f, -1});    // BOS
    nodes.push_back({len, 0, -1, 0.f, 0.f, -1});  // EOS
    end_nodes[0].push_back(0);
    begin_nodes[len].push_back(1);
    const float unk_score = min_score - 10.0f;  // kUnkPenalty
    for (int b = 0; b < len; ++b) {
      trie.CommonPrefixSearch(s.data() + surface[b], s.size() - surface[b], res);
      bool has_single = false;
      for (auto &r : *res) {
        const size_t e = surface[b] + r.second;
        int c = b;
        while (surface[c] < e) ++c;
        const int length = c - b;
        Insert(b, length, r.first, score[r.first]);
        if (length == 1) has_single = true;
      }
      if (!has_single) Insert(b, 1, 0, unk_score);
    }
  }
  void Insert(int pos, int length, int id, float sc) {
    const int k = static_cast<int>(nodes.size());
    nodes.push_back({pos, length, id, sc, 0.f, -1});
    begin_nodes[pos].push_back(k);
    end_nodes[pos + length].push_back(k);
  }
  std::vector<int> Viterbi() {
    for (int pos = 0; pos <= len; ++pos)
      for (int r : begin_nodes[pos]) {
        int best = -1;
        float best_score = 0.f;
        for (int l : end_nodes[pos]) {
          const float sc = nodes[l].bt + nodes[r].score;
          if (best < 0 || sc > best_score) {
            best = l;
            best_score = sc;
          }
        }
        if (best < 0) return {};
        nodes[r].prev = best;
        nodes[r].bt = best_score;
      }
    std::vector<int> out;
    for (int k = nodes[begin_nodes[len][0]].prev; nodes[k].prev >= 0; k = nodes[k].prev)
      out.push_back(k);
    std::reverse(out.begin(), out.end());
    return out;
  }
  // A* n-best with the same std::priority_queue ordering as the reference.
  std::vector<std::vector<int>> NBest2() {
    struct Hyp {
      int node;
      Hyp *next;
      float fx, gx;
    };
    struct Cmp {
      bool operator()(Hyp *a, Hyp *b) const { return a->fx < b->fx; }
    };
    using Agenda = std::priority_queue<Hyp *, std::vector<Hyp *>, Cmp>;
    const size_t nbest_size = 2;
    std::deque<Hyp> pool;
    Agenda agenda;
    std::vector<std::vector<int>> results;
    const int eos = begin_nodes[len][0], bos = end_nodes[0][0];
    pool.push_back(Hyp{eos, nullptr, nodes[eos].score, nodes[eos].score});
    agenda.push(&pool.back());
    Viterbi();
    while (!agenda.empty()) {
      Hyp *top = agenda.top();
      agenda.pop();
      if (top->node == bos) {
        results.emplace_back();
        for (Hyp *h = top->next; h->next != nullptr; h = h->next) results.back().push_back(h->node);
        if (results.size() == nbest_size) break;
        continue;
      }
      for (int l : end_nodes[nodes[top->node].pos]) {
        pool.push_back(Hyp{l, top, nodes[l].bt + top->gx, nodes[l].score + top->gx});
        agenda.push(&pool.back());
      }
      if (agenda.size() >= 100000) {
        Agenda na;
        const int size = std::min<int>(512, static_cast<int>(nbest_size * 10));
        for (int i = 0; i < size; ++i) {
          na.push(agenda.top());
          agenda.pop();
        }
        agenda = std::move(na);
      }
    }
    return results;
  }
};

using Pieces = std::vector<std::pair<std::string, float>>;

// Sentences as one CSR arena (no per-sentence allocations): trainer_interface
// Sentences = vector<pair<string, int64>> restated as bytes + offsets + freq.
// std::allocator that default-initializes (no zero fill on resize): the
// corpus arenas are written right after they grow.
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = DefaultInitAlloc<U>;
  };
  DefaultInitAlloc() = default;
  template <class U>
  DefaultInitAlloc(const DefaultInitAlloc<U> &) noexcept {}
  template <class U>
  void construct(U *p) noexcept {
    ::new (static_cast<void *>(p)) U;
  }
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
  }
};
using ByteVec = std::vector<char, DefaultInitAlloc<char>>;

struct Corpus {
  ByteVec bytes;
  std::vector<uint64_t> off{0};
  std::vector<int64_t> freq;
  uint64_t size() const { return freq.size(); }
  const char *data(uint64_t i) const { return bytes.data() + off[i]; }
  uint64_t len(uint64_t i) const { return off[i + 1] - off[i]; }
  void push(const char *p, size_t n, int64_t f) {
    bytes.insert(bytes.end(), p, p + n);
    off.push_back(bytes.size());
    freq.push_back(f);
  }
};

// Device CSR (bytes, offsets, freq) owned by the trainer.
struct DeviceCorpus {
  uint8_t *bytes = nullptr;
  uint64_t *off = nullptr;
  int64_t *freq = nullptr;
  uint64_t n = 0, total = 0;
  void Reset() {
    if (bytes) (void)DevFree(bytes);
    if (off) (void)DevFree(off);
    if (freq) (void)DevFree(freq);
    bytes = nullptr;
    off = nullptr;
    freq = nullptr;
    n = total = 0;
  }
  ~DeviceCorpus() { Reset(); }
};

// hipMalloc-owned scratch freed at scope exit.
struct DevScratch {
  std::vector<void *> p;
  template <typename T>
  T *Get(uint64_t count) {
    void *v = nullptr;
    if (DevMalloc(&v, std::max<uint64_t>(count, 1) * sizeof(T)) != hipSuccess) return nullptr;
    p.push_back(v);
    return static_cast<T *>(v);
  }
  ~DevScratch() {
    for (void *x : p) (void)DevFree(x);
  }
};

class UnigramTrainer {
 public:
  UnigramTrainer(const TrainerSpec &ts, const NormalizerSpec &ns, const TrainerOptions &opt)
      : spec_(ts), norm_(ns), opt_(opt), threads_(HostThreads(opt.host_threads)) {}

  Status Train(TrainerTimings *tm);

 private:
  void Log(const std::string &s) const {
    if (opt_.verbose) std::cerr << s << std::endl;
  }
  Status VerifySpec() const;
  Status InitMetaPieces();
  Status LoadSentences();
  Status ReadCorpus(Corpus *raw);
  Status ReadTextParallel(const std::string &filename, Corpus *raw, uint64_t *too_long, bool *handled);
  Status ReadTextDevice(const std::string &filename, ParsedLines *out, uint64_t *too_long, bool *handled);
  Status NormalizeOnDevice(const Corpus &raw);
  // d_raw / d_raw_off / d_freq: the loaded lines on the device; host_freq:
  // their freqs on the host (null: all 1, a text file read on the device).
  Status NormalizeDeviceCSR(const uint8_t *d_raw, const uint64_t *d_raw_off, const int64_t *d_freq, uint64_t n,
                            const std::vector<int64_t> *host_freq);
  Status MakeSeedSentencePieces(Pieces *out, TrainerTimings *tm);
  Status SplitSentencesByWhitespace();
  Status UploadCorpus(DeviceCorpus *out);
  Status SetUpRanks();
  Status RunRanks(const std::function<Status(int)> &f);
  Status ReduceToRank0(int mode, uint64_t V, int T);
  Status SetModel(Pieces &&p);
  Status RunEStep(std::vector<float> *expected, float *obj, int64_t *ntok);
  Pieces RunMStep(const std::vector<float> &expected) const;
  Status PruneSentencePieces(Pieces *out);
  Status TrainBpe(TrainerTimings *tm);
  bool IsValidSentencePiece(const uint32_t *b, const uint32_t *e) const;
  Pieces FinalizeSentencePieces() const;
  Status Save() const;
  Status Serialize(std::vector<PieceRec> *out) const;

  TrainerSpec spec_;
  NormalizerSpec norm_;
  TrainerOptions opt_;
  int threads_;
  std::map<int, std::pair<std::string, int32_t>> meta_pieces_;
  Corpus sentences_;          // host copy (after load / after the split)
  DeviceCorpus loaded_;       // normalized corpus on the device (seed mining)
  ParsedLines dev_lines_;     // ReadCorpus's device path: the raw lines (until normalized)
  void ReleaseDevLines() {
    for (void *x : {static_cast<void *>(dev_lines_.bytes), static_cast<void *>(dev_lines_.off),
                    static_cast<void *>(dev_lines_.freq)})
      if (x) (void)DevFree(x);
    dev_lines_ = ParsedLines();
  }
  std::unordered_map<uint32_t, int64_t> required_chars_;
  Pieces pieces_;      // current TrainerModel list
  double read_s_ = 0, trie_build_s_ = 0;  // TrainerTimings::read / trie_build
  float min_score_ = FLT_MAX;
  size_t desired_vocab_size_ = 0;
  Pieces final_pieces_;
  bool need_host_text_ = true;  // the whitespace split needs the text on the host
  bool host_freq_deferred_ = false;  // sentences_.freq not materialized (loaded_.n sentences)

  // One rank per GPU (--num_gpus; csrc/shard_plan.h): its shard of the EM
  // corpus (its plan segments concatenated), stream and E-step accumulators.
  struct Rank {
    int device = 0;
    hipStream_t stream = nullptr;
    DeviceCorpus shard;
    std::vector<ShardSegment> segs;
    std::vector<uint64_t> seg_begin;  // local index of each segment's first sentence
    char *acc = nullptr;              // [acc | obj | ntok], grow-only
    uint64_t acc_cap = 0;
    spm_hip_pieces *pieces = nullptr;  // the last E-step's piece trie on the rank's device
    std::vector<uint8_t> piece_bytes;  // ... and the piece list it was built from
    std::vector<uint64_t> piece_off;
    ~Rank() {
      if (pieces) spm_hip_pieces_free(pieces);
      if (acc) (void)DevFree(acc);
      if (stream) (void)hipStreamDestroy(stream);
    }
  };
  std::vector<std::unique_ptr<Rank>> ranks_;
  std::vector<ncclComm_t> comms_;  // one per rank when every rank has its own device
  uint64_t acc_obj_at_ = 0, acc_ntok_at_ = 0;  // accumulator layout of the current E-step
  uint64_t nbest_host_redo_ = 0;  // pruning NBest pieces redone on the host (device slab overflow)

 public:
  ~UnigramTrainer() {
    ReleaseDevLines();
    if (reaper_.joinable()) reaper_.join();
    for (ncclComm_t c : comms_) (void)ncclCommDestroy(c);
  }

 private:
  // Frees the loaded raw corpus (GBs of host pages at c5: ~0.3 s of munmap)
  // on another thread while seed mining runs.
  std::thread reaper_;
};

// trainer_interface.cc:32-89 VerifySpec
Status UnigramTrainer::VerifySpec() const {
  if (spec_.model_prefix.empty()) return Err(SPM_INTERNAL, "model_prefix is empty");
  if (spec_.input.empty()) return Err(SPM_INTERNAL, "input is empty");
  if (spec_.vocab_size <= 0) return Err(SPM_INTERNAL, "vocab_size <= 0");
  if (spec_.model_type != kUnigram && spec_.model_type != kBpe)
    return Err(SPM_UNIMPLEMENTED, "only --model_type=unigram|bpe are trained on the device path");
  if (spec_.use_all_vocab) return Err(SPM_INTERNAL, "--use_all_vocab=true is valid for WORD/CHAR model.");
  auto range = [](double v, double lo, double hi) { return v >= lo && v <= hi; };
  if (!range(spec_.character_coverage, 0.98, 1.0) ||
      !range(spec_.max_sentencepiece_length, 1, 512) || !range(spec_.num_sub_iterations, 1, 10) ||
      !range(spec_.num_threads, 1, 128) || !range(spec_.self_test_sample_size, 0, 1000) ||
      !range(spec_.shrinking_factor, 0.5, 0.95) ||
      !range(spec_.max_sentence_length, 10, 1073741824))
    return Err(SPM_INTERNAL, "a trainer spec value is out of range");
  if (!(spec_.input_sentence_size <= 0 || spec_.input_sentence_size > 100))
    return Err(SPM_INTERNAL, "input_sentence_size must be <= 0 or > 100");
  if (spec_.unk_piece.empty() || spec_.bos_piece.empty() || spec_.eos_piece.empty() ||
      spec_.pad_piece.empty())
    return Err(SPM_INTERNAL, "meta piece strings must not be empty");
  if (spec_.self_test_sample_size > 0)
    return Err(SPM_UNIMPLEMENTED, "self_test_sample_size > 0 is not supported");
  if (!norm_.escape_whitespaces) return Err(SPM_INTERNAL, "escape_whitespaces must be true");
  return Status::Ok();
}

// trainer_interface.cc:585-645
Status UnigramTrainer::InitMetaPieces() {
  bool has_unk = false;
  auto insert_id = [&](int id, const std::string &w) {
    if (id < 0) return true;
    if (id >= spec_.vocab_size || meta_pieces_.count(id) || (has_unk && w == spec_.unk_piece))
      return false;
    if (w == spec_.unk_piece) has_unk = true;
    meta_pieces_[id] = {w, w == spec_.unk_piece ? kUnknown : kControl};
    return true;
  };
  if (!insert_id(spec_.unk_id, spec_.unk_piece) || !insert_id(spec_.bos_id, spec_.bos_piece) ||
      !insert_id(spec_.eos_id, spec_.eos_piece) || !insert_id(spec_.pad_id, spec_.pad_piece))
    return Err(SPM_INTERNAL, "invalid meta piece id");
  if (!has_unk) return Err(SPM_INTERNAL, spec_.unk_piece + " must be defined.");
  std::set<std::string> dup;
  int id = 0;
  auto insert_meta = [&](const std::string &w, int32_t type) {
    if (!dup.insert(w).second) return false;
    if (w == spec_.unk_piece) return false;
    if (w == spec_.bos_piece && spec_.bos_id >= 0) meta_pieces_[spec_.bos_id].second = type;
    else if (w == spec_.eos_piece && spec_.eos_id >= 0) meta_pieces_[spec_.eos_id].second = type;
    else if (w == spec_.pad_piece && spec_.pad_id >= 0) meta_pieces_[spec_.pad_id].second = type;
    else {
      while (meta_pieces_.count(id)) ++id;
      meta_pieces_[id] = {w, type};
    }
    return true;
  };
  for (auto &w : spec_.control_symbols)
    if (!insert_meta(w, kControl)) return Err(SPM_INTERNAL, w + " is already defined.");
  for (auto &w : spec_.user_defined_symbols)
    if (!insert_meta(w, kUserDefined)) return Err(SPM_INTERNAL, w + " is already defined.");
  return Status::Ok();
}

// One input line → (sentence, freq) after the reference's per-line filters
// (trainer_interface.cc:295-331).  Returns 0 keep, 1 skip, 2 too long, -1 error.
int ParseLine(const char *b, size_t n, bool is_tsv, int max_len, std::string *out, int64_t *freq,
              std::string *err) {
  *freq = 1;
  if (is_tsv) {
    const std::vector<std::string> v = Split(std::string(b, n), '\t');
    if (v.size() != 2) {
      *err = "Input format must be: word <tab> freq. " + std::string(b, n);
      return -1;
    }
    *out = v[0];
    *freq = std::atoll(v[1].c_str());
    if (*freq < 1) {
      *err = "freq must be >= 1";
      return -1;
    }
  } else {
    out->assign(b, n);
  }
  if (out->empty()) return 1;
  if (static_cast<int>(out->size()) > max_len) return 2;
  if (out->find(kUNKStr) != std::string::npos) return 1;
  return 0;
}

// trainer_interface.cc:269-331: the input lines after the per-line filters
// and the SentenceSelector, as a raw CSR.  Files are read whole and, unless
// --input_sentence_size asks for the (order-dependent) selector, parsed by
// host threads over newline-aligned chunks and concatenated in file order.
// A regular text file, no sentence selector: the file is read by host
// threads (pread of 64 MB pieces into an uninitialized buffer) and split into
// lines in two passes — count the kept lines / bytes per thread range, then
// every thread copies its lines straight to their final place in `raw` — so
// no per-thread parts are concatenated afterwards.  Lines: std::getline
// semantics (filesystem.cc:42-44); empty lines and lines holding kUNKStr are
// dropped, lines over max_sentence_length counted as too long
// (trainer_interface.cc:287-316).  *handled = false: not a regular file, the
// caller streams it.
Status UnigramTrainer::ReadTextParallel(const std::string &filename, Corpus *raw, uint64_t *too_long,
                                        bool *handled) {
  *handled = false;
  const int fd = ::open(filename.c_str(), O_RDONLY);
  if (fd < 0) return Status::Ok();
  struct stat sb;
  if (::fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode) || sb.st_size <= 0) {
    ::close(fd);
    return Status::Ok();
  }
  const size_t size = static_cast<size_t>(sb.st_size);
  std::unique_ptr<char[]> data(new char[size]);
  {
    constexpr size_t kPiece = 64ull << 20;
    const size_t pieces = (size + kPiece - 1) / kPiece;
    std::atomic<size_t> next{0};
    std::atomic<bool> bad{false};
    std::vector<std::thread> th;
    const int T = static_cast<int>(std::max<size_t>(1, std::min<size_t>(threads_, pieces)));
    for (int t = 0; t < T; ++t)
      th.emplace_back([&]() {
        for (size_t k = next++; k < pieces && !bad; k = next++) {
          size_t o = k * kPiece;
          const size_t e = std::min(size, o + kPiece);
          while (o < e) {
            const ssize_t r = ::pread(fd, data.get() + o, e - o, static_cast<off_t>(o));
            if (r <= 0) {
              bad = true;
              break;
            }
            o += static_cast<size_t>(r);
          }
        }
      });
    for (auto &x : th) x.join();
    ::close(fd);
    if (bad) return Err(SPM_INTERNAL, "\"" + filename + "\": read error");
  }
  const int T = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(threads_, size / (1 << 20) + 1)));
  std::vector<size_t> cut(T + 1, size);
  cut[0] = 0;
  for (int t = 1; t < T; ++t) {
    const size_t c = size * t / T;
    const void *nl = c < size ? std::memchr(data.get() + c, '\n', size - c) : nullptr;
    cut[t] = std::max(nl ? static_cast<size_t>(static_cast<const char *>(nl) - data.get()) + 1 : size, cut[t - 1]);
  }
  const int max_len = spec_.max_sentence_length;
  // 0 keep, 1 drop (empty / holds kUNKStr), 2 drop (too long).  kUNKStr is
  // found through memchr of its lead byte (string_view::find walks char by
  // char: it was most of the load time at 100 M lines).
  auto has_unk = [](const char *s, size_t n) {
    const char *e = s + n;
    for (const char *p = s; (p = static_cast<const char *>(std::memchr(p, kUNKStr[0], e - p))) != nullptr; ++p)
      if (e - p >= 3 && p[1] == kUNKStr[1] && p[2] == kUNKStr[2]) return true;
    return false;
  };
  auto verdict = [&](const char *s, size_t n) {
    if (n == 0) return 1;
    if (static_cast<int64_t>(n) > max_len) return 2;
    return has_unk(s, n) ? 1 : 0;
  };
  std::vector<uint64_t> nl_t(T, 0), nb_t(T, 0), tl_t(T, 0);
  auto each_range = [&](const std::function<void(int)> &f) {  // one host thread per range
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(f, t);
    for (auto &x : th) x.join();
  };
  each_range([&](int t) {
    uint64_t nl_c = 0, nb_c = 0, tl_c = 0;  // (thread-local: no false sharing)
    for (size_t p = cut[t]; p < cut[t + 1];) {
      const void *nl = std::memchr(data.get() + p, '\n', cut[t + 1] - p);
      const size_t q = nl ? static_cast<size_t>(static_cast<const char *>(nl) - data.get()) : cut[t + 1];
      const int r = verdict(data.get() + p, q - p);
      if (r == 0) {
        ++nl_c;
        nb_c += q - p;
      } else if (r == 2) {
        ++tl_c;
      }
      p = q + 1;
    }
    nl_t[t] = nl_c;
    nb_t[t] = nb_c;
    tl_t[t] = tl_c;
  });
  const uint64_t n0 = raw->size(), b0 = raw->bytes.size();
  std::vector<uint64_t> ln(T + 1, n0), lb(T + 1, b0);
  for (int t = 0; t < T; ++t) {
    ln[t + 1] = ln[t] + nl_t[t];
    lb[t + 1] = lb[t] + nb_t[t];
    *too_long += tl_t[t];
  }
  raw->bytes.resize(lb[T]);
  raw->off.resize(ln[T] + 1);
  raw->freq.resize(ln[T], 1);
  each_range([&](int t) {
    {
      uint64_t li = ln[t], bi = lb[t];
      for (size_t p = cut[t]; p < cut[t + 1];) {
        const void *nl = std::memchr(data.get() + p, '\n', cut[t + 1] - p);
        const size_t q = nl ? static_cast<size_t>(static_cast<const char *>(nl) - data.get()) : cut[t + 1];
        if (verdict(data.get() + p, q - p) == 0) {
          std::memcpy(raw->bytes.data() + bi, data.get() + p, q - p);
          bi += q - p;
          raw->off[++li] = bi;
        }
        p = q + 1;
      }
    }
  });
  *handled = true;
  return Status::Ok();
}

// ReadCorpus's device path: a regular text file is read by host threads into
// small pinned buffers (pread of 16 MB pieces, two buffers per thread) and
// copied into one device buffer while the next piece is read; the lines are
// then found and filtered on the device (CorpusParseLines), so the file's
// bytes are never parsed, copied or held on the host.  *handled = false: not
// a regular non-empty file, or too many lines for the device scan (the
// caller takes the host path).
Status UnigramTrainer::ReadTextDevice(const std::string &filename, ParsedLines *out, uint64_t *too_long,
                                      bool *handled) {
  *handled = false;
  const double t_begin = Now();
  const int fd = ::open(filename.c_str(), O_RDONLY);
  if (fd < 0) return Status::Ok();
  struct FdGuard {
    int fd;
    ~FdGuard() { ::close(fd); }
  } fd_guard{fd};
  struct stat sb;
  if (::fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode) || sb.st_size <= 0) return Status::Ok();
  const uint64_t size = static_cast<uint64_t>(sb.st_size);
  uint8_t *d_file = nullptr;
  if (DevMalloc(&d_file, size) != hipSuccess) {
    (void)hipGetLastError();
    return Status::Ok();
  }
  struct DevGuard {
    uint8_t *p;
    ~DevGuard() { (void)DevFree(p); }
  } dev_guard{d_file};
  // SPM_HIP_LOAD_PIECE_MB: bytes per pread + copy (default 16 MB, two pinned
  // buffers per reader).
  static const uint64_t kPiece = [] {
    const char *v = std::getenv("SPM_HIP_LOAD_PIECE_MB");
    return (v && std::atoi(v) > 0 ? static_cast<uint64_t>(std::atoi(v)) : 16ull) << 20;
  }();
  const uint64_t pieces = (size + kPiece - 1) / kPiece;
  // SPM_HIP_LOAD_READERS: reader threads (default 8, at most the trainer's).
  static const int kReaders = [] {
    const char *v = std::getenv("SPM_HIP_LOAD_READERS");
    return v && std::atoi(v) > 0 ? std::atoi(v) : 8;
  }();
  const int T = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(std::min(threads_, kReaders), pieces)));
  std::atomic<uint64_t> next{0};
  std::atomic<bool> bad{false};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&]() {
      void *buf[2] = {nullptr, nullptr};
      hipEvent_t ev[2] = {nullptr, nullptr};
      bool used[2] = {false, false};
      hipStream_t st = nullptr;
      bool ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
      for (int b = 0; b < 2 && ok; ++b)
        ok = hipHostMalloc(&buf[b], kPiece, hipHostMallocDefault) == hipSuccess &&
             hipEventCreateWithFlags(&ev[b], hipEventDisableTiming) == hipSuccess;
      for (uint64_t k = next++, j = 0; ok && k < pieces && !bad; k = next++, ++j) {
        const int b = static_cast<int>(j & 1);
        if (used[b] && hipEventSynchronize(ev[b]) != hipSuccess) ok = false;
        const uint64_t o = k * kPiece, len = std::min(kPiece, size - o);
        for (uint64_t r = 0; ok && r < len;) {
          const ssize_t g = ::pread(fd, static_cast<char *>(buf[b]) + r, len - r, static_cast<off_t>(o + r));
          if (g <= 0) ok = false;
          else r += static_cast<uint64_t>(g);
        }
        if (ok) ok = hipMemcpyAsync(d_file + o, buf[b], len, hipMemcpyHostToDevice, st) == hipSuccess &&
                     hipEventRecord(ev[b], st) == hipSuccess;
        used[b] = true;
      }
      if (st && hipStreamSynchronize(st) != hipSuccess) ok = false;
      for (int b = 0; b < 2; ++b) {
        if (buf[b]) (void)hipHostFree(buf[b]);
        if (ev[b]) (void)hipEventDestroy(ev[b]);
      }
      if (st) (void)hipStreamDestroy(st);
      if (!ok) bad = true;
    });
  for (auto &x : th) x.join();
  if (bad) return Err(SPM_INTERNAL, "\"" + filename + "\": read error");
  const double t_read = Now();
  const hipError_t e = CorpusParseLines(d_file, size, spec_.max_sentence_length, out, nullptr);
  {
    std::ostringstream os;
    os << "ReadTextDevice: file to HBM " << t_read - t_begin << " s, line split " << Now() - t_read << " s ("
       << T << " readers)";
    Log(os.str());
  }
  if (e == hipErrorInvalidValue) {
    (void)hipGetLastError();
    return Status::Ok();  // host path
  }
  if (e != hipSuccess) return Err(SPM_INTERNAL, std::string("device line split: ") + hipGetErrorString(e));
  *too_long += out->too_long;
  *handled = true;
  return Status::Ok();
}

Status UnigramTrainer::ReadCorpus(Corpus *raw) {
  const bool is_tsv = spec_.input_format == "tsv";
  if (!(spec_.input_format.empty() || spec_.input_format == "text" || is_tsv))
    return Err(SPM_INTERNAL, "Supported formats are 'text' and 'tsv'.");
  const bool select = spec_.input_sentence_size > 0;
  const bool sample = select && spec_.shuffle_input_sentence;
  std::mt19937 engine(12345678);  // SentenceSelector kSeed (:100-104)
  std::vector<std::pair<std::string, int64_t>> picked;  // selector path only
  size_t total = 0;
  uint64_t too_long = 0;
  bool done = false;
  // One plain text file, no selector: read straight into device memory and
  // split into lines there (SPM_HIP_DEVICE_LOAD=0: the host path below).
  static const bool kDeviceLoad = [] {
    const char *e = std::getenv("SPM_HIP_DEVICE_LOAD");
    return !(e && std::atoi(e) == 0);
  }();
  if (!select && !is_tsv && spec_.input.size() == 1 && kDeviceLoad) {
    const std::string &filename = spec_.input[0];
    if (!std::ifstream(filename, std::ios::binary))
      return Err(SPM_NOT_FOUND, "\"" + filename + "\": No such file or directory");
    Log("Loading corpus: " + filename);
    bool handled = false;
    RETURN_IF_ERROR(ReadTextDevice(filename, &dev_lines_, &too_long, &handled));
    if (handled) {
      Log("Loaded " + std::to_string(dev_lines_.n) + " sentences");
      if (too_long > 0) Log("Skipped " + std::to_string(too_long) + " too long sentences.");
      if (dev_lines_.n == 0) {
        ReleaseDevLines();
        return Err(SPM_INTERNAL, "no sentences");
      }
      return Status::Ok();
    }
  }
  for (const auto &filename : spec_.input) {
    if (done) break;
    std::ifstream is(filename, std::ios::binary);
    if (!is) return Err(SPM_NOT_FOUND, "\"" + filename + "\": No such file or directory");
    Log("Loading corpus: " + filename);
    if (!select && !is_tsv) {
      bool handled = false;
      RETURN_IF_ERROR(ReadTextParallel(filename, raw, &too_long, &handled));
      if (handled) continue;
    }
    std::string data;
    is.seekg(0, std::ios::end);
    const std::streamoff fsize = is.tellg();
    is.seekg(0, std::ios::beg);
    if (fsize > 0) {
      data.resize(static_cast<size_t>(fsize));
      is.read(&data[0], fsize);
      data.resize(static_cast<size_t>(is.gcount()));
    } else {  // not seekable (pipe): stream it
      data.assign(std::istreambuf_iterator<char>(is), std::istreambuf_iterator<char>());
    }
    // Lines: std::getline semantics (filesystem.cc:42-44).
    if (!select) {
      const int T = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(threads_, data.size() / (1 << 20) + 1)));
      std::vector<size_t> cut(T + 1, data.size());
      cut[0] = 0;
      for (int t = 1; t < T; ++t) {
        const size_t c = data.size() * t / T;
        const void *nl = c < data.size() ? std::memchr(data.data() + c, '\n', data.size() - c) : nullptr;
        cut[t] = std::max(nl ? static_cast<size_t>(static_cast<const char *>(nl) - data.data()) + 1 : data.size(),
                          cut[t - 1]);
      }
      std::vector<Corpus> part(T);
      std::vector<uint64_t> tl(T, 0);
      std::vector<std::string> errs(T);
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t]() {
          size_t p = cut[t];
          const size_t end = cut[t + 1];
          part[t].bytes.reserve(end - p);
          std::string line;
          while (p < end) {
            const void *nl = std::memchr(data.data() + p, '\n', end - p);
            const size_t q = nl ? static_cast<size_t>(static_cast<const char *>(nl) - data.data()) : end;
            int64_t freq = 1;
            int r;
            if (is_tsv) {
              r = ParseLine(data.data() + p, q - p, true, spec_.max_sentence_length, &line, &freq, &errs[t]);
              if (r < 0) return;
              if (r == 0) part[t].push(line.data(), line.size(), freq);
            } else {
              // Text lines need no copy: the filters read the line in place.
              const size_t n = q - p;
              r = n == 0 ? 1 : static_cast<int>(n) > spec_.max_sentence_length ? 2 : 0;
              if (r == 0 && std::string_view(data.data() + p, n).find(kUNKStr) != std::string_view::npos) r = 1;
              if (r == 0) part[t].push(data.data() + p, n, 1);
            }
            if (r == 2) ++tl[t];
            p = q + 1;
          }
        });
      for (auto &x : th) x.join();
      for (int t = 0; t < T; ++t)
        if (!errs[t].empty()) return Err(SPM_INTERNAL, errs[t]);
      uint64_t add_b = 0, add_n = 0;
      for (auto &c : part) {
        add_b += c.bytes.size();
        add_n += c.size();
      }
      raw->bytes.reserve(raw->bytes.size() + add_b);
      raw->off.reserve(raw->off.size() + add_n);
      raw->freq.reserve(raw->freq.size() + add_n);
      for (int t = 0; t < T; ++t) {
        too_long += tl[t];
        const uint64_t base = raw->bytes.size();
        raw->bytes.insert(raw->bytes.end(), part[t].bytes.begin(), part[t].bytes.end());
        for (uint64_t k = 1; k < part[t].off.size(); ++k) raw->off.push_back(base + part[t].off[k]);
        raw->freq.insert(raw->freq.end(), part[t].freq.begin(), part[t].freq.end());
        part[t] = Corpus();
      }
      continue;
    }
    size_t p = 0;
    std::string sentence;
    while (p < data.size() && !done) {
      const void *nl = std::memchr(data.data() + p, '\n', data.size() - p);
      const size_t q = nl ? static_cast<size_t>(static_cast<const char *>(nl) - data.data()) : data.size();
      int64_t freq;
      std::string err;
      const int r = ParseLine(data.data() + p, q - p, is_tsv, spec_.max_sentence_length, &sentence,
                              &freq, &err);
      p = q + 1;
      if (r < 0) return Err(SPM_INTERNAL, err);
      if (r == 2) ++too_long;
      if (r != 0) continue;
      // SentenceSelector::Add (:121-141); ReservoirSampler::Add (util.h:757-768)
      if (sample) {
        ++total;
        if (picked.size() < size_t(spec_.input_sentence_size)) {
          picked.emplace_back(sentence, freq);
        } else {
          std::uniform_int_distribution<size_t> dist(0, total - 1);
          const size_t k = dist(engine);
          if (k < picked.size()) picked[k] = {sentence, freq};
        }
      } else {
        picked.emplace_back(sentence, freq);
        if (picked.size() >= size_t(spec_.input_sentence_size)) done = true;
      }
    }
  }
  for (auto &x : picked) raw->push(x.first.data(), x.first.size(), x.second);
  Log("Loaded " + std::to_string(raw->size()) + " sentences");
  if (too_long > 0) Log("Skipped " + std::to_string(too_long) + " too long sentences.");
  if (raw->size() == 0) return Err(SPM_INTERNAL, "no sentences");
  return Status::Ok();
}

#define HIP_OR_RETURN(expr)                                                                  \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return Err(SPM_INTERNAL, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// trainer_interface.cc:333-455 on the device: Normalize (Normalizer(spec),
// no suffix flag), PrefixMatcher::GlobalReplace of the meta pieces, the
// empty-sentence removal (swap-with-last, simulated on the host over the
// lengths), the char histogram, required_chars_ and the rare-char
// replacement.  The result stays on the device (loaded_) for seed mining;
// the host keeps the freq (and the text when the whitespace split needs it).
Status UnigramTrainer::NormalizeOnDevice(const Corpus &raw) {
  const uint64_t n = raw.size();
  DevScratch S;
  uint8_t *d_raw = S.Get<uint8_t>(raw.bytes.size());
  uint64_t *d_raw_off = S.Get<uint64_t>(n + 1);
  int64_t *d_freq = S.Get<int64_t>(n);
  if (!d_raw || !d_raw_off || !d_freq) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
  HIP_OR_RETURN(hipMemcpy(d_raw, raw.bytes.data(), raw.bytes.size(), hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(d_raw_off, raw.off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(d_freq, raw.freq.data(), n * 8, hipMemcpyHostToDevice));
  return NormalizeDeviceCSR(d_raw, d_raw_off, d_freq, n, &raw.freq);
}

Status UnigramTrainer::NormalizeDeviceCSR(const uint8_t *d_raw, const uint64_t *d_raw_off, const int64_t *d_freq,
                                          uint64_t n, const std::vector<int64_t> *host_freq) {
  hipStream_t st = nullptr;
  // SPM_HIP_TRACE_LOAD=1: synchronize and log after every step (debugging).
  static const bool kTrace = std::getenv("SPM_HIP_TRACE_LOAD") != nullptr;
  const double t_norm = Now();
  auto step = [&](const char *what) {
    if (!kTrace) return;
    const hipError_t e = hipDeviceSynchronize();
    std::ostringstream os;
    os << "normalize step " << what << " " << Now() - t_norm << " s (" << hipGetErrorString(e) << ")";
    Log(os.str());
  };
  DevScratch S;
  uint64_t *d_len = S.Get<uint64_t>(n);
  uint32_t *d_flag = S.Get<uint32_t>(4);
  if (!d_len || !d_flag) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
  HIP_OR_RETURN(hipMemset(d_flag, 0, 16));
  size_t tmp_bytes = 0;
  // (a size query: nothing is written)
  HIP_OR_RETURN(LengthsToOffsets(d_len, n, const_cast<uint64_t *>(d_raw_off), nullptr, &tmp_bytes, st));
  void *d_tmp = S.Get<uint8_t>(tmp_bytes);
  auto scan = [&](uint64_t *d_off_out, uint64_t *total) -> Status {
    size_t tb = tmp_bytes;
    HIP_OR_RETURN(LengthsToOffsets(d_len, n, d_off_out, d_tmp, &tb, st));
    HIP_OR_RETURN(hipMemcpy(total, d_off_out + n, 8, hipMemcpyDeviceToHost));
    return Status::Ok();
  };
  // Normalize.
  NormTables t;
  const std::string &blob = norm_.precompiled_charsmap;
  if (!blob.empty()) {
    uint32_t tsize = 0;
    if (blob.size() <= 4) return Err(SPM_INTERNAL, "Blob for normalization rule is broken.");
    std::memcpy(&tsize, blob.data(), 4);
    if (tsize >= blob.size() || tsize < 4) return Err(SPM_INTERNAL, "Blob for normalization rule is broken.");
    uint8_t *d_blob = S.Get<uint8_t>(blob.size() + 1);
    if (!d_blob) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    HIP_OR_RETURN(hipMemcpy(d_blob, blob.data(), blob.size(), hipMemcpyHostToDevice));
    HIP_OR_RETURN(hipMemset(d_blob + blob.size(), 0, 1));  // ends an unterminated pool string
    t.units = reinterpret_cast<const uint32_t *>(d_blob + 4);
    t.num_units = tsize / 4;
    t.pool = d_blob + 4 + tsize;
    t.pool_size = static_cast<uint32_t>(blob.size() - 4 - tsize);
  }
  t.add_dummy_prefix = norm_.add_dummy_prefix;
  t.remove_extra_whitespaces = norm_.remove_extra_whitespaces;
  t.escape_whitespaces = norm_.escape_whitespaces;
  t.suffix = false;
  step("start");
  HIP_OR_RETURN(NormalizeLengths(t, d_raw, d_raw_off, n, d_len, st));
  step("lengths");
  uint64_t *d_off = S.Get<uint64_t>(n + 1);
  uint64_t total = 0;
  RETURN_IF_ERROR(scan(d_off, &total));
  step("scan");
  uint8_t *d_text = S.Get<uint8_t>(total);
  if (!d_off || !d_text) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
  HIP_OR_RETURN(NormalizeWrite(t, d_raw, d_raw_off, n, d_text, d_off, st));
  step("write");
  // Meta pieces → "\\t" (GlobalReplace, normalizer.cc:391-405).
  {
    std::vector<std::pair<std::string, int32_t>> keys;
    for (auto &it : meta_pieces_) keys.emplace_back(it.second.first, 1);
    DoubleArray da;
    std::string err;
    if (!BuildDoubleArray(keys, &da, &err)) return Err(SPM_INTERNAL, err);
    uint32_t *d_units = S.Get<uint32_t>(da.units.size());
    if (!d_units) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    HIP_OR_RETURN(hipMemcpy(d_units, da.units.data(), da.units.size() * 4, hipMemcpyHostToDevice));
    HIP_OR_RETURN(MetaReplaceLengths(d_units, static_cast<uint32_t>(da.units.size()), d_text, d_off, n,
                                     d_len, d_flag + 1, st));
    uint32_t any = 0;
    HIP_OR_RETURN(hipMemcpy(&any, d_flag + 1, 4, hipMemcpyDeviceToHost));
    if (any) {
      uint64_t *d_off2 = S.Get<uint64_t>(n + 1);
      uint64_t total2 = 0;
      RETURN_IF_ERROR(scan(d_off2, &total2));
      uint8_t *d_text2 = S.Get<uint8_t>(total2);
      if (!d_off2 || !d_text2) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
      HIP_OR_RETURN(MetaReplaceWrite(d_units, static_cast<uint32_t>(da.units.size()), d_text, d_off, n,
                                     d_text2, d_off2, st));
      d_text = d_text2;
      d_off = d_off2;
      total = total2;
    }
  }
  // Char histogram (:401-420) + space / NUL / empty flags.
  std::vector<unsigned long long> counts(0x110000, 0);
  {
    unsigned long long *d_counts = S.Get<unsigned long long>(0x110000);
    if (!d_counts) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    HIP_OR_RETURN(hipMemset(d_counts, 0, 0x110000 * 8));
    HIP_OR_RETURN(hipMemset(d_flag, 0, 4));
    step("meta");
    HIP_OR_RETURN(CorpusCharHistogram(d_text, d_off, d_freq, n, d_counts, d_flag, st));
    step("histogram");
    HIP_OR_RETURN(hipMemcpy(counts.data(), d_counts, 0x110000 * 8, hipMemcpyDeviceToHost));
  }
  uint32_t flags = 0;
  HIP_OR_RETURN(hipMemcpy(&flags, d_flag, 4, hipMemcpyDeviceToHost));
  if (flags & 1u) return Err(SPM_INTERNAL, "Normalized string must not include spaces");
  // Empty sentences (:392-398): for i ascending, an empty sentence i is
  // swapped with the last and the vector shrinks; the swapped-in one is not
  // re-checked.  Simulated over the lengths, applied as a device gather.
  // Host freqs of the kept sentences (all 1 for a file read on the device).
  std::vector<int64_t> freq;
  if (host_freq) freq = *host_freq;
  uint64_t m = n;
  if (flags & 4u) {
    std::vector<uint64_t> off(n + 1);
    HIP_OR_RETURN(hipMemcpy(off.data(), d_off, (n + 1) * 8, hipMemcpyDeviceToHost));
    std::vector<uint64_t> idx(n);
    for (uint64_t i = 0; i < n; ++i) idx[i] = i;
    for (uint64_t i = 0; i < m; ++i) {
      if (off[idx[i] + 1] == off[idx[i]]) {
        std::swap(idx[i], idx[m - 1]);
        --m;
      }
    }
    idx.resize(m);
    if (host_freq) {
      for (uint64_t k = 0; k < m; ++k) freq[k] = (*host_freq)[idx[k]];
      freq.resize(m);
    }
    uint64_t *d_idx = S.Get<uint64_t>(m);
    uint64_t *d_off2 = S.Get<uint64_t>(m + 1);
    int64_t *d_freq2 = S.Get<int64_t>(m);
    if (!d_idx || !d_off2 || !d_freq2) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    HIP_OR_RETURN(hipMemcpy(d_idx, idx.data(), m * 8, hipMemcpyHostToDevice));
    HIP_OR_RETURN(CorpusGatherLengths(d_off, d_idx, m, d_len, st));
    size_t tb = tmp_bytes;
    HIP_OR_RETURN(LengthsToOffsets(d_len, m, d_off2, d_tmp, &tb, st));
    uint64_t total2 = 0;
    HIP_OR_RETURN(hipMemcpy(&total2, d_off2 + m, 8, hipMemcpyDeviceToHost));
    uint8_t *d_text2 = S.Get<uint8_t>(total2);
    if (!d_text2) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    HIP_OR_RETURN(CorpusGatherWrite(d_text, d_off, d_freq, d_idx, m, d_text2, d_off2, d_freq2, st));
    d_text = d_text2;
    d_off = d_off2;
    d_freq = d_freq2;
    total = total2;
  }
  if (m == 0) return Err(SPM_INTERNAL, "no sentences after normalization");
  // required_chars_ (:422-436)
  std::vector<std::pair<uint32_t, int64_t>> chars;
  int64_t all_chars_count = 0;
  for (uint32_t c = 0; c < 0x110000; ++c)
    if (counts[c]) {
      chars.emplace_back(c, static_cast<int64_t>(counts[c]));
      all_chars_count += static_cast<int64_t>(counts[c]);
    }
  int64_t accumulated = 0;
  for (auto &w : Sorted(chars)) {
    const float coverage = static_cast<float>(1.0 * accumulated / all_chars_count);
    if (!spec_.use_all_vocab && coverage >= spec_.character_coverage) break;
    accumulated += w.second;
    if (w.first == kUPPBoundaryChar) continue;
    required_chars_.insert(w);
  }
  Log("Alphabet size=" + std::to_string(required_chars_.size()));
  if (required_chars_.count(kUNKChar)) return Err(SPM_INTERNAL, "UNK char in required chars");
  // Rare chars → kUNKChar (:444-455); the identity when every char present is
  // required and no NUL occurs.
  if ((flags & 2u) || chars.size() != required_chars_.size()) {
    std::vector<uint32_t> bits(0x110000 / 32, 0);
    for (auto &kv : required_chars_) bits[kv.first >> 5] |= 1u << (kv.first & 31);
    uint32_t *d_bits = S.Get<uint32_t>(bits.size());
    uint64_t *d_off2 = S.Get<uint64_t>(m + 1);
    if (!d_bits || !d_off2) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    HIP_OR_RETURN(hipMemcpy(d_bits, bits.data(), bits.size() * 4, hipMemcpyHostToDevice));
    HIP_OR_RETURN(CorpusReplaceLengths(d_text, d_off, m, d_bits, d_len, st));
    size_t tb = tmp_bytes;
    HIP_OR_RETURN(LengthsToOffsets(d_len, m, d_off2, d_tmp, &tb, st));
    uint64_t total2 = 0;
    HIP_OR_RETURN(hipMemcpy(&total2, d_off2 + m, 8, hipMemcpyDeviceToHost));
    uint8_t *d_text2 = S.Get<uint8_t>(total2);
    if (!d_text2) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    HIP_OR_RETURN(CorpusReplaceWrite(d_text, d_off, m, d_bits, d_text2, d_off2, st));
    d_text = d_text2;
    d_off = d_off2;
    total = total2;
  }
  if (static_cast<int>(required_chars_.size() + meta_pieces_.size()) > spec_.vocab_size)
    return Err(SPM_INTERNAL, "Vocabulary size is smaller than required_chars.");
  // Keep the final corpus on the device (own copies; scratch is freed).
  loaded_.Reset();
  loaded_.n = m;
  loaded_.total = total;
  if (DevMalloc(&loaded_.bytes, std::max<uint64_t>(total, 1)) != hipSuccess ||
      DevMalloc(&loaded_.off, (m + 1) * 8) != hipSuccess || DevMalloc(&loaded_.freq, m * 8) != hipSuccess)
    return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
  HIP_OR_RETURN(hipMemcpy(loaded_.bytes, d_text, total, hipMemcpyDeviceToDevice));
  HIP_OR_RETURN(hipMemcpy(loaded_.off, d_off, (m + 1) * 8, hipMemcpyDeviceToDevice));
  HIP_OR_RETURN(hipMemcpy(loaded_.freq, d_freq, m * 8, hipMemcpyDeviceToDevice));
  sentences_ = Corpus();
  // A file read on the device has all freqs 1; when the whitespace split
  // comes next and needs no host text, the host copy is not made at all (the
  // split replaces the sentences; its host fallback downloads the freqs).
  host_freq_deferred_ = !host_freq && spec_.split_by_whitespace && !need_host_text_;
  if (!host_freq && !host_freq_deferred_) freq.assign(m, 1);
  sentences_.freq = std::move(freq);
  if (need_host_text_) {
    sentences_.bytes.resize(total);
    sentences_.off.resize(m + 1);
    HIP_OR_RETURN(hipMemcpy(&sentences_.bytes[0], d_text, total, hipMemcpyDeviceToHost));
    HIP_OR_RETURN(hipMemcpy(sentences_.off.data(), d_off, (m + 1) * 8, hipMemcpyDeviceToHost));
  }
  return Status::Ok();
}

Status UnigramTrainer::LoadSentences() {
  const double t0 = Now();
  Corpus raw;
  RETURN_IF_ERROR(ReadCorpus(&raw));
  const double t1 = Now();
  read_s_ = t1 - t0;
  if (dev_lines_.bytes) {
    struct Release {
      UnigramTrainer *t;
      ~Release() { t->ReleaseDevLines(); }
    } release{this};
    RETURN_IF_ERROR(NormalizeDeviceCSR(dev_lines_.bytes, dev_lines_.off, dev_lines_.freq, dev_lines_.n, nullptr));
  } else {
    RETURN_IF_ERROR(NormalizeOnDevice(raw));
  }
  if (reaper_.joinable()) reaper_.join();
  reaper_ = std::thread([c = std::move(raw)]() mutable { c = Corpus(); });
  std::ostringstream os;
  os << "LoadSentences: read+parse " << t1 - t0 << " s, device normalize/count/replace "
     << Now() - t1 << " s (" << threads_ << " host threads)";
  Log(os.str());
  return Status::Ok();
}

// unigram_model_trainer.cc:124-225 on the device (spm_hip_seed_mine).
Status UnigramTrainer::MakeSeedSentencePieces(Pieces *out, TrainerTimings *tm) {
  // all_chars (:131-139) == the required chars' counts (every other char is
  // now kUNKChar, which all_chars skips).
  std::vector<uint32_t> chars;
  std::vector<int64_t> freq;
  for (auto &kv : required_chars_) {
    chars.push_back(kv.first);
    freq.push_back(kv.second);
  }
  spm_hip_seed_options o{};
  o.max_sentencepiece_length = spec_.max_sentencepiece_length;
  o.split_by_unicode_script = spec_.split_by_unicode_script;
  o.split_by_number = spec_.split_by_number;
  o.split_by_whitespace = spec_.split_by_whitespace;
  o.treat_whitespace_as_suffix = spec_.treat_whitespace_as_suffix;
  o.seed_sentencepiece_size = spec_.seed_sentencepiece_size;
  spm_hip_seeds *seeds = nullptr;
  const int rc = spm_hip_seed_mine_device(loaded_.bytes, loaded_.off, loaded_.n, chars.data(),
                                          freq.data(), chars.size(), &o, &seeds);
  if (rc != SPM_OK) return Err(rc, std::string("seed mining: ") + spm_hip_seed_last_error());
  const uint64_t k = spm_hip_seeds_size(seeds);
  const uint8_t *b = spm_hip_seeds_bytes(seeds);
  const uint64_t *so = spm_hip_seeds_offsets(seeds);
  const float *sc = spm_hip_seeds_scores(seeds);
  out->clear();
  out->reserve(k);
  for (uint64_t i = 0; i < k; ++i)
    out->emplace_back(std::string(reinterpret_cast<const char *>(b) + so[i], so[i + 1] - so[i]), sc[i]);
  uint64_t nc = 0, cand = 0;
  float ms = 0.f;
  spm_hip_seeds_stats(seeds, &nc, &cand, &ms);
  uint32_t ns = 0;
  float stages[7] = {};
  spm_hip_seeds_stage_times(seeds, stages, 7, &ns);
  spm_hip_seeds_free(seeds);
  if (tm) {
    tm->seed_candidates = cand;
    tm->seed_device_ms = ms;
    for (uint32_t k = 0; k < ns; ++k) tm->seed_stages[k] = stages[k];
  }
  Log("Initialized " + std::to_string(k) + " seed sentencepieces");
  return Status::Ok();
}

// trainer_interface.cc:465-477 + SplitIntoWords (model_interface.cc:155-190),
// per-thread hash maps keyed by views into the corpus arena.
// FNV-1a over the split result (words and freqs in order), for the log.
static std::string WordsDigest(const Corpus &c) {
  uint64_t h = 0xcbf29ce484222325ull;
  auto mix = [&](const void *p, size_t n) {
    for (size_t k = 0; k < n; ++k) h = (h ^ static_cast<const uint8_t *>(p)[k]) * 0x100000001b3ull;
  };
  for (size_t i = 0; i < c.size(); ++i) {
    mix(c.data(i), c.len(i));
    mix(&c.freq[i], 8);
  }
  char buf[24];
  snprintf(buf, sizeof(buf), "%016llx", static_cast<unsigned long long>(h));
  return buf;
}

Status UnigramTrainer::SplitSentencesByWhitespace() {
  const bool suffix = spec_.treat_whitespace_as_suffix;
  if (loaded_.bytes) {
    // The normalized corpus is resident in HBM: split and count on the
    // device (split_kernels.hip); only the unique words come back.
    SplitWords sw;
    const hipError_t e = opt_.host_split ? hipSuccess
                                         : CorpusSplitWords(loaded_.bytes, loaded_.off, loaded_.freq, loaded_.n,
                                                            suffix, &sw, nullptr);
    if (opt_.host_split) sw.fallback = true;
    if (e == hipSuccess && !sw.fallback) {
      std::vector<std::pair<std::string_view, int64_t>> v;
      v.reserve(sw.freq.size());
      for (size_t k = 0; k < sw.freq.size(); ++k)
        v.emplace_back(std::string_view(reinterpret_cast<const char *>(sw.bytes.data()) + sw.off[k],
                                        sw.off[k + 1] - sw.off[k]),
                       sw.freq[k]);
      v = Sorted(std::move(v));
      Corpus words;
      words.bytes.reserve(sw.bytes.size());
      for (auto &w : v) words.push(w.first.data(), w.first.size(), w.second);
      sentences_ = std::move(words);
      Log("Done! " + std::to_string(sentences_.size()) + " words (device split of " +
          std::to_string(sw.occurrences) + " occurrences, digest " + WordsDigest(sentences_) + ")");
      return Status::Ok();
    }
    if (e != hipSuccess) (void)hipGetLastError();
    Log(opt_.host_split     ? std::string("--host_split: host split")
        : e != hipSuccess   ? std::string("device split failed (") + hipGetErrorString(e) + "), host split"
                            : std::string("device split: hash collision or size limit, host split"));
    if (sentences_.bytes.size() != loaded_.total || sentences_.off.size() != loaded_.n + 1) {
      sentences_.bytes.resize(loaded_.total);
      sentences_.off.resize(loaded_.n + 1);
      HIP_OR_RETURN(hipMemcpy(sentences_.bytes.data(), loaded_.bytes, loaded_.total, hipMemcpyDeviceToHost));
      HIP_OR_RETURN(hipMemcpy(sentences_.off.data(), loaded_.off, (loaded_.n + 1) * 8, hipMemcpyDeviceToHost));
    }
    if (sentences_.freq.size() != loaded_.n) {  // (deferred by the device load)
      sentences_.freq.resize(loaded_.n);
      HIP_OR_RETURN(hipMemcpy(sentences_.freq.data(), loaded_.freq, loaded_.n * 8, hipMemcpyDeviceToHost));
    }
  }
  using Map = std::unordered_map<std::string_view, int64_t>;
  std::vector<Map> maps(threads_);
  ParallelChunks(sentences_.size(), threads_, [&](int t, uint64_t lo, uint64_t hi) {
    Map &tokens = maps[t];
    for (uint64_t i = lo; i < hi; ++i) {
      const char *s = sentences_.data(i);
      const size_t n = sentences_.len(i);
      const int64_t f = sentences_.freq[i];
      size_t b = 0, start = 0;
      bool open = false;
      while (b < n) {
        const size_t mblen = std::min<size_t>(OneCharLen(static_cast<uint8_t>(s[b])), n - b);
        const bool is_ws = mblen == 3 && std::memcmp(s + b, kWSStr, 3) == 0;
        if (suffix) {
          if (!open) {
            open = true;
            start = b;
          }
          b += mblen;
          if (b < n && is_ws) {
            tokens[std::string_view(s + start, b - start)] += f;
            open = false;
          }
        } else {
          if (b == 0 || is_ws) {
            if (open) tokens[std::string_view(s + start, b - start)] += f;
            open = true;
            start = b;
          }
          b += mblen;
        }
      }
      if (open) tokens[std::string_view(s + start, n - start)] += f;
    }
  });
  for (int t = 1; t < threads_; ++t) {
    for (auto &kv : maps[t]) maps[0][kv.first] += kv.second;
    Map().swap(maps[t]);
  }
  std::vector<std::pair<std::string_view, int64_t>> v(maps[0].begin(), maps[0].end());
  v = Sorted(std::move(v));
  Corpus words;
  uint64_t tb = 0;
  for (auto &w : v) tb += w.first.size();
  words.bytes.reserve(tb);
  for (auto &w : v) words.push(w.first.data(), w.first.size(), w.second);
  sentences_ = std::move(words);
  Log("Done! " + std::to_string(sentences_.size()) + " words (host split, digest " + WordsDigest(sentences_) + ")");
  return Status::Ok();
}

// The EM corpus on the device: the split words, or (no split) the loaded
// corpus itself.
Status UnigramTrainer::UploadCorpus(DeviceCorpus *out) {
  if (!spec_.split_by_whitespace && loaded_.bytes) {
    std::swap(out->bytes, loaded_.bytes);
    std::swap(out->off, loaded_.off);
    std::swap(out->freq, loaded_.freq);
    out->n = loaded_.n;
    out->total = loaded_.total;
    loaded_.Reset();
    return Status::Ok();
  }
  loaded_.Reset();
  const uint64_t n = sentences_.size();
  out->Reset();
  out->n = n;
  out->total = sentences_.bytes.size();
  if (DevMalloc(&out->bytes, std::max<uint64_t>(out->total, 1)) != hipSuccess ||
      DevMalloc(&out->off, (n + 1) * 8) != hipSuccess ||
      DevMalloc(&out->freq, std::max<uint64_t>(n, 1) * 8) != hipSuccess)
    return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
  if (hipMemcpy(out->bytes, sentences_.bytes.data(), out->total, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(out->off, sentences_.off.data(), (n + 1) * 8, hipMemcpyHostToDevice) != hipSuccess ||
      (n && hipMemcpy(out->freq, sentences_.freq.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess))
    return Err(SPM_INTERNAL, "device upload failed");
  return Status::Ok();
}

// Runs f(r) for every rank on its own host thread (device set), first error wins.
Status UnigramTrainer::RunRanks(const std::function<Status(int)> &f) {
  const int W = static_cast<int>(ranks_.size());
  std::vector<Status> st(W);
  auto body = [&](int r) {
    if (hipSetDevice(ranks_[r]->device) != hipSuccess) {
      st[r] = Err(SPM_INTERNAL, "hipSetDevice failed");
      return;
    }
    st[r] = f(r);
  };
  if (W == 1) {
    body(0);
  } else {
    std::vector<std::thread> th;
    for (int r = 0; r < W; ++r) th.emplace_back(body, r);
    for (auto &t : th) t.join();
  }
  (void)hipSetDevice(ranks_[0]->device);
  for (auto &x : st)
    if (!x.ok()) return x;
  return Status::Ok();
}

// Ranks, shard plans and shards (unigram_model_trainer.cc:237-287's thread
// fan-out mapped onto GPUs).  W = 1 keeps the corpus where it is.
Status UnigramTrainer::SetUpRanks() {
  const int W = std::max(1, opt_.num_gpus);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return Err(SPM_INTERNAL, "no HIP device");
  const bool parity = opt_.estep_mode == SPM_ESTEP_PARITY;
  const uint64_t n = sentences_.size();
  ranks_.clear();
  for (int r = 0; r < W; ++r) {
    auto rk = std::make_unique<Rank>();
    rk->device = r % ndev;
    rk->segs = EStepShardPlan(n, parity, spec_.num_threads, W, r);
    uint64_t b = 0;
    for (auto &sg : rk->segs) {
      rk->seg_begin.push_back(b);
      b += sg.count;
    }
    ranks_.push_back(std::move(rk));
  }
  if (W == 1) {
    RETURN_IF_ERROR(UploadCorpus(&ranks_[0]->shard));
  } else {
    loaded_.Reset();
    RETURN_IF_ERROR(RunRanks([&](int r) -> Status {
      Rank &rk = *ranks_[r];
      std::string bytes;
      std::vector<uint64_t> off{0};
      std::vector<int64_t> freq;
      for (auto &sg : rk.segs)
        for (uint64_t k = 0; k < sg.count; ++k) {
          const uint64_t i = sg.index_base + k * sg.index_stride;
          bytes.append(sentences_.data(i), sentences_.len(i));
          off.push_back(bytes.size());
          freq.push_back(sentences_.freq[i]);
        }
      DeviceCorpus &d = rk.shard;
      d.n = freq.size();
      d.total = bytes.size();
      if (DevMalloc(&d.bytes, std::max<uint64_t>(d.total, 1)) != hipSuccess ||
          DevMalloc(&d.off, (d.n + 1) * 8) != hipSuccess ||
          DevMalloc(&d.freq, std::max<uint64_t>(d.n, 1) * 8) != hipSuccess)
        return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
      if (hipMemcpy(d.bytes, bytes.data(), d.total, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(d.off, off.data(), (d.n + 1) * 8, hipMemcpyHostToDevice) != hipSuccess ||
          (d.n && hipMemcpy(d.freq, freq.data(), d.n * 8, hipMemcpyHostToDevice) != hipSuccess))
        return Err(SPM_INTERNAL, "device upload failed");
      return Status::Ok();
    }));
  }
  RETURN_IF_ERROR(RunRanks([&](int r) -> Status {
    return hipStreamCreateWithFlags(&ranks_[r]->stream, hipStreamNonBlocking) == hipSuccess
               ? Status::Ok()
               : Err(SPM_INTERNAL, "hipStreamCreate failed");
  }));
  // RCCL needs one device per rank; ranks that share a device (more ranks
  // than GPUs) reduce through the host instead.
  if (W > 1 && ndev >= W) {
    comms_.assign(W, nullptr);
    std::vector<int> devs(W);
    for (int r = 0; r < W; ++r) devs[r] = ranks_[r]->device;
    if (ncclCommInitAll(comms_.data(), W, devs.data()) != ncclSuccess) {
      comms_.clear();
      return Err(SPM_INTERNAL, "ncclCommInitAll failed");
    }
  }
  if (W > 1) {
    std::ostringstream os;
    os << "E-step/pruning ranks: " << W << " (devices";
    for (auto &rk : ranks_) os << " " << rk->device;
    os << "), reduction " << (comms_.empty() ? "through the host (ranks share a device)" : "RCCL");
    Log(os.str());
  }
  return Status::Ok();
}

// TrainerModel::SetSentencePieces (unigram_model_trainer.cc:97-119)
Status UnigramTrainer::SetModel(Pieces &&p) {
  if (p.empty()) return Err(SPM_INTERNAL, "empty piece list");
  pieces_ = std::move(p);
  min_score_ = FLT_MAX;
  for (auto &w : pieces_) {
    if (std::isnan(w.second)) return Err(SPM_INTERNAL, "NaN score");
    min_score_ = std::min(min_score_, w.second);
  }
  return Status::Ok();
}

struct PieceCSR {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off{0};
  std::vector<float> score;
  explicit PieceCSR(const Pieces &p) {
    for (auto &w : p) {
      bytes.insert(bytes.end(), w.first.begin(), w.first.end());
      off.push_back(bytes.size());
      score.push_back(w.second);
    }
    if (bytes.empty()) bytes.push_back(0);
  }
};

// Every rank's accumulator onto rank 0.
//   FAST  : SUM of fp64[V] + obj + ntok (ncclReduce).
//   PARITY: bucket b's float row, obj and ntok are accumulated by rank
//           b % W alone (the shard plan), so rank 0 GATHERS each row from its
//           owner (ncclSend / ncclRecv of the T/W rows a rank owns) — no
//           arithmetic on the rows, bit-exact by construction, and 1/W of a
//           zero-padded reduce's payload (T = 16, V = 320k: 2.6 MB instead of
//           20 MB per rank).  obj[T] / ntok[T] (a few bytes) are SUM-reduced:
//           exact, since every entry has one non-zero contributor.
// Every RCCL call's status is checked; a failure inside the group still
// closes it before returning.
Status UnigramTrainer::ReduceToRank0(int mode, uint64_t V, int T) {
  spm_amd::TraceRange trace_range_("trainer_rccl_reduce_to_rank0");
  const int W = static_cast<int>(ranks_.size());
  const bool fast = mode == SPM_ESTEP_FAST;
  const uint64_t nacc = fast ? V : static_cast<uint64_t>(T) * V;
  const uint64_t nobj = fast ? 1 : static_cast<uint64_t>(T);
  if (!comms_.empty()) {
    const ncclDataType_t ft = fast ? ncclFloat64 : ncclFloat32;
    std::string failed;
    auto nc = [&](ncclResult_t e, const char *what) {
      if (e != ncclSuccess && failed.empty()) failed = std::string(what) + ": " + ncclGetErrorString(e);
    };
    nc(ncclGroupStart(), "ncclGroupStart");
    if (failed.empty()) {
      for (int r = 0; r < W; ++r) {
        Rank &rk = *ranks_[r];
        char *a = rk.acc;
        if (fast) {
          nc(ncclReduce(a, a, nacc, ft, ncclSum, 0, comms_[r], rk.stream), "ncclReduce(acc)");
        } else {
          for (int b = 0; b < T; ++b) {
            const int owner = EStepBucketOwner(b, W);
            if (owner == 0) continue;
            char *row = a + static_cast<uint64_t>(b) * V * 4;
            if (r == owner) nc(ncclSend(row, V, ft, 0, comms_[r], rk.stream), "ncclSend(row)");
            if (r == 0) nc(ncclRecv(row, V, ft, owner, comms_[0], rk.stream), "ncclRecv(row)");
          }
        }
        nc(ncclReduce(a + acc_obj_at_, a + acc_obj_at_, nobj, ft, ncclSum, 0, comms_[r], rk.stream),
           "ncclReduce(obj)");
        nc(ncclReduce(a + acc_ntok_at_, a + acc_ntok_at_, nobj, ncclInt64, ncclSum, 0, comms_[r], rk.stream),
           "ncclReduce(ntok)");
      }
      nc(ncclGroupEnd(), "ncclGroupEnd");
    }
    if (!failed.empty()) return Err(SPM_INTERNAL, "RCCL: " + failed);
    return RunRanks([&](int r) -> Status {
      return hipStreamSynchronize(ranks_[r]->stream) == hipSuccess ? Status::Ok()
                                                                    : Err(SPM_INTERNAL, "RCCL reduce failed");
    });
  }
  // Ranks sharing a device: the same reduction through the host.
  const uint64_t bytes = acc_ntok_at_ + nobj * 8;
  std::vector<std::vector<char>> h(W, std::vector<char>(bytes));
  RETURN_IF_ERROR(RunRanks([&](int r) -> Status {
    return hipMemcpy(h[r].data(), ranks_[r]->acc, bytes, hipMemcpyDeviceToHost) == hipSuccess
               ? Status::Ok()
               : Err(SPM_INTERNAL, "accumulator download failed");
  }));
  auto add = [&](auto *zero_type, uint64_t at, uint64_t cnt) {
    using X = std::remove_pointer_t<decltype(zero_type)>;
    X *d = reinterpret_cast<X *>(h[0].data() + at);
    for (int r = 1; r < W; ++r) {
      const X *x = reinterpret_cast<const X *>(h[r].data() + at);
      for (uint64_t k = 0; k < cnt; ++k) d[k] += x[k];
    }
  };
  if (fast) {
    add(static_cast<double *>(nullptr), 0, nacc);
    add(static_cast<double *>(nullptr), acc_obj_at_, nobj);
  } else {
    for (int b = 0; b < T; ++b) {
      const int owner = EStepBucketOwner(b, W);
      if (owner == 0) continue;
      const uint64_t at = static_cast<uint64_t>(b) * V * 4;
      std::memcpy(h[0].data() + at, h[owner].data() + at, V * 4);
    }
    add(static_cast<float *>(nullptr), acc_obj_at_, nobj);
  }
  add(static_cast<int64_t *>(nullptr), acc_ntok_at_, nobj);
  if (hipMemcpy(ranks_[0]->acc, h[0].data(), bytes, hipMemcpyHostToDevice) != hipSuccess)
    return Err(SPM_INTERNAL, "accumulator upload failed");
  return Status::Ok();
}

// unigram_model_trainer.cc:237-287 on the device (PARITY: T = num_threads
// ordered float buckets, owned whole by one rank each; FAST: fp64).
Status UnigramTrainer::RunEStep(std::vector<float> *expected, float *obj, int64_t *ntok) {
  spm_amd::TraceRange trace_range_("trainer_estep");
  const uint64_t V = pieces_.size();
  PieceCSR csr(pieces_);
  int64_t all_freq = 0;
  for (int64_t f : sentences_.freq) all_freq += f;
  const int mode = opt_.estep_mode;
  const bool fast = mode == SPM_ESTEP_FAST;
  const int T = fast ? 1 : spec_.num_threads;
  auto align = [](uint64_t x) { return (x + 255) / 256 * 256; };
  const uint64_t acc_bytes = fast ? V * 8 : static_cast<uint64_t>(T) * V * 4;
  acc_obj_at_ = align(acc_bytes);
  acc_ntok_at_ = acc_obj_at_ + align(fast ? 8 : static_cast<uint64_t>(T) * 4);
  const uint64_t total = acc_ntok_at_ + (fast ? 8 : static_cast<uint64_t>(T) * 8);
  RETURN_IF_ERROR(RunRanks([&](int r) -> Status {
    Rank &rk = *ranks_[r];
    const double tb = Now();
    // The same piece list as the last E-step (the M-step dropped nothing):
    // new scores into the existing trie.
    int rc = SPM_INTERNAL;
    if (rk.pieces && rk.piece_off == csr.off && rk.piece_bytes == csr.bytes)
      rc = spm_hip_pieces_set_scores(rk.pieces, csr.score.data(), V);
    if (rc != SPM_OK) {
      if (rk.pieces) spm_hip_pieces_free(rk.pieces);
      rk.pieces = nullptr;
      rk.piece_bytes.clear();
      rk.piece_off.clear();
      rc = spm_hip_pieces_create(csr.bytes.data(), csr.off.data(), csr.score.data(), V, &rk.pieces);
      if (rc != SPM_OK) return Err(rc, "pieces_create failed");
      rk.piece_bytes = csr.bytes;
      rk.piece_off = csr.off;
    }
    if (r == 0) trie_build_s_ += Now() - tb;
    if (rk.acc_cap < total) {
      if (rk.acc) (void)DevFree(rk.acc);
      rk.acc = nullptr;
      rk.acc_cap = 0;
      if (DevMalloc(&rk.acc, total) != hipSuccess) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
      rk.acc_cap = total;
    }
    if (hipMemsetAsync(rk.acc, 0, total, rk.stream) != hipSuccess) return Err(SPM_INTERNAL, "memset failed");
    for (size_t k = 0; k < rk.segs.size(); ++k) {
      const ShardSegment &sg = rk.segs[k];
      const uint64_t b = rk.seg_begin[k];
      rc = spm_hip_estep_accumulate(rk.pieces, rk.shard.bytes, rk.shard.off + b, rk.shard.freq + b,
                                    sg.count, all_freq, mode, T, sg.index_base, sg.index_stride, rk.acc,
                                    rk.acc + acc_obj_at_,
                                    reinterpret_cast<int64_t *>(rk.acc + acc_ntok_at_), rk.stream);
      if (rc != SPM_OK) return Err(rc, std::string("E-step: ") + spm_hip_pieces_last_error(rk.pieces));
    }
    return hipStreamSynchronize(rk.stream) == hipSuccess ? Status::Ok() : Err(SPM_INTERNAL, "E-step failed");
  }));
  if (ranks_.size() > 1) RETURN_IF_ERROR(ReduceToRank0(mode, V, T));
  Rank &r0 = *ranks_[0];
  DevScratch sc;
  float *d_exp = sc.Get<float>(V), *d_obj = sc.Get<float>(1);
  int64_t *d_ntok = sc.Get<int64_t>(1);
  if (!d_exp || !d_obj || !d_ntok) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
  int rc = spm_hip_estep_finalize(r0.pieces, mode, T, r0.acc, r0.acc + acc_obj_at_,
                                  reinterpret_cast<const int64_t *>(r0.acc + acc_ntok_at_), d_exp, d_obj,
                                  d_ntok, r0.stream);
  if (rc == SPM_OK && hipStreamSynchronize(r0.stream) != hipSuccess) rc = SPM_INTERNAL;
  expected->assign(V, 0.f);
  if (rc == SPM_OK) {
    if (hipMemcpy(expected->data(), d_exp, V * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(obj, d_obj, 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(ntok, d_ntok, 8, hipMemcpyDeviceToHost) != hipSuccess)
      rc = SPM_INTERNAL;
  }
  if (rc != SPM_OK) return Err(rc, std::string("E-step: ") + spm_hip_pieces_last_error(r0.pieces));
  if (std::isnan(*obj)) return Err(SPM_INTERNAL, "likelihood is NAN");
  return Status::Ok();
}

// unigram_model_trainer.cc:47-57
double Digamma(double x) {
  double result = 0.0;
  for (; x < 7; ++x) result -= 1 / x;
  x -= 1.0 / 2.0;
  const double xx = 1.0 / x;
  const double xx2 = xx * xx;
  const double xx4 = xx2 * xx2;
  result += std::log(x) + (1.0 / 24.0) * xx2 - (7.0 / 960.0) * xx4 +
            (31.0 / 8064.0) * xx4 * xx2 - (127.0 / 30720.0) * xx4 * xx4;
  return result;
}

// unigram_model_trainer.cc:298-332
Pieces UnigramTrainer::RunMStep(const std::vector<float> &expected) const {
  Pieces out;
  float sum = 0.0f;
  for (size_t i = 0; i < expected.size(); ++i) {
    const float freq = expected[i];
    if (freq < 0.5f) continue;  // kExpectedFrequencyThreshold
    out.emplace_back(pieces_[i].first, freq);
    sum += freq;
  }
  const float logsum = static_cast<float>(Digamma(sum));
  for (auto &w : out) w.second = static_cast<float>(Digamma(w.second) - logsum);
  return out;
}

// unigram_model_trainer.cc:337-491.  NBest(2) per piece on host threads;
// the Viterbi over every sentence on the device; the float accumulation in
// the reference's thread-bucket order on the host.
Status UnigramTrainer::PruneSentencePieces(Pieces *out) {
  const size_t V = pieces_.size();
  std::vector<float> score(V);
  std::vector<std::pair<std::string, int32_t>> keys(V);
  for (size_t i = 0; i < V; ++i) {
    score[i] = pieces_[i].second;
    keys[i] = {pieces_[i].first, static_cast<int32_t>(i)};
  }
  // NBest(2) of every piece on the device (rank 0, spm_hip_prune_nbest);
  // pieces whose A* agenda outgrows the device slab are redone on the host.
  PieceCSR csr(pieces_);
  std::vector<uint8_t> always_keep(V, 1);
  std::vector<std::vector<int>> alternatives(V);
  {
    std::vector<uint64_t> alt_off(V + 1, 0);
    uint32_t max_bytes = 1;
    for (size_t i = 0; i < V; ++i) {
      const std::string &w = pieces_[i].first;
      uint64_t chars = 0;
      for (size_t q = 0; q < w.size(); q += std::max<size_t>(OneCharLen(static_cast<uint8_t>(w[q])), 1)) ++chars;
      alt_off[i + 1] = alt_off[i] + chars;
      max_bytes = std::max<uint32_t>(max_bytes, static_cast<uint32_t>(w.size()));
    }
    Rank &r0 = *ranks_[0];
    // The last E-step's piece set when the M-step kept every piece (new
    // scores into its trie), else a piece set of its own.
    spm_hip_pieces *hp = nullptr;
    std::unique_ptr<spm_hip_pieces, void (*)(spm_hip_pieces *)> hg(nullptr, spm_hip_pieces_free);
    const double tb = Now();
    int rc = SPM_INTERNAL;
    if (r0.pieces && r0.piece_off == csr.off && r0.piece_bytes == csr.bytes &&
        spm_hip_pieces_set_scores(r0.pieces, csr.score.data(), V) == SPM_OK) {
      hp = r0.pieces;
      rc = SPM_OK;
    } else {
      rc = spm_hip_pieces_create(csr.bytes.data(), csr.off.data(), csr.score.data(), V, &hp);
      hg.reset(hp);
    }
    trie_build_s_ += Now() - tb;
    if (rc != SPM_OK) return Err(rc, "pieces_create failed");
    DevScratch sc;
    uint8_t *d_pb = sc.Get<uint8_t>(csr.bytes.size());
    uint64_t *d_po = sc.Get<uint64_t>(V + 1), *d_ao = sc.Get<uint64_t>(V + 1);
    uint8_t *d_keep = sc.Get<uint8_t>(V);
    int32_t *d_alt = sc.Get<int32_t>(alt_off[V]);
    uint32_t *d_altn = sc.Get<uint32_t>(V);
    if (!d_pb || !d_po || !d_ao || !d_keep || !d_alt || !d_altn)
      return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    std::vector<uint32_t> alt_n(V);
    std::vector<int32_t> alt(std::max<uint64_t>(alt_off[V], 1));
    if (hipMemcpy(d_pb, csr.bytes.data(), csr.bytes.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_po, csr.off.data(), (V + 1) * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_ao, alt_off.data(), (V + 1) * 8, hipMemcpyHostToDevice) != hipSuccess)
      return Err(SPM_INTERNAL, "device upload failed");
    rc = spm_hip_prune_nbest(hp, d_pb, d_po, d_keep, d_alt, d_ao, d_altn, max_bytes, r0.stream);
    if (rc != SPM_OK) return Err(rc, std::string("NBest: ") + spm_hip_pieces_last_error(hp));
    if (hipStreamSynchronize(r0.stream) != hipSuccess ||
        hipMemcpy(always_keep.data(), d_keep, V, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(alt_n.data(), d_altn, V * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        (alt_off[V] && hipMemcpy(alt.data(), d_alt, alt_off[V] * 4, hipMemcpyDeviceToHost) != hipSuccess))
      return Err(SPM_INTERNAL, "NBest download failed");
    std::vector<uint64_t> redo;
    for (size_t i = 0; i < V; ++i) {
      if (always_keep[i] == 2) {
        always_keep[i] = 1;
        redo.push_back(i);
      } else {
        alternatives[i].assign(alt.begin() + alt_off[i], alt.begin() + alt_off[i] + alt_n[i]);
      }
    }
    nbest_host_redo_ += redo.size();
    if (!redo.empty()) {
      Log("NBest: " + std::to_string(redo.size()) + " pieces outgrew the device slab, redone on the host");
      DoubleArray trie;
      std::string err;
      const double tb = Now();
      if (!BuildDoubleArray(keys, &trie, &err)) return Err(SPM_RESOURCE_EXHAUSTED, err);
      trie_build_s_ += Now() - tb;
      ParallelChunks(redo.size(), threads_, [&](int, uint64_t lo, uint64_t hi) {
        HostLattice L;
        std::vector<std::pair<int32_t, size_t>> res;
        for (uint64_t j = lo; j < hi; ++j) {
          const uint64_t i = redo[j];
          L.Build(pieces_[i].first, trie, score, min_score_, &res);
          const auto nb = L.NBest2();
          if (nb.size() == 1) {
            always_keep[i] = 1;
          } else if (nb[0].size() >= 2) {
            always_keep[i] = 0;
          } else if (nb[0].size() == 1) {
            always_keep[i] = 1;
            for (int k : nb[1]) alternatives[i].push_back(L.nodes[k].id);
          }
        }
      });
    }
  }
  // Viterbi over all sentences: every rank encodes its shard on its device.
  const int W = static_cast<int>(ranks_.size());
  std::vector<std::vector<uint64_t>> rtok(W);
  std::vector<std::vector<int32_t>> rids(W);
  RETURN_IF_ERROR(RunRanks([&](int r) -> Status {
    Rank &rk = *ranks_[r];
    spm_hip_model *m = nullptr;
    const double tb = Now();
    int rc = spm_hip_model_from_pieces(csr.bytes.data(), csr.off.data(), csr.score.data(), V, &m);
    if (r == 0) trie_build_s_ += Now() - tb;
    if (rc != SPM_OK) return Err(rc, std::string("model_from_pieces: ") + spm_hip_last_error());
    std::unique_ptr<spm_hip_model, void (*)(spm_hip_model *)> mg(m, spm_hip_model_free);
    const uint64_t nl = rk.shard.n;
    DevScratch sc;
    int32_t *d_ids = sc.Get<int32_t>(rk.shard.total);
    uint64_t *d_tok = sc.Get<uint64_t>(nl + 1);
    if (!d_ids || !d_tok) return Err(SPM_RESOURCE_EXHAUSTED, "device allocation failed");
    rtok[r].assign(nl + 1, 0);
    if (nl) {
      rc = spm_hip_encode_batch(m, rk.shard.bytes, rk.shard.off, nl, d_ids, nullptr, d_tok, rk.stream);
      if (rc == SPM_OK && (hipStreamSynchronize(rk.stream) != hipSuccess ||
                           hipMemcpy(rtok[r].data(), d_tok, (nl + 1) * 8, hipMemcpyDeviceToHost) != hipSuccess))
        rc = SPM_INTERNAL;
    }
    if (rc == SPM_OK) {
      rids[r].resize(std::max<uint64_t>(rtok[r][nl], 1));
      if (hipMemcpy(rids[r].data(), d_ids, rtok[r][nl] * 4, hipMemcpyDeviceToHost) != hipSuccess)
        rc = SPM_INTERNAL;
    }
    return rc == SPM_OK ? Status::Ok() : Err(rc, std::string("pruning Viterbi: ") + spm_hip_last_error());
  }));
  const uint64_t n = sentences_.size();
  std::vector<uint64_t> tok;
  std::vector<int32_t> ids;
  if (W == 1) {
    tok = std::move(rtok[0]);
    ids = std::move(rids[0]);
  } else {
    // Back to global sentence order through the shard plans.
    tok.assign(n + 1, 0);
    for (int r = 0; r < W; ++r) {
      const Rank &rk = *ranks_[r];
      for (size_t k = 0; k < rk.segs.size(); ++k)
        for (uint64_t j = 0; j < rk.segs[k].count; ++j) {
          const uint64_t l = rk.seg_begin[k] + j;
          tok[rk.segs[k].index_base + j * rk.segs[k].index_stride + 1] = rtok[r][l + 1] - rtok[r][l];
        }
    }
    for (uint64_t i = 0; i < n; ++i) tok[i + 1] += tok[i];
    ids.resize(std::max<uint64_t>(tok[n], 1));
    for (int r = 0; r < W; ++r) {
      const Rank &rk = *ranks_[r];
      for (size_t k = 0; k < rk.segs.size(); ++k)
        for (uint64_t j = 0; j < rk.segs[k].count; ++j) {
          const uint64_t l = rk.seg_begin[k] + j;
          const uint64_t g = rk.segs[k].index_base + j * rk.segs[k].index_stride;
          std::copy(rids[r].begin() + rtok[r][l], rids[r].begin() + rtok[r][l + 1], ids.begin() + tok[g]);
        }
    }
  }
  // Thread buckets (:383-421): sentence i → bucket i mod T, float sums in order.
  const int T = spec_.num_threads;
  std::vector<float> vsums(T, 0.0f);
  std::vector<std::vector<float>> freqs(T, std::vector<float>(V, 0.0f));
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        for (uint64_t i = t; i < n; i += T) {
          const int64_t f = sentences_.freq[i];
          vsums[t] += f;
          for (uint64_t k = tok[i]; k < tok[i + 1]; ++k) freqs[t][ids[k]] += f;
        }
      });
    for (auto &x : th) x.join();
  }
  float vsum = 0.0f;
  std::vector<float> freq(V, 0.0f);
  for (int t = 0; t < T; ++t) {
    vsum += vsums[t];
    for (size_t i = 0; i < V; ++i) freq[i] += freqs[t][i];
  }
  // F[i] = sum over inverted[i] (bucket 0's occurrences in sentence order,
  // then bucket 1, ...) of sentences_.freq[n], in float.
  std::vector<float> F(V, 0.0f);
  for (int t = 0; t < T; ++t)
    for (uint64_t i = t; i < n; i += T) {
      const int64_t f = sentences_.freq[i];
      for (uint64_t k = tok[i]; k < tok[i + 1]; ++k) F[ids[k]] += f;
    }
  double dsum = 0.0;  // std::accumulate(freq.begin(), freq.end(), 0.0)
  for (float f : freq) dsum += f;
  const float sum = static_cast<float>(dsum);
  const float logsum = static_cast<float>(std::log(static_cast<double>(sum)));
  std::vector<std::pair<int, float>> candidates;
  out->clear();
  for (size_t i = 0; i < V; ++i) {
    if (freq[i] == 0 || !always_keep[i]) {
      continue;
    } else if (alternatives[i].empty()) {
      out->push_back(pieces_[i]);
    } else {
      float Fi = F[i];
      Fi /= vsum;
      const float logprob_sp = static_cast<float>(std::log(static_cast<double>(freq[i])) - logsum);
      // Note (reference :461): alternatives.size() is the size of the OUTER
      // vector (the piece count), kept as is for bit parity.
      const float logsum_alt = static_cast<float>(
          std::log(static_cast<double>(sum + freq[i] * static_cast<float>(V - 1))));
      float logprob_alt = 0.0f;
      for (int k : alternatives[i])
        logprob_alt = static_cast<float>(static_cast<double>(logprob_alt) +
                                         (std::log(static_cast<double>(freq[k] + freq[i])) -
                                          static_cast<double>(logsum_alt)));
      const float loss = Fi * (logprob_sp - logprob_alt);
      candidates.emplace_back(static_cast<int>(i), loss);
    }
  }
  const int pruned_size = std::max<int>(static_cast<int>(desired_vocab_size_),
                                        static_cast<int>(spec_.shrinking_factor * static_cast<float>(V)));
  for (auto &w : Sorted(std::move(candidates))) {
    if (out->size() == static_cast<size_t>(pruned_size)) break;
    out->push_back(pieces_[w.first]);
  }
  return Status::Ok();
}

// unigram_model_trainer.cc:497-537
Pieces UnigramTrainer::FinalizeSentencePieces() const {
  std::unordered_map<std::string, float> fin;
  std::unordered_map<std::string, float> sp(pieces_.begin(), pieces_.end());
  float min_score_penalty = 0.0f;
  const float kMinScorePenaltyDelta = 0.0001f;
  std::vector<std::pair<uint32_t, int64_t>> req(required_chars_.begin(), required_chars_.end());
  for (auto &w : Sorted(std::move(req))) {
    std::string s;
    AppendUTF8(w.first, &s);
    auto it = sp.find(s);
    if (it != sp.end()) {
      fin[s] = it->second;
    } else {
      fin[s] = min_score_ + min_score_penalty;
      min_score_penalty += kMinScorePenaltyDelta;
    }
  }
  const int vocab_size_size = spec_.vocab_size - static_cast<int>(meta_pieces_.size());
  for (auto &w : Sorted(pieces_)) {
    if (fin.count(w.first)) continue;
    if (static_cast<size_t>(vocab_size_size) == fin.size()) break;
    fin[w.first] = w.second;
  }
  return Sorted(Pieces(fin.begin(), fin.end()));
}

// trainer_interface.cc:479-530
Status UnigramTrainer::Serialize(std::vector<PieceRec> *out) const {
  out->clear();
  std::set<std::string> dup;
  size_t fid = 0;
  for (int id = 0; id < spec_.vocab_size; ++id) {
    auto it = meta_pieces_.find(id);
    PieceRec p;
    if (it != meta_pieces_.end()) {
      p.piece = it->second.first;
      p.type = it->second.second;
      p.score = 0.0f;
    } else if (fid < final_pieces_.size()) {
      p.piece = final_pieces_[fid].first;
      p.score = final_pieces_[fid].second;
      p.type = kNormal;
      ++fid;
    } else {
      continue;
    }
    if (p.piece.empty() || !dup.insert(p.piece).second)
      return Err(SPM_INTERNAL, p.piece + " is already defined");
    out->push_back(p);
  }
  if (fid != final_pieces_.size()) return Err(SPM_INTERNAL, "final pieces do not fit the vocab");
  if (spec_.hard_vocab_limit && static_cast<int>(out->size()) != spec_.vocab_size)
    return Err(SPM_INTERNAL, "Vocabulary size too high (" + std::to_string(spec_.vocab_size) +
                                 "). Please set it to a value <= " + std::to_string(out->size()) + ".");
  return Status::Ok();
}

// trainer_interface.cc:532-583 SaveModel / SaveVocab
Status UnigramTrainer::Save() const {
  std::vector<PieceRec> pieces;
  RETURN_IF_ERROR(Serialize(&pieces));
  TrainerSpec ts = spec_;
  if (!ts.hard_vocab_limit) {
    ts.vocab_size = static_cast<int32_t>(pieces.size());
    ts.has.insert(4);
  }
  const std::string model = SerializeModelProto(pieces, ts, norm_);
  {
    std::ofstream os(spec_.model_prefix + ".model", std::ios::binary);
    if (!os) return Err(SPM_PERMISSION_DENIED, "cannot write " + spec_.model_prefix + ".model");
    os.write(model.data(), model.size());
  }
  std::ofstream os(spec_.model_prefix + ".vocab", std::ios::binary);
  if (!os) return Err(SPM_PERMISSION_DENIED, "cannot write " + spec_.model_prefix + ".vocab");
  for (auto &p : pieces) {
    std::ostringstream line;
    line << p.piece << "\t" << p.score;
    os << line.str() << "\n";
  }
  return Status::Ok();
}


// trainer_interface.cc:178-267 IsValidSentencePiece (the seed kernels carry
// the device version; the BPE trainer checks merged pairs on the host).
bool UnigramTrainer::IsValidSentencePiece(const uint32_t *b, const uint32_t *e) const {
  const size_t size = e - b;
  if (size == 0 || size > static_cast<size_t>(spec_.max_sentencepiece_length)) return false;
  constexpr int kAny = -1;
  int prev = kAny;
  for (size_t pos = 0; pos < size; ++pos) {
    const uint32_t c = b[pos];
    if (c == kUNKChar || c == 0 || c == kUPPBoundaryChar || c == 0x20 || !IsValidCodepoint(c)) return false;
    if (c == 0x2581) {  // kWSChar
      const bool bad = spec_.treat_whitespace_as_suffix
                           ? (spec_.split_by_whitespace ? pos < size - 1 : (pos < size - 1 && pos == 0))
                           : (spec_.split_by_whitespace ? pos > 0 : (pos > 0 && pos == size - 1));
      if (bad) return false;
      continue;
    }
    int lo = 0, hi = kNumScriptRanges - 1, sc = kScriptCommon;
    while (lo <= hi) {
      const int mid = (lo + hi) / 2;
      if (c < kScriptRanges[mid].lo) hi = mid - 1;
      else if (c > kScriptRanges[mid].hi) lo = mid + 1;
      else {
        sc = kScriptRanges[mid].script;
        break;
      }
    }
    if (sc == kScriptHiragana || sc == kScriptKatakana || c == 0x30FC) sc = kScriptHan;
    if (!spec_.split_by_number && c >= 0x30 && c <= 0x39) sc = kAny;
    if (spec_.split_by_unicode_script && sc != kAny && prev != kAny && prev != sc) return false;
    prev = sc;
  }
  return true;
}

// ---- bpe::Trainer (bpe_model_trainer.cc:27-330) ----------------------------
// The pair census (every adjacent pair, its positions and freq, symbols in
// first-occurrence order) runs on the device (spm_hip_bpe_pair_census); the
// greedy merge loop is inherently sequential and runs here with the
// reference's data structures: the symbol cache is a
// std::unordered_map<uint64, Symbol*> that sees the reference's insertion and
// erase sequence (so UpdateActiveSymbols' partial_sort sees the same order),
// positions are ordered sets, fingerprints are util.h's FingerprintCat.  The
// active set is ordered by symbol creation (the reference orders it by heap
// address); it only breaks ties between symbols of equal freq, length and
// string.
namespace {
struct BpeSymbol {
  const BpeSymbol *left = nullptr, *right = nullptr;
  std::vector<uint32_t> chars;
  std::string str;  // ToString(), fixed at creation
  bool is_unk = false;
  uint64_t fp = 0, seq = 0;
  uint32_t id = 0;  // index into the dense per-symbol arrays (freq, bigram flag)
  std::set<uint64_t> positions;
  // Active-set bookkeeping of the merge loop: member of the active set; in
  // the ordered set (with ord_freq, the freq it was inserted with); queued
  // for ComputeFreq before the next selection.
  bool active = false, ordered = false, dirty = false;
  uint64_t ord_freq = 0;
  bool IsBigram() const { return left && right; }
  const std::string &ToString() const { return str; }
};
// The reference's selection order: freq desc, length asc, string asc; the
// first in active-set order (creation sequence here) among equals.  The
// ordered set keeps (freq, length) in its nodes, so most comparisons never
// touch the symbols themselves (they are scattered over the heap).
struct OrdKey {
  uint64_t freq;
  uint64_t len;
  const BpeSymbol *p;
};
struct BySelection {
  bool operator()(const OrdKey &a, const OrdKey &b) const {
    if (a.freq != b.freq) return a.freq > b.freq;
    if (a.len != b.len) return a.len < b.len;
    if (a.p == b.p) return false;
    const int c = a.p->str.compare(b.p->str);
    if (c != 0) return c < 0;
    return a.p->seq < b.p->seq;
  }
};
// Bump allocator for the symbol cache's nodes: nodes sit contiguously in
// creation order instead of between the symbols, strings and position sets
// allocated alongside them, so the full-cache walk of UpdateActiveSymbols'
// replay chases pointers within a few MB.  (The allocator does not change the
// hash table's iteration order: that depends only on keys, hashes and the
// insert/erase/rehash sequence.)  Freed nodes are not reused; the arena lives
// as long as the merge loop.
struct NodeArena {
  std::vector<std::unique_ptr<char[]>> blocks;
  size_t used = 0, cap = 0;
  void *Get(size_t bytes, size_t align) {
    used = (used + align - 1) & ~(align - 1);
    if (blocks.empty() || used + bytes > cap) {
      cap = std::max<size_t>(bytes, 1 << 20);
      blocks.emplace_back(new char[cap]);
      used = 0;
    }
    void *p = blocks.back().get() + used;
    used += bytes;
    return p;
  }
};
template <class T>
struct ArenaAlloc {
  using value_type = T;
  NodeArena *arena;
  explicit ArenaAlloc(NodeArena *a) : arena(a) {}
  template <class U>
  ArenaAlloc(const ArenaAlloc<U> &o) : arena(o.arena) {}
  T *allocate(size_t n) {
    // Bucket arrays go to the heap (they are replaced on every rehash).
    if (n != 1) return std::allocator<T>().allocate(n);
    return static_cast<T *>(arena->Get(sizeof(T), alignof(T)));
  }
  void deallocate(T *p, size_t n) {
    if (n != 1) std::allocator<T>().deallocate(p, n);
  }
  template <class U>
  bool operator==(const ArenaAlloc<U> &o) const { return arena == o.arena; }
  template <class U>
  bool operator!=(const ArenaAlloc<U> &o) const { return arena != o.arena; }
};

// util.h:613-662
uint64_t FingerprintCat(uint64_t a, uint64_t c) {
  uint64_t b = 0xe08c1d668b756f82ull;
  auto round = [&](int s1, int s2, int s3) {  // one third of mix(a, b, c)
    a -= b; a -= c; a ^= (c >> s1);
    b -= c; b -= a; b ^= (a << s2);
    c -= a; c -= b; c ^= (b >> s3);
  };
  round(43, 9, 8);
  round(38, 23, 5);
  round(35, 49, 11);
  round(12, 18, 22);
  return c;
}
}  // namespace

Status UnigramTrainer::TrainBpe(TrainerTimings *tm) {
  const double t0 = Now();
  if (spec_.split_by_whitespace) RETURN_IF_ERROR(SplitSentencesByWhitespace());
  const uint64_t n = sentences_.size();
  Log("Using " + std::to_string(n) + " sentences for BPE training");
  tm->em_sentences = n;
  DeviceCorpus dc;
  RETURN_IF_ERROR(UploadCorpus(&dc));
  spm_hip_bpe_census *cs = nullptr;
  int rc = spm_hip_bpe_pair_census(dc.bytes, dc.off, dc.freq, n, &cs, nullptr);
  if (rc != SPM_OK) return Err(rc, std::string("BPE pair census: ") + spm_hip_bpe_census_last_error());
  std::unique_ptr<spm_hip_bpe_census, void (*)(spm_hip_bpe_census *)> cg(cs, spm_hip_bpe_census_free);
  dc.Reset();
  const uint32_t *codes, *uchars;
  const uint64_t *coff, *pkeys, *pfreq, *poff, *ppos;
  uint64_t nuc = 0, npairs = 0;
  float dev_ms = 0.f;
  spm_hip_bpe_census_view(cs, &codes, &coff, &uchars, &nuc, &pkeys, &pfreq, &poff, &ppos, &npairs, &dev_ms);
  tm->seed_device_ms = dev_ms;
  tm->seed_candidates = npairs;

  std::vector<std::unique_ptr<BpeSymbol>> alloc;
  // symbols_cache_: fingerprint -> symbol id.  Its iteration order (what
  // UpdateActiveSymbols' partial_sort sees) depends only on the keys and the
  // insert/erase sequence, not on the mapped type; the freqs and bigram flags
  // live in dense arrays indexed by id, so the full-cache scan every 100
  // merges walks the map's nodes and two small arrays instead of
  // dereferencing every (heap-scattered) symbol.
  // Two arenas: every 8 refreshes the map is copied into the other one
  // (`relayout`), which allocates its nodes in iteration order, so the
  // refresh's full walk reads them front to back instead of hopping over
  // the creation-order arena; the copy keeps the bucket count, the rehash
  // policy's state and the node order (libstdc++ _Hashtable's copy
  // constructor appends the nodes in the source's order), so every later
  // insert, erase and walk behaves as on the original map.
  using CacheAlloc = ArenaAlloc<std::pair<const uint64_t, uint32_t>>;
  using CacheMap = std::unordered_map<uint64_t, uint32_t, std::hash<uint64_t>, std::equal_to<uint64_t>, CacheAlloc>;
  NodeArena arenas[2];
  int arena_k = 0;
  std::unique_ptr<CacheMap> cache_p(new CacheMap(CacheAlloc(&arenas[0])));  // (no bucket hint: as default-constructed)
  static const bool kRelayoutCheck = [] {  // test knob: the copy's walk must equal the original's
    const char *v = std::getenv("SPM_HIP_BPE_RELAYOUT_CHECK");
    return v && v[0] == '1';
  }();
  uint64_t relayouts = 0;
  auto relayout = [&]() -> bool {
    const int nk = arena_k ^ 1;
    arenas[nk] = NodeArena();
    std::unique_ptr<CacheMap> fresh(new CacheMap(*cache_p, CacheAlloc(&arenas[nk])));
    if (kRelayoutCheck) {
      if (fresh->bucket_count() != cache_p->bucket_count() || fresh->size() != cache_p->size()) return false;
      auto x = cache_p->begin();
      for (auto y = fresh->begin(); y != fresh->end(); ++x, ++y)
        if (x->first != y->first || x->second != y->second) return false;
    }
    cache_p = std::move(fresh);
    arena_k = nk;
    ++relayouts;
    return true;
  };
  std::vector<uint64_t> sfreq;  // Symbol::freq
  std::vector<uint8_t> sbig;    // Symbol::IsBigram()
  // The bigram symbols in the cache as a dense list (any order) with each
  // id's slot, for the order-free work of UpdateActiveSymbols.
  std::vector<uint32_t> live_big, live_slot;
  // The device refresh's todo list: every live bigram whose freq may be 0
  // (created, or reset by a merge), compacted at each refresh; with dense
  // left / right ids, so building it touches no symbol object.
  std::vector<uint32_t> zlist, sleft, sright;
  std::vector<uint8_t> inz, slive;
  auto zero_push = [&](const BpeSymbol *x) {
    if (!inz[x->id]) {
      inz[x->id] = 1;
      zlist.push_back(x->id);
    }
  };
  auto live_erase = [&](const BpeSymbol *x) {
    const uint32_t k = live_slot[x->id], last = live_big.back();
    live_big[k] = last;
    live_slot[last] = k;
    live_big.pop_back();
    slive[x->id] = 0;
  };
  auto F = [&](const BpeSymbol *x) -> uint64_t & { return sfreq[x->id]; };
  // The reference scans the whole active set and recomputes every freq each
  // step (:213-226).  Equivalent and incremental: active symbols with a
  // computed freq sit in `order` (BySelection); a symbol whose freq was reset
  // or whose positions grew while its freq is 0 is queued in `dirty` and
  // recomputed before the next selection; the best is order.begin().
  std::set<OrdKey, BySelection> order;
  std::vector<BpeSymbol *> dirty;
  std::vector<BpeSymbol *> activated;  // every symbol set active since the last UpdateActiveSymbols
  auto key_of = [](const BpeSymbol *x) { return OrdKey{x->ord_freq, x->chars.size(), x}; };
  auto unorder = [&](BpeSymbol *x) {
    if (x->ordered) {
      order.erase(key_of(x));
      x->ordered = false;
    }
  };
  auto mark_dirty = [&](BpeSymbol *x) {
    unorder(x);
    if (!x->dirty) {
      x->dirty = true;
      dirty.push_back(x);
    }
  };
  auto place = [&](BpeSymbol *x) {  // active, freq computed
    unorder(x);
    x->ord_freq = F(x);
    order.insert(key_of(x));
    x->ordered = true;
  };
  auto deactivate = [&](BpeSymbol *x) {
    unorder(x);
    x->active = false;
  };
  auto new_symbol = [&]() {
    alloc.emplace_back(new BpeSymbol());
    alloc.back()->seq = alloc.size();
    alloc.back()->id = static_cast<uint32_t>(alloc.size() - 1);
    sfreq.push_back(0);
    sbig.push_back(0);
    live_slot.push_back(0);
    sleft.push_back(0);
    sright.push_back(0);
    inz.push_back(0);
    slive.push_back(0);
    return alloc.back().get();
  };
  auto char_symbol = [&](uint32_t c) -> BpeSymbol * {  // GetCharSymbol :30-50
    auto it = cache_p->find(c);
    if (it != cache_p->end()) return alloc[it->second].get();
    auto rq = required_chars_.find(c);
    BpeSymbol *s = new_symbol();
    s->is_unk = c == kUNKChar;
    s->fp = c;
    s->chars.push_back(c);
    AppendUTF8(c, &s->str);
    F(s) = rq == required_chars_.end() ? 1 : static_cast<uint64_t>(rq->second);
    cache_p->emplace(s->fp, s->id);
    return s;
  };
  auto pair_symbol = [&](const BpeSymbol *l, const BpeSymbol *r) -> BpeSymbol * {  // GetPairSymbol :52-85
    if (!l || !r || l->is_unk || r->is_unk) return nullptr;
    const uint64_t fp = FingerprintCat(l->fp, r->fp);
    auto it = cache_p->find(fp);
    if (it != cache_p->end()) return alloc[it->second].get();
    std::vector<uint32_t> ut(l->chars);
    ut.insert(ut.end(), r->chars.begin(), r->chars.end());
    if (!IsValidSentencePiece(ut.data(), ut.data() + ut.size())) return nullptr;
    BpeSymbol *s = new_symbol();
    s->fp = fp;
    s->left = l;
    s->right = r;
    s->chars = std::move(ut);
    s->str = l->str + r->str;
    sbig[s->id] = 1;
    live_slot[s->id] = static_cast<uint32_t>(live_big.size());
    live_big.push_back(s->id);
    sleft[s->id] = l->id;
    sright[s->id] = r->id;
    slive[s->id] = 1;
    zero_push(s);
    cache_p->emplace(s->fp, s->id);
    return s;
  };
  // Symbols in the census order (= the reference's creation order).
  for (uint64_t k = 0; k < nuc; ++k) char_symbol(uchars[k]);
  std::vector<std::vector<BpeSymbol *>> syms(n);
  for (uint64_t i = 0; i < n; ++i) {
    syms[i].reserve(coff[i + 1] - coff[i]);
    for (uint64_t q = coff[i]; q < coff[i + 1]; ++q) syms[i].push_back(alloc[cache_p->find(codes[q])->second].get());
  }
  for (uint64_t k = 0; k < npairs; ++k) {
    BpeSymbol *s = pair_symbol(alloc[cache_p->find(pkeys[k] >> 21)->second].get(),
                               alloc[cache_p->find(pkeys[k] & 0x1FFFFFu)->second].get());
    if (!s) continue;
    s->active = true;  // (the first UpdateActiveSymbols rebuilds the set anyway)
    activated.push_back(s);
    for (uint64_t q = poff[k]; q < poff[k + 1]; ++q) s->positions.insert(s->positions.end(), ppos[q]);
    F(s) = pfreq[k];  // the first ComputeFreq, done by the census
  }
  // The pair-frequency refresh of UpdateActiveSymbols runs on the device
  // (spm_hip_bpe_refresh): its state is the sentences' symbol ids and every
  // bigram's position set; the loop below logs its changes for it.
  // SPM_HIP_BPE_DEVICE_REFRESH=0 keeps the refresh on host threads (A/B);
  // SPM_HIP_BPE_REFRESH_CHECK=1 also recomputes every refreshed freq on the
  // host and fails on any difference (test knob).
  static const bool kDeviceRefresh = [] {
    const char *v = std::getenv("SPM_HIP_BPE_DEVICE_REFRESH");
    return !(v && v[0] == '0');
  }();
  static const bool kRefreshCheck = [] {
    const char *v = std::getenv("SPM_HIP_BPE_REFRESH_CHECK");
    return v && v[0] == '1';
  }();
  std::unique_ptr<spm_hip_bpe_refresh, void (*)(spm_hip_bpe_refresh *)> refresh(nullptr, spm_hip_bpe_refresh_free);
  std::vector<uint64_t> wlog, ins_k, del_k;  // logs since the last refresh
  std::vector<uint32_t> ins_s, del_s;
  if (kDeviceRefresh) {
    std::vector<int32_t> flat(coff[n]);
    for (uint64_t i = 0; i < n; ++i)
      for (uint64_t q = coff[i]; q < coff[i + 1]; ++q) flat[q] = static_cast<int32_t>(syms[i][q - coff[i]]->id);
    std::vector<uint32_t> ps;
    std::vector<uint64_t> pk;
    for (const auto &x : alloc)  // symbol id order, each set ascending: sorted by (symbol, position)
      for (uint64_t v : x->positions) {
        ps.push_back(x->id);
        pk.push_back(v);
      }
    spm_hip_bpe_refresh *r = nullptr;
    rc = spm_hip_bpe_refresh_create(flat.data(), coff, sentences_.freq.data(), n, ps.data(), pk.data(), ps.size(),
                                    nullptr, &r);
    if (rc != SPM_OK) return Err(rc, std::string("BPE refresh: ") + spm_hip_bpe_census_last_error());
    refresh.reset(r);
  }
  const double t1 = Now();
  tm->seed = t1 - t0;

  auto compute_freq = [&](BpeSymbol *s) {  // :87-113
    uint64_t &freq = F(s);
    if (freq > 0) return;
    int64_t psid = -1, pright = 0;
    for (auto it = s->positions.begin(); it != s->positions.end();) {
      const uint64_t v = *it;
      const int64_t sid = static_cast<int64_t>(v >> 32), l = (v >> 16) & 0xffff, r = v & 0xffff;
      if ((sid == psid && l == pright) || s->left != syms[sid][l] || s->right != syms[sid][r]) {
        if (refresh) {
          del_s.push_back(s->id);
          del_k.push_back(v);
        }
        it = s->positions.erase(it);
        psid = -1;
        pright = 0;
      } else {
        freq += static_cast<uint64_t>(sentences_.freq[sid]);
        psid = sid;
        pright = r;
        ++it;
      }
    }
  };
  auto next_index = [&](uint64_t sid, int i) {
    for (size_t k = i + 1; k < syms[sid].size(); ++k)
      if (syms[sid][k]) return static_cast<int>(k);
    return -1;
  };
  auto prev_index = [&](uint64_t sid, int i) {
    for (int k = i - 1; k >= 0; --k)
      if (syms[sid][k]) return k;
    return -1;
  };
  auto add_pair = [&](uint64_t sid, int l, int r) {  // AddNewPair :131-141
    if (l == -1 || r == -1) return;
    BpeSymbol *s = pair_symbol(syms[sid][l], syms[sid][r]);
    if (s) {
      const uint64_t key = sid << 32 | static_cast<uint64_t>(l) << 16 | static_cast<uint64_t>(r);
      if (s->positions.insert(key).second && refresh) {
        ins_s.push_back(s->id);
        ins_k.push_back(key);
      }
      if (!s->active) {
        s->active = true;
        activated.push_back(s);
        if (F(s) == 0) mark_dirty(s);
        else place(s);  // a stale positive freq is kept, as the reference does
      } else if (F(s) == 0) {
        mark_dirty(s);  // new positions: the next ComputeFreq may find some
      }
    }
  };
  auto reset_freq = [&](uint64_t sid, int l, int r, const BpeSymbol *best) {  // :143-151
    if (l == -1 || r == -1) return;
    BpeSymbol *s = pair_symbol(syms[sid][l], syms[sid][r]);
    if (s && s != best && F(s) != 0) {
      F(s) = 0;
      zero_push(s);
      if (s->active) mark_dirty(s);
    }
  };
  // The kept set is always found by replaying partial_sort's heap phase: at
  // 10 M lines the order-free shortcut below (nth_element + a count) was
  // followed by a replay anyway in 293 of 320 updates (f* ties across the
  // boundary), so it cost more than it saved (update sort 0.62 -> 0.47 s).
  // SPM_HIP_BPE_ALWAYS_REPLAY=0 turns the shortcut back on (same kept set).
  static const bool kAlwaysReplay = [] {
    const char *v = std::getenv("SPM_HIP_BPE_ALWAYS_REPLAY");
    return !(v && v[0] == '0');
  }();
  // ComputeFreq of the live bigrams whose freq was reset, on the device: the
  // logged changes go up with the todo list; the erased positions come back
  // and leave the host sets too, so both sides keep the same sets.
  std::vector<uint32_t> todo;
  std::vector<uint64_t> tfreq;
  auto device_refresh = [&]() -> Status {
    const double r0 = Now();
    todo.clear();
    {
      size_t o = 0;
      for (uint32_t id : zlist) {
        if (!slive[id] || sfreq[id] != 0) {
          inz[id] = 0;
          continue;
        }
        zlist[o++] = id;
        todo.push_back(id);
        todo.push_back(sleft[id]);
        todo.push_back(sright[id]);
      }
      zlist.resize(o);
    }
    const uint64_t nt = todo.size() / 3;
    tm->bpe_refreshed += nt;
    // Symbol writes: the last one per position (the device scatters them in
    // parallel; a position merged twice in one interval must end as -1).
    std::stable_sort(wlog.begin(), wlog.end(), [](uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); });
    {
      size_t o = 0;
      for (size_t k = 0; k < wlog.size(); ++k) {
        if (k + 1 < wlog.size() && (wlog[k + 1] >> 32) == (wlog[k] >> 32)) continue;
        wlog[o++] = wlog[k];
      }
      wlog.resize(o);
    }
    // Inserts still in their sets, sorted by (symbol, position), once each.
    std::vector<std::pair<uint32_t, uint64_t>> ins;
    ins.reserve(ins_s.size());
    for (size_t k = 0; k < ins_s.size(); ++k)
      if (alloc[ins_s[k]]->positions.count(ins_k[k])) ins.emplace_back(ins_s[k], ins_k[k]);
    std::sort(ins.begin(), ins.end());
    ins.erase(std::unique(ins.begin(), ins.end()), ins.end());
    ins_s.resize(ins.size());
    ins_k.resize(ins.size());
    for (size_t k = 0; k < ins.size(); ++k) {
      ins_s[k] = ins[k].first;
      ins_k[k] = ins[k].second;
    }
    // The check knob: the host's ComputeFreq of every todo symbol on copies
    // of its sets (freq and erased positions), before the device runs.
    std::vector<uint64_t> hfreq;
    std::vector<std::pair<uint32_t, uint64_t>> herased;
    if (kRefreshCheck)
      for (uint64_t k = 0; k < nt; ++k) {
        BpeSymbol *x = alloc[todo[3 * k]].get();
        const std::set<uint64_t> keep = x->positions;
        const uint64_t f0 = F(x);
        const size_t d0 = del_s.size();
        compute_freq(x);
        hfreq.push_back(F(x));
        for (uint64_t v : keep)
          if (!x->positions.count(v)) herased.emplace_back(x->id, v);
        x->positions = keep;
        F(x) = f0;
        del_s.resize(d0);
        del_k.resize(d0);
      }
    tfreq.assign(nt, 0);
    const double r1 = Now();
    tm->bpe_refresh_prep += r1 - r0;
    const uint32_t *es = nullptr;
    const uint64_t *ek = nullptr;
    uint64_t ne = 0;
    const int rc2 = spm_hip_bpe_refresh_run(refresh.get(), wlog.data(), wlog.size(), ins_s.data(), ins_k.data(),
                                            ins_s.size(), del_s.data(), del_k.data(), del_s.size(), todo.data(), nt,
                                            tfreq.data(), &es, &ek, &ne);
    if (rc2 != SPM_OK) return Err(rc2, std::string("BPE refresh: ") + spm_hip_bpe_census_last_error());
    wlog.clear();
    ins_s.clear();
    ins_k.clear();
    del_s.clear();
    del_k.clear();
    const double r2 = Now();
    tm->bpe_refresh_call += r2 - r1;
    tm->bpe_refresh_erased += ne;
    for (uint64_t k = 0; k < nt; ++k) sfreq[todo[3 * k]] = tfreq[k];
    for (uint64_t k = 0; k < ne; ++k) alloc[es[k]]->positions.erase(ek[k]);
    tm->bpe_refresh_post += Now() - r2;
    if (kRefreshCheck) {
      std::vector<std::pair<uint32_t, uint64_t>> der(ne);
      for (uint64_t k = 0; k < ne; ++k) der[k] = {es[k], ek[k]};
      std::sort(der.begin(), der.end());
      std::sort(herased.begin(), herased.end());
      if (hfreq != tfreq || der != herased)
        return Err(SPM_INTERNAL, "BPE refresh check: device ComputeFreq differs from the host's (" +
                                     std::to_string(nt) + " symbols, " + std::to_string(ne) + " vs " +
                                     std::to_string(herased.size()) + " erased)");
      ++tm->bpe_refresh_checked;
    }
    return Status::Ok();
  };
  auto update_active = [&]() -> Status {  // UpdateActiveSymbols :153-183
    const double u0 = Now();
    // ComputeFreq of every bigram (symbols with a positive freq return at
    // once): on the device, or on host threads (different symbols touch
    // disjoint position sets and only read the symbol arrays).
    if (refresh) {
      Status st = device_refresh();
      if (!st.ok()) return st;
    } else {
      for (uint32_t id : live_big) tm->bpe_refreshed += sfreq[id] == 0;
      ParallelChunks(live_big.size(), threads_, [&](int, uint64_t lo, uint64_t hi) {
        for (uint64_t k = lo; k < hi; ++k)
          if (sfreq[live_big[k]] == 0) compute_freq(alloc[live_big[k]].get());
      });
    }
    const double u1 = Now();
    tm->bpe_update_freq += u1 - u0;
    const int nbig = static_cast<int>(live_big.size());
    const int size = std::min<int>(std::max<int>(1000, static_cast<int>(cache_p->size() * 0.05f)), nbig);
    // The reference keeps partial_sort's first `size` symbols of the cache's
    // iteration order.  Let f* be the size-th largest freq: every symbol with
    // freq > f* is kept, and which of the freq == f* symbols are kept depends
    // on the order only when more than `size` symbols have freq >= f*.  So
    // the kept SET is order-free unless f* ties across the boundary; the
    // active set itself is ordered by (freq, length, string, creation), never
    // by partial_sort's output order.
    std::vector<uint32_t> keep;
    keep.reserve(size);
    bool replay = true;
    if (size == nbig) {
      replay = false;
      keep = live_big;
    } else if (size > 0 && !kAlwaysReplay) {
      std::vector<uint64_t> fs(nbig);
      for (int k = 0; k < nbig; ++k) fs[k] = sfreq[live_big[k]];
      std::nth_element(fs.begin(), fs.begin() + (size - 1), fs.end(), std::greater<uint64_t>());
      const uint64_t fstar = fs[size - 1];
      int ge = 0;
      for (int k = 0; k < nbig; ++k) ge += sfreq[live_big[k]] >= fstar;
      replay = ge != size;
      if (!replay)
        for (int k = 0; k < nbig; ++k)
          if (sfreq[live_big[k]] >= fstar) keep.push_back(live_big[k]);
    }
    const double u2 = Now();
    tm->bpe_update_sort += u2 - u1;
    if (replay) {
      // f* ties across the boundary: replay partial_sort over the cache's
      // iteration order.  Its moves depend only on the comparisons'
      // outcomes, so sorting (freq, id) pairs gives the reference's
      // permutation.  libstdc++'s partial_sort heapifies [0, size) and then
      // visits the rest in order, inserting an element only when its freq
      // exceeds the heap top (the smallest freq held), which never
      // decreases: a tail element whose freq is <= the first heap's
      // smallest is never inserted and changes nothing, so it is left out.
      ++tm->bpe_update_replays;
      if (tm->bpe_updates % 8 == 0 && !relayout())
        return Err(SPM_INTERNAL, "BPE symbol cache relayout: the copy's iteration order differs");
      std::vector<uint32_t> v;
      v.reserve(nbig);
      for (auto &it : *cache_p)
        if (sbig[it.second]) v.push_back(it.second);
      const double u3 = Now();
      tm->bpe_update_scan += u3 - u2;
      uint64_t head_min = ~0ull;
      for (int k = 0; k < size; ++k) head_min = std::min(head_min, sfreq[v[k]]);
      // Only the kept SET matters (the active set is re-sorted below), so
      // the heap phase of libstdc++'s partial_sort (heap_select.h) is run alone, without its
      // final sort_heap, which only permutes the first `size` elements.
      // Elements are (freq, id) packed into 8 bytes (freq above kIdBits) when
      // both fit — the comparisons, and so the heap's moves, are the same as
      // on (freq, id) pairs with the freq-only comparator; half the bytes moved.
      constexpr int kIdBits = 26;
      uint64_t max_f = 0;
      for (uint32_t id : v) max_f = std::max(max_f, sfreq[id]);
      if (alloc.size() < (1ull << kIdBits) && max_f < (1ull << (64 - kIdBits))) {
        std::vector<uint64_t> fv;
        fv.reserve(v.size());
        for (int k = 0; k < size; ++k) fv.push_back(sfreq[v[k]] << kIdBits | v[k]);
        for (size_t k = size; k < v.size(); ++k)
          if (sfreq[v[k]] > head_min) fv.push_back(sfreq[v[k]] << kIdBits | v[k]);
        auto by_freq = [](uint64_t a, uint64_t b) { return (a >> kIdBits) > (b >> kIdBits); };
        HeapSelect(fv.begin(), fv.begin() + size, fv.end(), by_freq);
        for (int k = 0; k < size; ++k) keep.push_back(static_cast<uint32_t>(fv[k] & ((1ull << kIdBits) - 1)));
      } else {
        std::vector<std::pair<uint64_t, uint32_t>> fv;
        fv.reserve(v.size());
        for (int k = 0; k < size; ++k) fv.emplace_back(sfreq[v[k]], v[k]);
        for (size_t k = size; k < v.size(); ++k)
          if (sfreq[v[k]] > head_min) fv.emplace_back(sfreq[v[k]], v[k]);
        auto by_freq = [](const std::pair<uint64_t, uint32_t> &a, const std::pair<uint64_t, uint32_t> &b) {
          return a.first > b.first;
        };
        HeapSelect(fv.begin(), fv.begin() + size, fv.end(), by_freq);
        for (int k = 0; k < size; ++k) keep.push_back(fv[k].second);
      }
      tm->bpe_update_sort += Now() - u3;
    }
    for (const OrdKey &k : order) const_cast<BpeSymbol *>(k.p)->ordered = false;
    order.clear();
    for (BpeSymbol *x : dirty) x->dirty = false;
    dirty.clear();
    for (BpeSymbol *x : activated) x->active = false;
    activated.clear();
    // The new active set, inserted in selection order (hinted at the end).
    std::vector<OrdKey> keys(size);
    for (int k = 0; k < size; ++k) {
      BpeSymbol *x = alloc[keep[k]].get();
      x->active = true;
      x->ord_freq = sfreq[keep[k]];
      x->ordered = true;
      activated.push_back(x);
      keys[k] = key_of(x);
    }
    std::sort(keys.begin(), keys.end(), BySelection());
    for (const OrdKey &k : keys) order.emplace_hint(order.end(), k);
    ++tm->bpe_updates;
    tm->bpe_update += Now() - u0;
    return Status::Ok();
  };
  const int vocab = spec_.vocab_size - static_cast<int>(meta_pieces_.size()) -
                    static_cast<int>(required_chars_.size());
  if (vocab < 0) return Err(SPM_INTERNAL, "vocab_size is smaller than required_chars");
  std::unordered_set<std::string> dup;
  Pieces fin;
  while (fin.size() < static_cast<size_t>(vocab)) {  // :209-303
    if (fin.size() % 100 == 0) RETURN_IF_ERROR(update_active());
    const double d0 = Now();
    for (BpeSymbol *x : dirty) {
      x->dirty = false;
      if (!x->active) continue;
      compute_freq(x);
      place(x);
    }
    dirty.clear();
    tm->bpe_dirty += Now() - d0;
    BpeSymbol *best = order.empty() ? nullptr : const_cast<BpeSymbol *>(order.begin()->p);
    if (!best) {
      Log("No valid symbol found");
      break;
    }
    if (!dup.insert(best->ToString()).second) {
      cache_p->erase(best->fp);
      live_erase(best);
      deactivate(best);
      continue;
    }
    fin.emplace_back(best->ToString(), -static_cast<float>(fin.size()));
    const double a0 = Now();
    tm->bpe_positions += best->positions.size();
    for (uint64_t v : best->positions) {
      const uint64_t sid = v >> 32;
      const int l = (v >> 16) & 0xffff, r = v & 0xffff;
      if (!syms[sid][l]) continue;
      if (!syms[sid][r]) return Err(SPM_INTERNAL, "BPE merge: right symbol missing");
      const int next = next_index(sid, r), prev = prev_index(sid, l);
      reset_freq(sid, prev, l, best);
      reset_freq(sid, r, next, best);
      syms[sid][l] = best;
      syms[sid][r] = nullptr;
      if (refresh) {
        wlog.push_back((coff[sid] + static_cast<uint64_t>(l)) << 32 | best->id);
        wlog.push_back((coff[sid] + static_cast<uint64_t>(r)) << 32 | 0xFFFFFFFFull);
      }
      add_pair(sid, prev, l);
      add_pair(sid, l, next);
    }
    cache_p->erase(best->fp);
    live_erase(best);
    deactivate(best);
    tm->bpe_apply += Now() - a0;
  }
  if (refresh) spm_hip_bpe_refresh_stats(refresh.get(), nullptr, &tm->bpe_refresh_device_ms);
  // required chars last, in Sorted order (:316-320)
  std::vector<std::pair<uint32_t, int64_t>> req(required_chars_.begin(), required_chars_.end());
  for (auto &w : Sorted(std::move(req))) fin.emplace_back(char_symbol(w.first)->ToString(), -static_cast<float>(fin.size()));
  final_pieces_ = std::move(fin);
  tm->em_iterations = static_cast<int>(final_pieces_.size());
  tm->estep = Now() - t1;
  return Status::Ok();
}

// ---- EM-round checkpoints (no counterpart in the reference) ----
// The loop state at the top of an EM round is the piece list alone: the
// sentences, their split and the rank plan are recomputed from the corpus and
// spec on a resumed run, so the resumed model equals the uninterrupted one.
// Binary file: magic, round, sentence count, piece count, then per piece
// (uint32 byte length, bytes, uint32 float bits); written to <path>.tmp and
// renamed, so a crash mid-write leaves the previous round's file.
static const char kEmCheckpointMagic[8] = {'S', 'P', 'M', 'E', 'M', 'C', 'K', '1'};

static Status WriteEmCheckpoint(const std::string &path, const Pieces &pieces, uint32_t round, uint64_t sentences) {
  const std::string tmp = path + ".tmp";
  {
    std::ofstream os(tmp, std::ios::binary | std::ios::trunc);
    if (!os) return Err(SPM_INTERNAL, "cannot write EM checkpoint " + tmp);
    const uint64_t n = pieces.size();
    os.write(kEmCheckpointMagic, 8);
    os.write(reinterpret_cast<const char *>(&round), 4);
    os.write(reinterpret_cast<const char *>(&sentences), 8);
    os.write(reinterpret_cast<const char *>(&n), 8);
    for (auto &w : pieces) {
      const uint32_t len = static_cast<uint32_t>(w.first.size());
      uint32_t bits;
      std::memcpy(&bits, &w.second, 4);
      os.write(reinterpret_cast<const char *>(&len), 4);
      os.write(w.first.data(), len);
      os.write(reinterpret_cast<const char *>(&bits), 4);
    }
    if (!os.flush()) return Err(SPM_INTERNAL, "cannot write EM checkpoint " + tmp);
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) return Err(SPM_INTERNAL, "cannot rename " + tmp);
  return Status::Ok();
}

static Status ReadEmCheckpoint(const std::string &path, Pieces *pieces, uint32_t *round, uint64_t *sentences) {
  std::ifstream is(path, std::ios::binary);
  if (!is) return Err(SPM_NOT_FOUND, "cannot open EM checkpoint " + path);
  char magic[8];
  uint64_t n = 0;
  is.read(magic, 8);
  is.read(reinterpret_cast<char *>(round), 4);
  is.read(reinterpret_cast<char *>(sentences), 8);
  is.read(reinterpret_cast<char *>(&n), 8);
  if (!is || std::memcmp(magic, kEmCheckpointMagic, 8) != 0 || n > (1ull << 32))
    return Err(SPM_INVALID_ARGUMENT, "not an EM checkpoint: " + path);
  pieces->clear();
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t len = 0, bits = 0;
    is.read(reinterpret_cast<char *>(&len), 4);
    if (!is || len > 4096) return Err(SPM_INVALID_ARGUMENT, "truncated EM checkpoint: " + path);
    std::string w(len, '\0');
    is.read(&w[0], len);
    is.read(reinterpret_cast<char *>(&bits), 4);
    if (!is) return Err(SPM_INVALID_ARGUMENT, "truncated EM checkpoint: " + path);
    float f;
    std::memcpy(&f, &bits, 4);
    pieces->emplace_back(std::move(w), f);
  }
  return Status::Ok();
}

// unigram_model_trainer.cc:539-603
Status UnigramTrainer::Train(TrainerTimings *tm) {
  TrainerTimings local;
  TrainerTimings &t = tm ? *tm : local;
  const double t0 = Now();
  // Device high-water marks per stage (scratch_cache.h DevMalloc accounting).
  DevPeakReset();
  auto stage_peak = [&t](int k) {
    t.stage_peak_bytes[k] = DevPeakBytes();
    t.peak_device_bytes = std::max(t.peak_device_bytes, t.stage_peak_bytes[k]);
    DevPeakReset();
  };
  RETURN_IF_ERROR(VerifySpec());
  RETURN_IF_ERROR(InitMetaPieces());
  // The BPE trainer (bpe_model_trainer.cc:185-330) runs on one device: its
  // merge loop is one sequential chain; --num_gpus shards only the unigram
  // E-step and pruning.  (escape_whitespaces, which both trainers require,
  // bpe_model_trainer.cc:189 / unigram_model_trainer.cc:543, is checked by
  // VerifySpec above.)
  const bool bpe = spec_.model_type == kBpe;
  if (bpe && opt_.num_gpus > 1) Log("--num_gpus is ignored for --model_type=bpe (one device)");
  // The whitespace split runs on the device corpus (host text only for its
  // rare fallback, fetched then); sharding the unsplit corpus over ranks
  // needs it on the host.
  need_host_text_ = opt_.num_gpus > 1 && !bpe && !spec_.split_by_whitespace;
  RETURN_IF_ERROR(LoadSentences());
  t.sentences = host_freq_deferred_ ? loaded_.n : sentences_.size();
  const double t1 = Now();
  t.load = t1 - t0;
  t.read = read_s_;
  stage_peak(0);
  if (spec_.model_type == kBpe) {  // bpe_model_trainer.cc:185-330
    RETURN_IF_ERROR(TrainBpe(&t));
    const double t4 = Now();
    RETURN_IF_ERROR(Save());
    t.finalize = Now() - t4;
    t.total = Now() - t0;
    t.trie_build = trie_build_s_;
    stage_peak(3);
    return Status::Ok();
  }
  Pieces seeds;
  // The seed and split stages' device scratch is recycled between them
  // (scratch_cache.h); the cache is emptied before the E-steps.
  auto cache = std::make_unique<ScratchCacheScope>();
  // SPM_HIP_EM_CHECKPOINT=<file>: the piece list at the top of every EM
  // round; SPM_HIP_EM_RESUME=<file>: start from such a file's round instead
  // of mining seeds; SPM_HIP_EM_STOP_BEFORE=<r>: fail once round r's
  // checkpoint is written (tests).  (spm_train: --em_checkpoint,
  // --resume_from.)
  const char *ck_env = std::getenv("SPM_HIP_EM_CHECKPOINT");
  const char *resume_env = std::getenv("SPM_HIP_EM_RESUME");
  const char *stop_env = std::getenv("SPM_HIP_EM_STOP_BEFORE");
  const std::string ck_path = ck_env ? ck_env : "";
  const long stop_before = stop_env && *stop_env ? std::atol(stop_env) : -1;
  uint32_t round = 0;
  if (resume_env && *resume_env) {
    uint64_t ck_sentences = 0;
    RETURN_IF_ERROR(ReadEmCheckpoint(resume_env, &seeds, &round, &ck_sentences));
    if (ck_sentences != t.sentences)
      return Err(SPM_INVALID_ARGUMENT, "EM checkpoint " + std::string(resume_env) + " is of another corpus (" +
                                           std::to_string(ck_sentences) + " sentences, this one " +
                                           std::to_string(t.sentences) + ")");
    Log("Resumed EM round " + std::to_string(round) + " with " + std::to_string(seeds.size()) + " pieces");
  } else {
    RETURN_IF_ERROR(MakeSeedSentencePieces(&seeds, &t));
  }
  if (!opt_.dump_seeds.empty()) {
    std::ofstream os(opt_.dump_seeds, std::ios::binary);
    for (auto &w : seeds) {
      os.write(w.first.data(), w.first.size());
      os << "\t";
      char buf[32];
      uint32_t u;
      std::memcpy(&u, &w.second, 4);
      snprintf(buf, sizeof(buf), "%08x", u);
      os << buf << "\n";
    }
  }
  RETURN_IF_ERROR(SetModel(std::move(seeds)));
  const double t2 = Now();
  t.seed = t2 - t1;
  stage_peak(1);
  if (spec_.split_by_whitespace) RETURN_IF_ERROR(SplitSentencesByWhitespace());
  cache.reset();
  Log("Using " + std::to_string(sentences_.size()) + " sentences for EM training");
  t.em_sentences = sentences_.size();
  RETURN_IF_ERROR(SetUpRanks());
  const double t3 = Now();
  t.split = t3 - t2;
  stage_peak(2);
  desired_vocab_size_ = static_cast<size_t>(spec_.vocab_size * 1.1);
  for (;; ++round) {
    if (!ck_path.empty()) RETURN_IF_ERROR(WriteEmCheckpoint(ck_path, pieces_, round, t.sentences));
    if (stop_before >= 0 && static_cast<long>(round) == stop_before)
      return Err(SPM_OUT_OF_RANGE, "stopped before EM round " + std::to_string(round) + " (SPM_HIP_EM_STOP_BEFORE)");
    for (int iter = 0; iter < spec_.num_sub_iterations; ++iter) {
      float objective = 0.0f;
      int64_t num_tokens = 0;
      std::vector<float> expected;
      const double a = Now();
      RETURN_IF_ERROR(RunEStep(&expected, &objective, &num_tokens));
      const double b = Now();
      RETURN_IF_ERROR(SetModel(RunMStep(expected)));
      t.estep += b - a;
      t.mstep += Now() - b;
      ++t.em_iterations;
      std::ostringstream os;
      os << "EM sub_iter=" << iter << " size=" << pieces_.size() << " obj=" << objective
         << " num_tokens=" << num_tokens
         << " num_tokens/piece=" << 1.0 * num_tokens / pieces_.size();
      Log(os.str());
    }
    if (pieces_.size() <= desired_vocab_size_) break;
    const double a = Now();
    Pieces pruned;
    RETURN_IF_ERROR(PruneSentencePieces(&pruned));
    RETURN_IF_ERROR(SetModel(std::move(pruned)));
    t.prune += Now() - a;
  }
  const double t4 = Now();
  final_pieces_ = FinalizeSentencePieces();
  RETURN_IF_ERROR(Save());
  t.finalize = Now() - t4;
  t.total = Now() - t0;
  t.trie_build = trie_build_s_;
  stage_peak(3);
  return Status::Ok();
}

}  // namespace

// ---- spec parsing ----------------------------------------------------------
Status SetTrainerField(const std::string &k, const std::string &v, TrainerSpec *s) {
  auto bad = [&](const char *ty) { return Err(SPM_INVALID_ARGUMENT, "cannot parse \"" + v + "\" as " + ty + "."); };
  auto i32 = [&](int field, int32_t *dst) -> Status {
    if (!LexicalCast(v, dst)) return bad("int32");
    s->has.insert(field);
    return Status::Ok();
  };
  auto f32 = [&](int field, float *dst) -> Status {
    if (!LexicalCast(v, dst)) return bad("float");
    s->has.insert(field);
    return Status::Ok();
  };
  auto bl = [&](int field, bool *dst) -> Status {
    if (!LexicalCastBool(v.empty() ? "true" : v, dst)) return bad("bool");
    s->has.insert(field);
    return Status::Ok();
  };
  auto str = [&](int field, std::string *dst) -> Status {
    *dst = v;
    s->has.insert(field);
    return Status::Ok();
  };
  auto rep = [&](int field, std::vector<std::string> *dst) -> Status {
    for (auto &x : Split(v, ',')) dst->push_back(x);
    s->has.insert(field);
    return Status::Ok();
  };
  if (k == "input") return rep(1, &s->input);
  if (k == "input_format") return str(7, &s->input_format);
  if (k == "model_prefix") return str(2, &s->model_prefix);
  if (k == "model_type") {
    std::string u = v;
    std::transform(u.begin(), u.end(), u.begin(), ::toupper);
    const std::map<std::string, int> m = {{"UNIGRAM", 1}, {"BPE", 2}, {"WORD", 3}, {"CHAR", 4}};
    auto it = m.find(u);
    if (it == m.end()) return Err(SPM_INVALID_ARGUMENT, "unknown enumeration value of \"" + v + "\" as ModelType.");
    s->model_type = it->second;
    s->has.insert(3);
    return Status::Ok();
  }
  if (k == "vocab_size") return i32(4, &s->vocab_size);
  if (k == "accept_language") return rep(5, &s->accept_language);
  if (k == "self_test_sample_size") return i32(6, &s->self_test_sample_size);
  if (k == "character_coverage") return f32(10, &s->character_coverage);
  if (k == "input_sentence_size") return i32(11, &s->input_sentence_size);
  if (k == "shuffle_input_sentence") return bl(19, &s->shuffle_input_sentence);
  if (k == "seed_sentencepiece_size") return i32(14, &s->seed_sentencepiece_size);
  if (k == "shrinking_factor") return f32(15, &s->shrinking_factor);
  if (k == "max_sentence_length") return i32(18, &s->max_sentence_length);
  if (k == "num_threads") return i32(16, &s->num_threads);
  if (k == "num_sub_iterations") return i32(17, &s->num_sub_iterations);
  if (k == "max_sentencepiece_length") return i32(20, &s->max_sentencepiece_length);
  if (k == "split_by_unicode_script") return bl(21, &s->split_by_unicode_script);
  if (k == "split_by_number") return bl(23, &s->split_by_number);
  if (k == "split_by_whitespace") return bl(22, &s->split_by_whitespace);
  if (k == "treat_whitespace_as_suffix") return bl(24, &s->treat_whitespace_as_suffix);
  if (k == "control_symbols") return rep(30, &s->control_symbols);
  if (k == "user_defined_symbols") return rep(31, &s->user_defined_symbols);
  if (k == "hard_vocab_limit") return bl(33, &s->hard_vocab_limit);
  if (k == "use_all_vocab") return bl(34, &s->use_all_vocab);
  if (k == "unk_id") return i32(40, &s->unk_id);
  if (k == "bos_id") return i32(41, &s->bos_id);
  if (k == "eos_id") return i32(42, &s->eos_id);
  if (k == "pad_id") return i32(43, &s->pad_id);
  if (k == "unk_surface") return str(44, &s->unk_surface);
  if (k == "unk_piece") return str(45, &s->unk_piece);
  if (k == "bos_piece") return str(46, &s->bos_piece);
  if (k == "eos_piece") return str(47, &s->eos_piece);
  if (k == "pad_piece") return str(48, &s->pad_piece);
  return Err(SPM_NOT_FOUND, "unknown field name \"" + k + "\" in TrainerSpec.");
}

Status SetNormalizerField(const std::string &k, const std::string &v, NormalizerSpec *s) {
  auto bl = [&](int field, bool *dst) -> Status {
    if (!LexicalCastBool(v.empty() ? "true" : v, dst))
      return Err(SPM_INVALID_ARGUMENT, "cannot parse \"" + v + "\" as bool.");
    s->has.insert(field);
    return Status::Ok();
  };
  if (k == "name") return s->name = v, s->has.insert(1), Status::Ok();
  if (k == "precompiled_charsmap") return s->precompiled_charsmap = v, s->has.insert(2), Status::Ok();
  if (k == "add_dummy_prefix") return bl(3, &s->add_dummy_prefix);
  if (k == "remove_extra_whitespaces") return bl(4, &s->remove_extra_whitespaces);
  if (k == "escape_whitespaces") return bl(5, &s->escape_whitespaces);
  if (k == "normalization_rule_tsv")
    return s->normalization_rule_tsv = v, s->has.insert(6), Status::Ok();
  return Err(SPM_NOT_FOUND, "unknown field name \"" + k + "\" in NormalizerSpec.");
}

// sentencepiece_trainer.cc:53-97
Status SentencePieceTrainer::MergeSpecsFromArgs(const std::string &args, TrainerSpec *ts,
                                                NormalizerSpec *ns) {
  for (auto arg : Split(args, ' ')) {
    if (arg.compare(0, 2, "--") == 0) arg = arg.substr(2);
    const size_t eq = arg.find('=');
    const std::string key = arg.substr(0, eq);
    const std::string value = eq == std::string::npos ? "" : arg.substr(eq + 1);
    if (key == "normalization_rule_name") {
      ns->name = value;
      ns->has.insert(1);
      continue;
    }
    if (key == "minloglevel") continue;
    Status st = SetTrainerField(key, value, ts);
    if (st.ok()) continue;
    if (st.code != SPM_NOT_FOUND) return st;
    Status sn = SetNormalizerField(key, value, ns);
    if (sn.ok()) continue;
    if (sn.code != SPM_NOT_FOUND) return sn;
    return st;
  }
  return Status::Ok();
}

// sentencepiece_trainer.cc:109-136 (+ Builder::GetPrecompiledCharsMap,
// builder.cc:280-299, with the rule blobs as files).
Status SentencePieceTrainer::PopulateNormalizerSpec(NormalizerSpec *ns, const std::string &rules_dir) {
  if (!ns->normalization_rule_tsv.empty())
    return Err(SPM_UNIMPLEMENTED, "--normalization_rule_tsv (charsmap compilation) is not supported");
  if (ns->name.empty()) {
    ns->name = "nmt_nfkc";
    ns->has.insert(1);
  }
  if (ns->precompiled_charsmap.empty()) {
    ns->has.insert(2);
    if (ns->name == "identity") return Status::Ok();
    const std::string path = rules_dir + "/" + ns->name + ".bin";
    std::ifstream is(path, std::ios::binary);
    if (!is) return Err(SPM_NOT_FOUND, "No precompiled charsmap is found: " + ns->name);
    ns->precompiled_charsmap.assign(std::istreambuf_iterator<char>(is), std::istreambuf_iterator<char>());
  }
  return Status::Ok();
}

Status SentencePieceTrainer::Train(const TrainerSpec &ts, const NormalizerSpec &ns,
                                   const TrainerOptions &opt, TrainerTimings *tm) {
  NormalizerSpec copied = ns;
  RETURN_IF_ERROR(PopulateNormalizerSpec(&copied, opt.rules_dir));
  UnigramTrainer trainer(ts, copied, opt);
  return trainer.Train(tm);
}

Status SentencePieceTrainer::Train(const std::string &args, const TrainerOptions &opt,
                                   TrainerTimings *tm) {
  TrainerSpec ts;
  NormalizerSpec ns;
  RETURN_IF_ERROR(MergeSpecsFromArgs(args, &ts, &ns));
  return Train(ts, ns, opt, tm);
}

// ModelProto (sentencepiece_model.proto:240-275): fields in number order, as
// protobuf's generated serializer writes them; optional fields only when set.
std::string SerializeModelProto(const std::vector<PieceRec> &pieces, const TrainerSpec &ts,
                                const NormalizerSpec &ns) {
  std::string out;
  for (const auto &p : pieces) {
    std::string sp;
    PutBytes(1, p.piece, &sp);
    PutFloat(2, p.score, &sp);
    if (p.type != kNormal) PutInt32(3, p.type, &sp);
    PutBytes(1, sp, &out);
  }
  std::string t;
  auto has = [&](int f) { return ts.has.count(f) > 0; };
  for (auto &x : ts.input) PutBytes(1, x, &t);
  if (has(2)) PutBytes(2, ts.model_prefix, &t);
  if (has(3)) PutInt32(3, ts.model_type, &t);
  if (has(4)) PutInt32(4, ts.vocab_size, &t);
  for (auto &x : ts.accept_language) PutBytes(5, x, &t);
  if (has(6)) PutInt32(6, ts.self_test_sample_size, &t);
  if (has(7)) PutBytes(7, ts.input_format, &t);
  if (has(10)) PutFloat(10, ts.character_coverage, &t);
  if (has(11)) PutInt32(11, ts.input_sentence_size, &t);
  if (has(14)) PutInt32(14, ts.seed_sentencepiece_size, &t);
  if (has(15)) PutFloat(15, ts.shrinking_factor, &t);
  if (has(16)) PutInt32(16, ts.num_threads, &t);
  if (has(17)) PutInt32(17, ts.num_sub_iterations, &t);
  if (has(18)) PutInt32(18, ts.max_sentence_length, &t);
  if (has(19)) PutBool(19, ts.shuffle_input_sentence, &t);
  if (has(20)) PutInt32(20, ts.max_sentencepiece_length, &t);
  if (has(21)) PutBool(21, ts.split_by_unicode_script, &t);
  if (has(22)) PutBool(22, ts.split_by_whitespace, &t);
  if (has(23)) PutBool(23, ts.split_by_number, &t);
  if (has(24)) PutBool(24, ts.treat_whitespace_as_suffix, &t);
  for (auto &x : ts.control_symbols) PutBytes(30, x, &t);
  for (auto &x : ts.user_defined_symbols) PutBytes(31, x, &t);
  if (has(33)) PutBool(33, ts.hard_vocab_limit, &t);
  if (has(34)) PutBool(34, ts.use_all_vocab, &t);
  if (has(40)) PutInt32(40, ts.unk_id, &t);
  if (has(41)) PutInt32(41, ts.bos_id, &t);
  if (has(42)) PutInt32(42, ts.eos_id, &t);
  if (has(43)) PutInt32(43, ts.pad_id, &t);
  if (has(44)) PutBytes(44, ts.unk_surface, &t);
  if (has(45)) PutBytes(45, ts.unk_piece, &t);
  if (has(46)) PutBytes(46, ts.bos_piece, &t);
  if (has(47)) PutBytes(47, ts.eos_piece, &t);
  if (has(48)) PutBytes(48, ts.pad_piece, &t);
  PutBytes(2, t, &out);
  std::string n;
  auto nhas = [&](int f) { return ns.has.count(f) > 0; };
  if (nhas(1)) PutBytes(1, ns.name, &n);
  if (nhas(2)) PutBytes(2, ns.precompiled_charsmap, &n);
  if (nhas(3)) PutBool(3, ns.add_dummy_prefix, &n);
  if (nhas(4)) PutBool(4, ns.remove_extra_whitespaces, &n);
  if (nhas(5)) PutBool(5, ns.escape_whitespaces, &n);
  if (nhas(6)) PutBytes(6, ns.normalization_rule_tsv, &n);
  PutBytes(3, n, &out);
  return out;
}

}  // namespace spm_amd
