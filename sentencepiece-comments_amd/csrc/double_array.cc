// Breadth-first double-array construction (see double_array.h).
#include "double_array.h"

#include <algorithm>
#include <cstddef>
#include <deque>
#include <mutex>
#include <thread>

namespace spm_amd {

int32_t DoubleArray::ExactMatch(const char *key, size_t len) const {
  uint32_t node = 0;
  for (size_t i = 0; i < len; ++i) {
    const uint32_t c = static_cast<uint8_t>(key[i]);
    if (c == 0) return -1;
    const uint32_t next = Base(units[node]) ^ c;
    if (next >= units.size() || Label(units[next]) != c) return -1;
    node = next;
  }
  return (node != 0 && Leaf(units[node])) ? values[node] : -1;
}

void DoubleArray::CommonPrefixSearch(const char *key, size_t len,
                                     std::vector<std::pair<int32_t, size_t>> *out) const {
  out->clear();
  uint32_t node = 0;
  for (size_t i = 0; i < len; ++i) {
    const uint32_t c = static_cast<uint8_t>(key[i]);
    if (c == 0) return;
    const uint32_t next = Base(units[node]) ^ c;
    if (next >= units.size() || Label(units[next]) != c) return;
    node = next;
    if (Leaf(units[node])) out->emplace_back(values[node], i + 1);
  }
}

namespace {

struct Pending {
  size_t lo, hi;   // key range sharing the first `depth` bytes
  size_t depth;
  uint32_t slot;   // unit index of this node
};

// Slots are handed out per 256-unit block: a node's children are base ^ byte,
// which stays inside base's block, so placing a node means choosing one free
// (block, base byte) pair.  Only a bounded window of recently opened blocks is
// searched (darts-clone keeps a similar window of "extra" blocks); when none
// fits, a fresh block is appended.  Cost per node is bounded, so building is
// O(nodes) instead of a scan over every free slot.
class Placer {
 public:
  static constexpr size_t kWindow = 32;
  explicit Placer(DoubleArray *da) : da_(da) { NewBlock(); }

  uint32_t FindBase(const std::vector<uint8_t> &labels, bool *ok) {
    for (size_t w = 0; w < open_.size(); ++w) {
      const size_t blk = open_[w];
      Block &b = blocks_[blk];
      if (b.nfree < static_cast<int>(labels.size())) continue;
      // Bases lo of this block that are unowned and whose child slots
      // lo ^ c are all free, as one 256-bit set: ~base_used AND, for each
      // label c, the free-slot set permuted by XOR c.
      uint64_t cand[4];
      for (int q = 0; q < 4; ++q) cand[q] = ~b.base_used[q];
      for (uint8_t c : labels) {
        uint64_t fr[4];
        for (int q = 0; q < 4; ++q) fr[q] = ~b.used[q];
        XorPermute(fr, c);
        for (int q = 0; q < 4; ++q) cand[q] &= fr[q];
      }
      if (!(cand[0] | cand[1] | cand[2] | cand[3])) {
        // A block that keeps failing has free slots but no free base that
        // reaches them: leave the window (scanning it for every node was
        // most of the build time: 30 blocks per placement at 350 k keys).
        if (++b.fails >= kMaxFails) {
          open_.erase(open_.begin() + static_cast<std::ptrdiff_t>(w));
          --w;
        }
        continue;
      }
      for (int q = 0; q < 4; ++q) {
        if (!cand[q]) continue;
        const uint32_t lo = static_cast<uint32_t>(q * 64 + __builtin_ctzll(cand[q]));
        const uint32_t base = static_cast<uint32_t>(blk) * 256u + lo;
        if (base >= DoubleArray::kBaseLimit) {
          *ok = false;
          return 0;
        }
        *ok = true;
        return base;
      }
    }
    const size_t blk = NewBlock();
    const uint32_t base = static_cast<uint32_t>(blk) * 256u;
    *ok = base < DoubleArray::kBaseLimit;
    return base;
  }
  void Claim(uint32_t base, const std::vector<uint8_t> &labels) {
    Block &b = blocks_[base >> 8];
    Set(b.base_used, base & 0xFFu);
    for (uint8_t c : labels) {
      Set(b.used, (base & 0xFFu) ^ c);
      --b.nfree;
    }
    if (b.nfree == 0) open_.erase(std::find(open_.begin(), open_.end(), base >> 8));
  }
  void MarkUsed(uint32_t s) {
    Block &b = blocks_[s >> 8];
    if (!Test(b.used, s & 0xFFu)) {
      Set(b.used, s & 0xFFu);
      --b.nfree;
    }
  }

 private:
  struct Block {
    uint64_t used[4] = {0, 0, 0, 0};
    uint64_t base_used[4] = {0, 0, 0, 0};
    int nfree = 256;
    int fails = 0;
  };
  static constexpr int kMaxFails = 16;
  static bool Test(const uint64_t *m, uint32_t i) { return (m[i >> 6] >> (i & 63)) & 1u; }
  // m'[i] = m[i ^ c] over a 256-bit set: words swap by c's top two bits,
  // bits inside a word by swapping aligned groups of 1, 2, ..., 32.
  static void XorPermute(uint64_t *m, uint32_t c) {
    static constexpr uint64_t kLow[6] = {0x5555555555555555ull, 0x3333333333333333ull, 0x0F0F0F0F0F0F0F0Full,
                                         0x00FF00FF00FF00FFull, 0x0000FFFF0000FFFFull, 0x00000000FFFFFFFFull};
    const uint32_t wx = c >> 6;
    if (wx) {
      uint64_t t[4];
      for (uint32_t q = 0; q < 4; ++q) t[q] = m[q ^ wx];
      for (uint32_t q = 0; q < 4; ++q) m[q] = t[q];
    }
    for (int k = 0; k < 6; ++k)
      if ((c >> k) & 1u) {
        const int sh = 1 << k;
        for (int q = 0; q < 4; ++q) m[q] = ((m[q] & kLow[k]) << sh) | ((m[q] >> sh) & kLow[k]);
      }
  }
  static void Set(uint64_t *m, uint32_t i) { m[i >> 6] |= uint64_t(1) << (i & 63); }
  size_t NewBlock() {
    const size_t blk = blocks_.size();
    blocks_.emplace_back();
    // A childless node has base 0: keep base 0 unowned.
    if (blk == 0) Set(blocks_[0].base_used, 0);
    da_->units.resize((blk + 1) * 256, 0);
    da_->values.resize((blk + 1) * 256, -1);
    open_.push_back(blk);
    if (open_.size() > kWindow) open_.pop_front();
    return blk;
  }
  DoubleArray *da_;
  std::vector<Block> blocks_;
  std::deque<size_t> open_;
};

}  // namespace

namespace {

// Keys in build order: NUL-truncated, sorted by bytes, the first value of
// equal keys kept, empty keys dropped.
void Canonicalize(std::vector<std::pair<std::string, int32_t>> *keys) {
  for (auto &k : *keys) {
    const size_t z = k.first.find('\0');
    if (z != std::string::npos) k.first.resize(z);
  }
  // Stable order by bytes: sort indices by the key bytes, ties by index.  The
  // first 8 bytes ride along big-endian (zero padded; keys hold no NUL), so
  // most comparisons never touch the strings.
  struct Ord {
    uint64_t head;
    uint32_t len, idx;
  };
  std::vector<Ord> order(keys->size());
  for (size_t i = 0; i < order.size(); ++i) {
    const std::string &k = (*keys)[i].first;
    uint64_t h = 0;
    for (size_t q = 0; q < 8; ++q) h = h << 8 | (q < k.size() ? static_cast<uint8_t>(k[q]) : 0u);
    order[i] = {h, static_cast<uint32_t>(std::min<size_t>(k.size(), UINT32_MAX)), static_cast<uint32_t>(i)};
  }
  std::sort(order.begin(), order.end(), [&](const Ord &a, const Ord &b) {
    if (a.head != b.head) return a.head < b.head;
    if (a.len > 8 && b.len > 8) {
      const int r = (*keys)[a.idx].first.compare(8, std::string::npos, (*keys)[b.idx].first, 8, std::string::npos);
      if (r) return r < 0;
    } else if (a.len != b.len) {
      return a.len < b.len;
    }
    return a.idx < b.idx;
  });
  std::vector<std::pair<std::string, int32_t>> sorted;
  sorted.reserve(keys->size());
  for (const Ord &o : order) sorted.push_back(std::move((*keys)[o.idx]));
  sorted.erase(std::unique(sorted.begin(), sorted.end(),
                           [](const std::pair<std::string, int32_t> &a,
                              const std::pair<std::string, int32_t> &b) { return a.first == b.first; }),
               sorted.end());
  // An empty key cannot be matched (the reference rejects empty pieces).
  size_t e = 0;
  while (e < sorted.size() && sorted[e].first.empty()) ++e;
  sorted.erase(sorted.begin(), sorted.begin() + static_cast<std::ptrdiff_t>(e));
  *keys = std::move(sorted);
}

// The trainer builds the same piece set's trie several times per EM round
// (E-step sub-iterations, the pruning NBest and Viterbi models, each listing
// the pieces in its own order): the last builds are kept by canonical key
// list and an identical list gets a copy.
struct BuildCache {
  struct Entry {
    std::vector<std::pair<std::string, int32_t>> raw, canonical;  // a caller's list, its canonical form
    DoubleArray da;
  };
  std::mutex mu;
  std::deque<Entry> entries;  // newest first
  static constexpr size_t kEntries = 3;
};
BuildCache &Cache() {
  static BuildCache c;
  return c;
}

bool Place(const std::vector<std::pair<std::string, int32_t>> &keys, DoubleArray *out, std::string *err);

void SetMaxPrefixMatches(const std::vector<std::pair<std::string, int32_t>> &keys, DoubleArray *out) {
  // trie_results_size_: max number of keys prefixing any key
  // (unigram_model.cc:656-667).
  const size_t n = keys.size();
  const size_t T = n >= (1u << 15) ? std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency())) : 1;
  std::vector<int32_t> part(T, 0);
  auto run = [&](size_t t) {
    std::vector<std::pair<int32_t, size_t>> res;
    for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) {
      out->CommonPrefixSearch(keys[i].first.data(), keys[i].first.size(), &res);
      part[t] = std::max<int32_t>(part[t], static_cast<int32_t>(res.size()));
    }
  };
  std::vector<std::thread> th;
  for (size_t t = 1; t < T; ++t) th.emplace_back(run, t);
  run(0);
  for (auto &x : th) x.join();
  out->max_prefix_matches = *std::max_element(part.begin(), part.end());
}

}  // namespace

bool BuildDoubleArray(std::vector<std::pair<std::string, int32_t>> keys, DoubleArray *out,
                      std::string *err) {
  BuildCache &c = Cache();
  {
    // The same list as a cached one (no canonicalization needed).
    std::lock_guard<std::mutex> lock(c.mu);
    for (auto &e : c.entries)
      if (e.raw == keys) {
        *out = e.da;
        return true;
      }
  }
  std::vector<std::pair<std::string, int32_t>> raw = keys;
  Canonicalize(&keys);
  {
    std::lock_guard<std::mutex> lock(c.mu);
    for (auto &e : c.entries)
      if (e.canonical == keys) {
        *out = e.da;
        e.raw = std::move(raw);  // (this caller's order next time)
        return true;
      }
  }
  if (!Place(keys, out, err)) return false;
  std::lock_guard<std::mutex> lock(c.mu);
  c.entries.push_front(BuildCache::Entry{std::move(raw), std::move(keys), *out});
  if (c.entries.size() > BuildCache::kEntries) c.entries.pop_back();
  return true;
}

namespace {

using Keys = std::vector<std::pair<std::string, int32_t>>;

struct Task {
  size_t lo, hi, depth;  // children still to place (the node's own leaf is set)
  uint32_t slot;         // the node's unit in the shared top array
  uint32_t base = 0;     // its children's base in the task group's own array
};

// Breadth-first placement from `queue` into `da`.  A pending node with
// task >= 0 is a task root living in another array: its base goes to
// tasks[task].base.  With split > 0, a node whose remaining key range is at
// most `split` keys is not expanded but appended to *tasks.
bool Expand(const Keys &keys, std::deque<Pending> *queue, std::vector<int32_t> *task_of, Placer *placer,
            DoubleArray *da, size_t split, std::vector<Task> *tasks, std::string *err) {
  std::vector<uint8_t> labels;
  std::vector<size_t> starts;
  size_t popped = 0;
  while (!queue->empty()) {
    Pending nd = queue->front();
    queue->pop_front();
    const int32_t task = task_of ? (*task_of)[popped] : -1;
    ++popped;
    size_t lo = nd.lo;
    if (task < 0 && lo < nd.hi && keys[lo].first.size() == nd.depth) {
      da->units[nd.slot] |= 1u << 8;
      da->values[nd.slot] = keys[lo].second;
      ++lo;
    }
    if (lo >= nd.hi) continue;
    if (split && nd.depth > 0 && nd.hi - lo <= split) {
      tasks->push_back({lo, nd.hi, nd.depth, nd.slot});
      continue;
    }
    labels.clear();
    starts.clear();
    for (size_t i = lo; i < nd.hi; ++i) {
      const uint8_t c = static_cast<uint8_t>(keys[i].first[nd.depth]);
      if (labels.empty() || labels.back() != c) {
        labels.push_back(c);
        starts.push_back(i);
      }
    }
    starts.push_back(nd.hi);
    bool ok = false;
    const uint32_t base = placer->FindBase(labels, &ok);
    if (!ok) {
      if (err) *err = "double array too large";
      return false;
    }
    placer->Claim(base, labels);
    if (task >= 0)
      (*tasks)[static_cast<size_t>(task)].base = base;
    else
      da->units[nd.slot] = (da->units[nd.slot] & 0x1FFu) | (base << 9);
    for (size_t j = 0; j < labels.size(); ++j) {
      const uint32_t slot = base ^ labels[j];
      da->units[slot] = labels[j];
      queue->push_back({starts[j], starts[j + 1], nd.depth + 1, slot});
      if (task_of) task_of->push_back(-1);
    }
  }
  return true;
}

// The top of the trie (nodes over more than `split` keys) is placed in one
// array; the subtrees below it are placed by several threads, each into an
// array of its own over a contiguous run of subtrees, and the arrays are
// appended with their bases shifted by whole blocks.  A base stays inside
// its block under XOR, so shifting by blocks keeps every child slot valid.
bool Place(const Keys &keys, DoubleArray *out, std::string *err) {
  *out = DoubleArray();
  const size_t n = keys.size();
  const size_t groups = n >= (1u << 15) ? std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency())) : 1;
  const size_t split = groups > 1 ? n / (groups * 16) : 0;
  std::vector<Task> tasks;
  {
    Placer placer(out);
    placer.MarkUsed(0);
    std::deque<Pending> queue;
    queue.push_back({0, n, 0, 0});
    if (!Expand(keys, &queue, nullptr, &placer, out, split, &tasks, err)) return false;
  }
  if (!tasks.empty()) {
    // Contiguous runs in key order with about the same key count each.
    std::sort(tasks.begin(), tasks.end(), [](const Task &a, const Task &b) { return a.lo < b.lo; });
    size_t total = 0;
    for (const Task &t : tasks) total += t.hi - t.lo;
    std::vector<size_t> cut(groups + 1, tasks.size());
    cut[0] = 0;
    {
      size_t g = 1, acc = 0;
      for (size_t i = 0; i < tasks.size() && g < groups; ++i) {
        acc += tasks[i].hi - tasks[i].lo;
        if (acc * groups >= total * g) cut[g++] = i + 1;
      }
    }
    std::vector<DoubleArray> part(groups);
    std::vector<std::string> perr(groups);
    std::vector<char> pok(groups, 1);
    std::vector<std::thread> th;
    for (size_t g = 0; g < groups; ++g) {
      if (cut[g] >= cut[g + 1]) continue;
      th.emplace_back([&, g] {
        Placer placer(&part[g]);
        std::deque<Pending> queue;
        std::vector<int32_t> task_of;
        for (size_t i = cut[g]; i < cut[g + 1]; ++i) {
          queue.push_back({tasks[i].lo, tasks[i].hi, tasks[i].depth, 0});
          task_of.push_back(static_cast<int32_t>(i));
        }
        pok[g] = Expand(keys, &queue, &task_of, &placer, &part[g], 0, &tasks, &perr[g]);
      });
    }
    for (auto &t : th) t.join();
    for (size_t g = 0; g < groups; ++g)
      if (!pok[g]) {
        if (err) *err = perr[g];
        return false;
      }
    // Append each group's array; its nonzero bases (local base 0 is never
    // handed out) shift by the group's first unit.
    for (size_t g = 0; g < groups; ++g) {
      if (cut[g] >= cut[g + 1]) continue;
      const uint64_t off = out->units.size();
      if ((off + part[g].units.size()) >> 8 > (DoubleArray::kBaseLimit >> 8)) {
        if (err) *err = "double array too large";
        return false;
      }
      const uint32_t shift = static_cast<uint32_t>(off);
      out->units.resize(off + part[g].units.size());
      out->values.insert(out->values.end(), part[g].values.begin(), part[g].values.end());
      for (size_t u = 0; u < part[g].units.size(); ++u) {
        const uint32_t v = part[g].units[u];
        out->units[off + u] = DoubleArray::Base(v) ? (v & 0x1FFu) | ((DoubleArray::Base(v) + shift) << 9) : v;
      }
      for (size_t i = cut[g]; i < cut[g + 1]; ++i) {
        const uint32_t nb = tasks[i].base + shift;
        if (nb >= DoubleArray::kBaseLimit) {
          if (err) *err = "double array too large";
          return false;
        }
        out->units[tasks[i].slot] = (out->units[tasks[i].slot] & 0x1FFu) | (nb << 9);
      }
      part[g] = DoubleArray();
    }
  }
  // Trim trailing free units (keep every slot a walk can address: base|0xFF).
  size_t last = 0;
  for (size_t i = 0; i < out->units.size(); ++i)
    if (out->units[i] != 0) last = std::max<size_t>(last, std::max<size_t>(i, (DoubleArray::Base(out->units[i]) | 0xFFu)));
  out->units.resize(last + 1);
  out->values.resize(last + 1);
  SetMaxPrefixMatches(keys, out);
  return true;
}

}  // namespace

}  // namespace spm_amd
