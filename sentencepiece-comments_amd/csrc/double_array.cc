// Breadth-first double-array construction (see double_array.h).
#include "double_array.h"

#include <algorithm>
#include <cstddef>
#include <deque>
#include <mutex>

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
  // Stable order by bytes: sort indices by the key bytes, ties by index.
  std::vector<uint32_t> order(keys->size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = static_cast<uint32_t>(i);
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    const int r = (*keys)[a].first.compare((*keys)[b].first);
    return r < 0 || (r == 0 && a < b);
  });
  std::vector<std::pair<std::string, int32_t>> sorted;
  sorted.reserve(keys->size());
  for (uint32_t i : order) sorted.push_back(std::move((*keys)[i]));
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
  out->max_prefix_matches = 0;
  std::vector<std::pair<int32_t, size_t>> res;
  for (const auto &k : keys) {
    out->CommonPrefixSearch(k.first.data(), k.first.size(), &res);
    out->max_prefix_matches = std::max<int32_t>(out->max_prefix_matches, static_cast<int32_t>(res.size()));
  }
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

bool Place(const std::vector<std::pair<std::string, int32_t>> &keys, DoubleArray *out, std::string *err) {
  *out = DoubleArray();
  Placer placer(out);
  placer.MarkUsed(0);
  std::deque<Pending> queue;
  queue.push_back({0, keys.size(), 0, 0});
  std::vector<uint8_t> labels;
  std::vector<size_t> starts;
  while (!queue.empty()) {
    Pending nd = queue.front();
    queue.pop_front();
    size_t lo = nd.lo;
    if (lo < nd.hi && keys[lo].first.size() == nd.depth) {
      out->units[nd.slot] |= 1u << 8;
      out->values[nd.slot] = keys[lo].second;
      ++lo;
    }
    if (lo >= nd.hi) continue;
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
    const uint32_t base = placer.FindBase(labels, &ok);
    if (!ok) {
      if (err) *err = "double array too large";
      return false;
    }
    placer.Claim(base, labels);
    out->units[nd.slot] = (out->units[nd.slot] & 0x1FFu) | (base << 9);
    for (size_t j = 0; j < labels.size(); ++j) {
      const uint32_t slot = base ^ labels[j];
      out->units[slot] = labels[j];
      queue.push_back({starts[j], starts[j + 1], nd.depth + 1, slot});
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
