// Breadth-first double-array construction (see double_array.h).
#include "double_array.h"

#include <algorithm>
#include <deque>

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

class Placer {
 public:
  explicit Placer(DoubleArray *da) : da_(da) {
    Grow(1024);
    base_used_[0] = 1;  // a childless node has base 0: keep it unowned
  }

  uint32_t FindBase(const std::vector<uint8_t> &labels, bool *ok) {
    // Scan free slots; try to put labels[0] there.
    for (size_t f = first_free_;; ++f) {
      if (f >= used_.size()) Grow(used_.size() * 2);
      if (used_[f]) {
        if (f == first_free_) ++first_free_;
        continue;
      }
      const uint32_t base = static_cast<uint32_t>(f) ^ labels[0];
      if (base >= DoubleArray::kBaseLimit) {
        *ok = false;
        return 0;
      }
      if ((base | 0xFFu) >= used_.size()) Grow(std::max<size_t>(used_.size() * 2, (base | 0xFFu) + 1));
      if (base_used_[base]) continue;
      bool fits = true;
      for (uint8_t c : labels) {
        const uint32_t s = base ^ c;
        if (s == 0 || used_[s]) {
          fits = false;
          break;
        }
      }
      if (fits) {
        *ok = true;
        return base;
      }
    }
  }
  void Claim(uint32_t base, const std::vector<uint8_t> &labels) {
    base_used_[base] = 1;
    for (uint8_t c : labels) used_[base ^ c] = 1;
  }
  void MarkUsed(uint32_t s) { used_[s] = 1; }

 private:
  void Grow(size_t n) {
    used_.resize(n, 0);
    base_used_.resize(n, 0);
    da_->units.resize(n, 0);
    da_->values.resize(n, -1);
  }
  DoubleArray *da_;
  std::vector<uint8_t> used_, base_used_;
  size_t first_free_ = 1;
};

}  // namespace

bool BuildDoubleArray(std::vector<std::pair<std::string, int32_t>> keys, DoubleArray *out,
                      std::string *err) {
  for (auto &k : keys) {
    const size_t z = k.first.find('\0');
    if (z != std::string::npos) k.first.resize(z);
  }
  std::stable_sort(keys.begin(), keys.end(),
                   [](const std::pair<std::string, int32_t> &a,
                      const std::pair<std::string, int32_t> &b) { return a.first < b.first; });
  keys.erase(std::unique(keys.begin(), keys.end(),
                         [](const std::pair<std::string, int32_t> &a,
                            const std::pair<std::string, int32_t> &b) { return a.first == b.first; }),
             keys.end());
  // An empty key cannot be matched (the reference rejects empty pieces).
  while (!keys.empty() && keys.front().first.empty()) keys.erase(keys.begin());

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
  // trie_results_size_: max number of keys prefixing any key
  // (unigram_model.cc:656-667).
  std::vector<std::pair<int32_t, size_t>> res;
  for (const auto &k : keys) {
    out->CommonPrefixSearch(k.first.data(), k.first.size(), &res);
    out->max_prefix_matches = std::max<int32_t>(out->max_prefix_matches, static_cast<int32_t>(res.size()));
  }
  return true;
}

}  // namespace spm_amd
