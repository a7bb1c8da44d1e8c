"""The BPE trainer's symbol-cache relayout (csrc/trainer.cc TrainBpe): a
std::unordered_map copied with the allocator-extended copy constructor into
a fresh node arena must keep the iteration order, bucket count and rehash
state, so that every later insert / erase / walk matches the original map's
(the reference's partial_sort reads the map's iteration order,
bpe_model_trainer.cc:153-183).  Checked on the toolchain's libstdc++ with the
trainer's kind of arena allocator, over random insert / erase / rehash
sequences with a copy every few hundred operations (CPU only)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include <cstdio>
#include <memory>
#include <random>
#include <unordered_map>
#include <vector>
struct Arena {
  std::vector<std::unique_ptr<char[]>> blocks;
  size_t used = 0, cap = 0;
  void *Get(size_t bytes, size_t align) {
    used = (used + align - 1) & ~(align - 1);
    if (blocks.empty() || used + bytes > cap) { cap = bytes > (1u << 16) ? bytes : (1u << 16); blocks.emplace_back(new char[cap]); used = 0; }
    void *p = blocks.back().get() + used; used += bytes; return p;
  }
};
template <class T> struct AA {
  using value_type = T;
  Arena *a;
  explicit AA(Arena *x) : a(x) {}
  template <class U> AA(const AA<U> &o) : a(o.a) {}
  T *allocate(size_t n) { return n != 1 ? std::allocator<T>().allocate(n) : static_cast<T *>(a->Get(sizeof(T), alignof(T))); }
  void deallocate(T *p, size_t n) { if (n != 1) std::allocator<T>().deallocate(p, n); }
  template <class U> bool operator==(const AA<U> &o) const { return a == o.a; }
  template <class U> bool operator!=(const AA<U> &o) const { return a != o.a; }
};
using Map = std::unordered_map<unsigned long, unsigned, std::hash<unsigned long>, std::equal_to<unsigned long>,
                               AA<std::pair<const unsigned long, unsigned>>>;
static bool same(const Map &x, const Map &y) {
  if (x.size() != y.size() || x.bucket_count() != y.bucket_count()) return false;
  auto i = x.begin();
  for (auto j = y.begin(); j != y.end(); ++i, ++j) if (i->first != j->first || i->second != j->second) return false;
  return true;
}
int main() {
  std::mt19937_64 rng(7);
  for (int t = 0; t < 40; ++t) {
    Arena a0, a1, ref_arena;
    Map ref{AA<std::pair<const unsigned long, unsigned>>(&ref_arena)};
    std::unique_ptr<Map> cur(new Map(AA<std::pair<const unsigned long, unsigned>>(&a0)));
    int k = 0;
    std::vector<unsigned long> keys;
    for (int op = 0; op < 60000; ++op) {
      const unsigned r = rng() % 100;
      if (r < 60 || keys.empty()) {
        const unsigned long key = rng() % (t % 2 ? 5000 : 1000000);
        ref.emplace(key, op); cur->emplace(key, op); keys.push_back(key);
      } else {
        const unsigned long key = keys[rng() % keys.size()];
        ref.erase(key); cur->erase(key);
      }
      if (op % 397 == 0) {  // relayout into the other arena
        Arena &next = k ? a0 : a1;
        next = Arena();
        std::unique_ptr<Map> fresh(new Map(*cur, AA<std::pair<const unsigned long, unsigned>>(&next)));
        if (!same(*fresh, *cur)) { std::printf("COPY ORDER t=%d op=%d\n", t, op); return 1; }
        cur = std::move(fresh);
        k ^= 1;
      }
      if (op % 1000 == 999 && !same(ref, *cur)) { std::printf("DIVERGED t=%d op=%d\n", t, op); return 1; }
    }
    if (!same(ref, *cur)) { std::printf("DIVERGED t=%d end\n", t); return 1; }
  }
  std::printf("ok\n");
  return 0;
}
"""


def test_cache_relayout_keeps_iteration_order(tmp_path):
    src = tmp_path / "relayout.cc"
    src.write_text(SRC)
    exe = tmp_path / "relayout"
    subprocess.run(["g++", "-O2", "-std=c++17", str(src), "-o", str(exe)], check=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, timeout=300)
    assert out.returncode == 0 and out.stdout.decode().strip() == "ok", out.stdout.decode()
