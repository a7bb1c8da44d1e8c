// Heap selection with the exact element moves of libstdc++'s partial_sort
// heap phase (bits/stl_heap.h + bits/stl_algo.h `__heap_select`, unchanged
// from GCC 4.x through GCC 14; the image's g++ 11 is what the reference build
// would use).  The BPE trainer's UpdateActiveSymbols (bpe_model_trainer.cc:
// 153-183) keeps the first `size` symbols of std::partial_sort over the symbol
// cache's iteration order; which of several equal-freq symbols survive depends
// on the heap's moves, so the kept SET must be produced by the same moves.
// Only the comparison outcomes drive the moves, so any element type works.
//
// Restated algorithm (no library internals are called):
//   make_heap(first, middle): sift down every parent from (len-2)/2 to 0;
//   for i in [middle, last): if comp(*i, *first): pop the top into *i and
//     sift *i's old value into the heap from the root (adjust + push).
// tests/test_heap_select_cpu.py checks the result against the toolchain's
// own std::__heap_select on random inputs with heavy ties.
#pragma once

#include <cstddef>
#include <utility>

namespace spm_amd {

// __push_heap: move `value` up from `hole` while its parent compares below it.
template <typename It, typename T, typename Cmp>
inline void HeapPushUp(It first, std::ptrdiff_t hole, std::ptrdiff_t top, T value, Cmp &comp) {
  std::ptrdiff_t parent = (hole - 1) / 2;
  while (hole > top && comp(first[parent], value)) {
    first[hole] = std::move(first[parent]);
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = std::move(value);
}

// __adjust_heap: walk the hole down to a leaf along the larger child, then
// push `value` back up from there.
template <typename It, typename T, typename Cmp>
inline void HeapAdjust(It first, std::ptrdiff_t hole, std::ptrdiff_t len, T value, Cmp &comp) {
  const std::ptrdiff_t top = hole;
  std::ptrdiff_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (comp(first[child], first[child - 1])) --child;
    first[hole] = std::move(first[child]);
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    first[hole] = std::move(first[child - 1]);
    hole = child - 1;
  }
  HeapPushUp(first, hole, top, std::move(value), comp);
}

template <typename It, typename Cmp>
inline void HeapMake(It first, It last, Cmp &comp) {
  const std::ptrdiff_t len = last - first;
  if (len < 2) return;
  for (std::ptrdiff_t parent = (len - 2) / 2;; --parent) {
    auto value = std::move(first[parent]);
    HeapAdjust(first, parent, len, std::move(value), comp);
    if (parent == 0) return;
  }
}

// [first, middle) ends up holding the heap of the selected elements.
template <typename It, typename Cmp>
inline void HeapSelect(It first, It middle, It last, Cmp comp) {
  HeapMake(first, middle, comp);
  const std::ptrdiff_t len = middle - first;
  for (It i = middle; i < last; ++i)
    if (comp(*i, *first)) {  // __pop_heap(first, middle, i)
      auto value = std::move(*i);
      *i = std::move(*first);
      HeapAdjust(first, std::ptrdiff_t(0), len, std::move(value), comp);
    }
}

}  // namespace spm_amd
