// pt_introsort.h -- internal: std::sort's result, computed in parallel.
//
// The reference builds its trees with std::sort (OpenglRayTracing/main.cpp:412-418,
// 467-469, 538-544) over records whose keys tie, and std::sort is not stable: which of two
// tied records comes first is whatever libstdc++'s introsort leaves, so a tree equal
// to the reference's needs that exact permutation. This header restates the
// algorithm of the libstdc++ the reference is built with here (GCC 11: median-of-three
// pivot moved to the front, Hoare partition, depth limit 2*floor(log2 n), heapsort
// below it, 16-element threshold, one final insertion sort) and makes the same
// comparisons on the same elements in the same order within each sub-range. The two
// sides of a partition never exchange elements again, so they are sorted on separate
// threads, and the final insertion sort moves an element only within its own
// partition block, so running it once over the whole range after the parallel phase
// gives std::sort's permutation exactly (tests/test_introsort.py checks it against
// std::sort on tie-heavy inputs).
#pragma once
#include <atomic>
#include <cstddef>
#include <thread>
#include <utility>
#include <vector>

namespace pt {

// A budget of helper threads shared by everything one build runs in parallel.
class Helpers {
 public:
  explicit Helpers(int spare) : spare_(spare) {}
  bool take() {
    int s = spare_.load(std::memory_order_relaxed);
    while (s > 0)
      if (spare_.compare_exchange_weak(s, s - 1)) return true;
    return false;
  }
  void give() { spare_.fetch_add(1); }

 private:
  std::atomic<int> spare_;
};

namespace introsort {

constexpr std::ptrdiff_t kThreshold = 16;    // _S_threshold
constexpr std::ptrdiff_t kParMin = 1 << 15;  // a partition side worth a thread

template <class T, class Less>
inline void medianToFirst(T* result, T* a, T* b, T* c, const Less& lt) {
  if (lt(*a, *b)) {
    if (lt(*b, *c)) std::swap(*result, *b);
    else if (lt(*a, *c)) std::swap(*result, *c);
    else std::swap(*result, *a);
  } else if (lt(*a, *c)) {
    std::swap(*result, *a);
  } else if (lt(*b, *c)) {
    std::swap(*result, *c);
  } else {
    std::swap(*result, *b);
  }
}

template <class T, class Less>
inline T* partitionPivot(T* first, T* last, const Less& lt) {
  T* mid = first + (last - first) / 2;
  medianToFirst(first, first + 1, mid, last - 1, lt);
  T* lo = first + 1;
  T* hi = last;
  const T& pivot = *first;
  while (true) {
    while (lt(*lo, pivot)) ++lo;
    --hi;
    while (lt(pivot, *hi)) --hi;
    if (!(lo < hi)) return lo;
    std::swap(*lo, *hi);
    ++lo;
  }
}

// heap primitives (the sift-down-to-leaf then sift-up form)
template <class T, class Less>
inline void adjustHeap(T* first, std::ptrdiff_t hole, std::ptrdiff_t len, T value, const Less& lt) {
  const std::ptrdiff_t top = hole;
  std::ptrdiff_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (lt(first[child], first[child - 1])) child--;
    first[hole] = first[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    first[hole] = first[child - 1];
    hole = child - 1;
  }
  std::ptrdiff_t parent = (hole - 1) / 2;
  while (hole > top && lt(first[parent], value)) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}

template <class T, class Less>
void heapSort(T* first, T* last, const Less& lt) {  // partial_sort(first, last, last)
  const std::ptrdiff_t len = last - first;
  if (len >= 2)
    for (std::ptrdiff_t parent = (len - 2) / 2;; parent--) {
      adjustHeap(first, parent, len, first[parent], lt);
      if (parent == 0) break;
    }
  while (last - first > 1) {
    --last;
    T v = *last;
    *last = *first;
    adjustHeap(first, std::ptrdiff_t(0), last - first, v, lt);
  }
}

template <class T, class Less>
void loop(T* first, T* last, int depth, const Less& lt, Helpers* h) {
  std::vector<std::thread> spawned;
  while (last - first > kThreshold) {
    if (depth == 0) {
#ifdef PT_INTROSORT_HEAPSORT_HOOK
      PT_INTROSORT_HEAPSORT_HOOK;
#endif
      heapSort(first, last, lt);
      break;
    }
    --depth;
    T* cut = partitionPivot(first, last, lt);
    if (h && last - cut >= kParMin && cut - first >= kParMin && h->take()) {
      spawned.emplace_back([=] {
        loop(cut, last, depth, lt, h);
        h->give();
      });
    } else {
      loop(cut, last, depth, lt, h);
    }
    last = cut;
  }
  for (auto& t : spawned) t.join();
}

template <class T, class Less>
void insertion(T* first, T* last, const Less& lt) {
  if (first == last) return;
  for (T* i = first + 1; i != last; ++i) {
    T v = *i;
    if (lt(v, *first)) {
      for (T* k = i; k != first; --k) *k = *(k - 1);
      *first = v;
    } else {
      T* k = i;
      while (lt(v, *(k - 1))) {
        *k = *(k - 1);
        --k;
      }
      *k = v;
    }
  }
}

template <class T, class Less>
void unguardedInsertion(T* first, T* last, const Less& lt) {
  for (T* i = first; i != last; ++i) {
    T v = *i;
    T* k = i;
    while (lt(v, *(k - 1))) {
      *k = *(k - 1);
      --k;
    }
    *k = v;
  }
}

inline int lg(std::ptrdiff_t n) {
  int r = 0;
  while (n > 1) {
    n >>= 1;
    r++;
  }
  return r;
}

}  // namespace introsort

// std::sort(first, last, lt)'s permutation; helper threads from h (may be null).
template <class T, class Less>
void exactSort(T* first, T* last, const Less& lt, Helpers* h) {
  if (first == last) return;
  introsort::loop(first, last, 2 * introsort::lg(last - first), lt, h);
  if (last - first > introsort::kThreshold) {
    introsort::insertion(first, first + introsort::kThreshold, lt);
    introsort::unguardedInsertion(first + introsort::kThreshold, last, lt);
  } else {
    introsort::insertion(first, last, lt);
  }
}

}  // namespace pt
