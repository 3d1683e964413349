// tests/native/introsort_check.cpp -- pt::exactSort (opengl_ray_tracing_amd/csrc/pt_introsort.h)
// against this toolchain's std::sort, and its heapsort against std::partial_sort, on
// tie-heavy (key, id) records: the permutations must be identical. Built and run by
// tests/test_introsort.py; prints "ok <cases>" or the first mismatch.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <random>
#include <vector>

static std::atomic<int> g_heapsorts{0};  // introsort's depth-limit fallbacks taken
#define PT_INTROSORT_HEAPSORT_HOOK g_heapsorts.fetch_add(1)
#include "pt_introsort.h"

struct KeyId {
  float k;
  int id;
};
struct Less {
  bool operator()(const KeyId& a, const KeyId& b) const { return a.k < b.k; }
};

static std::vector<KeyId> make(int n, int distinct, int shape, std::mt19937& g) {
  std::vector<KeyId> v(n);
  std::uniform_int_distribution<int> d(0, distinct - 1);
  for (int i = 0; i < n; i++) {
    int k = d(g);
    if (shape == 1) k = i / std::max(1, n / distinct);                  // sorted with runs of ties
    if (shape == 2) k = (n - i) / std::max(1, n / distinct);            // reversed
    if (shape == 3) k = std::min(i, n - 1 - i) % distinct;              // organ pipe
    v[i] = KeyId{(float)k * 0.25f, i};
  }
  return v;
}

static bool same(const std::vector<KeyId>& a, const std::vector<KeyId>& b) {
  for (size_t i = 0; i < a.size(); i++)
    if (a[i].id != b[i].id) return false;
  return true;
}

// McIlroy's adversary ("A Killer Adversary for Quicksort", 1999): keys fixed lazily so
// that every partition is as bad as possible -- an input that drives introsort past its
// depth limit into the heapsort fallback.
static std::vector<KeyId> killer(int n) {
  std::vector<int> val(n, n), idx(n);
  int nsolid = 0, candidate = 0;
  for (int i = 0; i < n; i++) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](int x, int y) {
    if (val[x] == n && val[y] == n) val[x == candidate ? x : y] = nsolid++;
    if (val[x] == n) candidate = x;
    else if (val[y] == n) candidate = y;
    return val[x] < val[y];
  });
  std::vector<KeyId> v(n);
  for (int i = 0; i < n; i++) v[i] = KeyId{(float)val[i], i};
  return v;
}

int main() {
  std::mt19937 g(12345);
  pt::Helpers helpers(7);
  int cases = 0;
  const int sizes[] = {0, 1, 2, 3, 15, 16, 17, 33, 100, 1000, 4097, 70000, 300000, 1 << 20};
  for (int n : sizes)
    for (int distinct : {1, 2, 7, 100, 1 << 30})
      for (int shape = 0; shape < 4; shape++) {
        std::vector<KeyId> a = make(n, distinct, shape, g), b = a, c = a, h1 = a, h2 = a;
        std::sort(a.begin(), a.end(), Less{});
        pt::exactSort(b.data(), b.data() + n, Less{}, nullptr);
        pt::exactSort(c.data(), c.data() + n, Less{}, &helpers);
        if (!same(a, b) || !same(a, c)) {
          std::printf("sort mismatch n=%d distinct=%d shape=%d serial=%d parallel=%d\n", n, distinct, shape,
                      (int)same(a, b), (int)same(a, c));
          return 1;
        }
        if (n <= 70000) {
          std::partial_sort(h1.begin(), h1.end(), h1.end(), Less{});
          pt::introsort::heapSort(h2.data(), h2.data() + n, Less{});
          if (!same(h1, h2)) {
            std::printf("heapsort mismatch n=%d distinct=%d shape=%d\n", n, distinct, shape);
            return 1;
          }
        }
        cases++;
      }
  for (int n : {1000, 4096, 100000, 1 << 20}) {
    std::vector<KeyId> a = killer(n), b = a, c = a;
    const int before = g_heapsorts.load();
    std::sort(a.begin(), a.end(), Less{});
    pt::exactSort(b.data(), b.data() + n, Less{}, nullptr);
    pt::exactSort(c.data(), c.data() + n, Less{}, &helpers);
    if (!same(a, b) || !same(a, c) || g_heapsorts.load() == before) {
      std::printf("killer mismatch n=%d serial=%d parallel=%d heapsorts=%d\n", n, (int)same(a, b), (int)same(a, c),
                  g_heapsorts.load() - before);
      return 1;
    }
    cases++;
  }
  std::printf("ok %d heapsort_fallbacks %d\n", cases, g_heapsorts.load());
  return 0;
}
