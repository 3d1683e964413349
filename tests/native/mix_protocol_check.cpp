// tests/native/mix_protocol_check.cpp -- the tile mix protocol of renderKernel's completeItem
// (opengl_ray_tracing_amd/csrc/pt_kernels.hip), restated over std::atomic with the same
// sequentially consistent operations, run by many threads on randomly split and shuffled
// work items of frames in flight. Each frame's items write a tile's sample values, the
// completer of a tile tries the tile's lock for its frame, and a mixer hands on to the next
// frame that already completed the tile. The running mean must come out bit for bit as if
// the frames had been mixed one after another, every frame must be mixed exactly once, and
// no thread ever waits. Built and run by tests/test_mix_protocol.py; prints "ok <mixes>
// <handoffs>" or the first mismatch.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

namespace {

constexpr int D = 8;        // frames in flight (slots)
constexpr int D1 = D + 1;   // colour buffers / completion-count rows
constexpr int TILES = 257;  // tiles (some with no pixels)
constexpr int FRAMES = 400;
constexpr int THREADS = 8;

struct State {
  std::vector<std::atomic<int>> done;        // D1 x TILES: pixels of the tile frame g has written
  std::vector<std::atomic<unsigned>> lock;   // TILES: 2 x next frame to mix (+1 while held)
  std::vector<float> accum;                  // TILES x 8: the running mean (pixels 0..need-1)
  std::vector<float> col;                    // D1 x TILES x 8: sample values of frame g
  std::vector<int> mixed;                    // FRAMES x TILES: times frame g was mixed into tile t
  std::atomic<long> handoffs{0};             // mixes done by a wave of another frame
  State() : done(D1 * TILES), lock(TILES), accum(TILES * 8, 0.0f), col(D1 * TILES * 8), mixed(FRAMES * TILES, 0) {
    for (auto& d : done) d.store(0);
    for (auto& l : lock) l.store(0);
  }
};

float mixf(float a, float b, float w) { return a * (1.0f - w) + b * w; }

// completeItem: frame seq's item of tile t wrote n of the tile's need pixels
void completeItem(State& s, unsigned seq, int t, int n, int need) {
  if (need == 0) return;
  const int done = s.done[(seq % D1) * TILES + t].fetch_add(n, std::memory_order_seq_cst) + n;
  if (done != need) return;
  unsigned g = seq;
  for (unsigned k = 0; k <= (unsigned)D; k++) {
    unsigned old = 2u * g;
    s.lock[t].compare_exchange_strong(old, 2u * g + 1u, std::memory_order_seq_cst);
    if (old != 2u * g) return;
    if (g != seq) s.handoffs.fetch_add(1);
    const float w = 1.0f / (float)(g + 1u);
    for (int i = 0; i < need; i++)
      s.accum[t * 8 + i] = mixf(s.accum[t * 8 + i], s.col[((g % D1) * TILES + t) * 8 + i], w);
    s.mixed[g * TILES + t]++;
    s.done[(g % D1) * TILES + t].store(0, std::memory_order_relaxed);
    s.lock[t].store(2u * (g + 1u), std::memory_order_seq_cst);
    const int next = s.done[((g + 1u) % D1) * TILES + t].load(std::memory_order_seq_cst);
    if (next != need) return;
    g++;
  }
}

}  // namespace

int main() {
  State s;
  std::mt19937 rng(12345);
  std::vector<int> need(TILES);
  for (int t = 0; t < TILES; t++) need[t] = (t % 37 == 5) ? 0 : 1 + (int)(rng() % 8);
  std::vector<float> ref(TILES * 8, 0.0f);
  std::vector<std::vector<float>> values(FRAMES, std::vector<float>(TILES * 8));
  for (auto& v : values)
    for (auto& x : v) x = std::uniform_real_distribution<float>(0.0f, 4.0f)(rng);
  // frames go in windows of D1 in flight at once (frame g + D1 starts after frame g is mixed,
  // as pt_runtime.cpp orders colour-buffer reuse)
  struct Item {
    unsigned g;
    int t, n, lo;
  };
  for (int w0 = 0; w0 < FRAMES; w0 += D1) {
    const int w1 = std::min(FRAMES, w0 + D1);
    std::vector<Item> items;
    for (int g = w0; g < w1; g++) {
      for (int t = 0; t < TILES; t++) {
        int left = need[t], lo = 0;
        do {  // the tile split into items of random sizes (adaptive tile splitting), or one empty item
          const int n = left <= 1 ? left : 1 + (int)(rng() % left);
          items.push_back({(unsigned)g, t, n, lo});
          lo += n;
          left -= n;
        } while (left > 0);
      }
    }
    std::shuffle(items.begin(), items.end(), rng);
    std::atomic<size_t> next{0};
    auto worker = [&](int id) {
      std::mt19937 r(id * 7919 + w0);
      for (size_t i; (i = next.fetch_add(1)) < items.size();) {
        const Item& it = items[i];
        for (int k = 0; k < it.n; k++)  // the item's pixels' sample values (accumulate's colour stores)
          s.col[((it.g % D1) * TILES + it.t) * 8 + it.lo + k] = values[it.g][it.t * 8 + it.lo + k];
        if (r() % 4 == 0) std::this_thread::yield();
        completeItem(s, it.g, it.t, it.n, need[it.t]);
      }
    };
    std::vector<std::thread> th;
    for (int k = 0; k < THREADS; k++) th.emplace_back(worker, k);
    for (auto& x : th) x.join();
    for (int g = w0; g < w1; g++)
      for (int t = 0; t < TILES; t++)
        for (int i = 0; i < need[t]; i++) ref[t * 8 + i] = mixf(ref[t * 8 + i], values[g][t * 8 + i], 1.0f / (float)(g + 1));
  }
  long mixes = 0;
  for (int g = 0; g < FRAMES; g++)
    for (int t = 0; t < TILES; t++) {
      const int want = need[t] ? 1 : 0;
      if (s.mixed[g * TILES + t] != want) {
        std::printf("frame %d tile %d mixed %d times\n", g, t, s.mixed[g * TILES + t]);
        return 1;
      }
      mixes += want;
    }
  for (int i = 0; i < TILES * 8; i++)
    if (s.accum[i] != ref[i]) {
      std::printf("tile %d pixel %d: %.9g != %.9g\n", i / 8, i % 8, s.accum[i], ref[i]);
      return 1;
    }
  std::printf("ok %ld %ld\n", mixes, s.handoffs.load());
  return 0;
}
