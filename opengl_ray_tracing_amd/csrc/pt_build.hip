// pt_build.hip -- the runtime's own tree built on the GPU (SURVEY.md 8(f)1:
// scene-prep acceleration; the host build it replaces is scene.cpp's threaded
// binned SAH, pt::buildAccel). A top-down binned-SAH builder, one tree level
// per step, every step a handful of kernels over the current frontier (the
// nodes still to split):
//
//   large nodes (> CHUNK triangles), many blocks each:
//     binLargeKernel     one block per CHUNK positions of a node: 3 axes x 32
//                        bins (count + triangle box) in LDS, merged into the
//                        node's global bins with ordered-uint atomics
//     splitLargeKernel   one wave per node: SAH sweep over the bins
//     partCountKernel    per chunk: left count + both children's boxes
//     (hipcub scan of the chunk left counts)
//     partScatterKernel  per chunk: stable partition into a scratch order
//     largeChildrenKernel, copyBackKernel
//   small nodes (<= CHUNK triangles): smallSplitKernel, one block per node
//     does all of the above in LDS and writes the children itself
//   nextFrontKernel      (hipcub scan of "child still to split") -> next frontier
//
// Nodes are numbered breadth-first as they are made (the root 0, a level's
// children after its parents), so the first internal nodes in id order are
// exactly the top of the tree the megakernel stages in LDS (pt_kernels.hip).
// encodeKernel then writes the wide records (pt_trace.h visitNodeF: both
// children's boxes, widened outward as pt_runtime.cpp encodeWideTree widens
// the host-built tree) and pairsKernel the leaf-order pair records.
//
// The SAH is scene.cpp splitBinned's: 32 bins per axis over the node's
// centroid bounds, cost = area(left) * n_left + area(right) * n_right, the
// first minimum in (axis, bin) order; a node whose centroids coincide is split
// at its median position. (splitBinned starts its search at the reference's
// INF = 2^31 and so falls back to the median on very large scenes; this search
// starts at +inf.) The tree is deterministic: every scatter position comes
// from scans, never from atomics' order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>
#include <cstring>

#include "pt_kernels.h"

namespace pt {

namespace {

constexpr int NB = 32;           // bins per axis (scene.cpp splitBinned)
constexpr int BT = 256;          // threads per block
constexpr int CHUNK = 1024;      // positions per block; nodes up to this size are split by one block
constexpr int PER = CHUNK / BT;  // positions per thread
constexpr int BW = 7;            // uints per bin: count, lo.xyz, hi.xyz (ordered-uint floats)
constexpr int BINS_U = 3 * NB * BW;
constexpr int ACC_U = 24;        // children accumulators: per side box lo/hi, centroid lo/hi (ordered uints)

// floats as order-preserving uints (atomicMin / atomicMax on the encoding
// give the float min / max)
__device__ __forceinline__ uint32_t fenc(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fdec(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
__device__ __forceinline__ uint32_t binInit(int i) {
  const int k = i % BW;
  return k == 0 ? 0u : (k <= 3 ? fenc(INFINITY) : fenc(-INFINITY));
}
__device__ __forceinline__ uint32_t accInit(int i) {  // per side: lo(3) hi(3) clo(3) chi(3)
  const int k = i % 12;
  return (k < 3 || (k >= 6 && k < 9)) ? fenc(INFINITY) : fenc(-INFINITY);
}

struct Prim {
  float lo[3], hi[3], c[3];
};
__device__ __forceinline__ Prim loadPrim(const float4* box, const float4* cen, int i) {
  const float4 a = box[2 * (size_t)i], b = box[2 * (size_t)i + 1], c = cen[i];
  return Prim{{a.x, a.y, a.z}, {b.x, b.y, b.z}, {c.x, c.y, c.z}};
}

__device__ __forceinline__ int nodeStart(const BuildNode& n) { return __float_as_int(n.lo.w); }
__device__ __forceinline__ int nodeCount(const BuildNode& n) { return __float_as_int(n.hi.w); }

// the bin of a centroid coordinate (scene.cpp splitBinned: (int)((c - lo) * (NB / ext)), clamped)
__device__ __forceinline__ int binOf(float c, float lo, float scale) {
  int b = (int)((c - lo) * scale);
  return b < 0 ? 0 : (b >= NB ? NB - 1 : b);
}

struct Axes {
  float lo[3], scale[3];
  bool on[3];  // axes with a positive centroid extent
};
__device__ __forceinline__ Axes nodeAxes(const BuildNode& n) {
  Axes a;
  const float clo[3] = {n.clo.x, n.clo.y, n.clo.z}, chi[3] = {n.chi.x, n.chi.y, n.chi.z};
  for (int k = 0; k < 3; k++) {
    const float ext = chi[k] - clo[k];
    a.on[k] = ext > 0.0f;
    a.lo[k] = clo[k];
    a.scale[k] = a.on[k] ? (float)NB / ext : 0.0f;
  }
  return a;
}

__device__ __forceinline__ void binPrim(uint32_t* bins, const Axes& ax, const Prim& p) {
  for (int a = 0; a < 3; a++) {
    if (!ax.on[a]) continue;
    uint32_t* b = bins + (a * NB + binOf(p.c[a], ax.lo[a], ax.scale[a])) * BW;
    atomicAdd(b, 1u);
    for (int k = 0; k < 3; k++) {
      atomicMin(b + 1 + k, fenc(p.lo[k]));
      atomicMax(b + 4 + k, fenc(p.hi[k]));
    }
  }
}
__device__ __forceinline__ void accPrim(uint32_t* acc, bool left, const Prim& p) {
  uint32_t* s = acc + (left ? 0 : 12);
  for (int k = 0; k < 3; k++) {
    atomicMin(s + k, fenc(p.lo[k]));
    atomicMax(s + 3 + k, fenc(p.hi[k]));
    atomicMin(s + 6 + k, fenc(p.c[k]));
    atomicMax(s + 9 + k, fenc(p.c[k]));
  }
}

__device__ __forceinline__ float boxArea(float lx, float ly, float lz, float hx, float hy, float hz) {
  if (hx < lx) return 0.0f;  // empty
  const float dx = hx - lx, dy = hy - ly, dz = hz - lz;
  return 2.0f * (dx * dy + dx * dz + dy * dz);
}

// One wave: the best split of one axis' NB bins (lanes 0..NB-1 hold a bin each).
// Returns (cost, bin) of the first minimum; cost +inf when no split leaves both
// sides non-empty.
__device__ __forceinline__ void sweepAxis(const uint32_t* bins, int axis, float& bestCost, int& bestBin) {
  const int lane = __lane_id();
  const bool in = lane < NB;
  const uint32_t* b = bins + (axis * NB + (in ? lane : 0)) * BW;
  int cnt = in ? (int)b[0] : 0;
  float lo[3], hi[3];
  for (int k = 0; k < 3; k++) {
    lo[k] = in ? fdec(b[1 + k]) : INFINITY;
    hi[k] = in ? fdec(b[4 + k]) : -INFINITY;
  }
  // inclusive prefix (left side: bins 0..lane) and suffix (right side: lane..NB-1)
  int lc = cnt, rc = cnt;
  float llo[3], lhi[3], rlo[3], rhi[3];
  for (int k = 0; k < 3; k++) { llo[k] = rlo[k] = lo[k]; lhi[k] = rhi[k] = hi[k]; }
  for (int off = 1; off < NB; off <<= 1) {
    const int uc = __shfl_up(lc, off, 64);
    const int dc = __shfl_down(rc, off, 64);
    float ul[3], uh[3], dl[3], dh[3];
    for (int k = 0; k < 3; k++) {
      ul[k] = __shfl_up(llo[k], off, 64);
      uh[k] = __shfl_up(lhi[k], off, 64);
      dl[k] = __shfl_down(rlo[k], off, 64);
      dh[k] = __shfl_down(rhi[k], off, 64);
    }
    if (lane >= off) {
      lc += uc;
      for (int k = 0; k < 3; k++) { llo[k] = fminf(llo[k], ul[k]); lhi[k] = fmaxf(lhi[k], uh[k]); }
    }
    if (lane + off < NB) {
      rc += dc;
      for (int k = 0; k < 3; k++) { rlo[k] = fminf(rlo[k], dl[k]); rhi[k] = fmaxf(rhi[k], dh[k]); }
    }
  }
  // split after bin `lane`: left = bins 0..lane, right = lane+1..NB-1
  const int nrc = __shfl_down(rc, 1, 64);
  float nrlo[3], nrhi[3];
  for (int k = 0; k < 3; k++) {
    nrlo[k] = __shfl_down(rlo[k], 1, 64);
    nrhi[k] = __shfl_down(rhi[k], 1, 64);
  }
  float cost = INFINITY;
  if (lane < NB - 1 && lc > 0 && nrc > 0)
    cost = boxArea(llo[0], llo[1], llo[2], lhi[0], lhi[1], lhi[2]) * (float)lc +
           boxArea(nrlo[0], nrlo[1], nrlo[2], nrhi[0], nrhi[1], nrhi[2]) * (float)nrc;
  int bin = lane;
  for (int off = 32; off > 0; off >>= 1) {
    const float oc = __shfl_xor(cost, off, 64);
    const int ob = __shfl_xor(bin, off, 64);
    if (oc < cost || (oc == cost && ob < bin)) { cost = oc; bin = ob; }
  }
  bestCost = cost;
  bestBin = bin;
}

// the split of a node from its bins: (axis, bin), axis -1 = median split
__device__ __forceinline__ int2 chooseSplit(const uint32_t* bins, const Axes& ax) {
  float best = INFINITY;
  int axis = -1, bin = 0;
  for (int a = 0; a < 3; a++) {
    if (!ax.on[a]) continue;
    float c;
    int b;
    sweepAxis(bins, a, c, b);
    if (c < best) { best = c; axis = a; bin = b; }
  }
  return make_int2(axis, bin);
}

__device__ __forceinline__ bool goesLeft(const Prim& p, const Axes& ax, int2 split, int offset, int leftMedian) {
  if (split.x < 0) return offset < leftMedian;
  return binOf(p.c[split.x], ax.lo[split.x], ax.scale[split.x]) <= split.y;
}

// block exclusive scan of one int per thread (BT threads); total returned
__device__ __forceinline__ int blockScan(int v, int* s_wave, int& total) {
  const int lane = __lane_id(), w = threadIdx.x >> 6;
  int incl = v;
  for (int off = 1; off < 64; off <<= 1) {
    const int u = __shfl_up(incl, off, 64);
    if (lane >= off) incl += u;
  }
  if (lane == 63) s_wave[w] = incl;
  __syncthreads();
  int base = 0;
  total = 0;
  for (int k = 0; k < BT / 64; k++) {
    if (k < w) base += s_wave[k];
    total += s_wave[k];
  }
  __syncthreads();
  return base + incl - v;
}

__device__ __forceinline__ BuildNode makeNode(int start, int count, const uint32_t* acc) {
  BuildNode n;
  n.lo = make_float4(fdec(acc[0]), fdec(acc[1]), fdec(acc[2]), __int_as_float(start));
  n.hi = make_float4(fdec(acc[3]), fdec(acc[4]), fdec(acc[5]), __int_as_float(count));
  n.clo = make_float4(fdec(acc[6]), fdec(acc[7]), fdec(acc[8]), __int_as_float(-1));
  n.chi = make_float4(fdec(acc[9]), fdec(acc[10]), fdec(acc[11]), __int_as_float(-1));
  return n;
}

// ------------------------------------------------------------------ kernels
// per triangle: its box and centroid ((p1 + p2 + p3) / 3, scene.cpp centre); the
// root's bounds accumulated into acc[0..11]
__global__ __launch_bounds__(BT) void primsKernel(const float4* geo, int n, float4* box, float4* cen, uint32_t* acc) {
  __shared__ uint32_t s[12];
  if (threadIdx.x < 12) s[threadIdx.x] = accInit(threadIdx.x);
  __syncthreads();
  const int i = blockIdx.x * BT + threadIdx.x;
  if (i < n) {
    const float4 a = geo[4 * (size_t)i], b = geo[4 * (size_t)i + 1], c = geo[4 * (size_t)i + 2];
    Prim p;
    p.lo[0] = fminf(a.x, fminf(b.x, c.x)); p.hi[0] = fmaxf(a.x, fmaxf(b.x, c.x));
    p.lo[1] = fminf(a.y, fminf(b.y, c.y)); p.hi[1] = fmaxf(a.y, fmaxf(b.y, c.y));
    p.lo[2] = fminf(a.z, fminf(b.z, c.z)); p.hi[2] = fmaxf(a.z, fmaxf(b.z, c.z));
    p.c[0] = ((a.x + b.x) + c.x) / 3.0f;
    p.c[1] = ((a.y + b.y) + c.y) / 3.0f;
    p.c[2] = ((a.z + b.z) + c.z) / 3.0f;
    box[2 * (size_t)i] = make_float4(p.lo[0], p.lo[1], p.lo[2], 0.0f);
    box[2 * (size_t)i + 1] = make_float4(p.hi[0], p.hi[1], p.hi[2], 0.0f);
    cen[i] = make_float4(p.c[0], p.c[1], p.c[2], 0.0f);
    accPrim(s, true, p);
  }
  __syncthreads();
  if (threadIdx.x < 12) {  // lo and centroid lo: min; hi and centroid hi: max
    if (threadIdx.x < 3 || (threadIdx.x >= 6 && threadIdx.x < 9)) atomicMin(acc + threadIdx.x, s[threadIdx.x]);
    else atomicMax(acc + threadIdx.x, s[threadIdx.x]);
  }
}

__global__ void initKernel(uint32_t* p, int n, int kind) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = kind == 0 ? binInit(i % BINS_U) : accInit(i % ACC_U);
}

__global__ void iotaKernel(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = i;
}

__global__ void rootKernel(BuildNode* nodes, int n, const uint32_t* acc, int* front) {
  nodes[0] = makeNode(0, n, acc);
  front[0] = 0;
}

// per frontier node: (is large) << 32 | (its chunks)
__global__ void classifyKernel(const BuildNode* nodes, const int* front, int F, unsigned long long* cls) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f > F) return;
  if (f == F) { cls[f] = 0; return; }
  const int c = nodeCount(nodes[front[f]]);
  cls[f] = c > CHUNK ? (1ull << 32) | (unsigned long long)((c + CHUNK - 1) / CHUNK) : 0ull;
}

__global__ void listLargeKernel(const unsigned long long* scan, const unsigned long long* cls, int F, int* largeList) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < F && cls[f]) largeList[scan[f] >> 32] = f;
}

// the frontier node owning chunk t: the last f whose chunk base is <= t
__device__ __forceinline__ int chunkOwner(const unsigned long long* scan, int F, int t) {
  int lo = 0, hi = F;  // invariant: base(lo) <= t < base(hi) (base(F) = total)
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if ((int)(uint32_t)scan[mid] <= t) lo = mid;
    else hi = mid;
  }
  return lo;
}

struct ChunkRef {
  int f, r, node, start, count, cs, ce, first;  // frontier index, large rank, node, node range, chunk range, first chunk
};
__device__ __forceinline__ ChunkRef chunkRef(const BuildNode* nodes, const int* front, const unsigned long long* scan,
                                             int F, int t) {
  ChunkRef c;
  c.f = chunkOwner(scan, F, t);
  c.r = (int)(scan[c.f] >> 32);
  c.first = (int)(uint32_t)scan[c.f];
  c.node = front[c.f];
  const BuildNode n = nodes[c.node];
  c.start = nodeStart(n);
  c.count = nodeCount(n);
  c.cs = c.start + (t - c.first) * CHUNK;
  c.ce = min(c.cs + CHUNK, c.start + c.count);
  return c;
}

__global__ __launch_bounds__(BT) void binLargeKernel(const BuildNode* nodes, const int* front,
                                                     const unsigned long long* scan, int F, const int* perm,
                                                     const float4* box, const float4* cen, uint32_t* gbins) {
  __shared__ uint32_t s[BINS_U];
  for (int i = threadIdx.x; i < BINS_U; i += BT) s[i] = binInit(i);
  __syncthreads();
  const ChunkRef c = chunkRef(nodes, front, scan, F, blockIdx.x);
  const Axes ax = nodeAxes(nodes[c.node]);
  for (int p = c.cs + threadIdx.x; p < c.ce; p += BT) binPrim(s, ax, loadPrim(box, cen, perm[p]));
  __syncthreads();
  uint32_t* g = gbins + (size_t)c.r * BINS_U;
  for (int i = threadIdx.x; i < BINS_U; i += BT) {
    const uint32_t v = s[i];
    const int k = i % BW;
    if (k == 0) { if (v) atomicAdd(g + i, v); }
    else if (v != binInit(i)) {
      if (k <= 3) atomicMin(g + i, v);
      else atomicMax(g + i, v);
    }
  }
}

// one wave per large node: its split from the global bins
__global__ __launch_bounds__(64) void splitLargeKernel(const BuildNode* nodes, const int* front, const int* largeList,
                                                       const uint32_t* gbins, int2* dec) {
  const int r = blockIdx.x;
  const BuildNode n = nodes[front[largeList[r]]];
  const int2 d = chooseSplit(gbins + (size_t)r * BINS_U, nodeAxes(n));
  if (threadIdx.x == 0) dec[r] = d;
}

__global__ __launch_bounds__(BT) void partCountKernel(const BuildNode* nodes, const int* front,
                                                      const unsigned long long* scan, int F, const int* perm,
                                                      const float4* box, const float4* cen, const int2* dec,
                                                      int* chunkLeft, uint32_t* gacc) {
  __shared__ uint32_t s[ACC_U];
  __shared__ int s_left;
  if (threadIdx.x < ACC_U) s[threadIdx.x] = accInit(threadIdx.x);
  if (threadIdx.x == 0) s_left = 0;
  __syncthreads();
  const ChunkRef c = chunkRef(nodes, front, scan, F, blockIdx.x);
  const Axes ax = nodeAxes(nodes[c.node]);
  const int2 d = dec[c.r];
  int left = 0;
  for (int p = c.cs + threadIdx.x; p < c.ce; p += BT) {
    const Prim pr = loadPrim(box, cen, perm[p]);
    const bool l = goesLeft(pr, ax, d, p - c.start, (c.count + 1) / 2);
    left += l;
    accPrim(s, l, pr);
  }
  atomicAdd(&s_left, left);
  __syncthreads();
  if (threadIdx.x == 0) chunkLeft[blockIdx.x] = s_left;
  if (threadIdx.x < ACC_U) {
    const uint32_t v = s[threadIdx.x];
    if (v != accInit(threadIdx.x)) {
      const int k = threadIdx.x % 12;
      if (k < 3 || (k >= 6 && k < 9)) atomicMin(gacc + (size_t)c.r * ACC_U + threadIdx.x, v);
      else atomicMax(gacc + (size_t)c.r * ACC_U + threadIdx.x, v);
    }
  }
}

// stable partition of every large node's chunks into tmp (left side first)
__global__ __launch_bounds__(BT) void partScatterKernel(const BuildNode* nodes, const int* front,
                                                        const unsigned long long* scan, int F, const int* perm,
                                                        const float4* box, const float4* cen, const int2* dec,
                                                        const int* leftScan, int* tmp) {
  __shared__ int s_wave[BT / 64];
  const ChunkRef c = chunkRef(nodes, front, scan, F, blockIdx.x);
  const Axes ax = nodeAxes(nodes[c.node]);
  const int2 d = dec[c.r];
  const int nChunks = (c.count + CHUNK - 1) / CHUNK;
  const int leftCount = leftScan[c.first + nChunks] - leftScan[c.first];
  const int leftBase = leftScan[blockIdx.x] - leftScan[c.first];  // lefts of this node before this chunk
  int idx[PER];
  bool fl[PER];
  int mine = 0;
  const int p0 = c.cs + threadIdx.x * PER;
  for (int j = 0; j < PER; j++) {
    const int p = p0 + j;
    fl[j] = false;
    idx[j] = -1;
    if (p < c.ce) {
      idx[j] = perm[p];
      fl[j] = goesLeft(loadPrim(box, cen, idx[j]), ax, d, p - c.start, (c.count + 1) / 2);
      mine += fl[j];
    }
  }
  int total;
  int lb = leftBase + blockScan(mine, s_wave, total);  // lefts before this thread's first position
  for (int j = 0; j < PER; j++) {
    const int p = p0 + j;
    if (p >= c.ce) break;
    const int o = p - c.start;
    const int dst = fl[j] ? c.start + lb : c.start + leftCount + (o - lb);
    tmp[dst] = idx[j];
    lb += fl[j];
  }
}

__global__ __launch_bounds__(BT) void copyBackKernel(const BuildNode* nodes, const int* front,
                                                     const unsigned long long* scan, int F, const int* tmp,
                                                     int* perm) {
  const ChunkRef c = chunkRef(nodes, front, scan, F, blockIdx.x);
  for (int p = c.cs + threadIdx.x; p < c.ce; p += BT) perm[p] = tmp[p];
}

// children of the large nodes: ids nextId + 2f, nextId + 2f + 1
__global__ void largeChildrenKernel(BuildNode* nodes, const int* front, const unsigned long long* scan,
                                    const int* largeList, int L, const int* leftScan, const uint32_t* gacc,
                                    int nextId) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= L) return;
  const int f = largeList[r];
  const int node = front[f];
  BuildNode& n = nodes[node];
  const int start = nodeStart(n), count = nodeCount(n);
  const int first = (int)(uint32_t)scan[f];
  const int nChunks = (count + CHUNK - 1) / CHUNK;
  const int leftCount = leftScan[first + nChunks] - leftScan[first];
  const int l = nextId + 2 * f;
  nodes[l] = makeNode(start, leftCount, gacc + (size_t)r * ACC_U);
  nodes[l + 1] = makeNode(start + leftCount, count - leftCount, gacc + (size_t)r * ACC_U + 12);
  n.clo.w = __int_as_float(l);
  n.chi.w = __int_as_float(l + 1);
}

// one block per small frontier node (<= CHUNK triangles): bins, SAH, stable
// in-place partition and both children, all in LDS
__global__ __launch_bounds__(BT) void smallSplitKernel(BuildNode* nodes, const int* front, int* perm,
                                                       const float4* box, const float4* cen, int nextId) {
  __shared__ uint32_t s_bins[BINS_U];
  __shared__ uint32_t s_acc[ACC_U];
  __shared__ int s_wave[BT / 64];
  __shared__ int2 s_dec[3];
  const int f = blockIdx.x;
  const int node = front[f];
  const BuildNode n = nodes[node];
  const int start = nodeStart(n), count = nodeCount(n);
  if (count > CHUNK) return;  // a large node (the multi-block path)
  for (int i = threadIdx.x; i < BINS_U; i += BT) s_bins[i] = binInit(i);
  if (threadIdx.x < ACC_U) s_acc[threadIdx.x] = accInit(threadIdx.x);
  __syncthreads();
  const Axes ax = nodeAxes(n);
  Prim pr[PER];
  int idx[PER];
  const int o0 = threadIdx.x * PER;  // node-relative offsets o0 .. o0 + PER - 1
  for (int j = 0; j < PER; j++) {
    idx[j] = -1;
    if (o0 + j < count) {
      idx[j] = perm[start + o0 + j];
      pr[j] = loadPrim(box, cen, idx[j]);
      binPrim(s_bins, ax, pr[j]);
    }
  }
  __syncthreads();
  // SAH: wave a sweeps axis a
  const int w = threadIdx.x >> 6;
  if (w < 3) {
    float c = INFINITY;
    int b = 0;
    if (ax.on[w]) sweepAxis(s_bins, w, c, b);
    if (__lane_id() == 0) s_dec[w] = make_int2(__float_as_int(c), b);
  }
  __syncthreads();
  int2 d = make_int2(-1, 0);
  {
    float best = INFINITY;
    for (int a = 0; a < 3; a++) {
      const float c = __int_as_float(s_dec[a].x);
      if (ax.on[a] && c < best) { best = c; d = make_int2(a, s_dec[a].y); }
    }
  }
  const int median = (count + 1) / 2;
  bool fl[PER];
  int mine = 0;
  for (int j = 0; j < PER; j++) {
    fl[j] = false;
    if (o0 + j < count) {
      fl[j] = goesLeft(pr[j], ax, d, o0 + j, median);
      mine += fl[j];
      accPrim(s_acc, fl[j], pr[j]);
    }
  }
  int leftCount;
  int lb = blockScan(mine, s_wave, leftCount);  // (the scan's barriers also order every read above)
  for (int j = 0; j < PER; j++) {
    const int o = o0 + j;
    if (o >= count) break;
    perm[start + (fl[j] ? lb : leftCount + (o - lb))] = idx[j];
    lb += fl[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int l = nextId + 2 * f;
    nodes[l] = makeNode(start, leftCount, s_acc);
    nodes[l + 1] = makeNode(start + leftCount, count - leftCount, s_acc + 12);
    BuildNode& p = nodes[node];
    p.clo.w = __int_as_float(l);
    p.chi.w = __int_as_float(l + 1);
  }
}

__global__ void needKernel(const BuildNode* nodes, int first, int n, int leafSize, int* need) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > n) return;
  need[k] = k < n && nodeCount(nodes[first + k]) > leafSize ? 1 : 0;
}
__global__ void nextFrontKernel(const int* need, const int* scan, int first, int n, int* front) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n && need[k]) front[scan[k]] = first + k;
}

// device ids of the internal nodes: breadth-first rank among them
__global__ void internalKernel(const BuildNode* nodes, int M, int leafSize, int* isInt) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > M) return;
  isInt[k] = k < M && nodeCount(nodes[k]) > leafSize ? 1 : 0;
}

__device__ __forceinline__ int childRef(const BuildNode* nodes, const int* devId, int k, int leafSize) {
  const BuildNode& c = nodes[k];
  const int cnt = nodeCount(c);
  if (cnt > leafSize) return devId[k];
  return (int)~(((uint32_t)nodeStart(c) << LEAF_CNT_BITS) | (uint32_t)(cnt - 1));
}
// pt_runtime.cpp encodeWideTree's widening of the host-built tree
__device__ __forceinline__ void widen(float4& lo, float4& hi, float inflate, float inflateAbs) {
  const float ex = inflate * (fabsf(lo.x) + fabsf(hi.x) + (hi.x - lo.x)) + inflateAbs + 1e-30f;
  const float ey = inflate * (fabsf(lo.y) + fabsf(hi.y) + (hi.y - lo.y)) + inflateAbs + 1e-30f;
  const float ez = inflate * (fabsf(lo.z) + fabsf(hi.z) + (hi.z - lo.z)) + inflateAbs + 1e-30f;
  lo.x -= ex; lo.y -= ey; lo.z -= ez;
  hi.x += ex; hi.y += ey; hi.z += ez;
}
// wide records of the internal nodes (pt_trace.h visitNode layout); inflateAbs is
// relAbs x the scene's largest coordinate magnitude (the root box's)
__global__ void encodeKernel(const BuildNode* nodes, int M, int leafSize, const int* devId, float inflate,
                             float relAbs, float4* bvh) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= M) return;
  const BuildNode n = nodes[k];
  if (nodeCount(n) <= leafSize) return;
  const BuildNode r0 = nodes[0];
  const float scale = fmaxf(fmaxf(fmaxf(fabsf(r0.lo.x), fabsf(r0.hi.x)), fmaxf(fabsf(r0.lo.y), fabsf(r0.hi.y))),
                            fmaxf(fabsf(r0.lo.z), fabsf(r0.hi.z)));
  const float inflateAbs = relAbs * scale;
  const int L = __float_as_int(n.clo.w), R = __float_as_int(n.chi.w);
  const BuildNode a = nodes[L], b = nodes[R];
  float4 la = make_float4(a.lo.x, a.lo.y, a.lo.z, 0), lb = make_float4(a.hi.x, a.hi.y, a.hi.z, 0);
  float4 ra = make_float4(b.lo.x, b.lo.y, b.lo.z, 0), rb = make_float4(b.hi.x, b.hi.y, b.hi.z, 0);
  widen(la, lb, inflate, inflateAbs);
  widen(ra, rb, inflate, inflateAbs);
  float4* o = bvh + 4 * (size_t)devId[k];
  o[0] = make_float4(la.x, ra.x, la.y, ra.y);
  o[1] = make_float4(la.z, ra.z, lb.x, rb.x);
  o[2] = make_float4(lb.y, rb.y, lb.z, rb.z);
  o[3] = make_float4(__int_as_float(childRef(nodes, devId, L, leafSize)),
                     __int_as_float(childRef(nodes, devId, R, leafSize)), 0.0f, 0.0f);
}

// pair records in the built order (pt_runtime.cpp buildPairs): position i holds
// triangles order[i] (x) and order[i + 1] (y; zeros past the last), and their uploaded
// indices (the record's last two floats, as int bits; -1 past the last)
__global__ void pairsKernel(const float4* geo, const int* order, int n, float4* pairs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4* A = geo + 4 * (size_t)order[i];
  const float4 z = make_float4(0, 0, 0, 0);
  const bool hasB = i + 1 < n;
  const float4* B = geo + 4 * (size_t)(hasB ? order[i + 1] : 0);
  const float4 a0 = A[0], a1 = A[1], a2 = A[2], a3 = A[3];
  const float4 b0 = hasB ? B[0] : z, b1 = hasB ? B[1] : z, b2 = hasB ? B[2] : z, b3 = hasB ? B[3] : z;
  float4* r = pairs + (size_t)i * PAIR_F4;
  r[0] = make_float4(a0.x, b0.x, a0.y, b0.y);
  r[1] = make_float4(a0.z, b0.z, a1.x, b1.x);
  r[2] = make_float4(a1.y, b1.y, a1.z, b1.z);
  r[3] = make_float4(a2.x, b2.x, a2.y, b2.y);
  r[4] = make_float4(a2.z, b2.z, a3.x, b3.x);
  r[5] = make_float4(a3.y, b3.y, a3.z, b3.z);
  r[6] = make_float4(a0.w, b0.w, __int_as_float(order[i]), __int_as_float(hasB ? order[i + 1] : -1));
}

// ------------------------------------------------------------ 4-wide collapse
// pt_runtime.cpp encodeWide4 on the device, level by level: every wide node of a
// level takes its binary node's two children and keeps replacing the internal
// child of largest surface area (first one on ties, areas in double as on the
// host) by that child's two children until it has four; the next level's wide
// nodes are the internal children in (node, child) order, so ids are
// breadth-first and identical to the host collapse of the same binary tree.
__device__ __forceinline__ bool bLeaf(const BuildNode& n, int leafSize) { return nodeCount(n) <= leafSize; }
__device__ __forceinline__ double bArea(const BuildNode& n) {
  const double dx = (double)n.hi.x - n.lo.x, dy = (double)n.hi.y - n.lo.y, dz = (double)n.hi.z - n.lo.z;
  return dx * dy + dx * dz + dy * dz;
}
__global__ void w4ExpandKernel(const BuildNode* nodes, const int* front, int F, int leafSize, int4* kids, int* cnt) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f > F) return;
  if (f == F) { cnt[f] = 0; return; }
  const BuildNode b = nodes[front[f]];
  int k[4] = {__float_as_int(b.clo.w), __float_as_int(b.chi.w), -1, -1};
  int n = 2;
  while (n < 4) {
    int pick = -1;
    double pa = -1.0;
    for (int i = 0; i < n; i++) {
      const BuildNode c = nodes[k[i]];
      if (!bLeaf(c, leafSize) && bArea(c) > pa) { pa = bArea(c); pick = i; }
    }
    if (pick < 0) break;
    const BuildNode c = nodes[k[pick]];
    k[pick] = __float_as_int(c.clo.w);
    k[n++] = __float_as_int(c.chi.w);
  }
  int internal = 0;
  for (int i = 0; i < n; i++) internal += !bLeaf(nodes[k[i]], leafSize);
  kids[f] = make_int4(k[0], k[1], k[2], k[3]);
  cnt[f] = internal;
}
// the level's records (wide ids base + f) and the next level's frontier (wide ids base + F + scan)
__global__ void w4EncodeKernel(const BuildNode* nodes, const int4* kids, const int* scan, int F, int base,
                               int leafSize, float inflate, float relAbs, float4* out, int* nextFront) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  const BuildNode r0 = nodes[0];
  const float scale = fmaxf(fmaxf(fmaxf(fabsf(r0.lo.x), fabsf(r0.hi.x)), fmaxf(fabsf(r0.lo.y), fabsf(r0.hi.y))),
                            fmaxf(fabsf(r0.lo.z), fabsf(r0.hi.z)));
  const float inflateAbs = relAbs * scale;
  const int4 kv = kids[f];
  const int k[4] = {kv.x, kv.y, kv.z, kv.w};
  float lo[3][4], hi[3][4];
  int ref[4];
  int next = scan[f];
  for (int i = 0; i < 4; i++) {
    if (k[i] < 0) {
      ref[i] = REF_NONE;
      for (int a = 0; a < 3; a++) { lo[a][i] = INFINITY; hi[a][i] = -INFINITY; }
      continue;
    }
    const BuildNode c = nodes[k[i]];
    if (bLeaf(c, leafSize)) {
      ref[i] = (int)~(((uint32_t)nodeStart(c) << LEAF_CNT_BITS) | (uint32_t)(nodeCount(c) - 1));
    } else {
      nextFront[next] = k[i];
      ref[i] = base + F + next;
      next++;
    }
    float4 l = make_float4(c.lo.x, c.lo.y, c.lo.z, 0.0f), h = make_float4(c.hi.x, c.hi.y, c.hi.z, 0.0f);
    widen(l, h, inflate, inflateAbs);
    lo[0][i] = l.x; lo[1][i] = l.y; lo[2][i] = l.z;
    hi[0][i] = h.x; hi[1][i] = h.y; hi[2][i] = h.z;
  }
  float4* r = out + (size_t)(base + f) * W4_F4;
  for (int a = 0; a < 3; a++) {
    r[a] = make_float4(lo[a][0], lo[a][1], lo[a][2], lo[a][3]);
    r[3 + a] = make_float4(hi[a][0], hi[a][1], hi[a][2], hi[a][3]);
  }
  r[6] = make_float4(__int_as_float(ref[0]), __int_as_float(ref[1]), __int_as_float(ref[2]), __int_as_float(ref[3]));
  r[7] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

inline int blocks(long n, int t = 256) { return (int)((n + t - 1) / t); }

}  // namespace

#define BK(x)                              \
  do {                                     \
    hipError_t e_ = (x);                   \
    if (e_ != hipSuccess) return e_;       \
  } while (0)

hipError_t buildAccelDevice(const float4* geo, int nTri, int leafSize, float inflate, float inflateRelAbs,
                            AccelBuild& out, hipStream_t s) {
  if (nTri < 1 || leafSize < 1 || leafSize > MAX_LEAF || nTri > MAX_TRIS) return hipErrorInvalidValue;
  out = AccelBuild{};
  const size_t N = (size_t)nTri, maxNodes = 2 * N + 1;
  float4 *box = nullptr, *cen = nullptr;
  int *tmp = nullptr, *frontA = nullptr, *frontB = nullptr, *need = nullptr, *needScan = nullptr, *largeList = nullptr,
      *chunkLeft = nullptr, *leftScan = nullptr;
  unsigned long long *cls = nullptr, *clsScan = nullptr;
  uint32_t *acc = nullptr, *gbins = nullptr, *gacc = nullptr;
  int2* dec = nullptr;
  void* cubTmp = nullptr;
  BuildNode* nodes = nullptr;
  // a large node of c triangles has ceil(c / CHUNK) < 2 c / CHUNK chunks
  const size_t maxChunks = 2 * (N / CHUNK) + 2, maxLarge = N / CHUNK + 1;
  hipError_t e = hipSuccess;
  auto alloc = [&](auto** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc((void**)p, bytes);
  };
  alloc(&box, 2 * N * sizeof(float4));
  alloc(&cen, N * sizeof(float4));
  alloc(&out.order, N * sizeof(int));
  alloc(&tmp, N * sizeof(int));
  alloc(&nodes, maxNodes * sizeof(BuildNode));
  alloc(&frontA, (N + 1) * sizeof(int));
  alloc(&frontB, (N + 1) * sizeof(int));
  alloc(&need, (maxNodes + 1) * sizeof(int));
  alloc(&needScan, (maxNodes + 1) * sizeof(int));
  alloc(&cls, (N + 2) * sizeof(unsigned long long));
  alloc(&clsScan, (N + 2) * sizeof(unsigned long long));
  alloc(&largeList, maxLarge * sizeof(int));
  alloc(&chunkLeft, (maxChunks + 1) * sizeof(int));
  alloc(&leftScan, (maxChunks + 1) * sizeof(int));
  alloc(&acc, 12 * sizeof(uint32_t));
  alloc(&gbins, maxLarge * BINS_U * sizeof(uint32_t));
  alloc(&gacc, maxLarge * ACC_U * sizeof(uint32_t));
  alloc(&dec, maxLarge * sizeof(int2));
  size_t cubBytes = 0;
  if (e == hipSuccess) {
    size_t a = 0, b = 0;
    e = hipcub::DeviceScan::ExclusiveSum(nullptr, a, cls, clsScan, (int)(N + 1), s);
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, b, need, needScan, (int)(maxNodes + 1), s);
    cubBytes = std::max(a, b);
  }
  alloc(&cubTmp, cubBytes);
  unsigned long long* hostCls = nullptr;
  if (e == hipSuccess) e = hipHostMalloc((void**)&hostCls, 2 * sizeof(unsigned long long));
  int M = 1, depth = 1;
  if (e == hipSuccess) {
    e = [&]() -> hipError_t {
      hipLaunchKernelGGL(initKernel, dim3(1), dim3(64), 0, s, acc, 12, 1);
      hipLaunchKernelGGL(primsKernel, dim3(blocks(N, BT)), dim3(BT), 0, s, geo, nTri, box, cen, acc);
      hipLaunchKernelGGL(iotaKernel, dim3(blocks(N)), dim3(256), 0, s, out.order, nTri);
      hipLaunchKernelGGL(rootKernel, dim3(1), dim3(1), 0, s, nodes, nTri, acc, frontA);
      BK(hipGetLastError());
      int F = nTri > leafSize ? 1 : 0;
      int* front = frontA;
      int* nextFront = frontB;
      int nextId = 1;
      while (F > 0) {
        // large nodes and their chunks
        hipLaunchKernelGGL(classifyKernel, dim3(blocks(F + 1)), dim3(256), 0, s, nodes, front, F, cls);
        size_t cb = cubBytes;
        BK(hipcub::DeviceScan::ExclusiveSum(cubTmp, cb, cls, clsScan, F + 1, s));
        BK(hipMemcpyAsync(hostCls, clsScan + F, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        BK(hipStreamSynchronize(s));
        const int L = (int)(hostCls[0] >> 32), T = (int)(uint32_t)hostCls[0];
        if (T > 0) {
          hipLaunchKernelGGL(initKernel, dim3(blocks((long)L * BINS_U)), dim3(256), 0, s, gbins, L * BINS_U, 0);
          hipLaunchKernelGGL(initKernel, dim3(blocks((long)L * ACC_U)), dim3(256), 0, s, gacc, L * ACC_U, 1);
          hipLaunchKernelGGL(listLargeKernel, dim3(blocks(F)), dim3(256), 0, s, clsScan, cls, F, largeList);
          hipLaunchKernelGGL(binLargeKernel, dim3(T), dim3(BT), 0, s, nodes, front, clsScan, F, out.order, box, cen,
                             gbins);
          hipLaunchKernelGGL(splitLargeKernel, dim3(L), dim3(64), 0, s, nodes, front, largeList, gbins, dec);
          hipLaunchKernelGGL(partCountKernel, dim3(T), dim3(BT), 0, s, nodes, front, clsScan, F, out.order, box, cen,
                             dec, chunkLeft, gacc);
          BK(hipMemsetAsync(chunkLeft + T, 0, sizeof(int), s));
          cb = cubBytes;
          BK(hipcub::DeviceScan::ExclusiveSum(cubTmp, cb, chunkLeft, leftScan, T + 1, s));
          hipLaunchKernelGGL(partScatterKernel, dim3(T), dim3(BT), 0, s, nodes, front, clsScan, F, out.order, box,
                             cen, dec, leftScan, tmp);
          hipLaunchKernelGGL(copyBackKernel, dim3(T), dim3(BT), 0, s, nodes, front, clsScan, F, tmp, out.order);
          hipLaunchKernelGGL(largeChildrenKernel, dim3(blocks(L)), dim3(256), 0, s, nodes, front, clsScan, largeList,
                             L, leftScan, gacc, nextId);
        }
        if (T == 0 || L < F)
          hipLaunchKernelGGL(smallSplitKernel, dim3(F), dim3(BT), 0, s, nodes, front, out.order, box, cen, nextId);
        // the next frontier: children still larger than a leaf, in id order
        const int nc = 2 * F;
        hipLaunchKernelGGL(needKernel, dim3(blocks(nc + 1)), dim3(256), 0, s, nodes, nextId, nc, leafSize, need);
        cb = cubBytes;
        BK(hipcub::DeviceScan::ExclusiveSum(cubTmp, cb, need, needScan, nc + 1, s));
        hipLaunchKernelGGL(nextFrontKernel, dim3(blocks(nc)), dim3(256), 0, s, need, needScan, nextId, nc, nextFront);
        BK(hipGetLastError());
        int nf = 0;
        BK(hipMemcpyAsync(hostCls + 1, needScan + nc, sizeof(int), hipMemcpyDeviceToHost, s));
        BK(hipStreamSynchronize(s));
        std::memcpy(&nf, hostCls + 1, sizeof(int));
        nextId += nc;
        if (++depth > nTri + 1) return hipErrorUnknown;  // every split shrinks its node: unreachable
        F = nf;
        std::swap(front, nextFront);
      }
      M = nextId;
      // device ids (breadth-first among the internal nodes), wide records, pair records
      hipLaunchKernelGGL(internalKernel, dim3(blocks(M + 1)), dim3(256), 0, s, nodes, M, leafSize, need);
      size_t cb = cubBytes;
      BK(hipcub::DeviceScan::ExclusiveSum(cubTmp, cb, need, needScan, M + 1, s));
      int nDev = 0;
      BK(hipMemcpyAsync(hostCls, needScan + M, sizeof(int), hipMemcpyDeviceToHost, s));
      BK(hipStreamSynchronize(s));
      std::memcpy(&nDev, hostCls, sizeof(int));
      BK(hipMalloc(&out.bvh, (size_t)std::max(nDev, 1) * 4 * sizeof(float4)));
      BK(hipMemsetAsync(out.bvh, 0, (size_t)std::max(nDev, 1) * 4 * sizeof(float4), s));
      BK(hipMalloc(&out.pairs, N * PAIR_F4 * sizeof(float4)));
      hipLaunchKernelGGL(encodeKernel, dim3(blocks(M)), dim3(256), 0, s, nodes, M, leafSize, needScan, inflate,
                         inflateRelAbs, out.bvh);
      hipLaunchKernelGGL(pairsKernel, dim3(blocks(N)), dim3(256), 0, s, geo, out.order, nTri, out.pairs);
      BK(hipGetLastError());
      out.nDev = nDev;
      out.rootRef = nTri > leafSize ? 0 : (int)~(uint32_t)(nTri - 1);  // root: device id 0, or one leaf [0, n)
      return hipSuccess;
    }();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  out.nNodes = M;
  out.depth = depth;
  if (e == hipSuccess) {
    out.nodes = nodes;  // kept for pt_build_bvh_device; freeAccelBuild releases it
    nodes = nullptr;
  }
  (void)hipFree(box); (void)hipFree(cen); (void)hipFree(tmp); (void)hipFree(nodes);
  (void)hipFree(frontA); (void)hipFree(frontB); (void)hipFree(need); (void)hipFree(needScan);
  (void)hipFree(cls); (void)hipFree(clsScan); (void)hipFree(largeList); (void)hipFree(chunkLeft);
  (void)hipFree(leftScan); (void)hipFree(acc); (void)hipFree(gbins); (void)hipFree(gacc); (void)hipFree(dec);
  (void)hipFree(cubTmp);
  if (hostCls) (void)hipHostFree(hostCls);
  if (e != hipSuccess) freeAccelBuild(out);
  return e;
}

hipError_t collapseWide4Device(const BuildNode* nodes, int nNodes, int leafSize, float inflate, float inflateRelAbs,
                               float4** out, int* rootRef, int* nDev, int* depth, hipStream_t s) {
  *out = nullptr;
  *nDev = 0;
  *depth = 1;
  if (nNodes < 1) return hipErrorInvalidValue;
  BuildNode root;
  hipError_t e = hipMemcpyAsync(&root, nodes, sizeof(root), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  int rootCount;
  std::memcpy(&rootCount, &root.hi.w, 4);
  if (rootCount <= leafSize) {  // one leaf: no wide node
    int start;
    std::memcpy(&start, &root.lo.w, 4);
    *rootRef = (int)~(((uint32_t)start << LEAF_CNT_BITS) | (uint32_t)(rootCount - 1));
    BK(hipMalloc(out, W4_F4 * sizeof(float4)));
    return hipMemsetAsync(*out, 0, W4_F4 * sizeof(float4), s);
  }
  // every wide node holds >= 2 binary nodes' worth of children: at most nNodes / 2 of them
  const size_t maxW = (size_t)nNodes / 2 + 1;
  int *frontA = nullptr, *frontB = nullptr, *cnt = nullptr, *scan = nullptr, *host = nullptr;
  int4* kids = nullptr;
  void* cub = nullptr;
  size_t cubBytes = 0;
  auto fin = [&](hipError_t r) {
    (void)hipFree(frontA); (void)hipFree(frontB); (void)hipFree(cnt); (void)hipFree(scan); (void)hipFree(kids);
    (void)hipFree(cub);
    if (host) (void)hipHostFree(host);
    if (r != hipSuccess) { (void)hipFree(*out); *out = nullptr; }
    return r;
  };
  if ((e = hipMalloc(out, maxW * W4_F4 * sizeof(float4))) != hipSuccess || (e = hipMalloc(&frontA, maxW * sizeof(int))) ||
      (e = hipMalloc(&frontB, maxW * sizeof(int))) || (e = hipMalloc(&cnt, (maxW + 1) * sizeof(int))) ||
      (e = hipMalloc(&scan, (maxW + 1) * sizeof(int))) || (e = hipMalloc(&kids, maxW * sizeof(int4))) ||
      (e = hipHostMalloc((void**)&host, sizeof(int))))
    return fin(e);
  if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, cubBytes, cnt, scan, (int)(maxW + 1), s)) ||
      (e = hipMalloc(&cub, std::max<size_t>(cubBytes, 1))))
    return fin(e);
  const int zero = 0;
  if ((e = hipMemcpyAsync(frontA, &zero, sizeof(int), hipMemcpyHostToDevice, s))) return fin(e);
  int F = 1, base = 0, d = 0;
  int* front = frontA;
  int* next = frontB;
  while (F > 0) {
    hipLaunchKernelGGL(w4ExpandKernel, dim3(blocks(F + 1)), dim3(256), 0, s, nodes, front, F, leafSize, kids, cnt);
    size_t cb = cubBytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(cub, cb, cnt, scan, F + 1, s))) return fin(e);
    hipLaunchKernelGGL(w4EncodeKernel, dim3(blocks(F)), dim3(256), 0, s, nodes, kids, scan, F, base, leafSize, inflate,
                       inflateRelAbs, *out, next);
    if ((e = hipGetLastError()) || (e = hipMemcpyAsync(host, scan + F, sizeof(int), hipMemcpyDeviceToHost, s)) ||
        (e = hipStreamSynchronize(s)))
      return fin(e);
    base += F;
    F = *host;
    d++;
    if ((size_t)base + F > maxW) return fin(hipErrorUnknown);  // cannot happen: every wide node splits a binary one
    std::swap(front, next);
  }
  *nDev = base;
  *depth = d;
  *rootRef = 0;
  return fin(hipSuccess);
}

void freeAccelBuild(AccelBuild& a) {
  (void)hipFree(a.bvh);
  (void)hipFree(a.pairs);
  (void)hipFree(a.order);
  (void)hipFree(a.nodes);
  a = AccelBuild{};
}

}  // namespace pt
