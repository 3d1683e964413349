// pt_primary.hip -- camera-ray bins: for one camera, the triangles each 8x8
// pixel tile's camera rays can hit, so the megakernel finds a camera ray's
// closest hit by testing its tile's few triangles (pass1.fsh hitTriangle
// IS:251-301, the same test as the traversal's) instead of walking the BVH
// (pt_kernels.hip primaryPacket).
//
// Every camera ray of pixel (px, py) leaves the eye through the image-plane
// point (x, y, -1.5) of camera space with x within a quarter pixel of the
// pixel's centre (IS:846-850: the AA jitter is +-0.5/W in NDC). A triangle
// point q (camera space, q = R^T (P - eye), R = cameraRotate's rotation) lies on
// such a ray iff it projects to that image point, and a hit needs t >= 0.0005
// (IS:281), so q.z < -2.5e-4 for every point a camera ray can hit. A triangle's
// bins are the tiles its projection -- clipped to q.z <= -2.5e-4 -- touches,
// widened by two pixels (far beyond the float rounding of the ray directions):
// conservative, so every triangle a camera ray hits is in its tile's bin.
// Results stay the reference's: a tie or an unreachable winner is retraced
// through the uploaded tree (as for the runtime tree, pt_trace.h refReachable).
//
// Build (once per camera and scene, on the frame's stream):
//   binRectKernel   per triangle: its tile rectangle (empty if off-screen / behind)
//   scan            per-triangle tile counts -> offsets (hipcub)
//   binCountKernel  per (triangle, tile) entry: count the tile's triangles
//   scan            per-tile counts -> bin starts (hipcub)
//   binFillKernel   per entry: place the triangle in its tile's bin
//   binGatherKernel per entry: its triangle's geometry record and leaf box, in bin order
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "pt_kernels.h"

namespace pt {

struct BinCam {
  double eye[3];
  double R[9];  // columns c0, c1, c2 of cameraRotate's upper 3x3
  int width, height, tilesX, tilesY;
};

constexpr double kNearZ = -2.5e-4;  // a hit point of a camera ray has q.z below this (t >= 0.0005)
constexpr double kMarginPx = 2.0;   // bins widened by this many pixels

__device__ __forceinline__ void toCam(const BinCam& c, const float4 v, double q[3]) {
  const double r0 = (double)v.x - c.eye[0], r1 = (double)v.y - c.eye[1], r2 = (double)v.z - c.eye[2];
  for (int a = 0; a < 3; a++) q[a] = c.R[3 * a] * r0 + c.R[3 * a + 1] * r1 + c.R[3 * a + 2] * r2;
}

// tile rectangle of triangle i -> rect[i] = (tx0, ty0, tx1, ty1) (tx0 > tx1: none), count[i] = its tiles
__global__ void binRectKernel(BinCam c, const float4* geo, int nTri, int4* rect, int* count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nTri) return;
  double q[3][3];
  for (int k = 0; k < 3; k++) toCam(c, geo[4 * (size_t)i + k], q[k]);
  // clip the triangle to q.z <= kNearZ (Sutherland-Hodgman, one plane): <= 4 points
  double px[4], py[4];
  int n = 0;
  for (int k = 0; k < 3; k++) {
    const double* a = q[k];
    const double* b = q[(k + 1) % 3];
    const bool ain = a[2] <= kNearZ, bin = b[2] <= kNearZ;
    if (ain) {
      px[n] = -1.5 * a[0] / a[2];
      py[n] = -1.5 * a[1] / a[2];
      n++;
    }
    if (ain != bin) {
      const double s = (kNearZ - a[2]) / (b[2] - a[2]);
      const double x = a[0] + s * (b[0] - a[0]), y = a[1] + s * (b[1] - a[1]);
      px[n] = -1.5 * x / kNearZ;
      py[n] = -1.5 * y / kNearZ;
      n++;
    }
  }
  int4 r = make_int4(1, 1, 0, 0);
  int cnt = 0;
  if (n > 0) {
    double x0 = 1e300, x1 = -1e300, y0 = 1e300, y1 = -1e300;
    for (int k = 0; k < n; k++) {
      // image plane -> pixel-centre coordinates (pix = (2 p + 1) / W - 1, IS:846)
      const double X = (px[k] + 1.0) * 0.5 * c.width - 0.5, Y = (py[k] + 1.0) * 0.5 * c.height - 0.5;
      x0 = fmin(x0, X); x1 = fmax(x1, X); y0 = fmin(y0, Y); y1 = fmax(y1, Y);
    }
    x0 -= kMarginPx; y0 -= kMarginPx; x1 += kMarginPx; y1 += kMarginPx;
    if (x1 >= 0.0 && y1 >= 0.0 && x0 <= c.width - 1.0 && y0 <= c.height - 1.0) {
      const int tx0 = (int)fmax(0.0, floor(x0 / 8.0)), ty0 = (int)fmax(0.0, floor(y0 / 8.0));
      const int tx1 = (int)fmin((double)(c.tilesX - 1), floor(x1 / 8.0));
      const int ty1 = (int)fmin((double)(c.tilesY - 1), floor(y1 / 8.0));
      if (tx0 <= tx1 && ty0 <= ty1) {
        r = make_int4(tx0, ty0, tx1, ty1);
        cnt = (tx1 - tx0 + 1) * (ty1 - ty0 + 1);
      }
    }
  }
  rect[i] = r;
  count[i] = cnt;
}

// entry e -> (triangle, tile): the triangle is the last one whose offset is <= e
__device__ __forceinline__ void entryOf(const int* offset, const int4* rect, int nTri, int tilesX, int e, int& tri,
                                        int& tile) {
  int lo = 0, hi = nTri - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (offset[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  tri = lo;
  const int4 r = rect[lo];
  const int k = e - offset[lo], w = r.z - r.x + 1;
  tile = (r.y + k / w) * tilesX + r.x + k % w;
}

__global__ void binCountKernel(const int* offset, const int4* rect, int nTri, int tilesX, int entries, int* tileCount) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= entries) return;
  int tri, tile;
  entryOf(offset, rect, nTri, tilesX, e, tri, tile);
  atomicAdd(tileCount + tile, 1);
}

__global__ void binFillKernel(const int* offset, const int4* rect, int nTri, int tilesX, int entries, const int* binStart,
                              int* cursor, int* binTris) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= entries) return;
  int tri, tile;
  entryOf(offset, rect, nTri, tilesX, e, tri, tile);
  binTris[binStart[tile] + atomicAdd(cursor + tile, 1)] = tri;
}

// per entry: its triangle's geometry record and reference leaf box, next to each other in bin order
__global__ void binGatherKernel(const int* binTris, int entries, const float4* geo, const float4* leafBox,
                                float4* binGeo, float4* binBox) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= entries) return;
  const int i = binTris[e];
  for (int q = 0; q < 4; q++) binGeo[4 * (size_t)e + q] = geo[4 * (size_t)i + q];
  for (int q = 0; q < 2; q++) binBox[2 * (size_t)e + q] = leafBox[2 * (size_t)i + q];
}

// exclusive prefix sum of n ints in place-free form (out may not alias in); the total lands in out[n]
static hipError_t scanInts(const int* in, int* out, int n, void*& tmp, size_t& tmpBytes, hipStream_t s) {
  size_t need = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, in, out, n + 1, s);
  if (e != hipSuccess) return e;
  if (need > tmpBytes) {
    if (tmp) (void)hipFree(tmp);
    tmp = nullptr;
    e = hipMalloc(&tmp, need);
    if (e != hipSuccess) { tmpBytes = 0; return e; }
    tmpBytes = need;
  }
  return hipcub::DeviceScan::ExclusiveSum(tmp, need, in, out, n + 1, s);
}

hipError_t buildPrimaryBins(const float eye[3], const float cam[16], int width, int height, const float4* geo,
                            const float4* leafBox, int nTri, PrimaryBins& b, hipStream_t s) {
  // the camera-ray pass reads each bin entry's geometry and reference leaf box from the gathered
  // binGeo / binBox only (binGatherKernel): without leaf boxes it would test unwritten records
  if (!geo || !leafBox) return hipErrorInvalidValue;
  BinCam c;
  for (int a = 0; a < 3; a++) c.eye[a] = eye[a];
  // columns c0 = cam[0..2], c1 = cam[4..6], c2 = cam[8..10] (column-major, IS:849)
  for (int a = 0; a < 3; a++) {
    c.R[3 * a + 0] = cam[4 * a + 0];
    c.R[3 * a + 1] = cam[4 * a + 1];
    c.R[3 * a + 2] = cam[4 * a + 2];
  }
  c.width = width;
  c.height = height;
  c.tilesX = (width + 7) / 8;
  c.tilesY = (height + 7) / 8;
  const int nTiles = c.tilesX * c.tilesY;
  hipError_t e;
  auto grow = [&](auto*& p, size_t& cap, size_t need) -> hipError_t {
    if (need <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t r = hipMalloc(&p, need * sizeof(*p));
    if (r == hipSuccess) cap = need;
    return r;
  };
  if ((e = grow(b.rect, b.rectCap, (size_t)nTri)) != hipSuccess) return e;
  if ((e = grow(b.triCount, b.triCountCap, (size_t)nTri + 1)) != hipSuccess) return e;
  if ((e = grow(b.triOffset, b.triOffsetCap, (size_t)nTri + 1)) != hipSuccess) return e;
  if ((e = grow(b.tileCount, b.tileCountCap, (size_t)nTiles + 1)) != hipSuccess) return e;
  if ((e = grow(b.binStart, b.binStartCap, (size_t)nTiles + 1)) != hipSuccess) return e;
  const int B = 256;
  hipLaunchKernelGGL(binRectKernel, dim3((nTri + B - 1) / B), dim3(B), 0, s, c, geo, nTri, b.rect, b.triCount);
  if ((e = hipMemsetAsync(b.triCount + nTri, 0, sizeof(int), s)) != hipSuccess) return e;
  if ((e = scanInts(b.triCount, b.triOffset, nTri, b.tmp, b.tmpBytes, s)) != hipSuccess) return e;
  int entries = 0;  // the one host sync of a bin build (sizes the entry passes and the bin array)
  if ((e = hipMemcpyAsync(&entries, b.triOffset + nTri, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  if ((e = grow(b.binTris, b.binTrisCap, (size_t)std::max(entries, 1))) != hipSuccess) return e;
  if ((e = hipMemsetAsync(b.tileCount, 0, ((size_t)nTiles + 1) * sizeof(int), s)) != hipSuccess) return e;
  if (entries > 0)
    hipLaunchKernelGGL(binCountKernel, dim3((entries + B - 1) / B), dim3(B), 0, s, b.triOffset, b.rect, nTri, c.tilesX,
                       entries, b.tileCount);
  if ((e = scanInts(b.tileCount, b.binStart, nTiles, b.tmp, b.tmpBytes, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(b.tileCount, 0, ((size_t)nTiles + 1) * sizeof(int), s)) != hipSuccess) return e;  // cursors
  if (entries > 0)
    hipLaunchKernelGGL(binFillKernel, dim3((entries + B - 1) / B), dim3(B), 0, s, b.triOffset, b.rect, nTri, c.tilesX,
                       entries, b.binStart, b.tileCount, b.binTris);
  if ((e = grow(b.binGeo, b.binGeoCap, 4 * (size_t)std::max(entries, 1))) != hipSuccess) return e;
  if ((e = grow(b.binBox, b.binBoxCap, 2 * (size_t)std::max(entries, 1))) != hipSuccess) return e;
  if (entries > 0 && leafBox)
    hipLaunchKernelGGL(binGatherKernel, dim3((entries + B - 1) / B), dim3(B), 0, s, b.binTris, entries, geo, leafBox,
                       b.binGeo, b.binBox);
  b.tilesX = c.tilesX;
  b.tilesY = c.tilesY;
  b.entries = entries;
  return hipGetLastError();
}

void freePrimaryBins(PrimaryBins& b) {
  for (void* p : {(void*)b.rect, (void*)b.triCount, (void*)b.triOffset, (void*)b.tileCount, (void*)b.binStart,
                  (void*)b.binTris, (void*)b.binGeo, (void*)b.binBox, b.tmp})
    if (p) (void)hipFree(p);
  b = PrimaryBins{};
}

}  // namespace pt
