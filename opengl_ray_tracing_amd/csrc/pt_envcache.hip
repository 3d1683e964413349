// pt_envcache.hip -- calculateHdrCache (ImportanceSampling_LowDiscrepancySequence/
// main.cpp:555-652) on the GPU, bit-identical to the host restatement
// (scene.cpp pt_hdr_cache): every floating-point sum runs in the reference's
// order. Its one inherently sequential step, the float sum of all luminances
// in scanline order, is a single dependent chain (hdrSumKernel). The per-column sums and prefix sums are
// one thread per column (serial over rows, as the reference), the row prefix
// is one thread, and the sample table is one thread per texel (two
// lower_bound searches).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_device.h"
#include "pt_kernels.h"

namespace pt {

// lum = 0.2 * R + 0.7 * G + 0.1 * B in double (the reference's double literals), stored as float
__global__ void hdrLumKernel(const float* hdr, float* lum, int n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double R = hdr[3 * (size_t)k], G = hdr[3 * (size_t)k + 1], B = hdr[3 * (size_t)k + 2];
  lum[k] = (float)((0.2 * R + 0.7 * G) + 0.1 * B);
}

// lumSum += lum, k = 0 .. n-1 in order (main.cpp:561-570). A float sum is not
// associative, so only this one dependent chain gives the reference's bits: no
// parallel reduction can. Wave 1 streams the next 4096 values into one LDS
// buffer while lane 0 of wave 0 adds the current buffer's, four values per
// LDS read.
constexpr int SUM_CHUNK = 4096;
__global__ __launch_bounds__(128) void hdrSumKernel(const float* lum, int n, float* out) {
  __shared__ float4 buf[2][SUM_CHUNK / 4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int chunks = (n + SUM_CHUNK - 1) / SUM_CHUNK;
  auto load = [&](int c) {
    float* b = reinterpret_cast<float*>(buf[c & 1]);
    const int base = c * SUM_CHUNK, m = min(SUM_CHUNK, n - base);
    for (int i = lane; i < SUM_CHUNK; i += 64) b[i] = i < m ? lum[base + i] : 0.0f;
  };
  if (w == 1 && chunks > 0) load(0);
  __syncthreads();
  float sum = 0.0f;
  for (int c = 0; c < chunks; c++) {
    if (w == 1 && c + 1 < chunks) {
      load(c + 1);
    } else if (w == 0 && lane == 0) {
      const int m = min(SUM_CHUNK, n - c * SUM_CHUNK);
      const float4* b = buf[c & 1];
      int i = 0;
#pragma unroll 8
      for (; i < m / 4; i++) {
        const float4 v = b[i];
        sum += v.x;
        sum += v.y;
        sum += v.z;
        sum += v.w;
      }
      const float* t = reinterpret_cast<const float*>(b);
      for (int k = 4 * i; k < m; k++) sum += t[k];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sum;
}

// pdf = lum / lumSum (main.cpp:573-575)
__global__ void hdrPdfKernel(float* pdf, int n, const float* lumSum) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  pdf[k] /= *lumSum;
}

// per column j: margin[j] = sum_i pdf[i][j] (rows in order), then the
// conditional CDF over rows, stored column-major cdfY[j * h + i] (main.cpp:578-605)
__global__ void hdrColumnKernel(const float* pdf, int w, int h, float* margin, float* cdfY) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= w) return;
  float m = 0.0f;
  for (int i = 0; i < h; i++) m += pdf[(size_t)i * w + j];
  margin[j] = m;
  float* col = cdfY + (size_t)j * h;
  float acc = 0.0f;
  for (int i = 0; i < h; i++) {
    const float v = pdf[(size_t)i * w + j] / m;
    acc = i == 0 ? v : acc + v;
    col[i] = acc;
  }
}

// cdfX = prefix sum of margin (main.cpp:584-586)
__global__ void hdrRowPrefixKernel(const float* margin, int w, float* cdfX) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  float acc = 0.0f;
  for (int j = 0; j < w; j++) {
    acc = j == 0 ? margin[0] : acc + margin[j];
    cdfX[j] = acc;
  }
}

__device__ __forceinline__ int lowerBound(const float* a, int n, float v) {
  int lo = 0, hi = n;  // first index with !(a[idx] < v)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// sample table (main.cpp:617-640): (x/w, y/h, pdf) per texel; the row CDF index
// is clamped like the host restatement (the reference reads past the end there)
__global__ void hdrSampleKernel(const float* pdf, const float* cdfX, const float* cdfY, int w, int h, float4* cache) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= w * h) return;
  const int i = k / w, j = k - i * w;
  const float xi_1 = (float)i / (float)h;
  const float xi_2 = (float)j / (float)w;
  const int x = lowerBound(cdfX, w, xi_1);
  const int xr = x < w ? x : w - 1;
  const int y = lowerBound(cdfY + (size_t)xr * h, h, xi_2);
  cache[k] = make_float4((float)x / (float)w, (float)y / (float)h, pdf[k], 0.0f);
}

// scratch: 2*w*h + 2*w + 1 floats
// render layout of an env map (pt_kernels.h Env): the pdf (cache.z) joins the
// texel's colour, the sampling table keeps (x, y)
__global__ void envPackKernel(float4* hdr, const float4* cache, float2* samp, int n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const float4 c = cache[k];
  hdr[k].w = c.z;
  samp[k] = make_float2(c.x, c.y);
}

// The compact env texels (pt_kernels.h Env::hdr8 / cache4), each kept only if it decodes to the
// float texel bit for bit with the decoder the frame kernels use (pt_device.h decodeHdr8 /
// decodeCache4); *bad is set otherwise (an env not from a Radiance file, or a sample table not
// from calculateHdrCache) and the float texels stay in use.
__global__ void envCompactKernel(const float4* hdr, const float2* cache, int w, int h, uint2* hdr8, uint32_t* cache4,
                                 int n, int* bad) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const float4 c = hdr[k];
  const float mx = fmaxf(c.x, fmaxf(c.y, c.z));
  bool ok = c.x >= 0.0f && c.y >= 0.0f && c.z >= 0.0f;  // (false for NaN)
  uint32_t word = 0;
  if (ok && mx > 0.0f) {
    int ex;
    (void)frexpf(mx, &ex);  // mx = f * 2^ex, f in [0.5, 1): the largest channel's m in [128, 256)
    const int E = ex + 128;
    ok = E >= 0 && E <= 255;
    if (ok) {
      const float inv = ldexpf(1.0f, 136 - E);  // exact scalings by powers of two
      const float mr = c.x * inv, mg = c.y * inv, mb = c.z * inv;
      ok = mr == floorf(mr) && mg == floorf(mg) && mb == floorf(mb) && mr <= 255.0f && mg <= 255.0f && mb <= 255.0f;
      if (ok) word = (uint32_t)mr | (uint32_t)mg << 8 | (uint32_t)mb << 16 | (uint32_t)E << 24;
    }
  }
  const uint2 t = make_uint2(word, __float_as_uint(c.w));
  const float4 d = decodeHdr8(t);
  ok = ok && __float_as_uint(d.x) == __float_as_uint(c.x) && __float_as_uint(d.y) == __float_as_uint(c.y) &&
       __float_as_uint(d.z) == __float_as_uint(c.z);
  hdr8[k] = t;
  const float2 q = cache[k];
  const float fx = rintf(q.x * (float)w), fy = rintf(q.y * (float)h);
  bool okc = fx >= 0.0f && fx <= 65535.0f && fy >= 0.0f && fy <= 65535.0f;
  const uint32_t v = okc ? ((uint32_t)fx | (uint32_t)fy << 16) : 0u;
  const float2 e = decodeCache4(v, w, h);
  okc = okc && __float_as_uint(e.x) == __float_as_uint(q.x) && __float_as_uint(e.y) == __float_as_uint(q.y);
  cache4[k] = v;
  if (!ok || !okc) atomicOr(bad, 1);
}

hipError_t launchEnvCompact(const float4* hdr, const float2* cache, int w, int h, uint2* hdr8, uint32_t* cache4,
                            int* bad, hipStream_t s) {
  const int n = w * h;
  hipLaunchKernelGGL(envCompactKernel, dim3((n + 255) / 256), dim3(256), 0, s, hdr, cache, w, h, hdr8, cache4, n, bad);
  return hipGetLastError();
}

hipError_t launchEnvPack(float4* hdr, const float4* cache, float2* samp, int n, hipStream_t s) {
  hipLaunchKernelGGL(envPackKernel, dim3((n + 255) / 256), dim3(256), 0, s, hdr, cache, samp, n);
  return hipGetLastError();
}

hipError_t launchHdrCache(const float* hdr, int w, int h, float4* cache, float* scratch, hipStream_t s) {
  const int n = w * h;
  float* pdf = scratch;
  float* cdfY = pdf + n;
  float* margin = cdfY + n;
  float* cdfX = margin + w;
  float* lumSum = cdfX + w;
  const int B = 256;
  hipLaunchKernelGGL(hdrLumKernel, dim3((n + B - 1) / B), dim3(B), 0, s, hdr, pdf, n);
  hipLaunchKernelGGL(hdrSumKernel, dim3(1), dim3(128), 0, s, pdf, n, lumSum);
  hipLaunchKernelGGL(hdrPdfKernel, dim3((n + B - 1) / B), dim3(B), 0, s, pdf, n, lumSum);
  hipLaunchKernelGGL(hdrColumnKernel, dim3((w + 63) / 64), dim3(64), 0, s, pdf, w, h, margin, cdfY);
  hipLaunchKernelGGL(hdrRowPrefixKernel, dim3(1), dim3(1), 0, s, margin, w, cdfX);
  hipLaunchKernelGGL(hdrSampleKernel, dim3((n + B - 1) / B), dim3(B), 0, s, pdf, cdfX, cdfY, w, h, cache);
  return hipGetLastError();
}

}  // namespace pt
