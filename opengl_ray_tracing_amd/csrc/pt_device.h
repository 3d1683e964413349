// pt_device.h -- device-side math, RNG, environment and BRDF for the MI355X
// path tracer. Every function restates one routine of the reference's
// pass1.fsh (cited), in the same float evaluation order as oracle/pt_oracle.c
// so the GPU and the CPU checker round identically wherever the hardware
// operations are correctly rounded (+,-,*,/,sqrt; the build uses
// -ffp-contract=off and IEEE fp32 division/sqrt). Transcendentals come from
// include/pt_fmath.h (explicit-fma polynomials), shared by the CPU checker, so
// they round identically too.
//
// IS = ImportanceSampling_LowDiscrepancySequence/shaders/pass1.fsh,
// D = DisneyBRDF/shaders/pass1.fsh, O = OpenglRayTracing/shaders/pass1.fsh.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_fmath.h"
#include "pt_kernels.h"

#define PT_PI 3.1415926f          // IS:23
#define PT_INF 2147483647.0f      // IS:24 (2^31 in f32)

namespace pt {

struct V3 {
  float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 operator/(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
__device__ __forceinline__ V3 normalize(V3 v) {
  float inv = 1.0f / sqrtf(dot(v, v));
  return v * inv;
}
__device__ __forceinline__ float mixf(float x, float y, float a) { return x * (1.0f - a) + y * a; }
__device__ __forceinline__ V3 mixv(V3 x, V3 y, float a) {
  return v3(mixf(x.x, y.x, a), mixf(x.y, y.y, a), mixf(x.z, y.z, a));
}
__device__ __forceinline__ float sqr(float x) { return x * x; }
__device__ __forceinline__ V3 reflect3(V3 I, V3 N) {
  float k = 2.0f * dot(N, I);
  return I - N * k;
}
__device__ __forceinline__ V3 ld3(const float* p) { return v3(p[0], p[1], p[2]); }

// ------------------------------------------------------------------ RNG
// wang_hash IS:78-85
__device__ __forceinline__ uint32_t wang(uint32_t& s) {
  uint32_t x = s;
  x = (x ^ 61u) ^ (x >> 16);
  x *= 9u;
  x = x ^ (x >> 4);
  x *= 0x27d4eb2du;
  x = x ^ (x >> 15);
  s = x;
  return x;
}
// rand IS:87-89
__device__ __forceinline__ float randf(uint32_t& s) { return (float)wang(s) / 4294967296.0f; }

// Sobol direction numbers IS:92-94 (8 dims x 32), in constant memory (one copy per
// translation unit).
static __constant__ uint32_t kSobolV[8 * 32] = {
    2147483648u,1073741824u,536870912u,268435456u,134217728u,67108864u,33554432u,16777216u,8388608u,4194304u,2097152u,1048576u,524288u,262144u,131072u,65536u,32768u,16384u,8192u,4096u,2048u,1024u,512u,256u,128u,64u,32u,16u,8u,4u,2u,1u,
    2147483648u,3221225472u,2684354560u,4026531840u,2281701376u,3422552064u,2852126720u,4278190080u,2155872256u,3233808384u,2694840320u,4042260480u,2290614272u,3435921408u,2863267840u,4294901760u,2147516416u,3221274624u,2684395520u,4026593280u,2281736192u,3422604288u,2852170240u,4278255360u,2155905152u,3233857728u,2694881440u,4042322160u,2290649224u,3435973836u,2863311530u,4294967295u,
    2147483648u,3221225472u,1610612736u,2415919104u,3892314112u,1543503872u,2382364672u,3305111552u,1753219072u,2629828608u,3999268864u,1435500544u,2154299392u,3231449088u,1626210304u,2421489664u,3900735488u,1556135936u,2388680704u,3314585600u,1751705600u,2627492864u,4008611328u,1431684352u,2147543168u,3221249216u,1610649184u,2415969680u,3892340840u,1543543964u,2382425838u,3305133397u,
    2147483648u,3221225472u,536870912u,1342177280u,4160749568u,1946157056u,2717908992u,2466250752u,3632267264u,624951296u,1507852288u,3872391168u,2013790208u,3020685312u,2181169152u,3271884800u,546275328u,1363623936u,4226424832u,1977167872u,2693105664u,2437829632u,3689389568u,635137280u,1484783744u,3846176960u,2044723232u,3067084880u,2148008184u,3222012020u,537002146u,1342505107u,
    2147483648u,1073741824u,536870912u,2952790016u,4160749568u,3690987520u,2046820352u,2634022912u,1518338048u,801112064u,2707423232u,4038066176u,3666345984u,1875116032u,2170683392u,1085997056u,579305472u,3016343552u,4217741312u,3719483392u,2013407232u,2617981952u,1510979072u,755882752u,2726789248u,4090085440u,3680870432u,1840435376u,2147625208u,1074478300u,537900666u,2953698205u,
    2147483648u,1073741824u,1610612736u,805306368u,2818572288u,335544320u,2113929216u,3472883712u,2290089984u,3829399552u,3059744768u,1127219200u,3089629184u,4199809024u,3567124480u,1891565568u,394297344u,3988799488u,920674304u,4193267712u,2950604800u,3977188352u,3250028032u,129093376u,2231568512u,2963678272u,4281226848u,432124720u,803643432u,1633613396u,2672665246u,3170194367u,
    2147483648u,3221225472u,2684354560u,3489660928u,1476395008u,2483027968u,1040187392u,3808428032u,3196059648u,599785472u,505413632u,4077912064u,1182269440u,1736704000u,2017853440u,2221342720u,3329785856u,2810494976u,3628507136u,1416089600u,2658719744u,864310272u,3863387648u,3076993792u,553150080u,272922560u,4167467040u,1148698640u,1719673080u,2009075780u,2149644390u,3222291575u,
    2147483648u,1073741824u,2684354560u,1342177280u,2281701376u,1946157056u,436207616u,2566914048u,2625634304u,3208642560u,2720006144u,2098200576u,111673344u,2354315264u,3464626176u,4027383808u,2886631424u,3770826752u,1691164672u,3357462528u,1993345024u,3752330240u,873073152u,2870150400u,1700563072u,87021376u,1097028000u,1222351248u,1560027592u,2977959924u,23268898u,437609937u};

// sobol IS:101-109 with the documented dims >= 8 extension (oracle: sobol_bits)
__device__ __forceinline__ float sobolf(uint32_t d, uint32_t i) {
  uint32_t result = 0;
  const uint32_t* V = kSobolV + (d & 7u) * 32u;
  for (uint32_t j = 0; i != 0; i >>= 1, j++)
    if ((i & 1u) != 0) result ^= V[j];
  if (d >= 8u) {
    uint32_t h = d;
    result ^= wang(h);
  }
  return (float)result * (1.0f / (float)0xFFFFFFFFu);
}
__device__ __forceinline__ uint32_t grayCode(uint32_t i) { return i ^ (i >> 1); }

// CranleyPattersonRotation IS:118-136
// split into the per-pixel shift (constant across bounces and frames) and its
// application, so a path computes the shift once
__device__ __forceinline__ void cranleyPattersonShift(int px, int py, float& u, float& v) {
  uint32_t pseed = ((uint32_t)px * 1973u + (uint32_t)py * 9277u + 59u * 26699u) | 1u;
  u = (float)wang(pseed) / 4294967296.0f;
  v = (float)wang(pseed) / 4294967296.0f;
}
__device__ __forceinline__ void cranleyPattersonApply(float u, float v, float& u_, float& v_) {
  float x = u_ + u;
  if (x > 1.0f) x -= 1.0f;
  if (x < 0.0f) x += 1.0f;
  float y = v_ + v;
  if (y > 1.0f) y -= 1.0f;
  if (y < 0.0f) y += 1.0f;
  u_ = x;
  v_ = y;
}
__device__ __forceinline__ void cranleyPatterson(int px, int py, float& u_, float& v_) {
  float u, v;
  cranleyPattersonShift(px, py, u, v);
  cranleyPattersonApply(u, v, u_, v_);
}

// ------------------------------------------------------------ material
struct Material {  // IS:41-56
  V3 emissive, baseColor;
  float subsurface, metallic, specular, specularTint, roughness, anisotropic;
  float sheen, sheenTint, clearcoat, clearcoatGloss;
};
// getMaterial IS:207-232 from floats 16..35 of a Triangle_encoded record (5 float4)
__device__ __forceinline__ Material loadMaterial(const float4* q) {
  float4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
  // floats: 16 17 18 | 19 20 21 | 22 23 24 | 25 26 27 | 28 29 30 | 31 32 33 | 34 35
  // emissive = 18,19,20; baseColor = 21,22,23; param1 = 24..26; param2 = 27..29; param3 = 30..32; param4 = 33..35
  Material m;
  m.emissive = v3(a.z, a.w, b.x);
  m.baseColor = v3(b.y, b.z, b.w);
  m.subsurface = c.x; m.metallic = c.y; m.specular = c.z;
  m.specularTint = c.w; m.roughness = d.x; m.anisotropic = d.y;
  m.sheen = d.z; m.sheenTint = d.w; m.clearcoat = e.x;
  m.clearcoatGloss = e.y;
  return m;
}

// ------------------------------------------------------------ environment
// Streaming (non-temporal) loads and stores for the env map and the
// accumulation buffer: their lines are touched about once per frame, so they
// are marked to leave L2 first and not evict the BVH and triangle lines every
// traversal re-reads (PT_NT_STREAM=0: plain accesses).
#ifndef PT_NT_STREAM
#define PT_NT_STREAM 1
#endif
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 ldStream(const float4* p) {
#if PT_NT_STREAM
  const f32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}
__device__ __forceinline__ float2 ldStream(const float2* p) {
#if PT_NT_STREAM
  const f32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const f32x2_t*>(p));
  return make_float2(v.x, v.y);
#else
  return *p;
#endif
}
// a pipelined frame's sample colour: COL_F = 3 floats per pixel (alpha is always 1, IS:871), 12 bytes
// written by the frame kernel and read once by mixKernel (16 until round 6: c2 33 -> 25 MB each way)
__device__ __forceinline__ void stCol(float* p, float r, float g, float b) {
#if PT_DIAG_NO_STORE
  if (r != -1234.5f) return;
#endif
#if PT_NT_STREAM
  __builtin_nontemporal_store(r, p);
  __builtin_nontemporal_store(g, p + 1);
  __builtin_nontemporal_store(b, p + 2);
#else
  p[0] = r;
  p[1] = g;
  p[2] = b;
#endif
}
__device__ __forceinline__ float3 ldCol(const float* p) {
#if PT_NT_STREAM
  return make_float3(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1), __builtin_nontemporal_load(p + 2));
#else
  return make_float3(p[0], p[1], p[2]);
#endif
}
__device__ __forceinline__ void stStream(float4* p, float4 v) {
#if PT_DIAG_NO_STORE  // diagnostics build (traffic attribution): colours almost never stored
  if (v.x != -1234.5f) return;
#endif
#if PT_NT_STREAM
  const f32x4_t x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<f32x4_t*>(p));
#else
  *p = v;
#endif
}

// GL_NEAREST + GL_CLAMP_TO_EDGE addressing (OpenglRayTracing/main.cpp:184-194): the texel of (u, v)
__device__ __forceinline__ void texXY(int w, int h, float u, float v, int& x, int& y) {
  float fx = floorf(u * (float)w);
  float fy = floorf(v * (float)h);
  fx = fminf(fmaxf(fx, 0.0f), (float)(w - 1));
  fy = fminf(fmaxf(fy, 0.0f), (float)(h - 1));
  x = (int)fx;
  y = (int)fy;
}
__device__ __forceinline__ int texIndex(int w, int h, float u, float v) {
  int x, y;
  texXY(w, h, u, v, x, y);
  return y * w + x;
}
template <class T>
__device__ __forceinline__ T texNearest(const T* img, int w, int h, float u, float v) {
  return ldStream(img + texIndex(w, h, u, v));
}
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 ldStream(const uint2* p) {
#if PT_NT_STREAM
  const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(p));
  return make_uint2(v.x, v.y);
#else
  return *p;
#endif
}
__device__ __forceinline__ uint32_t ldStream(const uint32_t* p) {
#if PT_NT_STREAM
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
// the compact env texels (pt_kernels.h Env): RGBE channels m * 2^(E - 136) -- exact products of an
// integer below 256 and a power of two -- and the pdf's own bits; the sample table's float(x) / w,
// float(y) / h with IEEE division, as calculateHdrCache computes them (IS main.cpp:630-631)
__device__ __forceinline__ float4 decodeHdr8(uint2 t) {
  const float sc = ldexpf(1.0f, (int)(t.x >> 24) - 136);
  return make_float4((float)(t.x & 255u) * sc, (float)((t.x >> 8) & 255u) * sc, (float)((t.x >> 16) & 255u) * sc,
                     __uint_as_float(t.y));
}
__device__ __forceinline__ float2 decodeCache4(uint32_t v, int w, int h) {
  return make_float2((float)(v & 0xffffu) / (float)w, (float)(v >> 16) / (float)h);
}
// the env texel (r, g, b, pdf) of (u, v), from the compact or the float4 texels
// PT_DIAG_ENV_SMALL (diagnostics builds, traffic attribution): bit 0 keeps every env texel read, bit 1
// every sample-table read, within the first 1024 texels
#ifndef PT_DIAG_ENV_SMALL
#define PT_DIAG_ENV_SMALL 0
#endif
__device__ __forceinline__ float4 envTexelK(const Env& e, int k) {
  k &= (PT_DIAG_ENV_SMALL & 1) ? 1023 : -1;
  if (e.nt) return e.hdr8 ? decodeHdr8(ldStream(e.hdr8 + k)) : ldStream(e.hdr + k);
  return e.hdr8 ? decodeHdr8(e.hdr8[k]) : e.hdr[k];
}
__device__ __forceinline__ float4 envTexel(const Env& e, float u, float v) { return envTexelK(e, texIndex(e.w, e.h, u, v)); }
// SampleSphericalMap IS:175-181 / toSphericalCoord IS:638-644
__device__ __forceinline__ void toSpherical(V3 v, float& u, float& w) {
  float a = ptm_atan2f(v.z, v.x), b = ptm_asinf(v.y);
  a = a / (2.0f * PT_PI);
  b = b / PT_PI;
  a = a + 0.5f;
  b = b + 0.5f;
  u = a;
  w = 1.0f - b;
}
// The texel of toSpherical(v) (v normalized) under GL_NEAREST / CLAMP_TO_EDGE, as computed with the
// correctly rounded atan2 / asin -- decided by their float approximations (include/pt_fmath.h
// ptm_*_fast, at most 4 / 3 ulp) whenever the approximate texel coordinates lie farther from a
// texel edge than the approximation can move them (4e-7 of the map's size: the bound from those ulps
// through toSpherical's float operations is 3e-7, the largest difference measured over 4e6 random
// directions 1.2e-7), else by the correctly rounded functions themselves. The same texel either way;
// c2's sky lookups (every camera ray and bounce ray that escapes) at the float functions' cost
// (c2 0.189 -> ~0.174 ms per frame)
// (the correctly rounded fallback: a call, so its double-precision registers are not the caller's)
__device__ __noinline__ int sphTexelExact(int W, int H, V3 v) {
  float u, w;
  toSpherical(v, u, w);
  return texIndex(W, H, u, w);
}
__device__ __forceinline__ int sphTexel(int W, int H, V3 v) {
  float a = ptm_atan2f_fast(v.z, v.x), b = ptm_asinf_fast(v.y);
  a = a / (2.0f * PT_PI);
  b = b / PT_PI;
  a = a + 0.5f;
  b = b + 0.5f;
  const float fx = a * (float)W, fy = (1.0f - b) * (float)H;
  if (fabsf(fx - rintf(fx)) > 4e-7f * (float)W && fabsf(fy - rintf(fy)) > 4e-7f * (float)H) {
    const int x = (int)fminf(fmaxf(floorf(fx), 0.0f), (float)(W - 1));
    const int y = (int)fminf(fmaxf(floorf(fy), 0.0f), (float)(H - 1));
    return y * W + x;
  }
  return sphTexelExact(W, H, v);
}
// sampleHdr IS:184-189 (clamped at 10)
__device__ __forceinline__ V3 sampleHdr(const Env& e, V3 v) {
  if (!e.hdr) return v3(0, 0, 0);
  float4 c = envTexelK(e, sphTexel(e.w, e.h, normalize(v)));
  return v3(fminf(c.x, 10.0f), fminf(c.y, 10.0f), fminf(c.z, 10.0f));
}
// hdrColor IS:647-651 (unclamped)
__device__ __forceinline__ V3 hdrColor(const Env& e, V3 L) {
  if (!e.hdr) return v3(0, 0, 0);
  float u, w;
  toSpherical(normalize(L), u, w);
  float4 c = envTexel(e, u, w);
  return v3(c.x, c.y, c.z);
}
// SampleHdr IS:573-585, in two parts: the cache texel of (xi1, xi2) and the
// direction it encodes (split so a caller can issue the fetch early)
__device__ __forceinline__ float2 hdrCacheTexel(const Env& e, float xi1, float xi2) {
  if (!e.cache) return make_float2(0.0f, 0.0f);
  if (e.cacheRow) {  // the row form (Env::cacheRow): the same entry, as decodeCache4 decodes it
    int col, row;
    texXY(e.w, e.h, xi1, xi2, col, row);
    const uint32_t r = e.cacheRow[row];
    const uint32_t y = e.cacheY[(size_t)(r >> 16) * e.w + (col & ((PT_DIAG_ENV_SMALL & 2) ? 1023 : -1))];
    return decodeCache4((r & 0xffffu) | y << 16, e.w, e.h);
  }
  const int k = texIndex(e.w, e.h, xi1, xi2) & ((PT_DIAG_ENV_SMALL & 2) ? 1023 : -1);
  if (e.nt) return e.cache4 ? decodeCache4(ldStream(e.cache4 + k), e.w, e.h) : ldStream(e.cache + k);
  return e.cache4 ? decodeCache4(e.cache4[k], e.w, e.h) : e.cache[k];
}
// SampleHdr's angles of a sample-table entry (x, y), IS:576-580
__device__ __forceinline__ float hdrTheta(float y) { return PT_PI * ((1.0f - y) - 0.5f); }
__device__ __forceinline__ float hdrPhi(float x) { return 2.0f * PT_PI * (x - 0.5f); }
__device__ __forceinline__ V3 hdrDirFromCache(float2 c) {
  float st, ct, sp, cp;
  ptm_sincosf(hdrTheta(c.y), &st, &ct);
  ptm_sincosf(hdrPhi(c.x), &sp, &cp);
  return v3(ct * cp, st, ct * sp);  // IS:583
}
__device__ __forceinline__ V3 sampleHdrDir(const Env& e, float xi1, float xi2, int* entry = nullptr) {
  // A compact sample table's entries are integers over (w, h) (decodeCache4), so SampleHdr's sines
  // and cosines take w + h values: Env::trig holds them (envTrigKernel, the same functions of the
  // same floats), one 8-byte load per angle instead of a double-precision sincos each
  if (e.trig && (e.cacheRow || e.cache4)) {
    int col, row;
    texXY(e.w, e.h, xi1, xi2, col, row);
    uint32_t v;
    if (e.cacheRow) {
      const uint32_t r = e.cacheRow[row];
      v = (r & 0xffffu) | (uint32_t)e.cacheY[(size_t)(r >> 16) * e.w + col] << 16;
    } else {
      const int k = row * e.w + col;
      v = e.nt ? ldStream(e.cache4 + k) : e.cache4[k];
    }
    const float2 t = e.trig[v >> 16], f = e.trig[e.h + 1 + (v & 0xffffu)];
    if (entry) *entry = (int)(v >> 16) * (e.w + 1) + (int)(v & 0xffffu);
    return v3(t.y * f.y, t.x, t.y * f.x);
  }
  if (entry) *entry = -1;
  return hdrDirFromCache(hdrCacheTexel(e, xi1, xi2));
}
// hdrPdf IS:655-666 (sin of the elevation: reference quirk kept)
__device__ __forceinline__ float hdrPdf(const Env& e, V3 L) {
  float u, w;
  toSpherical(normalize(L), u, w);
  float pdf = e.hdr ? envTexel(e, u, w).w : 0.0f;
  float theta = PT_PI * (0.5f - w);
  float sin_theta = fmaxf(ptm_sinf(theta), 1e-10f);
  float p_convert = (float)(e.res * e.res / 2) / (2.0f * PT_PI * PT_PI * sin_theta);
  return pdf * p_convert;
}

// hdrColor(L) and hdrPdf(L) of the same direction (every MIS use pairs them):
// one toSphericalCoord, the same operations and results as the two calls.
// Split in two like sampleHdrDir: the texel of L (and the elevation coordinate
// w its pdf needs), then color and pdf from them.
__device__ __forceinline__ float4 hdrTexelOf(const Env& e, V3 L, float& w) {
  float u;
  toSpherical(normalize(L), u, w);
  return e.hdr ? envTexel(e, u, w) : make_float4(0, 0, 0, 0);
}
__device__ __forceinline__ void hdrColorPdfOf(const Env& e, float4 c, float w, V3& color, float& pdf) {
  color = v3(c.x, c.y, c.z);
  const float p = c.w;  // the cache pdf of the same texel
  const float theta = PT_PI * (0.5f - w);
  const float sin_theta = fmaxf(ptm_sinf(theta), 1e-10f);
  const float p_convert = (float)(e.res * e.res / 2) / (2.0f * PT_PI * PT_PI * sin_theta);
  pdf = p * p_convert;
}
// (a call: the correctly rounded atan2 / asin / sin in double precision stay out of the MIS kernels'
// register allocation -- c5's MIS regen kernel spilled 8 VGPRs with them inlined. Arguments and result
// by value: an Env or an output passed by reference would live in scratch memory.)
__device__ __noinline__ float4 hdrColorPdfCall(const uint2* hdr8, const float4* hdr, int w, int h, int res, int nt,
                                              V3 L) {
  Env e;
  e.hdr8 = hdr8;
  e.hdr = hdr;
  e.w = w;
  e.h = h;
  e.res = res;
  e.nt = nt;
  float wv;
  const float4 c = hdrTexelOf(e, L, wv);
  V3 color;
  float pdf;
  hdrColorPdfOf(e, c, wv, color, pdf);
  return make_float4(color.x, color.y, color.z, pdf);
}
__device__ __forceinline__ void hdrColorPdf(const Env& e, V3 L, V3& color, float& pdf) {
  const float4 r = hdrColorPdfCall(e.hdr8, e.hdr, e.w, e.h, e.res, e.nt, L);
  color = v3(r.x, r.y, r.z);
  pdf = r.w;
}
// hdrColor and hdrPdf of a light sample's direction (IS:778-779): from Env::light when the sample
// came from a compact table's entry (sampleHdrDir's *entry) -- the texel's RGBE and the finished pdf,
// computed at upload by envLightKernel with the operations below -- else computed
__device__ __forceinline__ void hdrLightColorPdf(const Env& e, int entry, V3 L, V3& color, float& pdf) {
  if (entry >= 0 && e.light) {
    const float4 c = decodeHdr8(e.nt ? ldStream(e.light + entry) : e.light[entry]);
    color = v3(c.x, c.y, c.z);
    pdf = c.w;
    return;
  }
  hdrColorPdf(e, L, color, pdf);
}

// ------------------------------------------------------------ BRDF IS:386-711
__device__ __forceinline__ float SchlickFresnel(float u) {
  float m = fminf(fmaxf(1.0f - u, 0.0f), 1.0f);
  float m2 = m * m;
  return m2 * m2 * m;
}
__device__ __forceinline__ float GTR1(float NdotH, float a) {
  if (a >= 1.0f) return 1.0f / PT_PI;
  float a2 = a * a;
  float t = 1.0f + (a2 - 1.0f) * NdotH * NdotH;
  return (a2 - 1.0f) / (PT_PI * ptm_logf(a2) * t);
}
__device__ __forceinline__ float GTR2(float NdotH, float a) {
  float a2 = a * a;
  float t = 1.0f + (a2 - 1.0f) * NdotH * NdotH;
  return a2 / (PT_PI * t * t);
}
__device__ __forceinline__ float GTR2_aniso(float NdotH, float HdotX, float HdotY, float ax, float ay) {
  return 1.0f / (PT_PI * ax * ay * sqr(sqr(HdotX / ax) + sqr(HdotY / ay) + NdotH * NdotH));
}
__device__ __forceinline__ float smithG_GGX(float NdotV, float alphaG) {
  float a = alphaG * alphaG;
  float b = NdotV * NdotV;
  return 1.0f / (NdotV + sqrtf(a + b - a * b));
}
__device__ __forceinline__ float smithG_GGX_aniso(float NdotV, float VdotX, float VdotY, float ax, float ay) {
  return 1.0f / (NdotV + sqrtf(sqr(VdotX * ax) + sqr(VdotY * ay) + sqr(NdotV)));
}
struct Tints {
  V3 Cdlin, Cspec0, Csheen;
};
__device__ __forceinline__ Tints tints(const Material& m) {
  Tints t;
  V3 Cdlin = m.baseColor;
  float Cdlum = 0.3f * Cdlin.x + 0.6f * Cdlin.y + 0.1f * Cdlin.z;
  V3 Ctint = (Cdlum > 0.0f) ? Cdlin / Cdlum : v3(1, 1, 1);
  V3 Cspec = mixv(v3(1, 1, 1), Ctint, m.specularTint) * m.specular;
  t.Cdlin = Cdlin;
  t.Cspec0 = mixv(Cspec * 0.08f, Cdlin, m.metallic);
  t.Csheen = mixv(v3(1, 1, 1), Ctint, m.sheenTint);
  return t;
}
// BRDF_Evaluate_aniso IS:423-482 == D:381-440
__device__ __forceinline__ V3 brdfAniso(V3 V, V3 N, V3 L, V3 X, V3 Y, const Material& m) {
  float NdotL = dot(N, L);
  float NdotV = dot(N, V);
  if (NdotL < 0 || NdotV < 0) return v3(0, 0, 0);
  V3 H = normalize(L + V);
  float NdotH = dot(N, H);
  float LdotH = dot(L, H);
  Tints tt = tints(m);
  float Fd90 = 0.5f + 2.0f * LdotH * LdotH * m.roughness;
  float FL = SchlickFresnel(NdotL);
  float FV = SchlickFresnel(NdotV);
  float Fd = mixf(1.0f, Fd90, FL) * mixf(1.0f, Fd90, FV);
  float Fss90 = LdotH * LdotH * m.roughness;
  float Fss = mixf(1.0f, Fss90, FL) * mixf(1.0f, Fss90, FV);
  float ss = 1.25f * (Fss * (1.0f / (NdotL + NdotV) - 0.5f) + 0.5f);
  float aspect = sqrtf(1.0f - m.anisotropic * 0.9f);
  float ax = fmaxf(0.001f, sqr(m.roughness) / aspect);
  float ay = fmaxf(0.001f, sqr(m.roughness) * aspect);
  float Ds = GTR2_aniso(NdotH, dot(H, X), dot(H, Y), ax, ay);
  float FH = SchlickFresnel(LdotH);
  V3 Fs = mixv(tt.Cspec0, v3(1, 1, 1), FH);
  float Gs = smithG_GGX_aniso(NdotL, dot(L, X), dot(L, Y), ax, ay);
  Gs *= smithG_GGX_aniso(NdotV, dot(V, X), dot(V, Y), ax, ay);
  V3 specular = (Fs * Gs) * Ds;
  float Dr = GTR1(NdotH, mixf(0.1f, 0.001f, m.clearcoatGloss));
  float Fr = mixf(0.04f, 1.0f, FH);
  float Gr = smithG_GGX(NdotL, 0.25f) * smithG_GGX(NdotV, 0.25f);
  float cc = 0.25f * Gr * Fr * Dr * m.clearcoat;
  V3 Fsheen = tt.Csheen * (FH * m.sheen);
  float kd = (1.0f / PT_PI) * mixf(Fd, ss, m.subsurface);
  V3 diffuse = tt.Cdlin * kd + Fsheen;
  V3 r = diffuse * (1.0f - m.metallic) + specular;
  return r + v3(cc, cc, cc);
}
// BRDF_Evaluate IS:587-636
__device__ __forceinline__ V3 brdfIso(V3 V, V3 N, V3 L, const Material& m) {
  float NdotL = dot(N, L);
  float NdotV = dot(N, V);
  if (NdotL < 0 || NdotV < 0) return v3(0, 0, 0);
  V3 H = normalize(L + V);
  float NdotH = dot(N, H);
  float LdotH = dot(L, H);
  Tints tt = tints(m);
  float Fd90 = 0.5f + 2.0f * LdotH * LdotH * m.roughness;
  float FL = SchlickFresnel(NdotL);
  float FV = SchlickFresnel(NdotV);
  float Fd = mixf(1.0f, Fd90, FL) * mixf(1.0f, Fd90, FV);
  float Fss90 = LdotH * LdotH * m.roughness;
  float Fss = mixf(1.0f, Fss90, FL) * mixf(1.0f, Fss90, FV);
  float ss = 1.25f * (Fss * (1.0f / (NdotL + NdotV) - 0.5f) + 0.5f);
  float alpha = fmaxf(0.001f, sqr(m.roughness));
  float Ds = GTR2(NdotH, alpha);
  float FH = SchlickFresnel(LdotH);
  V3 Fs = mixv(tt.Cspec0, v3(1, 1, 1), FH);
  float Gs = smithG_GGX(NdotL, m.roughness);
  Gs *= smithG_GGX(NdotV, m.roughness);
  float Dr = GTR1(NdotH, mixf(0.1f, 0.001f, m.clearcoatGloss));
  float Fr = mixf(0.04f, 1.0f, FH);
  float Gr = smithG_GGX(NdotL, 0.25f) * smithG_GGX(NdotV, 0.25f);
  V3 Fsheen = tt.Csheen * (FH * m.sheen);
  float kd = (1.0f / PT_PI) * mixf(Fd, ss, m.subsurface);
  V3 diffuse = tt.Cdlin * kd + Fsheen;
  V3 specular = (Fs * Gs) * Ds;
  float cc = 0.25f * Gr * Fr * Dr * m.clearcoat;
  V3 r = diffuse * (1.0f - m.metallic) + specular;
  return r + v3(cc, cc, cc);
}
// BRDF_Pdf IS:669-706
__device__ __forceinline__ float brdfPdf(V3 V, V3 N, V3 L, const Material& m) {
  float NdotL = dot(N, L);
  float NdotV = dot(N, V);
  if (NdotL < 0 || NdotV < 0) return 0.0f;
  V3 H = normalize(L + V);
  float NdotH = dot(N, H);
  float LdotH = dot(L, H);
  float alpha = fmaxf(0.001f, sqr(m.roughness));
  float Ds = GTR2(NdotH, alpha);
  float Dr = GTR1(NdotH, mixf(0.1f, 0.001f, m.clearcoatGloss));
  float pdf_diffuse = NdotL / PT_PI;
  float pdf_specular = Ds * NdotH / (4.0f * LdotH);
  float pdf_clearcoat = Dr * NdotH / (4.0f * LdotH);
  float r_diffuse = 1.0f - m.metallic;
  float r_specular = 1.0f;
  float r_clearcoat = 0.25f * m.clearcoat;
  float r_sum = r_diffuse + r_specular + r_clearcoat;
  float p_diffuse = r_diffuse / r_sum;
  float p_specular = r_specular / r_sum;
  float p_clearcoat = r_clearcoat / r_sum;
  float pdf = p_diffuse * pdf_diffuse + p_specular * pdf_specular + p_clearcoat * pdf_clearcoat;
  return fmaxf(1e-10f, pdf);
}
__device__ __forceinline__ float misWeight(float a, float b) {  // IS:708-711
  float t = a * a;
  return t / (b * b + t);
}
// toNormalHemisphere IS:153-159
__device__ __forceinline__ V3 toNormalHemisphere(V3 v, V3 N) {
  V3 helper = v3(1, 0, 0);
  if (fabsf(N.x) > 0.999f) helper = v3(0, 0, 1);
  V3 tangent = normalize(cross(N, helper));
  V3 bitangent = normalize(cross(N, tangent));
  return (tangent * v.x + bitangent * v.y) + N * v.z;
}
// getTangent IS:161-172 (swapped naming kept)
__device__ __forceinline__ void getTangent(V3 N, V3& tangent, V3& bitangent) {
  V3 helper = v3(1, 0, 0);
  if (fabsf(N.x) > 0.999f) helper = v3(0, 0, 1);
  bitangent = normalize(cross(N, helper));
  tangent = normalize(cross(N, bitangent));
}
// SampleHemisphere D:90-95
__device__ __forceinline__ V3 sampleHemisphereRand(uint32_t& seed) {
  float z = randf(seed);
  float r = fmaxf(0.0f, sqrtf(1.0f - z * z));
  float phi = 2.0f * PT_PI * randf(seed);
  float s, c;
  ptm_sincosf(phi, &s, &c);  // the same bits as ptm_sinf / ptm_cosf, one range reduction
  return v3(r * c, r * s, z);
}
// SampleCosineHemisphere IS:485-496
__device__ __forceinline__ V3 sampleCosine(float xi_1, float xi_2, V3 N) {
  float r = sqrtf(xi_1);
  float theta = xi_2 * 2.0f * PT_PI;
  float st, ct;
  ptm_sincosf(theta, &st, &ct);
  float x = r * ct;
  float y = r * st;
  float z = sqrtf(1.0f - x * x - y * y);
  return toNormalHemisphere(v3(x, y, z), N);
}
// SampleGTR2 IS:499-516 / SampleGTR1 IS:519-536
__device__ __forceinline__ V3 sampleGTR(float xi_1, float xi_2, V3 V, V3 N, float alpha, bool gtr1) {
  float phi_h = 2.0f * PT_PI * xi_1;
  float sin_phi_h, cos_phi_h;
  ptm_sincosf(phi_h, &sin_phi_h, &cos_phi_h);
  float cos_theta_h;
  if (gtr1)
    cos_theta_h = sqrtf((1.0f - ptm_powf(alpha * alpha, 1.0f - xi_2)) / (1.0f - alpha * alpha));
  else
    cos_theta_h = sqrtf((1.0f - xi_2) / (1.0f + (alpha * alpha - 1.0f) * xi_2));
  float sin_theta_h = sqrtf(fmaxf(0.0f, 1.0f - cos_theta_h * cos_theta_h));
  V3 H = v3(sin_theta_h * cos_phi_h, sin_theta_h * sin_phi_h, cos_theta_h);
  H = toNormalHemisphere(H, N);
  return reflect3(-V, H);
}
// SampleBRDF IS:539-570
__device__ __forceinline__ V3 sampleBRDF(float xi_1, float xi_2, float xi_3, V3 V, V3 N, const Material& m) {
  float alpha_GTR1 = mixf(0.1f, 0.001f, m.clearcoatGloss);
  float alpha_GTR2 = fmaxf(0.001f, sqr(m.roughness));
  float r_diffuse = 1.0f - m.metallic;
  float r_specular = 1.0f;
  float r_clearcoat = 0.25f * m.clearcoat;
  float r_sum = r_diffuse + r_specular + r_clearcoat;
  float p_diffuse = r_diffuse / r_sum;
  float p_specular = r_specular / r_sum;
  float rd = xi_3;
  if (rd <= p_diffuse) return sampleCosine(xi_1, xi_2, N);
  if (p_diffuse < rd && rd <= p_diffuse + p_specular) return sampleGTR(xi_1, xi_2, V, N, alpha_GTR2, false);
  if (p_diffuse + p_specular < rd) return sampleGTR(xi_1, xi_2, V, N, alpha_GTR1, true);
  return v3(0, 1, 0);
}

}  // namespace pt
