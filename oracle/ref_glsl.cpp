// ref_glsl.cpp -- TEST INFRASTRUCTURE ONLY: the reference's three per-pixel
// kernels (the pass1.fsh fragment shaders) compiled from their own GLSL text as
// C++ over the reference's vendored glm, so the oracle's restatement
// (oracle/pt_oracle.c) can be compared with the reference's code itself --
// function by function on random inputs and frame by frame through each
// shader's own main() (tests/test_glsl_ref.py, tests/golden/glsl/).
//
// oracle/ref_build.py copies each shader, from line 3 (after `#version`) to the
// end, into oracle/_ref/{o,d,is}_pass1.inc with ONE textual rule applied:
// a GLSL `inout T name` parameter becomes `T& name` (3 sites in IS and D, 1 in O:
// wang_hash and getTangent), since C++ has no spelling of a by-reference
// parameter that a macro in front of the type can produce. Every other token is
// the reference's. Each extract is included inside a struct (below), so the
// shader's globals (`in`, `uniform`, the `seed` initialiser of IS:73-76) become
// per-fragment members and its functions member functions.
//
// What this file supplies is the GLSL language and the GL pipeline around the
// text, each piece stated here:
//  * qualifiers: `in`, `out`, `uniform` expand to nothing (inputs, outputs and
//    uniforms become members set per fragment by the constructor);
//  * literals: clang with -cl-single-precision-constant, so 0.5 and 3.1415926 are
//    float literals as in GLSL (4.30 spec 4.1.4); the evaluation of a call's
//    arguments is left to right as in GLSL (5.9) -- clang's order on x86-64,
//    checked at load (ref_glsl_selfcheck);
//  * GLSL's implicit int -> float conversion in built-in calls (4.1.10):
//    max(int, float), max(float, int), clamp(float, int, int);
//  * swizzles: glm's swizzle operators (GLM_FORCE_SWIZZLE) for pix.xy / dir.xyz,
//    a texel type with xyz / rgb / rg / b members for texture results;
//  * texelFetch(samplerBuffer, i): texel i of a GL_RGB32F buffer as (r, g, b, 1);
//    texture2D(sampler2D, uv): GL_NEAREST + GL_CLAMP_TO_EDGE (the reference's
//    sampler state, OpenglRayTracing/main.cpp:184-194): texel (floor(u w),
//    floor(v h)) clamped to the image, row 0 = the first row uploaded;
//  * the transcendental built-ins (sin, cos, atan(y, x), asin, log, pow) bound to
//    include/pt_fmath.h: GLSL leaves their precision to the GL driver, which is
//    not in the reference; this build defines them there for the oracle and the
//    GPU alike, so the comparison isolates everything else. sqrt, / and the
//    rest are IEEE (-ffp-contract=off);
//  * pix, the vertex shader's NDC position (vshader.vsh:7-10) interpolated to the
//    fragment centre, as the oracle forms it: (2 px + 1) / w - 1 in float.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>

#define GLM_FORCE_SWIZZLE
#include <glm/glm.hpp>

#include "pt_fmath.h"

using namespace glm;

namespace glsl {

struct samplerBuffer {
  const float* t = nullptr;  // GL_RGB32F texels
  int n = 0;
};
struct sampler2D {
  const float* t = nullptr;
  int w = 0, h = 0, comps = 3;  // GL_RGB32F (3) or GL_RGBA32F (4)
};
struct texel {
  vec3 xyz, rgb;
  vec2 rg;
  float b;
};
inline texel mk(float r, float g, float b, float a) {
  (void)a;
  texel t;
  t.xyz = t.rgb = vec3(r, g, b);
  t.rg = vec2(r, g);
  t.b = b;
  return t;
}
inline texel texelFetch(const samplerBuffer& s, int i) {
  if (i < 0 || i >= s.n) return mk(0, 0, 0, 0);
  return mk(s.t[3 * (size_t)i], s.t[3 * (size_t)i + 1], s.t[3 * (size_t)i + 2], 1.0f);
}
inline texel texture2D(const sampler2D& s, vec2 uv) {
  if (!s.t) return mk(0, 0, 0, 1);
  float fx = std::floor(uv.x * (float)s.w), fy = std::floor(uv.y * (float)s.h);
  fx = std::fmin(std::fmax(fx, 0.0f), (float)(s.w - 1));  // (a NaN coordinate lands on texel 0)
  fy = std::fmin(std::fmax(fy, 0.0f), (float)(s.h - 1));
  const float* p = s.t + ((size_t)fy * s.w + (size_t)fx) * s.comps;
  return mk(p[0], p[1], p[2], s.comps == 4 ? p[3] : 1.0f);
}

// the built-ins the shaders call with mixed int / float arguments, and the ones
// bound to the numerics contract
using glm::abs;
using glm::clamp;
using glm::max;
using glm::min;
inline float max(int a, float b) { return glm::max((float)a, b); }
inline float max(float a, int b) { return glm::max(a, (float)b); }
inline float clamp(float x, int a, int b) { return glm::clamp(x, (float)a, (float)b); }
inline float sin(float x) { return ptm_sinf(x); }
inline float cos(float x) { return ptm_cosf(x); }
inline float atan(float y, float x) { return ptm_atan2f(y, x); }
inline float asin(float x) { return ptm_asinf(x); }
inline float log(float x) { return ptm_logf(x); }
inline float pow(float x, float y) { return ptm_powf(x, y); }
inline float sqrt(float x) { return std::sqrt(x); }
// a swizzle is a vector wherever GLSL passes one to a built-in
using glm::normalize;
template <class S, class V = decltype(std::declval<const S&>()())>
inline V normalize(const S& s) { return glm::normalize(s()); }

struct Uniforms {
  vec3 pix;
  uint frameCounter;
  int nTriangles, nNodes, width, height, hdrResolution;
  samplerBuffer triangles, nodes;
  sampler2D lastFrame, hdrMap, hdrCache;
  vec3 eye;
  mat4 cameraRotate;
};

#define in
#define out
#define uniform

#define PT_GL_COMMON(u)                                                                              \
  pix(u.pix), frameCounter(u.frameCounter), nTriangles(u.nTriangles), nNodes(u.nNodes), width(u.width), \
      height(u.height), triangles(u.triangles), nodes(u.nodes), lastFrame(u.lastFrame), hdrMap(u.hdrMap),  \
      eye(u.eye), cameraRotate(u.cameraRotate)

struct PassO {  // OpenglRayTracing/shaders/pass1.fsh
#include "_ref/o_pass1.inc"
  vec4 gl_FragData[1];
  explicit PassO(const Uniforms& u) : PT_GL_COMMON(u) {}
};
#undef PI
#undef INF
#undef SIZE_TRIANGLE
#undef SIZE_BVHNODE

struct PassD {  // DisneyBRDF/shaders/pass1.fsh
#include "_ref/d_pass1.inc"
  vec4 gl_FragData[1];
  explicit PassD(const Uniforms& u) : PT_GL_COMMON(u) {}
};
#undef PI
#undef INF
#undef SIZE_TRIANGLE
#undef SIZE_BVHNODE

struct PassIS {  // ImportanceSampling_LowDiscrepancySequence/shaders/pass1.fsh
#include "_ref/is_pass1.inc"
  vec4 gl_FragData[1];
  explicit PassIS(const Uniforms& u)
      : pix(u.pix), frameCounter(u.frameCounter), nTriangles(u.nTriangles), nNodes(u.nNodes), width(u.width),
        height(u.height), hdrResolution(u.hdrResolution), triangles(u.triangles), nodes(u.nodes),
        lastFrame(u.lastFrame), hdrMap(u.hdrMap), hdrCache(u.hdrCache), eye(u.eye), cameraRotate(u.cameraRotate) {}
};
#undef PI
#undef INF
#undef SIZE_TRIANGLE
#undef SIZE_BVHNODE

#undef in
#undef out
#undef uniform

}  // namespace glsl

using namespace glsl;

extern "C" {

typedef struct ref_scene {
  const float* tris;   // nTriangles x 36 (Triangle_encoded)
  int nTriangles;
  const float* nodes;  // nNodes x 12 (BVHNode_encoded)
  int nNodes;
  const float* hdr;    // hdrW x hdrH x 3 (nullable)
  const float* cache;  // calculateHdrCache output, same size (nullable)
  int hdrW, hdrH;
} ref_scene;

// GLSL evaluates call arguments left to right (GLSL 4.30 5.9); this build relies on
// the compiler doing the same for the shaders' two-rand() calls (IS:772, IS:848, ...).
static int g_order = 0;
static int nextOrder() { return ++g_order; }
static int firstOf(int a, int b) { return a < b ? 1 : 2; }
int ref_glsl_selfcheck(void) {
  g_order = 0;
  return firstOf(nextOrder(), nextOrder()) == 1 ? 0 : -1;
}

// One frame of shader `which` (0 O, 1 D, 2 IS) over the listed pixels (px, py pairs,
// py from the bottom; NULL = all): each fragment runs the shader's own main() and
// writes gl_FragData[0] into accum_out; lastFrame reads accum_in (W x H x 4).
int ref_glsl_render(int which, const ref_scene* s, int W, int H, const float eye[3], const float cam[16],
                    uint32_t frameCounter, const int* pixels, int nPix, const float* accum_in, float* accum_out) {
  if (!s || !accum_in || !accum_out || which < 0 || which > 2) return -1;
  if (ref_glsl_selfcheck() != 0) return -2;
  Uniforms u;
  u.frameCounter = frameCounter;
  u.nTriangles = s->nTriangles;
  u.nNodes = s->nNodes;
  u.width = W;
  u.height = H;
  u.hdrResolution = s->hdrW;  // IS main.cpp:853
  u.triangles.t = s->tris;
  u.triangles.n = s->nTriangles * 12;
  u.nodes.t = s->nodes;
  u.nodes.n = s->nNodes * 4;
  u.lastFrame.t = accum_in;
  u.lastFrame.w = W;
  u.lastFrame.h = H;
  u.lastFrame.comps = 4;
  u.hdrMap.t = s->hdr;
  u.hdrMap.w = s->hdrW;
  u.hdrMap.h = s->hdrH;
  u.hdrCache.t = s->cache;
  u.hdrCache.w = s->hdrW;
  u.hdrCache.h = s->hdrH;
  u.eye = vec3(eye[0], eye[1], eye[2]);
  std::memcpy(&u.cameraRotate[0][0], cam, 16 * sizeof(float));
  const long total = pixels ? nPix : (long)W * H;
  for (long k = 0; k < total; k++) {
    const int px = pixels ? pixels[2 * k] : (int)(k % W);
    const int py = pixels ? pixels[2 * k + 1] : (int)(k / W);
    u.pix = vec3((float)(2 * px + 1) / (float)W - 1.0f, (float)(2 * py + 1) / (float)H - 1.0f, 0.0f);
    vec4 c;
    if (which == 0) { PassO f(u); f.main(); c = f.gl_FragData[0]; }
    else if (which == 1) { PassD f(u); f.main(); c = f.gl_FragData[0]; }
    else { PassIS f(u); f.main(); c = f.gl_FragData[0]; }
    float* o = accum_out + 4 * ((size_t)py * W + px);
    o[0] = c.x; o[1] = c.y; o[2] = c.z; o[3] = c.w;
  }
  return 0;
}

}  // extern "C"
