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
//  * the transcendental built-ins (sin, cos, atan(y, x), asin, log, pow): GLSL leaves
//    their precision to the GL driver, which is not in the reference. They are bound
//    here to the host C library's double-precision sin / cos / atan2 / asin / log / pow
//    (glibc) rounded to float, i.e. the correctly rounded value in all but rare cases,
//    computed by code this repository did not write. (Until round 6 they were bound to
//    include/pt_fmath.h, the functions the GPU itself calls, which made this pin a
//    self-comparison for every transcendental site.) sqrt, / and the rest are IEEE
//    (-ffp-contract=off);
//  * pix, the vertex shader's NDC position (vshader.vsh:7-10) interpolated to the
//    fragment centre, as the oracle forms it: (2 px + 1) / w - 1 in float.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>

// glm enables its swizzle operators (pix.xy as a member) only with MS language
// extensions or x86 intrinsics; the former changes no arithmetic (glm/detail/setup.hpp:75)
#define GLM_FORCE_SWIZZLE
#ifndef _MSC_EXTENSIONS
#define _MSC_EXTENSIONS
#define PT_UNDEF_MSC_EXTENSIONS
#endif
#include <glm/glm.hpp>
#ifdef PT_UNDEF_MSC_EXTENSIONS
#undef _MSC_EXTENSIONS
#endif


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
// GLSL's transcendental built-ins: the host C library's double-precision functions (glibc),
// rounded to float -- the correctly rounded value in all but rare cases, from an implementation
// this repository did not write (the GPU's include/pt_fmath.h computes the same correctly rounded
// values its own way; tests/test_fmath.py, tests/test_gpu_libm_pin.py)
inline float sin(float x) { return (float)::sin((double)x); }
inline float cos(float x) { return (float)::cos((double)x); }
inline float atan(float y, float x) { return (float)::atan2((double)y, (double)x); }
inline float asin(float x) { return (float)::asin((double)x); }
inline float log(float x) { return (float)::log((double)x); }
inline float pow(float x, float y) { return (float)::pow((double)x, (double)y); }
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

// ---------------------------------------------------------------- per-function
// Function fn of the compiled shader text on n inputs (fixed strides, tests/test_glsl_ref.py
// FUNCS; the oracle's orc_glsl_fn takes the same layout). Unsigned ints travel as float bits.
// Member functions are called on one fragment object whose uniforms the input sets
// (CranleyPatterson reads pix / width / height).
static inline uint32_t ubits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static inline float fbits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static inline vec3 v3at(const float* p) { return vec3(p[0], p[1], p[2]); }
static inline void put3(float* o, vec3 v) { o[0] = v.x; o[1] = v.y; o[2] = v.z; }
}  // extern "C"
template <class M>
static M matAt(const float* p) {
  M m;
  m.emissive = v3at(p);
  m.baseColor = v3at(p + 3);
  m.subsurface = p[6]; m.metallic = p[7]; m.specular = p[8]; m.specularTint = p[9];
  m.roughness = p[10]; m.anisotropic = p[11]; m.sheen = p[12]; m.sheenTint = p[13];
  m.clearcoat = p[14]; m.clearcoatGloss = p[15]; m.IOR = p[16]; m.transmission = p[17];
  return m;
}
extern "C" {

static const int FN_IN[] = {1, 2, 2, 6, 6, 3, 24, 12, 1, 2, 2, 5, 2, 5, 33, 33, 27, 27, 5, 9, 9, 26, 3, 2, 1};
static const int FN_OUT[] = {2, 1, 2, 2, 3, 6, 9, 1, 1, 1, 1, 1, 1, 1, 3, 3, 3, 1, 3, 3, 3, 3, 2, 1, 4};
#define REF_NFN ((int)(sizeof(FN_IN) / sizeof(FN_IN[0])))

int ref_glsl_fn_arity(int fn, int* nin, int* nout) {
  if (fn < 0 || fn >= REF_NFN) return -1;
  *nin = FN_IN[fn];
  *nout = FN_OUT[fn];
  return 0;
}

int ref_glsl_fn(int fn, const float* in, float* out, int n) {
  if (fn < 0 || fn >= REF_NFN || n < 0) return -1;
  if (ref_glsl_selfcheck() != 0) return -2;
  Uniforms u{};
  u.width = u.height = 1;
  for (int k = 0; k < n; k++) {
    const float* a = in + (size_t)k * FN_IN[fn];
    float* o = out + (size_t)k * FN_OUT[fn];
    PassIS is(u);
    PassD d(u);
    switch (fn) {
      case 0: {  // wang_hash IS:78-85
        uint32_t sd = ubits(a[0]);
        uint32_t r = is.wang_hash(sd);
        o[0] = fbits(r); o[1] = fbits(sd);
        break;
      }
      case 1: o[0] = is.sobol(ubits(a[0]), ubits(a[1])); break;  // IS:101-109
      case 2: { vec2 v = is.sobolVec2(ubits(a[0]), ubits(a[1])); o[0] = v.x; o[1] = v.y; break; }  // IS:112-116
      case 3: {  // CranleyPatterson IS:118-136: pix of pixel (a0, a1) in an a2 x a3 frame
        Uniforms w = u;
        w.width = (int)a[2];
        w.height = (int)a[3];
        w.pix = vec3((float)(2 * (int)a[0] + 1) / (float)w.width - 1.0f, (float)(2 * (int)a[1] + 1) / (float)w.height - 1.0f, 0.0f);
        PassIS f(w);
        vec2 r = f.CranleyPattersonRotation(vec2(a[4], a[5]));
        o[0] = r.x; o[1] = r.y;
        break;
      }
      case 4: put3(o, is.toNormalHemisphere(v3at(a), v3at(a + 3))); break;  // IS:153-159
      case 5: { vec3 t(0), b(0); is.getTangent(v3at(a), t, b); put3(o, t); put3(o + 3, b); break; }  // IS:161-172
      case 6: {  // hitTriangle IS:251-301
        PassIS::Triangle t;
        t.p1 = v3at(a); t.p2 = v3at(a + 3); t.p3 = v3at(a + 6);
        t.n1 = v3at(a + 9); t.n2 = v3at(a + 12); t.n3 = v3at(a + 15);
        PassIS::Ray r;
        r.startPosition = v3at(a + 18);
        r.direction = v3at(a + 21);
        PassIS::HitResult h = is.hitTriangle(t, r);
        o[0] = h.isHit ? 1.0f : 0.0f; o[1] = h.isInside ? 1.0f : 0.0f; o[2] = h.distance;
        put3(o + 3, h.isHit ? h.hitPoint : vec3(0)); put3(o + 6, h.isHit ? h.normal : vec3(0));
        break;
      }
      case 7: {  // hitAABB IS:303-316
        PassIS::Ray r;
        r.startPosition = v3at(a);
        r.direction = v3at(a + 3);
        o[0] = is.hitAABB(r, v3at(a + 6), v3at(a + 9));
        break;
      }
      case 8: o[0] = is.SchlickFresnel(a[0]); break;              // IS:390-394
      case 9: o[0] = is.GTR1(a[0], a[1]); break;                   // IS:396-401
      case 10: o[0] = is.GTR2(a[0], a[1]); break;                  // IS:403-407
      case 11: o[0] = is.GTR2_aniso(a[0], a[1], a[2], a[3], a[4]); break;  // IS:409-411
      case 12: o[0] = is.smithG_GGX(a[0], a[1]); break;            // IS:413-417
      case 13: o[0] = is.smithG_GGX_aniso(a[0], a[1], a[2], a[3], a[4]); break;  // IS:419-421
      case 14:  // BRDF_Evaluate_aniso IS:423-482
        put3(o, is.BRDF_Evaluate_aniso(v3at(a), v3at(a + 3), v3at(a + 6), v3at(a + 9), v3at(a + 12),
                                       matAt<PassIS::Material>(a + 15)));
        break;
      case 15:  // BRDF_Evaluate D:381-440 (the DisneyBRDF kernel's own text)
        put3(o, d.BRDF_Evaluate(v3at(a), v3at(a + 3), v3at(a + 6), v3at(a + 9), v3at(a + 12),
                                matAt<PassD::Material>(a + 15)));
        break;
      case 16: put3(o, is.BRDF_Evaluate(v3at(a), v3at(a + 3), v3at(a + 6), matAt<PassIS::Material>(a + 9))); break;  // IS:587-636
      case 17: o[0] = is.BRDF_Pdf(v3at(a), v3at(a + 3), v3at(a + 6), matAt<PassIS::Material>(a + 9)); break;  // IS:669-706
      case 18: put3(o, is.SampleCosineHemisphere(a[0], a[1], v3at(a + 2))); break;  // IS:485-496
      case 19: put3(o, is.SampleGTR2(a[0], a[1], v3at(a + 2), v3at(a + 5), a[8])); break;  // IS:499-516
      case 20: put3(o, is.SampleGTR1(a[0], a[1], v3at(a + 2), v3at(a + 5), a[8])); break;  // IS:519-536
      case 21:  // SampleBRDF IS:539-570
        put3(o, is.SampleBRDF(a[0], a[1], a[2], v3at(a + 3), v3at(a + 6), matAt<PassIS::Material>(a + 8)));
        break;
      case 22: { vec2 v = is.toSphericalCoord(v3at(a)); o[0] = v.x; o[1] = v.y; break; }  // IS:638-644
      case 23: o[0] = is.misMixWeight(a[0], a[1]); break;  // IS:708-711
      case 24: {  // SampleHemisphere() D:90-95 (z = rand(), then phi), from seed a0
        d.seed = ubits(a[0]);
        vec3 v = d.SampleHemisphere();
        put3(o, v);
        o[3] = fbits(d.seed);
        break;
      }
    }
  }
  return 0;
}

}  // extern "C"
