/*
 * pt_oracle.c -- TEST INFRASTRUCTURE ONLY (see pt_oracle.h).
 *
 * A line-by-line CPU restatement of the reference's per-pixel fragment kernel
 * (three variants) and of its CPU tracer. Compiled with -ffp-contract=off so
 * every float operation rounds exactly once, in the order written here. The
 * evaluation orders chosen for expressions the GLSL spec leaves open are the
 * glm 0.9.9.8 orders (dot = (x+y)+z, mat4*vec4 = (c0x+c1y)+(c2z+c3w)), and the
 * HIP kernel follows the same orders.
 *
 * References cited as IS = ImportanceSampling_LowDiscrepancySequence/shaders/pass1.fsh,
 * D = DisneyBRDF/shaders/pass1.fsh, O = OpenglRayTracing/shaders/pass1.fsh,
 * B = BasicRayTracingWithC++/main.cpp, H = OpenglRayTracing/main.cpp.
 */
#include "pt_oracle.h"
#include "pt_fmath.h" /* the numerics contract for transcendentals (include/) */

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PI 3.1415926f            /* IS:23 */
#define INF 2147483647.0f        /* IS:24 (rounds to 2^31 in f32) */

typedef struct { float x, y, z; } v3;

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 scl(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 sdiv(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
  return V3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline v3 normalize(v3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return scl(v, inv); }
static inline float mixf(float x, float y, float a) { return x * (1.0f - a) + y * a; }
static inline v3 mixv(v3 x, v3 y, float a) { return V3(mixf(x.x, y.x, a), mixf(x.y, y.y, a), mixf(x.z, y.z, a)); }
static inline float sqr(float x) { return x * x; }   /* IS:386 */
static inline v3 vminf(v3 a, float m) { return V3(fminf(a.x, m), fminf(a.y, m), fminf(a.z, m)); }
/* GLSL reflect(I, N) = I - 2*dot(N,I)*N */
static inline v3 reflect3(v3 I, v3 N) { float k = 2.0f * dot(N, I); return sub(I, scl(N, k)); }

/* ------------------------------------------------------------------ RNG */
/* wang_hash IS:78-85 */
static inline uint32_t wang(uint32_t* s) {
  uint32_t x = *s;
  x = (x ^ 61u) ^ (x >> 16);
  x *= 9u;
  x = x ^ (x >> 4);
  x *= 0x27d4eb2du;
  x = x ^ (x >> 15);
  *s = x;
  return x;
}
/* rand IS:87-89 */
static inline float randf(uint32_t* s) { return (float)wang(s) / 4294967296.0f; }

/* Sobol direction numbers, verbatim from IS:92-94 (8 dims x 32). */
static const uint32_t SOBOL_V[8 * 32] = {
    2147483648u,1073741824u,536870912u,268435456u,134217728u,67108864u,33554432u,16777216u,8388608u,4194304u,2097152u,1048576u,524288u,262144u,131072u,65536u,32768u,16384u,8192u,4096u,2048u,1024u,512u,256u,128u,64u,32u,16u,8u,4u,2u,1u,
    2147483648u,3221225472u,2684354560u,4026531840u,2281701376u,3422552064u,2852126720u,4278190080u,2155872256u,3233808384u,2694840320u,4042260480u,2290614272u,3435921408u,2863267840u,4294901760u,2147516416u,3221274624u,2684395520u,4026593280u,2281736192u,3422604288u,2852170240u,4278255360u,2155905152u,3233857728u,2694881440u,4042322160u,2290649224u,3435973836u,2863311530u,4294967295u,
    2147483648u,3221225472u,1610612736u,2415919104u,3892314112u,1543503872u,2382364672u,3305111552u,1753219072u,2629828608u,3999268864u,1435500544u,2154299392u,3231449088u,1626210304u,2421489664u,3900735488u,1556135936u,2388680704u,3314585600u,1751705600u,2627492864u,4008611328u,1431684352u,2147543168u,3221249216u,1610649184u,2415969680u,3892340840u,1543543964u,2382425838u,3305133397u,
    2147483648u,3221225472u,536870912u,1342177280u,4160749568u,1946157056u,2717908992u,2466250752u,3632267264u,624951296u,1507852288u,3872391168u,2013790208u,3020685312u,2181169152u,3271884800u,546275328u,1363623936u,4226424832u,1977167872u,2693105664u,2437829632u,3689389568u,635137280u,1484783744u,3846176960u,2044723232u,3067084880u,2148008184u,3222012020u,537002146u,1342505107u,
    2147483648u,1073741824u,536870912u,2952790016u,4160749568u,3690987520u,2046820352u,2634022912u,1518338048u,801112064u,2707423232u,4038066176u,3666345984u,1875116032u,2170683392u,1085997056u,579305472u,3016343552u,4217741312u,3719483392u,2013407232u,2617981952u,1510979072u,755882752u,2726789248u,4090085440u,3680870432u,1840435376u,2147625208u,1074478300u,537900666u,2953698205u,
    2147483648u,1073741824u,1610612736u,805306368u,2818572288u,335544320u,2113929216u,3472883712u,2290089984u,3829399552u,3059744768u,1127219200u,3089629184u,4199809024u,3567124480u,1891565568u,394297344u,3988799488u,920674304u,4193267712u,2950604800u,3977188352u,3250028032u,129093376u,2231568512u,2963678272u,4281226848u,432124720u,803643432u,1633613396u,2672665246u,3170194367u,
    2147483648u,3221225472u,2684354560u,3489660928u,1476395008u,2483027968u,1040187392u,3808428032u,3196059648u,599785472u,505413632u,4077912064u,1182269440u,1736704000u,2017853440u,2221342720u,3329785856u,2810494976u,3628507136u,1416089600u,2658719744u,864310272u,3863387648u,3076993792u,553150080u,272922560u,4167467040u,1148698640u,1719673080u,2009075780u,2149644390u,3222291575u,
    2147483648u,1073741824u,2684354560u,1342177280u,2281701376u,1946157056u,436207616u,2566914048u,2625634304u,3208642560u,2720006144u,2098200576u,111673344u,2354315264u,3464626176u,4027383808u,2886631424u,3770826752u,1691164672u,3357462528u,1993345024u,3752330240u,873073152u,2870150400u,1700563072u,87021376u,1097028000u,1222351248u,1560027592u,2977959924u,23268898u,437609937u};

/* sobol IS:101-109. Dims >= 8 index past V[] in the reference (bounce >= 4:
 * undefined). Documented extension: dim d >= 8 reuses table dim
 * d % 8 with a digital XOR shift by wang_hash(d). */
static uint32_t sobol_bits(uint32_t d, uint32_t i) {
  uint32_t result = 0;
  uint32_t offset = (d & 7u) * 32u;
  for (uint32_t j = 0; i != 0; i >>= 1, j++)
    if ((i & 1u) != 0) result ^= SOBOL_V[j + offset];
  if (d >= 8u) { uint32_t h = d; result ^= wang(&h); }
  return result;
}
static inline float sobolf(uint32_t d, uint32_t i) {
  return (float)sobol_bits(d, i) * (1.0f / (float)0xFFFFFFFFu);
}
static inline uint32_t grayCode(uint32_t i) { return i ^ (i >> 1); } /* IS:96-98 */

/* CranleyPattersonRotation IS:118-136 (114514/1919 == 59 in integer math) */
static void cranley_patterson(int px, int py, float* u_, float* v_) {
  uint32_t pseed = ((uint32_t)px * 1973u + (uint32_t)py * 9277u + 59u * 26699u) | 1u;
  float u = (float)wang(&pseed) / 4294967296.0f;
  float v = (float)wang(&pseed) / 4294967296.0f;
  float x = *u_ + u;
  if (x > 1.0f) x -= 1.0f;
  if (x < 0.0f) x += 1.0f;
  float y = *v_ + v;
  if (y > 1.0f) y -= 1.0f;
  if (y < 0.0f) y += 1.0f;
  *u_ = x; *v_ = y;
}

/* ------------------------------------------------------------ scene fetch */
typedef struct {
  v3 emissive, baseColor;
  float subsurface, metallic, specular, specularTint, roughness, anisotropic;
  float sheen, sheenTint, clearcoat, clearcoatGloss, IOR, transmission;
} Material;

typedef struct {
  int isHit, isInside;
  float distance;
  v3 hitPoint, normal, viewDir;
  Material material;
  int tri;
} Hit;

typedef struct { v3 p1, p2, p3, n1, n2, n3; } Tri;

typedef struct {
  const orc_scene* s;
  orc_counters c;
} Ctx;

static inline v3 texel3(const float* base, int k) { return V3(base[3 * k], base[3 * k + 1], base[3 * k + 2]); }

/* getTriangle IS:191-205 */
static Tri getTriangle(Ctx* cx, int i) {
  const float* t = cx->s->tris + (size_t)i * 36;
  Tri r;
  r.p1 = texel3(t, 0); r.p2 = texel3(t, 1); r.p3 = texel3(t, 2);
  r.n1 = texel3(t, 3); r.n2 = texel3(t, 4); r.n3 = texel3(t, 5);
  cx->c.tris++;
  return r;
}
/* getMaterial IS:207-232 */
static Material getMaterial(Ctx* cx, int i) {
  const float* t = cx->s->tris + (size_t)i * 36;
  Material m;
  v3 p1 = texel3(t, 8), p2 = texel3(t, 9), p3 = texel3(t, 10), p4 = texel3(t, 11);
  m.emissive = texel3(t, 6);
  m.baseColor = texel3(t, 7);
  m.subsurface = p1.x; m.metallic = p1.y; m.specular = p1.z;
  m.specularTint = p2.x; m.roughness = p2.y; m.anisotropic = p2.z;
  m.sheen = p3.x; m.sheenTint = p3.y; m.clearcoat = p3.z;
  m.clearcoatGloss = p4.x; m.IOR = p4.y; m.transmission = p4.z;
  cx->c.mats++;
  return m;
}
typedef struct { int left, right, n, index; v3 AA, BB; } Node;
/* getBVHNode IS:234-249 (ivec3(float) truncation) */
static Node getBVHNode(Ctx* cx, int i) {
  const float* t = cx->s->nodes + (size_t)i * 12;
  Node n;
  n.left = (int)t[0]; n.right = (int)t[1];
  n.n = (int)t[3]; n.index = (int)t[4];
  n.AA = texel3(t, 2); n.BB = texel3(t, 3);
  cx->c.nodes++;
  return n;
}

/* hitTriangle IS:251-301 */
static Hit hitTriangle(Tri tr, v3 S, v3 d) {
  Hit res;
  memset(&res, 0, sizeof(res));
  res.distance = INF;
  v3 p1 = tr.p1, p2 = tr.p2, p3 = tr.p3;
  v3 N = normalize(cross(sub(p2, p1), sub(p3, p1)));
  if (dot(N, d) > 0.0f) { N = neg(N); res.isInside = 1; }
  if (fabsf(dot(N, d)) < 0.00001f) return res;
  float t = (dot(N, p1) - dot(S, N)) / dot(d, N);
  if (t < 0.0005f) return res;
  v3 P = add(S, scl(d, t));
  v3 c1 = cross(sub(p2, p1), sub(P, p1));
  v3 c2 = cross(sub(p3, p2), sub(P, p2));
  v3 c3 = cross(sub(p1, p3), sub(P, p3));
  float s1 = dot(c1, N), s2 = dot(c2, N), s3 = dot(c3, N);
  int r1 = (s1 > 0 && s2 > 0 && s3 > 0);
  int r2 = (s1 < 0 && s2 < 0 && s3 < 0);
  if (r1 || r2) {
    res.isHit = 1;
    res.hitPoint = P;
    res.distance = t;
    res.viewDir = d;
    float alpha = (-(P.x - p2.x) * (p3.y - p2.y) + (P.y - p2.y) * (p3.x - p2.x)) /
                  (-(p1.x - p2.x - 0.00005f) * (p3.y - p2.y + 0.00005f) +
                   (p1.y - p2.y + 0.00005f) * (p3.x - p2.x + 0.00005f));
    float beta = (-(P.x - p3.x) * (p1.y - p3.y) + (P.y - p3.y) * (p1.x - p3.x)) /
                 (-(p2.x - p3.x - 0.00005f) * (p1.y - p3.y + 0.00005f) +
                  (p2.y - p3.y + 0.00005f) * (p1.x - p3.x + 0.00005f));
    float gama = 1.0f - alpha - beta;
    v3 Ns = add(add(scl(tr.n1, alpha), scl(tr.n2, beta)), scl(tr.n3, gama));
    Ns = normalize(Ns);
    res.normal = res.isInside ? neg(Ns) : Ns;
  }
  return res;
}

/* hitAABB IS:303-316 */
static float hitAABB(v3 S, v3 d, v3 AA, v3 BB) {
  v3 invdir = V3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  v3 f = mul(sub(BB, S), invdir);
  v3 n = mul(sub(AA, S), invdir);
  v3 tmax = V3(fmaxf(f.x, n.x), fmaxf(f.y, n.y), fmaxf(f.z, n.z));
  v3 tmin = V3(fminf(f.x, n.x), fminf(f.y, n.y), fminf(f.z, n.z));
  float t1 = fminf(tmax.x, fminf(tmax.y, tmax.z));
  float t0 = fmaxf(tmin.x, fmaxf(tmin.y, tmin.z));
  return (t1 >= t0) ? ((t0 > 0.0f) ? t0 : t1) : -1.0f;
}

/* hitArray IS:319-332 */
static Hit hitArray(Ctx* cx, v3 S, v3 d, int l, int r) {
  Hit res;
  memset(&res, 0, sizeof(res));
  res.distance = INF;
  res.tri = -1;
  for (int i = l; i <= r; i++) {
    Tri tr = getTriangle(cx, i);
    Hit h = hitTriangle(tr, S, d);
    if (h.isHit && h.distance < res.distance) {
      res = h;
      res.tri = i;
      res.material = getMaterial(cx, i);
    }
  }
  return res;
}

#define ORC_STACK 8192 /* the reference's int stack[256] (IS:340) is UB when exceeded */

/* hitBVH IS:335-382 */
static Hit hitBVH(Ctx* cx, v3 S, v3 d) {
  Hit res;
  memset(&res, 0, sizeof(res));
  res.distance = INF;
  res.tri = -1;
  cx->c.rays++;
  int stack[ORC_STACK];
  int sp = 0;
  stack[sp++] = 1;
  while (sp > 0) {
    int top = stack[--sp];
    Node node = getBVHNode(cx, top);
    if (node.n > 0) {
      int L = node.index;
      int R = node.index + node.n - 1;
      Hit r = hitArray(cx, S, d, L, R);
      if (r.isHit && r.distance < res.distance) res = r;
      continue;
    }
    float d1 = INF, d2 = INF;
    if (node.left > 0) {
      Node ln = getBVHNode(cx, node.left);
      d1 = hitAABB(S, d, ln.AA, ln.BB);
    }
    if (node.right > 0) {
      Node rn = getBVHNode(cx, node.right);
      d2 = hitAABB(S, d, rn.AA, rn.BB);
    }
    /* A child index <= 0 is never produced by the reference builders (H:430-551);
     * the reference would push it (d = INF > 0) and read the dummy node 0 with an
     * uninitialised index. Documented deviation: missing children are skipped. */
    int lok = node.left > 0, rok = node.right > 0;
    if (sp + 2 > ORC_STACK) break;
    if (d1 > 0 && d2 > 0 && lok && rok) {
      if (d1 < d2) { stack[sp++] = node.right; stack[sp++] = node.left; }
      else { stack[sp++] = node.left; stack[sp++] = node.right; }
    } else if (d1 > 0 && lok) {
      stack[sp++] = node.left;
    } else if (d2 > 0 && rok) {
      stack[sp++] = node.right;
    }
  }
  return res;
}

/* ------------------------------------------------------------ environment */
static v3 tex_nearest(Ctx* cx, const float* img, float u, float v) {
  const orc_scene* s = cx->s;
  cx->c.texels++;
  if (!img) return V3(0, 0, 0);
  float fx = floorf(u * (float)s->hdrW);
  float fy = floorf(v * (float)s->hdrH);
  fx = fminf(fmaxf(fx, 0.0f), (float)(s->hdrW - 1));
  fy = fminf(fmaxf(fy, 0.0f), (float)(s->hdrH - 1));
  int x = (int)fx, y = (int)fy;
  return texel3(img, y * s->hdrW + x);
}
/* SampleSphericalMap IS:175-181 == toSphericalCoord IS:638-644 */
static void toSpherical(v3 v, float* u, float* w) {
  float a = ptm_atan2f(v.z, v.x), b = ptm_asinf(v.y);
  a = a / (2.0f * PI);
  b = b / PI;
  a = a + 0.5f;
  b = b + 0.5f;
  *u = a;
  *w = 1.0f - b;
}
/* sampleHdr IS:184-189 (clamped at 10) */
static v3 sampleHdr(Ctx* cx, v3 v) {
  float u, w;
  toSpherical(normalize(v), &u, &w);
  return vminf(tex_nearest(cx, cx->s->hdr, u, w), 10.0f);
}
/* hdrColor IS:647-651 (unclamped) */
static v3 hdrColor(Ctx* cx, v3 L) {
  float u, w;
  toSpherical(normalize(L), &u, &w);
  return tex_nearest(cx, cx->s->hdr, u, w);
}
/* SampleHdr IS:573-585 */
static v3 SampleHdrDir(Ctx* cx, float xi1, float xi2) {
  v3 xy = tex_nearest(cx, cx->s->cache, xi1, xi2);
  float x = xy.x, y = 1.0f - xy.y;
  float phi = 2.0f * PI * (x - 0.5f);
  float theta = PI * (y - 0.5f);
  return V3(ptm_cosf(theta) * ptm_cosf(phi), ptm_sinf(theta), ptm_cosf(theta) * ptm_sinf(phi));
}
/* hdrPdf IS:655-666 (sin of the elevation: reference bug kept) */
static float hdrPdf(Ctx* cx, v3 L, int hdrResolution) {
  float u, w;
  toSpherical(normalize(L), &u, &w);
  float pdf = tex_nearest(cx, cx->s->cache, u, w).z;
  float theta = PI * (0.5f - w);
  float sin_theta = fmaxf(ptm_sinf(theta), 1e-10f);
  float p_convert = (float)(hdrResolution * hdrResolution / 2) / (2.0f * PI * PI * sin_theta);
  return pdf * p_convert;
}

/* ------------------------------------------------------------ BRDF IS:386-706 */
static float SchlickFresnel(float u) {
  float m = fminf(fmaxf(1.0f - u, 0.0f), 1.0f);
  float m2 = m * m;
  return m2 * m2 * m;
}
static float GTR1(float NdotH, float a) {
  if (a >= 1.0f) return 1.0f / PI;
  float a2 = a * a;
  float t = 1.0f + (a2 - 1.0f) * NdotH * NdotH;
  return (a2 - 1.0f) / (PI * ptm_logf(a2) * t);
}
static float GTR2(float NdotH, float a) {
  float a2 = a * a;
  float t = 1.0f + (a2 - 1.0f) * NdotH * NdotH;
  return a2 / (PI * t * t);
}
static float GTR2_aniso(float NdotH, float HdotX, float HdotY, float ax, float ay) {
  return 1.0f / (PI * ax * ay * sqr(sqr(HdotX / ax) + sqr(HdotY / ay) + NdotH * NdotH));
}
static float smithG_GGX(float NdotV, float alphaG) {
  float a = alphaG * alphaG;
  float b = NdotV * NdotV;
  return 1.0f / (NdotV + sqrtf(a + b - a * b));
}
static float smithG_GGX_aniso(float NdotV, float VdotX, float VdotY, float ax, float ay) {
  return 1.0f / (NdotV + sqrtf(sqr(VdotX * ax) + sqr(VdotY * ay) + sqr(NdotV)));
}

typedef struct { v3 Cdlin, Cspec0, Csheen; } Tints;
static Tints tints(const Material* m) {
  Tints t;
  v3 Cdlin = m->baseColor;
  float Cdlum = 0.3f * Cdlin.x + 0.6f * Cdlin.y + 0.1f * Cdlin.z;
  v3 Ctint = (Cdlum > 0.0f) ? sdiv(Cdlin, Cdlum) : V3(1, 1, 1);
  v3 Cspec = scl(mixv(V3(1, 1, 1), Ctint, m->specularTint), m->specular);
  t.Cdlin = Cdlin;
  t.Cspec0 = mixv(scl(Cspec, 0.08f), Cdlin, m->metallic);
  t.Csheen = mixv(V3(1, 1, 1), Ctint, m->sheenTint);
  return t;
}

/* BRDF_Evaluate_aniso IS:423-482 == D:381-440 */
static v3 BRDF_Evaluate_aniso(v3 V, v3 N, v3 L, v3 X, v3 Y, const Material* m) {
  float NdotL = dot(N, L);
  float NdotV = dot(N, V);
  if (NdotL < 0 || NdotV < 0) return V3(0, 0, 0);
  v3 H = normalize(add(L, V));
  float NdotH = dot(N, H);
  float LdotH = dot(L, H);
  Tints tt = tints(m);
  float Fd90 = 0.5f + 2.0f * LdotH * LdotH * m->roughness;
  float FL = SchlickFresnel(NdotL);
  float FV = SchlickFresnel(NdotV);
  float Fd = mixf(1.0f, Fd90, FL) * mixf(1.0f, Fd90, FV);
  float Fss90 = LdotH * LdotH * m->roughness;
  float Fss = mixf(1.0f, Fss90, FL) * mixf(1.0f, Fss90, FV);
  float ss = 1.25f * (Fss * (1.0f / (NdotL + NdotV) - 0.5f) + 0.5f);
  float aspect = sqrtf(1.0f - m->anisotropic * 0.9f);
  float ax = fmaxf(0.001f, sqr(m->roughness) / aspect);
  float ay = fmaxf(0.001f, sqr(m->roughness) * aspect);
  float Ds = GTR2_aniso(NdotH, dot(H, X), dot(H, Y), ax, ay);
  float FH = SchlickFresnel(LdotH);
  v3 Fs = mixv(tt.Cspec0, V3(1, 1, 1), FH);
  float Gs = smithG_GGX_aniso(NdotL, dot(L, X), dot(L, Y), ax, ay);
  Gs *= smithG_GGX_aniso(NdotV, dot(V, X), dot(V, Y), ax, ay);
  v3 specular = scl(scl(Fs, Gs), Ds);
  float Dr = GTR1(NdotH, mixf(0.1f, 0.001f, m->clearcoatGloss));
  float Fr = mixf(0.04f, 1.0f, FH);
  float Gr = smithG_GGX(NdotL, 0.25f) * smithG_GGX(NdotV, 0.25f);
  float cc = 0.25f * Gr * Fr * Dr * m->clearcoat;
  v3 Fsheen = scl(tt.Csheen, FH * m->sheen);
  float kd = (1.0f / PI) * mixf(Fd, ss, m->subsurface);
  v3 diffuse = add(scl(tt.Cdlin, kd), Fsheen);
  v3 r = add(scl(diffuse, 1.0f - m->metallic), specular);
  return add(r, V3(cc, cc, cc));
}

/* BRDF_Evaluate IS:587-636 */
static v3 BRDF_Evaluate(v3 V, v3 N, v3 L, const Material* m) {
  float NdotL = dot(N, L);
  float NdotV = dot(N, V);
  if (NdotL < 0 || NdotV < 0) return V3(0, 0, 0);
  v3 H = normalize(add(L, V));
  float NdotH = dot(N, H);
  float LdotH = dot(L, H);
  Tints tt = tints(m);
  float Fd90 = 0.5f + 2.0f * LdotH * LdotH * m->roughness;
  float FL = SchlickFresnel(NdotL);
  float FV = SchlickFresnel(NdotV);
  float Fd = mixf(1.0f, Fd90, FL) * mixf(1.0f, Fd90, FV);
  float Fss90 = LdotH * LdotH * m->roughness;
  float Fss = mixf(1.0f, Fss90, FL) * mixf(1.0f, Fss90, FV);
  float ss = 1.25f * (Fss * (1.0f / (NdotL + NdotV) - 0.5f) + 0.5f);
  float alpha = fmaxf(0.001f, sqr(m->roughness));
  float Ds = GTR2(NdotH, alpha);
  float FH = SchlickFresnel(LdotH);
  v3 Fs = mixv(tt.Cspec0, V3(1, 1, 1), FH);
  float Gs = smithG_GGX(NdotL, m->roughness);
  Gs *= smithG_GGX(NdotV, m->roughness);
  float Dr = GTR1(NdotH, mixf(0.1f, 0.001f, m->clearcoatGloss));
  float Fr = mixf(0.04f, 1.0f, FH);
  float Gr = smithG_GGX(NdotL, 0.25f) * smithG_GGX(NdotV, 0.25f);
  v3 Fsheen = scl(tt.Csheen, FH * m->sheen);
  float kd = (1.0f / PI) * mixf(Fd, ss, m->subsurface);
  v3 diffuse = add(scl(tt.Cdlin, kd), Fsheen);
  v3 specular = scl(scl(Fs, Gs), Ds);
  float cc = 0.25f * Gr * Fr * Dr * m->clearcoat;
  v3 r = add(scl(diffuse, 1.0f - m->metallic), specular);
  return add(r, V3(cc, cc, cc));
}

/* BRDF_Pdf IS:669-706 */
static float BRDF_Pdf(v3 V, v3 N, v3 L, const Material* m) {
  float NdotL = dot(N, L);
  float NdotV = dot(N, V);
  if (NdotL < 0 || NdotV < 0) return 0.0f;
  v3 H = normalize(add(L, V));
  float NdotH = dot(N, H);
  float LdotH = dot(L, H);
  float alpha = fmaxf(0.001f, sqr(m->roughness));
  float Ds = GTR2(NdotH, alpha);
  float Dr = GTR1(NdotH, mixf(0.1f, 0.001f, m->clearcoatGloss));
  float pdf_diffuse = NdotL / PI;
  float pdf_specular = Ds * NdotH / (4.0f * LdotH);
  float pdf_clearcoat = Dr * NdotH / (4.0f * LdotH);
  float r_diffuse = 1.0f - m->metallic;
  float r_specular = 1.0f;
  float r_clearcoat = 0.25f * m->clearcoat;
  float r_sum = r_diffuse + r_specular + r_clearcoat;
  float p_diffuse = r_diffuse / r_sum;
  float p_specular = r_specular / r_sum;
  float p_clearcoat = r_clearcoat / r_sum;
  float pdf = p_diffuse * pdf_diffuse + p_specular * pdf_specular + p_clearcoat * pdf_clearcoat;
  return fmaxf(1e-10f, pdf);
}
static float misMixWeight(float a, float b) { float t = a * a; return t / (b * b + t); } /* IS:708-711 */

/* toNormalHemisphere IS:153-159 */
static v3 toNormalHemisphere(v3 v, v3 N) {
  v3 helper = V3(1, 0, 0);
  if (fabsf(N.x) > 0.999f) helper = V3(0, 0, 1);
  v3 tangent = normalize(cross(N, helper));
  v3 bitangent = normalize(cross(N, tangent));
  return add(add(scl(tangent, v.x), scl(bitangent, v.y)), scl(N, v.z));
}
/* getTangent IS:161-172 (note the swapped naming) */
static void getTangent(v3 N, v3* tangent, v3* bitangent) {
  v3 helper = V3(1, 0, 0);
  if (fabsf(N.x) > 0.999f) helper = V3(0, 0, 1);
  *bitangent = normalize(cross(N, helper));
  *tangent = normalize(cross(N, *bitangent));
}
/* SampleHemisphere D:90-95 (rand order: z first) */
static v3 SampleHemisphereRand(uint32_t* seed) {
  float z = randf(seed);
  float r = fmaxf(0.0f, sqrtf(1.0f - z * z));
  float phi = 2.0f * PI * randf(seed);
  return V3(r * ptm_cosf(phi), r * ptm_sinf(phi), z);
}
/* SampleCosineHemisphere IS:485-496 */
static v3 SampleCosineHemisphere(float xi_1, float xi_2, v3 N) {
  float r = sqrtf(xi_1);
  float theta = xi_2 * 2.0f * PI;
  float x = r * ptm_cosf(theta);
  float y = r * ptm_sinf(theta);
  float z = sqrtf(1.0f - x * x - y * y);
  return toNormalHemisphere(V3(x, y, z), N);
}
/* SampleGTR2 IS:499-516 */
static v3 SampleGTR2(float xi_1, float xi_2, v3 V, v3 N, float alpha) {
  float phi_h = 2.0f * PI * xi_1;
  float sin_phi_h = ptm_sinf(phi_h);
  float cos_phi_h = ptm_cosf(phi_h);
  float cos_theta_h = sqrtf((1.0f - xi_2) / (1.0f + (alpha * alpha - 1.0f) * xi_2));
  float sin_theta_h = sqrtf(fmaxf(0.0f, 1.0f - cos_theta_h * cos_theta_h));
  v3 H = V3(sin_theta_h * cos_phi_h, sin_theta_h * sin_phi_h, cos_theta_h);
  H = toNormalHemisphere(H, N);
  return reflect3(neg(V), H);
}
/* SampleGTR1 IS:519-536 */
static v3 SampleGTR1(float xi_1, float xi_2, v3 V, v3 N, float alpha) {
  float phi_h = 2.0f * PI * xi_1;
  float sin_phi_h = ptm_sinf(phi_h);
  float cos_phi_h = ptm_cosf(phi_h);
  float cos_theta_h = sqrtf((1.0f - ptm_powf(alpha * alpha, 1.0f - xi_2)) / (1.0f - alpha * alpha));
  float sin_theta_h = sqrtf(fmaxf(0.0f, 1.0f - cos_theta_h * cos_theta_h));
  v3 H = V3(sin_theta_h * cos_phi_h, sin_theta_h * sin_phi_h, cos_theta_h);
  H = toNormalHemisphere(H, N);
  return reflect3(neg(V), H);
}
/* SampleBRDF IS:539-570 */
static v3 SampleBRDF(float xi_1, float xi_2, float xi_3, v3 V, v3 N, const Material* m) {
  float alpha_GTR1 = mixf(0.1f, 0.001f, m->clearcoatGloss);
  float alpha_GTR2 = fmaxf(0.001f, sqr(m->roughness));
  float r_diffuse = 1.0f - m->metallic;
  float r_specular = 1.0f;
  float r_clearcoat = 0.25f * m->clearcoat;
  float r_sum = r_diffuse + r_specular + r_clearcoat;
  float p_diffuse = r_diffuse / r_sum;
  float p_specular = r_specular / r_sum;
  float rd = xi_3;
  if (rd <= p_diffuse) return SampleCosineHemisphere(xi_1, xi_2, N);
  else if (p_diffuse < rd && rd <= p_diffuse + p_specular) return SampleGTR2(xi_1, xi_2, V, N, alpha_GTR2);
  else if (p_diffuse + p_specular < rd) return SampleGTR1(xi_1, xi_2, V, N, alpha_GTR1);
  return V3(0, 1, 0);
}

/* ------------------------------------------------------------ integrators */
/* pathTracing O:329-364 (Lambert, uniform hemisphere) */
static v3 pt_lambert(Ctx* cx, Hit hit, int maxBounce, uint32_t* seed) {
  v3 Lo = V3(0, 0, 0), history = V3(1, 1, 1);
  for (int bounce = 0; bounce < maxBounce; bounce++) {
    v3 wi = toNormalHemisphere(SampleHemisphereRand(seed), hit.normal);
    Hit nh = hitBVH(cx, hit.hitPoint, wi);
    float pdf = 1.0f / (2.0f * PI);
    float cosine_i = fmaxf(0.0f, dot(wi, hit.normal));
    v3 f_r = sdiv(hit.material.baseColor, PI);
    if (!nh.isHit) {
      v3 sky = sampleHdr(cx, wi);
      Lo = add(Lo, sdiv(scl(mul(mul(history, sky), f_r), cosine_i), pdf));
      break;
    }
    v3 Le = nh.material.emissive;
    Lo = add(Lo, sdiv(scl(mul(mul(history, Le), f_r), cosine_i), pdf));
    hit = nh;
    history = mul(history, sdiv(scl(f_r, cosine_i), pdf));
  }
  return Lo;
}

/* pathTracing D:443-481 (anisotropic Disney, uniform hemisphere) */
static v3 pt_disney_uniform(Ctx* cx, Hit hit, int maxBounce, uint32_t* seed) {
  v3 Lo = V3(0, 0, 0), history = V3(1, 1, 1);
  for (int bounce = 0; bounce < maxBounce; bounce++) {
    v3 V = neg(hit.viewDir);
    v3 N = hit.normal;
    v3 L = toNormalHemisphere(SampleHemisphereRand(seed), hit.normal);
    float pdf = 1.0f / (2.0f * PI);
    float cosine_i = fmaxf(0.0f, dot(L, N));
    v3 tangent, bitangent;
    getTangent(N, &tangent, &bitangent);
    v3 f_r = BRDF_Evaluate_aniso(V, N, L, tangent, bitangent, &hit.material);
    Hit nh = hitBVH(cx, hit.hitPoint, L);
    if (!nh.isHit) {
      v3 sky = sampleHdr(cx, L);
      Lo = add(Lo, sdiv(scl(mul(mul(history, sky), f_r), cosine_i), pdf));
      break;
    }
    v3 Le = nh.material.emissive;
    Lo = add(Lo, sdiv(scl(mul(mul(history, Le), f_r), cosine_i), pdf));
    hit = nh;
    history = mul(history, sdiv(scl(f_r, cosine_i), pdf));
  }
  return Lo;
}

/* pathTracingImportanceSampling IS:761-841 */
/* sample index of the frame: the reference's frameCounter unless sample-parallel */
static inline uint32_t sample_index(const orc_frame* f) {
  uint32_t w = f->sampleWorld > 0 ? (uint32_t)f->sampleWorld : 1u;
  return f->frameCounter * w + (uint32_t)f->sampleRank;
}

static v3 pt_mis(Ctx* cx, Hit hit, int maxBounce, uint32_t* seed, int px, int py, uint32_t frameCounter) {
  const orc_scene* s = cx->s;
  v3 Lo = V3(0, 0, 0), history = V3(1, 1, 1);
  for (int bounce = 0; bounce < maxBounce; bounce++) {
    v3 V = neg(hit.viewDir);
    v3 N = hit.normal;
    float r1 = randf(seed);
    float r2 = randf(seed);
    v3 Ldir = SampleHdrDir(cx, r1, r2);
    if (dot(N, Ldir) > 0.0f) {
      Hit hh = hitBVH(cx, hit.hitPoint, Ldir);
      if (!hh.isHit) {
        v3 L = Ldir;
        v3 color = hdrColor(cx, L);
        float pdf_light = hdrPdf(cx, L, s->hdrResolution);
        v3 f_r = BRDF_Evaluate(V, N, L, &hit.material);
        float pdf_brdf = BRDF_Pdf(V, N, L, &hit.material);
        float mis_weight = misMixWeight(pdf_light, pdf_brdf);
        v3 c = mul(mul(scl(history, mis_weight), color), f_r);
        Lo = add(Lo, sdiv(scl(c, dot(N, L)), pdf_light));
      }
    }
    uint32_t gi = grayCode(frameCounter + 1u);
    float u = sobolf(2u * (uint32_t)bounce, gi);
    float v = sobolf(2u * (uint32_t)bounce + 1u, gi);
    cranley_patterson(px, py, &u, &v);
    float xi_3 = randf(seed);
    v3 L = SampleBRDF(u, v, xi_3, V, N, &hit.material);
    float NdotL = dot(N, L);
    if (NdotL <= 0.0f) break;
    Hit nh = hitBVH(cx, hit.hitPoint, L);
    v3 f_r = BRDF_Evaluate(V, N, L, &hit.material);
    float pdf_brdf = BRDF_Pdf(V, N, L, &hit.material);
    if (pdf_brdf <= 0.0f) break;
    if (!nh.isHit) {
      v3 color = hdrColor(cx, L);
      float pdf_light = hdrPdf(cx, L, s->hdrResolution);
      float mis_weight = misMixWeight(pdf_brdf, pdf_light);
      v3 c = mul(mul(scl(history, mis_weight), color), f_r);
      Lo = add(Lo, sdiv(scl(c, NdotL), pdf_brdf));
      break;
    }
    v3 Le = nh.material.emissive;
    Lo = add(Lo, sdiv(scl(mul(mul(history, Le), f_r), NdotL), pdf_brdf));
    hit = nh;
    history = mul(history, sdiv(scl(f_r, NdotL), pdf_brdf));
  }
  return Lo;
}

static int default_bounce(int integrator) {
  switch (integrator) {
    case ORC_LAMBERT_O: return 2;          /* O:385 */
    case ORC_DISNEY_UNIFORM_D: return 5;   /* D:502 */
    case ORC_DISNEY_MIS_SOBOL_IS: return 2;/* IS:861 */
    default: return 8;                     /* B:254 */
  }
}

/* main IS:844-872 (one pixel) */
static void shade_gl_pixel(Ctx* cx, const orc_frame* f, int px, int py, float* accum) {
  const int W = f->width, H = f->height;
  const uint32_t sidx = sample_index(f);
  uint32_t seed = ((uint32_t)px * 1973u + (uint32_t)py * 9277u + sidx * 26699u) | 1u;
  float pixx = (float)(2 * px + 1) / (float)W - 1.0f;
  float pixy = (float)(2 * py + 1) / (float)H - 1.0f;
  float ax = (randf(&seed) - 0.5f) / (float)W;
  float ay = (randf(&seed) - 0.5f) / (float)H;
  float x = pixx + ax, y = pixy + ay, z = -1.5f;
  const float* M = f->cameraRotate;
  v3 c0 = V3(M[0], M[1], M[2]), c1 = V3(M[4], M[5], M[6]), c2 = V3(M[8], M[9], M[10]), c3 = V3(M[12], M[13], M[14]);
  v3 dir = add(add(scl(c0, x), scl(c1, y)), add(scl(c2, z), scl(c3, 0.0f)));
  dir = normalize(dir);
  v3 eye = V3(f->eye[0], f->eye[1], f->eye[2]);
  Hit first = hitBVH(cx, eye, dir);
  v3 color;
  int mb = f->maxBounce >= 0 ? f->maxBounce : default_bounce(f->integrator);
  if (!first.isHit) {
    color = sampleHdr(cx, dir);
  } else {
    v3 Le = first.material.emissive;
    v3 Li;
    if (f->integrator == ORC_LAMBERT_O) Li = pt_lambert(cx, first, mb, &seed);
    else if (f->integrator == ORC_DISNEY_UNIFORM_D) Li = pt_disney_uniform(cx, first, mb, &seed);
    else Li = pt_mis(cx, first, mb, &seed, px, py, sidx);
    color = add(Le, Li);
  }
  float* a = accum + 4 * ((size_t)py * W + px);
  cx->c.texels++; /* lastFrame read, IS:868 */
  float w = 1.0f / (float)(f->frameCounter + 1u);
  a[0] = mixf(a[0], color.x, w);
  a[1] = mixf(a[1], color.y, w);
  a[2] = mixf(a[2], color.z, w);
  a[3] = 1.0f;
}

/* ---------------------------------------------------- BASIC (CPU tracer B) */
/* The arithmetic is the reference binary's: glm vec3 is float, the Material
 * rates, the sphere radius, HitResult::distance and the image are double
 * (B:49-68, :130, :356), and every mixed expression is evaluated in the type
 * C++ promotes it to. Pinned byte for byte against the reference compiled here
 * (tests/golden/basic/, oracle/ref_basic.cpp; test_basic_serial_equals_reference). */
typedef struct {
  int isHit;
  double distance;
  v3 hitPoint;
  v3 normal, color;
  int emissive;
  double specularRate, roughness, refractRate, refractAngle, refractRoughness;
} BHit;

/* The random stream. ORC_RNG_COUNTER: a per-pixel wang-hash stream (the
 * parallel CPU baseline and the GPU kernel); ORC_RNG_MT19937: the reference's
 * one global std::mt19937 read through uniform_real_distribution<double>
 * (B:208-214), consumed in the reference's serial loop order. */
typedef struct { uint32_t mt[624]; int idx; } Mt19937;
static void mt_seed(Mt19937* m, uint32_t s) {
  m->mt[0] = s;
  for (int i = 1; i < 624; i++) m->mt[i] = 1812433253u * (m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) + (uint32_t)i;
  m->idx = 624;
}
static uint32_t mt_next(Mt19937* m) {
  if (m->idx >= 624) {
    for (int i = 0; i < 624; i++) {
      uint32_t y = (m->mt[i] & 0x80000000u) | (m->mt[(i + 1) % 624] & 0x7fffffffu);
      m->mt[i] = m->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    m->idx = 0;
  }
  uint32_t y = m->mt[m->idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
/* libstdc++ generate_canonical<double, 53> over a 32-bit engine: two draws,
 * (g1 + g2 * 2^32) / 2^64 summed in double, 1.0 mapped to the largest double
 * below it; uniform_real_distribution(0, 1) returns it unchanged (x * 1 + 0). */
static double mt_canonical(Mt19937* m) {
  double sum = (double)mt_next(m);
  sum += (double)mt_next(m) * 4294967296.0;
  double r = sum / 18446744073709551616.0;
  if (r >= 1.0) r = nextafter(1.0, 0.0);
  return r;
}

enum { ORC_RNG_COUNTER = 0, ORC_RNG_MT19937 = 1 };
typedef struct {
  int kind;
  uint32_t seed;     /* counter */
  Mt19937* mt;       /* mt19937 */
  int64_t draws;     /* randf() calls so far (mt19937) */
} BRng;
/* randf B:211-214 */
static double b_rand(BRng* g) {
  if (g->kind == ORC_RNG_MT19937) { g->draws++; return mt_canonical(g->mt); }
  return (double)wang(&g->seed) / 4294967296.0;
}

static void bfill(BHit* r, const double* sh) {
  r->color = V3((float)sh[10], (float)sh[11], (float)sh[12]);
  r->emissive = sh[16] != 0.0;
  r->specularRate = sh[17]; r->roughness = sh[18]; r->refractRate = sh[19];
  r->refractAngle = sh[20]; r->refractRoughness = sh[21];
}
/* Triangle::intersect B:90-122: the accept test and distance; the winner's normal
 * (n, flipped to face the ray) and material are filled in once by b_shoot. */
static int b_tri(const double* sh, v3 S, v3 d, float* tOut, v3* POut) {
  v3 p1 = V3((float)sh[1], (float)sh[2], (float)sh[3]), p2 = V3((float)sh[4], (float)sh[5], (float)sh[6]);
  v3 p3 = V3((float)sh[7], (float)sh[8], (float)sh[9]);
  v3 n = V3((float)sh[13], (float)sh[14], (float)sh[15]);
  v3 N = n;
  if (dot(N, d) > 0.0f) N = neg(N);
  if (fabsf(dot(N, d)) < 0.00001f) return 0;
  float t = (dot(N, p1) - dot(S, N)) / dot(d, N);
  if (t < 0.0005f) return 0;
  v3 P = add(S, scl(d, t));
  v3 c1 = cross(sub(p2, p1), sub(P, p1));
  v3 c2 = cross(sub(p3, p2), sub(P, p2));
  v3 c3 = cross(sub(p1, p3), sub(P, p3));
  if (dot(c1, n) < 0 || dot(c2, n) < 0 || dot(c3, n) < 0) return 0;
  *tOut = t;
  *POut = P;
  return 1;
}
/* Sphere::intersect B:135-164: OS, SH, t are float (glm length / dot); pow(x, 2)
 * of a float is exact in double; R is double, so OH > R and PH are double
 * expressions (pow(R, 2) == R * R for the scene's radii, test_basic_sphere_pow);
 * length(SH) of a float is |SH|. */
static int b_sphere(const double* sh, v3 S, v3 d, float* tOut, v3* POut) {
  v3 O = V3((float)sh[1], (float)sh[2], (float)sh[3]);
  double R = sh[22];
  v3 OSv = sub(O, S);
  float OS = sqrtf(dot(OSv, OSv));
  float SH = dot(OSv, d);
  float OH = (float)sqrt((double)OS * (double)OS - (double)SH * (double)SH);
  if ((double)OH > R) return 0;
  float PH = (float)sqrt(R * R - (double)OH * (double)OH);
  float t1 = fabsf(SH) - PH;
  float t2 = fabsf(SH) + PH;
  float t = (t1 < 0) ? t2 : t1;
  v3 P = add(S, scl(d, t));
  if (fabsf(t1) < 0.0005f || fabsf(t2) < 0.0005f) return 0;
  *tOut = t;
  *POut = P;
  return 1;
}
/* shoot B:192-205 (res.distance is a double initialised from 1145141919.810f): the
 * first shape at the least distance wins; only its HitResult is formed */
static BHit b_shoot(Ctx* cx, v3 S, v3 d) {
  const orc_scene* s = cx->s;
  BHit res;
  res.isHit = 0;
  res.distance = (double)1145141919.810f;
  cx->c.rays++;
  int win = -1;
  v3 wP = V3(0, 0, 0);
  for (int k = 0; k < s->nShapes; k++) {
    const double* sh = s->shapes + (size_t)k * ORC_SHAPE_DOUBLES;
    float t;
    v3 P;
    const int h = (sh[0] == 1.0) ? b_sphere(sh, S, d, &t, &P) : b_tri(sh, S, d, &t, &P);
    if (h && (double)t < res.distance) {
      res.distance = t;
      win = k;
      wP = P;
    }
  }
  if (win < 0) return res;
  const double* sh = s->shapes + (size_t)win * ORC_SHAPE_DOUBLES;
  res.isHit = 1;
  res.hitPoint = wP;
  bfill(&res, sh);
  if (sh[0] == 1.0) {
    res.normal = normalize(sub(wP, V3((float)sh[1], (float)sh[2], (float)sh[3])));
  } else {
    v3 N = V3((float)sh[13], (float)sh[14], (float)sh[15]);
    if (dot(N, d) > 0.0f) N = neg(N);
    res.normal = N;
  }
  return res;
}
/* randomVec3 B:217-234: vec3(randf(), randf(), randf()) -- the compiled reference
 * evaluates the three arguments right to left (g++ and MSVC on x86-64), so z takes
 * the first draw; 2.0f * v - vec3(1) in float, dot(d, d) > 1.0 in double.
 * randomDirection B:237-250. */
static v3 b_randomDirection(v3 n, BRng* g) {
  v3 d;
  do {
    double z = b_rand(g), y = b_rand(g), x = b_rand(g);
    d = sub(scl(V3((float)x, (float)y, (float)z), 2.0f), V3(1, 1, 1));
  } while ((double)dot(d, d) > 1.0);
  return normalize(add(normalize(d), n));
}
/* glm reflect (func_geometric.inl:104-110): I - N * dot(N, I) * 2 */
static v3 b_reflect(v3 I, v3 N) { return sub(I, scl(scl(N, dot(N, I)), 2.0f)); }
/* glm refract (func_geometric.inl:113-123) */
static v3 b_refract(v3 I, v3 N, float eta) {
  float dotValue = dot(N, I);
  float k = 1.0f - eta * eta * (1.0f - dotValue * dotValue);
  if (!(k >= 0.0f)) return V3(0, 0, 0);
  return sub(scl(I, eta), scl(N, eta * dotValue + sqrtf(k)));
}
/* glm mix(vec3, vec3, double) (func_common.inl:103-111): computed in double, stored as float */
static v3 b_mixd(v3 x, v3 y, double a) {
  const double b = 1.0 - a;
  return V3((float)((double)x.x * b + (double)y.x * a), (float)((double)x.y * b + (double)y.y * a),
            (float)((double)x.z * b + (double)y.z * a));
}
/* One lobe choice + new direction, shared by the primary vertex (B:399-422) and
 * pathTracing (B:268-294). Returns the lobe: 0 specular, 1 refract, 2 diffuse. */
static int b_lobe(const BHit* res, v3 din, BRng* g, v3* dout) {
  v3 rd = b_randomDirection(res->normal, g);
  double r = b_rand(g);
  if (r < res->specularRate) {
    v3 ref = normalize(b_reflect(din, res->normal));
    *dout = b_mixd(ref, rd, res->roughness);
    return 0;
  } else if (res->specularRate <= r && r <= res->refractRate) {
    v3 ref = normalize(b_refract(din, res->normal, (float)res->refractAngle));
    *dout = b_mixd(ref, neg(rd), res->refractRoughness);
    return 1;
  }
  *dout = rd;
  return 2;
}
#define ORC_BASIC_MAX_DEPTH 64
/* pathTracing B:252-297 from depth 0. The recursion's products are formed on the
 * way back up (color = pathTracing(depth + 1) * cosine [* srcColor], / P), so each
 * vertex's factors are kept and folded from the deepest vertex upward. */
static v3 b_path(Ctx* cx, v3 S, v3 d, int maxDepth, BRng* g) {
  float cosv[ORC_BASIC_MAX_DEPTH + 1];
  v3 col[ORC_BASIC_MAX_DEPTH + 1];
  int diffuse[ORC_BASIC_MAX_DEPTH + 1];
  const float P = 0.8f; /* B:264 float P = 0.8 */
  v3 v = V3(0, 0, 0);
  int n = 0;
  if (maxDepth > ORC_BASIC_MAX_DEPTH) maxDepth = ORC_BASIC_MAX_DEPTH;
  for (int depth = 0;; depth++) {
    if (depth > maxDepth) break;
    BHit res = b_shoot(cx, S, d);
    if (!res.isHit) break;
    if (res.emissive) { v = res.color; break; }
    double r = b_rand(g);
    if (r > (double)P) break;
    v3 nd;
    int lobe = b_lobe(&res, d, g, &nd);  /* randomDirection, then randf() (B:270, :276) */
    cosv[n] = fabsf(dot(neg(d), res.normal));
    col[n] = res.color;
    diffuse[n] = lobe == 2;
    n++;
    S = res.hitPoint;
    d = nd;
  }
  for (int k = n - 1; k >= 0; k--) {
    v = scl(v, cosv[k]);
    if (diffuse[k]) v = mul(v, col[k]);
    v = sdiv(v, P);
  }
  return v;
}
/* pixel loop body B:367-429 for pixel (j, i) of one sample: the value added to image */
static v3 b_pixel(Ctx* cx, int j, int i, int W, int H, int maxDepth, float brightness, BRng* g) {
  double xd = 2.0 * (double)j / (double)W - 1.0;
  double yd = 2.0 * (double)(H - i) / (double)H - 1.0;
  xd += (b_rand(g) - 0.5) / (double)W;
  yd += (b_rand(g) - 0.5) / (double)H;
  v3 coord = V3((float)xd, (float)yd, (float)1.1);  /* SCREEN_Z B:27 is a double */
  v3 dir = normalize(sub(coord, V3(0, 0, 4.0f)));
  BHit res = b_shoot(cx, coord, dir);
  v3 color = V3(0, 0, 0);
  if (res.isHit) {
    if (res.emissive) {
      color = res.color;
    } else {
      v3 nd;
      int lobe = b_lobe(&res, dir, g, &nd);
      v3 pt = b_path(cx, res.hitPoint, nd, maxDepth, g);
      color = (lobe == 2) ? mul(pt, res.color) : pt;
      color = scl(color, brightness); /* color *= BRIGHTNESS: glm casts the double to float */
    }
  }
  return color;
}
/* BRIGHTNESS B:20: (2.0f * 3.1415926f) * (1.0f / double(SAMPLE)), a double */
static float b_brightness(int samples) { return (float)((double)(2.0f * 3.1415926f) * (1.0 / (double)samples)); }

/* one sample of pixel (j, i) with the counter stream, added to the double image */
static void shade_basic_pixel(Ctx* cx, const orc_frame* f, int j, int i, float* accum) {
  const int W = f->width, H = f->height;
  uint32_t k = sample_index(f);
  BRng g;
  memset(&g, 0, sizeof(g));
  g.kind = ORC_RNG_COUNTER;
  g.seed = ((uint32_t)j * 1973u + (uint32_t)i * 9277u + k * 26699u + f->basicSeed * 0x9E3779B9u) | 1u;
  int maxDepth = f->maxBounce >= 0 ? f->maxBounce : 8;
  v3 color = b_pixel(cx, j, i, W, H, maxDepth, b_brightness(f->basicSamples), &g);
  double* im = f->basicImage + 3 * ((size_t)i * W + j);
  if (f->frameCounter == 0) im[0] = im[1] = im[2] = 0.0;  /* sample 0 starts the image (B:356-357) */
  im[0] += color.x; im[1] += color.y; im[2] += color.z;
  float* a = accum + 4 * ((size_t)i * W + j);
  a[0] = (float)im[0]; a[1] = (float)im[1]; a[2] = (float)im[2]; a[3] = 1.0f;
}

int orc_basic_serial(const orc_scene* s, int W, int H, int samples, uint32_t seed, int maxDepth, double* image,
                     int64_t* offsets, int64_t* nDraws, orc_counters* counters) {
  if (!s || !image || W <= 0 || H <= 0 || samples <= 0) return -1;
  Mt19937* mt = (Mt19937*)malloc(sizeof(Mt19937));
  if (!mt) return -3;
  mt_seed(mt, seed);
  Ctx cx;
  cx.s = s;
  memset(&cx.c, 0, sizeof(cx.c));
  BRng g;
  memset(&g, 0, sizeof(g));
  g.kind = ORC_RNG_MT19937;
  g.mt = mt;
  const float br = b_brightness(samples);
  memset(image, 0, sizeof(double) * (size_t)W * H * 3);
  for (int k = 0; k < samples; k++)          /* B:361-432, serial as shipped (no /openmp) */
    for (int i = 0; i < H; i++)
      for (int j = 0; j < W; j++) {
        if (offsets) offsets[((size_t)k * H + i) * W + j] = g.draws;
        v3 c = b_pixel(&cx, j, i, W, H, maxDepth, br, &g);
        double* p = image + 3 * ((size_t)i * W + j);
        p[0] += c.x; p[1] += c.y; p[2] += c.z;
      }
  if (nDraws) *nDraws = g.draws;
  if (counters) *counters = cx.c;
  free(mt);
  return 0;
}

int orc_mt_doubles(uint32_t seed, int64_t n, double* out) {
  if (n < 0 || (n > 0 && !out)) return -1;
  Mt19937* mt = (Mt19937*)malloc(sizeof(Mt19937));
  if (!mt) return -3;
  mt_seed(mt, seed);
  for (int64_t k = 0; k < n; k++) out[k] = mt_canonical(mt);
  free(mt);
  return 0;
}

/* ------------------------------------------------------------ entry points */
int orc_render_pixels(const orc_scene* s, const orc_frame* f, const int* pix, int nPix,
                      float* accum, int nthreads, orc_counters* counters) {
  if (!s || !f || !accum) return -1;
  if (f->integrator != ORC_BASIC_CPU_COMPAT && (!s->tris || !s->nodes || s->nNodes < 2)) return -2;
  if (f->integrator == ORC_BASIC_CPU_COMPAT && (!s->shapes || !f->basicImage)) return -2;
  long total = pix ? nPix : (long)f->width * f->height;
  orc_counters sum = {0, 0, 0, 0, 0};
#ifdef _OPENMP
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
  {
    Ctx cx;
    cx.s = s;
    memset(&cx.c, 0, sizeof(cx.c));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
    for (long k = 0; k < total; k++) {
      int px, py;
      if (pix) { px = pix[2 * k]; py = pix[2 * k + 1]; }
      else { px = (int)(k % f->width); py = (int)(k / f->width); }
      if (f->integrator == ORC_BASIC_CPU_COMPAT) shade_basic_pixel(&cx, f, px, py, accum);
      else shade_gl_pixel(&cx, f, px, py, accum);
    }
#ifdef _OPENMP
#pragma omp critical
#endif
    {
      sum.rays += cx.c.rays; sum.nodes += cx.c.nodes; sum.tris += cx.c.tris;
      sum.mats += cx.c.mats; sum.texels += cx.c.texels;
    }
  }
  if (counters) *counters = sum;
  return 0;
}

int orc_trace_closest(const orc_scene* s, const float* rays, int n, float* t_out, int* tri_out,
                      int brute, orc_counters* counters) {
  Ctx cx;
  cx.s = s;
  memset(&cx.c, 0, sizeof(cx.c));
  for (int k = 0; k < n; k++) {
    v3 S = V3(rays[6 * k], rays[6 * k + 1], rays[6 * k + 2]);
    v3 d = V3(rays[6 * k + 3], rays[6 * k + 4], rays[6 * k + 5]);
    Hit h = brute ? hitArray(&cx, S, d, 0, s->nTriangles - 1) : hitBVH(&cx, S, d);
    t_out[k] = h.isHit ? h.distance : INF;
    tri_out[k] = h.isHit ? h.tri : -1;
  }
  if (counters) *counters = cx.c;
  return 0;
}

uint32_t orc_wang_hash(uint32_t seed) { return wang(&seed); }
float orc_sobol(uint32_t d, uint32_t i) { return sobolf(d, i); }
/* RNG stream of one pixel: seed (IS:73-76) then n successive rand() values */
void orc_pixel_rng(int px, int py, uint32_t frameCounter, int n, float* out) {
  uint32_t seed = ((uint32_t)px * 1973u + (uint32_t)py * 9277u + frameCounter * 26699u) | 1u;
  for (int k = 0; k < n; k++) out[k] = randf(&seed);
}

/* calculateHdrCache IS main.cpp:555-652. The luminance weights are double
 * literals in the C++ source, so lum is computed in double and stored as f32. */
static int lower_bound_f(const float* a, int n, float x) {
  int lo = 0, hi = n;
  while (lo < hi) { int mid = lo + (hi - lo) / 2; if (a[mid] < x) lo = mid + 1; else hi = mid; }
  return lo;
}
int orc_hdr_cache(const float* HDR, int width, int height, float* cache) {
  if (!HDR || !cache || width <= 0 || height <= 0) return -1;
  size_t n = (size_t)width * height;
  float* pdf = (float*)malloc(n * sizeof(float));
  float* margin = (float*)calloc((size_t)width, sizeof(float));
  float* cdfx = (float*)malloc((size_t)width * sizeof(float));
  float* cdfy = (float*)malloc(n * sizeof(float)); /* transposed: [x][y] */
  if (!pdf || !margin || !cdfx || !cdfy) { free(pdf); free(margin); free(cdfx); free(cdfy); return -3; }
  float lumSum = 0.0f;
  for (int i = 0; i < height; i++)
    for (int j = 0; j < width; j++) {
      size_t k = (size_t)i * width + j;
      float R = HDR[3 * k], G = HDR[3 * k + 1], B = HDR[3 * k + 2];
      float lum = (float)(0.2 * R + 0.7 * G + 0.1 * B);
      pdf[k] = lum;
      lumSum += lum;
    }
  for (size_t k = 0; k < n; k++) pdf[k] /= lumSum;
  for (int j = 0; j < width; j++)
    for (int i = 0; i < height; i++) margin[j] += pdf[(size_t)i * width + j];
  for (int j = 0; j < width; j++) cdfx[j] = margin[j];
  for (int j = 1; j < width; j++) cdfx[j] += cdfx[j - 1];
  for (int j = 0; j < width; j++) {
    for (int i = 0; i < height; i++) cdfy[(size_t)j * height + i] = pdf[(size_t)i * width + j] / margin[j];
    for (int i = 1; i < height; i++) cdfy[(size_t)j * height + i] += cdfy[(size_t)j * height + i - 1];
  }
  for (int j = 0; j < width; j++)
    for (int i = 0; i < height; i++) {
      float xi_1 = (float)i / height;
      float xi_2 = (float)j / width;
      int x = lower_bound_f(cdfx, width, xi_1);
      /* x == width (cdf rounding below xi_1) indexes past cdf_y_condiciton in the
       * reference (UB); the row lookup is clamped, the stored x/width is not. */
      int xr = x < width ? x : width - 1;
      int y = lower_bound_f(cdfy + (size_t)xr * height, height, xi_2);
      size_t k = (size_t)i * width + j;
      cache[3 * k] = (float)x / width;
      cache[3 * k + 1] = (float)y / height;
      cache[3 * k + 2] = pdf[k];
    }
  free(pdf); free(margin); free(cdfx); free(cdfy);
  return 0;
}

/* ------------------------------------------------- per-function parity hooks */
/* Function fn of this restatement on n inputs, in the layout of the reference
 * shader harness's ref_glsl_fn (oracle/ref_glsl.cpp: the pass1.fsh text compiled
 * as C++), so tests/test_glsl_ref.py can compare them on random inputs. Each case
 * calls the function the integrators call, composed as the integrators compose it. */
static inline uint32_t o_ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float o_fbits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline v3 o_v3(const float* p) { return V3(p[0], p[1], p[2]); }
static inline void o_put3(float* o, v3 v) { o[0] = v.x; o[1] = v.y; o[2] = v.z; }
static Material o_mat(const float* p) {
  Material m;
  m.emissive = o_v3(p); m.baseColor = o_v3(p + 3);
  m.subsurface = p[6]; m.metallic = p[7]; m.specular = p[8]; m.specularTint = p[9];
  m.roughness = p[10]; m.anisotropic = p[11]; m.sheen = p[12]; m.sheenTint = p[13];
  m.clearcoat = p[14]; m.clearcoatGloss = p[15]; m.IOR = p[16]; m.transmission = p[17];
  return m;
}
static const int O_FN_IN[] = {1, 2, 2, 6, 6, 3, 24, 12, 1, 2, 2, 5, 2, 5, 33, 33, 27, 27, 5, 9, 9, 26, 3, 2, 1};
static const int O_FN_OUT[] = {2, 1, 2, 2, 3, 6, 9, 1, 1, 1, 1, 1, 1, 1, 3, 3, 3, 1, 3, 3, 3, 3, 2, 1, 4};

int orc_glsl_fn(int fn, const float* in, float* out, int n) {
  if (fn < 0 || fn >= (int)(sizeof(O_FN_IN) / sizeof(O_FN_IN[0])) || n < 0) return -1;
  for (int k = 0; k < n; k++) {
    const float* a = in + (size_t)k * O_FN_IN[fn];
    float* o = out + (size_t)k * O_FN_OUT[fn];
    switch (fn) {
      case 0: { uint32_t sd = o_ubits(a[0]); uint32_t r = wang(&sd); o[0] = o_fbits(r); o[1] = o_fbits(sd); break; }
      case 1: o[0] = sobolf(o_ubits(a[0]), o_ubits(a[1])); break;
      case 2: {  /* sobolVec2(frameCounter + 1, bounce) as pt_mis forms it */
        uint32_t gi = grayCode(o_ubits(a[0]));
        uint32_t b = o_ubits(a[1]);
        o[0] = sobolf(2u * b, gi);
        o[1] = sobolf(2u * b + 1u, gi);
        break;
      }
      case 3: { float u = a[4], v = a[5]; cranley_patterson((int)a[0], (int)a[1], &u, &v); o[0] = u; o[1] = v; break; }
      case 4: o_put3(o, toNormalHemisphere(o_v3(a), o_v3(a + 3))); break;
      case 5: { v3 t, b; getTangent(o_v3(a), &t, &b); o_put3(o, t); o_put3(o + 3, b); break; }
      case 6: {
        Tri t;
        t.p1 = o_v3(a); t.p2 = o_v3(a + 3); t.p3 = o_v3(a + 6);
        t.n1 = o_v3(a + 9); t.n2 = o_v3(a + 12); t.n3 = o_v3(a + 15);
        Hit h = hitTriangle(t, o_v3(a + 18), o_v3(a + 21));
        o[0] = h.isHit ? 1.0f : 0.0f; o[1] = h.isInside ? 1.0f : 0.0f; o[2] = h.distance;
        o_put3(o + 3, h.isHit ? h.hitPoint : V3(0, 0, 0)); o_put3(o + 6, h.isHit ? h.normal : V3(0, 0, 0));
        break;
      }
      case 7: o[0] = hitAABB(o_v3(a), o_v3(a + 3), o_v3(a + 6), o_v3(a + 9)); break;
      case 8: o[0] = SchlickFresnel(a[0]); break;
      case 9: o[0] = GTR1(a[0], a[1]); break;
      case 10: o[0] = GTR2(a[0], a[1]); break;
      case 11: o[0] = GTR2_aniso(a[0], a[1], a[2], a[3], a[4]); break;
      case 12: o[0] = smithG_GGX(a[0], a[1]); break;
      case 13: o[0] = smithG_GGX_aniso(a[0], a[1], a[2], a[3], a[4]); break;
      case 14: case 15: {
        Material m = o_mat(a + 15);
        o_put3(o, BRDF_Evaluate_aniso(o_v3(a), o_v3(a + 3), o_v3(a + 6), o_v3(a + 9), o_v3(a + 12), &m));
        break;
      }
      case 16: { Material m = o_mat(a + 9); o_put3(o, BRDF_Evaluate(o_v3(a), o_v3(a + 3), o_v3(a + 6), &m)); break; }
      case 17: { Material m = o_mat(a + 9); o[0] = BRDF_Pdf(o_v3(a), o_v3(a + 3), o_v3(a + 6), &m); break; }
      case 18: o_put3(o, SampleCosineHemisphere(a[0], a[1], o_v3(a + 2))); break;
      case 19: o_put3(o, SampleGTR2(a[0], a[1], o_v3(a + 2), o_v3(a + 5), a[8])); break;
      case 20: o_put3(o, SampleGTR1(a[0], a[1], o_v3(a + 2), o_v3(a + 5), a[8])); break;
      case 21: { Material m = o_mat(a + 8); o_put3(o, SampleBRDF(a[0], a[1], a[2], o_v3(a + 3), o_v3(a + 6), &m)); break; }
      case 22: { float u, w; toSpherical(o_v3(a), &u, &w); o[0] = u; o[1] = w; break; }
      case 23: o[0] = misMixWeight(a[0], a[1]); break;
      case 24: { uint32_t sd = o_ubits(a[0]); o_put3(o, SampleHemisphereRand(&sd)); o[3] = o_fbits(sd); break; }
    }
  }
  return 0;
}
