// pt_kernels.hip -- MI355X (gfx950) kernels of the progressive path tracer:
// BVH traversal, triangle test, the three pass1.fsh integrators, the
// BasicRayTracingWithC++ integrator, pass3 tonemap and the multi-GPU tile
// pack/unpack. Host-side launchers live in pt_runtime.cpp.
//
// Execution model (DESIGN.md "Kernels"):
//  * persistent grid sized to residency; each wave64 dequeues 8x8 pixel tiles
//    from 8 per-XCD-group work counters (blockIdx % 8), stealing when its own
//    queue drains;
//  * one lane per pixel runs the whole path (megakernel): ray gen, closest-hit
//    traversal, env any-hit shadow rays, BRDF/MIS, running-mean accumulate;
//  * traversal keeps the current node in registers and the deferred siblings in
//    an LDS stack (LDS_STACK entries per lane, lane-interleaved so a wave's
//    push/pop is bank-conflict free) that spills to a per-thread HBM region
//    only for trees deeper than LDS_STACK;
//  * node records are re-laid out at upload as 64-byte "wide" records holding
//    both children's boxes (one dependent fetch per visited internal node
//    instead of the reference's three); triangles as 64-byte records with the
//    precomputed unit normal and plane offset.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_device.h"
#include "pt_kernels.h"

namespace pt {

__constant__ uint32_t kSobolV[8 * 32] = {
    2147483648u,1073741824u,536870912u,268435456u,134217728u,67108864u,33554432u,16777216u,8388608u,4194304u,2097152u,1048576u,524288u,262144u,131072u,65536u,32768u,16384u,8192u,4096u,2048u,1024u,512u,256u,128u,64u,32u,16u,8u,4u,2u,1u,
    2147483648u,3221225472u,2684354560u,4026531840u,2281701376u,3422552064u,2852126720u,4278190080u,2155872256u,3233808384u,2694840320u,4042260480u,2290614272u,3435921408u,2863267840u,4294901760u,2147516416u,3221274624u,2684395520u,4026593280u,2281736192u,3422604288u,2852170240u,4278255360u,2155905152u,3233857728u,2694881440u,4042322160u,2290649224u,3435973836u,2863311530u,4294967295u,
    2147483648u,3221225472u,1610612736u,2415919104u,3892314112u,1543503872u,2382364672u,3305111552u,1753219072u,2629828608u,3999268864u,1435500544u,2154299392u,3231449088u,1626210304u,2421489664u,3900735488u,1556135936u,2388680704u,3314585600u,1751705600u,2627492864u,4008611328u,1431684352u,2147543168u,3221249216u,1610649184u,2415969680u,3892340840u,1543543964u,2382425838u,3305133397u,
    2147483648u,3221225472u,536870912u,1342177280u,4160749568u,1946157056u,2717908992u,2466250752u,3632267264u,624951296u,1507852288u,3872391168u,2013790208u,3020685312u,2181169152u,3271884800u,546275328u,1363623936u,4226424832u,1977167872u,2693105664u,2437829632u,3689389568u,635137280u,1484783744u,3846176960u,2044723232u,3067084880u,2148008184u,3222012020u,537002146u,1342505107u,
    2147483648u,1073741824u,536870912u,2952790016u,4160749568u,3690987520u,2046820352u,2634022912u,1518338048u,801112064u,2707423232u,4038066176u,3666345984u,1875116032u,2170683392u,1085997056u,579305472u,3016343552u,4217741312u,3719483392u,2013407232u,2617981952u,1510979072u,755882752u,2726789248u,4090085440u,3680870432u,1840435376u,2147625208u,1074478300u,537900666u,2953698205u,
    2147483648u,1073741824u,1610612736u,805306368u,2818572288u,335544320u,2113929216u,3472883712u,2290089984u,3829399552u,3059744768u,1127219200u,3089629184u,4199809024u,3567124480u,1891565568u,394297344u,3988799488u,920674304u,4193267712u,2950604800u,3977188352u,3250028032u,129093376u,2231568512u,2963678272u,4281226848u,432124720u,803643432u,1633613396u,2672665246u,3170194367u,
    2147483648u,3221225472u,2684354560u,3489660928u,1476395008u,2483027968u,1040187392u,3808428032u,3196059648u,599785472u,505413632u,4077912064u,1182269440u,1736704000u,2017853440u,2221342720u,3329785856u,2810494976u,3628507136u,1416089600u,2658719744u,864310272u,3863387648u,3076993792u,553150080u,272922560u,4167467040u,1148698640u,1719673080u,2009075780u,2149644390u,3222291575u,
    2147483648u,1073741824u,2684354560u,1342177280u,2281701376u,1946157056u,436207616u,2566914048u,2625634304u,3208642560u,2720006144u,2098200576u,111673344u,2354315264u,3464626176u,4027383808u,2886631424u,3770826752u,1691164672u,3357462528u,1993345024u,3752330240u,873073152u,2870150400u,1700563072u,87021376u,1097028000u,1222351248u,1560027592u,2977959924u,23268898u,437609937u};

// ----------------------------------------------------------------- counters
struct Counters {
  uint32_t rays, nodes, tris, mats, texels;
};

// ----------------------------------------------------------------- stack
// LDS stack of LDS_STACK entries per lane, entry e of thread t at
// lds[(e % LDS_STACK) * BLOCK + t]; entries older than the newest LDS_STACK
// live in the thread's HBM overflow region gbl[e] (only when the tree is
// deeper than LDS_STACK).
struct Stack {
  int* lds;   // &s_stack[threadIdx.x]
  int* gbl;   // overflow region (may be null when maxStack <= LDS_STACK)
  int sp;
  __device__ __forceinline__ void push(int v) {
    int slot = sp & (LDS_STACK - 1);
    if (sp >= LDS_STACK) gbl[sp - LDS_STACK] = lds[slot * BLOCK];
    lds[slot * BLOCK] = v;
    sp++;
  }
  __device__ __forceinline__ int pop() {
    sp--;
    int slot = sp & (LDS_STACK - 1);
    int v = lds[slot * BLOCK];
    if (sp >= LDS_STACK) lds[slot * BLOCK] = gbl[sp - LDS_STACK];
    return v;
  }
};

// hitAABB IS:303-316 with the precomputed reciprocal direction (the reference
// recomputes the same 1/d per box). Returns the reference's d; t0 (the slab
// entry) is returned for culling.
__device__ __forceinline__ float hitAABB(V3 o, V3 inv, float4 lo, float4 hi, float& t0out) {
  float fx = (hi.x - o.x) * inv.x, fy = (hi.y - o.y) * inv.y, fz = (hi.z - o.z) * inv.z;
  float nx = (lo.x - o.x) * inv.x, ny = (lo.y - o.y) * inv.y, nz = (lo.z - o.z) * inv.z;
  float t1 = fminf(fmaxf(fx, nx), fminf(fmaxf(fy, ny), fmaxf(fz, nz)));
  float t0 = fmaxf(fminf(fx, nx), fmaxf(fminf(fy, ny), fminf(fz, nz)));
  t0out = t0;
  return (t1 >= t0) ? ((t0 > 0.0f) ? t0 : t1) : -1.0f;
}

// hitTriangle IS:251-301, accept/reject and distance only. With the stored unit
// normal Ng = normalize(cross(p2-p1,p3-p1)) and w = dot(Ng,p1) (computed on the
// host in the reference's order) this rounds exactly like the reference: the
// orientation flip negates numerator, denominator and all three edge tests
// exactly, so it changes neither t nor the accept decision.
__device__ __forceinline__ bool triHit(const float4* g, V3 o, V3 d, float& t) {
  float4 A = g[0], B = g[1], C = g[2], Nn = g[3];
  V3 N = v3(Nn.x, Nn.y, Nn.z);
  float dn = dot(N, d);
  if (fabsf(dn) < 0.00001f) return false;
  float tt = (A.w - dot(o, N)) / dn;
  if (tt < 0.0005f) return false;
  V3 p1 = v3(A.x, A.y, A.z), p2 = v3(B.x, B.y, B.z), p3 = v3(C.x, C.y, C.z);
  V3 P = o + d * tt;
  float s1 = dot(cross(p2 - p1, P - p1), N);
  float s2 = dot(cross(p3 - p2, P - p2), N);
  float s3 = dot(cross(p1 - p3, P - p3), N);
  bool r1 = (s1 > 0 && s2 > 0 && s3 > 0);
  bool r2 = (s1 < 0 && s2 < 0 && s3 < 0);
  t = tt;
  return r1 || r2;
}

// hitBVH IS:335-382: same visiting order (nearer child by the reference's d
// first, ties to the right child), strict '<' closest update, so the same
// triangle wins. CULL skips children whose slab entry lies beyond the current
// closest hit (plus a margin); ANYHIT returns on the first accepted triangle
// (used for env shadow rays, where only isHit is read: IS:776-779).
template <bool ANYHIT, bool CULL, bool COUNT>
__device__ int traceRay(const SceneView& S, V3 o, V3 d, float& tOut, Stack& st, Counters& C) {
  V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float tbest = PT_INF;
  int best = -1;
  int ref = S.rootRef;
  st.sp = 0;
  C.rays++;
  while (true) {
    if (ref >= 0) {
      const float4* nd = S.bvh + 4 * (size_t)ref;
      float4 la = nd[0], lb = nd[1], ra = nd[2], rb = nd[3];
      int lref = __float_as_int(la.w), rref = __float_as_int(lb.w);
      float t0l, t0r;
      float d1 = hitAABB(o, inv, la, lb, t0l);
      float d2 = hitAABB(o, inv, ra, rb, t0r);
      bool h1 = (lref != REF_NONE) && d1 > 0.0f;
      bool h2 = (rref != REF_NONE) && d2 > 0.0f;
      if (COUNT) C.nodes += 1u + (lref != REF_NONE) + (rref != REF_NONE);
      if (CULL) {
        float lim = tbest + 1e-3f * fmaxf(1.0f, tbest);
        h1 = h1 && !(t0l > lim);
        h2 = h2 && !(t0r > lim);
      }
      if (h1 && h2) {
        bool leftFirst = d1 < d2;
        st.push(leftFirst ? rref : lref);
        ref = leftFirst ? lref : rref;
        continue;
      }
      if (h1) { ref = lref; continue; }
      if (h2) { ref = rref; continue; }
    } else if (ref != REF_NONE) {
      uint32_t v = ~(uint32_t)ref;
      int start = (int)(v >> LEAF_CNT_BITS);
      int cnt = (int)(v & ((1u << LEAF_CNT_BITS) - 1u)) + 1;
      if (COUNT) C.nodes++;
      float localBest = PT_INF;
      for (int k = 0; k < cnt; k++) {
        int i = start + k;
        float t;
        bool hit = triHit(S.geo + 4 * (size_t)i, o, d, t);
        if (COUNT) {
          C.tris++;
          if (hit && t < localBest) { localBest = t; C.mats++; }
        }
        if (hit && t < tbest) {
          tbest = t;
          best = i;
          if (ANYHIT) { tOut = tbest; return best; }
        }
      }
    }
    if (st.sp == 0) break;
    ref = st.pop();
  }
  tOut = tbest;
  return best;
}

// The full HitResult (IS:63-71) of the winning triangle, computed once.
struct Hit {
  V3 P, N, viewDir;
  Material m;
};
__device__ __forceinline__ void finishHit(const SceneView& S, int tri, V3 o, V3 d, float t, Hit& h) {
  const float4* g = S.geo + 4 * (size_t)tri;
  float4 A = g[0], B = g[1], C4 = g[2], Nn = g[3];
  V3 p1 = v3(A.x, A.y, A.z), p2 = v3(B.x, B.y, B.z), p3 = v3(C4.x, C4.y, C4.z);
  bool inside = dot(v3(Nn.x, Nn.y, Nn.z), d) > 0.0f;
  V3 P = o + d * t;
  float alpha = (-(P.x - p2.x) * (p3.y - p2.y) + (P.y - p2.y) * (p3.x - p2.x)) /
                (-(p1.x - p2.x - 0.00005f) * (p3.y - p2.y + 0.00005f) + (p1.y - p2.y + 0.00005f) * (p3.x - p2.x + 0.00005f));
  float beta = (-(P.x - p3.x) * (p1.y - p3.y) + (P.y - p3.y) * (p1.x - p3.x)) /
               (-(p2.x - p3.x - 0.00005f) * (p1.y - p3.y + 0.00005f) + (p2.y - p3.y + 0.00005f) * (p1.x - p3.x + 0.00005f));
  float gama = 1.0f - alpha - beta;
  const float* rec = S.attr + 36 * (size_t)tri;
  const float4* q = reinterpret_cast<const float4*>(rec + 8);
  float4 q0 = q[0], q1 = q[1], q2 = q[2];  // floats 8..19
  V3 n1 = v3(q0.y, q0.z, q0.w), n2 = v3(q1.x, q1.y, q1.z), n3 = v3(q1.w, q2.x, q2.y);
  V3 Ns = normalize((n1 * alpha + n2 * beta) + n3 * gama);
  h.P = P;
  h.N = inside ? -Ns : Ns;
  h.viewDir = d;
  h.m = loadMaterial(rec);
}

// ------------------------------------------------------------ integrators
template <bool CULL, bool COUNT>
struct Tracer {
  const SceneView& S;
  Stack& st;
  Counters& C;
  __device__ __forceinline__ bool closest(V3 o, V3 d, Hit& h) {
    float t;
    int tri = traceRay<false, CULL, COUNT>(S, o, d, t, st, C);
    if (tri < 0) return false;
    finishHit(S, tri, o, d, t, h);
    return true;
  }
  __device__ __forceinline__ bool occluded(V3 o, V3 d) {
    float t;
    // COUNT reproduces the reference's closest-hit shadow query fetch by fetch
    return traceRay<!COUNT, CULL, COUNT>(S, o, d, t, st, C) >= 0;
  }
};

// pathTracing O:329-364
template <class T>
__device__ V3 pathLambert(T& tr, const Env& env, Hit hit, int maxBounce, uint32_t& seed, Counters& C, bool count) {
  V3 Lo = v3(0, 0, 0), history = v3(1, 1, 1);
  for (int bounce = 0; bounce < maxBounce; bounce++) {
    V3 wi = toNormalHemisphere(sampleHemisphereRand(seed), hit.N);
    Hit nh;
    bool isHit = tr.closest(hit.P, wi, nh);
    float pdf = 1.0f / (2.0f * PT_PI);
    float cosine_i = fmaxf(0.0f, dot(wi, hit.N));
    V3 f_r = hit.m.baseColor / PT_PI;
    if (!isHit) {
      V3 sky = sampleHdr(env, wi);
      if (count) C.texels++;
      Lo = Lo + ((history * sky) * f_r * cosine_i) / pdf;
      break;
    }
    V3 Le = nh.m.emissive;
    Lo = Lo + ((history * Le) * f_r * cosine_i) / pdf;
    hit = nh;
    history = history * ((f_r * cosine_i) / pdf);
  }
  return Lo;
}

// pathTracing D:443-481
template <class T>
__device__ V3 pathDisneyUniform(T& tr, const Env& env, Hit hit, int maxBounce, uint32_t& seed, Counters& C,
                                bool count) {
  V3 Lo = v3(0, 0, 0), history = v3(1, 1, 1);
  for (int bounce = 0; bounce < maxBounce; bounce++) {
    V3 V = -hit.viewDir;
    V3 N = hit.N;
    V3 L = toNormalHemisphere(sampleHemisphereRand(seed), hit.N);
    float pdf = 1.0f / (2.0f * PT_PI);
    float cosine_i = fmaxf(0.0f, dot(L, N));
    V3 tangent, bitangent;
    getTangent(N, tangent, bitangent);
    V3 f_r = brdfAniso(V, N, L, tangent, bitangent, hit.m);
    Hit nh;
    bool isHit = tr.closest(hit.P, L, nh);
    if (!isHit) {
      V3 sky = sampleHdr(env, L);
      if (count) C.texels++;
      Lo = Lo + ((history * sky) * f_r * cosine_i) / pdf;
      break;
    }
    V3 Le = nh.m.emissive;
    Lo = Lo + ((history * Le) * f_r * cosine_i) / pdf;
    hit = nh;
    history = history * ((f_r * cosine_i) / pdf);
  }
  return Lo;
}

// pathTracingImportanceSampling IS:761-841
template <class T>
__device__ V3 pathMIS(T& tr, const Env& env, Hit hit, int maxBounce, uint32_t& seed, int px, int py,
                      uint32_t frameCounter, Counters& C, bool count) {
  V3 Lo = v3(0, 0, 0), history = v3(1, 1, 1);
  const uint32_t gi = grayCode(frameCounter + 1u);
  for (int bounce = 0; bounce < maxBounce; bounce++) {
    V3 V = -hit.viewDir;
    V3 N = hit.N;
    float r1 = randf(seed);
    float r2 = randf(seed);
    V3 Ldir = sampleHdrDir(env, r1, r2);
    if (count) C.texels++;
    if (dot(N, Ldir) > 0.0f) {
      if (!tr.occluded(hit.P, Ldir)) {
        V3 L = Ldir;
        V3 color = hdrColor(env, L);
        float pdf_light = hdrPdf(env, L);
        if (count) C.texels += 2;
        V3 f_r = brdfIso(V, N, L, hit.m);
        float pdf_brdf = brdfPdf(V, N, L, hit.m);
        float mis_weight = misWeight(pdf_light, pdf_brdf);
        V3 c = ((history * mis_weight) * color) * f_r;
        Lo = Lo + (c * dot(N, L)) / pdf_light;
      }
    }
    float u = sobolf(2u * (uint32_t)bounce, gi);
    float v = sobolf(2u * (uint32_t)bounce + 1u, gi);
    cranleyPatterson(px, py, u, v);
    float xi_3 = randf(seed);
    V3 L = sampleBRDF(u, v, xi_3, V, N, hit.m);
    float NdotL = dot(N, L);
    if (NdotL <= 0.0f) break;
    Hit nh;
    bool isHit = tr.closest(hit.P, L, nh);
    V3 f_r = brdfIso(V, N, L, hit.m);
    float pdf_brdf = brdfPdf(V, N, L, hit.m);
    if (pdf_brdf <= 0.0f) break;
    if (!isHit) {
      V3 color = hdrColor(env, L);
      float pdf_light = hdrPdf(env, L);
      if (count) C.texels += 2;
      float mis_weight = misWeight(pdf_brdf, pdf_light);
      V3 c = ((history * mis_weight) * color) * f_r;
      Lo = Lo + (c * NdotL) / pdf_brdf;
      break;
    }
    V3 Le = nh.m.emissive;
    Lo = Lo + ((history * Le) * f_r * NdotL) / pdf_brdf;
    hit = nh;
    history = history * ((f_r * NdotL) / pdf_brdf);
  }
  return Lo;
}

// main IS:844-872 for one pixel (px, py from the bottom-left)
template <int INTEG, bool CULL, bool COUNT>
__device__ __forceinline__ void shadePixel(const RenderParams& p, int px, int py, Stack& st, Counters& C) {
  Tracer<CULL, COUNT> tr{p.scene, st, C};
  const int W = p.width, H = p.height;
  uint32_t seed = ((uint32_t)px * 1973u + (uint32_t)py * 9277u + p.frameCounter * 26699u) | 1u;
  float pixx = (float)(2 * px + 1) / (float)W - 1.0f;
  float pixy = (float)(2 * py + 1) / (float)H - 1.0f;
  float ax = (randf(seed) - 0.5f) / (float)W;
  float ay = (randf(seed) - 0.5f) / (float)H;
  float x = pixx + ax, y = pixy + ay, z = -1.5f;
  const float* M = p.cam;
  V3 c0 = v3(M[0], M[1], M[2]), c1 = v3(M[4], M[5], M[6]), c2 = v3(M[8], M[9], M[10]), c3 = v3(M[12], M[13], M[14]);
  V3 dir = (c0 * x + c1 * y) + (c2 * z + c3 * 0.0f);
  dir = normalize(dir);
  V3 eye = v3(p.eye[0], p.eye[1], p.eye[2]);
  Hit first;
  V3 color;
  if (!tr.closest(eye, dir, first)) {
    color = sampleHdr(p.env, dir);
    if (COUNT) C.texels++;
  } else {
    V3 Li;
    if (INTEG == 0) Li = pathLambert(tr, p.env, first, p.maxBounce, seed, C, COUNT);
    else if (INTEG == 1) Li = pathDisneyUniform(tr, p.env, first, p.maxBounce, seed, C, COUNT);
    else Li = pathMIS(tr, p.env, first, p.maxBounce, seed, px, py, p.frameCounter, C, COUNT);
    color = first.m.emissive + Li;
  }
  float4* a = p.accum + (size_t)py * W + px;
  float4 old = *a;
  if (COUNT) C.texels++;
  float w = 1.0f / (float)(p.frameCounter + 1u);
  *a = make_float4(mixf(old.x, color.x, w), mixf(old.y, color.y, w), mixf(old.z, color.z, w), 1.0f);
}

// ------------------------------------------------ BASIC (BasicRayTracingWithC++)
struct BHit {
  float distance;
  V3 P, N, color;
  bool emissive;
  float specularRate, roughness, refractRate, refractAngle, refractRoughness;
};
// Triangle::intersect B:90-122 / Sphere::intersect B:135-164
__device__ __forceinline__ bool bIntersect(const float* sh, V3 S, V3 d, BHit& res) {
  if (sh[0] == 1.0f) {
    V3 O = ld3(sh + 1);
    float R = sh[22];
    float OS = sqrtf(dot(O - S, O - S));
    float SH = dot(O - S, d);
    float OH = sqrtf(OS * OS - SH * SH);
    if (OH > R) return false;
    float PH = sqrtf(R * R - OH * OH);
    float t1 = fabsf(SH) - PH;
    float t2 = fabsf(SH) + PH;
    float t = (t1 < 0) ? t2 : t1;
    V3 P = S + d * t;
    if (fabsf(t1) < 0.0005f || fabsf(t2) < 0.0005f) return false;
    res.distance = t;
    res.P = P;
    res.N = normalize(P - O);
  } else {
    V3 p1 = ld3(sh + 1), p2 = ld3(sh + 4), p3 = ld3(sh + 7), n = ld3(sh + 13);
    V3 N = n;
    if (dot(N, d) > 0.0f) N = -N;
    if (fabsf(dot(N, d)) < 0.00001f) return false;
    float t = (dot(N, p1) - dot(S, N)) / dot(d, N);
    if (t < 0.0005f) return false;
    V3 P = S + d * t;
    V3 c1 = cross(p2 - p1, P - p1), c2 = cross(p3 - p2, P - p2), c3 = cross(p1 - p3, P - p3);
    if (dot(c1, n) < 0 || dot(c2, n) < 0 || dot(c3, n) < 0) return false;
    res.distance = t;
    res.P = P;
    res.N = N;
  }
  res.color = ld3(sh + 10);
  res.emissive = sh[16] != 0.0f;
  res.specularRate = sh[17]; res.roughness = sh[18]; res.refractRate = sh[19];
  res.refractAngle = sh[20]; res.refractRoughness = sh[21];
  return true;
}
// shoot B:192-205
__device__ __forceinline__ bool bShoot(const float* shapes, int n, V3 S, V3 d, BHit& best) {
  bool any = false;
  best.distance = 1145141919.810f;
  for (int k = 0; k < n; k++) {
    BHit r;
    if (bIntersect(shapes + (size_t)k * 24, S, d, r) && r.distance < best.distance) {
      best = r;
      any = true;
    }
  }
  return any;
}
// randomDirection B:237-250
__device__ __forceinline__ V3 bRandomDirection(V3 n, uint32_t& seed) {
  V3 dd;
  do {
    float a = randf(seed), b = randf(seed), c = randf(seed);
    dd = v3(a, b, c) * 2.0f - v3(1, 1, 1);
  } while (dot(dd, dd) > 1.0f);
  return normalize(normalize(dd) + n);
}
__device__ __forceinline__ V3 bRefract(V3 I, V3 N, float eta) {  // glm refract
  float dv = dot(N, I);
  float k = 1.0f - eta * eta * (1.0f - dv * dv);
  if (k < 0.0f) return v3(0, 0, 0);
  return I * eta - N * (eta * dv + sqrtf(k));
}
__device__ __forceinline__ int bLobe(const BHit& res, V3 din, uint32_t& seed, V3& dout) {
  V3 rd = bRandomDirection(res.N, seed);
  float r = randf(seed);
  if (r < res.specularRate) {
    dout = mixv(normalize(reflect3(din, res.N)), rd, res.roughness);
    return 0;
  } else if (res.specularRate <= r && r <= res.refractRate) {
    dout = mixv(normalize(bRefract(din, res.N, res.refractAngle)), -rd, res.refractRoughness);
    return 1;
  }
  dout = rd;
  return 2;
}

__global__ __launch_bounds__(BLOCK) void basicKernel(BasicParams p) {
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  uint32_t rays = 0;
  if (j < p.width && i < p.height) {
    const int W = p.width, H = p.height;
    uint32_t seed = ((uint32_t)j * 1973u + (uint32_t)i * 9277u + p.sample * 26699u + p.seed * 0x9E3779B9u) | 1u;
    double xd = 2.0 * (double)j / (double)W - 1.0;
    double yd = 2.0 * (double)(H - i) / (double)H - 1.0;
    xd += (double)(randf(seed) - 0.5f) / (double)W;
    yd += (double)(randf(seed) - 0.5f) / (double)H;
    V3 coord = v3((float)xd, (float)yd, 1.1f);
    V3 dir = normalize(coord - v3(0, 0, 4.0f));
    BHit res;
    V3 color = v3(0, 0, 0);
    rays++;
    if (bShoot(p.shapes, p.nShapes, coord, dir, res)) {
      if (res.emissive) {
        color = res.color;
      } else {
        V3 nd;
        int lobe = bLobe(res, dir, seed, nd);
        // pathTracing B:252-297, recursion unrolled into a throughput product
        V3 S = res.P, d = nd, thr = v3(1, 1, 1), pt = v3(0, 0, 0);
        for (int depth = 0; depth <= p.maxDepth; depth++) {
          BHit h;
          rays++;
          if (!bShoot(p.shapes, p.nShapes, S, d, h)) break;
          if (h.emissive) { pt = thr * h.color; break; }
          float r = randf(seed);
          if (r > 0.8f) break;
          float cosine = fabsf(dot(-d, h.N));
          V3 nd2;
          int lb = bLobe(h, d, seed, nd2);
          thr = thr * cosine;
          if (lb == 2) thr = thr * h.color;
          thr = thr / 0.8f;
          S = h.P;
          d = nd2;
        }
        color = (lobe == 2) ? pt * res.color : pt;
        color = color * p.brightness;
      }
    }
    float4* a = p.accum + (size_t)i * W + j;
    float4 o = *a;
    *a = make_float4(o.x + color.x, o.y + color.y, o.z + color.z, 1.0f);
  }
  // wave-reduce the ray count, one atomic per wave
  for (int off = 32; off > 0; off >>= 1) rays += __shfl_down(rays, off, 64);
  if ((threadIdx.x & 63) == 0 && rays) atomicAdd(reinterpret_cast<unsigned long long*>(p.stats), (unsigned long long)rays);
}

// ------------------------------------------------------------ render kernel
__device__ __forceinline__ uint32_t waveSum(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

template <int INTEG, bool CULL, bool COUNT>
__global__ __launch_bounds__(BLOCK) void renderKernel(RenderParams p) {
  __shared__ int s_stack[LDS_STACK * BLOCK];
  Stack st;
  st.lds = s_stack + threadIdx.x;
  st.gbl = p.ovf ? p.ovf + (size_t)(blockIdx.x * BLOCK + threadIdx.x) * p.ovfDepth : nullptr;
  st.sp = 0;
  Counters C = {0, 0, 0, 0, 0};
  const int lane = threadIdx.x & 63;
  const int home = blockIdx.x & (NUM_QUEUES - 1);
  const int tilesPerShard = p.shardTiles;  // 8x8 wave tiles per shard tile
  const int sub = p.shardSize >> 3;        // wave tiles per shard-tile edge
  for (int qi = 0; qi < NUM_QUEUES;) {
    const int q = (home + qi) & (NUM_QUEUES - 1);
    int item = 0;
    if (lane == 0) item = atomicAdd(p.queue + q, 1);
    item = __shfl(item, 0, 64);
    const int base = q * p.perQueue;
    if (item >= p.perQueue || base + item >= p.numItems) {
      qi++;
      continue;
    }
    const int w = base + item;
    const int j = w / tilesPerShard, s = w - j * tilesPerShard;
    const int g = j * p.world + p.rank;  // global shard tile id (row-major)
    const int gy = g / p.shardsX, gx = g - gy * p.shardsX;
    const int px = gx * p.shardSize + (s % sub) * 8 + (lane & 7);
    const int py = gy * p.shardSize + (s / sub) * 8 + (lane >> 3);
    if (px < p.width && py < p.height) shadePixel<INTEG, CULL, COUNT>(p, px, py, st, C);
  }
  uint32_t r = waveSum(C.rays);
  if (COUNT) {
    uint32_t n = waveSum(C.nodes), t = waveSum(C.tris), m = waveSum(C.mats), x = waveSum(C.texels);
    if (lane == 0) {
      atomicAdd(reinterpret_cast<unsigned long long*>(p.stats + 1), (unsigned long long)n);
      atomicAdd(reinterpret_cast<unsigned long long*>(p.stats + 2), (unsigned long long)t);
      atomicAdd(reinterpret_cast<unsigned long long*>(p.stats + 3), (unsigned long long)m);
      atomicAdd(reinterpret_cast<unsigned long long*>(p.stats + 4), (unsigned long long)x);
    }
  }
  if (lane == 0 && r) atomicAdd(reinterpret_cast<unsigned long long*>(p.stats), (unsigned long long)r);
}

// ------------------------------------------------------------ batch query
template <bool CULL>
__global__ __launch_bounds__(BLOCK) void traceKernel(TraceParams p) {
  __shared__ int s_stack[LDS_STACK * BLOCK];
  Stack st;
  st.lds = s_stack + threadIdx.x;
  const size_t gtid = (size_t)blockIdx.x * BLOCK + threadIdx.x;
  st.gbl = p.ovf ? p.ovf + gtid * p.ovfDepth : nullptr;
  Counters C = {0, 0, 0, 0, 0};
  for (size_t k = gtid; k < (size_t)p.n; k += (size_t)gridDim.x * BLOCK) {
    const float* r = p.rays + 6 * k;
    V3 o = v3(r[0], r[1], r[2]), d = v3(r[3], r[4], r[5]);
    float t;
    int tri = traceRay<false, CULL, false>(p.scene, o, d, t, st, C);
    p.t[k] = tri >= 0 ? t : PT_INF;
    p.tri[k] = tri;
  }
}

// ------------------------------------------------------------ epilogues
// pass3.fsh:14-24 tonemap (+ optional gamma, commented out in the reference)
__global__ void tonemapKernel(const float4* accum, float* rgb, int n, float limit, float gamma) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float4 c = accum[i];
  float lum = 0.3f * c.x + 0.6f * c.y + 0.1f * c.z;
  float s = 1.0f / (1.0f + lum / limit);
  float r = c.x * s, g = c.y * s, b = c.z * s;
  if (gamma > 0.0f) {
    r = ptm_powf(r, 1.0f / gamma);
    g = ptm_powf(g, 1.0f / gamma);
    b = ptm_powf(b, 1.0f / gamma);
  }
  rgb[3 * i] = r;
  rgb[3 * i + 1] = g;
  rgb[3 * i + 2] = b;
}

// pack (unpack) the pixels of shard tiles t % world == rank in (tile, row, col) order
__device__ __forceinline__ bool packedPixel(const PackParams& p, long k, int& px, int& py) {
  const long perTile = (long)p.shardSize * p.shardSize;
  long j = k / perTile;
  int within = (int)(k - j * perTile);
  long g = j * p.world + p.rank;
  int gy = (int)(g / p.shardsX), gx = (int)(g - (long)gy * p.shardsX);
  px = gx * p.shardSize + within % p.shardSize;
  py = gy * p.shardSize + within / p.shardSize;
  return px < p.width && py < p.height;
}
__global__ void packKernel(PackParams p, const float4* accum, float4* packed) {
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.count) return;
  int px, py;
  packed[k] = packedPixel(p, k, px, py) ? accum[(size_t)py * p.width + px] : make_float4(0, 0, 0, 0);
}
__global__ void unpackKernel(PackParams p, float4* accum, const float4* packed) {
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.count) return;
  int px, py;
  if (packedPixel(p, k, px, py)) accum[(size_t)py * p.width + px] = packed[k];
}

// include/pt_fmath.h evaluated on the device (diagnostics; bit-equality with the host)
__device__ __forceinline__ float fmathEval(int fn, float x, float y) {
  switch (fn) {
    case 0: return ptm_sinf(x);
    case 1: return ptm_cosf(x);
    case 2: return ptm_atan2f(x, y);
    case 3: return ptm_asinf(x);
    case 4: return ptm_logf(x);
    case 5: return ptm_expf(x);
    default: return ptm_powf(x, y);
  }
}
__global__ void fmathKernel(int fn, const float* x, const float* y, int n, float* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = fmathEval(fn, x[i], y ? y[i] : 0.0f);
}

}  // namespace pt

// ------------------------------------------------------------ launchers
namespace pt {

template <int I>
static hipError_t launchRenderI(const RenderParams& p, int grid, hipStream_t s, bool cull, bool count) {
  if (count) {
    hipLaunchKernelGGL((renderKernel<I, false, true>), dim3(grid), dim3(BLOCK), 0, s, p);
  } else if (cull) {
    hipLaunchKernelGGL((renderKernel<I, true, false>), dim3(grid), dim3(BLOCK), 0, s, p);
  } else {
    hipLaunchKernelGGL((renderKernel<I, false, false>), dim3(grid), dim3(BLOCK), 0, s, p);
  }
  return hipGetLastError();
}

hipError_t launchRender(const RenderParams& p, int integrator, int grid, hipStream_t s, bool cull, bool count) {
  switch (integrator) {
    case 0: return launchRenderI<0>(p, grid, s, cull, count);
    case 1: return launchRenderI<1>(p, grid, s, cull, count);
    default: return launchRenderI<2>(p, grid, s, cull, count);
  }
}

hipError_t renderBlocksPerCU(int integrator, bool cull, bool count, int* nb) {
  const void* f;
#define PT_SEL(I)                                                                              \
  f = count ? (const void*)renderKernel<I, false, true>                                        \
            : (cull ? (const void*)renderKernel<I, true, false> : (const void*)renderKernel<I, false, false>)
  if (integrator == 0) { PT_SEL(0); }
  else if (integrator == 1) { PT_SEL(1); }
  else { PT_SEL(2); }
#undef PT_SEL
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(nb, f, BLOCK, 0);
}

hipError_t launchTrace(const TraceParams& p, int grid, hipStream_t s, bool cull) {
  if (cull) hipLaunchKernelGGL((traceKernel<true>), dim3(grid), dim3(BLOCK), 0, s, p);
  else hipLaunchKernelGGL((traceKernel<false>), dim3(grid), dim3(BLOCK), 0, s, p);
  return hipGetLastError();
}

hipError_t launchBasic(const BasicParams& p, hipStream_t s) {
  dim3 grid((p.width + 15) / 16, (p.height + 15) / 16);
  hipLaunchKernelGGL(basicKernel, grid, dim3(BLOCK), 0, s, p);
  return hipGetLastError();
}

hipError_t launchTonemap(const float4* accum, float* rgb, int n, float limit, float gamma, hipStream_t s) {
  hipLaunchKernelGGL(tonemapKernel, dim3((n + 255) / 256), dim3(256), 0, s, accum, rgb, n, limit, gamma);
  return hipGetLastError();
}

hipError_t launchFmath(int fn, const float* x, const float* y, int n, float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fmathKernel, dim3((n + 255) / 256), dim3(256), 0, s, fn, x, y, n, out);
  return hipGetLastError();
}

hipError_t launchPack(const PackParams& p, const float4* accum, float4* packed, hipStream_t s) {
  if (p.count <= 0) return hipSuccess;
  hipLaunchKernelGGL(packKernel, dim3((unsigned)((p.count + 255) / 256)), dim3(256), 0, s, p, accum, packed);
  return hipGetLastError();
}
hipError_t launchUnpack(const PackParams& p, float4* accum, const float4* packed, hipStream_t s) {
  if (p.count <= 0) return hipSuccess;
  hipLaunchKernelGGL(unpackKernel, dim3((unsigned)((p.count + 255) / 256)), dim3(256), 0, s, p, accum, packed);
  return hipGetLastError();
}

}  // namespace pt
