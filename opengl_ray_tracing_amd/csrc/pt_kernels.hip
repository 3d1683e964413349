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
#include "pt_scene.h"
#include "pt_trace.h"

namespace pt {



// ------------------------------------------------------------ integrators
template <bool CULL, bool COUNT>
struct Tracer {
  const SceneView& S;
  Stack& st;
  Counters& C;
  const float4* top;  // LDS copy of the top of the tree traversed first (null = none)
  // closest hit: the triangle (-1 = miss) and its t. With S.fast, through the
  // runtime's tree and checked against the reference's (pt_trace.h refReachable).
  __device__ __forceinline__ int trace(V3 o, V3 d, float& t) {
    if (PT_WIDE4 && !COUNT && S.fast) {  // the 4-wide runtime tree (PT_WIDE4), checked as the binary one
      bool tie = false;
      int tri = traceRay4<CULL, Stack, (PT_WIDE4 == 2)>(S, o, d, t, st, C, false, top, &tie);
      if (tie || (tri >= 0 && !refReachable(S, tri, o, d, t))) {
        C.rays--;
        tri = traceRay<false, CULL, false, Stack>(S, o, d, t, st, C);
      }
      return tri;
    }
    if (!COUNT && S.fast) {
      bool tie = false;
      const SceneView F = fastView(S);
      const int pos = traceRay<false, CULL, false, Stack, (LDS_NODES > 0), true, FAST_KIND>(F, o, d, t, st, C, false, top, &tie);
      int tri = pos >= 0 ? S.fastTri[pos] : -1;
      if (tie || (tri >= 0 && !refReachable(S, tri, o, d, t))) {
        C.rays--;  // the same ray, counted once
        tri = traceRay<false, CULL, false, Stack>(S, o, d, t, st, C);
      }
      return tri;
    }
    return traceRay<false, CULL, COUNT, Stack, (LDS_NODES > 0)>(S, o, d, t, st, C, false, top);
  }
  __device__ __forceinline__ bool closest(V3 o, V3 d, Hit& h) {
    float t;
    const int tri = trace(o, d, t);
    if (tri < 0) return false;
    finishHit(S, tri, o, d, t, h);
    return true;
  }
  __device__ __forceinline__ bool occluded(V3 o, V3 d) {
    float t;
    if (PT_WIDE4 && !COUNT && S.fast) {
      bool tie = false;
      const int tri = traceRay4<CULL, Stack, (PT_WIDE4 == 2)>(S, o, d, t, st, C, true, top, &tie);
      if (tri < 0) return false;
      if (refReachable(S, tri, o, d, t)) return true;
      C.rays--;
      return traceRay<true, CULL, false, Stack>(S, o, d, t, st, C) >= 0;
    }
    if (!COUNT && S.fast) {
      const SceneView F = fastView(S);
      const int pos = traceRay<true, CULL, false, Stack, (LDS_NODES > 0), false, FAST_KIND>(F, o, d, t, st, C, false, top);
      if (pos < 0) return false;
      if (refReachable(S, S.fastTri[pos], o, d, t)) return true;
      C.rays--;
      return traceRay<true, CULL, false, Stack>(S, o, d, t, st, C) >= 0;
    }
    // COUNT reproduces the reference's closest-hit shadow query fetch by fetch
    return traceRay<!COUNT, CULL, COUNT, Stack, (LDS_NODES > 0)>(S, o, d, t, st, C, false, top) >= 0;
  }
  // closest (anyhit false) or env-shadow (anyhit true: >= 0 = occluded) query through ONE call site
  // of the traversal, so a path loop that traces its shadow and BRDF rays from the same place
  // keeps one copy of the walk (and its registers) live: trace() / occluded() per lane
  __device__ __forceinline__ int traceK(V3 o, V3 d, bool anyhit, float& t) {
    if (PT_WIDE4 && !COUNT && S.fast) {
      bool tie = false;
      int tri = traceRay4<CULL, Stack, (PT_WIDE4 == 2)>(S, o, d, t, st, C, anyhit, top, &tie);
      if ((tie && !anyhit) || (tri >= 0 && !refReachable(S, tri, o, d, t))) {
        C.rays--;  // the same ray, counted once
        tri = traceRay<false, CULL, false, Stack>(S, o, d, t, st, C, anyhit);
      }
      return tri;
    }
    if (anyhit) return occluded(o, d) ? 0 : -1;
    return trace(o, d, t);
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
//
// Evaluated in a different order from the reference, with the same operations
// on the same values (so the same bits): everything that needs the hit's
// material -- the light sample's contribution and the BRDF sample with its
// f_r and pdf -- is computed before either ray of the bounce is traced, and
// the light contribution is added only if the shadow ray is unoccluded. No
// material, view vector or normal is live across a traversal. Random numbers are
// drawn in the reference's order (r1, r2, then xi_3); the shadow ray is traced and
// counted exactly when the reference traces it. Both rays of a bounce go through
// one traversal call site (Tracer::traceK): the loop's phase says which ray is in
// flight, so a lane whose bounce has no shadow ray walks its BRDF ray beside
// another lane's shadow ray, and the kernel holds one copy of the walk.
template <class T>
__device__ V3 pathMIS(T& tr, const Env& env, Hit hit, int maxBounce, uint32_t& seed, int px, int py,
                      uint32_t frameCounter, Counters& C, bool count) {
  V3 Lo = v3(0, 0, 0), history = v3(1, 1, 1);
  if (maxBounce <= 0) return Lo;
  const uint32_t gi = grayCode(frameCounter + 1u);  // frameCounter = the sample index here
  float cpu, cpv;
  cranleyPattersonShift(px, py, cpu, cpv);
  for (int bounce = 0; bounce < maxBounce; bounce++) {
    const V3 V = -hit.viewDir;
    const V3 N = hit.N;
    // (1) light sample IS:772-789
    const float r1 = randf(seed);
    const float r2 = randf(seed);
    int ent;
    const V3 Ldir = sampleHdrDir(env, r1, r2, &ent);
    if (count) C.texels++;
    const bool tryLight = dot(N, Ldir) > 0.0f;
    V3 lightC = v3(0, 0, 0);
    if (tryLight) {
      V3 color;
      float pdf_light;
      hdrLightColorPdf(env, ent, Ldir, color, pdf_light);
      const V3 fl = brdfIso(V, N, Ldir, hit.m);
      const float pb = brdfPdf(V, N, Ldir, hit.m);
      const float mis_weight = misWeight(pdf_light, pb);
      const V3 c = ((history * mis_weight) * color) * fl;
      lightC = (c * dot(N, Ldir)) / pdf_light;
    }
    // (2) BRDF sample IS:791-840
    float u = sobolf(2u * (uint32_t)bounce, gi);
    float v = sobolf(2u * (uint32_t)bounce + 1u, gi);
    cranleyPattersonApply(cpu, cpv, u, v);
    const float xi_3 = randf(seed);
    const V3 L = sampleBRDF(u, v, xi_3, V, N, hit.m);
    const float NdotL = dot(N, L);
    const V3 f_r = brdfIso(V, N, L, hit.m);
    const float pdf_brdf = brdfPdf(V, N, L, hit.m);
    const V3 P = hit.P;
    if (!tryLight && NdotL <= 0.0f) break;  // IS:818: no ray left in this bounce
    // (3) the bounce's rays, the env shadow ray first when there is one, through one call site
    bool shadow = tryLight, end = false;
    int tri;
    float t;
    while (true) {
      tri = tr.traceK(P, shadow ? Ldir : L, shadow, t);
      if (!shadow) break;
      if (tri < 0) {  // IS:776-790
        Lo = Lo + lightC;
        if (count) C.texels += 2;
      }
      shadow = false;
      if (NdotL <= 0.0f) {
        end = true;
        break;
      }
    }
    if (end) break;
    if (pdf_brdf <= 0.0f) break;  // IS:816: the ray is traced, then discarded
    if (tri < 0) {  // IS:819-829
      V3 color;
      float pdf_light;
      hdrColorPdf(env, L, color, pdf_light);
      if (count) C.texels += 2;
      const float mis_weight = misWeight(pdf_brdf, pdf_light);
      const V3 c = ((history * mis_weight) * color) * f_r;
      Lo = Lo + (c * NdotL) / pdf_brdf;
      break;
    }
    finishHit(tr.S, tri, P, L, t, hit);  // IS:831-840: the next bounce's hit
    const V3 Le = hit.m.emissive;
    Lo = Lo + ((history * Le) * f_r * NdotL) / pdf_brdf;
    history = history * ((f_r * NdotL) / pdf_brdf);
  }
  return Lo;
}

// main IS:844-872 for one pixel (px, py from the bottom-left), in two parts:
// the camera ray (cameraRay + primaryPixel) and the rest of the path
// (finishPixel, which recomputes the camera ray and RNG state from the pixel).
__device__ __forceinline__ V3 cameraRay(const RenderParams& p, uint32_t sampleIndex, int px, int py, uint32_t& seed) {
  const int W = p.width, H = p.height;
  seed = ((uint32_t)px * 1973u + (uint32_t)py * 9277u + sampleIndex * 26699u) | 1u;
  float pixx = (float)(2 * px + 1) / (float)W - 1.0f;
  float pixy = (float)(2 * py + 1) / (float)H - 1.0f;
  float ax = (randf(seed) - 0.5f) / (float)W;
  float ay = (randf(seed) - 0.5f) / (float)H;
  float x = pixx + ax, y = pixy + ay, z = -1.5f;
  const float* M = p.cam;
  V3 c0 = v3(M[0], M[1], M[2]), c1 = v3(M[4], M[5], M[6]), c2 = v3(M[8], M[9], M[10]), c3 = v3(M[12], M[13], M[14]);
  V3 dir = (c0 * x + c1 * y) + (c2 * z + c3 * 0.0f);
  return normalize(dir);
}

// f: the frame the pixel belongs to (its sample index and colour buffer)
__device__ __forceinline__ void accumulate(const RenderParams& p, const FrameRef& f, int px, int py, V3 color, Counters& C,
                                           bool count) {
  float* col = f.col;
  if (!count && col) {  // pipelined frame: the sample colour, mixed into the running mean in frame order (mixKernel)
    stCol(col + shareIndex(p, px, py) * COL_F, color.x, color.y, color.z);
    return;
  }
  float4* a = p.accum + (size_t)py * p.width + px;
  float4 old = ldStream(a);
  if (count) C.texels++;
  float w = 1.0f / (float)(p.frameCounter + 1u);
  stStream(a, make_float4(mixf(old.x, color.x, w), mixf(old.y, color.y, w), mixf(old.z, color.z, w), 1.0f));
}

// the camera ray's closest hit; a miss is finished here (sky colour accumulated)
template <bool CULL, bool COUNT>
__device__ __forceinline__ int primaryPixel(const RenderParams& p, const FrameRef& f, int px, int py, Stack& st,
                                            Counters& C, const float4* top, float& t) {
  uint32_t seed;
  const V3 dir = cameraRay(p, f.sampleIndex, px, py, seed);
  const V3 eye = v3(p.eye[0], p.eye[1], p.eye[2]);
  Tracer<CULL, COUNT> tr{p.scene, st, C, top};
  const int tri = tr.trace(eye, dir, t);
  if (tri < 0) {
    const V3 color = sampleHdr(p.env, dir);
    if (COUNT) C.texels++;
    accumulate(p, f, px, py, color, C, COUNT);
  }
  return tri;
}

// primaryPixel for a whole wave: the camera rays of the wave's pixels traced as
// one packet (tracePacket); a ray that met an exact tie is retraced in the
// reference order. All 64 lanes call it; valid marks the lanes with a pixel.
template <bool CULL>
__device__ __forceinline__ int primaryPacket(const RenderParams& p, const FrameRef& f, int px, int py, bool valid,
                                             Stack& st, Counters& C, const float4* top, PacketEntry* pstack, float& t) {
  uint32_t seed;
  const V3 dir = cameraRay(p, f.sampleIndex, valid ? px : 0, valid ? py : 0, seed);
  const V3 eye = v3(p.eye[0], p.eye[1], p.eye[2]);
  bool tie;
  int tri;
  // camera-ray bins (pt_primary.hip): the tile's candidate triangles, each tested
  // with hitTriangle's exact arithmetic (IS:251-301); the closest stands when no
  // other candidate ties it and the reference traversal reaches it (refReachable),
  // else the ray is retraced in the reference order
  int b0 = 0, b1 = 0;  // an 8x8 tile of a shard wholly outside the image (no valid lane) has no bin
  if (p.binStart) {
    // every lane calls this function, so the first active lane is lane 0, whose pixel lies in the tile
    const int tx = __builtin_amdgcn_readfirstlane(px) >> 3, ty = __builtin_amdgcn_readfirstlane(py) >> 3;
    if (tx < p.binTilesX && ty < p.binTilesY) {
      const int tile = ty * p.binTilesX + tx;
      b0 = p.binStart[tile];
      b1 = p.binStart[tile + 1];
    }
  }
  if (p.binStart && b1 - b0 <= PT_BIN_CAP) {
    // the bin's triangles staged in the wave's own (still empty) part of the LDS stack:
    // every lane loads one float4 of one triangle, so the whole bin costs two memory round
    // trips instead of one per triangle; the test loop then reads broadcast LDS records.
    // Triangle t's 16 floats at wb + (t >> 2) * BLOCK + (t & 3) * 16, its index at row IDX.
    constexpr int IDX = (PT_BIN_CAP + 3) / 4;
    static_assert(PT_BIN_CAP <= 64 && IDX < LDS_STACK, "bin staging fits the wave's stack rows 0..IDX");
    const int n = b1 - b0;
    int* wb = st.lds - __lane_id();  // column 0 of this wave's stack columns
    const int lane = __lane_id();
    for (int t = lane >> 2; t < n; t += 16) {
      const int i = p.binTris[b0 + t];
      const float4 v = p.scene.geo[4 * (size_t)i + (lane & 3)];
      *reinterpret_cast<float4*>(wb + (t >> 2) * BLOCK + (t & 3) * 16 + 4 * (lane & 3)) = v;
      if ((lane & 3) == 0) wb[IDX * BLOCK + t] = i;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float tbest = PT_INF;
    int best = -1;
    tie = false;
    for (int k = 0; k < n; k++) {
      const float4* g = reinterpret_cast<const float4*>(wb + (k >> 2) * BLOCK + (k & 3) * 16);
      float tt;
      const bool h = valid && triTest(g[0], g[1], g[2], g[3], eye, dir, PT_INF, tt);
      if (h && tt == tbest) tie = true;
      if (h && tt < tbest) {
        tbest = tt;
        best = k;
      }
    }
    if (best >= 0) best = wb[IDX * BLOCK + best];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // every lane has read the staging before the stack is used
    __builtin_amdgcn_wave_barrier();
    if (valid) C.rays++;
    tri = best;
    t = tbest;
    if (valid && (tie || (tri >= 0 && !refReachable(p.scene, tri, eye, dir, t)))) {
      C.rays--;  // the same ray, counted once
      tri = traceRay<false, CULL, false, Stack>(p.scene, eye, dir, t, st, C);
    }
  } else if (!p.packets) {  // a tree too deep for the packet stack: each ray on its own
    tri = -1;
    if (valid) {
      Tracer<CULL, false> tr{p.scene, st, C, top};
      tri = tr.trace(eye, dir, t);
    }
  } else if (p.scene.fast) {  // through the runtime's tree, checked against the reference's
    const int pos = tracePacket<CULL, FAST_KIND>(fastView(p.scene), eye, dir, valid, t, tie, pstack, C,
                                                  PT_WIDE4 == 2 ? nullptr : top);
    tri = pos >= 0 ? p.scene.fastTri[pos] : -1;
    if (valid && (tie || (tri >= 0 && !refReachable(p.scene, tri, eye, dir, t)))) {
      C.rays--;  // the same ray, counted once
      tri = traceRay<false, CULL, false, Stack>(p.scene, eye, dir, t, st, C);
    }
  } else {
    tri = tracePacket<CULL>(p.scene, eye, dir, valid, t, tie, pstack, C, top);
    if (valid && tie) {
      C.rays--;
      tri = traceRay<false, CULL, false, Stack, (LDS_NODES > 0)>(p.scene, eye, dir, t, st, C, false, top);
    }
  }
  if (valid && tri < 0) {
    const V3 color = sampleHdr(p.env, dir);
    accumulate(p, f, px, py, color, C, false);
  }
  return tri;
}

// Camera-ray pass: the bin path of primaryPacket for every 8x8 tile of the
// rank, one wave per tile, before the megakernel. Inside the persistent
// megakernel (3 waves/SIMD) a tile's camera rays are a chain of dependent
// round trips (claim, bin, triangles, refReachable, env) that the few resident
// waves cannot hide; here a launch of one short wave per tile keeps up to 8
// waves per SIMD in flight and claims nothing. Sky pixels are finished here;
// every other pixel's result goes to primHit for the megakernel.
__global__ __launch_bounds__(64) void primaryKernel(RenderParams p) {
  __shared__ float4 s_tri[PT_PASS_BIN_CAP * 4];
  __shared__ float4 s_box[PT_PASS_BIN_CAP * 2];
  __shared__ int s_idx[PT_PASS_BIN_CAP];
  // block b: tile b / nFrames of frame b % nFrames (a batch's frames of one tile side by side).
  // (Blocks of 2 / 4 / 8 such one-wave items, fewer workgroups for the dispatcher: c2's 1/8 share of
  // a 20-frame batch 88.6 -> 92.2 / 93.4 / 102.2 us; one block per tile for several frames: DESIGN.md 3b.)
  const int fr = (int)(blockIdx.x % (unsigned)p.nFrames);
  const int w = (int)(blockIdx.x / (unsigned)p.nFrames);
  const int lane = threadIdx.x;
  if (p.zeroQueue && blockIdx.x == 0)  // the frame kernel's work-queue counters, zeroed for it (it runs next on this stream)
    for (int q = lane; q < NUM_QUEUES; q += 64) p.queue[q * CTL_LINE_INTS] = 0;
  const int sub = p.shardSize >> 3;
  const int j = w / p.shardTiles, s = w - j * p.shardTiles;
  const int g = j * p.world + p.rank;
  const int gy = g / p.shardsX, gx = g - gy * p.shardsX;
  const int px = gx * p.shardSize + (s % sub) * 8 + (lane & 7);
  const int py = gy * p.shardSize + (s / sub) * 8 + (lane >> 3);
  const bool valid = px < p.width && py < p.height;
  const int tx = (gx * p.shardSize + (s % sub) * 8) >> 3, ty = (gy * p.shardSize + (s / sub) * 8) >> 3;
  int b0 = 0, b1 = 0;  // a tile wholly outside the image has no bin (and no valid lane)
  if (tx < p.binTilesX && ty < p.binTilesY) {
    b0 = p.binStart[ty * p.binTilesX + tx];
    b1 = p.binStart[ty * p.binTilesX + tx + 1];
  }
  const int n = b1 - b0;
  // the tile's results compacted (RenderParams::primMask): the slots that need a path, in slot order
  int2* out = p.primHit + ((size_t)fr * p.numItems + w) * 64;
  unsigned long long* mask = p.primMask + (size_t)fr * p.numItems + w;
  FrameRef fp;  // this block's frame (accumulate's colour buffer)
  fp.col = p.col ? p.col + (size_t)fr * p.colStride * COL_F : nullptr;
  fp.sampleIndex = p.sampleIndex + (uint32_t)fr * p.sampleStride;
  if (n > PT_PASS_BIN_CAP) {  // the frame kernel traces this tile's camera rays (the megakernel as a packet)
    const unsigned long long m = __ballot(valid);
    if (valid) out[__popcll(m & ((1ull << lane) - 1ull))] = make_int2(PRIM_TILE, 0);
    if (lane == 0) *mask = m;
    return;
  }
  // the bin's triangles and their leaf boxes in bin order (binGeo / binBox, gathered at bin build): one
  // round trip after binStart instead of binTris -> geo, and refReachable's leaf box from LDS
  for (int t = lane >> 2; t < n; t += 16) {  // one float4 of one triangle (and of its leaf box) per lane
    s_tri[4 * t + (lane & 3)] = p.binGeo[4 * (size_t)(b0 + t) + (lane & 3)];
    if ((lane & 3) < 2) s_box[2 * t + (lane & 3)] = p.binBox[2 * (size_t)(b0 + t) + (lane & 3)];
    else if ((lane & 3) == 2) s_idx[t] = p.binTris[b0 + t];
  }
  __syncthreads();
  uint32_t seed;
  const V3 dir = cameraRay(p, fp.sampleIndex, valid ? px : 0, valid ? py : 0, seed);
  const V3 eye = v3(p.eye[0], p.eye[1], p.eye[2]);
  float tbest = PT_INF;
  int best = -1;
  bool tie = false;
  for (int k = 0; k < n; k++) {
    float tt;
    const bool h = valid && triTest(s_tri[4 * k], s_tri[4 * k + 1], s_tri[4 * k + 2], s_tri[4 * k + 3], eye, dir,
                                    PT_INF, tt);
    if (h && tt == tbest) tie = true;
    if (h && tt < tbest) {
      tbest = tt;
      best = k;
    }
  }
  uint32_t rays = 0;
  int res = PRIM_MISS;
  if (valid) {
    res = best >= 0 ? s_idx[best] : PRIM_MISS;
    if (tie || (res >= 0 && !refReachableBox(p.scene, s_box[2 * best], s_box[2 * best + 1], eye, dir, tbest))) {
      res = PRIM_RETRACE;  // counted by the megakernel's retrace
    } else {
      rays = 1;
      if (res == PRIM_MISS) {
        Counters C = {0, 0, 0, 0, 0};
        accumulate(p, fp, px, py, sampleHdr(p.env, dir), C, false);
      }
    }
  }
  const bool need = valid && res != PRIM_MISS;
  const unsigned long long m = __ballot(need);
  if (need) out[__popcll(m & ((1ull << lane) - 1ull))] = make_int2(res, __float_as_int(tbest));
  if (lane == 0) *mask = m;
  addRays(p.rayShards, rays);
}

hipError_t launchPrimary(const RenderParams& p, hipStream_t s) {
  if (!p.primHit || !p.primMask || !p.binStart || !p.binGeo || !p.binBox || p.numItems <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(primaryKernel, dim3((unsigned)p.numItems * (unsigned)p.nFrames), dim3(64), 0, s, p);
  return hipGetLastError();
}

// the rest of the path of a pixel whose camera ray hit triangle tri at t
template <int INTEG, bool CULL, bool COUNT>
__device__ __forceinline__ void finishPixel(const RenderParams& p, const FrameRef& f, int px, int py, int tri, float t,
                                            Stack& st, Counters& C, const float4* top) {
  Tracer<CULL, COUNT> tr{p.scene, st, C, top};
  uint32_t seed;
  const uint32_t sampleIndex = f.sampleIndex;
  const V3 dir = cameraRay(p, sampleIndex, px, py, seed);  // the same ray and RNG state as primaryPixel
  const V3 eye = v3(p.eye[0], p.eye[1], p.eye[2]);
  Hit first;
  finishHit(p.scene, tri, eye, dir, t, first);
  V3 Li;
  if (INTEG == 0) Li = pathLambert(tr, p.env, first, p.maxBounce, seed, C, COUNT);
  else if (INTEG == 1) Li = pathDisneyUniform(tr, p.env, first, p.maxBounce, seed, C, COUNT);
  else Li = pathMIS(tr, p.env, first, p.maxBounce, seed, px, py, sampleIndex, C, COUNT);
  // MIS (8-16 bounces): the camera hit's emission reloaded once the path has ended rather than
  // held across every bounce (the megakernel at its 168-VGPR limit: 37 -> 28 VGPRs spilled)
  const V3 Le0 = INTEG == 2 ? emissiveOf(p.scene, tri) : first.m.emissive;
  accumulate(p, f, px, py, Le0 + Li, C, COUNT);
}

// ------------------------------------------------ BASIC (BasicRayTracingWithC++)
// The reference binary's arithmetic (oracle/pt_oracle.c b_*, pinned byte for byte
// against the reference compiled from its source): glm vec3 is float, the Material
// rates, the sphere radius, HitResult::distance and the image are double
// (B:49-68, :130, :356), each mixed expression in the type C++ promotes it to.
struct BHit {
  double distance;
  V3 P, N, color;
  bool emissive;
  double specularRate, roughness, refractRate, refractAngle, refractRoughness;
};
// randf B:211-214: the per-pixel counter stream, or the replayed reference stream
struct BRng {
  uint32_t seed;
  const double* rep;
  long long pos, end;
  bool over;
};
__device__ __forceinline__ double bRand(BRng& g) {
  if (g.rep) {
    if (g.pos < g.end) return g.rep[g.pos++];
    g.over = true;
    return 0.5;
  }
  return (double)wang(g.seed) / 4294967296.0;
}
__device__ __forceinline__ V3 ldf3(const double* p) { return v3((float)p[0], (float)p[1], (float)p[2]); }
// Triangle::intersect B:90-122 / Sphere::intersect B:135-164 (OS, SH, t float; pow(x, 2)
// of a float exact in double; R double, so OH > R and PH double expressions)
__device__ __forceinline__ bool bIntersect(const double* sh, V3 S, V3 d, BHit& res) {
  if (sh[0] == 1.0) {
    V3 O = ldf3(sh + 1);
    double R = sh[22];
    V3 OSv = O - S;
    float OS = sqrtf(dot(OSv, OSv));
    float SH = dot(OSv, d);
    float OH = (float)sqrt((double)OS * (double)OS - (double)SH * (double)SH);
    if ((double)OH > R) return false;
    float PH = (float)sqrt(R * R - (double)OH * (double)OH);
    float t1 = fabsf(SH) - PH;
    float t2 = fabsf(SH) + PH;
    float t = (t1 < 0) ? t2 : t1;
    V3 P = S + d * t;
    if (fabsf(t1) < 0.0005f || fabsf(t2) < 0.0005f) return false;
    res.distance = t;
    res.P = P;
    res.N = normalize(P - O);
  } else {
    V3 p1 = ldf3(sh + 1), p2 = ldf3(sh + 4), p3 = ldf3(sh + 7), n = ldf3(sh + 13);
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
  res.color = ldf3(sh + 10);
  res.emissive = sh[16] != 0.0;
  res.specularRate = sh[17]; res.roughness = sh[18]; res.refractRate = sh[19];
  res.refractAngle = sh[20]; res.refractRoughness = sh[21];
  return true;
}
// shoot B:192-205 (res.distance a double initialised from 1145141919.810f)
__device__ __forceinline__ bool bShoot(const double* shapes, int n, V3 S, V3 d, BHit& best) {
  bool any = false;
  best.distance = (double)1145141919.810f;
  for (int k = 0; k < n; k++) {
    BHit r;
    if (bIntersect(shapes + (size_t)k * PT_SHAPE_DOUBLES, S, d, r) && r.distance < best.distance) {
      best = r;
      any = true;
    }
  }
  return any;
}
// randomVec3 B:217-234 (the compiled reference evaluates vec3(randf(), randf(), randf())
// right to left: z takes the first draw) / randomDirection B:237-250
__device__ __forceinline__ V3 bRandomDirection(V3 n, BRng& g) {
  V3 dd;
  do {
    double z = bRand(g), y = bRand(g), x = bRand(g);
    dd = v3((float)x, (float)y, (float)z) * 2.0f - v3(1, 1, 1);
  } while ((double)dot(dd, dd) > 1.0);
  return normalize(normalize(dd) + n);
}
// glm reflect / refract (func_geometric.inl:104-123), glm mix(vec3, vec3, double) in double
__device__ __forceinline__ V3 bReflect(V3 I, V3 N) { return I - (N * dot(N, I)) * 2.0f; }
__device__ __forceinline__ V3 bRefract(V3 I, V3 N, float eta) {
  float dv = dot(N, I);
  float k = 1.0f - eta * eta * (1.0f - dv * dv);
  if (!(k >= 0.0f)) return v3(0, 0, 0);
  return I * eta - N * (eta * dv + sqrtf(k));
}
__device__ __forceinline__ V3 bMixd(V3 x, V3 y, double a) {
  const double b = 1.0 - a;
  return v3((float)((double)x.x * b + (double)y.x * a), (float)((double)x.y * b + (double)y.y * a),
            (float)((double)x.z * b + (double)y.z * a));
}
// lobe choice + new direction (B:399-422, B:268-294): 0 specular, 1 refract, 2 diffuse
__device__ __forceinline__ int bLobe(const BHit& res, V3 din, BRng& g, V3& dout) {
  V3 rd = bRandomDirection(res.N, g);
  double r = bRand(g);
  if (r < res.specularRate) {
    dout = bMixd(normalize(bReflect(din, res.N)), rd, res.roughness);
    return 0;
  } else if (res.specularRate <= r && r <= res.refractRate) {
    dout = bMixd(normalize(bRefract(din, res.N, (float)res.refractAngle)), -rd, res.refractRoughness);
    return 1;
  }
  dout = rd;
  return 2;
}

__global__ __launch_bounds__(BLOCK) void basicKernel(BasicParams p) {
  const int j = blockIdx.x * 16 + (threadIdx.x & 15);
  const int i = blockIdx.y * 16 + (threadIdx.x >> 4);
  uint32_t rays = 0;
  bool over = false;
  if (j < p.width && i < p.height) {
    const int W = p.width, H = p.height;
    BRng g;
    g.seed = ((uint32_t)j * 1973u + (uint32_t)i * 9277u + p.sample * 26699u + p.seed * 0x9E3779B9u) | 1u;
    g.rep = p.stream;
    g.pos = g.end = 0;
    g.over = false;
    if (p.stream) {
      const long long idx = ((long long)p.sample * H + i) * W + j;
      if (idx < p.nOffsets) {
        g.pos = p.offsets[idx];
        g.end = idx + 1 < p.nOffsets ? p.offsets[idx + 1] : p.streamN;
        g.end = g.end < p.streamN ? g.end : p.streamN;
      }
    }
    // pixel loop body B:367-429
    double xd = 2.0 * (double)j / (double)W - 1.0;
    double yd = 2.0 * (double)(H - i) / (double)H - 1.0;
    xd += (bRand(g) - 0.5) / (double)W;
    yd += (bRand(g) - 0.5) / (double)H;
    V3 coord = v3((float)xd, (float)yd, (float)1.1);  // SCREEN_Z B:27 is a double
    V3 dir = normalize(coord - v3(0, 0, 4.0f));
    BHit res;
    V3 color = v3(0, 0, 0);
    rays++;
    if (bShoot(p.shapes, p.nShapes, coord, dir, res)) {
      if (res.emissive) {
        color = res.color;
      } else {
        V3 nd;
        int lobe = bLobe(res, dir, g, nd);
        // pathTracing B:252-297 from depth 0: the recursion forms its products on the way
        // back up (pathTracing(depth + 1) * cosine [* srcColor] / P), so each vertex's
        // factors are kept and folded from the deepest vertex upward
        float cosv[BASIC_MAX_DEPTH + 1];
        V3 col[BASIC_MAX_DEPTH + 1];
        bool diff[BASIC_MAX_DEPTH + 1];
        const float P = 0.8f;  // B:264
        V3 S = res.P, d = nd, v = v3(0, 0, 0);
        int n = 0;
        for (int depth = 0; depth <= p.maxDepth; depth++) {
          BHit h;
          rays++;
          if (!bShoot(p.shapes, p.nShapes, S, d, h)) break;
          if (h.emissive) { v = h.color; break; }
          double r = bRand(g);
          if (r > (double)P) break;
          V3 nd2;
          int lb = bLobe(h, d, g, nd2);
          cosv[n] = fabsf(dot(-d, h.N));
          col[n] = h.color;
          diff[n] = lb == 2;
          n++;
          S = h.P;
          d = nd2;
        }
        for (int k = n - 1; k >= 0; k--) {
          v = v * cosv[k];
          if (diff[k]) v = v * col[k];
          v = v / P;
        }
        color = (lobe == 2) ? v * res.color : v;
        color = color * p.brightness;  // color *= BRIGHTNESS (glm casts the double to float)
      }
    }
    double* im = p.image + 3 * ((size_t)i * W + j);
    double r0 = p.reset ? 0.0 : im[0], r1 = p.reset ? 0.0 : im[1], r2 = p.reset ? 0.0 : im[2];
    r0 += color.x; r1 += color.y; r2 += color.z;  // *p += color.x ... (B:427-429)
    im[0] = r0; im[1] = r1; im[2] = r2;
    p.accum[(size_t)i * W + j] = make_float4((float)r0, (float)r1, (float)r2, 1.0f);
    over = g.over;
  }
  // wave-reduce the ray count, one atomic per wave
  for (int off = 32; off > 0; off >>= 1) rays += __shfl_down(rays, off, 64);
  if ((threadIdx.x & 63) == 0 && rays) atomicAdd(reinterpret_cast<unsigned long long*>(p.stats), (unsigned long long)rays);
  const unsigned long long ov = __ballot(over);
  if ((threadIdx.x & 63) == 0 && ov) atomicAdd(p.overruns, (unsigned long long)__popcll(ov));
}

// ------------------------------------------------------------ tile order
// One block per queue band, between frames: build the next frame's work items
// (TileCursor) from the costs the megakernel measured in this one.
//  * Split state: a wave runs its item's paths in lock step, so a tile whose
//    lanes take turns at long traversals lasts the sum of its slowest lanes --
//    for a few tiles most of a frame. A tile whose longest item cost more than
//    splitPct % of a wave's share of the band (band cost / waves per band)
//    is split once more (2^lg items of 64 >> lg pixels, lg <= 6); one whose
//    items became cheap (< 1/4 of that) is merged back one step.
//  * Order: items by their tile's longest item, descending, so the long ones
//    start first: a counting sort over 128 cost buckets (the cost's octave and
//    two more bits, ~19 % wide; order within a bucket is arbitrary) -- one pass
//    of LDS atomics instead of a bitonic sort's 55 barrier phases. Progressive
//    frames share camera and scene, so this frame's costs predict the next's.
// group > 1 sorts groups of consecutive tiles by summed cost and never splits.
constexpr int REORDER_BUCKETS = 128;
__device__ __forceinline__ int costBucket(unsigned long long c) {  // 0 = most expensive
  const unsigned v = (unsigned)min(c, 0xffffffffull) | 1u;
  const int oct = 31 - __clz(v);
  const int frac = oct >= 2 ? (int)((v >> (oct - 2)) & 3u) : (int)((v << (2 - oct)) & 3u);
  return REORDER_BUCKETS - 1 - (oct * 4 + frac);
}
__global__ __launch_bounds__(1024) void reorderKernel(int* cost, int* costMax, int* splitLg, int* ema, int* order,
                                                       int perQueue,
                                                       int orderCap, int numItems, int group, int numWaves,
                                                       int splitPct) {
  __shared__ int bucketOf[REORDER_MAX];  // each group's bucket
  __shared__ int rankG[REORDER_MAX];     // the group at each rank, most expensive first
  __shared__ int start[REORDER_BUCKETS];
  __shared__ int scan[1024];
  __shared__ int partialPos;
  __shared__ unsigned long long sumCost;
  const int q = blockIdx.x;
  const int base = q * perQueue;
  const int n = max(0, min(perQueue, numItems - base));
  const int ng = (n + group - 1) / group;  // groups of `group` consecutive tiles (the last may be short)
  const int lastSize = n - (ng - 1) * group;
  const bool splitting = group == 1 && splitLg != nullptr && splitPct > 0;
  if (threadIdx.x == 0) sumCost = 0;
  if (threadIdx.x < REORDER_BUCKETS) start[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long mySum = 0;
  for (int g = threadIdx.x; g < ng; g += blockDim.x) {
    const int t0 = base + g * group, t1 = min(t0 + group, base + n);
    for (int t = t0; t < t1; t++) mySum += (unsigned)max(cost[t], 0);
  }
  atomicAdd(&sumCost, mySum);
  __syncthreads();
  // a wave's share of the band's work: the cost above which an item forms the tail
  const unsigned long long share = sumCost / (unsigned long long)max(1, numWaves / NUM_QUEUES);
  const unsigned long long target = max(share * (unsigned long long)splitPct / 100ull, 1ull);
  for (int g = threadIdx.x; g < ng; g += blockDim.x) {
    unsigned long long c = 0;
    const int t0 = base + g * group, t1 = min(t0 + group, base + n);
    if (splitting) {
      const int t = t0;
      const unsigned long long m = (unsigned)max(costMax[t], 1);
      int lg = splitLg[t];
      if (m > target && lg < MAX_SPLIT_LG) lg++;
      else if (lg > 0 && 4 * m < target) lg--;
      splitLg[t] = lg;
      c = m;
      costMax[t] = 0;
    } else {
      for (int t = t0; t < t1; t++) c += (unsigned)max(cost[t], 1);
      if (costMax)
        for (int t = t0; t < t1; t++) costMax[t] = 0;
    }
    for (int t = t0; t < t1; t++) cost[t] = 0;
    if constexpr (PT_COST_EMA > 0) {  // a path's cost varies frame to frame: rank by the running estimate
      const unsigned long long e = (unsigned)ema[base + g];
      constexpr int S = PT_COST_EMA > 0 ? PT_COST_EMA : 1;  // weight of this frame: 2^-S
      c = e ? (((1ull << S) - 1) * e + min(c, 0x7fffffffull) + (1ull << (S - 1))) >> S : min(c, 0x7fffffffull);
      ema[base + g] = (int)c;
    }
    const int bk = costBucket(c);
    bucketOf[g] = bk;
    atomicAdd(&start[bk], 1);
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of the bucket counts, one wave
    const int lane = threadIdx.x;
    const int c0 = start[2 * lane], c1 = start[2 * lane + 1];
    int incl = c0 + c1;
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off, 64);
      if (lane >= off) incl += v;
    }
    const int excl = incl - c0 - c1;
    start[2 * lane] = excl;
    start[2 * lane + 1] = excl + c0;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < ng; g += blockDim.x) rankG[atomicAdd(&start[bucketOf[g]], 1)] = g;
  __syncthreads();
  int* out = order + (size_t)q * orderCap;
  if (splitting) {
    // item offsets: exclusive scan of 2^lg over the ranks (ceil(ng / 1024) ranks per thread)
    const int per = (ng + 1023) / 1024;
    const int r0 = min(ng, (int)threadIdx.x * per), r1 = min(ng, r0 + per);
    int local = 0;
    for (int r = r0; r < r1; r++) local += 1 << splitLg[base + rankG[r]];
    scan[threadIdx.x] = local;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int v = threadIdx.x >= (unsigned)off ? scan[threadIdx.x - off] : 0;
      __syncthreads();
      scan[threadIdx.x] += v;
      __syncthreads();
    }
    const int total = scan[1023];
    if (total <= orderCap) {
      int pos = scan[threadIdx.x] - local;
      for (int r = r0; r < r1; r++) {
        const int t = base + rankG[r];
        const int lg = splitLg[t];
        for (int sIdx = 0; sIdx < (1 << lg); sIdx++) out[pos++] = t | sIdx << ITEM_TILE_BITS | lg << 28;
      }
      if (threadIdx.x == 0) order[(size_t)NUM_QUEUES * orderCap + q] = total;
      return;
    }
    // no room: this frame unsplit, and the band starts over
    for (int r = threadIdx.x; r < ng; r += blockDim.x) splitLg[base + r] = 0;
  }
  for (int r = threadIdx.x; r < ng; r += blockDim.x)
    if (rankG[r] == ng - 1) partialPos = r;
  __syncthreads();
  for (int r = threadIdx.x; r < ng; r += blockDim.x) {
    const int g = rankG[r];
    const int off = r * group - (r > partialPos ? group - lastSize : 0);
    const int len = g == ng - 1 ? lastSize : group;
    for (int k = 0; k < len; k++) out[off + k] = base + g * group + k;
  }
  if (threadIdx.x == 0) order[(size_t)NUM_QUEUES * orderCap + q] = n;
}

hipError_t launchReorder(int* cost, int* costMax, int* splitLg, int* ema, int* order, int perQueue, int orderCap,
                         int numItems, int group, int numWaves, int splitPct, hipStream_t s) {
  if ((perQueue + group - 1) / group > REORDER_MAX || orderCap < perQueue) return hipErrorInvalidValue;
  hipLaunchKernelGGL(reorderKernel, dim3(NUM_QUEUES), dim3(1024), 0, s, cost, costMax, splitLg, ema, order, perQueue,
                     orderCap, numItems, group, numWaves, splitPct);
  return hipGetLastError();
}

// ------------------------------------------------------------ render kernel
__device__ __forceinline__ uint32_t waveSum(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// WAVES > 0: compiled for that many waves per SIMD (the latency-bound large
// scenes' variant, pt_runtime.cpp renderFrame)
template <int INTEG, bool CULL, bool COUNT, int WAVES = 0>
__global__ __launch_bounds__(BLOCK, WAVES > 0 ? WAVES
                                             : (INTEG == 0 ? PT_MIN_WAVES_LAMBERT
                                                           : INTEG == 2 ? PT_MIN_WAVES_MIS : PT_MIN_WAVES)) void renderKernel(
    RenderParams p) {
  __shared__ int s_stack[LDS_STACK * BLOCK];
  Stack st;
  st.init(s_stack, p.ovf, p.ovfDepth);
  st.reset();
  __shared__ unsigned s_drained;  // the work queues this block's waves found drained (TileCursor)
  if (threadIdx.x == 0) s_drained = 0;
  // the top of the tree (every ray's first node visits) staged in LDS once per block
#if PT_LDS_NODES > 0
  __shared__ float4 s_nodes[LDS_NODES * 4];
  {
    const bool w4 = PT_WIDE4 == 2 && !COUNT && p.scene.fast;  // the 4-wide tree's top
    const float4* src = w4 ? p.scene.fbvh4 : p.scene.fast ? p.scene.fbvh : p.scene.bvh;  // the tree traversed first
    // the copy's size from the staged tree's own record kind (never the other tree's: DESIGN.md §8)
    const int n = w4 ? p.scene.f4nTop * W4_F4 : p.scene.fast ? p.scene.fnTop * 4 : p.scene.nTop * 4;
    for (int i = threadIdx.x; i < n; i += BLOCK) s_nodes[i] = src[i];
  }
  __syncthreads();
  const float4* top = s_nodes;
#else
  __syncthreads();
  const float4* top = nullptr;
#endif
  Counters C = {0, 0, 0, 0, 0};
  const int lane = threadIdx.x & 63;
  const int home = blockIdx.x & (NUM_QUEUES - 1);
  __shared__ PacketEntry s_packet[BLOCK / 64][COUNT ? 1 : PKT_DEPTH];  // camera-ray packet stacks
  PacketEntry* pstack = s_packet[threadIdx.x >> 6];
  const int tilesPerShard = p.shardTiles;  // 8x8 wave tiles per shard tile
  const int sub = p.shardSize >> 3;        // wave tiles per shard-tile edge
#if PT_WAVE_TRACE
  const unsigned long long wStart = wall_clock64();
  unsigned long long wTiles = 0, wLongest = 0, wLongestAt = 0, wNodeIt = 0, wLeafIt = 0;
#endif
  TileCursor cur;
  cur.drained = &s_drained;
  // Each lane runs its pixel's whole path right after the tile's camera rays.
  // (Deferring the paths of the pixels that hit something to a per-wave LDS
  // queue and running them 64 at a time keeps every lane busy, but it mixes
  // tiles: 64-path batches made c2 0.77 ms instead of 0.55, 32-path batches
  // 0.59 -- the coherence of one tile's rays is worth more than full lanes.)
  int fr = 0;  // the claimed item's frame in the launch's batch
  int item = cur.next(p.queue, p.perQueue, p.numItems, home, fr, p.nFrames, p.tileOrder, p.orderCap);
  while (item >= 0) {
    // the item's frame: its sample index and colour buffer (accumulate)
    FrameRef fv;
    fv.col = p.col ? p.col + (size_t)fr * p.colStride * COL_F : nullptr;
    fv.sampleIndex = p.sampleIndex + (uint32_t)fr * p.sampleStride;
    const int w = itemTile(item);
    const long long t0 = COUNT ? 0 : clock64();
#if PT_WAVE_TRACE
    const unsigned long long tw0 = wall_clock64();
    const uint32_t n0 = C.nodes, l0 = C.tris, m0 = C.mats;
#endif
    const int j = w / tilesPerShard, s = w - j * tilesPerShard;
    const int g = j * p.world + p.rank;  // global shard tile id (row-major)
    const int gy = g / p.shardsX, gx = g - gy * p.shardsX;
    // a split item runs pixels [sub * n, (sub + 1) * n) of the tile (n = 64 >> lg), one per lane
    const int lg = itemLg(item), nLanes = 64 >> lg;
    const int k = itemSub(item) * nLanes + lane;
    const int px = gx * p.shardSize + (s % sub) * 8 + (k & 7);
    const int py = gy * p.shardSize + (s / sub) * 8 + (k >> 3);
    const bool valid = lane < nLanes && px < p.width && py < p.height;
    if (!COUNT && p.primHit) {  // camera rays already traced by primaryKernel
      const unsigned long long pm = primTileMask(p, fr, w);
      const int2 h = valid ? primOfSlot(pm, primTileEntries(p, fr, w), k) : make_int2(PRIM_MISS, 0);
      int tri = h.x;
      float t = __int_as_float(h.y);
      if (__ballot(valid && tri == PRIM_TILE)) {  // wave-uniform: the whole tile
        tri = primaryPacket<CULL>(p, fv, px, py, valid, st, C, top, pstack, t);
      } else if (valid && tri == PRIM_RETRACE) {  // in the reference order, as primaryPacket does
        uint32_t seed;
        const V3 dir = cameraRay(p, fv.sampleIndex, px, py, seed);
        const V3 eye = v3(p.eye[0], p.eye[1], p.eye[2]);
        tri = traceRay<false, CULL, false, Stack>(p.scene, eye, dir, t, st, C);
        if (tri < 0) accumulate(p, fv, px, py, sampleHdr(p.env, dir), C, false);
      }
      if (valid && tri >= 0) finishPixel<INTEG, CULL, COUNT>(p, fv, px, py, tri, t, st, C, top);
    } else if (!COUNT && (p.packets || p.binStart)) {
      float t;
      const int tri = primaryPacket<CULL>(p, fv, px, py, valid, st, C, top, pstack, t);
      if (valid && tri >= 0) finishPixel<INTEG, CULL, COUNT>(p, fv, px, py, tri, t, st, C, top);
    } else if (valid) {
      float t;
      const int tri = primaryPixel<CULL, COUNT>(p, fv, px, py, st, C, top, t);
      if (tri >= 0) finishPixel<INTEG, CULL, COUNT>(p, fv, px, py, tri, t, st, C, top);
    }
    if (!COUNT && p.tileCost && lane == 0) {
      const int dt = (int)min(clock64() - t0, (long long)0x3fffffff);
      atomicAdd(p.tileCost + w, dt);
      atomicMax(p.tileCostMax + w, dt);
    }
#if PT_WAVE_TRACE
    const unsigned long long tEnd = wall_clock64();
    wTiles++;
    uint32_t dn = C.nodes - n0, dl = C.tris - l0, dw = C.mats - m0;
    for (int off = 32; off > 0; off >>= 1) dw += (uint32_t)__shfl_xor(dw, off, 64);
    for (int off = 32; off > 0; off >>= 1) {
      dn = max(dn, (uint32_t)__shfl_xor(dn, off, 64));
      dl = max(dl, (uint32_t)__shfl_xor(dl, off, 64));
    }
    if (tEnd - tw0 > wLongest) {
      wNodeIt = dn;
      wLeafIt = dl | (unsigned long long)dw << 32;
      wLongest = tEnd - tw0;
      wLongestAt = (unsigned long long)__shfl(px, 0, 64) << 16 | (unsigned long long)__shfl(py, 0, 64);
    }
#endif
    item = cur.next(p.queue, p.perQueue, p.numItems, home, fr, p.nFrames, p.tileOrder, p.orderCap);
  }
#if PT_WAVE_TRACE
  if (p.waveTrace && lane == 0) {
    unsigned long long* r = p.waveTrace + 6 * ((size_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6));
    r[0] = wStart; r[1] = wall_clock64(); r[2] = wTiles | wLongestAt << 32; r[3] = wLongest;
    r[4] = wNodeIt; r[5] = wLeafIt;
  }
#endif
  addRays(p.rayShards, C.rays);
  if (COUNT) {
    uint32_t n = waveSum(C.nodes), t = waveSum(C.tris), m = waveSum(C.mats), x = waveSum(C.texels);
    if (lane == 0) {
      atomicAdd(reinterpret_cast<unsigned long long*>(p.stats + 1), (unsigned long long)n);
      atomicAdd(reinterpret_cast<unsigned long long*>(p.stats + 2), (unsigned long long)t);
      atomicAdd(reinterpret_cast<unsigned long long*>(p.stats + 3), (unsigned long long)m);
      atomicAdd(reinterpret_cast<unsigned long long*>(p.stats + 4), (unsigned long long)x);
    }
  }
}

// ------------------------------------------------------------ batch query
template <bool CULL>
__global__ __launch_bounds__(BLOCK) void traceKernel(TraceParams p) {
  __shared__ int s_stack[LDS_STACK * BLOCK];
  Stack st;
  st.init(s_stack, p.ovf, p.ovfDepth);
  const size_t gtid = (size_t)blockIdx.x * BLOCK + threadIdx.x;
  Counters C = {0, 0, 0, 0, 0};
  SceneView S = p.scene;  // no LDS copy of the top of the tree here
  S.nTop = 0;
  S.fnTop = 0;
  S.f4nTop = 0;
  Tracer<CULL, false> tr{S, st, C, nullptr};  // the runtime's tree when S.fast (reference-exact)
  for (size_t k = gtid; k < (size_t)p.n; k += (size_t)gridDim.x * BLOCK) {
    const float* r = p.rays + 6 * k;
    V3 o = v3(r[0], r[1], r[2]), d = v3(r[3], r[4], r[5]);
    float t;
    int tri = tr.trace(o, d, t);
    p.t[k] = tri >= 0 ? t : PT_INF;
    p.tri[k] = tri;
  }
}

// ------------------------------------------------------------ epilogues
// pass3.fsh:14-24 tonemap (+ optional gamma, commented out in the reference)
__device__ __forceinline__ V3 tonemapPixel(float4 c, float limit, float gamma) {
  float lum = 0.3f * c.x + 0.6f * c.y + 0.1f * c.z;
  float s = 1.0f / (1.0f + lum / limit);
  float r = c.x * s, g = c.y * s, b = c.z * s;
  if (gamma > 0.0f) {
    r = ptm_powf(r, 1.0f / gamma);
    g = ptm_powf(g, 1.0f / gamma);
    b = ptm_powf(b, 1.0f / gamma);
  }
  return v3(r, g, b);
}
__global__ void tonemapKernel(const float4* accum, float* rgb, int n, float limit, float gamma) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const V3 c = tonemapPixel(accum[i], limit, gamma);
  rgb[3 * i] = c.x;
  rgb[3 * i + 1] = c.y;
  rgb[3 * i + 2] = c.z;
}
// pass3's fragColor as the GLUT_RGBA window stores it (OpenglRayTracing/main.cpp glutInitDisplayMode,
// an 8-bit unsigned-normalised framebuffer): round(clamp(x, 0, 1) * 255), as one fused multiply-add
// (NaN -> 0)
__device__ __forceinline__ uint32_t unorm8(float x) {
  const float c = fminf(fmaxf(x, 0.0f), 1.0f);
  return (uint32_t)__builtin_fmaf(c, 255.0f, 0.5f);
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
// packed slots are (r, g, b): the running mean's alpha is 1 for every rendered pixel
// (IS:868-871 writes vec4(color, 1)), so the gather moves 12 bytes per pixel, not 16
__global__ void packKernel(PackParams p, const float4* accum, float* packed) {
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.count) return;
  int px, py;
  const float4 c = packedPixel(p, k, px, py) ? accum[(size_t)py * p.width + px] : make_float4(0, 0, 0, 0);
  packed[3 * k] = c.x;
  packed[3 * k + 1] = c.y;
  packed[3 * k + 2] = c.z;
}
__global__ void unpackKernel(PackParams p, float4* accum, const float* packed) {
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.count) return;
  int px, py;
  if (packedPixel(p, k, px, py))
    accum[(size_t)py * p.width + px] = make_float4(packed[3 * k], packed[3 * k + 1], packed[3 * k + 2], 1.0f);
}

// The displayed frame (pass3 into the 8-bit window) of a screen-tile split: each rank packs its
// own tiles' display values (3 bytes per pixel, packed order) and rank 0 writes its own tiles and
// unpacks every other rank's into one RGBA8 image -- a quarter of the f32 gather's bytes over xGMI.
__global__ void displayPackKernel(PackParams p, const float4* accum, float limit, float gamma, uint8_t* packed) {
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.count) return;
  int px, py;
  uint32_t r = 0, g = 0, b = 0;
  if (packedPixel(p, k, px, py)) {
    const V3 c = tonemapPixel(accum[(size_t)py * p.width + px], limit, gamma);
    r = unorm8(c.x), g = unorm8(c.y), b = unorm8(c.z);
  }
  packed[3 * k] = (uint8_t)r;
  packed[3 * k + 1] = (uint8_t)g;
  packed[3 * k + 2] = (uint8_t)b;
}
__global__ void displayOwnKernel(PackParams p, const float4* accum, float limit, float gamma, uchar4* image) {
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.count) return;
  int px, py;
  if (!packedPixel(p, k, px, py)) return;
  const size_t i = (size_t)py * p.width + px;
  const V3 c = tonemapPixel(accum[i], limit, gamma);
  image[i] = make_uchar4((uint8_t)unorm8(c.x), (uint8_t)unorm8(c.y), (uint8_t)unorm8(c.z), 255);
}
// blockIdx.y = rank - 1 of ranks 1..world-1 (their packed buffers in d.src)
__global__ void displayUnpackKernel(RanksUnpack d, uchar4* image) {
  const int rank = blockIdx.y + 1;
  const uint8_t* src = static_cast<const uint8_t*>(d.src[rank]);
  if (!src) return;
  PackParams p = d.base;
  p.rank = rank;
  p.count = d.count[rank];
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.count) return;
  int px, py;
  if (packedPixel(p, k, px, py))
    image[(size_t)py * p.width + px] = make_uchar4(src[3 * k], src[3 * k + 1], src[3 * k + 2], 255);
}

// unpackKernel of ranks 1..world-1 in one launch (blockIdx.y = rank - 1): rank 0's reassembly of
// a gather of the f32 running means after each batch of frames
__global__ void unpackRanksKernel(RanksUnpack d, float4* accum) {
  const int rank = blockIdx.y + 1;
  const float* src = static_cast<const float*>(d.src[rank]);
  if (!src) return;
  PackParams p = d.base;
  p.rank = rank;
  p.count = d.count[rank];
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.count) return;
  int px, py;
  if (packedPixel(p, k, px, py))
    accum[(size_t)py * p.width + px] = make_float4(src[3 * k], src[3 * k + 1], src[3 * k + 2], 1.0f);
}

// the running means of a batch of pipelined frames (accumulate's update, deferred to frame
// order): frame f's colours at col + f * colStride, its weight 1 / (frameCounter + f + 1); the
// pixel's mean after each frame is the one serial frames store (mixf of the same floats)
__global__ void mixKernel(PackParams p, float4* accum, const float* col, size_t colStride, int nFrames,
                          uint32_t frameCounter) {
  long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.count) return;
  int px, py;
  if (!packedPixel(p, k, px, py)) return;
  const size_t i = (size_t)py * p.width + px;
  float4 a = ldStream(accum + i);
  for (int f = 0; f < nFrames; f++) {
    const float3 c = ldCol(col + ((size_t)f * colStride + k) * COL_F);  // slot k of the share (shareIndex)
    const float w = 1.0f / (float)(frameCounter + (uint32_t)f + 1u);
    a = make_float4(mixf(a.x, c.x, w), mixf(a.y, c.y, w), mixf(a.z, c.z, w), 1.0f);
  }
  stStream(accum + i, a);
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
static hipError_t launchRenderI(const RenderParams& p, int grid, hipStream_t s, bool cull, bool count, bool wide) {
  if (count) {
    hipLaunchKernelGGL((renderKernel<I, false, true>), dim3(grid), dim3(BLOCK), 0, s, p);
  } else if (cull && wide && I != 0) {
    hipLaunchKernelGGL((renderKernel<I, true, false, WIDE_WAVES>), dim3(grid), dim3(BLOCK), 0, s, p);
  } else if (cull) {
    hipLaunchKernelGGL((renderKernel<I, true, false>), dim3(grid), dim3(BLOCK), 0, s, p);
  } else {
    hipLaunchKernelGGL((renderKernel<I, false, false>), dim3(grid), dim3(BLOCK), 0, s, p);
  }
  return hipGetLastError();
}

hipError_t launchRender(const RenderParams& p, int integrator, int grid, hipStream_t s, bool cull, bool count,
                        bool wide) {
  switch (integrator) {
    case 0: return launchRenderI<0>(p, grid, s, cull, count, wide);
    case 1: return launchRenderI<1>(p, grid, s, cull, count, wide);
    default: return launchRenderI<2>(p, grid, s, cull, count, wide);
  }
}

hipError_t renderBlocksPerCU(int integrator, bool cull, bool count, bool wide, int* nb) {
  const void* f;
#define PT_SEL(I)                                                                              \
  f = count ? (const void*)renderKernel<I, false, true>                                        \
            : (cull ? (wide && I != 0 ? (const void*)renderKernel<I, true, false, WIDE_WAVES>   \
                                      : (const void*)renderKernel<I, true, false>)             \
                    : (const void*)renderKernel<I, false, false>)
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

__global__ void basicWidenKernel(const float4* accum, double* image, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 a = accum[i];
  image[3 * i] = (double)a.x;
  image[3 * i + 1] = (double)a.y;
  image[3 * i + 2] = (double)a.z;
}
__global__ void basicNarrowKernel(const double* image, float4* accum, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  accum[i] = make_float4((float)image[3 * i], (float)image[3 * i + 1], (float)image[3 * i + 2], 1.0f);  // basicKernel's store
}
hipError_t launchBasicWiden(const float4* accum, double* image, long n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(basicWidenKernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, accum, image, n);
  return hipGetLastError();
}
hipError_t launchBasicNarrow(const double* image, float4* accum, long n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(basicNarrowKernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, image, accum, n);
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

hipError_t launchPack(const PackParams& p, const float4* accum, float* packed, hipStream_t s) {
  if (p.count <= 0) return hipSuccess;
  hipLaunchKernelGGL(packKernel, dim3((unsigned)((p.count + 255) / 256)), dim3(256), 0, s, p, accum, packed);
  return hipGetLastError();
}
hipError_t launchMix(const PackParams& p, float4* accum, const float* col, size_t colStride, int nFrames,
                     uint32_t frameCounter, hipStream_t s) {
  if (p.count <= 0 || nFrames <= 0) return hipSuccess;
  hipLaunchKernelGGL(mixKernel, dim3((unsigned)((p.count + 255) / 256)), dim3(256), 0, s, p, accum, col, colStride,
                     nFrames, frameCounter);
  return hipGetLastError();
}
// Env::trig: SampleHdr's sines and cosines (IS:582-583) of every integer entry of a compact sample
// table, by the same device functions of the same floats as hdrDirFromCache
__global__ void envTrigKernel(float2* trig, int w, int h) {
  const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (k > w + h + 1) return;
  float sn, cs;
  if (k <= h) ptm_sincosf(hdrTheta((float)k / (float)h), &sn, &cs);
  else ptm_sincosf(hdrPhi((float)(k - h - 1) / (float)w), &sn, &cs);
  trig[k] = make_float2(sn, cs);
}
hipError_t launchEnvTrig(float2* trig, int w, int h, hipStream_t s) {
  if (!trig || w <= 0 || h <= 0) return hipErrorInvalidValue;
  const int n = w + h + 2;
  hipLaunchKernelGGL(envTrigKernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, trig, w, h);
  return hipGetLastError();
}
// Env::light: what a light sample of each sample-table entry reads (IS:778-779), computed once with
// the operations sampleHdrDir + hdrColorPdf apply to it in a frame
__global__ void envLightKernel(Env e, uint2* light) {
  const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (k >= (e.w + 1) * (e.h + 1)) return;
  const int y = k / (e.w + 1), x = k - y * (e.w + 1);
  const float2 t = e.trig[y], f = e.trig[e.h + 1 + x];
  const V3 L = v3(t.y * f.y, t.x, t.y * f.x);
  float u, w;
  toSpherical(normalize(L), u, w);
  const uint2 raw = e.hdr8[texIndex(e.w, e.h, u, w)];
  V3 color;
  float pdf;
  hdrColorPdfOf(e, decodeHdr8(raw), w, color, pdf);
  light[k] = make_uint2(raw.x, __float_as_uint(pdf));
}
hipError_t launchEnvLight(const Env& e, uint2* light, hipStream_t s) {
  if (!light || !e.trig || !e.hdr8 || e.w <= 0 || e.h <= 0) return hipErrorInvalidValue;
  const int n = (e.w + 1) * (e.h + 1);
  hipLaunchKernelGGL(envLightKernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, e, light);
  return hipGetLastError();
}
hipError_t launchDisplayPack(const PackParams& p, const float4* accum, float limit, float gamma, uint8_t* packed,
                             hipStream_t s) {
  if (p.count <= 0) return hipSuccess;
  hipLaunchKernelGGL(displayPackKernel, dim3((unsigned)((p.count + 255) / 256)), dim3(256), 0, s, p, accum, limit,
                     gamma, packed);
  return hipGetLastError();
}
hipError_t launchDisplayOwn(const PackParams& p, const float4* accum, float limit, float gamma, uchar4* image,
                            hipStream_t s) {
  if (p.count <= 0) return hipSuccess;
  hipLaunchKernelGGL(displayOwnKernel, dim3((unsigned)((p.count + 255) / 256)), dim3(256), 0, s, p, accum, limit,
                     gamma, image);
  return hipGetLastError();
}
hipError_t launchUnpackRanks(const RanksUnpack& d, int world, float4* accum, hipStream_t s) {
  long most = 0;
  for (int k = 1; k < world; k++) most = d.count[k] > most ? d.count[k] : most;
  if (world < 2 || most <= 0) return hipSuccess;
  hipLaunchKernelGGL(unpackRanksKernel, dim3((unsigned)((most + 255) / 256), (unsigned)(world - 1)), dim3(256), 0, s,
                     d, accum);
  return hipGetLastError();
}
hipError_t launchDisplayUnpack(const RanksUnpack& d, int world, uchar4* image, hipStream_t s) {
  long most = 0;
  for (int k = 1; k < world; k++) most = d.count[k] > most ? d.count[k] : most;
  if (world < 2 || most <= 0) return hipSuccess;
  hipLaunchKernelGGL(displayUnpackKernel, dim3((unsigned)((most + 255) / 256), (unsigned)(world - 1)), dim3(256), 0, s,
                     d, image);
  return hipGetLastError();
}
hipError_t launchUnpack(const PackParams& p, float4* accum, const float* packed, hipStream_t s) {
  if (p.count <= 0) return hipSuccess;
  hipLaunchKernelGGL(unpackKernel, dim3((unsigned)((p.count + 255) / 256)), dim3(256), 0, s, p, accum, packed);
  return hipGetLastError();
}

}  // namespace pt
