// pt_regen.hip -- frame kernel selected by PT_FLAG_REGEN: a persistent path state machine
// with per-lane path regeneration.
//
// Every lane owns one path at a time and runs one loop: trace the lane's
// current ray (closest hit, or any hit for an env shadow ray) through the single
// traversal call site, then advance the path by one event (primary hit/miss,
// bounce hit/miss, shadow result). A lane whose path has ended writes its
// pixel's running mean and immediately takes the next pixel of its wave's 8x8
// tile (ballot + prefix over the idle lanes); a wave takes a new tile from the
// per-XCD-group work queues when its tile is used up. Lanes therefore never
// idle while their neighbours finish longer paths, and only path state (not the
// traversal or BRDF temporaries) is live across the traversal loop, which keeps
// the register file -- and so occupancy -- well below the one-call-per-bounce
// megakernel's.
//
// Per path the sequence of random numbers, rays and floating-point operations
// is exactly that of main()/pathTracing*() in pass1.fsh (and of the lock-step
// megakernel in pt_kernels.hip and the CPU checker), so images are bit-identical.
// Reference: ImportanceSampling_LowDiscrepancySequence/shaders/pass1.fsh (IS)
// main IS:844-872, pathTracingImportanceSampling IS:761-841; DisneyBRDF
// pathTracing D:443-481; OpenglRayTracing pathTracing O:329-364.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_device.h"
#include "pt_kernels.h"
#include "pt_trace.h"

namespace pt {

#ifndef PT_REGEN_LDS_STACK
#define PT_REGEN_LDS_STACK 16
#endif
constexpr int REGEN_LDS_STACK = PT_REGEN_LDS_STACK;
// minimum waves per SIMD the register allocator must allow (uniform integrators
// fit 128 VGPRs without spilling; the MIS state machine does not)
// Dynamic ray fetch for the 4-wide walk (pt_trace.h walk4Run): a wave stops walking as soon
// as this many of its walking lanes are done, and those lanes shade and take their next ray
// while the others resume their walks (0 = every walk runs to its end first, traceRay4).
#ifndef PT_REGEN_YIELD
#define PT_REGEN_YIELD 40  // c5: 0 (off) 6.97 ms, 8 6.98, 16 6.59, 32 5.78, 40 5.64, 48 5.63-5.71, 56 5.85, 60 6.17
#endif
#ifndef PT_REGEN_MIN_WAVES_U
#define PT_REGEN_MIN_WAVES_U 4
#endif
#ifndef PT_REGEN_MIN_WAVES_MIS
#define PT_REGEN_MIN_WAVES_MIS 1
#endif

// 4-wide nodes of the runtime tree (breadth-first ids) the wide variant stages in LDS per block:
// 128 (16 KB, with the 16 KB stack rows 4 blocks per CU) measured c2 0.248 -> 0.245 ms and
// c5 7.98 -> 7.28 ms against 64; 192 (the LDS limit at 4 blocks) c2 0.247, c5 7.60
#ifndef PT_REGEN_TOP4
#define PT_REGEN_TOP4 128
#endif
// ... and at 3 waves per SIMD (the uniform integrators' variant): 128 too (c2 0.235 ms per frame;
// 256, which 3 blocks per CU would fit, 0.240)
#ifndef PT_REGEN_TOP4_3
#define PT_REGEN_TOP4_3 128
#endif
constexpr int regenTop4W(int waves) { return waves == 3 ? PT_REGEN_TOP4_3 : PT_REGEN_TOP4; }

// The camera-ray pass's results of a claimed tile loaded at once (lane k: slot k) and read by
// the refilling lanes from their neighbours (0: each refilling lane loads its own). For the
// uniform integrators only: c2 0.2226 -> 0.2173 ms per frame; the MIS kernel (4 waves, at its
// register limit) spills more with the tile's results live, c5 5.69 -> 5.95 ms.
#ifndef PT_TILE_PRIM
#define PT_TILE_PRIM 1
#endif
// (The MIS kernel keeps the per-lane load: at its 128-VGPR limit it spilled 36 more VGPRs with the
// hand-out's state; materials staged in LDS per block measured c2 -0.6 %, within noise. Both knobs
// were deleted in round 6, git history keeps them.)

enum : int { K_NONE = 0, K_PRIMARY = 1, K_BOUNCE = 2, K_SHADOW = 3 };

struct PathState {
  int px, py;
  int fr;        // the pixel's frame in the launch's batch (RenderParams::nFrames)
  int kind;      // the ray in flight (K_*)
  int bounce;    // bounce index of the K_BOUNCE / K_SHADOW ray
  uint32_t seed;
  V3 o, d;       // ray in flight
  V3 Lo, hist;
  V3 Le0;        // the camera hit's emission (uniform integrators) ...
  int mat0;      // ... or its material (MIS: the emission reloaded when the path ends, camEmission)
  V3 f_r;        // BRDF value of the bounce ray in flight
  float cosL;    // cosine_i (uniform) / NdotL (MIS) of the bounce ray
  float pdfB;    // pdf_brdf of the MIS bounce ray
  V3 Lb;         // MIS: the BRDF ray traced after the shadow ray
  V3 shC;        // MIS: unoccluded env contribution of the shadow ray
  bool haveB;    // MIS: a BRDF ray follows the shadow ray
};

__device__ __forceinline__ uint32_t sampleOf(const RenderParams& p, const PathState& s) {
  return p.sampleIndex + (uint32_t)s.fr * p.sampleStride;
}

__device__ __forceinline__ void writeAccum(const RenderParams& p, const PathState& s, V3 color) {
  const int px = s.px, py = s.py;
  if (p.col) {  // pipelined frame: the sample colour; mixKernel updates the running mean in frame order
    stCol(p.col + ((size_t)s.fr * p.colStride + shareIndex(p, px, py)) * COL_F, color.x, color.y, color.z);
    return;
  }
  float4* a = p.accum + (size_t)py * p.width + px;
  float4 old = ldStream(a);
  float w = 1.0f / (float)(p.frameCounter + 1u);
  stStream(a, make_float4(mixf(old.x, color.x, w), mixf(old.y, color.y, w), mixf(old.z, color.z, w), 1.0f));
}

// the camera hit's emission Le (IS:865 color = Le + Li): the MIS paths (8-16 bounces) keep its
// material index and reload it at the end rather than hold three floats across every walk (c5
// 5.74 -> 5.57 ms per frame, the MIS kernel's scratch 164 -> 148 B per lane); the 2-bounce
// uniform paths keep the floats (c2 0.2090 vs 0.2108 ms with the reload)
template <int INTEG>
__device__ __forceinline__ V3 camEmission(const RenderParams& p, const PathState& s) {
  return INTEG == 2 ? emissiveMat(p.scene, s.mat0) : s.Le0;
}

// the set bits of a wave-wide mask below the calling lane (v_mbcnt: no 64-bit lane mask held in VGPRs)
__device__ __forceinline__ int rankBelow(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// the first pixel of 8x8 wave tile `tile` of this context's screen-tile share
__device__ __forceinline__ int tilePx(const RenderParams& p, int tile, int sub) {
  const int j = tile / p.shardTiles, sI = tile - j * p.shardTiles;
  const int g = j * p.world + p.rank;
  return (g % p.shardsX) * p.shardSize + (sI % sub) * 8;
}
__device__ __forceinline__ int tilePy(const RenderParams& p, int tile, int sub) {
  const int j = tile / p.shardTiles, sI = tile - j * p.shardTiles;
  const int g = j * p.world + p.rank;
  return (g / p.shardsX) * p.shardSize + (sI / sub) * 8;
}

// main IS:846-850: seed and camera ray of pixel (px, py)
__device__ __forceinline__ void startPath(const RenderParams& p, PathState& s) {
  const int W = p.width, H = p.height;
  s.seed = ((uint32_t)s.px * 1973u + (uint32_t)s.py * 9277u + sampleOf(p, s) * 26699u) | 1u;
  float pixx = (float)(2 * s.px + 1) / (float)W - 1.0f;
  float pixy = (float)(2 * s.py + 1) / (float)H - 1.0f;
  float ax = (randf(s.seed) - 0.5f) / (float)W;
  float ay = (randf(s.seed) - 0.5f) / (float)H;
  float x = pixx + ax, y = pixy + ay, z = -1.5f;
  const float* M = p.cam;
  V3 c0 = v3(M[0], M[1], M[2]), c1 = v3(M[4], M[5], M[6]), c2 = v3(M[8], M[9], M[10]), c3 = v3(M[12], M[13], M[14]);
  s.d = normalize((c0 * x + c1 * y) + (c2 * z + c3 * 0.0f));
  s.o = v3(p.eye[0], p.eye[1], p.eye[2]);
  s.kind = K_PRIMARY;
  s.bounce = 0;
  s.Lo = v3(0, 0, 0);
  s.hist = v3(1, 1, 1);
}

// The path has a new surface hit `hit` at bounce index nb: sample the next
// ray(s) (O:335-345, D:448-456, IS:766-816) or end the path. Returns false when
// the path ends.
template <int INTEG>
__device__ __forceinline__ bool continueFromHit(const RenderParams& p, PathState& s, const Hit& hit, int nb) {
  if (nb >= p.maxBounce) return false;
  s.bounce = nb;
  s.o = hit.P;
  if (INTEG != 2) {
    V3 N = hit.N;
    V3 L = toNormalHemisphere(sampleHemisphereRand(s.seed), N);
    s.cosL = fmaxf(0.0f, dot(L, N));
    if (INTEG == 0) {
      s.f_r = hit.m.baseColor / PT_PI;
    } else {
      V3 tangent, bitangent;
      getTangent(N, tangent, bitangent);
      s.f_r = brdfAniso(-hit.viewDir, N, L, tangent, bitangent, hit.m);
    }
    s.d = L;
    s.kind = K_BOUNCE;
    return true;
  }
  V3 V = -hit.viewDir;
  V3 N = hit.N;
  float r1 = randf(s.seed);
  float r2 = randf(s.seed);
  int ent;
  V3 Ldir = sampleHdrDir(p.env, r1, r2, &ent);
  bool shadow = false;
  if (dot(N, Ldir) > 0.0f) {  // IS:775-790; added if the shadow ray escapes
    V3 L = Ldir;
    V3 color;
    float pdf_light;
    hdrLightColorPdf(p.env, ent, L, color, pdf_light);
    V3 f_r = brdfIso(V, N, L, hit.m);
    float pdf_brdf = brdfPdf(V, N, L, hit.m);
    float mis_weight = misWeight(pdf_light, pdf_brdf);
    V3 c = ((s.hist * mis_weight) * color) * f_r;
    s.shC = (c * dot(N, L)) / pdf_light;
    shadow = true;
  }
  const uint32_t gi = grayCode(sampleOf(p, s) + 1u);
  float u = sobolf(2u * (uint32_t)nb, gi);
  float v = sobolf(2u * (uint32_t)nb + 1u, gi);
  cranleyPatterson(s.px, s.py, u, v);
  float xi_3 = randf(s.seed);
  V3 L = sampleBRDF(u, v, xi_3, V, N, hit.m);
  float NdotL = dot(N, L);
  s.haveB = false;
  if (NdotL > 0.0f) {
    V3 f_r = brdfIso(V, N, L, hit.m);
    float pdf_brdf = brdfPdf(V, N, L, hit.m);
    // IS:816: pdf <= 0 ends the path (the reference traces the ray first and discards it)
    if (pdf_brdf > 0.0f) {
      s.f_r = f_r;
      s.cosL = NdotL;
      s.pdfB = pdf_brdf;
      s.Lb = L;
      s.haveB = true;
    }
  }
  if (shadow) {
    s.d = Ldir;
    s.kind = K_SHADOW;
    return true;
  }
  if (s.haveB) {
    s.d = s.Lb;
    s.kind = K_BOUNCE;
    return true;
  }
  return false;
}

// Advance the path by the result (tri, t) of its ray in flight. Returns false
// when the path has ended (its final color in `color`). A camera ray's hit and a
// bounce ray's hit go through ONE finishHit and ONE continueFromHit (the same
// operations on the same values as separate paths would make): the lanes of a wave
// holding either kind shade together, and each call site of advance holds one copy
// of the shading code (the MIS wide kernel 14.3k -> 11.0k instructions; c2 and c5
// frame times unchanged, tools/tune.py). Shading the camera-ray pass's hits in the
// main loop instead of the refill loop (no second call site) made the kernel smaller
// still (7.5k) but slower -- c2 0.233 -> 0.266 ms, c5 5.55 -> 5.64 -- the lanes
// holding them sat out a walk step before their first bounce.
template <int INTEG>
__device__ __forceinline__ bool advance(const RenderParams& p, PathState& s, int tri, float t, V3& color) {
  const SceneView& S = p.scene;
  if (s.kind == K_SHADOW) {  // IS:776-790
    if (tri < 0) s.Lo = s.Lo + s.shC;
    if (!s.haveB) {
      color = camEmission<INTEG>(p, s) + s.Lo;
      return false;
    }
    s.d = s.Lb;
    s.kind = K_BOUNCE;
    return true;
  }
  const bool primary = s.kind == K_PRIMARY;
  if (tri < 0) {
    if (primary) {  // IS:857-859
      color = sampleHdr(p.env, s.d);
      return false;
    }
    if (INTEG == 2) {  // IS:819-829
      V3 c;
      float pdf_light;
      hdrColorPdf(p.env, s.d, c, pdf_light);
      float mis_weight = misWeight(s.pdfB, pdf_light);
      V3 cc = ((s.hist * mis_weight) * c) * s.f_r;
      s.Lo = s.Lo + (cc * s.cosL) / s.pdfB;
    } else {  // O:347-360 / D:463-479
      const float pdf = 1.0f / (2.0f * PT_PI);
      V3 sky = sampleHdr(p.env, s.d);
      s.Lo = s.Lo + ((s.hist * sky) * s.f_r * s.cosL) / pdf;
    }
    color = camEmission<INTEG>(p, s) + s.Lo;
    return false;
  }
  Hit hit;
  finishHit(S, tri, s.o, s.d, t, hit);  // IS:833-837 (a bounce), IS:852-856 (the camera ray)
  const V3 Le = hit.m.emissive;
  if (primary) {
    if (INTEG == 2) s.mat0 = hit.matId;
    else s.Le0 = Le;
  } else {
    const float pdf = INTEG == 2 ? s.pdfB : 1.0f / (2.0f * PT_PI);
    s.Lo = s.Lo + ((s.hist * Le) * s.f_r * s.cosL) / pdf;
    s.hist = s.hist * ((s.f_r * s.cosL) / pdf);
  }
  if (continueFromHit<INTEG>(p, s, hit, primary ? 0 : s.bounce + 1)) return true;
  color = camEmission<INTEG>(p, s) + s.Lo;
  return false;
}

// WAVES > 0: compiled for that many waves per SIMD (large scenes, pt_runtime.cpp renderOne).
// W4: rays walk the 4-wide runtime tree when p.scene.fast (pt_trace.h traceRay4), results
// checked against the uploaded tree and retraced through it on a tie or an unreachable hit.
// FULL (with W4): the whole 4-wide tree in LDS -- dynamic shared memory, p.scene.f4nTop =
// every node, swizzled (pt_trace.h loadNode4Lds) -- one block of BS threads (all the waves a CU
// holds) sharing one copy: a walk's node visits leave the texture data path to the leaf
// records.
template <int INTEG, bool CULL, int WAVES = 0, bool W4 = false, int BS = BLOCK, bool FULL = false>
__global__ __launch_bounds__(BS, WAVES > 0 ? WAVES : (INTEG == 2 ? PT_REGEN_MIN_WAVES_MIS : PT_REGEN_MIN_WAVES_U)) void regenKernel(
    RenderParams p) {
  static_assert(!FULL || W4, "the LDS tree is the 4-wide one");
  static_assert(!FULL || PT_REGEN_YIELD > 0, "the whole LDS tree is walked by walk4Run (loadNode4Lds) only");
  constexpr bool TILE_PRIM = PT_TILE_PRIM && INTEG != 2;
  __shared__ int s_stack[REGEN_LDS_STACK * BS];
  StackT<REGEN_LDS_STACK, BS> st;
  st.init(s_stack, p.ovf, p.ovfDepth);
  st.reset();
  __shared__ unsigned s_drained;  // the work queues this block's waves found drained (TileCursor)
  if (threadIdx.x == 0) s_drained = 0;
  // the top of the tree (every ray's first node visits) -- or all of it -- staged in LDS once per block
#if PT_LDS_NODES > 0
  constexpr int TOP4 = regenTop4W(WAVES);
  constexpr int TOPF4 = FULL ? 1 : (W4 && TOP4 * W4_F4 > LDS_NODES * 4) ? TOP4 * W4_F4 : LDS_NODES * 4;
  __shared__ float4 s_nodes[TOPF4];
  extern __shared__ float4 s_tree[];  // FULL: f4nTop * W4_LDS_F4 float4 (launch's dynamic LDS)
  if (FULL) {
    const float4* src = p.scene.fbvh4;
    const int n = p.scene.f4nTop * W4_LDS_F4;
    for (int i = threadIdx.x; i < n; i += BS) s_tree[i] = src[W4_F4 * (i / W4_LDS_F4) + i % W4_LDS_F4];
  } else {
    const bool w4 = W4 && p.scene.fast;
    const float4* src = w4 ? p.scene.fbvh4 : p.scene.bvh;
    const int n = w4 ? p.scene.f4nTop * W4_F4 : p.scene.nTop * 4;  // the staged tree's own record size
    for (int i = threadIdx.x; i < n; i += BS) s_nodes[i] = src[i];
  }
  __syncthreads();
  const float4* top = FULL ? s_tree : s_nodes;
#else
  __syncthreads();
  const float4* top = nullptr;
#endif
  Counters C = {0, 0, 0, 0, 0};
  const int lane = threadIdx.x & 63;
  const int home = blockIdx.x & (NUM_QUEUES - 1);
  const int sub = p.shardSize >> 3;
  TileCursor cur;     // wave-uniform
  cur.drained = &s_drained;
  int tile = -1;      // current 8x8 wave tile (wave-uniform)
  int tileFr = 0;     // its frame in the launch's batch (wave-uniform)
  int cursor = 64;    // next unused pixel slot of the tile (wave-uniform; TILE_PRIM: index into s_slot)
  int nValid = 0;     // TILE_PRIM: slots of the tile that need a path (wave-uniform)
  bool drained = false;  // TILE_PRIM: the work queues had nothing left for this wave (wave-uniform)
  uint32_t tmaskLo = 0, tmaskHi = 0;  // !TILE_PRIM: the claimed tile's camera-ray mask (wave-uniform)
  // TILE_PRIM: the tile's slots that need a path, in slot order, and their camera-ray results (this
  // wave's rows; in LDS rather than registers, which the walk needs)
  __shared__ unsigned char s_slotAll[TILE_PRIM ? BS : 1];
  __shared__ int2 s_hitAll[TILE_PRIM ? BS : 1];
  const int waveBase = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));  // scalar
  unsigned char* s_slot = s_slotAll + (TILE_PRIM ? waveBase : 0);
  int2* s_hit = s_hitAll + (TILE_PRIM ? waveBase : 0);
  bool active = false;
  bool walking = false;  // PT_REGEN_YIELD: the lane's ray has a walk in progress (w, st)
  Walk4 w;
  PathState s;
  s.px = s.py = s.fr = 0;
  s.kind = K_NONE;
#if PT_WAVE_TRACE
  // diagnostics build: {start, end, tiles | last lone lane's pixel << 32, last successful claim,
  // loop iterations, iterations with at most 4 lanes active} (100 MHz wall clock, tools/wave_trace.py --regen)
  const unsigned long long wStart = wall_clock64();
  unsigned long long wTiles = 0, wLastClaim = wStart, wIters = 0, wThin = 0, wLonePix = 0;
#endif
#if PT_PHASE_STATS
  // diagnostics build: per wave, in LDS (first active lane adds): [0] refill cycles, [1] walk
  // cycles, [2] reference-check cycles, [3] shading cycles, [4] main-loop iterations, [5] lanes
  // walking, [6] lanes shading, [7]/[8] node iterations / lanes, [9]/[10] pair tests / lanes,
  // [11] refill iterations, [12] lanes whose walk ran out of the yield, [13] walk calls that end
  // every walk, [14] retraced lanes, [15] wave lifetime (clock64 cycles); the TILE_PRIM hand-out:
  // [16] hand-out cycles, [17] tile claims, [18] claim cycles (atomic + camera-ray results),
  // [19] camera-hit shading cycles, [20] lanes shaded there, [21] camera-hit shading passes
  __shared__ unsigned long long s_ph[BS / 64][PHASE_WORDS];
  unsigned long long* ph = s_ph[threadIdx.x >> 6];
  if (lane < PHASE_WORDS) ph[lane] = 0;
  const long long phStart = clock64();
#define PH_ADD(k, x)                                                         \
  do {                                                                       \
    const unsigned long long v_ = (unsigned long long)(x); /* every lane */ \
    const unsigned long long m_ = __ballot(1);                               \
    if (__lane_id() == __ffsll((unsigned long long)m_) - 1) ph[k] += v_;     \
  } while (0)
#else
  unsigned long long* ph = nullptr;
#define PH_ADD(k, x) \
  do {               \
  } while (0)
#endif
  while (true) {
#if PT_PHASE_STATS
    const long long phA = clock64();
#endif
    if constexpr (TILE_PRIM) {
      // regenerate (uniform integrators): idle lanes take the next pixels of the wave's tile that
      // need a path -- the claimed tile's camera-ray results are loaded at once (lane k: slot k)
      // and its non-sky slots compacted into s_slot, so one pass hands every idle lane a pixel
      // (sky pixels, finished by the camera-ray pass, are never handed out) -- and then the camera
      // hits taken here are shaded together, once (shading inside the hand-out loop ran that code
      // once per hand-out pass, for a few lanes each time)
      while (true) {
        bool pend = false;
        int2 hP = make_int2(0, 0);
#if PT_PHASE_STATS
        const long long phH = clock64();
#endif
        while (true) {
          PH_ADD(11, 1);
          const unsigned long long idle = __ballot(!active);
          if (idle == 0) break;
          if (cursor >= nValid) {
#if PT_PHASE_STATS
            const long long phC = clock64();
            PH_ADD(17, 1);
#endif
            // (a claim -- the device-scope atomic, then the tile's camera-ray results -- is 1.6-2.3 us
            // and 10-13 % of a c2 wave's time, PT_PHASE_STATS; measured slower: claiming the wave's
            // next tile ahead, c2 0.1807 -> 0.1841 ms, c5 4.25 -> 4.29; 2 / 4 consecutive items per
            // atomic, c2 0.2106 -> 0.2160 / 0.2390 at 4 hardware queues; claiming once the tile has
            // 8 / 16 / 32 slots left, c2 0.1783 -> 0.1786 / 0.1792 / 0.1793)
            const int item = cur.next(p.queue, p.perQueue, p.numItems, home, tileFr, p.nFrames);
            if (item < 0) {
              drained = true;
              break;  // no tiles left for this wave
            }
            tile = item;
#if PT_WAVE_TRACE
            wTiles++;
            wLastClaim = wall_clock64();
#endif
            if (p.primHit) {
              // the camera-ray pass's compacted results: the tile's mask (scalar), then its first nValid
              // entries (one coalesced read of 8 bytes per path; sky slots cost nothing)
              const unsigned long long m = primTileMask(p, tileFr, tile);
              const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)m);
              const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(m >> 32));
              if ((lane < 32 ? lo >> lane : hi >> (lane - 32)) & 1u)
                s_slot[__builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u))] = (unsigned char)lane;
              nValid = __popc(lo) + __popc(hi);
              if (lane < nValid) s_hit[lane] = primTileEntries(p, tileFr, tile)[lane];
            } else {  // without the pass every pixel's camera ray is traced here (PRIM_RETRACE)
              const int px = tilePx(p, tile, sub) + (lane & 7), py = tilePy(p, tile, sub) + (lane >> 3);
              const bool in = px < p.width && py < p.height;
              const unsigned long long valid = __ballot(in);
              if (in) {
                const int k = rankBelow(valid);
                s_slot[k] = (unsigned char)lane;
                s_hit[k] = make_int2(PRIM_RETRACE, 0);
              }
              nValid = __popcll(valid);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            cursor = 0;
#if PT_PHASE_STATS
            PH_ADD(18, clock64() - phC);
#endif
            continue;  // an all-sky tile (nValid 0) is skipped without starting a path
          }
          const int r = cursor + rankBelow(idle);
          if (!active && r < nValid) {
            const int slot = s_slot[r];
            const int2 h = s_hit[r];
            s.px = tilePx(p, tile, sub) + (slot & 7);
            s.py = tilePy(p, tile, sub) + (slot >> 3);
            s.fr = tileFr;
            active = true;
            pend = true;
            hP = h;
          }
          cursor = min(nValid, cursor + __popcll(idle));
        }
        // the camera hits just taken, shaded together (a PRIM_RETRACE / PRIM_TILE camera ray is
        // traced below like any ray)
#if PT_PHASE_STATS
        PH_ADD(16, clock64() - phH);
        const long long phS = clock64();
        if (__ballot(pend)) {
          PH_ADD(21, 1);
          PH_ADD(20, __popcll(__ballot(pend)));
        }
#endif
        bool ended = false;
        if (pend) {
          startPath(p, s);
          if (hP.x >= 0) {
            V3 color;
            if (!advance<INTEG>(p, s, hP.x, __int_as_float(hP.y), color)) {
              writeAccum(p, s, color);
              active = false;
              ended = true;
            }
          }
        }
#if PT_PHASE_STATS
        PH_ADD(19, clock64() - phS);
#endif
        // a path that ended at its camera hit (max_bounce 0) leaves its lane idle: hand out again
        if (drained || __ballot(ended) == 0) break;
      }
    } else {
      // regenerate: idle lanes take the next pixels of the wave's tile
      while (true) {
        PH_ADD(11, 1);
        const unsigned long long idle = __ballot(!active);
        if (idle == 0) break;
        if (cursor >= 64) {
          const int item = cur.next(p.queue, p.perQueue, p.numItems, home, tileFr, p.nFrames);
          if (item < 0) break;  // no tiles left for this wave
          tile = item;
          cursor = 0;
          if (p.primHit) {  // the tile's mask of the camera-ray pass's compacted results (wave-uniform)
            const unsigned long long m = primTileMask(p, tileFr, tile);
            tmaskLo = __builtin_amdgcn_readfirstlane((uint32_t)m);
            tmaskHi = __builtin_amdgcn_readfirstlane((uint32_t)(m >> 32));
          }
#if PT_WAVE_TRACE
          wTiles++;
          wLastClaim = wall_clock64();
#endif
        }
        const int slot = cursor + rankBelow(idle);
        if (!active && slot < 64) {
          const int px = tilePx(p, tile, sub) + (slot & 7);
          const int py = tilePy(p, tile, sub) + (slot >> 3);
          int2 h = make_int2(0, 0);
          if (p.primHit)
            h = primOfSlot((unsigned long long)tmaskHi << 32 | tmaskLo, primTileEntries(p, tileFr, tile), slot);
          if (px < p.width && py < p.height && !(p.primHit && h.x == PRIM_MISS)) {
            s.px = px;
            s.py = py;
            s.fr = tileFr;
            startPath(p, s);
            active = true;
            // the camera ray's result from the camera-ray pass (primaryKernel; a sky pixel, finished
            // by the pass, is never started: the lane takes another slot)
            if (p.primHit && h.x >= 0) {
              V3 color;
              if (!advance<INTEG>(p, s, h.x, __int_as_float(h.y), color)) {
                writeAccum(p, s, color);
                active = false;
              }
            }  // PRIM_RETRACE / PRIM_TILE: traced below like any camera ray
          }
        }
        cursor = min(64, cursor + __popcll(idle));
      }
    }
#if PT_PHASE_STATS
    PH_ADD(0, clock64() - phA);
#endif
    const unsigned long long act = __ballot(active);
    if (act == 0) break;
#if PT_WAVE_TRACE
    wIters++;
    if (__popcll(act) <= 4) {
      wThin++;
      const int l = __ffsll((long long)act) - 1;
      wLonePix = (unsigned long long)__shfl(s.px, l, 64) << 16 | (unsigned long long)__shfl(s.py, l, 64);
    }
#endif
    if (!active) continue;
    float t;
    int tri;
#if PT_PHASE_STATS
    long long phT = 0;
#endif
    if (PT_REGEN_YIELD > 0 && W4 && p.scene.fast) {
      if (!walking) {
        walk4Begin(p.scene, w, st, C);
        walking = true;
      }
#if PT_PHASE_STATS
      PH_ADD(4, 1);
      PH_ADD(5, __popcll(act));
      phT = clock64();
#endif
      walk4Run<CULL, StackT<REGEN_LDS_STACK, BS>, (LDS_NODES > 0), FULL,
               INTEG == 2 ? PT_LEAF_WAIT_MIS : PT_LEAF_WAIT_U>(p.scene, s.o, s.d, s.kind == K_SHADOW, w, st, top,
                                                              PT_REGEN_YIELD, ph);
#if PT_PHASE_STATS
      PH_ADD(1, clock64() - phT);
      if (__ballot(!walk4Done(w)) == 0) PH_ADD(13, 1);
      PH_ADD(12, __popcll(__ballot(!walk4Done(w))));
#endif
      if (!walk4Done(w)) continue;  // stopped for the lanes that are done: resumes next iteration
      walking = false;
#if PT_PHASE_STATS
      phT = clock64();
#endif
      t = w.tbest;
      tri = w.best;
      // (the MIS kernel of the large scenes, whose reference trees are deep: the walk up stops early)
      const bool retrace =
          w.tie || (tri >= 0 && !refReachable<INTEG == 2 && WAVES == PT_WIDE_REGEN_WAVES>(p.scene, tri, s.o, s.d, t));
      PH_ADD(14, __popcll(__ballot(retrace)));
      if (retrace) {
        C.rays--;  // the same ray, counted once
        tri = traceRay<false, CULL, false>(p.scene, s.o, s.d, t, st, C, s.kind == K_SHADOW);
      }
#if PT_PHASE_STATS
      PH_ADD(2, clock64() - phT);
      PH_ADD(6, __popcll(__ballot(1)));
      phT = clock64();
#endif
    } else if (W4 && p.scene.fast) {
      bool tie = false;
      tri = traceRay4<CULL, StackT<REGEN_LDS_STACK, BS>, (LDS_NODES > 0)>(p.scene, s.o, s.d, t, st, C,
                                                                         s.kind == K_SHADOW, top, &tie);
      if (tie || (tri >= 0 && !refReachable(p.scene, tri, s.o, s.d, t))) {
        C.rays--;  // the same ray, counted once
        tri = traceRay<false, CULL, false>(p.scene, s.o, s.d, t, st, C, s.kind == K_SHADOW);
      }
    } else {
      tri = traceRay<false, CULL, false, StackT<REGEN_LDS_STACK, BS>, (LDS_NODES > 0)>(
          p.scene, s.o, s.d, t, st, C, s.kind == K_SHADOW, top);
    }
    V3 color;
    if (!advance<INTEG>(p, s, tri, t, color)) {
      writeAccum(p, s, color);
      active = false;
    }
#if PT_PHASE_STATS
    PH_ADD(3, clock64() - phT);
#endif
  }
#undef PH_ADD
#if PT_PHASE_STATS
  if (lane == 0) ph[15] = clock64() - phStart;
  if (p.waveTrace && lane < PHASE_WORDS)
    p.waveTrace[PHASE_WORDS * ((size_t)blockIdx.x * (BS / 64) + (threadIdx.x >> 6)) + lane] = ph[lane];
#elif PT_WAVE_TRACE
  if (p.waveTrace && lane == 0) {
    unsigned long long* r = p.waveTrace + 6 * ((size_t)blockIdx.x * (BS / 64) + (threadIdx.x >> 6));
    r[0] = wStart; r[1] = wall_clock64(); r[2] = wTiles | wLonePix << 32; r[3] = wLastClaim;
    r[4] = wIters; r[5] = wThin;
  }
#endif
  addRays(p.rayShards, C.rays);
}

// The FULL variant: the uniform integrators' wide kernel (PT_WIDE_REGEN_WAVES_U = 4 waves per
// SIMD) as one block of all the CU's waves, the whole tree beside their 16-entry LDS stacks
// (PT_LDS_TREE = 0: never)
#ifndef PT_LDS_TREE
#define PT_LDS_TREE 1
#endif
constexpr int FULL_BS = 256 * PT_WIDE_REGEN_WAVES_U;  // one block per CU: all its waves share the tree
constexpr size_t LDS_BYTES = 160 * 1024;
template <int I>
static const void* regenFn(bool cull, bool wide, bool full, bool small) {
  if constexpr (I != 2 && PT_REGEN_YIELD > 0)  // the uniform integrators' variant only
    if (full) return (const void*)regenKernel<I, true, wideRegenWaves(I), true, FULL_BS, true>;
  if constexpr (I == 2 && PT_WIDE_REGEN_WAVES_SMALL != PT_WIDE_REGEN_WAVES)
    if (wide && small) return (const void*)regenKernel<I, true, PT_WIDE_REGEN_WAVES_SMALL, true>;
  if (wide) return (const void*)regenKernel<I, true, wideRegenWaves(I), true>;
  return cull ? (const void*)regenKernel<I, true> : (const void*)regenKernel<I, false>;
}
static const void* regenFnI(int integrator, bool cull, bool wide, bool full, bool small = false) {
  return integrator == 0   ? regenFn<0>(cull, wide, full, small)
         : integrator == 1 ? regenFn<1>(cull, wide, full, small)
                           : regenFn<2>(cull, wide, full, small);
}

static long long fullStaticLds(int integrator) {
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, regenFnI(integrator, true, true, true)) != hipSuccess) return -1;
  return (long long)fa.sharedSizeBytes;
}

hipError_t regenShape(int integrator, bool cull, bool wide, int f4nDev, bool smallScene, RegenShape* out) {
  RegenShape r;
  r.wide = wide && cull;
  r.small = integrator == 2 && r.wide && smallScene && PT_WIDE_REGEN_WAVES_SMALL != PT_WIDE_REGEN_WAVES;
  const size_t treeBytes = (size_t)f4nDev * W4_LDS_F4 * sizeof(float4);
  // the FULL variant's static LDS (stack rows, hand-out rows, phase counters) as compiled
  // (a property of the code object, the same on every device: read once per integrator)
  size_t staticBytes = 0;
  if (PT_LDS_TREE && PT_REGEN_YIELD > 0 && r.wide && integrator != 2 && f4nDev > 0) {
    static const long long cached[2] = {fullStaticLds(0), fullStaticLds(1)};
    if (cached[integrator] < 0) return hipErrorInvalidDeviceFunction;
    staticBytes = (size_t)cached[integrator];
  }
  // the whole tree in LDS needs the resumable walk (walk4Run's ALL records): with PT_REGEN_YIELD = 0
  // the walks run traceRay4, which reads an LDS top at the built 8-float4 stride
  r.fullTree = PT_LDS_TREE && PT_REGEN_YIELD > 0 && r.wide && integrator != 2 && f4nDev > 0 &&
               treeBytes + staticBytes <= LDS_BYTES;
  r.block = r.fullTree ? FULL_BS : BLOCK;
  r.dynLds = r.fullTree ? treeBytes : 0;
  const void* f = regenFnI(integrator, cull, r.wide, r.fullTree, r.small);
  if (r.fullTree) {
    // room for any tree that fits beside the static LDS; a function attribute is per device, and
    // setting it is cheap, so every shape query on the current device sets it
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(LDS_BYTES - staticBytes));
    if (e != hipSuccess) return e;
  }
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&r.blocksPerCU, f, r.block, r.dynLds);
  *out = r;
  return e;
}

template <int I>
static hipError_t launchRegenI(const RenderParams& p, int grid, hipStream_t s, bool cull, const RegenShape& r) {
  if constexpr (I != 2 && PT_REGEN_YIELD > 0) {
    if (r.fullTree) {
      hipLaunchKernelGGL((regenKernel<I, true, wideRegenWaves(I), true, FULL_BS, true>), dim3(grid), dim3(FULL_BS),
                         r.dynLds, s, p);
      return hipGetLastError();
    }
  }
  if (r.fullTree) return hipErrorInvalidValue;
  if constexpr (I == 2 && PT_WIDE_REGEN_WAVES_SMALL != PT_WIDE_REGEN_WAVES)
    if (r.wide && r.small) {
      hipLaunchKernelGGL((regenKernel<I, true, PT_WIDE_REGEN_WAVES_SMALL, true>), dim3(grid), dim3(BLOCK), 0, s, p);
      return hipGetLastError();
    }
  if (r.wide)
    hipLaunchKernelGGL((regenKernel<I, true, wideRegenWaves(I), true>), dim3(grid), dim3(BLOCK), 0, s, p);
  else if (cull) hipLaunchKernelGGL((regenKernel<I, true>), dim3(grid), dim3(BLOCK), 0, s, p);
  else hipLaunchKernelGGL((regenKernel<I, false>), dim3(grid), dim3(BLOCK), 0, s, p);
  return hipGetLastError();
}

hipError_t launchRegen(const RenderParams& p, int integrator, int grid, hipStream_t s, bool cull, const RegenShape& r) {
  if (r.fullTree && p.scene.f4nTop * W4_LDS_F4 * sizeof(float4) > r.dynLds) return hipErrorInvalidValue;
  switch (integrator) {
    case 0: return launchRegenI<0>(p, grid, s, cull, r);
    case 1: return launchRegenI<1>(p, grid, s, cull, r);
    default: return launchRegenI<2>(p, grid, s, cull, r);
  }
}

int regenLdsStack() { return REGEN_LDS_STACK; }
int regenTop4(const RegenShape& r, int integrator) {
  return regenTop4W(r.small ? PT_WIDE_REGEN_WAVES_SMALL : wideRegenWaves(integrator));
}

}  // namespace pt
