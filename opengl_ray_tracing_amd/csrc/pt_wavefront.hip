// pt_wavefront.hip -- wavefront formulation of the three pass1.fsh integrators.
//
// One frame = gen -> [trace_closest (+ trace_shadow) -> shade] x (maxBounce + 1).
// Path state lives in HBM in per-pixel structure-of-arrays (pixel id = py*W+px);
// the work lists between stages are compacted queues of pixel ids, appended with
// one atomic per wave (__ballot + popcount + mbcnt prefix) into one of WF_NSEG
// segment counters. The trace kernels are small (no shading code) and run a
// flattened traversal loop in which a lane that finishes its ray immediately
// starts its next one; the shade kernels see only live paths. Every
// floating-point operation is the one the megakernel (pt_kernels.hip) and the
// CPU checker perform, in the same order, so the image is bit-identical to both.
//
// Reference: ImportanceSampling_LowDiscrepancySequence/shaders/pass1.fsh (IS),
// DisneyBRDF/shaders/pass1.fsh (D), OpenglRayTracing/shaders/pass1.fsh (O).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_device.h"
#include "pt_kernels.h"
#include "pt_trace.h"
#include "pt_wavefront.h"

namespace pt {

// -------------------------------------------------------------- helpers
__device__ __forceinline__ int laneId() { return threadIdx.x & 63; }

// Append pred lanes' values to queue segment q (counter cnt): one atomic per wave.
__device__ __forceinline__ void waveAppend(int* q, int* cnt, bool pred, int value) {
  unsigned long long m = __ballot(pred);
  if (m == 0) return;
  const int lane = laneId();
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(cnt, __popcll(m));
  base = __shfl(base, leader, 64);
  if (pred) {
    unsigned long long below = m & ((1ull << lane) - 1ull);
    q[base + __popcll(below)] = value;
  }
}

__device__ __forceinline__ V3 xyz(float4 a) { return v3(a.x, a.y, a.z); }
__device__ __forceinline__ float4 f4(V3 a, float w) { return make_float4(a.x, a.y, a.z, w); }

// pixel of owned slot k (8x8 wave tiles inside shard tiles, as the megakernel)
__device__ __forceinline__ bool ownedPixel(const WFParams& p, int k, int& px, int& py) {
  const int w = k >> 6, lane = k & 63;
  const int sub = p.shardSize >> 3;
  const int tilesPerShard = sub * sub;
  const int j = w / tilesPerShard, s = w - j * tilesPerShard;
  const int g = j * p.world + p.rank;
  const int gy = g / p.shardsX, gx = g - gy * p.shardsX;
  px = gx * p.shardSize + (s % sub) * 8 + (lane & 7);
  py = gy * p.shardSize + (s / sub) * 8 + (lane >> 3);
  return px < p.width && py < p.height;
}

__device__ __forceinline__ void finishPixel(const WFParams& p, int pid, V3 color) {
  float4* a = p.accum + pid;
  float4 old = ldStream(a);
  float w = 1.0f / (float)(p.frameCounter + 1u);
  stStream(a, make_float4(mixf(old.x, color.x, w), mixf(old.y, color.y, w), mixf(old.z, color.z, w), 1.0f));
}

// -------------------------------------------------------------- gen: main() IS:846-850
// Owned slot k -> wave tile k/64 dealt round-robin over the segments; no atomics.
// Slots outside the frame hold -1.
__global__ __launch_bounds__(BLOCK) void wfGenKernel(WFParams p) {
  const int k = blockIdx.x * BLOCK + threadIdx.x;
  const int tiles = p.numOwned >> 6;
  if (blockIdx.x == 0 && threadIdx.x < WF_NSEG) {
    const int s = threadIdx.x;
    const int n = (tiles > s ? (tiles - s + WF_NSEG - 1) / WF_NSEG : 0) * 64;
    p.q.cnt[wfCnt(0, WF_CNT_CLS, s)] = n;
    p.q.cnt[wfCnt(0, WF_CNT_ACT, s)] = n;
  }
  if (k >= p.numOwned) return;
  int px = 0, py = 0;
  const bool ok = ownedPixel(p, k, px, py);
  const int pid = ok ? py * p.width + px : -1;
  const int tile = k >> 6;
  const int slot = (tile & (WF_NSEG - 1)) * p.q.segCap + ((tile / WF_NSEG) << 6) + (k & 63);
  p.q.cls[0][slot] = pid;
  p.q.act[0][slot] = pid;
  if (!ok) return;
  const int W = p.width, H = p.height;
  uint32_t seed = ((uint32_t)px * 1973u + (uint32_t)py * 9277u + p.sampleIndex * 26699u) | 1u;
  float pixx = (float)(2 * px + 1) / (float)W - 1.0f;
  float pixy = (float)(2 * py + 1) / (float)H - 1.0f;
  float ax = (randf(seed) - 0.5f) / (float)W;
  float ay = (randf(seed) - 0.5f) / (float)H;
  float x = pixx + ax, y = pixy + ay, z = -1.5f;
  const float* M = p.cam;
  V3 c0 = v3(M[0], M[1], M[2]), c1 = v3(M[4], M[5], M[6]), c2 = v3(M[8], M[9], M[10]), c3 = v3(M[12], M[13], M[14]);
  V3 dir = normalize((c0 * x + c1 * y) + (c2 * z + c3 * 0.0f));
  const WFState& S = p.st;
  S.rayO[pid] = make_float4(p.eye[0], p.eye[1], p.eye[2], 0.0f);
  S.rayD[pid] = f4(dir, 0.0f);
  S.seed[pid] = seed;
  S.flags[pid] = WF_PRIMARY | WF_CLS;
  S.hist[pid] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
  S.Lo[pid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

// -------------------------------------------------------------- trace
// hitBVH (IS:335-382) as a flattened per-lane state machine: each iteration a
// lane either tests one triangle of its current leaf or one internal node; a
// lane whose ray is finished writes the result and loads its next ray from its
// segment (grid-stride), so no lane waits for the slowest ray of its wave.
// Visiting order, culling and the strict '<' update are those of traceRay.
template <bool ANYHIT, bool CULL>
__global__ __launch_bounds__(BLOCK) void wfTraceKernel(WFTraceParams p) {
  __shared__ int s_stack[WF_LDS_STACK * BLOCK];
  StackT<WF_LDS_STACK, BLOCK> st;
  st.lds = s_stack + threadIdx.x;
  const size_t gtid = (size_t)blockIdx.x * BLOCK + threadIdx.x;
  st.gbl = p.ovf ? p.ovf + gtid * p.ovfDepth : nullptr;
  st.reset();
  const int seg = blockIdx.x & (WF_NSEG - 1);
  const int n = p.count[seg * CTL_LINE_INTS];
  const int* q = p.queue + (size_t)seg * p.segCap;
  const int stride = (gridDim.x / WF_NSEG) * BLOCK;
  int next = (blockIdx.x / WF_NSEG) * BLOCK + threadIdx.x;
  const SceneView& S = p.scene;

  int pid = -1;
  V3 o = v3(0, 0, 0), d = v3(0, 0, 0), inv = v3(0, 0, 0);
  float tbest = PT_INF;
  int best = -1, ref = REF_NONE, leafI = 0, leafEnd = 0;
  uint32_t nrays = 0;
  while (true) {
    while (pid < 0 && next < n) {
      const int c = q[next];
      next += stride;
      if (c < 0) continue;
      float4 a = p.rayO[c], b = p.rayD[c];
      o = xyz(a);
      d = xyz(b);
      inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
      tbest = PT_INF;
      best = -1;
      st.reset();
      ref = S.rootRef;
      leafI = leafEnd = 0;
      if (ref < 0 && ref != REF_NONE) {
        uint32_t v = ~(uint32_t)ref;
        leafI = (int)(v >> LEAF_CNT_BITS);
        leafEnd = leafI + (int)(v & ((1u << LEAF_CNT_BITS) - 1u)) + 1;
        ref = REF_NONE;
      }
      nrays++;
      if (leafI >= leafEnd && ref == REF_NONE) {  // empty tree: a miss
        if (ANYHIT) p.occ[c] = 0;
        else p.hit[c] = make_int2(-1, __float_as_int(PT_INF));
        continue;
      }
      pid = c;
    }
    if (__ballot(pid >= 0) == 0) break;
    if (pid < 0) continue;
    bool finished = false;
    if (leafI < leafEnd) {
      float t;
      if (triHit(S.geo + 4 * (size_t)leafI, o, d, tbest, t)) {
        tbest = t;
        best = leafI;
        if (ANYHIT) finished = true;
      }
      leafI++;
    } else {
      NodeHit nh;
      visitNode(S.bvh + 4 * (size_t)ref, o, inv, nh);
      const int lref = nh.lref, rref = nh.rref;
      const float d1 = nh.d1, d2 = nh.d2, t0l = nh.t0l, t0r = nh.t0r;
      bool h1 = (lref != REF_NONE) && d1 > 0.0f;
      bool h2 = (rref != REF_NONE) && d2 > 0.0f;
      if (CULL) {
        float lim = tbest + 1e-3f * fmaxf(1.0f, tbest);
        h1 = h1 && !(t0l > lim);
        h2 = h2 && !(t0r > lim);
      }
      if (h1 && h2) {
        bool leftFirst = d1 < d2;
        st.push(leftFirst ? rref : lref);
        ref = leftFirst ? lref : rref;
      } else if (h1) {
        ref = lref;
      } else if (h2) {
        ref = rref;
      } else {
        ref = REF_NONE;
      }
    }
    if (!finished && leafI >= leafEnd) {
      if (ref == REF_NONE) {
        if (st.sp > 0) ref = st.pop();
        else finished = true;
      }
      if (!finished && ref < 0) {  // a leaf: its triangles come next
        uint32_t v = ~(uint32_t)ref;
        leafI = (int)(v >> LEAF_CNT_BITS);
        leafEnd = leafI + (int)(v & ((1u << LEAF_CNT_BITS) - 1u)) + 1;
        ref = REF_NONE;
      }
    }
    if (finished) {
      if (ANYHIT) p.occ[pid] = best >= 0 ? 1 : 0;
      else p.hit[pid] = make_int2(best, __float_as_int(tbest));
      pid = -1;
    }
  }
  // per-wave ray count into the block's counter shard
  addRays(p.rays, nrays);
}

// The same as a walk of the 4-wide runtime tree (pt_trace.h walk4Run), results made the
// reference's by refReachable / a retrace through the uploaded tree as in every other frame
// kernel. One launch traces a bounce's closest-hit rays and then its env shadow rays. A lane
// whose walk is done writes its result and loads its next ray as soon as the wave has
// PT_WF_YIELD such lanes, so the walks run with nearly full waves (the regen kernel's lanes
// wait for their paths' shading instead: 16 of 64 lanes per node iteration on c5). No path
// state is live here; the kernel is compiled for PT_WF_WAVES waves per SIMD; blocks of
// WF4_BS threads share one LDS copy of the tree's top WF4_TOP nodes.
#ifndef PT_WF_YIELD
#define PT_WF_YIELD 16
#endif
#ifndef PT_WF_WAVES
#define PT_WF_WAVES 4  // the walk needs ~112 VGPRs: 5 waves spill 25, 6 waves 61, 8 waves 103
#endif
constexpr int WF4_BS = PT_WF_WAVES >= 8 ? 1024 : PT_WF_WAVES == 5 ? 256 : 512;
constexpr int WF4_TOP = 128;
template <bool CULL>
__global__ __launch_bounds__(WF4_BS, PT_WF_WAVES) void wfTrace4Kernel(WFTraceParams p) {
  __shared__ int s_stack[WF_LDS_STACK * WF4_BS];
  __shared__ float4 s_top[WF4_TOP * W4_F4];
  StackT<WF_LDS_STACK, WF4_BS> st;
  st.lds = s_stack + threadIdx.x;
  const size_t gtid = (size_t)blockIdx.x * WF4_BS + threadIdx.x;
  st.gbl = p.ovf ? p.ovf + gtid * p.ovfDepth : nullptr;
  st.reset();
  const SceneView& S = p.scene;
  for (int i = threadIdx.x; i < S.f4nTop * W4_F4; i += WF4_BS) s_top[i] = S.fbvh4[i];
  __syncthreads();
  const int seg = blockIdx.x & (WF_NSEG - 1);
  const int nC = p.count[seg * CTL_LINE_INTS];
  const int nS = p.queueS ? p.countS[seg * CTL_LINE_INTS] : 0;
  const int* qC = p.queue + (size_t)seg * p.segCap;
  const int* qS = p.queueS ? p.queueS + (size_t)seg * p.segCap : nullptr;
  const int stride = (gridDim.x / WF_NSEG) * WF4_BS;
  int next = (blockIdx.x / WF_NSEG) * WF4_BS + threadIdx.x;
  Counters C = {0, 0, 0, 0, 0};
  int pid = -1;
  bool shadow = false;
  V3 o = v3(0, 0, 0), d = v3(0, 0, 0);
  Walk4 w;
  w.ref = w.leaf = REF_NONE;
  while (true) {
    while (pid < 0 && next < nC + nS) {
      const bool sh = next >= nC;
      const int c = sh ? qS[next - nC] : qC[next];
      next += stride;
      if (c < 0) continue;
      o = xyz(p.rayO[c]);
      d = xyz(sh ? p.rayDS[c] : p.rayD[c]);
      shadow = sh;
      pid = c;
      walk4Begin(S, w, st, C);
    }
    if (__ballot(pid >= 0) == 0) break;
    if (pid < 0) continue;
    walk4Run<CULL, StackT<WF_LDS_STACK, WF4_BS>, true>(S, o, d, shadow, w, st, s_top, PT_WF_YIELD);
    if (!walk4Done(w)) continue;
    float t = w.tbest;
    int tri = w.best;
    if ((w.tie && !shadow) || (tri >= 0 && !refReachable(S, tri, o, d, t))) {
      C.rays--;  // the same ray, counted once
      tri = traceRay<false, CULL, false>(S, o, d, t, st, C, shadow);
    }
    if (shadow) p.occ[pid] = tri >= 0 ? 1 : 0;
    else p.hit[pid] = make_int2(tri, __float_as_int(t));
    pid = -1;
  }
  addRays(p.rays, C.rays);
}

// -------------------------------------------------------------- shade
// Sample the next bounce from `hit` for the uniform-hemisphere integrators
// (O:335-345, D:448-456): stores the pending f_r and cosine, the new ray.
template <int INTEG>
__device__ __forceinline__ void prepareUniform(const WFState& S, int pid, const Hit& hit, uint32_t& seed) {
  V3 N = hit.N;
  V3 L = toNormalHemisphere(sampleHemisphereRand(seed), N);
  float cosine_i = fmaxf(0.0f, dot(L, N));
  V3 f_r;
  if (INTEG == 0) {
    f_r = hit.m.baseColor / PT_PI;
  } else {
    V3 tangent, bitangent;
    getTangent(N, tangent, bitangent);
    f_r = brdfAniso(-hit.viewDir, N, L, tangent, bitangent, hit.m);
  }
  S.pend[pid] = f4(f_r, cosine_i);
  S.rayO[pid] = f4(hit.P, 0.0f);
  S.rayD[pid] = f4(L, 0.0f);
}

// One bounce of pathTracingImportanceSampling IS:766-811 up to the two traces.
// Returns the flags of the rays cast (WF_SHD / WF_CLS).
__device__ __forceinline__ uint32_t prepareMIS(const WFParams& p, int pid, int px, int py, int bounce, const Hit& hit,
                                               V3 history, uint32_t& seed) {
  const WFState& S = p.st;
  V3 V = -hit.viewDir;
  V3 N = hit.N;
  uint32_t cast = 0;
  float r1 = randf(seed);
  float r2 = randf(seed);
  V3 Ldir = sampleHdrDir(p.env, r1, r2);
  float4 shc = make_float4(0, 0, 0, 0);
  if (dot(N, Ldir) > 0.0f) {
    // the unoccluded contribution (IS:781-789), added by the next stage if the ray escapes
    V3 L = Ldir;
    V3 color;
    float pdf_light;
    hdrColorPdf(p.env, L, color, pdf_light);
    V3 f_r = brdfIso(V, N, L, hit.m);
    float pdf_brdf = brdfPdf(V, N, L, hit.m);
    float mis_weight = misWeight(pdf_light, pdf_brdf);
    V3 c = ((history * mis_weight) * color) * f_r;
    shc = f4((c * dot(N, L)) / pdf_light, 0.0f);
    S.shD[pid] = f4(Ldir, 0.0f);
    cast |= WF_SHD;
  }
  const uint32_t gi = grayCode(p.sampleIndex + 1u);
  float u = sobolf(2u * (uint32_t)bounce, gi);
  float v = sobolf(2u * (uint32_t)bounce + 1u, gi);
  cranleyPatterson(px, py, u, v);
  float xi_3 = randf(seed);
  V3 L = sampleBRDF(u, v, xi_3, V, N, hit.m);
  float NdotL = dot(N, L);
  if (NdotL > 0.0f) {
    V3 f_r = brdfIso(V, N, L, hit.m);
    float pdf_brdf = brdfPdf(V, N, L, hit.m);
    // IS:816: pdf <= 0 ends the path; the reference traces the ray first and discards it
    if (pdf_brdf > 0.0f) {
      S.pend[pid] = f4(f_r, NdotL);
      shc.w = pdf_brdf;
      S.rayD[pid] = f4(L, 0.0f);
      cast |= WF_CLS;
    }
  }
  S.rayO[pid] = f4(hit.P, 0.0f);
  S.shC[pid] = shc;
  return cast;
}

template <int INTEG>
__global__ __launch_bounds__(BLOCK) void wfShadeKernel(WFParams p, int stage) {
  const int in = stage & 1, out = in ^ 1;
  const int seg = blockIdx.x & (WF_NSEG - 1);
  const int n = p.q.cnt[wfCnt(stage, WF_CNT_ACT, seg)];
  const int* qin = p.q.act[in] + (size_t)seg * p.q.segCap;

  const WFState& S = p.st;
  const int stride = (gridDim.x / WF_NSEG) * BLOCK;
  const int waveBase = (blockIdx.x / WF_NSEG) * BLOCK + (threadIdx.x & ~63);
  for (int base = waveBase; base < n; base += stride) {
    const int idx = base + laneId();
    bool toCls = false, toShd = false, toAct = false;
    const int pid = idx < n ? qin[idx] : -1;
    if (pid >= 0) {
      const int px = pid % p.width, py = pid / p.width;
      uint32_t flags = S.flags[pid];
      uint32_t seed = S.seed[pid];
      const int bounce = (int)(flags & WF_BOUNCE_MASK);
      const bool primary = (flags & WF_PRIMARY) != 0;
      bool done = false;
      V3 color = v3(0, 0, 0);
      V3 Lo = v3(0, 0, 0);
      V3 history = v3(1, 1, 1);
      V3 Le0 = v3(0, 0, 0);
      Hit hit;
      bool haveHit = false;
      int nextBounce = 0;
      if (primary) {
        int2 h = S.hit[pid];
        V3 o = xyz(S.rayO[pid]), d = xyz(S.rayD[pid]);
        if (h.x < 0) {
          color = sampleHdr(p.env, d);  // IS:857-859
          done = true;
        } else {
          finishHit(p.scene, h.x, o, d, __int_as_float(h.y), hit);
          Le0 = hit.m.emissive;
          haveHit = true;
          nextBounce = 0;
        }
      } else {
        Lo = xyz(S.Lo[pid]);
        history = xyz(S.hist[pid]);
        Le0 = xyz(S.Le0[pid]);
        float4 pend = S.pend[pid];
        V3 f_r = xyz(pend);
        if (INTEG == 2) {
          float4 shc = S.shC[pid];
          if ((flags & WF_SHD) && S.occ[pid] == 0) Lo = Lo + xyz(shc);  // IS:789
          if (!(flags & WF_CLS)) {
            done = true;  // IS:805 / IS:816 break
          } else {
            float NdotL = pend.w, pdf_brdf = shc.w;
            int2 h = S.hit[pid];
            V3 o = xyz(S.rayO[pid]), L = xyz(S.rayD[pid]);
            if (h.x < 0) {  // IS:819-829
              V3 c;
              float pdf_light;
              hdrColorPdf(p.env, L, c, pdf_light);
              float mis_weight = misWeight(pdf_brdf, pdf_light);
              V3 cc = ((history * mis_weight) * c) * f_r;
              Lo = Lo + (cc * NdotL) / pdf_brdf;
              done = true;
            } else {  // IS:833-837
              finishHit(p.scene, h.x, o, L, __int_as_float(h.y), hit);
              V3 Le = hit.m.emissive;
              Lo = Lo + ((history * Le) * f_r * NdotL) / pdf_brdf;
              history = history * ((f_r * NdotL) / pdf_brdf);
              haveHit = true;
              nextBounce = bounce + 1;
            }
          }
        } else {  // O:347-360 / D:463-479
          const float pdf = 1.0f / (2.0f * PT_PI);
          float cosine_i = pend.w;
          int2 h = S.hit[pid];
          V3 o = xyz(S.rayO[pid]), L = xyz(S.rayD[pid]);
          if (h.x < 0) {
            V3 sky = sampleHdr(p.env, L);
            Lo = Lo + ((history * sky) * f_r * cosine_i) / pdf;
            done = true;
          } else {
            finishHit(p.scene, h.x, o, L, __int_as_float(h.y), hit);
            V3 Le = hit.m.emissive;
            Lo = Lo + ((history * Le) * f_r * cosine_i) / pdf;
            history = history * ((f_r * cosine_i) / pdf);
            haveHit = true;
            nextBounce = bounce + 1;
          }
        }
      }
      if (haveHit) {
        if (nextBounce >= p.maxBounce) {
          done = true;
        } else if (INTEG == 2) {
          uint32_t cast = prepareMIS(p, pid, px, py, nextBounce, hit, history, seed);
          toCls = (cast & WF_CLS) != 0;
          toShd = (cast & WF_SHD) != 0;
          if (cast == 0) done = true;  // neither ray: the loop breaks here (IS:805)
          else flags = (uint32_t)nextBounce | cast;
        } else {
          prepareUniform<INTEG>(S, pid, hit, seed);
          toCls = true;
          flags = (uint32_t)nextBounce | WF_CLS;
        }
      }
      if (done) {
        if (!primary || haveHit) color = Le0 + Lo;  // IS:865 color = Le + Li
        finishPixel(p, pid, color);
      } else {
        toAct = true;
        if (primary) S.Le0[pid] = f4(Le0, 0.0f);
        S.flags[pid] = flags;
        S.seed[pid] = seed;
        S.hist[pid] = f4(history, 0.0f);
        S.Lo[pid] = f4(Lo, 0.0f);
      }
    }
    waveAppend(p.q.cls[out] + (size_t)seg * p.q.segCap, p.q.cnt + wfCnt(stage + 1, WF_CNT_CLS, seg), toCls, pid);
    waveAppend(p.q.shd[out] + (size_t)seg * p.q.segCap, p.q.cnt + wfCnt(stage + 1, WF_CNT_SHD, seg), toShd, pid);
    waveAppend(p.q.act[out] + (size_t)seg * p.q.segCap, p.q.cnt + wfCnt(stage + 1, WF_CNT_ACT, seg), toAct, pid);
  }
}

// -------------------------------------------------------------- launchers
hipError_t wfLaunchGen(const WFParams& p, hipStream_t s) {
  hipLaunchKernelGGL(wfGenKernel, dim3((p.numOwned + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p);
  return hipGetLastError();
}
hipError_t wfLaunchTrace(const WFTraceParams& p, bool anyhit, bool cull, int grid, hipStream_t s) {
  if (anyhit) {
    if (cull) hipLaunchKernelGGL((wfTraceKernel<true, true>), dim3(grid), dim3(BLOCK), 0, s, p);
    else hipLaunchKernelGGL((wfTraceKernel<true, false>), dim3(grid), dim3(BLOCK), 0, s, p);
  } else {
    if (cull) hipLaunchKernelGGL((wfTraceKernel<false, true>), dim3(grid), dim3(BLOCK), 0, s, p);
    else hipLaunchKernelGGL((wfTraceKernel<false, false>), dim3(grid), dim3(BLOCK), 0, s, p);
  }
  return hipGetLastError();
}
hipError_t wfTraceBlocksPerCU(bool anyhit, bool cull, int* nb) {
  const void* f = anyhit ? (cull ? (const void*)wfTraceKernel<true, true> : (const void*)wfTraceKernel<true, false>)
                         : (cull ? (const void*)wfTraceKernel<false, true> : (const void*)wfTraceKernel<false, false>);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(nb, f, BLOCK, 0);
}
hipError_t wfLaunchTrace4(const WFTraceParams& p, bool cull, int grid, hipStream_t s) {
  if (p.scene.f4nTop > WF4_TOP || !p.scene.fast) return hipErrorInvalidValue;
  if (cull) hipLaunchKernelGGL((wfTrace4Kernel<true>), dim3(grid), dim3(WF4_BS), 0, s, p);
  else hipLaunchKernelGGL((wfTrace4Kernel<false>), dim3(grid), dim3(WF4_BS), 0, s, p);
  return hipGetLastError();
}
hipError_t wfTrace4Shape(bool cull, int* blockSize, int* blocksPerCU) {
  *blockSize = WF4_BS;
  const void* f = cull ? (const void*)wfTrace4Kernel<true> : (const void*)wfTrace4Kernel<false>;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocksPerCU, f, WF4_BS, 0);
}
int wfTrace4Top() { return WF4_TOP; }
hipError_t wfLaunchShade(const WFParams& p, int integrator, int stage, int grid, hipStream_t s) {
  switch (integrator) {
    case 0: hipLaunchKernelGGL(wfShadeKernel<0>, dim3(grid), dim3(BLOCK), 0, s, p, stage); break;
    case 1: hipLaunchKernelGGL(wfShadeKernel<1>, dim3(grid), dim3(BLOCK), 0, s, p, stage); break;
    default: hipLaunchKernelGGL(wfShadeKernel<2>, dim3(grid), dim3(BLOCK), 0, s, p, stage); break;
  }
  return hipGetLastError();
}

}  // namespace pt
