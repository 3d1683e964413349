// pt_trace.h -- BVH traversal and triangle intersection shared by the
// megakernel (pt_kernels.hip), the path-regeneration kernel (pt_regen.hip) and the
// camera-ray pass (pt_primary.hip). Restates hitBVH / hitArray / hitTriangle / hitAABB of
// ImportanceSampling_LowDiscrepancySequence/shaders/pass1.fsh:251-382 over the
// re-laid-out device scene (pt_kernels.h SceneView).
#pragma once
#include "pt_device.h"
#include "pt_kernels.h"

namespace pt {

// ----------------------------------------------------------------- counters
struct Counters {
  uint32_t rays, nodes, tris, mats, texels;
};

// The node phase of a while-while walk (traceRay, traceRay4; walk4Run has PT_LEAF_WAIT) ends once
// at most this many of its lanes still look for a leaf (0: every lane holds one)
#ifndef PT_LEAF_WAIT_MK
#define PT_LEAF_WAIT_MK 0
#endif

// ----------------------------------------------------------------- stack
// LDS stack of up to DEPTH entries per lane, entry e of thread t at
// lds[(e % DEPTH) * STRIDE + t] (lane-interleaved: a wave's push/pop is bank
// conflict free). Entries [0, base) live in the thread's HBM overflow region
// the thread's overflow region gbl() (only trees deeper than DEPTH get there): a push onto a full LDS part
// moves its older half to HBM, and a pop from an empty LDS part brings back up
// to half a stack at once -- one memory round trip per DEPTH/2 pops. (Moving
// one entry per push/pop past the LDS depth stalled every deep pop on an L2
// round trip: the rays that walk deep into a chain-shaped reference-SAH tree
// made single 8x8 tiles last most of a c4 frame.)
template <int DEPTH, int STRIDE>
struct StackT {
  static_assert((DEPTH & (DEPTH - 1)) == 0, "LDS stack depth must be a power of two");
  static constexpr int HALF = DEPTH / 2;
  int* lds;       // &s_stack[threadIdx.x]
  int* ovf;       // the launch's overflow area (RenderParams::ovf, wave-uniform; may be null when
  int ovfDepth;   // maxStack <= DEPTH), ovfDepth entries per thread: this thread's region is
                  // computed where it is used (a per-lane pointer held across every walk cost two
                  // VGPRs: the regen kernel's spills)
  int sp;         // entries on the stack
  int base;       // entries in the overflow region
  __device__ __forceinline__ void init(int* ldsBase, int* ovfArea, int depth) {
    lds = ldsBase + threadIdx.x;
    ovf = ovfArea;
    ovfDepth = depth;
  }
  __device__ __forceinline__ int* gbl() const {
    return ovf + ((size_t)blockIdx.x * STRIDE + threadIdx.x) * (size_t)ovfDepth;
  }
  __device__ __forceinline__ void reset() { sp = 0; base = 0; }
  __device__ __forceinline__ void push(int v) {
    if (sp - base == DEPTH) {
      int* g = gbl();
      for (int i = 0; i < HALF; i++) g[base + i] = lds[((base + i) & (DEPTH - 1)) * STRIDE];
      base += HALF;
    }
    lds[(sp & (DEPTH - 1)) * STRIDE] = v;
    sp++;
  }
  __device__ __forceinline__ int pop() {
    if (sp == base) {
      const int n = base < HALF ? base : HALF;
      base -= n;
      const int* g = gbl();
      for (int i = 0; i < n; i++) lds[((base + i) & (DEPTH - 1)) * STRIDE] = g[base + i];
    }
    sp--;
    return lds[(sp & (DEPTH - 1)) * STRIDE];
  }
};
using Stack = StackT<LDS_STACK, BLOCK>;

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

// Both children's hitAABB of one wide node. Node record (pt_runtime.cpp):
// {L.lo.x, R.lo.x, L.lo.y, R.lo.y}, {L.lo.z, R.lo.z, L.hi.x, R.hi.x},
// {L.hi.y, R.hi.y, L.hi.z, R.hi.z}, {left ref, right ref, -, -}: the slab
// differences and products of the two boxes run as packed pairs
// (v_pk_add_f32 / v_pk_mul_f32, the same IEEE operations as hitAABB); the
// min/max reductions are hitAABB's, component by component.
typedef float f32x2 __attribute__((ext_vector_type(2)));
struct NodeHit {
  float d1, d2;    // the reference's d for the left / right child
  float t0l, t0r;  // slab entries (culling)
  int lref, rref;
};
// the slab tests of both children from their boxes as float pairs
__device__ __forceinline__ void slabPair(f32x2 lox, f32x2 loy, f32x2 loz, f32x2 hix, f32x2 hiy, f32x2 hiz, V3 o, V3 inv,
                                         NodeHit& h) {
  const f32x2 ox = {o.x, o.x}, oy = {o.y, o.y}, oz = {o.z, o.z};
  const f32x2 ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
  const f32x2 fx = (hix - ox) * ix, fy = (hiy - oy) * iy, fz = (hiz - oz) * iz;
  const f32x2 nx = (lox - ox) * ix, ny = (loy - oy) * iy, nz = (loz - oz) * iz;
  float t1 = fminf(fmaxf(fx.x, nx.x), fminf(fmaxf(fy.x, ny.x), fmaxf(fz.x, nz.x)));
  float t0 = fmaxf(fminf(fx.x, nx.x), fmaxf(fminf(fy.x, ny.x), fminf(fz.x, nz.x)));
  h.t0l = t0;
  h.d1 = (t1 >= t0) ? ((t0 > 0.0f) ? t0 : t1) : -1.0f;
  t1 = fminf(fmaxf(fx.y, nx.y), fminf(fmaxf(fy.y, ny.y), fmaxf(fz.y, nz.y)));
  t0 = fmaxf(fminf(fx.y, nx.y), fmaxf(fminf(fy.y, ny.y), fminf(fz.y, nz.y)));
  h.t0r = t0;
  h.d2 = (t1 >= t0) ? ((t0 > 0.0f) ? t0 : t1) : -1.0f;
}
__device__ __forceinline__ void visitNode(const float4* nd, V3 o, V3 inv, NodeHit& h) {
  const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
  const f32x2 lox = {q0.x, q0.y}, loy = {q0.z, q0.w}, loz = {q1.x, q1.y};
  const f32x2 hix = {q1.z, q1.w}, hiy = {q2.x, q2.y}, hiz = {q2.z, q2.w};
  slabPair(lox, loy, loz, hix, hiy, hiz, o, inv, h);
  h.lref = __float_as_int(q3.x);
  h.rref = __float_as_int(q3.y);
}
// The runtime tree's slab tests fused: (plane - o) * inv as fma(plane, inv,
// -o * inv), one packed FMA per axis and child pair instead of a subtract and a
// multiply. The rounding differs from hitAABB's by about |o| * 2^-23 along each
// axis, far inside the widening of the runtime tree's boxes (pt_runtime.cpp
// uploadAccel), so the walk still meets every triangle the ray hits; results
// found through it are checked against the reference tree as before. Never
// used on the reference tree, whose d must be hitAABB's bit for bit.
__device__ __forceinline__ void visitNodeF(const float4* nd, V3 inv, V3 noi, NodeHit& h) {
  const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
  const f32x2 lox = {q0.x, q0.y}, loy = {q0.z, q0.w}, loz = {q1.x, q1.y};
  const f32x2 hix = {q1.z, q1.w}, hiy = {q2.x, q2.y}, hiz = {q2.z, q2.w};
  const f32x2 ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
  const f32x2 ox = {noi.x, noi.x}, oy = {noi.y, noi.y}, oz = {noi.z, noi.z};
  const f32x2 fx = __builtin_elementwise_fma(hix, ix, ox), fy = __builtin_elementwise_fma(hiy, iy, oy),
              fz = __builtin_elementwise_fma(hiz, iz, oz);
  const f32x2 nx = __builtin_elementwise_fma(lox, ix, ox), ny = __builtin_elementwise_fma(loy, iy, oy),
              nz = __builtin_elementwise_fma(loz, iz, oz);
  float t1 = fminf(fmaxf(fx.x, nx.x), fminf(fmaxf(fy.x, ny.x), fmaxf(fz.x, nz.x)));
  float t0 = fmaxf(fminf(fx.x, nx.x), fmaxf(fminf(fy.x, ny.x), fminf(fz.x, nz.x)));
  h.t0l = t0;
  h.d1 = (t1 >= t0) ? ((t0 > 0.0f) ? t0 : t1) : -1.0f;
  t1 = fminf(fmaxf(fx.y, nx.y), fminf(fmaxf(fy.y, ny.y), fmaxf(fz.y, nz.y)));
  t0 = fmaxf(fminf(fx.y, nx.y), fmaxf(fminf(fy.y, ny.y), fminf(fz.y, nz.y)));
  h.t0r = t0;
  h.d2 = (t1 >= t0) ? ((t0 > 0.0f) ? t0 : t1) : -1.0f;
  h.lref = __float_as_int(q3.x);
  h.rref = __float_as_int(q3.y);
}
// The fused walk's per-ray constants: 1/d clamped to +-2^64 (a direction
// component of 0 or near it would make plane * inv - o * inv an inf - inf NaN
// or an overflow), and -o * inv. With the clamp, an axis the ray runs
// (nearly) parallel to still gives a slab interval of the right sign that spans
// at least +-2^64 x the origin's distance from the planes -- every t of
// interest when the origin is inside, none when it is outside -- so the test
// stays conservative there too.
struct FusedRay {
  V3 inv, noi;
};
__device__ __forceinline__ float clampInv(float v) { return copysignf(fminf(fabsf(v), 0x1p64f), v); }
// fma(a, s.x, s.y) on both halves of a, s = {1/d, -o/d} of one axis, as two scalar FMAs: a
// 4-wide walk holds its ray as three such pairs. Packed FMAs need both scalars broadcast into
// register pairs of their own (six pairs, twelve VGPRs, live across the whole walk); the
// scalar form has six VGPRs fewer and twelve more VALU instructions per visit, and measured
// faster everywhere (c2 0.2122 -> 0.2056 ms, c4 0.2926 -> 0.2775, c5 5.59 -> 5.51; spills of
// the MIS kernels 28 -> 13 and 88 -> 76 VGPRs). The same IEEE fma, so the same results.
__device__ __forceinline__ f32x2 fmaBcast(f32x2 a, f32x2 s) {
  // (v_pk_fma_f32 with op_sel broadcasting s's halves, as inline asm, halves these FMAs but makes the
  // compiler canonicalise every result before the IEEE-mode min/max: 24 v_max added, not kept)
  return f32x2{__builtin_fmaf(a.x, s.x, s.y), __builtin_fmaf(a.y, s.x, s.y)};
}
__device__ __forceinline__ FusedRay fusedRay(V3 o, V3 inv) {
  FusedRay f;
  f.inv = v3(clampInv(inv.x), clampInv(inv.y), clampInv(inv.z));
  f.noi = v3(-(o.x * f.inv.x), -(o.y * f.inv.y), -(o.z * f.inv.z));
  return f;
}
// Node kinds, a compile-time property of a traversal: the reference tree's
// exact records and slab tests (NODE_EXACT) or the runtime tree's records with
// fused slab tests (NODE_FUSED).
constexpr int NODE_EXACT = 0, NODE_FUSED = 2;
constexpr int FAST_KIND = PT_FUSED_SLABS ? NODE_FUSED : NODE_EXACT;
template <int KIND>
__device__ __forceinline__ void visitAny(const float4* nd, V3 o, V3 inv, const FusedRay& fr, NodeHit& h) {
  if (KIND == NODE_FUSED) visitNodeF(nd, fr.inv, fr.noi, h);
  else visitNode(nd, o, inv, h);
}

// hitTriangle IS:251-301, accept/reject and distance only. With the stored unit
// normal Ng = normalize(cross(p2-p1,p3-p1)) and w = dot(Ng,p1) (computed on the
// host in the reference's order) this rounds exactly like the reference: the
// orientation flip negates numerator, denominator and all three edge tests
// exactly, so it changes neither t nor the accept decision. A triangle at or
// beyond tmax cannot win (the caller keeps a hit only if t < tbest), so it is
// rejected before the edge tests; pass PT_INF to get the plain hitTriangle.
__device__ __forceinline__ bool triTest(float4 A, float4 B, float4 C, float4 Nn, V3 o, V3 d, float tmax, float& t) {
  // Every test is evaluated without branching: an early return would let the
  // compiler sink the vertex loads behind the normal test, turning one memory
  // round trip into three.
  V3 N = v3(Nn.x, Nn.y, Nn.z);
  float dn = dot(N, d);
  float tt = (A.w - dot(o, N)) / dn;
  V3 p1 = v3(A.x, A.y, A.z), p2 = v3(B.x, B.y, B.z), p3 = v3(C.x, C.y, C.z);
  V3 P = o + d * tt;
  float s1 = dot(cross(p2 - p1, P - p1), N);
  float s2 = dot(cross(p3 - p2, P - p2), N);
  float s3 = dot(cross(p1 - p3, P - p3), N);
  bool r1 = (s1 > 0 && s2 > 0 && s3 > 0);
  bool r2 = (s1 < 0 && s2 < 0 && s3 < 0);
  t = tt;
  return !(fabsf(dn) < 0.00001f) && !(tt < 0.0005f) && (tt < tmax) && (r1 || r2);
}
// triTest of triangles i and i+1 from their pair record (pt_runtime.cpp): the two triangles'
// data arrive in one memory round trip, component-interleaved. Every operation of triTest per
// triangle, in scalar VALU. (Until round 4 the pair ran as packed v_pk_mul/v_pk_add math, half
// the VALU, but with o and d broadcast into six register pairs that the compiler hoists out of
// the walks and holds across them: scalar, the Lambert LDS-tree kernel drops 159 -> 135 VGPRs
// and the MIS kernels' spills 13 -> 2 (megakernel) and 76 -> 14 (regen), c2 0.2029 -> 0.1931 ms,
// c4 0.2888 -> 0.2803, c5 5.48 -> 5.34.)
// g0/g1: accepted apart from the caller's closest-hit bound.
// ids (pairTestIds): the two triangles' uploaded indices stored in the record (buildPairs)
__device__ __forceinline__ void pairHalf(float p1x, float p1y, float p1z, float p2x, float p2y, float p2z, float p3x,
                                         float p3y, float p3z, float nx, float ny, float nz, float w, V3 o, V3 d,
                                         float& t, bool& g) {
  const float dn = (nx * d.x + ny * d.y) + nz * d.z;        // dot(N, d)
  const float num = w - ((o.x * nx + o.y * ny) + o.z * nz);  // A.w - dot(o, N)
  const float tt = num / dn;
  const float Px = o.x + d.x * tt, Py = o.y + d.y * tt, Pz = o.z + d.z * tt;
  // dot(cross(b - a, P - a), N)
  auto edge = [&](float ax, float ay, float az, float bx, float by, float bz) -> float {
    const float ex = bx - ax, ey = by - ay, ez = bz - az;
    const float vx = Px - ax, vy = Py - ay, vz = Pz - az;
    const float cx = ey * vz - vy * ez, cy = ez * vx - vz * ex, cz = ex * vy - vx * ey;
    return (cx * nx + cy * ny) + cz * nz;
  };
  const float s1 = edge(p1x, p1y, p1z, p2x, p2y, p2z);
  const float s2 = edge(p2x, p2y, p2z, p3x, p3y, p3z);
  const float s3 = edge(p3x, p3y, p3z, p1x, p1y, p1z);
  t = tt;
  g = !(fabsf(dn) < 0.00001f) && !(tt < 0.0005f) && ((s1 > 0 && s2 > 0 && s3 > 0) || (s1 < 0 && s2 < 0 && s3 < 0));
}
template <bool IDS = false>
__device__ __forceinline__ void pairTestT(const float4* r, V3 o, V3 d, float& t0, float& t1, bool& g0, bool& g1,
                                          int* ids = nullptr) {
  const float4 q0 = r[0], q1 = r[1], q2 = r[2], q3 = r[3], q4 = r[4], q5 = r[5], q6 = r[6];
  if (IDS) ids[0] = __float_as_int(q6.z), ids[1] = __float_as_int(q6.w);
  // (p1.x, p1.y, p1.z, p2.x, ..., Ng.z, w) of triangle i in the x halves, i + 1 in the y halves
  pairHalf(q0.x, q0.z, q1.x, q1.z, q2.x, q2.z, q3.x, q3.z, q4.x, q4.z, q5.x, q5.z, q6.x, o, d, t0, g0);
  pairHalf(q0.y, q0.w, q1.y, q1.w, q2.y, q2.w, q3.y, q3.w, q4.y, q4.w, q5.y, q5.w, q6.y, o, d, t1, g1);
}
__device__ __forceinline__ void pairTest(const float4* r, V3 o, V3 d, float& t0, float& t1, bool& g0, bool& g1) {
  pairTestT<false>(r, o, d, t0, t1, g0, g1);
}
__device__ __forceinline__ void pairTestIds(const float4* r, V3 o, V3 d, float& t0, float& t1, bool& g0, bool& g1,
                                            int& id0, int& id1) {
  int ids[2];
  pairTestT<true>(r, o, d, t0, t1, g0, g1, ids);
  id0 = ids[0];
  id1 = ids[1];
}

__device__ __forceinline__ bool triHit(const float4* g, V3 o, V3 d, float tmax, float& t) {
  return triTest(g[0], g[1], g[2], g[3], o, d, tmax, t);
}

__device__ __forceinline__ bool isLeafRef(int ref) { return ref < 0 && ref != REF_NONE; }

// hitBVH IS:335-382: same visiting order of the leaves (nearer child by the
// reference's d first, ties to the right child), strict '<' closest update, so
// the same triangle wins even on exact-t ties. CULL skips children whose slab
// entry lies beyond the current closest hit (plus a margin, so tied triangles
// are still visited); ANYHIT returns on the first accepted triangle (env shadow
// rays, where only isHit is read: IS:776-779); anyRT is the same switch chosen
// per lane at run time.
//
// Loop structure ("while-while" with speculative node traversal): a lane that
// reaches a leaf parks it and keeps visiting the nodes that follow it in the
// visiting order until every lane still walking nodes holds a parked leaf; the
// wave then intersects the parked leaves together. Leaves are still intersected
// in the reference's order (the parked leaf precedes every node visited
// speculatively); node visits use a possibly stale tbest for culling, which
// only culls less.
//
// top (LDSTOP): the LDS copy of device node ids [0, S.nTop) -- the top of the
// tree -- read in place of the global records (one flat load serves lanes in
// both address spaces).
//
// TIES: *tie is set when a lane meets a triangle at exactly its current closest
// t (the visiting order decides such ties; see refReachable).
template <bool ANYHIT, bool CULL, bool COUNT, class StackType, bool LDSTOP = false, bool TIES = false,
          int KIND = NODE_EXACT>
__device__ __forceinline__ int traceRay(const SceneView& S, V3 o, V3 d, float& tOut, StackType& st, Counters& C,
                                        bool anyRT = false, const float4* top = nullptr, bool* tie = nullptr) {
  V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const FusedRay fr = fusedRay(o, inv);  // NODE_FUSED
  float tbest = PT_INF;
  int best = -1;
  int ref = S.rootRef;   // next item in visiting order (REF_NONE only when the stack is empty too)
  int leaf = REF_NONE;   // parked leaf, precedes ref
  st.reset();
  C.rays++;
  while (true) {
    // node phase
    while (ref >= 0) {
      if (PT_WAVE_TRACE && !COUNT) {  // diagnostics build: node-loop iterations (lane, wave)
        C.nodes++;
        if (__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) C.mats++;
      }
      NodeHit nh;
      const float4* nd = S.bvh + (size_t)4 * ref;
      if (LDSTOP && ref < S.nTop) nd = top + 4 * ref;
      visitAny<KIND>(nd, o, inv, fr, nh);
      const int lref = nh.lref, rref = nh.rref;
      const float d1 = nh.d1, d2 = nh.d2, t0l = nh.t0l, t0r = nh.t0r;
      bool h1 = (lref != REF_NONE) && d1 > 0.0f;
      bool h2 = (rref != REF_NONE) && d2 > 0.0f;
      if (COUNT) C.nodes += 1u + (lref != REF_NONE) + (rref != REF_NONE);
      if (CULL) {
        float lim = tbest + 1e-3f * fmaxf(1.0f, tbest);
        h1 = h1 && !(t0l > lim);
        h2 = h2 && !(t0r > lim);
      }
      int next;
      if (h1 && h2) {
        bool leftFirst = d1 < d2;
        st.push(leftFirst ? rref : lref);
        next = leftFirst ? lref : rref;
      } else if (h1) {
        next = lref;
      } else if (h2) {
        next = rref;
      } else {
        next = st.sp > 0 ? st.pop() : REF_NONE;
      }
      if (isLeafRef(next) && leaf == REF_NONE) {  // park it, walk on
        leaf = next;
        next = st.sp > 0 ? st.pop() : REF_NONE;
      }
      ref = next;
      // every lane still walking holds a leaf (or at most PT_LEAF_WAIT_MK still look for one)
      if (__popcll(__ballot(leaf == REF_NONE)) <= PT_LEAF_WAIT_MK) break;
    }
    // leaf phase
    if (leaf == REF_NONE && isLeafRef(ref)) {
      leaf = ref;
      ref = st.sp > 0 ? st.pop() : REF_NONE;
    }
    if (leaf == REF_NONE) {
      if (ref >= 0) continue;  // left the node phase early (PT_LEAF_WAIT_MK): on with its nodes
      break;                   // ref == REF_NONE too: done
    }
    {
      uint32_t v = ~(uint32_t)leaf;
      int start = (int)(v >> LEAF_CNT_BITS);
      int cnt = (int)(v & ((1u << LEAF_CNT_BITS) - 1u)) + 1;
      leaf = REF_NONE;
      if (COUNT) C.nodes++;
      float localBest = PT_INF;
      // two triangles per iteration from one pair record (one memory round trip,
      // packed math: pairTest; the last record pairs with zeros), accepted in
      // index order against the running tbest
      for (int k = 0; k < cnt; k += 2) {
        if (PT_WAVE_TRACE && !COUNT) {  // diagnostics build: leaf-loop iterations (lane, wave)
          C.tris++;
          if (__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) C.mats++;
        }
        const int i = start + k;
        const bool second = k + 1 < cnt;
        float t0, t1;
        bool g0, g1;
        pairTest(S.pairs + PAIR_F4 * (size_t)i, o, d, t0, t1, g0, g1);
        if (COUNT) {
          const bool h0 = g0 && t0 < PT_INF;
          const bool h1 = g1 && t1 < PT_INF && second;
          C.tris += 1u + (second ? 1u : 0u);
          if (h0 && t0 < localBest) { localBest = t0; C.mats++; }
          if (h0 && t0 < tbest) { tbest = t0; best = i; }
          if (h1 && t1 < localBest) { localBest = t1; C.mats++; }
          if (h1 && t1 < tbest) { tbest = t1; best = i + 1; }
        } else {
          if (TIES && g0 && t0 == tbest) *tie = true;
          if (g0 && t0 < tbest) {
            tbest = t0;
            best = i;
            if (ANYHIT || anyRT) { tOut = tbest; return best; }
          }
          if (TIES && g1 && second && t1 == tbest) *tie = true;
          if (g1 && second && t1 < tbest) {
            tbest = t1;
            best = i + 1;
            if (ANYHIT || anyRT) { tOut = tbest; return best; }
          }
        }
      }
    }
  }
  tOut = tbest;
  return best;
}

// ----------------------------------------------------------------- 4-wide runtime tree
// The runtime tree collapsed to 4-wide nodes (pt_runtime.cpp encodeWide4): per
// node {lo.x of children 0..3}, {lo.y}, {lo.z}, {hi.x}, {hi.y}, {hi.z}, {refs},
// {-}: 128 bytes, one line. A visit tests the four (widened) child boxes with
// fused slabs, visits the nearest hit child next and pushes the others far to
// near: about half the dependent node fetches of the binary walk, for
// memory-latency-bound walks of large scenes (the regen kernel on scenes past
// PT_WIDE_SCENE_MB). Results are checked exactly like the binary runtime
// tree's (the order of visits only matters for exact-t ties, which are
// flagged: refReachable, the retrace in the reference order). The walks return the
// winner's uploaded triangle index, read from its pair record (pairTestIds), so the
// reference check starts without a lookup of S.fastTri.
constexpr float PT_INF_KEY = __builtin_huge_valf();  // sort key of a missed child (every entry t is finite)
__device__ __forceinline__ void cswap(float& ka, int& ra, float& kb, int& rb) {
  const bool s = kb < ka;
  const float k = s ? kb : ka;
  const int r = s ? rb : ra;
  kb = s ? ka : kb;
  rb = s ? ra : rb;
  ka = k;
  ra = r;
}
// one 4-wide record: child planes lo/hi per axis (children 0..3 in x..w) and the refs
__device__ __forceinline__ void loadNode4(const float4* nd, float4& lx, float4& ly, float4& lz, float4& hx, float4& hy,
                                          float4& hz, float4& rf) {
  lx = nd[0], ly = nd[1], lz = nd[2], hx = nd[3], hy = nd[4], hz = nd[5], rf = nd[6];
}
// The whole 4-wide tree in LDS (the regen kernel's FULL variant): node k's float4 j (the 7
// a visit reads) at 7k + j. Lanes of a wave read different nodes; at the built 8-float4
// stride the j-th float4 of every node would sit in the same bank quad and a ds_read_b128 of
// 16 lanes would serialise on it; at 7 float4 node k's records start k quads apart (mod 8),
// spread over all of them. (Round 4's first layout rotated each record within its 128 B,
// 8k + ((j + k) & 7), with the same banks; the unrotated stride lets the seven reads share one
// address with immediate offsets: ~20 fewer VALU instructions per node visit.)
constexpr int W4_LDS_F4 = 7;
__device__ __forceinline__ void loadNode4Lds(const float4* tree, int k, float4& lx, float4& ly, float4& lz, float4& hx,
                                             float4& hy, float4& hz, float4& rf) {
  const float4* n = tree + W4_LDS_F4 * k;
  lx = n[0], ly = n[1], lz = n[2], hx = n[3], hy = n[4], hz = n[5], rf = n[6];
}
template <bool CULL, class StackType, bool LDSTOP>
__device__ __forceinline__ int traceRay4(const SceneView& S, V3 o, V3 d, float& tOut, StackType& st, Counters& C,
                                         bool anyRT, const float4* top, bool* tie) {
  const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const FusedRay fr = fusedRay(o, inv);
  const f32x2 sx = {fr.inv.x, fr.noi.x}, sy = {fr.inv.y, fr.noi.y}, sz = {fr.inv.z, fr.noi.z};
  float tbest = PT_INF;
  int best = -1;
  int ref = S.f4Root;
  int leaf = REF_NONE;
  st.reset();
  C.rays++;
  while (true) {
    while (ref >= 0) {
      if (PT_WAVE_TRACE) {  // diagnostics build: node-loop iterations (lane, wave)
        C.nodes++;
        if (__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) C.mats++;
      }
      const float4* nd = S.fbvh4 + (size_t)W4_F4 * ref;
      if (LDSTOP && ref < S.f4nTop) nd = top + W4_F4 * ref;
      float4 lx, ly, lz, hx, hy, hz, rf;
      loadNode4(nd, lx, ly, lz, hx, hy, hz, rf);
      float key[4];
      int r[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
      const float lim = tbest + 1e-3f * fmaxf(1.0f, tbest);
#pragma unroll
      for (int h = 0; h < 2; h++) {  // children (0, 1) and (2, 3) as packed pairs
        const f32x2 Lx = h ? f32x2{lx.z, lx.w} : f32x2{lx.x, lx.y}, Ly = h ? f32x2{ly.z, ly.w} : f32x2{ly.x, ly.y};
        const f32x2 Lz = h ? f32x2{lz.z, lz.w} : f32x2{lz.x, lz.y}, Hx = h ? f32x2{hx.z, hx.w} : f32x2{hx.x, hx.y};
        const f32x2 Hy = h ? f32x2{hy.z, hy.w} : f32x2{hy.x, hy.y}, Hz = h ? f32x2{hz.z, hz.w} : f32x2{hz.x, hz.y};
        const f32x2 fx = fmaBcast(Hx, sx), fy = fmaBcast(Hy, sy), fz = fmaBcast(Hz, sz);
        const f32x2 nx = fmaBcast(Lx, sx), ny = fmaBcast(Ly, sy), nz = fmaBcast(Lz, sz);
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int c = 2 * h + e;
          const float t1 = fminf(fmaxf(fx[e], nx[e]), fminf(fmaxf(fy[e], ny[e]), fmaxf(fz[e], nz[e])));
          const float t0 = fmaxf(fminf(fx[e], nx[e]), fmaxf(fminf(fy[e], ny[e]), fminf(fz[e], nz[e])));
          bool hit = r[c] != REF_NONE && t1 >= t0 && t1 > 0.0f;
          if (CULL) hit = hit && !(t0 > lim);
          key[c] = hit ? t0 : PT_INF_KEY;
        }
      }
      // nearest first: sort the four (entry t, ref) pairs, misses last
      cswap(key[0], r[0], key[1], r[1]);
      cswap(key[2], r[2], key[3], r[3]);
      cswap(key[0], r[0], key[2], r[2]);
      cswap(key[1], r[1], key[3], r[3]);
      cswap(key[1], r[1], key[2], r[2]);
      int next;
      if (key[0] < PT_INF_KEY) {
        if (key[3] < PT_INF_KEY) st.push(r[3]);
        if (key[2] < PT_INF_KEY) st.push(r[2]);
        if (key[1] < PT_INF_KEY) st.push(r[1]);
        next = r[0];
      } else {
        next = st.sp > 0 ? st.pop() : REF_NONE;
      }
      if (isLeafRef(next) && leaf == REF_NONE) {  // park it, walk on (traceRay's while-while)
        leaf = next;
        next = st.sp > 0 ? st.pop() : REF_NONE;
      }
      ref = next;
      if (__popcll(__ballot(leaf == REF_NONE)) <= PT_LEAF_WAIT_MK) break;
    }
    if (leaf == REF_NONE && isLeafRef(ref)) {
      leaf = ref;
      ref = st.sp > 0 ? st.pop() : REF_NONE;
    }
    if (leaf == REF_NONE) {
      if (ref >= 0) continue;  // left the node phase early (PT_LEAF_WAIT_MK): on with its nodes
      break;
    }
    const uint32_t v = ~(uint32_t)leaf;
    const int start = (int)(v >> LEAF_CNT_BITS);
    const int cnt = (int)(v & ((1u << LEAF_CNT_BITS) - 1u)) + 1;
    leaf = REF_NONE;
    for (int k = 0; k < cnt; k += 2) {
      if (PT_WAVE_TRACE) {  // diagnostics build: leaf-loop iterations (lane, wave)
        C.tris++;
        if (__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) C.mats++;
      }
      const int i = start + k;
      const bool second = k + 1 < cnt;
      float t0, t1;
      bool g0, g1;
      int id0, id1;
      pairTestIds(S.fpairs + PAIR_F4 * (size_t)i, o, d, t0, t1, g0, g1, id0, id1);
      if (g0 && t0 == tbest) *tie = true;
      if (g0 && t0 < tbest) {
        tbest = t0;
        best = id0;
        if (anyRT) { tOut = tbest; return best; }
      }
      if (g1 && second && t1 == tbest) *tie = true;
      if (g1 && second && t1 < tbest) {
        tbest = t1;
        best = id1;
        if (anyRT) { tOut = tbest; return best; }
      }
    }
  }
  tOut = tbest;
  return best;
}

// ----------------------------------------------------------------- resumable 4-wide walk
// The resumable walk's node phase ends once at most LW of its lanes still look for a leaf (0: every
// lane holds one, the while-while); the few still looking go on after the leaf phase. Measured
// (profiles/r5/ab, wall ms per frame): c2 (Lambert) LW 0 / 4 / 8 / 12 / 16: 0.1864 / 0.1807-0.1814 /
// 0.1795 / 0.1805 / 0.1853; c5 (MIS) 0 / 4 / 8 / 12 / 16: 4.88 / 4.25-4.28 / 4.21 / 4.17 / 4.16
#ifndef PT_LEAF_WAIT_U
#define PT_LEAF_WAIT_U 8
#endif
#ifndef PT_LEAF_WAIT_MIS
#define PT_LEAF_WAIT_MIS 12
#endif
// traceRay4 as a walk that can stop and resume (the regen kernel's dynamic ray
// fetch, PT_REGEN_YIELD): the walk's state is a Walk4 plus the lane's stack, and
// walk4Run returns once the lane's walk is done -- or, for the whole wave, as
// soon as `yield` of the lanes walking with it are done, so that those lanes go
// on with their paths (shade, take the next ray or pixel) instead of idling
// until the wave's longest walk ends; the others resume where they stopped on
// the next call. Per ray the sequence of node visits, leaf tests and closest-hit
// updates is traceRay4's (stopping between outer iterations changes nothing a
// lane computes), so results are identical.
struct Walk4 {
  float tbest;
  int best;  // the closest hit's uploaded triangle index (-1: none)
  int ref;   // next item in visiting order (REF_NONE: none)
  int leaf;  // parked leaf (REF_NONE: none)
  bool tie;
};
__device__ __forceinline__ bool walk4Done(const Walk4& w) { return w.ref == REF_NONE && w.leaf == REF_NONE; }
template <class StackType>
__device__ __forceinline__ void walk4Begin(const SceneView& S, Walk4& w, StackType& st, Counters& C) {
  w.tbest = PT_INF;
  w.best = -1;
  w.ref = S.f4Root;
  w.leaf = REF_NONE;
  w.tie = false;
  st.reset();
  C.rays++;
}
// ALL: every node is in LDS at `top`, swizzled (loadNode4Lds); else the first S.f4nTop are, in order
template <bool CULL, class StackType, bool LDSTOP, bool ALL = false, int LW = PT_LEAF_WAIT_U>
__device__ __forceinline__ void walk4Run(const SceneView& S, V3 o, V3 d, bool anyRT, Walk4& w, StackType& st,
                                         const float4* top, int yield, unsigned long long* ph = nullptr) {
  const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const FusedRay fr = fusedRay(o, inv);
  const f32x2 sx = {fr.inv.x, fr.noi.x}, sy = {fr.inv.y, fr.noi.y}, sz = {fr.inv.z, fr.noi.z};
  while (true) {
    const bool done = walk4Done(w);
    if (__ballot(!done) == 0 || __popcll(__ballot(done)) >= yield) break;  // wave-uniform
    if (done) continue;
    while (w.ref >= 0) {
      if (PT_PHASE_STATS && ph) {  // diagnostics build: node-loop iterations (wave, lanes)
        const unsigned long long m = __ballot(1);
        if (__lane_id() == __ffsll((unsigned long long)m) - 1) ph[7] += 1, ph[8] += __popcll(m);
      }
      float4 lx, ly, lz, hx, hy, hz, rf;
      if (ALL) {
        loadNode4Lds(top, w.ref, lx, ly, lz, hx, hy, hz, rf);
      } else {
        const float4* nd = S.fbvh4 + (size_t)W4_F4 * w.ref;
        if (LDSTOP && w.ref < S.f4nTop) nd = top + W4_F4 * w.ref;
        loadNode4(nd, lx, ly, lz, hx, hy, hz, rf);
      }
      float key[4];
      int r[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
      const float lim = w.tbest + 1e-3f * fmaxf(1.0f, w.tbest);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const f32x2 Lx = h ? f32x2{lx.z, lx.w} : f32x2{lx.x, lx.y}, Ly = h ? f32x2{ly.z, ly.w} : f32x2{ly.x, ly.y};
        const f32x2 Lz = h ? f32x2{lz.z, lz.w} : f32x2{lz.x, lz.y}, Hx = h ? f32x2{hx.z, hx.w} : f32x2{hx.x, hx.y};
        const f32x2 Hy = h ? f32x2{hy.z, hy.w} : f32x2{hy.x, hy.y}, Hz = h ? f32x2{hz.z, hz.w} : f32x2{hz.x, hz.y};
        const f32x2 fx = fmaBcast(Hx, sx), fy = fmaBcast(Hy, sy), fz = fmaBcast(Hz, sz);
        const f32x2 nx = fmaBcast(Lx, sx), ny = fmaBcast(Ly, sy), nz = fmaBcast(Lz, sz);
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int c = 2 * h + e;
          const float t1 = fminf(fmaxf(fx[e], nx[e]), fminf(fmaxf(fy[e], ny[e]), fmaxf(fz[e], nz[e])));
          const float t0 = fmaxf(fminf(fx[e], nx[e]), fmaxf(fminf(fy[e], ny[e]), fminf(fz[e], nz[e])));
          bool hit = r[c] != REF_NONE && t1 >= t0 && t1 > 0.0f;
          if (CULL) hit = hit && !(t0 > lim);
          key[c] = hit ? t0 : PT_INF_KEY;
        }
      }
      cswap(key[0], r[0], key[1], r[1]);
      cswap(key[2], r[2], key[3], r[3]);
      cswap(key[0], r[0], key[2], r[2]);
      cswap(key[1], r[1], key[3], r[3]);
      cswap(key[1], r[1], key[2], r[2]);
      int next;
      if (key[0] < PT_INF_KEY) {
        if (key[3] < PT_INF_KEY) st.push(r[3]);
        if (key[2] < PT_INF_KEY) st.push(r[2]);
        if (key[1] < PT_INF_KEY) st.push(r[1]);
        next = r[0];
      } else {
        next = st.sp > 0 ? st.pop() : REF_NONE;
      }
      if (isLeafRef(next) && w.leaf == REF_NONE) {
        w.leaf = next;
        next = st.sp > 0 ? st.pop() : REF_NONE;
      }
      w.ref = next;
      // the node phase ends once at most LW of its lanes still look for a leaf (above)
      if (__popcll(__ballot(w.leaf == REF_NONE)) <= LW) break;
    }
    if (w.leaf == REF_NONE && isLeafRef(w.ref)) {
      w.leaf = w.ref;
      w.ref = st.sp > 0 ? st.pop() : REF_NONE;
    }
    if (w.leaf == REF_NONE) continue;  // w.ref == REF_NONE too: this lane's walk is done
    const uint32_t v = ~(uint32_t)w.leaf;
    const int start = (int)(v >> LEAF_CNT_BITS);
    const int cnt = (int)(v & ((1u << LEAF_CNT_BITS) - 1u)) + 1;
    w.leaf = REF_NONE;
    for (int k = 0; k < cnt; k += 2) {
      if (PT_PHASE_STATS && ph) {  // diagnostics build: pair tests (wave, lanes)
        const unsigned long long m = __ballot(1);
        if (__lane_id() == __ffsll((unsigned long long)m) - 1) ph[9] += 1, ph[10] += __popcll(m);
      }
      const int i = start + k;
      const bool second = k + 1 < cnt;
      float t0, t1;
      bool g0, g1;
      int id0, id1;
      pairTestIds(S.fpairs + PAIR_F4 * (size_t)i, o, d, t0, t1, g0, g1, id0, id1);
      if (g0 && t0 == w.tbest) w.tie = true;
      if (g0 && t0 < w.tbest) {
        w.tbest = t0;
        w.best = id0;
        if (anyRT) { w.ref = REF_NONE; break; }  // any hit: the walk ends here (traceRay4's return)
      }
      if (g1 && second && t1 == w.tbest) w.tie = true;
      if (g1 && second && t1 < w.tbest) {
        w.tbest = t1;
        w.best = id1;
        if (anyRT) { w.ref = REF_NONE; break; }
      }
    }
  }
}

// ----------------------------------------------------------------- reference-exact results
// Reference-exact results through the runtime's tree. The reference's closest
// hit is the first, in its traversal order, of the triangles with the least t
// among those its traversal reaches; it reaches a triangle iff the ray's
// hitAABB is > 0 for every box on the path from the root to the triangle's
// leaf. The runtime's tree has conservative (widened) boxes, so its traversal
// meets every triangle the ray hits. Its result w (least t, no tie met) is
// therefore the reference's iff the reference reaches w, which refReachable
// decides: cheaply when the hit point lies inside w's reference leaf box by a
// margin far above the rounding of the slab arithmetic (the exact ray then
// crosses every enclosing box with room to spare, so every rounded slab test on
// the path passes), else by evaluating hitAABB up the reference path. A tie, or
// an unreachable w, sends the ray through the reference traversal itself.
// A miss in the runtime's tree is a miss in the reference's (it meets every
// triangle the ray hits). An any-hit result stands when its triangle is reachable.
// refReachable with the triangle's leaf box (leafBox[2 tri], [2 tri + 1]) at hand
// P (the hit point o + d t) inside box [lo, hi] by a margin far above the rounding of the box's slab
// arithmetic: the ray then passes the rounded slab test of this box and of every box enclosing it
__device__ __forceinline__ bool insideByMargin(V3 P, V3 o, float t, const float4 lo, const float4 hi) {
  const float scale = fmaxf(fmaxf(fabsf(P.x), fmaxf(fabsf(P.y), fabsf(P.z))),
                            fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)))) +
                      fmaxf(fmaxf(fmaxf(fabsf(lo.x), fabsf(hi.x)), fmaxf(fabsf(lo.y), fabsf(hi.y))),
                            fmaxf(fabsf(lo.z), fabsf(hi.z))) +
                      t + 1.0f;
  const float mu = 6.103515625e-05f * scale;  // 2^-14: >= 2^8 x the slab rounding
  return P.x - lo.x > mu && hi.x - P.x > mu && P.y - lo.y > mu && hi.y - P.y > mu && P.z - lo.z > mu &&
         hi.z - P.z > mu;
}
// UP: the walk up the reference path stops at the first box that holds the hit point by the margin
// (the large-scene MIS kernel, whose reference trees are deep: c5 4.46 -> 4.33 ms per frame; elsewhere
// the plain walk: the extra registers cost c2's whole-tree kernel 1.8 % (spills) and c3's 3.8 %)
template <bool UP = false>
__device__ __forceinline__ bool refReachableBox(const SceneView& S, const float4 lo, const float4 hi, V3 o, V3 d,
                                                float t) {
  const int leaf = __float_as_int(lo.w);  // the triangle's reference leaf (-1: in none)
  if (leaf < 0) return false;
  const V3 P = o + d * t;
  if (insideByMargin(P, o, t, lo, hi)) return true;
  // A leaf box flat in one axis a (a floor or a light quad: lo.a == hi.a bitwise) never passes the
  // margin test above. Every box on its path brackets the flat plane in a (the boxes nest), so each
  // box's a-slab values (lo.a - o.a) * inv.a and (hi.a - o.a) * inv.a bracket the plane's own value
  // ta exactly -- IEEE subtraction and multiplication by one reciprocal are monotone -- and the leaf's
  // a-slab is [ta, ta]. The path therefore passes when ta > 0 and the ray meets the plane inside the
  // other two axes' ranges by the margin: their slabs then hold ta with room to spare in every box.
  const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const bool flx = lo.x == hi.x, fly = lo.y == hi.y, flz = lo.z == hi.z;
  if ((int)flx + (int)fly + (int)flz == 1) {
    const float ta = flx ? (lo.x - o.x) * inv.x : fly ? (lo.y - o.y) * inv.y : (lo.z - o.z) * inv.z;
    if (ta > 0.0f && ta < PT_INF) {  // finite (a NaN fails too)
      const V3 Q = o + d * ta;
      const float sq = fmaxf(fmaxf(fabsf(Q.x), fmaxf(fabsf(Q.y), fabsf(Q.z))),
                             fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)))) +
                       fmaxf(fmaxf(fmaxf(fabsf(lo.x), fabsf(hi.x)), fmaxf(fabsf(lo.y), fabsf(hi.y))),
                             fmaxf(fabsf(lo.z), fabsf(hi.z))) +
                       ta + 1.0f;
      const float mq = 6.103515625e-05f * sq;
      if ((flx || (Q.x - lo.x > mq && hi.x - Q.x > mq)) && (fly || (Q.y - lo.y > mq && hi.y - Q.y > mq)) &&
          (flz || (Q.z - lo.z > mq && hi.z - Q.z > mq)))
        return true;
    }
  }
  // up the reference path: each box by hitAABB itself -- UP: until one holds P by the margin (that box
  // and every box enclosing it pass, as for the leaf box above; the boxes of a reference tree nest,
  // pt_runtime.cpp prepareAccel)
  for (int c = leaf; c != 1; c = S.refParent[c]) {
    if (c <= 0) return false;
    const float4 blo = S.refBox[2 * (size_t)c], bhi = S.refBox[2 * (size_t)c + 1];
    if (UP && c != leaf && insideByMargin(P, o, t, blo, bhi)) return true;
    float t0;
    if (!(hitAABB(o, inv, blo, bhi, t0) > 0.0f)) return false;
  }
  return true;
}
template <bool UP = false>
__device__ __forceinline__ bool refReachable(const SceneView& S, int tri, V3 o, V3 d, float t) {
  return refReachableBox<UP>(S, S.leafBox[2 * (size_t)tri], S.leafBox[2 * (size_t)tri + 1], o, d, t);
}
// the runtime's tree as a SceneView for traceRay / tracePacket
__device__ __forceinline__ SceneView fastView(const SceneView& S) {
  SceneView F = S;
  F.bvh = S.fbvh;
  F.pairs = S.fpairs;
  F.rootRef = S.fRoot;
  F.nTop = S.fnTop;
  return F;
}

// ----------------------------------------------------------------- camera-ray packets
// Closest hit of a wave's 64 camera rays as one packet (the rays of an 8x8 tile
// share the eye and nearly their direction, so they walk nearly the same
// nodes): the wave walks the tree once, each node record is a wave-uniform
// (scalar) load, every lane tests its own ray against both children's boxes
// with hitAABB, and a child is entered with the mask of the lanes whose own
// test hit it -- so each ray intersects exactly the leaves the reference
// traversal of that ray reaches (minus the ones culled by its current closest
// hit), only in a different order. Order only matters for exact ties (two
// triangles at the same t): a lane that meets a triangle at exactly its current
// closest t reports tie = true, and the caller retraces that ray with traceRay
// (the reference order). Children are entered nearer-first by majority vote of
// the lanes that hit both. pstack: this wave's LDS stack of (node, mask),
// PKT_DEPTH deep (the host enables packets only for trees that fit).
struct PacketEntry {
  int ref;
  int pad;
  unsigned long long mask;
};
template <bool CULL, int KIND = NODE_EXACT>
__device__ __forceinline__ int tracePacket(const SceneView& S, V3 o, V3 d, bool valid, float& tOut, bool& tie,
                                           PacketEntry* pstack, Counters& C, const float4* top) {
  const int lane = __lane_id();
  const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const FusedRay fr = fusedRay(o, inv);  // NODE_FUSED
  float tbest = PT_INF;
  int best = -1;
  tie = false;
  unsigned long long mask = __ballot(valid);
  if (valid) C.rays++;
  int ref = __builtin_amdgcn_readfirstlane(S.rootRef);
  int sp = 0;
  while (true) {
    if (ref >= 0) {  // internal node: one scalar record for the wave
      NodeHit nh;
      if (top && ref < S.nTop) visitAny<KIND>(top + 4 * ref, o, inv, fr, nh);  // LDS broadcast
      else visitAny<KIND>(S.bvh + (size_t)4 * ref, o, inv, fr, nh);
      nh.lref = __builtin_amdgcn_readfirstlane(nh.lref);
      nh.rref = __builtin_amdgcn_readfirstlane(nh.rref);
      const bool active = (mask >> lane) & 1ull;
      bool h1 = active && nh.lref != REF_NONE && nh.d1 > 0.0f;
      bool h2 = active && nh.rref != REF_NONE && nh.d2 > 0.0f;
      if (CULL) {
        const float lim = tbest + 1e-3f * fmaxf(1.0f, tbest);
        h1 = h1 && !(nh.t0l > lim);
        h2 = h2 && !(nh.t0r > lim);
      }
      const unsigned long long m1 = __ballot(h1), m2 = __ballot(h2);
      if (m1 && m2) {
        const int left = __popcll(__ballot(h1 && h2 && nh.d1 < nh.d2));
        const int right = __popcll(__ballot(h1 && h2 && !(nh.d1 < nh.d2)));
        const bool leftFirst = left >= right;
        if (lane == 0) {
          pstack[sp].ref = leftFirst ? nh.rref : nh.lref;
          pstack[sp].mask = leftFirst ? m2 : m1;
        }
        sp++;
        ref = leftFirst ? nh.lref : nh.rref;
        mask = leftFirst ? m1 : m2;
        continue;
      }
      if (m1 | m2) {
        ref = m1 ? nh.lref : nh.rref;
        mask = m1 ? m1 : m2;
        continue;
      }
    } else if (ref != REF_NONE) {  // leaf: its triangle pairs, scalar records
      const uint32_t v = ~(uint32_t)ref;
      const int start = (int)(v >> LEAF_CNT_BITS);
      const int cnt = (int)(v & ((1u << LEAF_CNT_BITS) - 1u)) + 1;
      const bool active = (mask >> lane) & 1ull;
      for (int k = 0; k < cnt; k += 2) {  // wave-uniform loop: the pair records are scalar loads
        const int i = start + k;
        float t0, t1;
        bool g0, g1;
        pairTest(S.pairs + PAIR_F4 * (size_t)i, o, d, t0, t1, g0, g1);
        g0 = g0 && active;
        g1 = g1 && active && k + 1 < cnt;
        if (g0 && t0 == tbest) tie = true;
        if (g0 && t0 < tbest) { tbest = t0; best = i; }
        if (g1 && t1 == tbest) tie = true;
        if (g1 && t1 < tbest) { tbest = t1; best = i + 1; }
      }
    }
    // pop the next (node, lanes) the packet still has to visit
    if (sp == 0) break;
    sp--;
    ref = __builtin_amdgcn_readfirstlane(pstack[sp].ref);
    const unsigned long long m = pstack[sp].mask;
    mask = (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)m) |
           (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(m >> 32)) << 32;
  }
  tOut = tbest;
  return best;
}

// ----------------------------------------------------------------- work queue
// The next 8x8 wave tile for the calling wave (wave-uniform; -1 when every queue is
// drained). Queue q holds tiles [q*perQueue, (q+1)*perQueue): one contiguous
// band of the frame, served first by the blocks with blockIdx % NUM_QUEUES == q
// (and so by one XCD under round-robin block placement), which keeps a band's
// BVH and env-map lines in that XCD's L2; after its home queue a wave steals
// round-robin. One tile per atomic measured best:
// claiming 2 or 4 per atomic, interleaving the queues or grouping an XCD's
// queues into one band were all slower or neutral; so was a launch-wide
// mask of drained queues that let a wave skip them without a failing atomic each (c2's
// shares and 100 frames within noise: 0.1699 vs 0.1704 ms).
// order (may be null = identity) replaces each queue's band by a list of work
// items built from the previous frame (reorderKernel): a tile whose paths form
// the frame's tail runs as 2^lg items of 64 >> lg pixels each (lg adapted per
// tile from frame to frame), longest items first, so the longest paths of a
// frame run side by side on otherwise idle SIMDs instead of forming its tail.
// Item encoding: tile | sub << 22 | lg << 28 (pixels [sub*(64>>lg), (sub+1)*(64>>lg))
// of the tile, row-major); order[q * orderCap + i], i < order[NUM_QUEUES * orderCap + q].
constexpr int ITEM_TILE_BITS = 22;
#ifndef PT_MAX_SPLIT_LG
#define PT_MAX_SPLIT_LG 6
#endif
constexpr int MAX_SPLIT_LG = PT_MAX_SPLIT_LG;
__device__ __forceinline__ int itemTile(int item) { return item & ((1 << ITEM_TILE_BITS) - 1); }
__device__ __forceinline__ int itemSub(int item) { return (item >> ITEM_TILE_BITS) & 63; }
__device__ __forceinline__ int itemLg(int item) { return (item >> 28) & 7; }
// A batch of nFrames frames (RenderParams::nFrames): claim `it` of queue q is work item
// it / nFrames of the band for frame it % nFrames, so a band's claims cover its items once
// per frame and the frames of one item are claimed one after another (set in *frame).
// (Round 6, a display() call's single frame: probing every queue not yet found empty in one round
// trip once the home queue drains -- 31 lanes, one counter each -- made c2 per call 0.455 -> 0.554
// ms: the probes of 4096 draining waves hammer every counter line at once. An agent-scope load
// instead of the atomic is served stale from the XCD's L2, 0.78 ms.)
static_assert(NUM_QUEUES <= 32, "TileCursor::drained holds one bit per work queue");
struct TileCursor {
  int qi = 0;  // queues found empty (wave-uniform)
  // optional: the block's LDS mask of the queues its waves found drained. A drained queue stays
  // drained for the rest of the launch, so once its home queue has drained a wave skips the queues
  // another wave of its block found empty instead of paying a device-scope claim (~3 us) on each;
  // without it every wave walks up to 31 drained queues one claim at a time while its in-flight
  // lanes wait. Per display() call (round 6, one box): c2 0.441 -> 0.425 ms, c3 0.370 -> 0.360, c4
  // and batched frames unchanged; consulting the mask before every claim (the home queue's too)
  // cost the batched frames 1-2 %. Not kept: a launch-wide mask in device memory beside it (set by
  // the first claim past a queue's end, read once when the home queue drains): c2 per call -1.4 %,
  // its batched frames +1.2 %, c3 / c4 unchanged
  unsigned* drained = nullptr;
  __device__ __forceinline__ int next(int* queue, int perQueue, int numItems, int home, int& frame, int nFrames = 1,
                                      const int* order = nullptr, int orderCap = 0) {
    while (qi < NUM_QUEUES) {
      const int q = (home + qi) & (NUM_QUEUES - 1);
      if (drained && qi > 0 &&
          ((__builtin_amdgcn_readfirstlane(*(volatile unsigned*)drained) >> q) & 1u)) {
        qi++;
        continue;
      }
      int it = 0;
      if ((threadIdx.x & 63) == 0) it = atomicAdd(queue + q * CTL_LINE_INTS, 1);
      it = __builtin_amdgcn_readfirstlane(it);  // lane 0's claim, as a scalar (the item is wave-uniform)
      const int k = nFrames == 1 ? it : it / nFrames;
      if (order) {
        if (it < order[NUM_QUEUES * orderCap + q] * nFrames) {
          frame = it - k * nFrames;
          return order[q * orderCap + k];
        }
      } else {
        const int t = q * perQueue + k;
        if (k < perQueue && t < numItems) {
          frame = it - k * nFrames;
          return t;
        }
      }
      if (drained && (threadIdx.x & 63) == 0) atomicOr(drained, 1u << q);
      qi++;
    }
    return -1;
  }
};

// Slot of pixel (px, py) in this context's screen-tile share, in the packed order of pt_pack_owned
// (pt_kernels.hip packedPixel): the index of a pipelined frame's colour and camera-ray buffers
// (RenderParams::colStride slots per frame). (px, py) must be one of the share's pixels.
__device__ __forceinline__ size_t shareIndex(const RenderParams& p, int px, int py) {
  const int ss = p.shardSize;
  const int gx = px / ss, gy = py / ss;
  const int j = (gy * p.shardsX + gx) / p.world;  // the share's j-th shard tile
  return (size_t)j * ss * ss + (size_t)((py - gy * ss) * ss + (px - gx * ss));
}

// The camera-ray pass's compacted results (RenderParams::primMask / primHit) of wave tile w of frame fr:
// the tile's mask, its entries, and slot k's result (PRIM_MISS for a slot outside the mask)
__device__ __forceinline__ unsigned long long primTileMask(const RenderParams& p, int fr, int w) {
  return p.primMask[(size_t)fr * p.numItems + w];
}
__device__ __forceinline__ const int2* primTileEntries(const RenderParams& p, int fr, int w) {
  return p.primHit + ((size_t)fr * p.numItems + w) * 64;
}
__device__ __forceinline__ int2 primOfSlot(unsigned long long m, const int2* e, int slot) {
  if (!((m >> slot) & 1ull)) return make_int2(PRIM_MISS, 0);
  return e[__popcll(m & ((1ull << slot) - 1ull))];
}

// per-wave sum of a lane counter into the block's padded shard
__device__ __forceinline__ void addRays(unsigned long long* shards, uint32_t r) {
  for (int off = 32; off > 0; off >>= 1) r += __shfl_down(r, off, 64);
  if ((threadIdx.x & 63) == 0 && r)
    atomicAdd(shards + (blockIdx.x & (RAY_SHARDS - 1)) * RAY_SHARD_STRIDE, (unsigned long long)r);
}

// The full HitResult (IS:63-71) of the winning triangle, computed once.
struct Hit {
  V3 P, N, viewDir;
  Material m;
  int matId;  // m's index in S.mats
};
// the emission of material matId (loadMaterial's emissive), for a path that keeps the camera
// hit's material index instead of its emission across its bounces
__device__ __forceinline__ V3 emissiveMat(const SceneView& S, int matId) {
  const float4* m = S.mats + MAT_F4 * (size_t)matId;
  const float4 a = m[0], b = m[1];
  return v3(a.z, a.w, b.x);
}
// the emission of triangle tri's material (finishHit's h.m.emissive)
__device__ __forceinline__ V3 emissiveOf(const SceneView& S, int tri) {
  return emissiveMat(S, __float_as_int(S.hitRec[HIT_F4 * (size_t)tri + 2].y));
}
__device__ __forceinline__ void finishHit(const SceneView& S, int tri, V3 o, V3 d, float t, Hit& h) {
  // the triangle's vertices and normal from its pair record (the x halves), the
  // record the leaf test of an uploaded-tree traversal has just read
  const float4* pr = S.pairs + PAIR_F4 * (size_t)tri;
  const float4 r0 = pr[0], r1 = pr[1], r2 = pr[2], r3 = pr[3], r4 = pr[4], r5 = pr[5];
  V3 p1 = v3(r0.x, r0.z, r1.x), p2 = v3(r1.z, r2.x, r2.z), p3 = v3(r3.x, r3.z, r4.x);
  bool inside = dot(v3(r4.z, r5.x, r5.z), d) > 0.0f;
  V3 P = o + d * t;
  float alpha = (-(P.x - p2.x) * (p3.y - p2.y) + (P.y - p2.y) * (p3.x - p2.x)) /
                (-(p1.x - p2.x - 0.00005f) * (p3.y - p2.y + 0.00005f) + (p1.y - p2.y + 0.00005f) * (p3.x - p2.x + 0.00005f));
  float beta = (-(P.x - p3.x) * (p1.y - p3.y) + (P.y - p3.y) * (p1.x - p3.x)) /
               (-(p2.x - p3.x - 0.00005f) * (p1.y - p3.y + 0.00005f) + (p2.y - p3.y + 0.00005f) * (p1.x - p3.x + 0.00005f));
  float gama = 1.0f - alpha - beta;
  const float4* q = S.hitRec + HIT_F4 * (size_t)tri;
  const float4 q0 = q[0], q1 = q[1], q2 = q[2];  // Triangle_encoded floats 9..17 + the material id
  V3 n1 = v3(q0.x, q0.y, q0.z), n2 = v3(q0.w, q1.x, q1.y), n3 = v3(q1.z, q1.w, q2.x);
  V3 Ns = normalize((n1 * alpha + n2 * beta) + n3 * gama);
  h.P = P;
  h.N = inside ? -Ns : Ns;
  h.viewDir = d;
  h.matId = __float_as_int(q2.y);
  h.m = loadMaterial(S.mats + MAT_F4 * (size_t)h.matId);
}

}  // namespace pt
