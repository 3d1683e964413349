// scene.cpp -- host-side scene preparation (pt_scene.h).
//
// Compiled with -ffp-contract=off: every float operation rounds once, in the
// order the reference's glm 0.9.9.8 code performs it, so the encoded arrays
// match what the reference host program would upload (OpenglRayTracing/main.cpp).
#include "pt_scene.h"
#include "pt_accel.h"
#include "pt_introsort.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

const float kINF = 2147483647.0f;  // #define INF 2147483647.0 (main.cpp:20), stored in floats

struct f3 {
  float x, y, z;
};
inline f3 F3(float x, float y, float z) { return f3{x, y, z}; }
inline f3 operator+(f3 a, f3 b) { return F3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline f3 operator-(f3 a, f3 b) { return F3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline f3 operator*(f3 a, float s) { return F3(a.x * s, a.y * s, a.z * s); }
inline float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline f3 cross(f3 a, f3 b) { return F3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
// glm::normalize = v * inversesqrt(dot(v,v)), inversesqrt(x) = 1/sqrt(x)
inline f3 normalize(f3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }
inline float gmax(float a, float b) { return (a < b) ? b : a; }  // glm/std max
inline float gmin(float a, float b) { return (b < a) ? b : a; }  // glm/std min

struct Mat4 {
  float m[4][4];  // m[col][row], glm layout
};
Mat4 identity() {
  Mat4 r;
  std::memset(&r, 0, sizeof(r));
  for (int i = 0; i < 4; i++) r.m[i][i] = 1.0f;
  return r;
}
// glm operator*(mat4, mat4) (type_mat4x4.inl:630-648)
Mat4 mul(const Mat4& a, const Mat4& b) {
  Mat4 r;
  for (int c = 0; c < 4; c++)
    for (int k = 0; k < 4; k++)
      r.m[c][k] = a.m[0][k] * b.m[c][0] + a.m[1][k] * b.m[c][1] + a.m[2][k] * b.m[c][2] + a.m[3][k] * b.m[c][3];
  return r;
}
// glm operator*(mat4, vec4) (type_mat4x4.inl:536-571): (m0*x + m1*y) + (m2*z + m3*w)
void mulv(const Mat4& M, const float v[4], float out[4]) {
  for (int k = 0; k < 4; k++) {
    float a0 = M.m[0][k] * v[0] + M.m[1][k] * v[1];
    float a1 = M.m[2][k] * v[2] + M.m[3][k] * v[3];
    out[k] = a0 + a1;
  }
}
// glm::inverse 4x4 (func_matrix.inl:294-351)
Mat4 inverse(const Mat4& M) {
  auto m = M.m;
  float Coef00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
  float Coef02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
  float Coef03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
  float Coef04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
  float Coef06 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
  float Coef07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
  float Coef08 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
  float Coef10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
  float Coef11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
  float Coef12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
  float Coef14 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
  float Coef15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
  float Coef16 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
  float Coef18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
  float Coef19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
  float Coef20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
  float Coef22 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
  float Coef23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
  float Fac[6][4] = {{Coef00, Coef00, Coef02, Coef03}, {Coef04, Coef04, Coef06, Coef07},
                     {Coef08, Coef08, Coef10, Coef11}, {Coef12, Coef12, Coef14, Coef15},
                     {Coef16, Coef16, Coef18, Coef19}, {Coef20, Coef20, Coef22, Coef23}};
  float Vec[4][4] = {{m[1][0], m[0][0], m[0][0], m[0][0]}, {m[1][1], m[0][1], m[0][1], m[0][1]},
                     {m[1][2], m[0][2], m[0][2], m[0][2]}, {m[1][3], m[0][3], m[0][3], m[0][3]}};
  float Inv[4][4];
  for (int k = 0; k < 4; k++) {
    Inv[0][k] = Vec[1][k] * Fac[0][k] - Vec[2][k] * Fac[1][k] + Vec[3][k] * Fac[2][k];
    Inv[1][k] = Vec[0][k] * Fac[0][k] - Vec[2][k] * Fac[3][k] + Vec[3][k] * Fac[4][k];
    Inv[2][k] = Vec[0][k] * Fac[1][k] - Vec[1][k] * Fac[3][k] + Vec[3][k] * Fac[5][k];
    Inv[3][k] = Vec[0][k] * Fac[2][k] - Vec[1][k] * Fac[4][k] + Vec[2][k] * Fac[5][k];
  }
  const float SignA[4] = {+1, -1, +1, -1}, SignB[4] = {-1, +1, -1, +1};
  Mat4 I;
  for (int k = 0; k < 4; k++) {
    I.m[0][k] = Inv[0][k] * SignA[k];
    I.m[1][k] = Inv[1][k] * SignB[k];
    I.m[2][k] = Inv[2][k] * SignA[k];
    I.m[3][k] = Inv[3][k] * SignB[k];
  }
  float Row0[4] = {I.m[0][0], I.m[1][0], I.m[2][0], I.m[3][0]};
  float Dot0[4];
  for (int k = 0; k < 4; k++) Dot0[k] = m[0][k] * Row0[k];
  float Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
  float One = 1.0f / Dot1;
  for (int c = 0; c < 4; c++)
    for (int k = 0; k < 4; k++) I.m[c][k] = I.m[c][k] * One;
  return I;
}
float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }
// glm::rotate (ext/matrix_transform.inl)
Mat4 rotate(const Mat4& m, float angle, f3 v) {
  float a = angle, c = std::cos(a), s = std::sin(a);
  f3 axis = normalize(v);
  f3 temp = axis * (1.0f - c);
  float R[3][3];
  R[0][0] = c + temp.x * axis.x;
  R[0][1] = temp.x * axis.y + s * axis.z;
  R[0][2] = temp.x * axis.z - s * axis.y;
  R[1][0] = temp.y * axis.x - s * axis.z;
  R[1][1] = c + temp.y * axis.y;
  R[1][2] = temp.y * axis.z + s * axis.x;
  R[2][0] = temp.z * axis.x + s * axis.y;
  R[2][1] = temp.z * axis.y - s * axis.x;
  R[2][2] = c + temp.z * axis.z;
  Mat4 r;
  for (int col = 0; col < 3; col++)
    for (int k = 0; k < 4; k++)
      r.m[col][k] = m.m[0][k] * R[col][0] + m.m[1][k] * R[col][1] + m.m[2][k] * R[col][2];
  for (int k = 0; k < 4; k++) r.m[3][k] = m.m[3][k];
  return r;
}

struct Material {
  f3 emissive, baseColor;
  float subsurface, metallic, specular, specularTint, roughness, anisotropic;
  float sheen, sheenTint, clearcoat, clearcoatGloss, IOR, transmission;
};
Material from_pt(const pt_material* m) {
  Material r;
  r.emissive = F3(m->emissive[0], m->emissive[1], m->emissive[2]);
  r.baseColor = F3(m->baseColor[0], m->baseColor[1], m->baseColor[2]);
  r.subsurface = m->subsurface; r.metallic = m->metallic; r.specular = m->specular;
  r.specularTint = m->specularTint; r.roughness = m->roughness; r.anisotropic = m->anisotropic;
  r.sheen = m->sheen; r.sheenTint = m->sheenTint; r.clearcoat = m->clearcoat;
  r.clearcoatGloss = m->clearcoatGloss; r.IOR = m->IOR; r.transmission = m->transmission;
  return r;
}

struct Triangle {  // main.cpp:45-49
  f3 p1, p2, p3, n1, n2, n3;
  Material material;
  int id = 0;  // uploaded index (buildAccel only)
};
struct BVHNode {  // main.cpp:63-67
  int left, right, n, index;
  f3 AA, BB;
};

// centre comparators (main.cpp:152-166): (p1+p2+p3)/vec3(3)
inline float centre(const Triangle& t, int axis) {
  f3 c = t.p1 + t.p2 + t.p3;
  float v = axis == 0 ? c.x : (axis == 1 ? c.y : c.z);
  return v / 3.0f;
}
struct CmpAxis {
  int axis;
  bool operator()(const Triangle& a, const Triangle& b) const { return centre(a, axis) < centre(b, axis); }
};

void node_bounds(const std::vector<Triangle>& tr, int l, int r, BVHNode& node) {
  node.AA = F3(kINF, kINF, kINF);
  node.BB = F3(-kINF, -kINF, -kINF);
  for (int i = l; i <= r; i++) {
    const Triangle& t = tr[i];
    float minx = gmin(t.p1.x, gmin(t.p2.x, t.p3.x));
    float miny = gmin(t.p1.y, gmin(t.p2.y, t.p3.y));
    float minz = gmin(t.p1.z, gmin(t.p2.z, t.p3.z));
    node.AA.x = gmin(node.AA.x, minx);
    node.AA.y = gmin(node.AA.y, miny);
    node.AA.z = gmin(node.AA.z, minz);
    float maxx = gmax(t.p1.x, gmax(t.p2.x, t.p3.x));
    float maxy = gmax(t.p1.y, gmax(t.p2.y, t.p3.y));
    float maxz = gmax(t.p1.z, gmax(t.p2.z, t.p3.z));
    node.BB.x = gmax(node.BB.x, maxx);
    node.BB.y = gmax(node.BB.y, maxy);
    node.BB.z = gmax(node.BB.z, maxz);
  }
}

int new_node(std::vector<BVHNode>& nodes) {
  nodes.push_back(BVHNode());
  int id = (int)nodes.size() - 1;
  nodes[id].left = nodes[id].right = nodes[id].n = nodes[id].index = 0;
  return id;
}

// appends a privately built subtree (ids from 1) to nodes, preserving preorder
int splice(std::vector<BVHNode>& nodes, const std::vector<BVHNode>& local, int root) {
  if (root == 0) return 0;
  const int shift = (int)nodes.size() - 1;  // local ids start at 1 (slot 0 is a placeholder)
  for (size_t k = 1; k < local.size(); k++) {
    BVHNode x = local[k];
    if (x.left > 0) x.left += shift;
    if (x.right > 0) x.right += shift;
    nodes.push_back(x);
  }
  return root + shift;
}

// ---- the reference builders (buildBVH main.cpp:376-427, buildBVHwithSAH main.cpp:430-551)
// The reference sorts Triangle records with std::sort by centre. Here the recursion orders
// triangle ids instead: (centre, id) pairs compared by centre make the same comparisons, so
// pt::exactSort (std::sort's permutation, computed in parallel -- pt_introsort.h) leaves the
// ids in the order the records would be in, and the per-triangle bounds the SAH sweeps read
// come from flat arrays rather than 140-byte records.
struct TriBox {
  float lo[3], hi[3];  // min / max over the three vertices
  float loZL, hiZL;    // the SAH left sweep's z bounds: main.cpp:480,484 read p2.x
};
struct RefInput {
  std::vector<float> c[3];  // centre per axis (main.cpp:152-166)
  std::vector<TriBox> box;  // one 32-byte record per triangle: a sweep step reads one line
};
RefInput ref_input(const std::vector<Triangle>& tr) {
  RefInput in;
  const size_t n = tr.size();
  for (int a = 0; a < 3; a++) in.c[a].resize(n);
  in.box.resize(n);
  for (size_t i = 0; i < n; i++) {
    const Triangle& t = tr[i];
    for (int a = 0; a < 3; a++) in.c[a][i] = centre(t, a);
    TriBox& b = in.box[i];
    b.lo[0] = gmin(t.p1.x, gmin(t.p2.x, t.p3.x));
    b.lo[1] = gmin(t.p1.y, gmin(t.p2.y, t.p3.y));
    b.lo[2] = gmin(t.p1.z, gmin(t.p2.z, t.p3.z));
    b.hi[0] = gmax(t.p1.x, gmax(t.p2.x, t.p3.x));
    b.hi[1] = gmax(t.p1.y, gmax(t.p2.y, t.p3.y));
    b.hi[2] = gmax(t.p1.z, gmax(t.p2.z, t.p3.z));
    b.loZL = gmin(t.p1.z, gmin(t.p2.x, t.p3.z));
    b.hiZL = gmax(t.p1.z, gmax(t.p2.x, t.p3.z));
  }
  return in;
}
struct KeyId {
  float k;
  int id;
};
struct KeyLess {
  bool operator()(const KeyId& a, const KeyId& b) const { return a.k < b.k; }
};
enum class RefKind { Median, SAH, FixedSAH };

struct RefScratch {
  std::vector<KeyId> kv;
  std::vector<float> right;  // suffix bounds of the SAH sweep, 6 per position
};

class RefBuilder {
 public:
  RefBuilder(const RefInput& in, RefKind kind, int leaf, int* id, pt::Helpers* h)
      : in_(in), kind_(kind), leaf_(leaf), id_(id), h_(h) {}

  // the recursion of main.cpp:376-427 / 430-551 with preorder node ids
  int build(std::vector<BVHNode>& nodes, int l, int r, RefScratch& s) {
    if (l > r) return 0;
    const int nid = new_node(nodes);
    bounds(l, r, nodes[nid]);
    if ((r - l + 1) <= leaf_) {
      nodes[nid].n = r - l + 1;
      nodes[nid].index = l;
      return nid;
    }
    const int mid = kind_ == RefKind::Median ? splitMedian(nodes[nid], l, r, s) : splitSAH(l, r, s);
    int left, right;
    if (std::min(mid - l + 1, r - mid) >= kParMin && h_->take()) {
      std::vector<BVHNode> ln(1), rn(1);
      int lr = 0;
      std::thread th([&] {
        RefScratch s2;
        lr = build(ln, l, mid, s2);
        h_->give();
      });
      const int rr = build(rn, mid + 1, r, s);
      th.join();
      left = splice(nodes, ln, lr);
      right = splice(nodes, rn, rr);
    } else {
      left = build(nodes, l, mid, s);
      right = build(nodes, mid + 1, r, s);
    }
    nodes[nid].left = left;
    nodes[nid].right = right;
    return nid;
  }

 private:
  static constexpr int kParMin = 4096;

  void bounds(int l, int r, BVHNode& node) const {
    node.AA = F3(kINF, kINF, kINF);
    node.BB = F3(-kINF, -kINF, -kINF);
    for (int i = l; i <= r; i++) {
      const TriBox& b = in_.box[id_[i]];
      node.AA.x = gmin(node.AA.x, b.lo[0]);
      node.AA.y = gmin(node.AA.y, b.lo[1]);
      node.AA.z = gmin(node.AA.z, b.lo[2]);
      node.BB.x = gmax(node.BB.x, b.hi[0]);
      node.BB.y = gmax(node.BB.y, b.hi[1]);
      node.BB.z = gmax(node.BB.z, b.hi[2]);
    }
  }

  // std::sort(tr + l, tr + r + 1, cmpx|cmpy|cmpz), on the ids. A range already strictly
  // increasing in the key is its own (unique) sorted order: no sort needed.
  void sortAxis(int l, int r, int axis, RefScratch& s) {
    const int cnt = r - l + 1;
    const float* key = in_.c[axis].data();
    s.kv.resize((size_t)cnt);
    bool strict = true;
    for (int i = 0; i < cnt; i++) {
      const int t = id_[l + i];
      s.kv[i] = KeyId{key[t], t};
      if (i && !(s.kv[i - 1].k < s.kv[i].k)) strict = false;
    }
    if (strict) return;
    pt::exactSort(s.kv.data(), s.kv.data() + cnt, KeyLess{}, cnt >= (1 << 16) ? h_ : nullptr);
    for (int i = 0; i < cnt; i++) id_[l + i] = s.kv[i].id;
  }

  int splitMedian(const BVHNode& node, int l, int r, RefScratch& s) {
    float lenx = node.BB.x - node.AA.x;
    float leny = node.BB.y - node.AA.y;
    float lenz = node.BB.z - node.AA.z;
    if (lenx >= leny && lenx >= lenz) sortAxis(l, r, 0, s);
    if (leny >= lenx && leny >= lenz) sortAxis(l, r, 1, s);
    if (lenz >= lenx && lenz >= leny) sortAxis(l, r, 2, s);
    return (l + r) / 2;
  }

  int splitSAH(int l, int r, RefScratch& s) {
    const bool zTypo = kind_ == RefKind::SAH;
    float Cost = kINF;
    int Axis = 0;
    int Split = (l + r) / 2;
    const int cnt = r - l + 1;
    s.right.resize((size_t)cnt * 6);
    float* R = s.right.data();
    for (int axis = 0; axis < 3; axis++) {
      sortAxis(l, r, axis, s);
      // suffix bounds (main.cpp:487-503)
      float Mx = -kINF, My = -kINF, Mz = -kINF, mx = kINF, my = kINF, mz = kINF;
      for (int i = r; i >= l; i--) {
        const TriBox& b = in_.box[id_[i]];
        Mx = gmax(Mx, b.hi[0]); My = gmax(My, b.hi[1]); Mz = gmax(Mz, b.hi[2]);
        mx = gmin(mx, b.lo[0]); my = gmin(my, b.lo[1]); mz = gmin(mz, b.lo[2]);
        float* o = R + (size_t)(i - l) * 6;
        o[0] = Mx; o[1] = My; o[2] = Mz; o[3] = mx; o[4] = my; o[5] = mz;
      }
      // prefix bounds (main.cpp:471-485) and the cost sweep (main.cpp:505-534)
      Mx = My = Mz = -kINF;
      mx = my = mz = kINF;
      float cost = kINF;
      int split = l;
      for (int i = l; i <= r - 1; i++) {
        const TriBox& b = in_.box[id_[i]];
        Mx = gmax(Mx, b.hi[0]); My = gmax(My, b.hi[1]); Mz = gmax(Mz, zTypo ? b.hiZL : b.hi[2]);
        mx = gmin(mx, b.lo[0]); my = gmin(my, b.lo[1]); mz = gmin(mz, zTypo ? b.loZL : b.lo[2]);
        float lenx = Mx - mx, leny = My - my, lenz = Mz - mz;
        float leftS = (float)(2.0 * (double)((lenx * leny) + (lenx * lenz) + (leny * lenz)));
        float leftCost = leftS * (float)(i - l + 1);
        const float* o = R + (size_t)(i + 1 - l) * 6;
        lenx = o[0] - o[3]; leny = o[1] - o[4]; lenz = o[2] - o[5];
        float rightS = (float)(2.0 * (double)((lenx * leny) + (lenx * lenz) + (leny * lenz)));
        float rightCost = rightS * (float)(r - i);
        float totalCost = leftCost + rightCost;
        if (totalCost < cost) {
          cost = totalCost;
          split = i;
        }
      }
      if (cost < Cost) {
        Cost = cost;
        Axis = axis;
        Split = split;
      }
    }
    sortAxis(l, r, Axis, s);  // main.cpp:537-544
    return Split;
  }

  const RefInput& in_;
  RefKind kind_;
  int leaf_;
  int* id_;
  pt::Helpers* h_;
};

// Binned SAH (32 bins over centroid bounds), O(n log n). Not a reference
// routine: a fast builder for the 1M-triangle stress scene. Same node
// encoding, preorder node ids, contiguous leaf ranges.
struct Box {
  f3 lo, hi;
};
inline Box empty_box() { return Box{F3(kINF, kINF, kINF), F3(-kINF, -kINF, -kINF)}; }
inline void grow(Box& b, f3 p) {
  b.lo = F3(gmin(b.lo.x, p.x), gmin(b.lo.y, p.y), gmin(b.lo.z, p.z));
  b.hi = F3(gmax(b.hi.x, p.x), gmax(b.hi.y, p.y), gmax(b.hi.z, p.z));
}
inline void grow(Box& b, const Box& o) {
  if (o.hi.x < o.lo.x) return;  // empty bin
  grow(b, o.lo);
  grow(b, o.hi);
}
inline float area(const Box& b) {
  if (b.hi.x < b.lo.x) return 0.0f;
  f3 d = b.hi - b.lo;
  return 2.0f * (d.x * d.y + d.x * d.z + d.y * d.z);
}
int splitBinned(std::vector<Triangle>& tr, const BVHNode&, int l, int r, bool) {
  Box cb = empty_box();
  for (int i = l; i <= r; i++) grow(cb, F3(centre(tr[i], 0), centre(tr[i], 1), centre(tr[i], 2)));
  const int NB = 32;
  float bestCost = kINF;
  int bestAxis = -1, bestBin = -1;
  float ext[3] = {cb.hi.x - cb.lo.x, cb.hi.y - cb.lo.y, cb.hi.z - cb.lo.z};
  float lo[3] = {cb.lo.x, cb.lo.y, cb.lo.z};
  for (int axis = 0; axis < 3; axis++) {
    if (!(ext[axis] > 0.0f)) continue;
    Box bb[NB];
    int bc[NB];
    for (int b = 0; b < NB; b++) { bb[b] = empty_box(); bc[b] = 0; }
    float scale = NB / ext[axis];
    for (int i = l; i <= r; i++) {
      int b = (int)((centre(tr[i], axis) - lo[axis]) * scale);
      b = b < 0 ? 0 : (b >= NB ? NB - 1 : b);
      bc[b]++;
      grow(bb[b], tr[i].p1); grow(bb[b], tr[i].p2); grow(bb[b], tr[i].p3);
    }
    float rightArea[NB];
    int rightCnt[NB];
    Box acc = empty_box();
    int c = 0;
    for (int b = NB - 1; b > 0; b--) {
      grow(acc, bb[b]); c += bc[b];
      rightArea[b] = area(acc); rightCnt[b] = c;
    }
    acc = empty_box(); c = 0;
    for (int b = 0; b < NB - 1; b++) {
      grow(acc, bb[b]); c += bc[b];
      if (c == 0 || rightCnt[b + 1] == 0) continue;
      float cost = area(acc) * c + rightArea[b + 1] * rightCnt[b + 1];
      if (cost < bestCost) { bestCost = cost; bestAxis = axis; bestBin = b; }
    }
  }
  int mid;
  if (bestAxis < 0) {
    mid = (l + r) / 2;  // all centroids coincide: median split
  } else {
    float scale = NB / ext[bestAxis];
    auto it = std::partition(tr.begin() + l, tr.begin() + r + 1, [&](const Triangle& t) {
      int b = (int)((centre(t, bestAxis) - lo[bestAxis]) * scale);
      b = b < 0 ? 0 : (b >= NB ? NB - 1 : b);
      return b <= bestBin;
    });
    mid = (int)(it - tr.begin()) - 1;
    if (mid < l || mid >= r) mid = (l + r) / 2;
  }
  return mid;
}

// Recursive build shared by the builders: preorder node ids (a node, then its
// left subtree, then its right subtree), contiguous leaf ranges. Subtrees of
// more than kParMin triangles are built on their own threads (up to parDepth
// levels deep) into private arrays that are spliced back in preorder, so the
// node array and the triangle order are identical to a serial build.
typedef int (*SplitFn)(std::vector<Triangle>&, const BVHNode&, int, int, bool);
constexpr int kParMin = 8192;

int buildTree(std::vector<Triangle>& tr, std::vector<BVHNode>& nodes, int l, int r, int n, SplitFn split, bool flag,
              int parDepth) {
  if (l > r) return 0;
  const int id = new_node(nodes);
  node_bounds(tr, l, r, nodes[id]);
  if ((r - l + 1) <= n) {
    nodes[id].n = r - l + 1;
    nodes[id].index = l;
    return id;
  }
  const int mid = split(tr, nodes[id], l, r, flag);
  int left, right;
  if (parDepth > 0 && r - l + 1 >= kParMin) {
    std::vector<BVHNode> ln(1), rn(1);
    int lr = 0;
    std::thread th([&] { lr = buildTree(tr, ln, l, mid, n, split, flag, parDepth - 1); });
    const int rr = buildTree(tr, rn, mid + 1, r, n, split, flag, parDepth - 1);
    th.join();
    left = splice(nodes, ln, lr);
    right = splice(nodes, rn, rr);
  } else {
    left = buildTree(tr, nodes, l, mid, n, split, flag, 0);
    right = buildTree(tr, nodes, mid + 1, r, n, split, flag, 0);
  }
  nodes[id].left = left;
  nodes[id].right = right;
  return id;
}



int tree_depth(const std::vector<BVHNode>& nodes) {
  if (nodes.size() < 2) return 0;
  std::vector<std::pair<int, int>> st{{1, 1}};
  int depth = 0;
  while (!st.empty()) {
    auto [k, d] = st.back();
    st.pop_back();
    depth = std::max(depth, d);
    if (nodes[k].n > 0) continue;
    if (nodes[k].left > 0) st.push_back({nodes[k].left, d + 1});
    if (nodes[k].right > 0) st.push_back({nodes[k].right, d + 1});
  }
  return depth;
}

}  // namespace

int pt::buildAccel(const float* tris, int nTri, int leafSize, std::vector<float>& out, std::vector<int>& order) {
  if (!tris || nTri < 1 || leafSize < 1) return -1;
  std::vector<Triangle> tr((size_t)nTri);
  for (int i = 0; i < nTri; i++) {
    const float* t = tris + (size_t)i * 36;
    tr[i].p1 = F3(t[0], t[1], t[2]);
    tr[i].p2 = F3(t[3], t[4], t[5]);
    tr[i].p3 = F3(t[6], t[7], t[8]);
    tr[i].id = i;
  }
  std::vector<BVHNode> nodes(1);
  nodes[0] = BVHNode{0, 0, 0, 0, F3(0, 0, 0), F3(0, 0, 0)};
  nodes.reserve(2 * (size_t)nTri / (size_t)leafSize + 16);
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  int parDepth = 0;
  while ((1u << parDepth) < hw) parDepth++;
  buildTree(tr, nodes, 0, nTri - 1, leafSize, splitBinned, false, parDepth);
  out.assign(nodes.size() * 12, 0.0f);
  for (size_t i = 0; i < nodes.size(); i++) {
    const BVHNode& n = nodes[i];
    float* o = out.data() + i * 12;
    o[0] = (float)n.left;
    o[1] = (float)n.right;
    o[3] = (float)n.n;
    o[4] = (float)n.index;
    o[6] = n.AA.x; o[7] = n.AA.y; o[8] = n.AA.z;
    o[9] = n.BB.x; o[10] = n.BB.y; o[11] = n.BB.z;
  }
  order.resize((size_t)nTri);
  for (int i = 0; i < nTri; i++) order[i] = tr[i].id;
  return tree_depth(nodes);
}

struct pt_scene {
  std::vector<Triangle> triangles;
  std::vector<BVHNode> nodes;
  int depth = 0;
};

extern "C" {

void pt_material_default(pt_material* m) {
  std::memset(m, 0, sizeof(*m));
  m->baseColor[0] = m->baseColor[1] = m->baseColor[2] = 1.0f;
  m->IOR = 1.0f;
}

int pt_scene_create(pt_scene** out) {
  if (!out) return -1;
  *out = new (std::nothrow) pt_scene();
  return *out ? 0 : -5;
}
void pt_scene_destroy(pt_scene* s) { delete s; }

// readObj steps after parsing (main.cpp:320-371)
static int finish_mesh(pt_scene* s, std::vector<f3>& vertices, const std::vector<int>& indices, float maxx,
                       float maxy, float maxz, float minx, float miny, float minz, const pt_material* pm,
                       const float trans[16], int smoothNormal) {
  for (int ix : indices)
    if (ix < 0 || ix >= (int)vertices.size()) return -4;
  float lenx = maxx - minx;
  float leny = maxy - miny;
  float lenz = maxz - minz;
  float maxaxis = gmax(lenx, gmax(leny, lenz));
  for (auto& v : vertices) {
    v.x /= maxaxis;
    v.y /= maxaxis;
    v.z /= maxaxis;
  }
  Mat4 T;
  if (trans) std::memcpy(T.m, trans, sizeof(float) * 16);
  else T = identity();
  for (auto& v : vertices) {
    float vv[4] = {v.x, v.y, v.z, 1.0f}, o[4];
    mulv(T, vv, o);
    v = F3(o[0], o[1], o[2]);
  }
  std::vector<f3> normals(vertices.size(), F3(0, 0, 0));
  for (size_t i = 0; i + 2 < indices.size(); i += 3) {
    f3 p1 = vertices[indices[i]], p2 = vertices[indices[i + 1]], p3 = vertices[indices[i + 2]];
    f3 n = normalize(cross(p2 - p1, p3 - p1));
    normals[indices[i]] = normals[indices[i]] + n;
    normals[indices[i + 1]] = normals[indices[i + 1]] + n;
    normals[indices[i + 2]] = normals[indices[i + 2]] + n;
  }
  pt_material dm;
  if (!pm) { pt_material_default(&dm); pm = &dm; }
  Material mat = from_pt(pm);
  size_t offset = s->triangles.size();
  s->triangles.resize(offset + indices.size() / 3);
  for (size_t i = 0; i + 2 < indices.size(); i += 3) {
    Triangle& t = s->triangles[offset + i / 3];
    t.p1 = vertices[indices[i]];
    t.p2 = vertices[indices[i + 1]];
    t.p3 = vertices[indices[i + 2]];
    if (!smoothNormal) {
      f3 n = normalize(cross(t.p2 - t.p1, t.p3 - t.p1));
      t.n1 = t.n2 = t.n3 = n;
    } else {
      t.n1 = normalize(normals[indices[i]]);
      t.n2 = normalize(normals[indices[i + 1]]);
      t.n3 = normalize(normals[indices[i + 2]]);
    }
    t.material = mat;
  }
  s->nodes.clear();
  return 0;
}

// readObj parse loop (main.cpp:280-318), including the AABB typo at :297-298
static int parse_obj(pt_scene* s, std::istream& fin, const pt_material* m, const float trans[16], int smooth) {
  std::vector<f3> vertices;
  std::vector<int> indices;
  float maxx = -kINF, maxy = -kINF, maxz = -kINF, minx = kINF, miny = kINF, minz = kINF;
  std::string line;
  while (std::getline(fin, line)) {
    std::istringstream sin(line);
    std::string type;
    float x = 0, y = 0, z = 0;
    int v0 = 0, v1 = 0, v2 = 0, vn0 = 0, vn1 = 0, vn2 = 0, vt0 = 0, vt1 = 0, vt2 = 0;  // vt, vn parsed and dropped (main.cpp:284-286)
    char slash;
    int slashCnt = 0;
    for (char c : line)
      if (c == '/') slashCnt++;
    sin >> type;
    if (type == "v") {
      sin >> x >> y >> z;
      vertices.push_back(F3(x, y, z));
      maxx = gmax(maxx, x); maxy = gmax(maxx, y); maxz = gmax(maxx, z);
      minx = gmin(minx, x); miny = gmin(minx, y); minz = gmin(minx, z);
    }
    if (type == "f") {
      if (slashCnt == 6) {
        sin >> v0 >> slash >> vt0 >> slash >> vn0;
        sin >> v1 >> slash >> vt1 >> slash >> vn1;
        sin >> v2 >> slash >> vt2 >> slash >> vn2;
      } else if (slashCnt == 3) {
        sin >> v0 >> slash >> vt0;
        sin >> v1 >> slash >> vt1;
        sin >> v2 >> slash >> vt2;
      } else {
        sin >> v0 >> v1 >> v2;
      }
      indices.push_back(v0 - 1);
      indices.push_back(v1 - 1);
      indices.push_back(v2 - 1);
    }
  }
  return finish_mesh(s, vertices, indices, maxx, maxy, maxz, minx, miny, minz, m, trans, smooth);
}

int pt_scene_read_obj(pt_scene* s, const char* path, const pt_material* m, const float trans[16], int smoothNormal) {
  if (!s || !path) return -1;
  std::ifstream fin(path);
  if (!fin.is_open()) return -6;
  return parse_obj(s, fin, m, trans, smoothNormal);
}

int pt_scene_read_obj_text(pt_scene* s, const char* text, const pt_material* m, const float trans[16],
                           int smoothNormal) {
  if (!s || !text) return -1;
  std::istringstream fin{std::string(text)};
  return parse_obj(s, fin, m, trans, smoothNormal);
}

int pt_scene_add_mesh(pt_scene* s, const float* verts, int nv, const int* idx, int nTri, const pt_material* m,
                      const float trans[16], int smoothNormal) {
  if (!s || !verts || !idx || nv <= 0 || nTri < 0) return -1;
  std::vector<f3> vertices((size_t)nv);
  float maxx = -kINF, maxy = -kINF, maxz = -kINF, minx = kINF, miny = kINF, minz = kINF;
  for (int i = 0; i < nv; i++) {
    float x = verts[3 * i], y = verts[3 * i + 1], z = verts[3 * i + 2];
    vertices[i] = F3(x, y, z);
    maxx = gmax(maxx, x); maxy = gmax(maxx, y); maxz = gmax(maxx, z);
    minx = gmin(minx, x); miny = gmin(minx, y); minz = gmin(minx, z);
  }
  std::vector<int> indices(idx, idx + (size_t)nTri * 3);
  return finish_mesh(s, vertices, indices, maxx, maxy, maxz, minx, miny, minz, m, trans, smoothNormal);
}

int pt_scene_num_triangles(const pt_scene* s) { return s ? (int)s->triangles.size() : 0; }
int pt_scene_num_nodes(const pt_scene* s) { return s ? (int)s->nodes.size() : 0; }
int pt_scene_depth(const pt_scene* s) { return s ? s->depth : 0; }

int pt_scene_build_bvh(pt_scene* s, int builder, int leafSize) {
  if (!s || leafSize < 1 || s->triangles.empty()) return -1;
  // dummy node 0 (main.cpp:675-681); its index is uninitialised there, 0 here
  BVHNode testNode;
  testNode.left = 255;
  testNode.right = 128;
  testNode.n = 30;
  testNode.index = 0;
  testNode.AA = F3(1, 1, 0);
  testNode.BB = F3(0, 1, 0);
  s->nodes.assign(1, testNode);
  s->nodes.reserve(2 * s->triangles.size() / (size_t)leafSize + 16);
  const int r = (int)s->triangles.size() - 1;
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (builder == PT_BVH_BINNED_SAH) {
    int parDepth = 0;  // up to 2^parDepth subtrees in flight
    while ((1u << parDepth) < hw) parDepth++;
    buildTree(s->triangles, s->nodes, 0, r, leafSize, splitBinned, false, parDepth);
  } else {
    RefKind kind;
    switch (builder) {
      case PT_BVH_REFERENCE_SAH: kind = RefKind::SAH; break;
      case PT_BVH_REFERENCE_MEDIAN: kind = RefKind::Median; break;
      case PT_BVH_FIXED_SAH: kind = RefKind::FixedSAH; break;
      default: return -1;
    }
    const RefInput in = ref_input(s->triangles);
    std::vector<int> id((size_t)r + 1);
    for (int i = 0; i <= r; i++) id[i] = i;
    pt::Helpers helpers((int)hw - 1);
    RefScratch scratch;
    RefBuilder(in, kind, leafSize, id.data(), &helpers).build(s->nodes, 0, r, scratch);
    std::vector<Triangle> built((size_t)r + 1);
    for (int i = 0; i <= r; i++) built[i] = s->triangles[id[i]];
    s->triangles.swap(built);
  }
  s->depth = tree_depth(s->nodes);
  return 0;
}

// encode (main.cpp:687-716)
int pt_scene_encode(const pt_scene* s, float* tris_out, float* nodes_out) {
  if (!s) return -1;
  if (tris_out) {
    for (size_t i = 0; i < s->triangles.size(); i++) {
      const Triangle& t = s->triangles[i];
      const Material& m = t.material;
      float* o = tris_out + i * 36;
      const f3 v[8] = {t.p1, t.p2, t.p3, t.n1, t.n2, t.n3, m.emissive, m.baseColor};
      for (int k = 0; k < 8; k++) { o[3 * k] = v[k].x; o[3 * k + 1] = v[k].y; o[3 * k + 2] = v[k].z; }
      const float p[12] = {m.subsurface, m.metallic,  m.specular,  m.specularTint,   m.roughness, m.anisotropic,
                           m.sheen,      m.sheenTint, m.clearcoat, m.clearcoatGloss, m.IOR,       m.transmission};
      std::memcpy(o + 24, p, sizeof(p));
    }
  }
  if (nodes_out) {
    for (size_t i = 0; i < s->nodes.size(); i++) {
      const BVHNode& n = s->nodes[i];
      float* o = nodes_out + i * 12;
      o[0] = (float)n.left; o[1] = (float)n.right; o[2] = 0.0f;
      o[3] = (float)n.n; o[4] = (float)n.index; o[5] = 0.0f;
      o[6] = n.AA.x; o[7] = n.AA.y; o[8] = n.AA.z;
      o[9] = n.BB.x; o[10] = n.BB.y; o[11] = n.BB.z;
    }
  }
  return 0;
}

void pt_transform_matrix(const float rotateDeg[3], const float translate[3], const float scale[3], float out[16]) {
  Mat4 unit = identity();
  Mat4 S = unit;  // glm::scale
  for (int k = 0; k < 4; k++) {
    S.m[0][k] = unit.m[0][k] * scale[0];
    S.m[1][k] = unit.m[1][k] * scale[1];
    S.m[2][k] = unit.m[2][k] * scale[2];
  }
  Mat4 Tm = unit;  // glm::translate: Result[3] = m0*v0 + m1*v1 + m2*v2 + m3
  for (int k = 0; k < 4; k++)
    Tm.m[3][k] = unit.m[0][k] * translate[0] + unit.m[1][k] * translate[1] + unit.m[2][k] * translate[2] + unit.m[3][k];
  Mat4 R = unit;
  R = rotate(R, radians(rotateDeg[0]), F3(1, 0, 0));
  R = rotate(R, radians(rotateDeg[1]), F3(0, 1, 0));
  R = rotate(R, radians(rotateDeg[2]), F3(0, 0, 1));
  Mat4 model = mul(mul(Tm, R), S);
  std::memcpy(out, model.m, sizeof(float) * 16);
}

void pt_orbit_camera(float rotateAngle, float upAngle, float r, float eye_out[3], float cameraRotate[16]) {
  f3 eye = F3(-std::sin(radians(rotateAngle)) * std::cos(radians(upAngle)), std::sin(radians(upAngle)),
              std::cos(radians(rotateAngle)) * std::cos(radians(upAngle)));
  eye.x *= r; eye.y *= r; eye.z *= r;
  // lookAtRH (ext/matrix_transform.inl:99-119)
  f3 center = F3(0, 0, 0), up = F3(0, 1, 0);
  f3 f = normalize(center - eye);
  f3 s = normalize(cross(f, up));
  f3 u = cross(s, f);
  Mat4 L = identity();
  L.m[0][0] = s.x; L.m[1][0] = s.y; L.m[2][0] = s.z;
  L.m[0][1] = u.x; L.m[1][1] = u.y; L.m[2][1] = u.z;
  L.m[0][2] = -f.x; L.m[1][2] = -f.y; L.m[2][2] = -f.z;
  L.m[3][0] = -dot(s, eye); L.m[3][1] = -dot(u, eye); L.m[3][2] = dot(f, eye);
  Mat4 I = inverse(L);
  eye_out[0] = eye.x; eye_out[1] = eye.y; eye_out[2] = eye.z;
  std::memcpy(cameraRotate, I.m, sizeof(float) * 16);
}

// ---------------------------------------------------------------- HDR
// In-memory restatement of HDRLoader (hdrloader.cpp:29-191). fgetc/feof/fseek
// semantics are emulated on a byte buffer so malformed files behave the same.
namespace {
struct Reader {
  const unsigned char* p;
  int64_t n, pos = 0;
  bool eof = false;
  int getc() {
    if (pos >= n) { eof = true; return -1; }
    return p[pos++];
  }
  void back() { if (pos > 0) pos--; eof = false; }
};
typedef unsigned char RGBE[4];
bool oldDecrunch(RGBE* scanline, int len, Reader& f, RGBE* base) {
  int rshift = 0;
  while (len > 0) {
    scanline[0][0] = (unsigned char)f.getc();
    scanline[0][1] = (unsigned char)f.getc();
    scanline[0][2] = (unsigned char)f.getc();
    scanline[0][3] = (unsigned char)f.getc();
    if (f.eof) return false;
    if (scanline[0][0] == 1 && scanline[0][1] == 1 && scanline[0][2] == 1) {
      for (int i = scanline[0][3] << rshift; i > 0; i--) {
        if (scanline == base || len <= 0) return false;  // reference reads scanline[-1] / overruns here
        std::memcpy(&scanline[0][0], &scanline[-1][0], 4);
        scanline++;
        len--;
      }
      rshift += 8;
    } else {
      scanline++;
      len--;
      rshift = 0;
    }
  }
  return true;
}
bool decrunch(RGBE* scanline, int len, Reader& f) {
  if (len < 8 || len > 0x7fff) return oldDecrunch(scanline, len, f, scanline);
  int i = f.getc();
  if (i != 2) {
    f.back();
    return oldDecrunch(scanline, len, f, scanline);
  }
  scanline[0][1] = (unsigned char)f.getc();
  scanline[0][2] = (unsigned char)f.getc();
  i = f.getc();
  if (scanline[0][1] != 2 || scanline[0][2] & 128) {
    scanline[0][0] = 2;
    scanline[0][3] = (unsigned char)i;
    return oldDecrunch(scanline + 1, len - 1, f, scanline);
  }
  for (i = 0; i < 4; i++) {
    for (int j = 0; j < len;) {
      unsigned char code = (unsigned char)f.getc();
      if (code > 128) {
        code &= 127;
        unsigned char val = (unsigned char)f.getc();
        while (code-- && j < len) scanline[j++][i] = val;
      } else {
        while (code-- && j < len) scanline[j++][i] = (unsigned char)f.getc();
      }
      if (f.eof) return false;
    }
  }
  return !f.eof;
}
}  // namespace

int pt_hdr_decode(const unsigned char* bytes, int64_t nbytes, int* w_out, int* h_out, float** cols_out) {
  if (!bytes || !w_out || !h_out || !cols_out) return -1;
  Reader f{bytes, nbytes};
  if (nbytes < 11 || std::memcmp(bytes, "#?RADIANCE", 10) != 0) return -6;
  f.pos = 11;
  int c = 0, oldc;
  while (true) {
    oldc = c;
    c = f.getc();
    if (c < 0) return -6;
    if (c == 0xa && oldc == 0xa) break;
  }
  std::string reso;
  while (true) {
    c = f.getc();
    if (c < 0) return -6;
    reso.push_back((char)c);
    if (c == 0xa) break;
  }
  int w = 0, h = 0;
  // hdrloader.cpp:68 uses "%ld" into int (an LP64 bug); parsed as int here.
  if (std::sscanf(reso.c_str(), "-Y %d +X %d", &h, &w) != 2 || w <= 0 || h <= 0) return -6;
  float* cols = (float*)std::calloc((size_t)w * h * 3, sizeof(float));
  if (!cols) return -5;
  std::vector<unsigned char> scan((size_t)w * 4);
  RGBE* scanline = reinterpret_cast<RGBE*>(scan.data());
  // convertComponent (hdrloader.cpp:99-104) = val/256 * (float)pow(2, expo):
  // the 256 possible scale factors are tabulated with the same expression
  float scale[256];
  for (int e = 0; e < 256; e++) scale[e] = (float)std::pow(2.0, (double)(e - 128));
  float* out = cols;
  for (int y = h - 1; y >= 0; y--) {
    if (!decrunch(scanline, w, f)) break;
    for (int k = 0; k < w; k++) {
      const float d = scale[scanline[k][3]];
      out[3 * k] = (scanline[k][0] / 256.0f) * d;
      out[3 * k + 1] = (scanline[k][1] / 256.0f) * d;
      out[3 * k + 2] = (scanline[k][2] / 256.0f) * d;
    }
    out += (size_t)w * 3;
  }
  *w_out = w;
  *h_out = h;
  *cols_out = cols;
  return 0;
}

int pt_hdr_load(const char* path, int* w, int* h, float** cols) {
  if (!path) return -1;
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return -6;
  std::vector<unsigned char> buf;
  unsigned char tmp[1 << 16];
  size_t k;
  while ((k = std::fread(tmp, 1, sizeof(tmp), fp)) > 0) buf.insert(buf.end(), tmp, tmp + k);
  std::fclose(fp);
  return pt_hdr_decode(buf.data(), (int64_t)buf.size(), w, h, cols);
}

void pt_free(void* p) { std::free(p); }

int pt_image_write_pfm(const char* path, const float* px, int w, int h, int channels) {
  if (!path || !px || w <= 0 || h <= 0 || (channels != 3 && channels != 4)) return -1;
  FILE* fp = std::fopen(path, "wb");
  if (!fp) return -6;
  std::fprintf(fp, "PF\n%d %d\n-1.0\n", w, h);
  std::vector<float> row((size_t)w * 3);
  bool ok = true;
  for (int y = 0; y < h && ok; y++) {
    const float* src = px + (size_t)y * w * channels;
    for (int x = 0; x < w; x++)
      for (int c = 0; c < 3; c++) row[(size_t)x * 3 + c] = src[(size_t)x * channels + c];
    ok = std::fwrite(row.data(), sizeof(float), row.size(), fp) == row.size();
  }
  return (std::fclose(fp) == 0 && ok) ? 0 : -6;
}

namespace {
uint32_t crc32_update(uint32_t crc, const unsigned char* p, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  for (size_t i = 0; i < n; i++) crc = table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return crc;
}
void put_be32(std::vector<unsigned char>& v, uint32_t x) {
  v.push_back((unsigned char)(x >> 24)); v.push_back((unsigned char)(x >> 16));
  v.push_back((unsigned char)(x >> 8)); v.push_back((unsigned char)x);
}
void png_chunk(std::vector<unsigned char>& out, const char* type, const std::vector<unsigned char>& data) {
  put_be32(out, (uint32_t)data.size());
  const size_t start = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), data.begin(), data.end());
  put_be32(out, crc32_update(0xffffffffu, out.data() + start, out.size() - start) ^ 0xffffffffu);
}
}  // namespace

int pt_image_write_png(const char* path, const float* px, int w, int h, int channels, float gamma, int flip_rows) {
  if (!path || !px || w <= 0 || h <= 0 || (channels != 3 && channels != 4) || w > (1 << 24)) return -1;
  // raw scanlines: filter byte 0 + RGB
  const size_t stride = (size_t)w * 3 + 1;
  std::vector<unsigned char> raw(stride * h);
  const double e = gamma > 0.0f ? (double)(1.0f / gamma) : 1.0;  // imshow: pow(double, 1.0f / 2.2f)
  for (int y = 0; y < h; y++) {
    const int sy = flip_rows ? h - 1 - y : y;
    const float* src = px + (size_t)sy * w * channels;
    unsigned char* dst = raw.data() + (size_t)y * stride;
    *dst++ = 0;
    for (int x = 0; x < w; x++)
      for (int c = 0; c < 3; c++) {
        double v = (double)src[(size_t)x * channels + c];
        double g = gamma > 0.0f ? std::pow(v, e) * 255.0 : v * 255.0;
        g = g < 0.0 ? 0.0 : (g > 255.0 ? 255.0 : g);  // clamp (NaN stays NaN -> 0 below)
        *dst++ = (unsigned char)(g == g ? g : 0.0);
      }
  }
  // zlib stream of stored deflate blocks (<= 65535 bytes each) + adler32
  std::vector<unsigned char> z = {0x78, 0x01};
  uint32_t a = 1, b = 0;
  for (size_t off = 0; off < raw.size() || raw.empty();) {
    const size_t n = std::min<size_t>(65535, raw.size() - off);
    const bool last = off + n >= raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back((unsigned char)(n & 0xff)); z.push_back((unsigned char)(n >> 8));
    z.push_back((unsigned char)(~n & 0xff)); z.push_back((unsigned char)((~n >> 8) & 0xff));
    for (size_t i = 0; i < n; i++) {
      const unsigned char c = raw[off + i];
      z.push_back(c);
      a = (a + c) % 65521u;
      b = (b + a) % 65521u;
    }
    off += n;
    if (last) break;
  }
  put_be32(z, (b << 16) | a);
  std::vector<unsigned char> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<unsigned char> ihdr;
  put_be32(ihdr, (uint32_t)w);
  put_be32(ihdr, (uint32_t)h);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit RGB, deflate, no filter, no interlace
  png_chunk(out, "IHDR", ihdr);
  png_chunk(out, "IDAT", z);
  png_chunk(out, "IEND", {});
  FILE* fp = std::fopen(path, "wb");
  if (!fp) return -6;
  const bool ok = std::fwrite(out.data(), 1, out.size(), fp) == out.size();
  return (std::fclose(fp) == 0 && ok) ? 0 : -6;
}

// calculateHdrCache (ImportanceSampling_LowDiscrepancySequence/main.cpp:555-652)
int pt_hdr_cache(const float* HDR, int width, int height, float* cache) {
  if (!HDR || !cache || width <= 0 || height <= 0) return -1;
  const size_t n = (size_t)width * height;
  std::vector<float> pdf(n);
  float lumSum = 0.0f;
  for (int i = 0; i < height; i++)
    for (int j = 0; j < width; j++) {
      size_t k = (size_t)i * width + j;
      float R = HDR[3 * k], G = HDR[3 * k + 1], B = HDR[3 * k + 2];
      float lum = (float)(0.2 * R + 0.7 * G + 0.1 * B);  // double literals in the reference
      pdf[k] = lum;
      lumSum += lum;
    }
  for (size_t k = 0; k < n; k++) pdf[k] /= lumSum;
  std::vector<float> margin((size_t)width, 0.0f);
  for (int j = 0; j < width; j++)
    for (int i = 0; i < height; i++) margin[j] += pdf[(size_t)i * width + j];
  std::vector<float> cdfx = margin;
  for (int j = 1; j < width; j++) cdfx[j] += cdfx[j - 1];
  std::vector<float> cdfy(n);  // [x][y]
  for (int j = 0; j < width; j++) {
    float* col = &cdfy[(size_t)j * height];
    for (int i = 0; i < height; i++) col[i] = pdf[(size_t)i * width + j] / margin[j];
    for (int i = 1; i < height; i++) col[i] += col[i - 1];
  }
  for (int j = 0; j < width; j++)
    for (int i = 0; i < height; i++) {
      float xi_1 = float(i) / height;
      float xi_2 = float(j) / width;
      int x = (int)(std::lower_bound(cdfx.begin(), cdfx.end(), xi_1) - cdfx.begin());
      int xr = x < width ? x : width - 1;  // reference indexes past the end here (UB)
      const float* col = &cdfy[(size_t)xr * height];
      int y = (int)(std::lower_bound(col, col + height, xi_2) - col);
      size_t k = (size_t)i * width + j;
      cache[3 * k] = float(x) / width;
      cache[3 * k + 1] = float(y) / height;
      cache[3 * k + 2] = pdf[k];
    }
  return 0;
}

}  // extern "C"
