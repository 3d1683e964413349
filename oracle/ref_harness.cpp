// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY: runs the reference's own host
// scene preparation, compiled from its sources, to make the golden fixtures
// under tests/golden/ref/ (tests/golden/make_ref_fixtures.py).
//
// oracle/ref_build.py copies these reference functions, by line range and
// unmodified, from /root/reference into oracle/_ref/ref_extract.inc (never
// committed) and compiles this file against the reference's vendored glm and
// GLEW headers (only GLEW's GL typedefs are used; nothing is linked from them):
//   OpenglRayTracing/main.cpp:20        INF
//   OpenglRayTracing/main.cpp:27-73     Material, Triangle, Triangle_encoded, BVHNode, BVHNode_encoded
//   OpenglRayTracing/main.cpp:151-166   cmpx / cmpy / cmpz
//   OpenglRayTracing/main.cpp:241-372   getTransformMatrix, readObj
//   OpenglRayTracing/main.cpp:374-551   buildBVH, buildBVHwithSAH
//   ImportanceSampling_LowDiscrepancySequence/main.cpp:554-652   calculateHdrCache
// What main() of OpenglRayTracing/main.cpp:646-716 does inline around them (the
// dummy node 0, the builder call, the encode) is restated below.
//
//   ref_harness scene <spec.txt> <sah|median|none> <tris.f32> <nodes.f32>
//       spec: one line per readObj call:
//       <obj path> <smooth 0/1> <rotate xyz> <translate xyz> <scale xyz> <16 material floats:
//        emissive.xyz baseColor.xyz subsurface metallic specular specularTint roughness
//        anisotropic sheen sheenTint clearcoat clearcoatGloss>   (IOR, transmission stay default)
//   ref_harness hdrcache <hdr.f32 (h*w*3)> <w> <h> <cache.f32>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include <GL/glew.h>
#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>

using namespace glm;

#include "_ref/ref_extract.inc"

namespace {

template <class T>
bool writeAll(const char* path, const std::vector<T>& v) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return false;
  const size_t n = v.empty() ? 0 : std::fwrite(v.data(), sizeof(T), v.size(), f);
  std::fclose(f);
  return n == v.size();
}

int scene(const char* specPath, const std::string& builder, const char* trisOut, const char* nodesOut) {
  std::ifstream spec(specPath);
  if (!spec) return 2;
  std::vector<Triangle> triangles;
  std::string line;
  while (std::getline(spec, line)) {
    std::istringstream in(line);
    std::string obj;
    int smooth = 1;
    float r[3], t[3], s[3], m[16];
    if (!(in >> obj >> smooth)) continue;
    for (float& x : r) in >> x;
    for (float& x : t) in >> x;
    for (float& x : s) in >> x;
    for (float& x : m) in >> x;
    if (!in) return 3;
    Material mat;
    mat.emissive = vec3(m[0], m[1], m[2]);
    mat.baseColor = vec3(m[3], m[4], m[5]);
    mat.subsurface = m[6];
    mat.metallic = m[7];
    mat.specular = m[8];
    mat.specularTint = m[9];
    mat.roughness = m[10];
    mat.anisotropic = m[11];
    mat.sheen = m[12];
    mat.sheenTint = m[13];
    mat.clearcoat = m[14];
    mat.clearcoatGloss = m[15];
    readObj(obj, triangles, mat, getTransformMatrix(vec3(r[0], r[1], r[2]), vec3(t[0], t[1], t[2]),
                                                    vec3(s[0], s[1], s[2])), smooth != 0);
  }
  // main.cpp:675-683 (the dummy node's index is left uninitialised there; 0 here)
  BVHNode testNode;
  testNode.left = 255;
  testNode.right = 128;
  testNode.n = 30;
  testNode.index = 0;
  testNode.AA = vec3(1, 1, 0);
  testNode.BB = vec3(0, 1, 0);
  std::vector<BVHNode> nodes{testNode};
  if (builder == "sah") buildBVHwithSAH(triangles, nodes, 0, (int)triangles.size() - 1, 8);
  else if (builder == "median") buildBVH(triangles, nodes, 0, (int)triangles.size() - 1, 8);
  else if (builder != "none") return 4;
  // main.cpp:688-716
  std::vector<Triangle_encoded> te(triangles.size());
  for (size_t i = 0; i < triangles.size(); i++) {
    const Triangle& tr = triangles[i];
    const Material& mm = tr.material;
    te[i].p1 = tr.p1; te[i].p2 = tr.p2; te[i].p3 = tr.p3;
    te[i].n1 = tr.n1; te[i].n2 = tr.n2; te[i].n3 = tr.n3;
    te[i].emissive = mm.emissive;
    te[i].baseColor = mm.baseColor;
    te[i].param1 = vec3(mm.subsurface, mm.metallic, mm.specular);
    te[i].param2 = vec3(mm.specularTint, mm.roughness, mm.anisotropic);
    te[i].param3 = vec3(mm.sheen, mm.sheenTint, mm.clearcoat);
    te[i].param4 = vec3(mm.clearcoatGloss, mm.IOR, mm.transmission);
  }
  std::vector<BVHNode_encoded> ne(builder == "none" ? 0 : nodes.size());
  for (size_t i = 0; i < ne.size(); i++) {
    ne[i].childs = vec3(nodes[i].left, nodes[i].right, 0);
    ne[i].leafInfo = vec3(nodes[i].n, nodes[i].index, 0);
    ne[i].AA = nodes[i].AA;
    ne[i].BB = nodes[i].BB;
  }
  static_assert(sizeof(Triangle_encoded) == 36 * sizeof(float), "Triangle_encoded layout");
  static_assert(sizeof(BVHNode_encoded) == 12 * sizeof(float), "BVHNode_encoded layout");
  return writeAll(trisOut, te) && writeAll(nodesOut, ne) ? 0 : 5;
}

int hdrcache(const char* in, int w, int h, const char* out) {
  std::vector<float> hdr((size_t)w * h * 3);
  FILE* f = std::fopen(in, "rb");
  if (!f) return 2;
  const size_t got = std::fread(hdr.data(), sizeof(float), hdr.size(), f);
  std::fclose(f);
  if (got != hdr.size()) return 3;
  float* cache = calculateHdrCache(hdr.data(), w, h);
  std::vector<float> c(cache, cache + (size_t)w * h * 3);
  delete[] cache;
  return writeAll(out, c) ? 0 : 5;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string cmd = argc > 1 ? argv[1] : "";
  if (cmd == "scene" && argc == 6) return scene(argv[2], argv[3], argv[4], argv[5]);
  if (cmd == "hdrcache" && argc == 6) return hdrcache(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), argv[5]);
  std::fprintf(stderr, "usage: ref_harness scene <spec> <sah|median|none> <tris> <nodes> | hdrcache <hdr> <w> <h> <out>\n");
  return 1;
}
