// pt_accel.h -- internal (not part of the C ABI): the runtime's own
// acceleration tree over an uploaded scene, built by scene.cpp's threaded
// binned-SAH builder (the pt_scene_build_bvh code path).
#pragma once
#include <vector>

namespace pt {
// Binned-SAH tree over nTri triangles given as Triangle_encoded records (36 f32,
// only p1..p3 are read). nodes: reference node encoding (12 f32 per node, dummy
// node 0, root 1, leaf ranges into the built order); order[i] = the uploaded
// index of the triangle at built position i. Returns the tree depth, or -1.
int buildAccel(const float* tris, int nTri, int leafSize, std::vector<float>& nodes, std::vector<int>& order);
}  // namespace pt
