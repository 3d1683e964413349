// abi_caller.cpp -- a compiled reference-side caller of the C ABI (test infrastructure).
//
// What a maintainer of the reference would write when dropping libpt.so into
// DisneyBRDF/main.cpp: the host keeps its own scene preparation up to
// the encoded arrays (here read from files, standing in for the Triangle_encoded /
// BVHNode_encoded vectors main() builds at DisneyBRDF/main.cpp:750-777), then
//   main():    pt_create -> pt_upload_scene (replaces the texture-buffer uploads :780-796)
//              -> pt_hdr_load + pt_upload_env(cache = NULL) (replaces HDRLoader::load + hdrMap, :800-804;
//                 the library computes calculateHdrCache, ImportanceSampling.../main.cpp:555-652)
//   display(): the camera of :569-573 (pt_orbit_camera = inverse(lookAt(eye, 0, up))), then
//              pt_render_frame(..., frameCounter++) in place of pass1.draw(); pass2.draw() (:574-599)
//              and pt_tonemap in place of pass3.draw() (:600), once per frame
//   BVH/main.cpp:566-575: the debug ray from (0, 0, 1) along normalize(0.1, -0.1, -0.7) through
//              pt_trace_closest (hitBVH as a query)
// Built with g++ against include/pt_abi.h and include/pt_scene.h only, linked with -lpt.
//
//   abi_caller --version                      print the loaded library's PT_ABI_VERSION (no GPU)
//   abi_caller DIR INTEGRATOR W H FRAMES [ROTATE UP R]
//     reads  DIR/tris.f32 (nTri x 36 f32), DIR/nodes.f32 (nNodes x 12 f32), DIR/env.hdr (Radiance)
//     writes DIR/accum.f32 (H x W x 4 f32 running mean), DIR/rgb.f32 (H x W x 3 f32, pass3),
//            DIR/debug_ray.txt ("tri t" of the debug ray), DIR/stats.txt ("rays frames")
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pt_abi.h"
#include "pt_scene.h"

static bool readFloats(const std::string& path, std::vector<float>& out) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize((size_t)n / sizeof(float));
  const size_t got = std::fread(out.data(), sizeof(float), out.size(), f);
  std::fclose(f);
  return got == out.size();
}

static bool writeFloats(const std::string& path, const float* p, size_t n) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  const size_t put = std::fwrite(p, sizeof(float), n, f);
  std::fclose(f);
  return put == n;
}

#define CHECK(call)                                                                       \
  do {                                                                                    \
    const int rc_ = (call);                                                               \
    if (rc_ != PT_OK) {                                                                   \
      std::fprintf(stderr, "%s failed: %d %s\n", #call, rc_, pt_last_error(g_pt));       \
      return 2;                                                                           \
    }                                                                                     \
  } while (0)

static pt_ctx* g_pt = nullptr;

int main(int argc, char** argv) {
  if (argc == 2 && std::strcmp(argv[1], "--version") == 0) {
    std::printf("%d\n", pt_abi_version());
    return pt_abi_version() == PT_ABI_VERSION ? 0 : 1;
  }
  if (argc < 6) {
    std::fprintf(stderr, "usage: abi_caller DIR INTEGRATOR W H FRAMES [ROTATE UP R]\n");
    return 1;
  }
  const std::string dir = argv[1];
  pt_config cfg;
  std::memset(&cfg, 0, sizeof(cfg));
  cfg.width = std::atoi(argv[3]);
  cfg.height = std::atoi(argv[4]);
  cfg.integrator = std::atoi(argv[2]);  // PT_DISNEY_UNIFORM_D for DisneyBRDF/, PT_LAMBERT_O, PT_DISNEY_MIS_SOBOL_IS
  cfg.max_bounce = -1;                  // the shader's own default
  cfg.device_id = 0;
  cfg.tile_rank = 0;
  cfg.tile_world = 1;
  const int frames = std::atoi(argv[5]);
  const float rotateAngle = argc > 6 ? (float)std::atof(argv[6]) : 0.0f;  // DisneyBRDF/main.cpp globals
  const float upAngle = argc > 7 ? (float)std::atof(argv[7]) : 0.0f;
  const float r = argc > 8 ? (float)std::atof(argv[8]) : 4.0f;

  std::vector<float> tris, nodes;
  if (!readFloats(dir + "/tris.f32", tris) || !readFloats(dir + "/nodes.f32", nodes)) {
    std::fprintf(stderr, "cannot read the encoded scene in %s\n", dir.c_str());
    return 1;
  }
  if (pt_create(&g_pt, &cfg) != PT_OK) {
    std::fprintf(stderr, "pt_create: %s\n", pt_last_error(nullptr));
    return 2;
  }
  CHECK(pt_upload_scene(g_pt, tris.data(), (int)(tris.size() / 36), nodes.data(), (int)(nodes.size() / 12)));
  int hw = 0, hh = 0;
  float* cols = nullptr;
  CHECK(pt_hdr_load((dir + "/env.hdr").c_str(), &hw, &hh, &cols));
  CHECK(pt_upload_env(g_pt, cols, hw, hh, nullptr));  // cache = NULL: calculateHdrCache on the device
  pt_free(cols);

  // display(), frame after frame (frameCounter++ is the uniform of :579)
  std::vector<float> rgb((size_t)cfg.width * cfg.height * 3);
  unsigned int frameCounter = 0;
  for (int f = 0; f < frames; f++) {
    float eye[3], cameraRotate[16];
    pt_orbit_camera(rotateAngle, upAngle, r, eye, cameraRotate);
    CHECK(pt_render_frame(g_pt, eye, cameraRotate, frameCounter++, nullptr));
    CHECK(pt_tonemap(g_pt, 1.5f, 0.0f, rgb.data()));  // pass3.fsh:14-24
  }
  std::vector<float> accum((size_t)cfg.width * cfg.height * 4);
  CHECK(pt_download_accum(g_pt, accum.data()));

  // BVH/main.cpp:566-575: one debug ray through hitBVH
  const float dx = 0.1f, dy = -0.1f, dz = -0.7f;
  const float inv = 1.0f / std::sqrt(dx * dx + dy * dy + dz * dz);
  const float ray[6] = {0.0f, 0.0f, 1.0f, dx * inv, dy * inv, dz * inv};
  float t = 0.0f;
  int tri = -2;
  CHECK(pt_trace_closest(g_pt, ray, 1, &t, &tri));

  pt_frame_stats st;
  CHECK(pt_get_stats(g_pt, &st));
  pt_destroy(g_pt);

  if (!writeFloats(dir + "/accum.f32", accum.data(), accum.size()) || !writeFloats(dir + "/rgb.f32", rgb.data(), rgb.size()))
    return 1;
  FILE* f = std::fopen((dir + "/debug_ray.txt").c_str(), "w");
  if (!f) return 1;
  std::fprintf(f, "%d %.9g\n", tri, (double)t);
  std::fclose(f);
  f = std::fopen((dir + "/stats.txt").c_str(), "w");
  if (!f) return 1;
  std::fprintf(f, "%llu %lld\n", (unsigned long long)st.rays, (long long)st.frames);
  std::fclose(f);
  std::printf("abi_caller ok: %d frames, debug ray tri %d t %.9g, rays %llu\n", frames, tri, (double)t,
              (unsigned long long)st.rays);
  return 0;
}
