// ref_basic.cpp -- TEST INFRASTRUCTURE ONLY: runs the reference's own CPU path
// tracer (BasicRayTracingWithC++/main.cpp), compiled from its source, to make the
// golden images under tests/golden/basic/ (tests/golden/make_ref_fixtures.py).
//
// oracle/ref_build.py copies these line ranges of BasicRayTracingWithC++/main.cpp,
// unmodified, into oracle/_ref/ (never committed):
//   ref_basic_head.inc   :1-16     includes, using namespace glm / std
//   ref_basic_body.inc   :18-168   BRIGHTNESS, sizes, camera, colours, Ray, Material,
//                                  HitResult, Shape, Triangle, Sphere
//                        :191-297  shoot, dis / rd / gen / randf, randomVec3,
//                                  randomDirection, pathTracing
//   ref_basic_scene.inc  :306-357  main()'s scene and the zeroed double image
//   ref_basic_loop.inc   :361-432  main()'s sample / row / column loop
//   ref_basic_png.inc    :172-174, :179-187   imshow()'s 8-bit conversion
// What this file adds around them:
//   * SAMPLE (:17 hard-codes 128) comes from -DREF_SAMPLE: the reference's
//     author edited that constant per run; BRIGHTNESS (:20) follows it;
//   * gen (:210, seeded by random_device) is re-seeded to 5489 (std::mt19937's
//     default seed) before the loop, so a run is deterministic;
//   * :359-360 (omp_set_num_threads + the OpenMP pragma) are left out: the
//     shipped project does not enable /openmp (BasicRayTracingWithC++.vcxproj),
//     so the reference runs the loop serially -- and so does this build;
//   * imshow's file output (fopen_s / svpng, :176-177, :189) is replaced by
//     writing the double image and the 8-bit bytes to the given files.
//
//   ref_basic_s<N> <image.f64 (H*W*3 doubles, row 0 = top)> <image.u8 (H*W*3)>
#include <cstdio>
#include <cstring>  // memset (:357): MSVC's <iostream> brings it in, libstdc++'s does not

#include "_ref/ref_basic_head.inc"
const int SAMPLE = REF_SAMPLE;
#include "_ref/ref_basic_body.inc"

static unsigned char* ref_bytes(double* SRC) {
#include "_ref/ref_basic_png.inc"
  return image;
}

static double* ref_render() {
#include "_ref/ref_basic_scene.inc"
  gen.seed(5489u);
#include "_ref/ref_basic_loop.inc"
  return image;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s image.f64 image.u8\n", argv[0]);
    return 2;
  }
  double* img = ref_render();
  unsigned char* bytes = ref_bytes(img);
  FILE* a = std::fopen(argv[1], "wb");
  FILE* b = std::fopen(argv[2], "wb");
  if (!a || !b) return 1;
  std::fwrite(img, sizeof(double), (size_t)WIDTH * HEIGHT * 3, a);
  std::fwrite(bytes, 1, (size_t)WIDTH * HEIGHT * 3, b);
  std::fclose(a);
  std::fclose(b);
  return 0;
}
