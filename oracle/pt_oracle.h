/*
 * pt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference path tracer's per-pixel hot path, used as
 * the parity checker for the HIP kernels and as the CPU baseline in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so. The product (opengl_ray_tracing_amd/) never links it.
 *
 * Parity pinning (see DESIGN.md "Oracle"): the GLSL kernels cannot execute in
 * this container (no GL context, no GPU), so this restatement is pinned
 * piecewise: Sobol table verbatim (pass1.fsh:92-94), wang hash (pass1.fsh:78-85),
 * BVH traversal == brute force (the reference's own switch, pass1.fsh:853-854),
 * HDR decode statistics recorded in SURVEY.md section 8(c), and the reference's
 * shipped CPU-tracer images (BasicRayTracingWithC++/{200spp,4000spp}.png, statistical).
 * Transcendental ulp behaviour of the GL driver is "parity unpinned".
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Integrator ids: identical to include/pt_abi.h */
#define ORC_LAMBERT_O 0          /* OpenglRayTracing/shaders/pass1.fsh */
#define ORC_DISNEY_UNIFORM_D 1   /* DisneyBRDF/shaders/pass1.fsh */
#define ORC_DISNEY_MIS_SOBOL_IS 2 /* ImportanceSampling_LowDiscrepancySequence/shaders/pass1.fsh */
#define ORC_BASIC_CPU_COMPAT 3   /* BasicRayTracingWithC++/main.cpp */

typedef struct orc_scene {
  const float* tris;   /* nTriangles x 36 f32 (Triangle_encoded, OpenglRayTracing/main.cpp:51-60) */
  int nTriangles;
  const float* nodes;  /* nNodes x 12 f32 (BVHNode_encoded, OpenglRayTracing/main.cpp:69-73) */
  int nNodes;
  const float* hdr;    /* hdrW x hdrH x 3 f32, row 0 = first scanline (nullable = black env) */
  const float* cache;  /* calculateHdrCache output, same dims (nullable) */
  int hdrW, hdrH;
  int hdrResolution;   /* uniform hdrResolution (IS main.cpp:853: = width) */
  /* BASIC_CPU_COMPAT shape list (nShapes x ORC_SHAPE_DOUBLES) */
  const double* shapes;
  int nShapes;
} orc_scene;

/* BASIC shape record layout (doubles; include/pt_scene.h PT_SHAPE_DOUBLES) */
#define ORC_SHAPE_DOUBLES 24
/* [0]=type (0 triangle, 1 sphere) [1..3]=p1 or sphere centre [4..6]=p2 [7..9]=p3
 * [10..12]=color [13..15]=normal (triangle: normalize(cross(p2-p1,p3-p1)))
 * [16]=isEmissive [17]=specularRate [18]=roughness [19]=refractRate
 * [20]=refractAngle [21]=refractRoughness [22]=sphere radius [23]=pad
 * The vec3 fields hold float values (glm vec3), the rates and the radius the
 * reference's doubles (Material: BasicRayTracingWithC++/main.cpp:49-59; shapes :78-165) */

typedef struct orc_frame {
  int width, height;
  int integrator;
  int maxBounce;            /* -1 = reference default (O:2, D:5, IS:2, BASIC depth 8) */
  uint32_t frameCounter;
  float eye[3];
  float cameraRotate[16];   /* column-major (glm value_ptr order) */
  int basicSamples;         /* BASIC: SAMPLE (BasicRayTracingWithC++/main.cpp:17) */
  uint32_t basicSeed;       /* BASIC: per-run seed of the counter RNG */
  int sampleRank, sampleWorld; /* RNG/Sobol sample = frameCounter*sampleWorld + sampleRank (0/0 = frameCounter);
                                  the running-mean weight stays 1/(frameCounter+1) (pt_abi.h pt_config) */
  double* basicImage;       /* BASIC: the reference's double image (width x height x 3, B:356), summed in
                               place (frameCounter 0 starts it); accum receives it as float */
} orc_frame;

typedef struct orc_counters {
  /* fetch counts of the reference algorithm */
  uint64_t rays;      /* hitBVH invocations (primary + BRDF + env shadow) */
  uint64_t nodes;     /* getBVHNode calls       (48 B each) */
  uint64_t tris;      /* getTriangle calls      (72 B each) */
  uint64_t mats;      /* getMaterial calls      (72 B each) */
  uint64_t texels;    /* hdrMap/hdrCache/lastFrame reads (12 B each) */
} orc_counters;

/* Render the listed pixels (px, py pairs; py from the bottom for the GL
 * integrators, row-from-top for BASIC) of one frame. accum is the full
 * width x height x 4 f32 running-mean buffer, read and written in place
 * (pass1.fsh:868-871). Multi-threaded with OpenMP when nthreads > 1.
 * pix == NULL renders every pixel. Returns 0 on success. */
int orc_render_pixels(const orc_scene* s, const orc_frame* f, const int* pix, int nPix,
                      float* accum, int nthreads, orc_counters* counters);

/* BasicRayTracingWithC++/main.cpp run as shipped: one global std::mt19937 seeded
 * with `seed`, the sample / row / column loop B:361-432 serially. image: W x H x 3
 * doubles (row 0 = top). offsets (nullable, samples x H x W): the stream position
 * (number of randf() draws before) at which each pixel sample starts; *nDraws the
 * total. This is what the reference binary computes, byte for byte
 * (tests/golden/basic/, test_basic_serial_equals_reference). */
int orc_basic_serial(const orc_scene* s, int W, int H, int samples, uint32_t seed, int maxDepth, double* image,
                     int64_t* offsets, int64_t* nDraws, orc_counters* counters);
/* The reference's randf() stream (B:208-214) from std::mt19937(seed): n doubles. */
int orc_mt_doubles(uint32_t seed, int64_t n, double* out);

/* Batch hitBVH (pass1.fsh:335-382): rays n x 6 (origin, direction). Miss: t = INF
 * (2147483648.f), tri = -1. brute != 0 uses hitArray over all triangles
 * (pass1.fsh:854, the reference's own differential switch). */
int orc_trace_closest(const orc_scene* s, const float* rays, int n, float* t_out, int* tri_out,
                      int brute, orc_counters* counters);

/* Debug: RNG / Sobol / CP value dumps for integer parity (bit-exact). */
uint32_t orc_wang_hash(uint32_t seed);
float orc_sobol(uint32_t d, uint32_t i);
void orc_pixel_rng(int px, int py, uint32_t frameCounter, int n, float* out);

/* Per-function parity hook: function fn (0..24, the layout of oracle/ref_glsl.cpp
 * ref_glsl_fn) on n inputs. */
int orc_glsl_fn(int fn, const float* in, float* out, int n);

/* calculateHdrCache restatement (IS main.cpp:555-652): cache_out w*h*3. */
int orc_hdr_cache(const float* hdr, int w, int h, float* cache_out);

#ifdef __cplusplus
}
#endif
#endif
