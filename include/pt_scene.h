/*
 * pt_scene.h -- host-side scene preparation (C ABI), the CPU half of the
 * reference's host surface that feeds pt_upload_scene / pt_upload_env.
 *
 * Everything here runs on the host and needs no GPU. Each function restates
 * one reference routine, cited on its declaration, with the reference's
 * numerical quirks kept (readObj AABB typo, SAH z-typo) unless a *_FIXED /
 * binned variant is asked for explicitly.
 */
#ifndef PT_SCENE_H
#define PT_SCENE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Material (OpenglRayTracing/main.cpp:27-42), defaults as there. */
typedef struct pt_material {
  float emissive[3];
  float baseColor[3];
  float subsurface, metallic, specular, specularTint, roughness, anisotropic;
  float sheen, sheenTint, clearcoat, clearcoatGloss, IOR, transmission;
} pt_material;

void pt_material_default(pt_material* m);

/* BVH builders */
#define PT_BVH_REFERENCE_SAH 0 /* buildBVHwithSAH (main.cpp:430-551), z-typo at :480,484 kept */
#define PT_BVH_REFERENCE_MEDIAN 1 /* buildBVH (main.cpp:376-427) */
#define PT_BVH_FIXED_SAH 2     /* buildBVHwithSAH with the z-typo fixed */
#define PT_BVH_BINNED_SAH 3    /* O(n log n) 32-bin SAH, same node encoding */

typedef struct pt_scene pt_scene;

int pt_scene_create(pt_scene** out);
void pt_scene_destroy(pt_scene* s);

/* readObj (OpenglRayTracing/main.cpp:261-372) from a file or an in-memory text. */
int pt_scene_read_obj(pt_scene* s, const char* path, const pt_material* m, const float trans[16], int smoothNormal);
int pt_scene_read_obj_text(pt_scene* s, const char* text, const pt_material* m, const float trans[16], int smoothNormal);
/* Same pipeline (normalise by the typo'd AABB, transform, normals) from arrays:
 * verts nv x 3 f32 as parsed, idx nTri x 3 zero-based. */
int pt_scene_add_mesh(pt_scene* s, const float* verts, int nv, const int* idx, int nTri,
                      const pt_material* m, const float trans[16], int smoothNormal);
int pt_scene_num_triangles(const pt_scene* s);

/* Build the BVH over all triangles (reorders triangles, as the reference does).
 * Node 0 is the reference's dummy node (main.cpp:675-681), root = 1. */
int pt_scene_build_bvh(pt_scene* s, int builder, int leafSize);
int pt_scene_num_nodes(const pt_scene* s);
int pt_scene_depth(const pt_scene* s);
/* Encode (main.cpp:687-716): tris_out nTri x 36 f32, nodes_out nNodes x 12 f32. */
int pt_scene_encode(const pt_scene* s, float* tris_out, float* nodes_out);

/* getTransformMatrix (main.cpp:242-258), glm conventions, column-major out. */
void pt_transform_matrix(const float rotateDeg[3], const float translate[3], const float scale[3], float out[16]);
/* display() camera (main.cpp:569-573): eye on a sphere of radius r, and
 * cameraRotate = inverse(lookAt(eye, 0, (0,1,0))), column-major. */
void pt_orbit_camera(float rotateAngleDeg, float upAngleDeg, float r, float eye[3], float cameraRotate[16]);

/* Radiance .hdr decode (hdrloader.cpp:29-191; LP64-safe). *cols is malloc'd
 * (w*h*3 f32, row 0 = first scanline); free with pt_free. */
int pt_hdr_load(const char* path, int* w, int* h, float** cols);
int pt_hdr_decode(const unsigned char* bytes, int64_t nbytes, int* w, int* h, float** cols);
void pt_free(void* p);
/* calculateHdrCache (ImportanceSampling_LowDiscrepancySequence/main.cpp:555-652). */
int pt_hdr_cache(const float* hdr, int w, int h, float* cache_out);

/* BASIC_CPU_COMPAT shape records, 24 f64 each (BasicRayTracingWithC++/main.cpp:42-165):
 * [0] type (0 triangle, 1 sphere), [1..3] p1 or sphere centre, [4..6] p2, [7..9] p3,
 * [10..12] color, [13..15] triangle normal normalize(cross(p2-p1, p3-p1)) (:85),
 * [16] isEmissive, [17] specularRate, [18] roughness, [19] refractRate,
 * [20] refractAngle, [21] refractRoughness, [22] sphere radius, [23] unused.
 * The vec3 fields hold float values (glm vec3), the rates and the radius doubles. */
#define PT_SHAPE_DOUBLES 24

/* Image output. The GL demos only display; BasicRayTracingWithC++ writes its
 * image with imshow + svpng (main.cpp:169-190). pixels: h rows of w pixels of
 * `channels` (3 or 4; alpha is dropped) f32, row 0 first.
 * PFM ("PF", little-endian): linear values, rows written in stored order, which
 * PFM reads bottom-to-top -- the accumulation's row 0 is the bottom (GL).
 * PNG (8-bit RGB, uncompressed deflate like svpng): each component
 * (unsigned char)clamp(pow(v, 1/gamma) * 255, 0, 255) in double as imshow does
 * (gamma <= 0: no gamma); flip_rows writes the last row first (GL -> image). */
int pt_image_write_pfm(const char* path, const float* pixels, int w, int h, int channels);
int pt_image_write_png(const char* path, const float* pixels, int w, int h, int channels, float gamma,
                       int flip_rows);

#ifdef __cplusplus
}
#endif
#endif /* PT_SCENE_H */
