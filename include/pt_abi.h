/*
 * pt_abi.h -- C-ABI drop-in boundary of the MI355X progressive path tracer.
 *
 * The reference has no plugin/FFI API; its de-facto boundary is the GL
 * contract around pass1.draw() (OpenglRayTracing/main.cpp:558-603,
 * DisneyBRDF/main.cpp:558-603, ImportanceSampling_LowDiscrepancySequence/
 * main.cpp:659-709). Each entry point below replaces one piece of that
 * contract; the reference call it replaces is cited on each declaration.
 *
 * Conventions
 *  - Return codes: 0 = OK, negative = PT_E_* (no exit(), unlike the reference's
 *    exit(-1) at OpenglRayTracing/main.cpp:175,214,225,269).
 *  - The caller owns host arrays; the library owns device buffers.
 *  - One host thread per pt_ctx; calls are stream-ordered and synchronous on
 *    return unless the name ends in _async.
 *  - Images are row-major, row 0 = the bottom row (GL window coordinates,
 *    pass1.fsh pix.y) for the GL integrators, row 0 = the top row for
 *    PT_BASIC_CPU_COMPAT (BasicRayTracingWithC++/main.cpp:364-370).
 */
#ifndef PT_ABI_H
#define PT_ABI_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 7  /* 2: in-process multi-GPU fields at the end of pt_config / pt_frame_stats;
                             3: scene-upload fields at the end of pt_frame_stats, pt_build_bvh_device;
                             4: BASIC shapes as doubles, its double image, the replayed random stream;
                             5: the displayed frame of a screen-tile split (pt_display_*);
                             6: batches of frames (pt_render_frames_async, pt_config.frame_batch,
                                pt_frame_stats.frames), pt_config.hw_queues;
                             7: pt_unpack_ranks (every other rank's f32 gather in one launch);
                                PT_FLAG_WAVEFRONT retired; pt_frame_stats.env_compact, tree4_nodes */

/* error codes */
#define PT_OK 0
#define PT_E_INVALID -1      /* bad argument */
#define PT_E_HIP -2          /* HIP runtime error (see pt_last_error) */
#define PT_E_NOSCENE -3      /* render before pt_upload_scene */
#define PT_E_BADSCENE -4     /* malformed node / triangle arrays */
#define PT_E_NOMEM -5
#define PT_E_IO -6           /* file open / parse failure */
#define PT_E_NODEVICE -7     /* no HIP device / extension missing */

/* integrators (one per reference kernel variant) */
#define PT_LAMBERT_O 0            /* OpenglRayTracing/shaders/pass1.fsh: Lambert, uniform hemisphere, 2 bounces */
#define PT_DISNEY_UNIFORM_D 1     /* DisneyBRDF/shaders/pass1.fsh: aniso Disney, uniform hemisphere, 5 bounces */
#define PT_DISNEY_MIS_SOBOL_IS 2  /* ImportanceSampling_LowDiscrepancySequence/shaders/pass1.fsh: MIS + Sobol, 2 bounces */
#define PT_BASIC_CPU_COMPAT 3     /* BasicRayTracingWithC++/main.cpp: spheres+triangles, RR 0.8, depth 8 */

/* flags */
#define PT_FLAG_NO_CULL 0x1u      /* traverse exactly like pass1.fsh:335-382 (no closest-t culling) */
#define PT_FLAG_CLOSEST_SHADOW 0x2u /* env shadow rays use closest-hit instead of any-hit */
#define PT_FLAG_COUNT_FETCHES 0x4u /* count reference-algorithm fetches (implies NO_CULL, closest shadow) */
#define PT_FLAG_WAVEFRONT 0x8u    /* retired (round 5): the staged wavefront pipeline measured slower than the
                                     regen kernel on every config; pt_create rejects it (PT_E_INVALID) */
#define PT_FLAG_REGEN 0x10u       /* path-regeneration state-machine kernel instead of the megakernel */
#define PT_FLAG_NO_TILE_ORDER 0x20u /* megakernel: hand out tiles in fixed order, not longest-first */
#define PT_FLAG_REFERENCE_TREE 0x40u /* megakernel: traverse only the uploaded tree (not the runtime's own) */
#define PT_FLAG_SERIAL_FRAMES 0x80u /* megakernel: no frames in flight (each frame starts after the previous one ends) */
#define PT_FLAG_NO_BINS 0x100u    /* megakernel: camera rays walk the BVH (no per-tile camera-ray bins) */
#define PT_FLAG_PRIMARY_PASS 0x800u /* camera rays traced by a one-wave-per-tile pass (camera-ray bins) before
                                       the frame kernel instead of inside it: same images; the default for
                                       the large-scene regen kernel (c5 -9 %), slower for the megakernel
                                       on c2-c4. PT_FLAG_NO_BINS turns the pass off */
#define PT_FLAG_MEGAKERNEL 0x400u /* the lock-step megakernel instead of the path-regeneration kernel (4-wide
                                     walk with dynamic ray fetch, camera-ray pass) that large scenes (> 48 MB
                                     of records) and the Lambert integrator on any scene default to */
#define PT_FLAG_HOST_ACCEL 0x200u /* pt_upload_scene builds the runtime's own tree on the host (threaded binned
                                     SAH) instead of on the GPU (pt_build.hip) */

/* in-process multi-GPU (pt_config.n_devices > 1) */
#define PT_MAX_DEVICES 8
#define PT_GATHER_AUTO 0  /* RCCL send/recv when the devices are distinct and RCCL loads, else peer copies */
#define PT_GATHER_COPY 1  /* hipMemcpyPeerAsync of each device's packed tiles to the first device (xGMI) */
#define PT_GATHER_RCCL 2  /* RCCL send/recv group (ncclCommInitAll over device_ids); error if unavailable */

typedef struct pt_config {
  int width;          /* RenderPass::width  (OpenglRayTracing/main.cpp:83), e.g. 1920 */
  int height;         /* RenderPass::height (OpenglRayTracing/main.cpp:84), e.g. 1080 */
  int integrator;     /* PT_LAMBERT_O .. PT_BASIC_CPU_COMPAT */
  int max_bounce;     /* -1 = the reference's default for the integrator */
  int device_id;      /* HIP device ordinal */
  int tile_rank;      /* screen-tile shard owned by this context: tiles t with t % tile_world == tile_rank */
  int tile_world;     /* 1 = whole frame */
  int tile_size;      /* shard tile edge in pixels (0 = 32) */
  uint32_t flags;     /* PT_FLAG_* */
  int basic_samples;  /* PT_BASIC_CPU_COMPAT: SAMPLE (BasicRayTracingWithC++/main.cpp:17), 0 = 128 */
  uint32_t basic_seed;/* PT_BASIC_CPU_COMPAT: seed of the per-pixel counter RNG */
  int sample_rank;    /* sample-parallel rendering: this context draws the RNG/Sobol streams of   */
  int sample_world;   /* samples frameCounter*sample_world + sample_rank (0/1 = the reference's   */
                      /* frameCounter itself); the running-mean weight stays 1/(frameCounter+1)   */
  /* In-process multi-GPU: n_devices >= 2 makes this one context drive
   * device_ids[0..n_devices-1] (device_id is ignored; ids may repeat). Device k renders the
   * 32x32 screen tiles t with t % n_devices == k; every pt_render_frame then gathers the
   * other devices' tiles into device_ids[0]'s accumulation (gather = PT_GATHER_*), so the
   * context's image is bit-identical to a one-device render. tile_world and sample_world
   * must be <= 1 with n_devices >= 2. 0 or 1 = one device (device_id). */
  int n_devices;
  int device_ids[PT_MAX_DEVICES];
  int gather;
  /* ABI 6 */
  int frame_batch;    /* pt_render_frames_async: most frames per launch, at most 32 (0 = automatic:
                         2 x tile_world frames with the Lambert integrator, 4 x tile_world with
                         Disney/MIS, tile_world with Disney/MIS on scenes of more than 48 MB of
                         records -- 12 x / 16 x (32 x for MIS beyond 2 bounces) / 2 x when the hardware queues allow at most 3
                         frames in flight, e.g. HIP's default GPU_MAX_HW_QUEUES = 4) */
  int hw_queues;      /* hardware queues of the process's HIP runtime (GPU_MAX_HW_QUEUES in effect when
                         HIP initialised; bounds the frames in flight); 0 = read GPU_MAX_HW_QUEUES now */
} pt_config;

/* Counters accumulate over every launch since pt_create / pt_reset_stats. */
typedef struct pt_frame_stats {
  uint64_t rays;        /* hitBVH invocations (primary + BRDF + env shadow) */
  uint64_t node_fetch;  /* PT_FLAG_COUNT_FETCHES only: getBVHNode calls (48 B) */
  uint64_t tri_fetch;   /* PT_FLAG_COUNT_FETCHES only: getTriangle calls (72 B) */
  uint64_t mat_fetch;   /* PT_FLAG_COUNT_FETCHES only: getMaterial calls (72 B) */
  uint64_t tex_fetch;   /* PT_FLAG_COUNT_FETCHES only: texel reads (12 B) */
  float kernel_ms;      /* device time of the last render launch (HIP events on its stream) */
  float kernel_ms_total;/* summed device time of the render launches since the reset */
  int launches;         /* render launches since the reset */
  int max_stack;        /* traversal stack bound used (tree depth + 1) */
  int split_items;      /* megakernel: work items the next frame's schedule adds by splitting
                           long-path tiles (0 = one item per tile) */
  int runtime_tree;     /* megakernel: 1 when the last frame traversed the runtime's own tree
                           (results checked against the uploaded one), 0 the uploaded tree */
  int waves_per_simd;   /* megakernel: waves per SIMD the last frame's kernel was compiled for
                           (3 = the large-scene Disney/MIS variant, else its default bound) */
  int devices;          /* devices the context renders on (1, or pt_config.n_devices) */
  int gather;           /* PT_GATHER_COPY / PT_GATHER_RCCL in use (0 with one device) */
  int frames_in_flight; /* megakernel frames that may overlap (1 = serial; >1: kernel_ms of
                           overlapping launches add up to more than the wall time) */
  /* the last pt_upload_scene (kept across pt_reset_stats) */
  float upload_ms;      /* its wall time: host re-layout, copies and the runtime tree build */
  float accel_build_ms; /* wall time of the runtime tree's build (GPU, or host with PT_FLAG_HOST_ACCEL) */
  int accel_device;     /* 1: the runtime tree was built on the GPU, 0: on the host, -1: none */
  int accel_nodes;      /* the runtime tree's nodes (internal + leaves) */
  int accel_depth;      /* and its depth (root = 1) */
  int regen;            /* 1: the last frame ran the path-regeneration kernel (PT_FLAG_REGEN, or a large
                           Disney/MIS scene), 0: the lock-step megakernel */
  /* ABI 6 */
  int64_t frames;       /* frames rendered by the launches since the reset (a batch launch renders
                           several: pt_render_frames_async) */
  int frame_batch;      /* most frames per launch of this context (pt_config.frame_batch, resolved) */
  /* ABI 7 */
  int env_compact;      /* 1: the env is read from its compact texels (RGBE + pdf, 16-bit sample table),
                           which decode to the uploaded floats bit for bit; 2: and the sample table by
                           rows (a row record plus the distinct rows, equal entry by entry); 0: from
                           the float texels */
  int tree4_nodes;      /* 4-wide runtime-tree nodes (0: none) */
} pt_frame_stats;

typedef struct pt_ctx pt_ctx;

/* Device selection, resolution, integrator (replaces glutInit/glewInit/RenderPass
 * setup, OpenglRayTracing/main.cpp:639-644,749-768). */
int pt_create(pt_ctx** out, const pt_config* cfg);
void pt_destroy(pt_ctx* ctx);
const char* pt_last_error(pt_ctx* ctx);  /* ctx may be NULL: last create error */
int pt_device_count(int* n);
int pt_abi_version(void);  /* PT_ABI_VERSION of the loaded library */

/* Upload the encoded scene (replaces the two GL_RGB32F texture buffers,
 * OpenglRayTracing/main.cpp:720-735). tris = nTriangles x 36 f32 exactly as
 * Triangle_encoded (main.cpp:51-60); nodes = nNodes x 12 f32 exactly as
 * BVHNode_encoded (main.cpp:69-73) including the dummy node 0, root at 1. */
int pt_upload_scene(pt_ctx* ctx, const float* tris, int nTriangles, const float* nodes, int nNodes);

/* Upload the HDR environment (replaces hdrMap/hdrCache textures,
 * ImportanceSampling_LowDiscrepancySequence/main.cpp:843-853). hdr = w x h x 3
 * f32, row 0 = first scanline; cache = calculateHdrCache output (nullable: the
 * library computes it). hdrResolution := w. hdr == NULL clears the env (black). */
int pt_upload_env(pt_ctx* ctx, const float* hdr, int w, int h, const float* cache);

/* PT_BASIC_CPU_COMPAT shape list (the vector<Shape*> of BasicRayTracingWithC++/main.cpp:306-353):
 * n x 24 f64 records (layout in pt_scene.h; the reference's Material rates and sphere radius
 * are doubles, its vec3 fields floats). */
int pt_upload_shapes(pt_ctx* ctx, const double* shapes, int n);

/* PT_BASIC_CPU_COMPAT: the reference's `double* image` (BasicRayTracingWithC++/main.cpp:356,
 * summed by :427-429; row 0 = top), width x height x 3 f64 host buffer. The f32 accumulation
 * (pt_download_accum) holds the same sums rounded to float. */
int pt_download_basic_image(pt_ctx* ctx, double* rgb);
/* PT_BASIC_CPU_COMPAT checkpoint restore: the double image (as pt_download_basic_image wrote it);
 * the next frame adds its sample to it, bit for bit as if the frames had not been interrupted.
 * (pt_upload_accum on a BASIC context restores from the f32 sums: the double image is set to
 * them, widened.) */
int pt_upload_basic_image(pt_ctx* ctx, const double* rgb);

/* PT_BASIC_CPU_COMPAT: replay a recorded random stream instead of the per-pixel counter RNG,
 * so a frame consumes exactly the random numbers the reference's serial run consumed
 * (its one global std::mt19937 read by randf(), main.cpp:208-214). stream = n doubles in
 * draw order; offsets[(k * height + i) * width + j] = the stream position at which sample k
 * of pixel (row i from the top, column j) starts (n_offsets = samples * width * height; a
 * sample's draws end where the next one's start). A pixel sample that would read past its
 * end gets 0.5 and is counted (pt_basic_replay_overruns). stream == NULL switches back to
 * the counter RNG. Frame frameCounter renders sample k = frameCounter. */
int pt_set_basic_stream(pt_ctx* ctx, const double* stream, int64_t n, const int64_t* offsets, int64_t n_offsets);
int pt_basic_replay_overruns(pt_ctx* ctx, int64_t* count);

/* calculateHdrCache (ImportanceSampling_LowDiscrepancySequence/main.cpp:555-652)
 * computed on this context's GPU; output as pt_hdr_cache (w*h*3 f32: sample x,
 * sample y, pdf), bit-identical to it. pt_upload_env with cache = NULL uses it. */
int pt_hdr_cache_device(pt_ctx* ctx, const float* hdr, int w, int h, float* cache_out);

/* One display() (OpenglRayTracing/main.cpp:558-603): 1 spp per owned pixel and
 * the running-mean update of the device-resident accumulation (pass1.fsh:868-871);
 * frameCounter = 0 resets the mean (mix weight 1). eye[3]; cameraRotate[16]
 * column-major = inverse(lookAt(eye, 0, up)) (main.cpp:570-573). accum_rgba
 * (nullable) receives width x height x 4 f32 after the frame. For
 * PT_BASIC_CPU_COMPAT frameCounter is the sample index k and accum is the sum
 * buffer `image` (BasicRayTracingWithC++/main.cpp:356-431). */
int pt_render_frame(pt_ctx* ctx, const float eye[3], const float cameraRotate[16],
                    uint32_t frameCounter, float* accum_rgba);
/* Same without synchronising or downloading. */
int pt_render_frame_async(pt_ctx* ctx, const float eye[3], const float cameraRotate[16],
                          uint32_t frameCounter);
/* nFrames display() calls of one camera: frames frameCounter .. frameCounter + nFrames - 1, each
 * 1 spp per owned pixel with its own running-mean update (bit for bit nFrames calls of
 * pt_render_frame_async). Consecutive frames are rendered side by side in one launch (up to
 * pt_config.frame_batch; while the tree / split policies are being measured, one each) and
 * their running-mean updates applied together, pixel by pixel in frame order; the accumulation
 * holds the last frame's mean when the call's work completes (a frame in between is not
 * materialised in it). Without synchronising. */
int pt_render_frames_async(pt_ctx* ctx, const float eye[3], const float cameraRotate[16],
                           uint32_t frameCounter, int nFrames);

/* The GPU binned-SAH builder (pt_build.hip), exposed as a scene
 * builder in the reference's node encoding -- the role of buildBVH / buildBVHwithSAH
 * (OpenglRayTracing/main.cpp:376-551), with pt_scene.h PT_BVH_BINNED_SAH's split rule.
 * tris = nTriangles x 36 f32 (Triangle_encoded; only p1..p3 are read). Writes
 * *nNodes_out nodes (12 f32 each: dummy node 0, root 1, leaves of <= leafSize
 * triangles whose ranges index the built order) to nodes_out when they fit in
 * max_nodes (else PT_E_INVALID, *nNodes_out still set), and order_out[i] = the input
 * index of the triangle at built position i (nTriangles ints). */
int pt_build_bvh_device(pt_ctx* ctx, const float* tris, int nTriangles, int leafSize, float* nodes_out,
                        int max_nodes, int* nNodes_out, int* order_out);

/* Batch hitBVH (pass1.fsh:335-382; BVH/main.cpp:571 debug-ray query). rays =
 * n x 6 f32 (origin, direction); miss -> t = 2147483648.f, tri = -1. */
int pt_trace_closest(pt_ctx* ctx, const float* rays, int n, float* t_out, int* tri_out);

/* Accumulation buffer access (lastFrame texture, main.cpp:763-764). */
int pt_download_accum(pt_ctx* ctx, float* accum_rgba);   /* host or device memory, width*height*4 f32 */
int pt_upload_accum(pt_ctx* ctx, const float* accum_rgba);
int pt_clear_accum(pt_ctx* ctx);
int pt_accum_device_ptr(pt_ctx* ctx, void** dptr); /* width*height*4 f32, device memory */

/* pass3.fsh tonemap c / (1 + (0.3r+0.6g+0.1b)/limit) of the accumulation,
 * optional gamma (pass3.fsh:14-24 keeps it commented out: gamma <= 0). rgb_out
 * = width x height x 3 f32 host buffer. */
int pt_tonemap(pt_ctx* ctx, float limit, float gamma, float* rgb_out);

/* Multi-process tile exchange (one process per GPU, pt_config.tile_rank/tile_world):
 * pack this rank's owned pixels into a contiguous device buffer (count =
 * pt_owned_pixel_count slots of 3 f32: r, g, b -- a rendered pixel's alpha is
 * always 1, and unpack writes 1), and unpack another rank's packed pixels into this
 * context's accumulation. Pointers are device memory; the caller moves the
 * packed buffers (RCCL gather over xGMI). Not for n_devices > 1 contexts, which
 * gather inside pt_render_frame. */
int pt_owned_pixel_count(pt_ctx* ctx, int rank, int world, int64_t* count);
int pt_pack_owned(pt_ctx* ctx, void* dpacked);
int pt_unpack_rank(pt_ctx* ctx, int rank, int world, const void* dpacked);
/* pt_unpack_rank of ranks 1..world-1 in one launch (dpacked[k] = rank k's packed buffer, [0] unused,
 * a NULL entry is skipped; world <= 16): rank 0's reassembly after a gather of the running means. */
int pt_unpack_ranks(pt_ctx* ctx, int world, const void* const* dpacked);

/* The displayed frame (pass3.fsh:14-24 drawn into the 8-bit GLUT_RGBA window,
 * ImportanceSampling_LowDiscrepancySequence/main.cpp:706,747): tonemap (and gamma > 0)
 * of the accumulation, stored as round(clamp(x, 0, 1) * 255) per channel, alpha 255.
 * A screen-tile split presents every frame from 3 bytes per pixel instead of the
 * accumulation's 12: each rank packs its owned pixels' display values
 * (pt_display_pack: pt_owned_pixel_count slots of 3 u8, packed order as pt_pack_owned),
 * the caller moves them to rank 0 (RCCL gather over xGMI), and rank 0 writes its own
 * tiles (pt_display_own) and the other ranks' (pt_display_unpack: dpacked[k] = rank k's
 * packed buffer for k = 1..world-1, world <= 16, one launch) into one width x height
 * RGBA8 device image. With tile_world 1, pt_display_own writes every pixel. All on the
 * context's current stream, after the frames rendered so far; device pointers (work
 * another stream queued on those buffers is not ordered before it: set that stream
 * with pt_set_stream, or synchronise it first). */
int pt_display_pack(pt_ctx* ctx, float limit, float gamma, void* dpacked);
int pt_display_own(pt_ctx* ctx, float limit, float gamma, void* dimage);
int pt_display_unpack(pt_ctx* ctx, int world, const void* const* dpacked, void* dimage);

/* Stream interop: render on the caller's HIP stream (e.g. torch's current
 * stream). NULL restores the context's own stream. */
int pt_set_stream(pt_ctx* ctx, void* hip_stream);
int pt_synchronize(pt_ctx* ctx);
int pt_get_stats(pt_ctx* ctx, pt_frame_stats* stats);   /* synchronises the stream */
int pt_reset_stats(pt_ctx* ctx);

/* Diagnostics: evaluate one include/pt_fmath.h function (0 sin, 1 cos, 2 atan2(x,y),
 * 3 asin, 4 log, 5 exp, 6 pow(x,y)) over n inputs on the host CPU or on the
 * context's GPU; the two must agree bit for bit. */
int pt_fmath_host(int fn, const float* x, const float* y, int n, float* out);
int pt_fmath_device(pt_ctx* ctx, int fn, const float* x, const float* y, int n, float* out);

#ifdef __cplusplus
}
#endif
#endif /* PT_ABI_H */
