// pt_runtime.cpp -- host implementation of the C-ABI in include/pt_abi.h:
// device selection, scene/env upload with the MI355X re-layout, frame
// launches, batch queries, accumulation access and multi-GPU tile pack.
//
// Compiled with -ffp-contract=off so the per-triangle unit normal and plane
// offset precomputed here round exactly like the reference computes them
// inline (pass1.fsh:263, :273).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <map>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pt_abi.h"
#include "pt_accel.h"
#include "pt_fmath.h"
#include "pt_kernels.h"
#include "pt_rccl.h"
#include "pt_scene.h"

using namespace pt;

static constexpr int EV_RING = 64;
// Frames in flight: the default megakernel's (or regen kernel's) launch g (its pipeline
// sequence number) runs on slot stream g % depth (8 by default) with its own work queues,
// overflow stack, tile order and camera-ray results, and writes its sample colours to colour
// buffer g % (2 * depth + 1). While k other launches are in flight its persistent grid is 1.5 /
// (k + 1) of residency (renderOne), so the frames in flight share the GPU by space: their waves
// are resident together, and a frame whose last long paths keep a few waves busy leaves the
// rest of the machine to the others. Its running-mean update (mixKernel) runs on the caller's
// stream, in frame order, once the launch's kernel has ended: the accumulation is updated in
// frame order, the image is bit for bit the one of serial frames, and whatever the caller
// queues behind a frame (pack, download, tonemap) follows its update with no further
// cross-queue wait. No launch waits for a mix except the one of the launch 2 * depth + 1 back,
// whose colour buffer it reuses.
//
// A launch may render a batch of consecutive frames of one camera (pt_render_frames_async,
// RenderParams::nFrames): every frame's colours in its own part of the colour buffer, and one
// mixKernel folds them into the running mean pixel by pixel in frame order. A small screen-tile
// share (1/8 of the image) gives one frame too little work to fill the machine; a batch of
// tile_world frames per launch is about one whole image's work, and the chain of running-mean
// updates on the caller's stream -- one cross-queue wait and one launch per update, which set
// an 8-way share's frame period before -- has one link per batch.
// (Measured alternatives, DESIGN.md 4: a separate mix stream is twice as slow at small
// shares -- each mix waited on two ~25 us cross-queue signals in a chain from mix to mix; and
// with full-residency grids a mix waits for a CU slot behind the next frame's persistent
// kernel, ~250 us on c2, which made deeper pipelines slower, not faster.)
#ifndef PT_PIPE
#define PT_PIPE 8  // frames in flight (PT_PIPE_DEPTH overrides; capped by the hardware queues)
#endif
static constexpr int PIPE = MAX_SLOTS;      // most frames in flight
// 32: c2's 1/8 share in the 20-frame bench window at 4 hardware queues 0.0417 -> 0.0351 ms per
// frame (its 20 frames one launch instead of 16 + 4), 1/4 share 0.0593 -> 0.0569, c4 0.2736 -> 0.2701
#ifndef PT_MAX_BATCH
#define PT_MAX_BATCH 32
#endif
static constexpr int MAX_BATCH = PT_MAX_BATCH;  // most frames per launch (pt_render_frames_async)
// colour buffers: a launch reuses the buffer of the launch 2 * depth + 1 back, whose running-mean
// update is then long done -- with depth + 1 the wait made a slot's next frame follow the
// running-mean update of the previous frame on another slot (two cross-queue hops), and an N = 8
// share of c2 kept only ~3 of its 8 frames in flight
static constexpr int COLS = 2 * MAX_SLOTS + 1;
// a launch of one frame while nothing else is in flight mixes its samples into the running mean in
// its own kernels (renderOne: no colour buffer, no mixKernel launch)
#ifndef PT_DIRECT_SOLO
#define PT_DIRECT_SOLO 1
#endif
// a single frame launched while nothing else is in flight (a display() call) runs on the megakernel
#ifndef PT_CALL_MEGAKERNEL
#define PT_CALL_MEGAKERNEL 1
#endif
static_assert(PT_PIPE >= 1 && PT_PIPE <= PIPE, "PT_PIPE: 1..MAX_SLOTS");
static_assert(PIPE * NUM_QUEUES * CTL_LINE_INTS * 4 <= (int)CTL_STATS, "queue counters of every slot fit the control block");

#ifndef PT_TILE_GROUP
#define PT_TILE_GROUP 1  // tiles ordered by cost in groups of this many consecutive tiles (1 measured best)
#endif


struct pt_ctx {
  pt_config cfg{};
  std::string err;
  hipStream_t own = nullptr, stream = nullptr;
  // Launch timing: a fixed ring of begin/end event pairs. Launch number i (since
  // pt_create) records into pair i % EV_RING; a launch's elapsed time is folded
  // into the running totals once its end event has completed (non-blocking on
  // every new launch, blocking only when the ring is full or stats are read), so
  // the cost per frame stays constant however long a caller renders.
  hipEvent_t ev[2 * EV_RING] = {};
  int evProbe[EV_RING] = {};    // probe slot of the launch in each ring position (-1 none)
  int evGen[EV_RING] = {};      // probe generation it was tagged in
  long long issued = 0, folded = 0;
  double msTotal = 0.0;         // summed device time of the folded launches since the reset
  float msLast = 0.0f;          // device time of the last folded launch
  int launches = 0;             // render launches since the reset
  long long frames = 0;         // frames those launches rendered (a batch launch renders several)
  int tagSlot = -1;             // probe slot for the launch being issued (probePolicy)
  int numCU = 0;
  // scene
  float4* d_geo = nullptr;
  float4* d_pairs = nullptr;  // triangles i and i+1 component-interleaved (SceneView::pairs)
  float4* d_hit = nullptr;   // per triangle: normals + material id (SceneView::hitRec)
  float4* d_mats = nullptr;  // the distinct materials (SceneView::mats)
  int nMats = 0;
  float4* d_bvh = nullptr;
  int nDevNodes = 0;  // internal nodes in d_bvh (device ids 0..nDevNodes-1)
  // the runtime's own tree (uploadAccel; SceneView::fast) and the reference
  // facts its results are checked against
  bool fastReady = false;
  float4* d_fbvh = nullptr;
  float4* d_fpairs = nullptr;
  int* d_fastTri = nullptr;
  int* d_refParent = nullptr;
  float4* d_refBox = nullptr;
  float4* d_leafBox = nullptr;
  int fRoot = REF_NONE, fnDev = 0, fDepth = 0;
  // the same tree collapsed to 4-wide nodes (encodeWide4; the large-scene regen kernel)
  float4* d_fbvh4 = nullptr;
  bool fast4Ready = false;
  int f4Root = REF_NONE, f4nDev = 0, f4Depth = 0;
  // the last pt_upload_scene (pt_frame_stats upload_ms, accel_*)
  float uploadMs = 0.0f, accelMs = 0.0f;
  int accelDevice = -1, accelNodes = 0, accelDepth = 0;
  int rootRef = REF_NONE;
  int nTri = 0, nNodes = 0, depth = 0, maxStack = 0;
  // env
  float4* d_hdr = nullptr;
  float2* d_cache = nullptr;  // sample table (x, y); the pdf lives in d_hdr[k].w
  uint2* d_hdr8 = nullptr;    // the same texels compacted (pt_kernels.h Env), null = not exact
  uint32_t* d_cache4 = nullptr;
  uint32_t* d_cacheRow = nullptr;           // the sample table by rows (pt_kernels.h Env::cacheRow)
  unsigned short* d_cacheY = nullptr;
  float2* d_trig = nullptr;                  // SampleHdr's sines and cosines (Env::trig)
  uint2* d_light = nullptr;                  // each sample-table entry's light-sample color and pdf (Env::light)
  int hdrW = 0, hdrH = 0;
  // BASIC shapes, the double image, the replayed random stream
  double* d_shapes = nullptr;
  int nShapes = 0;
  double* d_basicImg = nullptr;
  double* d_stream = nullptr;
  long long* d_offsets = nullptr;
  long long streamN = 0, nOffsets = 0;
  unsigned long long* d_overruns = nullptr;
  // frame state
  float4* d_accum = nullptr;
  // control block (pt_kernels.h CTL_*): padded queue counters (zeroed per
  // launch), cumulative fetch stats, padded sharded cumulative ray counters
  unsigned char* d_ctl = nullptr;
  int* d_ovf = nullptr;
  int* d_cost = nullptr;   // per slot: per-tile cost of its last frame, longest item, split state, estimate
  int* d_order = nullptr;  // per slot: per-band work items for its next frame
  bool lastFast = false;    // the last megakernel frame traversed the runtime's tree
  bool lastRegen = false;   // the last frame ran the path-regeneration kernel
  int lastWaves = 0;        // waves per SIMD of the last megakernel launch (occupancy query)
  // tree / tile-split policy probe (probePolicy): frames since the probe (re)started,
  // the summed frame times of each policy, the decision
  int probeFrame = 0;
  // camera-ray bins (pt_primary.hip) of the camera and scene they were built for
  PrimaryBins bins;
  bool binsValid = false;
  float binEye[3] = {}, binCam[16] = {};
  unsigned sceneVersion = 0, binVersion = 0;
  // frames in flight (PIPE slots; see PIPE above)
  bool pipe = false;                        // this context pipelines its megakernel frames
  int pipeDepth = PT_PIPE;                  // frames in flight (slot streams in use), 1..PIPE
  int pipeDepthBase = PT_PIPE;              // ... as chosen at creation (uploadScene may lower it for large scenes)
  bool pipeDepthFixed = false;              // PT_PIPE_DEPTH set: no scene-dependent choice
  // Frames of one pt_render_frames_async call rendered per launch (RenderParams::nFrames), at most:
  // pt_config.frame_batch, else as many as make one launch about a whole image's work (tile_world
  // frames of a screen-tile share, up to MAX_BATCH). Probe frames and frameCounter 0 run alone.
  int batchCap = 1;
  int colCap[COLS] = {};                    // frames each colour buffer holds
  int primCap[PIPE] = {};                   // frames each slot's camera-ray results hold
  // the large-scene path (regen kernel at 4 waves/SIMD, 4-wide walk with dynamic ray fetch,
  // camera-ray pass) on scenes of any size: -1 = for the Lambert integrator (c2 0.342 ->
  // 0.251 ms/frame) and the MIS integrator at 2 bounces (round 5: c3 0.1443 -> 0.1331; c4's 8
  // bounces keep the megakernel); PT_FLAG_REGEN / PT_FLAG_MEGAKERNEL choose per context,
  // PT_REGEN_WIDE = 1 / 0 (environment) for every / no scene
  int regenWide = -1;
  bool solo = true;                         // PT_SOLO = 0 (environment): every pipelined launch on a slot stream
  hipStream_t slotStream[PIPE] = {};
  hipEvent_t kernelDone[PIPE] = {};         // slot's last frame kernel (+ reorder) ended
  bool slotBusy[PIPE] = {};                 // kernelDone[k] has been recorded since the last sync
  hipEvent_t mixDone[COLS] = {};            // colour buffer's last running-mean update
  hipStream_t lastMixStream = nullptr;      // the stream the last update ran on (pt_set_stream may change it)
  // camera-ray bins built on one slot's stream: binsBuilt is recorded after the build, and
  // every other slot waits for it once before its first frame with those bins (binGen)
  hipEvent_t binsBuilt = nullptr;
  unsigned binGen = 0, binGenSeen[MAX_SLOTS] = {};
  float* d_col[COLS] = {};                  // per-colour-buffer sample colours (COL_F floats per slot)
  int2* d_prim[PIPE] = {};                  // per-slot camera-ray results (primaryKernel)
  int lastSlot = -1;                        // slot of the last pipelined frame
  int lastCol = -1;                         // colour buffer of the last pipelined frame
  bool mixPending = false;                  // a pipelined frame's update may still be running
  unsigned long long frameNo = 0;           // pipelined frames issued
  int probeN[4] = {0, 0, 0, 0};        // timed frames: runtime tree, uploaded tree (both unsplit), split
  double probeMs[4] = {0.0, 0.0, 0.0, 0.0};
  long long probeLast[4] = {-1, -1, -1, -1};  // launch number of each slot's last timed frame
  int probeGen = 0;
  int treeDecided = -1, splitDecided = -1;  // -1 probing, 0 off, 1 on
  unsigned policyKey = 0, probedKey = ~0u;  // bumped by every scene / env upload; the key the decisions were made for
  int orderCap = 0;        // work items per band in d_order
  bool orderValid[PIPE] = {};
  bool orderSplit[PIPE] = {};               // the slot's order list holds split items (a one-frame launch built it)
  size_t ovfInts = 0;
  // shards
  int shardSize = 32, shardsX = 0, shardsY = 0, numItems = 0, perQueue = 0;
  // scratch for queries / tonemap / pack
  float* d_rays = nullptr;
  float* d_t = nullptr;
  int* d_tri = nullptr;
  size_t traceCap = 0;
  float* d_rgb = nullptr;
  // in-process multi-GPU (pt_config.n_devices > 1): this context renders as
  // screen-tile rank 0 on device_ids[0] and owns the other ranks' contexts and
  // the per-frame gather of their tiles into its accumulation
  std::vector<pt_ctx*> peers;  // ranks 1 .. n_devices-1
  struct GroupGather* gather = nullptr;
};

// The per-frame gather of an in-process device group. Rank k >= 1 packs its
// tiles (packKernel) on its render stream into one of two send buffers; the
// packed tiles travel to rank 0's device -- an RCCL send/recv group over the
// communicator of all the devices, or hipMemcpyPeerAsync -- and are unpacked
// into rank 0's accumulation on rank 0's communication stream. Rank 0's next
// frame renders meanwhile (its own tiles only); a send buffer is packed again
// only after its previous transfer completed.
struct GroupGather {
  int mode = PT_GATHER_COPY;
  int n = 0;
  hipStream_t cstream = nullptr;  // rank 0's device: receives, copies, unpacks
  hipEvent_t done = nullptr;      // rank 0's device: the last frame's unpacks
  bool pending = false;
  unsigned frame = 0;
  struct Peer {
    int dev = 0;
    size_t count = 0;                       // packed pixels (float4) of this rank
    float* send[2] = {nullptr, nullptr};    // on the rank's device, PACK_F floats per slot
    float* recv = nullptr;                  // on rank 0's device
    hipStream_t mstream = nullptr;          // the rank's device: RCCL sends
    hipEvent_t packed[2] = {nullptr, nullptr};
    hipEvent_t sent[2] = {nullptr, nullptr};  // the buffer's transfer completed
    bool sentValid[2] = {false, false};
  };
  std::vector<Peer> peer;  // ranks 1 .. n-1
  ncclComm_t comms[PT_MAX_DEVICES] = {};
  bool commsReady = false;
};

static std::string g_create_err;

#define CK(expr)                                                                     \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) {                                                          \
      ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);                  \
      return PT_E_HIP;                                                               \
    }                                                                                \
  } while (0)

static int fail(pt_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

template <class T>
static void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

template <class T>
static int upload(pt_ctx* ctx, T** dst, const std::vector<T>& src) {
  dfree(*dst);
  if (src.empty()) return PT_OK;
  CK(hipMalloc(dst, src.size() * sizeof(T)));
  CK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return PT_OK;
}

extern "C" {

int pt_device_count(int* n) {
  if (!n) return PT_E_INVALID;
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  *n = c;
  return PT_OK;
}

const char* pt_last_error(pt_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

// Frames per launch of pt_render_frames_async: pt_config.frame_batch, else whole images' work per
// launch in multiples of tile_world frames, at most MAX_BATCH:
//  * 2 x for the Lambert regen kernel -- one image's is enough to fill the machine, the second
//    halves the launches and running-mean updates per frame: c2 0.244 -> 0.231 ms per frame at
//    N = 1, c2's 1/8 share 0.0354 -> 0.0344 (profiles/r4); 3 and 4 measured no better;
//  * 4 x for the megakernel (Disney/MIS on small scenes), whose longest-first launches end in their
//    longest tiles: c4 at N = 1 0.2566 -> 0.2531 ms per frame over 200 frames and 0.3288 -> 0.2860
//    over 20 from an idle GPU, N = 2 0.139 -> 0.131, N = 4 / 8 equal (profiles/r4/batch_c4/);
//  * 1 x on large Disney/MIS scenes, whose frames are long already (c5 5.66 ms at 1, 5.86 at 2).
// With few hardware queues (GPU_MAX_HW_QUEUES 4, HIP's default and the GPU box's: 2 frames in flight)
// a launch takes more frames, so that about as much work is in flight: Lambert 8 x, Disney/MIS 16 x,
// large scenes 2 x (round 5, 4 queues, the driver's 20-frame bench window from an idle GPU: c2 at
// 2 / 4 / 6 / 8 / 12 / 16 frames per launch 0.218 / 0.196 / 0.187 / 0.184 / 0.178 / 0.184 ms per
// frame; c4 at 4 / 8 / 16 0.342 / 0.302 / 0.271; c5 at 1 / 2 4.59 / 4.34; c2's shares at 20 frames,
// N = 2 / 4 / 8, at 2 x N 0.116 / 0.066 / 0.041 and 4 x N 0.107 / 0.060 / 0.041 ms).
static int defaultBounce(int integ);

static int batchFor(const pt_ctx* ctx, bool wideScene) {
  const pt_config& c = ctx->cfg;
  if (c.frame_batch > 0) return std::min(c.frame_batch, MAX_BATCH);
  const bool fewQueues = ctx->pipeDepth <= 3;
#ifndef PT_BATCH_LAMBERT
#define PT_BATCH_LAMBERT 12  // c2, 20 frames: 8 + 8 + 4 -> 12 + 8, 0.1789-0.1802 -> 0.1707-0.1729 ms (10: 0.1949); 200 frames equal
#endif
#ifndef PT_BATCH_MIS
#define PT_BATCH_MIS 16
#endif
#ifndef PT_BATCH_MIS_MK
// MIS beyond its shader's 2 bounces renders on the megakernel (c4): 32 frames per launch, c4 0.2599
// -> 0.2327 ms over 20 frames (one launch instead of 16 + 4), 0.2389 -> 0.2303 over 100; the MIS
// regen kernel (c3) keeps 16 (24 / 32: 0.1107 -> 0.1122 / 0.1148)
#define PT_BATCH_MIS_MK 32
#endif
  const int mb = c.max_bounce >= 0 ? c.max_bounce : defaultBounce(c.integrator);
  const int mis = c.integrator == 2 && mb > 2 ? PT_BATCH_MIS_MK : PT_BATCH_MIS;
  const int m = wideScene ? (fewQueues ? 2 : 1) : c.integrator == 0 ? (fewQueues ? PT_BATCH_LAMBERT : 2) : (fewQueues ? mis : 4);
  return std::max(1, std::min(m * std::max(1, c.tile_world), MAX_BATCH));
}

static int createOne(pt_ctx** out, const pt_config* cfg) {
  if (!out || !cfg) return PT_E_INVALID;
  *out = nullptr;
  // width, height < 65536: the megakernel packs a pixel as (px | py << 16)
  if (cfg->width <= 0 || cfg->height <= 0 || cfg->width > 65535 || cfg->height > 65535 || cfg->integrator < 0 ||
      cfg->integrator > PT_BASIC_CPU_COMPAT ||
      cfg->tile_world < 1 || cfg->tile_rank < 0 || cfg->tile_rank >= cfg->tile_world || cfg->sample_world < 0 ||
      cfg->sample_rank < 0 || cfg->sample_rank >= (cfg->sample_world > 0 ? cfg->sample_world : 1)) {
    g_create_err = "pt_create: invalid config";
    return PT_E_INVALID;
  }
  if (cfg->flags & PT_FLAG_WAVEFRONT) {  // retired in round 5; git history keeps it
    g_create_err = "pt_create: invalid config: PT_FLAG_WAVEFRONT (the staged wavefront pipeline) was retired";
    return PT_E_INVALID;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    g_create_err = "pt_create: no HIP device";
    return PT_E_NODEVICE;
  }
  if (cfg->device_id < 0 || cfg->device_id >= ndev) {
    g_create_err = "pt_create: device_id out of range";
    return PT_E_INVALID;
  }
  pt_ctx* ctx = new (std::nothrow) pt_ctx();
  if (!ctx) return PT_E_NOMEM;
  ctx->cfg = *cfg;
  if (ctx->cfg.basic_samples <= 0) ctx->cfg.basic_samples = 128;
  int ss = cfg->tile_size > 0 ? cfg->tile_size : 32;
  if (ss % 8 != 0) {
    delete ctx;
    g_create_err = "pt_create: tile_size must be a multiple of 8";
    return PT_E_INVALID;
  }
  ctx->shardSize = ss;
  auto bail = [&](int code) {
    g_create_err = ctx->err;
    pt_destroy(ctx);
    return code;
  };
#define CKC(expr)                                                     \
  do {                                                                \
    hipError_t e_ = (expr);                                           \
    if (e_ != hipSuccess) {                                           \
      ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);   \
      return bail(PT_E_HIP);                                          \
    }                                                                 \
  } while (0)
  CKC(hipSetDevice(cfg->device_id));
  hipDeviceProp_t prop;
  CKC(hipGetDeviceProperties(&prop, cfg->device_id));
  ctx->numCU = prop.multiProcessorCount;
  CKC(hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking));
  ctx->stream = ctx->own;
  const size_t npix = (size_t)cfg->width * cfg->height;
  CKC(hipMalloc(&ctx->d_accum, npix * sizeof(float4)));
  CKC(hipMemset(ctx->d_accum, 0, npix * sizeof(float4)));
  CKC(hipMalloc(&ctx->d_ctl, CTL_BYTES));
  CKC(hipMemset(ctx->d_ctl, 0, CTL_BYTES));
  ctx->shardsX = (cfg->width + ss - 1) / ss;
  ctx->shardsY = (cfg->height + ss - 1) / ss;
  const int numShards = ctx->shardsX * ctx->shardsY;
  const int owned = (numShards - cfg->tile_rank + cfg->tile_world - 1) / cfg->tile_world;
  ctx->numItems = owned * (ss / 8) * (ss / 8);
  ctx->perQueue = (ctx->numItems + NUM_QUEUES - 1) / NUM_QUEUES;
  // the default megakernel and the regen kernel pipeline their frames (not BASIC, the fetch
  // counter or PT_FLAG_SERIAL_FRAMES)
  // the path-regeneration kernel with the 4-wide walk for every integrator on any scene
  // (PT_REGEN_WIDE = 1; 0: never; unset: Lambert frames and large Disney/MIS scenes)
  if (const char* e = std::getenv("PT_REGEN_WIDE")) ctx->regenWide = std::atoi(e) != 0 ? 1 : 0;
  if (const char* e = std::getenv("PT_SOLO")) ctx->solo = std::atoi(e) != 0;
  ctx->pipe = cfg->integrator != PT_BASIC_CPU_COMPAT &&
              !(cfg->flags & (PT_FLAG_COUNT_FETCHES | PT_FLAG_SERIAL_FRAMES));
  if (ctx->pipe) {
    // a process has the hardware queues its HIP runtime was initialised with (GPU_MAX_HW_QUEUES,
    // HIP's default 4; the Python package asks for 12 when it is unset and HIP not yet initialised,
    // and passes what is in effect as pt_config.hw_queues): streams beyond them share queues and
    // serialise, so the slot streams, the context's own stream and the caller's (torch's) must fit
    int hwq = cfg->hw_queues;
    if (hwq <= 0) {
      const char* q = std::getenv("GPU_MAX_HW_QUEUES");
      hwq = q && std::atoi(q) > 0 ? std::atoi(q) : 4;
    }
    ctx->pipeDepth = std::min(ctx->pipeDepth, std::max(2, hwq - 2));
    // Whole Lambert frames (the regen kernel on every scene): 6 in flight. c2's bench line (20 frames
    // from an idle GPU) 0.254-0.257 ms per frame at 6 vs 0.259-0.277 at 8 and 0.259 at 4, 100 frames
    // 0.232 either way; the MIS megakernel keeps 8 (c4 0.366 at 8 vs 0.373-0.397 at 6, 0.41 at 4),
    // and so do screen-tile shares (c2's 1/8 share 0.061 at 8 vs 0.074 at 6)
    if (cfg->integrator == 0 && ctx->regenWide != 0 && cfg->tile_world <= 1) ctx->pipeDepth = std::min(ctx->pipeDepth, 6);
    if (const char* e = std::getenv("PT_PIPE_DEPTH")) {
      ctx->pipeDepth = std::min(PIPE, std::max(1, std::atoi(e)));
      ctx->pipeDepthFixed = true;
    }
    ctx->pipeDepthBase = ctx->pipeDepth;
    ctx->batchCap = batchFor(ctx, false);
    // slot streams are created as a depth first uses them (ensureSlots). (Created here instead,
    // before the context's own stream and the caller's, they take hardware queues of their own even
    // at GPU_MAX_HW_QUEUES = 4 -- created later they share one -- but c2's shares measured slower
    // that way in the 20-frame window, N = 2 / 4 / 8: 0.1091 / 0.0638 / 0.0439 -> 0.1164 / 0.0701 /
    // 0.0478 ms: the next launch's camera-ray pass then competes with the running launch's tail.)
    for (int k = 0; k < COLS; k++) CKC(hipEventCreateWithFlags(&ctx->mixDone[k], hipEventDisableTiming));
    CKC(hipEventCreateWithFlags(&ctx->binsBuilt, hipEventDisableTiming));
  }
#undef CKC
  *out = ctx;
  return PT_OK;
}

static void destroyGroup(pt_ctx* ctx);
static int createGroup(pt_ctx* ctx);

int pt_create(pt_ctx** out, const pt_config* cfg) {
  if (!out || !cfg) return PT_E_INVALID;
  *out = nullptr;
  const int n = cfg->n_devices;
  if (n < 0 || n > PT_MAX_DEVICES || cfg->gather < PT_GATHER_AUTO || cfg->gather > PT_GATHER_RCCL) {
    g_create_err = "pt_create: n_devices must be 0..8 and gather a PT_GATHER_* value";
    return PT_E_INVALID;
  }
  if (n <= 1) return createOne(out, cfg);
  if (cfg->tile_world > 1 || cfg->sample_world > 1 || cfg->integrator == PT_BASIC_CPU_COMPAT) {
    g_create_err = "pt_create: n_devices > 1 renders screen tiles of the GL integrators itself "
                   "(tile_world and sample_world must be <= 1)";
    return PT_E_INVALID;
  }
  // rank k: device_ids[k], screen tiles t % n == k
  pt_config c = *cfg;
  c.n_devices = 0;
  c.tile_world = n;
  c.tile_rank = 0;
  c.device_id = cfg->device_ids[0];
  int rc = createOne(out, &c);
  if (rc) return rc;
  pt_ctx* ctx = *out;
  ctx->cfg.n_devices = n;
  for (int k = 1; k < n; k++) {
    c.tile_rank = k;
    c.device_id = cfg->device_ids[k];
    pt_ctx* p = nullptr;
    if ((rc = createOne(&p, &c)) != PT_OK) {
      pt_destroy(ctx);
      *out = nullptr;
      return rc;
    }
    ctx->peers.push_back(p);
  }
  if ((rc = createGroup(ctx)) != PT_OK) {
    g_create_err = ctx->err;
    pt_destroy(ctx);
    *out = nullptr;
    return rc;
  }
  return PT_OK;
}

void pt_destroy(pt_ctx* ctx) {
  if (!ctx) return;
  destroyGroup(ctx);
  (void)hipSetDevice(ctx->cfg.device_id);
  if (ctx->own) (void)hipStreamSynchronize(ctx->own);
  dfree(ctx->d_geo); dfree(ctx->d_hit); dfree(ctx->d_mats); dfree(ctx->d_bvh); dfree(ctx->d_pairs);
  dfree(ctx->d_fbvh); dfree(ctx->d_fbvh4); dfree(ctx->d_fpairs); dfree(ctx->d_fastTri);
  dfree(ctx->d_refParent); dfree(ctx->d_refBox); dfree(ctx->d_leafBox);
  dfree(ctx->d_hdr); dfree(ctx->d_cache); dfree(ctx->d_hdr8); dfree(ctx->d_cache4); dfree(ctx->d_shapes);
  dfree(ctx->d_cacheRow); dfree(ctx->d_cacheY); dfree(ctx->d_trig); dfree(ctx->d_light);
  dfree(ctx->d_basicImg); dfree(ctx->d_stream); dfree(ctx->d_offsets); dfree(ctx->d_overruns);
  dfree(ctx->d_accum); dfree(ctx->d_ctl); dfree(ctx->d_ovf); dfree(ctx->d_cost); dfree(ctx->d_order);
  dfree(ctx->d_rays); dfree(ctx->d_t); dfree(ctx->d_tri); dfree(ctx->d_rgb);
  freePrimaryBins(ctx->bins);
  for (int k = 0; k < PIPE; k++) {
    if (ctx->slotStream[k]) (void)hipStreamSynchronize(ctx->slotStream[k]);
    dfree(ctx->d_prim[k]);
    if (ctx->kernelDone[k]) (void)hipEventDestroy(ctx->kernelDone[k]);
    if (ctx->slotStream[k]) (void)hipStreamDestroy(ctx->slotStream[k]);
  }
  for (int k = 0; k < COLS; k++) {
    dfree(ctx->d_col[k]);
    if (ctx->mixDone[k]) (void)hipEventDestroy(ctx->mixDone[k]);
  }
  if (ctx->binsBuilt) (void)hipEventDestroy(ctx->binsBuilt);
  for (hipEvent_t e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  delete ctx;
}

// ------------------------------------------------------------ scene upload
static inline void nrm3(const float* a, const float* b, const float* c, float N[3]) {
  // normalize(cross(p2 - p1, p3 - p1)), glm order (oracle: hitTriangle)
  float e1x = b[0] - a[0], e1y = b[1] - a[1], e1z = b[2] - a[2];
  float e2x = c[0] - a[0], e2y = c[1] - a[1], e2z = c[2] - a[2];
  float cx = e1y * e2z - e2y * e1z;
  float cy = e1z * e2x - e2z * e1x;
  float cz = e1x * e2y - e2x * e1y;
  float inv = 1.0f / std::sqrt((cx * cx + cy * cy) + cz * cz);
  N[0] = cx * inv; N[1] = cy * inv; N[2] = cz * inv;
}

// A tree in the reference node encoding (12 f32 per node, dummy node 0, root 1)
// re-laid out as device wide nodes (pt_kernels.h SceneView::bvh). inflate > 0
// widens every box outward by that relative amount plus inflateAbs (the
// runtime's own tree: conservative, so a ray that hits a triangle always enters
// its boxes).
struct WideTree {
  std::vector<float4> bvh;
  int rootRef = REF_NONE, nDev = 0, depth = 0;
};

static std::string encodeWideTree(const float* nodes, int nNodes, int nTri, float inflate, WideTree& out,
                                  float inflateAbs = 0.0f) {
  auto nodeN = [&](int k) { return (int)nodes[(size_t)k * 12 + 3]; };
  auto isInternal = [&](int k) { return k > 0 && k < nNodes && nodeN(k) <= 0; };
  // depth of the reachable tree (bounds the traversal stack; rejects cycles)
  int depth = 0;
  {
    std::vector<std::pair<int, int>> st{{1, 1}};
    long visits = 0;
    while (!st.empty()) {
      auto [k, d] = st.back();
      st.pop_back();
      if (++visits > 2L * nNodes) return "node graph is not a tree (cycle)";
      depth = std::max(depth, d);
      if (nodeN(k) > 0) continue;
      int L = (int)nodes[(size_t)k * 12 + 0], R = (int)nodes[(size_t)k * 12 + 1];
      if (L > 0 && L < nNodes) st.push_back({L, d + 1});
      if (R > 0 && R < nNodes) st.push_back({R, d + 1});
    }
  }
  // Device ids of the reachable internal nodes: the first LDS_NODES in
  // breadth-first order from the root (the top of the tree, which every ray
  // walks: the megakernel stages exactly these ids in LDS), the rest in the
  // tree's id order (the reference's preorder, which keeps subtrees together).
  // Only the storage order changes; traversal visits the same nodes in the same
  // order.
  std::vector<int> newId(nNodes, -1), order;
  {
    std::vector<char> reach(nNodes, 0);
    std::vector<int> bfs;
    if (isInternal(1)) { bfs.push_back(1); reach[1] = 1; }
    for (size_t h = 0; h < bfs.size(); h++) {
      const int k = bfs[h];
      for (int c = 0; c < 2; c++) {
        const int ch = (int)nodes[(size_t)k * 12 + c];
        if (isInternal(ch) && !reach[ch]) { reach[ch] = 1; bfs.push_back(ch); }
      }
    }
    for (size_t h = 0; h < bfs.size() && h < (size_t)LDS_NODES; h++) order.push_back(bfs[h]);
    for (int k : order) newId[k] = -2;
    for (int k = 1; k < nNodes; k++)
      if (reach[k] && newId[k] == -1) order.push_back(k);
    for (size_t i = 0; i < order.size(); i++) newId[order[i]] = (int)i;
  }
  std::string bad;
  // node references (ivec3(texelFetch) truncation, pass1.fsh:238-243)
  auto encodeRef = [&](int k) -> int {
    if (k <= 0 || k >= nNodes) return REF_NONE;
    int n = nodeN(k);
    if (n > 0) {
      int index = (int)nodes[(size_t)k * 12 + 4];
      if (index < 0 || (long)index + n > nTri) { bad = "leaf range out of bounds at node " + std::to_string(k); return REF_NONE; }
      if (n > MAX_LEAF) { bad = "leaf larger than 32 triangles at node " + std::to_string(k); return REF_NONE; }
      return (int)~(((uint32_t)index << LEAF_CNT_BITS) | (uint32_t)(n - 1));
    }
    return newId[k];
  };
  auto widen = [&](float4& lo, float4& hi) {
    if (inflate <= 0.0f && inflateAbs <= 0.0f) return;
    const float e[3] = {inflate * (std::fabs(lo.x) + std::fabs(hi.x) + (hi.x - lo.x)) + inflateAbs + 1e-30f,
                        inflate * (std::fabs(lo.y) + std::fabs(hi.y) + (hi.y - lo.y)) + inflateAbs + 1e-30f,
                        inflate * (std::fabs(lo.z) + std::fabs(hi.z) + (hi.z - lo.z)) + inflateAbs + 1e-30f};
    lo.x -= e[0]; lo.y -= e[1]; lo.z -= e[2];
    hi.x += e[0]; hi.y += e[1]; hi.z += e[2];
  };
  std::vector<float4>& bvh = out.bvh;
  bvh.assign(std::max<size_t>(order.size(), 1) * 4, make_float4(0, 0, 0, 0));
  const float inf = INFINITY;
  for (size_t id = 0; id < order.size(); id++) {
    const int k = order[id];
    int L = (int)nodes[(size_t)k * 12 + 0], R = (int)nodes[(size_t)k * 12 + 1];
    int lr = encodeRef(L), rr = encodeRef(R);
    if (!bad.empty()) return bad;
    float4 la = make_float4(inf, inf, inf, 0), lb = make_float4(-inf, -inf, -inf, 0);
    float4 ra = la, rb = lb;
    if (lr != REF_NONE) {
      const float* c = nodes + (size_t)L * 12;
      la = make_float4(c[6], c[7], c[8], 0); lb = make_float4(c[9], c[10], c[11], 0);
      widen(la, lb);
    }
    if (rr != REF_NONE) {
      const float* c = nodes + (size_t)R * 12;
      ra = make_float4(c[6], c[7], c[8], 0); rb = make_float4(c[9], c[10], c[11], 0);
      widen(ra, rb);
    }
    // children paired per component (left, right) so one packed op serves both boxes
    float refs[2];
    std::memcpy(&refs[0], &lr, 4);
    std::memcpy(&refs[1], &rr, 4);
    bvh[4 * id + 0] = make_float4(la.x, ra.x, la.y, ra.y);
    bvh[4 * id + 1] = make_float4(la.z, ra.z, lb.x, rb.x);
    bvh[4 * id + 2] = make_float4(lb.y, rb.y, lb.z, rb.z);
    bvh[4 * id + 3] = make_float4(refs[0], refs[1], 0.0f, 0.0f);
  }
  out.rootRef = encodeRef(1);
  if (!bad.empty()) return bad;
  out.nDev = (int)order.size();
  out.depth = depth;
  return "";
}

// The runtime tree (reference encoding, 12 f32 per node, root 1) collapsed to
// 4-wide nodes (pt_trace.h traceRay4): each wide node takes a binary node's two
// children and keeps replacing its internal child of largest surface area by
// that child's two children until it has four (or only leaves). Wide nodes get
// breadth-first ids (the first ones are the top the kernels stage in LDS); the
// children's boxes are widened like encodeWideTree's; leaves keep their
// references into the pair records. depth: wide levels (root = 1).
static void encodeWide4(const float* nodes, int nNodes, int nTri, float inflate, float inflateAbs,
                        std::vector<float4>& out, int& rootRef, int& nDev, int& depth) {
  auto N = [&](int k, int f) { return nodes[(size_t)k * 12 + f]; };
  auto isLeaf = [&](int k) { return N(k, 3) > 0.0f; };
  auto area = [&](int k) {
    const double dx = N(k, 9) - N(k, 6), dy = N(k, 10) - N(k, 7), dz = N(k, 11) - N(k, 8);
    return dx * dy + dx * dz + dy * dz;
  };
  auto leafRef = [&](int k) {
    return (int)~(((uint32_t)(int)N(k, 4) << LEAF_CNT_BITS) | (uint32_t)((int)N(k, 3) - 1));
  };
  out.clear();
  nDev = 0;
  depth = 1;
  if (nNodes < 2 || isLeaf(1)) {
    rootRef = nNodes >= 2 ? leafRef(1) : REF_NONE;
    out.assign(W4_F4, make_float4(0, 0, 0, 0));
    return;
  }
  std::vector<int> queue{1}, level{1};  // binary ids of the wide nodes, breadth-first, and their levels
  std::vector<std::array<int, 4>> kids;
  for (size_t q = 0; q < queue.size(); q++) {
    const int b = queue[q];
    std::array<int, 4> k = {(int)N(b, 0), (int)N(b, 1), 0, 0};
    int n = 2;
    while (n < 4) {
      int pick = -1;
      double pa = -1.0;
      for (int i = 0; i < n; i++)
        if (!isLeaf(k[i]) && area(k[i]) > pa) { pa = area(k[i]); pick = i; }
      if (pick < 0) break;
      const int c = k[pick];
      k[pick] = (int)N(c, 0);
      k[n++] = (int)N(c, 1);
    }
    for (int i = n; i < 4; i++) k[i] = 0;
    for (int i = 0; i < n; i++)
      if (!isLeaf(k[i])) {
        queue.push_back(k[i]);
        level.push_back(level[q] + 1);
        depth = std::max(depth, level[q] + 1);
      }
    kids.push_back(k);
  }
  nDev = (int)queue.size();
  std::vector<int> wideId(nNodes, -1);
  for (int i = 0; i < nDev; i++) wideId[queue[i]] = i;
  out.assign((size_t)nDev * W4_F4, make_float4(0, 0, 0, 0));
  for (int w = 0; w < nDev; w++) {
    float lo[3][4], hi[3][4];
    int ref[4];
    for (int i = 0; i < 4; i++) {
      const int c = kids[w][i];
      if (c <= 0) {
        ref[i] = REF_NONE;
        for (int a = 0; a < 3; a++) { lo[a][i] = INFINITY; hi[a][i] = -INFINITY; }
        continue;
      }
      ref[i] = isLeaf(c) ? leafRef(c) : wideId[c];
      for (int a = 0; a < 3; a++) {
        const float l = N(c, 6 + a), h = N(c, 9 + a);
        const float e = inflate * (std::fabs(l) + std::fabs(h) + (h - l)) + inflateAbs + 1e-30f;
        lo[a][i] = l - e;
        hi[a][i] = h + e;
      }
    }
    float4* r = &out[(size_t)w * W4_F4];
    for (int a = 0; a < 3; a++) {
      r[a] = make_float4(lo[a][0], lo[a][1], lo[a][2], lo[a][3]);
      r[3 + a] = make_float4(hi[a][0], hi[a][1], hi[a][2], hi[a][3]);
    }
    float fr[4];
    std::memcpy(fr, ref, sizeof(fr));
    r[6] = make_float4(fr[0], fr[1], fr[2], fr[3]);
  }
  rootRef = 0;
  (void)nTri;
}

// the device builder's nodes (pt_build.hip BuildNode, breadth-first from 0) in the
// reference encoding (BVHNode_encoded, main.cpp:69-73): build node k is node k + 1
static std::vector<float> refNodes(const std::vector<BuildNode>& bn, int leafSize) {
  const int M = (int)bn.size();
  std::vector<float> out((size_t)(M + 1) * 12, 0.0f);
  for (int k = 0; k < M; k++) {
    const BuildNode& b = bn[k];
    float* o = out.data() + 12 * (size_t)(k + 1);
    int start, count, left, right;
    std::memcpy(&start, &b.lo.w, 4);
    std::memcpy(&count, &b.hi.w, 4);
    std::memcpy(&left, &b.clo.w, 4);
    std::memcpy(&right, &b.chi.w, 4);
    const bool leaf = count <= leafSize;
    o[0] = leaf ? 0.0f : (float)(left + 1);
    o[1] = leaf ? 0.0f : (float)(right + 1);
    o[3] = leaf ? (float)count : 0.0f;
    o[4] = leaf ? (float)start : 0.0f;
    o[6] = b.lo.x; o[7] = b.lo.y; o[8] = b.lo.z;
    o[9] = b.hi.x; o[10] = b.hi.y; o[11] = b.hi.z;
  }
  return out;
}

// pair records: position i holds triangles order[i] (x) and order[i + 1] (y,
// zeros past the last), PAIR_F4 float4 each (pt_trace.h pairTest), and the two triangles'
// uploaded indices as int bits in the last two floats (-1 past the last): a walk of the
// runtime's tree reads its winner's index with the winner's record (pairTestIds)
static void buildPairs(const std::vector<float4>& geo, const int* order, int nTri, std::vector<float4>& pairs) {
  pairs.assign((size_t)nTri * PAIR_F4, make_float4(0, 0, 0, 0));
  const float4 zero[4] = {make_float4(0, 0, 0, 0), make_float4(0, 0, 0, 0), make_float4(0, 0, 0, 0),
                          make_float4(0, 0, 0, 0)};
  for (int i = 0; i < nTri; i++) {
    const float4* A = &geo[4 * (size_t)(order ? order[i] : i)];
    const float4* B = i + 1 < nTri ? &geo[4 * (size_t)(order ? order[i + 1] : i + 1)] : zero;
    float4* r = &pairs[(size_t)i * PAIR_F4];
    r[0] = make_float4(A[0].x, B[0].x, A[0].y, B[0].y);  // p1.x, p1.y
    r[1] = make_float4(A[0].z, B[0].z, A[1].x, B[1].x);  // p1.z, p2.x
    r[2] = make_float4(A[1].y, B[1].y, A[1].z, B[1].z);  // p2.y, p2.z
    r[3] = make_float4(A[2].x, B[2].x, A[2].y, B[2].y);  // p3.x, p3.y
    r[4] = make_float4(A[2].z, B[2].z, A[3].x, B[3].x);  // p3.z, Ng.x
    r[5] = make_float4(A[3].y, B[3].y, A[3].z, B[3].z);  // Ng.y, Ng.z
    const int ia = order ? order[i] : i, ib = i + 1 < nTri ? (order ? order[i + 1] : i + 1) : -1;
    float fa, fb;
    std::memcpy(&fa, &ia, sizeof(fa));
    std::memcpy(&fb, &ib, sizeof(fb));
    r[6] = make_float4(A[0].w, B[0].w, fa, fb);          // w = dot(Ng, p1); the uploaded indices
  }
}

// Everything pt_upload_scene derives on the host from the caller's arrays,
// computed once and uploaded to every device of a context.
struct SceneHost {
  int nTri = 0, nNodes = 0;
  std::vector<float4> geo, pairs;
  std::vector<float4> hit, mats;  // SceneView::hitRec / mats
  WideTree ref;
  // the runtime's own tree and the reference facts its results are checked against
  bool fast = false;
  bool deviceBuild = false;  // the tree itself is built on each device (pt_build.hip) by uploadScene
  float accelMs = 0.0f;      // host build time (deviceBuild false)
  int accelNodes = 0;
  std::vector<float> accelRef;  // host build: its nodes in the reference encoding (encodeWide4)
  WideTree fastTree;
  std::vector<float4> fpairs, refBox, leafBox;
  std::vector<int> order, leafOf, parent;
};

// The runtime's own tree (a binned-SAH build over the uploaded triangles) and
// the reference facts a result found through it is checked against
// (pt_trace.h refReachable): each triangle's reference leaf and its box, every
// reference node's parent and box. Any triangle in two reference leaves, or a
// failed build, leaves the runtime on the reference tree alone (h.fast false).
static void prepareAccel(const float* tris, int nTri, const float* nodes, int nNodes, SceneHost& h, bool hostBuild) {
  h.fast = false;
  if (!PT_FAST_TREE) return;
  auto nodeN = [&](int k) { return (int)nodes[(size_t)k * 12 + 3]; };
  std::vector<int>& leafOf = h.leafOf;
  std::vector<int>& parent = h.parent;
  leafOf.assign(nTri, -1);
  parent.assign(nNodes, 0);
  {
    std::vector<int> st{1};
    while (!st.empty()) {
      const int k = st.back();
      st.pop_back();
      if (nodeN(k) > 0) {
        const int index = (int)nodes[(size_t)k * 12 + 4];
        for (int i = index; i < index + nodeN(k); i++) {
          if (leafOf[i] != -1) return;  // a triangle in two leaves: reference tree only
          leafOf[i] = k;
        }
        continue;
      }
      for (int c = 0; c < 2; c++) {
        const int ch = (int)nodes[(size_t)k * 12 + c];
        if (ch > 0 && ch < nNodes) {
          // refReachable's margin test needs every box inside its parent's (true
          // of the reference builders, which bound each node's own triangles)
          const float* pb = nodes + (size_t)k * 12;
          const float* cb = nodes + (size_t)ch * 12;
          for (int a = 0; a < 3; a++)
            if (!(pb[6 + a] <= cb[6 + a] && cb[9 + a] <= pb[9 + a])) return;
          parent[ch] = k;
          st.push_back(ch);
        }
      }
    }
  }
  h.refBox.assign((size_t)nNodes * 2, make_float4(0, 0, 0, 0));
  h.leafBox.assign((size_t)nTri * 2, make_float4(0, 0, 0, 0));
  for (int k = 0; k < nNodes; k++) {
    const float* c = nodes + (size_t)k * 12;
    h.refBox[2 * (size_t)k] = make_float4(c[6], c[7], c[8], 0.0f);
    h.refBox[2 * (size_t)k + 1] = make_float4(c[9], c[10], c[11], 0.0f);
  }
  const float inf = INFINITY;
  for (int i = 0; i < nTri; i++) {
    // lo.w holds the reference leaf's node id (int bits), so the reachability check reads one
    // 32-byte record per hit instead of that record and a separate leaf-id array
    if (leafOf[i] < 0) {  // in no reference leaf: never a reference hit (empty box fails the margin test)
      h.leafBox[2 * (size_t)i] = make_float4(inf, inf, inf, 0.0f);
      h.leafBox[2 * (size_t)i + 1] = make_float4(-inf, -inf, -inf, 0.0f);
    } else {
      h.leafBox[2 * (size_t)i] = h.refBox[2 * (size_t)leafOf[i]];
      h.leafBox[2 * (size_t)i + 1] = h.refBox[2 * (size_t)leafOf[i] + 1];
    }
    int id = leafOf[i];
    std::memcpy(&h.leafBox[2 * (size_t)i].w, &id, sizeof(int));
  }
  // the tree itself: on the GPU by uploadScene (pt_build.hip), or here (scene.cpp's threaded binned SAH)
  if (!hostBuild) {
    h.deviceBuild = true;
    h.fast = true;
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<float> an;
  if (pt::buildAccel(tris, nTri, PT_ACCEL_LEAF, an, h.order) < 0 || an.size() / 12 >= (1u << 24)) return;
  h.accelNodes = (int)(an.size() / 12) - 1;
  h.accelRef = an;

  // widened by 1e-5 of each box's own magnitude plus 3e-5 of the scene's: above
  // the rounding of a slab test (~1.2e-7 x the origin-box distance) for ray origins
  // up to ~100x the scene scale away, so a ray that hits a triangle enters every box around it
  float sceneScale = 0.0f;
  for (int i = 0; i < nTri; i++)
    for (int k = 0; k < 9; k++) sceneScale = std::max(sceneScale, std::fabs(tris[(size_t)i * 36 + k]));
  if (!encodeWideTree(an.data(), (int)(an.size() / 12), nTri, 1e-5f, h.fastTree, 3e-5f * sceneScale).empty()) return;
  buildPairs(h.geo, h.order.data(), nTri, h.fpairs);
  h.accelMs = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  h.fast = true;
}

// host-side re-layout of the caller's arrays (pt_upload_scene); "" or the reason they are malformed
static std::string prepareScene(const float* tris, int nTri, const float* nodes, int nNodes, SceneHost& h,
                                bool hostBuild) {
  h.nTri = nTri;
  h.nNodes = nNodes;
  // geometry records (+1 zero record past the last triangle)
  h.geo.assign((size_t)(nTri + 1) * 4, make_float4(0, 0, 0, 0));
  for (int i = 0; i < nTri; i++) {
    const float* t = tris + (size_t)i * 36;
    float N[3];
    nrm3(t, t + 3, t + 6, N);
    float w = (N[0] * t[0] + N[1] * t[1]) + N[2] * t[2];
    h.geo[4 * i + 0] = make_float4(t[0], t[1], t[2], w);
    h.geo[4 * i + 1] = make_float4(t[3], t[4], t[5], 0.0f);
    h.geo[4 * i + 2] = make_float4(t[6], t[7], t[8], 0.0f);
    h.geo[4 * i + 3] = make_float4(N[0], N[1], N[2], 0.0f);
  }
  // shading records: the normals and a material id per triangle; each distinct
  // material (Triangle_encoded floats 18..35, compared bit for bit) stored once
  h.hit.assign((size_t)nTri * HIT_F4, make_float4(0, 0, 0, 0));
  {
    std::map<std::array<uint32_t, 18>, int> ids;
    std::array<uint32_t, 18> lastKey{};
    int lastId = 0;
    for (int i = 0; i < nTri; i++) {
      const float* t = tris + (size_t)i * 36;
      std::array<uint32_t, 18> key;
      std::memcpy(key.data(), t + 18, sizeof(key));
      int id;
      if (i > 0 && key == lastKey) {  // meshes share one material: most lookups are this one
        id = lastId;
      } else if (auto it = ids.find(key); it == ids.end()) {
        id = (int)ids.size();
        ids.emplace(key, id);
        for (int k = 0; k < MAT_F4; k++) h.mats.push_back(make_float4(t[16 + 4 * k], t[17 + 4 * k], t[18 + 4 * k], t[19 + 4 * k]));
      } else {
        id = it->second;
      }
      lastKey = key;
      lastId = id;
      float fid;
      std::memcpy(&fid, &id, 4);
      float4* r = &h.hit[(size_t)i * HIT_F4];
      r[0] = make_float4(t[9], t[10], t[11], t[12]);
      r[1] = make_float4(t[13], t[14], t[15], t[16]);
      r[2] = make_float4(t[17], fid, 0.0f, 0.0f);
    }
  }
  std::string bad = encodeWideTree(nodes, nNodes, nTri, 0.0f, h.ref);
  if (!bad.empty()) return bad;
  buildPairs(h.geo, nullptr, nTri, h.pairs);
  prepareAccel(tris, nTri, nodes, nNodes, h, hostBuild);
  return "";
}

static int syncStreams(pt_ctx* ctx);
static int ensureBasicImage(pt_ctx* ctx);

static int uploadScene(pt_ctx* ctx, const float* tris, const SceneHost& h) {
  if (int rc = syncStreams(ctx)) return rc;  // no frame in flight reads the buffers replaced here
  ctx->policyKey++;  // the tree / split policies are measured again at the next restart
  CK(hipSetDevice(ctx->cfg.device_id));
  int rc;
  if ((rc = upload(ctx, &ctx->d_pairs, h.pairs)) || (rc = upload(ctx, &ctx->d_geo, h.geo)) ||
      (rc = upload(ctx, &ctx->d_bvh, h.ref.bvh)))
    return rc;
  if ((rc = upload(ctx, &ctx->d_hit, h.hit)) || (rc = upload(ctx, &ctx->d_mats, h.mats))) return rc;
  ctx->nMats = (int)(h.mats.size() / MAT_F4);
  ctx->nTri = h.nTri;
  ctx->nNodes = h.nNodes;
  ctx->nDevNodes = h.ref.nDev;
  // Large Disney/MIS scenes (the regen kernel's, renderOne wideScene) run 4 frames in flight:
  // c5's frames last ~6 ms, and 8 in flight spend more on the pipeline's fill and drain than
  // they gain (bench line, 20 frames from idle: 5.60-5.66 ms per frame at 4 vs 5.88 at 8, 6.00 at 6)
  if (ctx->pipe && !ctx->pipeDepthFixed) {
    const size_t sceneBytes = (size_t)ctx->nTri * (PAIR_F4 * 16 + 64 + HIT_F4 * 16) + (size_t)ctx->nDevNodes * 64;
    const bool wideScene = ctx->cfg.integrator != 0 && !(ctx->cfg.flags & PT_FLAG_NO_CULL) &&
                           sceneBytes > ((size_t)PT_WIDE_SCENE_MB << 20);
    ctx->pipeDepth = wideScene ? std::min(ctx->pipeDepthBase, 4) : ctx->pipeDepthBase;
  }
  if (ctx->pipe) {
    const size_t sceneBytes = (size_t)ctx->nTri * (PAIR_F4 * 16 + 64 + HIT_F4 * 16) + (size_t)ctx->nDevNodes * 64;
    ctx->batchCap = batchFor(ctx, ctx->cfg.integrator != 0 && sceneBytes > ((size_t)PT_WIDE_SCENE_MB << 20));
  }
  ctx->rootRef = h.ref.rootRef;
  ctx->depth = h.ref.depth;
  ctx->maxStack = h.ref.depth + 1;
  ctx->fastReady = false;
  ctx->fast4Ready = false;
  ctx->accelDevice = -1;
  ctx->accelMs = 0.0f;
  ctx->accelNodes = ctx->accelDepth = 0;
  if (!h.fast) return PT_OK;
  if ((rc = upload(ctx, &ctx->d_refParent, h.parent)) ||
      (rc = upload(ctx, &ctx->d_refBox, h.refBox)) || (rc = upload(ctx, &ctx->d_leafBox, h.leafBox)))
    return rc;
  if (h.deviceBuild) {
    // the runtime's tree built here, from the geometry records just uploaded (pt_build.hip)
    const auto t0 = std::chrono::steady_clock::now();
    AccelBuild ab;
    hipError_t e = buildAccelDevice(ctx->d_geo, h.nTri, PT_ACCEL_LEAF, 1e-5f, 3e-5f, ab, ctx->stream);
    if (e != hipSuccess) return fail(ctx, PT_E_HIP, std::string("device tree build: ") + hipGetErrorString(e));
    if (ab.nNodes + 1 >= (1 << 24)) {  // as the host path: no runtime tree of 2^24 nodes or more
      freeAccelBuild(ab);
      return PT_OK;
    }
    // the 4-wide collapse, on the device too (the large-scene regen kernel's and the megakernel's tree)
    float4* w4 = nullptr;
    e = collapseWide4Device(ab.nodes, ab.nNodes, PT_ACCEL_LEAF, 1e-5f, 3e-5f, &w4, &ctx->f4Root, &ctx->f4nDev,
                            &ctx->f4Depth, ctx->stream);
    dfree(ab.nodes);
    if (e != hipSuccess) {
      freeAccelBuild(ab);
      return fail(ctx, PT_E_HIP, std::string("device 4-wide collapse: ") + hipGetErrorString(e));
    }
    dfree(ctx->d_fbvh4);
    ctx->d_fbvh4 = w4;
    dfree(ctx->d_fbvh);
    dfree(ctx->d_fpairs);
    dfree(ctx->d_fastTri);
    ctx->d_fbvh = ab.bvh;
    ctx->d_fpairs = ab.pairs;
    ctx->d_fastTri = ab.order;
    ctx->fRoot = ab.rootRef;
    ctx->fnDev = ab.nDev;
    ctx->fDepth = ab.depth;
    ctx->accelMs = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ctx->accelDevice = 1;
    ctx->accelNodes = ab.nNodes;
  } else {
    if ((rc = upload(ctx, &ctx->d_fbvh, h.fastTree.bvh)) || (rc = upload(ctx, &ctx->d_fpairs, h.fpairs)) ||
        (rc = upload(ctx, &ctx->d_fastTri, h.order)))
      return rc;
    ctx->fRoot = h.fastTree.rootRef;
    ctx->fnDev = h.fastTree.nDev;
    ctx->fDepth = h.fastTree.depth;
    ctx->accelMs = h.accelMs;
    ctx->accelDevice = 0;
    ctx->accelNodes = h.accelNodes;
  }
  ctx->accelDepth = ctx->fDepth;
  // the host-built tree's 4-wide collapse (the device build collapsed on the device above)
  if (!h.deviceBuild) {
    const std::vector<float>& an = h.accelRef;
    const int nn = (int)(an.size() / 12);
    float scale = 0.0f;  // the scene's largest coordinate magnitude: the root box's
    for (int k = 6; k < 12 && nn > 1; k++) scale = std::max(scale, std::fabs(an[12 + k]));
    std::vector<float4> w4;
    encodeWide4(an.data(), nn, h.nTri, 1e-5f, 3e-5f * scale, w4, ctx->f4Root, ctx->f4nDev, ctx->f4Depth);
    if ((rc = upload(ctx, &ctx->d_fbvh4, w4))) return rc;
  }
  ctx->fast4Ready = true;
  // a visit pushes up to three children: the traversal stack needs 3 entries per wide level
  ctx->maxStack = std::max(ctx->maxStack, 3 * ctx->f4Depth + 2);
  ctx->sceneVersion++;  // camera-ray bins are rebuilt for the new triangles
  ctx->maxStack = std::max(ctx->maxStack, ctx->fDepth + 1);
  ctx->fastReady = true;
  return PT_OK;
}

// every context of a device group (rank 0 first), or just ctx
static std::vector<pt_ctx*> members(pt_ctx* ctx) {
  std::vector<pt_ctx*> m{ctx};
  m.insert(m.end(), ctx->peers.begin(), ctx->peers.end());
  return m;
}

static int fromPeer(pt_ctx* ctx, pt_ctx* p, int rc) {
  if (rc && p != ctx) ctx->err = "device " + std::to_string(p->cfg.device_id) + ": " + p->err;
  return rc;
}

int pt_upload_scene(pt_ctx* ctx, const float* tris, int nTri, const float* nodes, int nNodes) {
  if (!ctx || !tris || !nodes) return PT_E_INVALID;
  if (nTri < 1 || nNodes < 2) return fail(ctx, PT_E_BADSCENE, "need >= 1 triangle and >= 2 nodes (dummy 0, root 1)");
  if (nTri > MAX_TRIS) return fail(ctx, PT_E_BADSCENE, "too many triangles for the leaf encoding");
  const auto t0 = std::chrono::steady_clock::now();
  SceneHost h;
  std::string bad = prepareScene(tris, nTri, nodes, nNodes, h, (ctx->cfg.flags & PT_FLAG_HOST_ACCEL) != 0);
  if (!bad.empty()) return fail(ctx, PT_E_BADSCENE, bad);
  for (pt_ctx* m : members(ctx))
    if (int rc = uploadScene(m, tris, h)) return fromPeer(ctx, m, rc);
  ctx->uploadMs = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return PT_OK;
}

int pt_build_bvh_device(pt_ctx* ctx, const float* tris, int nTri, int leafSize, float* nodes_out, int maxNodes,
                        int* nNodesOut, int* orderOut) {
  if (!ctx || !tris || !nodes_out || !nNodesOut || !orderOut || nTri < 1 || leafSize < 1 || leafSize > MAX_LEAF)
    return PT_E_INVALID;
  if (nTri > MAX_TRIS) return fail(ctx, PT_E_BADSCENE, "too many triangles for the leaf encoding");
  if (int rc = syncStreams(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  // the builder reads p1..p3 of the geometry records (the normal and plane offset only feed the pair records)
  std::vector<float4> geo((size_t)nTri * 4, make_float4(0, 0, 0, 0));
  for (int i = 0; i < nTri; i++)
    for (int k = 0; k < 3; k++) {
      const float* v = tris + (size_t)i * 36 + 3 * k;
      geo[4 * (size_t)i + k] = make_float4(v[0], v[1], v[2], 0.0f);
    }
  float4* dgeo = nullptr;
  if (int rc = upload(ctx, &dgeo, geo)) return rc;
  AccelBuild ab;
  hipError_t e = buildAccelDevice(dgeo, nTri, leafSize, 0.0f, 0.0f, ab, ctx->stream);
  dfree(dgeo);
  if (e != hipSuccess) return fail(ctx, PT_E_HIP, std::string("device tree build: ") + hipGetErrorString(e));
  const int M = ab.nNodes;
  *nNodesOut = M + 1;
  std::vector<BuildNode> bn(M);
  e = hipMemcpy(bn.data(), ab.nodes, (size_t)M * sizeof(BuildNode), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(orderOut, ab.order, (size_t)nTri * sizeof(int), hipMemcpyDeviceToHost);
  freeAccelBuild(ab);
  if (e != hipSuccess) return fail(ctx, PT_E_HIP, std::string("device tree download: ") + hipGetErrorString(e));
  if (M + 1 > maxNodes) return fail(ctx, PT_E_INVALID, "nodes_out holds fewer than *nNodes_out nodes");
  const std::vector<float> ref = refNodes(bn, leafSize);
  std::memcpy(nodes_out, ref.data(), ref.size() * sizeof(float));
  return PT_OK;
}

// calculateHdrCache of host image hdr (w*h*3) into the device table out (w*h float4)
static int deviceHdrCache(pt_ctx* ctx, const float* hdr, int w, int h, float4* out) {
  const size_t n = (size_t)w * h;
  float* d3 = nullptr;
  float* scratch = nullptr;
  CK(hipMalloc(&d3, n * 3 * sizeof(float)));
  if (hipMalloc(&scratch, (2 * n + 2 * (size_t)w + 1) * sizeof(float)) != hipSuccess) {
    (void)hipFree(d3);
    return fail(ctx, PT_E_NOMEM, "hdr cache scratch");
  }
  hipError_t e = hipMemcpyAsync(d3, hdr, n * 3 * sizeof(float), hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = launchHdrCache(d3, w, h, out, scratch, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(d3);
  (void)hipFree(scratch);
  if (e != hipSuccess) return fail(ctx, PT_E_HIP, std::string("hdr cache: ") + hipGetErrorString(e));
  return PT_OK;
}

static int envOne(pt_ctx* ctx, const float* hdr, int w, int h, const float* cache) {
  if (!ctx) return PT_E_INVALID;
  if (int rc = syncStreams(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  dfree(ctx->d_hdr);
  dfree(ctx->d_cache);
  dfree(ctx->d_hdr8);
  dfree(ctx->d_cache4);
  dfree(ctx->d_cacheRow);
  dfree(ctx->d_cacheY);
  dfree(ctx->d_trig);
  dfree(ctx->d_light);
  ctx->hdrW = ctx->hdrH = 0;
  if (!hdr) return PT_OK;
  if (w <= 0 || h <= 0) return PT_E_INVALID;
  const size_t n = (size_t)w * h;
  // render layout (pt_kernels.h Env): (r, g, b, pdf) texels + (x, y) sample table
  std::vector<float4> a(n);
  for (size_t k = 0; k < n; k++)
    a[k] = make_float4(hdr[3 * k], hdr[3 * k + 1], hdr[3 * k + 2], cache ? cache[3 * k + 2] : 0.0f);
  CK(hipMalloc(&ctx->d_hdr, n * sizeof(float4)));
  CK(hipMalloc(&ctx->d_cache, n * sizeof(float2)));
  CK(hipMemcpy(ctx->d_hdr, a.data(), n * sizeof(float4), hipMemcpyHostToDevice));
  if (cache) {
    std::vector<float2> b(n);
    for (size_t k = 0; k < n; k++) b[k] = make_float2(cache[3 * k], cache[3 * k + 1]);
    CK(hipMemcpy(ctx->d_cache, b.data(), n * sizeof(float2), hipMemcpyHostToDevice));
  } else {
    float4* full = nullptr;  // calculateHdrCache on the GPU, then packed into the render layout
    CK(hipMalloc(&full, n * sizeof(float4)));
    int rc = deviceHdrCache(ctx, hdr, w, h, full);
    if (!rc) {
      hipError_t e = launchEnvPack(ctx->d_hdr, full, ctx->d_cache, (int)n, ctx->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
      if (e != hipSuccess) rc = fail(ctx, PT_E_HIP, std::string("env pack: ") + hipGetErrorString(e));
    }
    (void)hipFree(full);
    if (rc) return rc;
  }
  // The compact texels (8 + 4 bytes instead of 16 + 8 per texel; pt_kernels.h Env), kept when every
  // texel decodes back to its float bits: a Radiance map's RGBE values and calculateHdrCache's
  // table always do. c4's MIS light samples read the sample table at uniformly random (xi1, xi2):
  // half the bytes per texel, twice the texels per cached line. PT_ENV_COMPACT=0: the float texels.
  static const bool compact = [] {
    const char* e = std::getenv("PT_ENV_COMPACT");
    return !e || std::atoi(e) != 0;
  }();
  // (built into locals and handed to the context only once verified: a failure part-way leaves the
  // float texels serving, never a half-built compact form)
  if (compact && w <= 65535 && h <= 65535) {
    uint2* hdr8 = nullptr;
    uint32_t* cache4 = nullptr;
    int* d_bad = nullptr;
    hipError_t e = hipMalloc(&hdr8, n * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&cache4, n * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&d_bad, sizeof(int));
    if (e == hipSuccess) e = hipMemsetAsync(d_bad, 0, sizeof(int), ctx->stream);
    if (e == hipSuccess) e = launchEnvCompact(ctx->d_hdr, ctx->d_cache, w, h, hdr8, cache4, d_bad, ctx->stream);
    int bad = 1;
    if (e == hipSuccess) e = hipMemcpyAsync(&bad, d_bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    dfree(d_bad);
    if (e != hipSuccess || bad) {  // not exact (or failed): the float texels serve
      dfree(hdr8);
      dfree(cache4);
      if (e != hipSuccess) return fail(ctx, PT_E_HIP, std::string("env compact: ") + hipGetErrorString(e));
    } else {
      ctx->d_hdr8 = hdr8;
      ctx->d_cache4 = cache4;
    }
  }
  if (ctx->d_cache4) {  // SampleHdr's sines and cosines of the compact table's integers (Env::trig)
    float2* trig = nullptr;
    hipError_t e2 = hipMalloc(&trig, (size_t)(w + h + 2) * sizeof(float2));
    if (e2 == hipSuccess) e2 = launchEnvTrig(trig, w, h, ctx->stream);
    if (e2 == hipSuccess) e2 = hipStreamSynchronize(ctx->stream);
    if (e2 != hipSuccess) {
      dfree(trig);
      return fail(ctx, PT_E_HIP, std::string("env trig: ") + hipGetErrorString(e2));
    }
    ctx->d_trig = trig;
    // ... and every entry's light-sample color and pdf (Env::light)
    Env e;
    std::memset(&e, 0, sizeof(e));
    e.hdr = ctx->d_hdr;
    e.hdr8 = ctx->d_hdr8;
    e.trig = ctx->d_trig;
    e.w = e.res = w;
    e.h = h;
    uint2* light = nullptr;
    e2 = hipMalloc(&light, (size_t)(w + 1) * (h + 1) * sizeof(uint2));
    if (e2 == hipSuccess) e2 = launchEnvLight(e, light, ctx->stream);
    if (e2 == hipSuccess) e2 = hipStreamSynchronize(ctx->stream);
    if (e2 != hipSuccess) {
      dfree(light);
      return fail(ctx, PT_E_HIP, std::string("env light: ") + hipGetErrorString(e2));
    }
    ctx->d_light = light;
  }
  if (ctx->d_cache4) {
    // the sample table by rows (pt_kernels.h Env::cacheRow), kept when every entry of every row equals
    // its row form: each row's x is one value, and the rows of one x hold the same y's
    std::vector<uint32_t> c4(n);
    CK(hipMemcpy(c4.data(), ctx->d_cache4, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<uint32_t> rows(h);
    std::vector<unsigned short> ys;
    std::vector<int> idOf(65536, -1);
    bool ok = true;
    for (int i = 0; i < h && ok; i++) {
      const uint32_t* row = c4.data() + (size_t)i * w;
      const uint32_t x = row[0] & 0xffffu;
      int id = idOf[x];
      if (id < 0) {
        id = idOf[x] = (int)(ys.size() / (size_t)w);
        for (int j = 0; j < w; j++) ys.push_back((unsigned short)(row[j] >> 16));
      }
      const unsigned short* yr = ys.data() + (size_t)id * w;
      for (int j = 0; j < w && ok; j++) ok = (row[j] & 0xffffu) == x && (row[j] >> 16) == yr[j];
      rows[i] = x | (uint32_t)id << 16;
    }
    if (ok) {  // both or neither (Env::cacheRow reads cacheY)
      uint32_t* cr = nullptr;
      unsigned short* cy = nullptr;
      hipError_t e = hipMalloc(&cr, rows.size() * sizeof(uint32_t));
      if (e == hipSuccess) e = hipMalloc(&cy, ys.size() * sizeof(unsigned short));
      if (e == hipSuccess) e = hipMemcpy(cr, rows.data(), rows.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(cy, ys.data(), ys.size() * sizeof(unsigned short), hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        dfree(cr);
        dfree(cy);
        return fail(ctx, PT_E_HIP, std::string("env rows: ") + hipGetErrorString(e));
      }
      ctx->d_cacheRow = cr;
      ctx->d_cacheY = cy;
    }
  }
  ctx->policyKey++;
  ctx->hdrW = w;
  ctx->hdrH = h;
  return PT_OK;
}

int pt_upload_env(pt_ctx* ctx, const float* hdr, int w, int h, const float* cache) {
  if (!ctx) return PT_E_INVALID;
  if (ctx->peers.empty()) return envOne(ctx, hdr, w, h, cache);
  // a device group computes calculateHdrCache once (on rank 0's GPU) and uploads it everywhere
  std::vector<float> own;
  if (hdr && !cache && w > 0 && h > 0) {
    own.resize((size_t)w * h * 3);
    if (int rc = pt_hdr_cache_device(ctx, hdr, w, h, own.data())) return rc;
    cache = own.data();
  }
  for (pt_ctx* m : members(ctx))
    if (int rc = envOne(m, hdr, w, h, cache)) return fromPeer(ctx, m, rc);
  return PT_OK;
}

int pt_hdr_cache_device(pt_ctx* ctx, const float* hdr, int w, int h, float* cache_out) {
  if (!ctx || !hdr || !cache_out || w <= 0 || h <= 0) return PT_E_INVALID;
  CK(hipSetDevice(ctx->cfg.device_id));
  const size_t n = (size_t)w * h;
  float4* d = nullptr;
  CK(hipMalloc(&d, n * sizeof(float4)));
  int rc = deviceHdrCache(ctx, hdr, w, h, d);
  std::vector<float4> b(rc ? 0 : n);
  if (!rc && hipMemcpy(b.data(), d, n * sizeof(float4), hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(ctx, PT_E_HIP, "pt_hdr_cache_device: copy");
  (void)hipFree(d);
  if (rc) return rc;
  for (size_t k = 0; k < n; k++) {
    cache_out[3 * k] = b[k].x;
    cache_out[3 * k + 1] = b[k].y;
    cache_out[3 * k + 2] = b[k].z;
  }
  return PT_OK;
}

int pt_upload_shapes(pt_ctx* ctx, const double* shapes, int n) {
  if (!ctx || (!shapes && n > 0) || n < 0) return PT_E_INVALID;
  if (!ctx->peers.empty()) return fail(ctx, PT_E_INVALID, "BASIC shapes: one device only");
  if (int rc = syncStreams(ctx)) return rc;
  dfree(ctx->d_shapes);
  ctx->nShapes = 0;
  if (n == 0) return PT_OK;
  CK(hipMalloc(&ctx->d_shapes, (size_t)n * PT_SHAPE_DOUBLES * sizeof(double)));
  CK(hipMemcpy(ctx->d_shapes, shapes, (size_t)n * PT_SHAPE_DOUBLES * sizeof(double), hipMemcpyHostToDevice));
  ctx->nShapes = n;
  return PT_OK;
}

int pt_download_basic_image(pt_ctx* ctx, double* rgb) {
  if (!ctx || !rgb) return PT_E_INVALID;
  if (ctx->cfg.integrator != PT_BASIC_CPU_COMPAT) return fail(ctx, PT_E_INVALID, "not a BASIC context");
  if (int rc = syncStreams(ctx)) return rc;
  const size_t n = (size_t)ctx->cfg.width * ctx->cfg.height * 3;
  if (!ctx->d_basicImg) {
    std::memset(rgb, 0, n * sizeof(double));
    return PT_OK;
  }
  CK(hipMemcpy(rgb, ctx->d_basicImg, n * sizeof(double), hipMemcpyDeviceToHost));
  return PT_OK;
}

int pt_set_basic_stream(pt_ctx* ctx, const double* stream, int64_t n, const int64_t* offsets, int64_t nOffsets) {
  if (!ctx) return PT_E_INVALID;
  if (ctx->cfg.integrator != PT_BASIC_CPU_COMPAT) return fail(ctx, PT_E_INVALID, "not a BASIC context");
  if (int rc = syncStreams(ctx)) return rc;
  dfree(ctx->d_stream);
  dfree(ctx->d_offsets);
  ctx->streamN = ctx->nOffsets = 0;
  if (!stream) return PT_OK;
  if (n < 1 || !offsets || nOffsets < 1) return fail(ctx, PT_E_INVALID, "pt_set_basic_stream: empty stream or offsets");
  for (int64_t k = 0; k < nOffsets; k++)
    if (offsets[k] < 0 || offsets[k] > n || (k > 0 && offsets[k] < offsets[k - 1]))
      return fail(ctx, PT_E_INVALID, "pt_set_basic_stream: offsets must be non-decreasing within [0, n]");
  CK(hipMalloc(&ctx->d_stream, (size_t)n * sizeof(double)));
  CK(hipMalloc(&ctx->d_offsets, (size_t)nOffsets * sizeof(long long)));
  CK(hipMemcpy(ctx->d_stream, stream, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
  CK(hipMemcpy(ctx->d_offsets, offsets, (size_t)nOffsets * sizeof(long long), hipMemcpyHostToDevice));
  ctx->streamN = n;
  ctx->nOffsets = nOffsets;
  return PT_OK;
}

int pt_basic_replay_overruns(pt_ctx* ctx, int64_t* count) {
  if (!ctx || !count) return PT_E_INVALID;
  if (int rc = syncStreams(ctx)) return rc;
  unsigned long long v = 0;
  if (ctx->d_overruns) CK(hipMemcpy(&v, ctx->d_overruns, sizeof(v), hipMemcpyDeviceToHost));
  *count = (int64_t)v;
  return PT_OK;
}

static int defaultBounce(int integ) {
  switch (integ) {
    case PT_LAMBERT_O: return 2;           // O:385
    case PT_DISNEY_UNIFORM_D: return 5;    // D:502
    case PT_DISNEY_MIS_SOBOL_IS: return 2; // IS:861
    default: return 8;                     // BasicRayTracingWithC++/main.cpp:254
  }
}

// Fold the oldest unfolded launch's device time into the totals (and into its
// probe slot). blocking = false returns false instead of waiting for it.
static bool foldOne(pt_ctx* ctx, bool blocking) {
  if (ctx->folded >= ctx->issued) return false;
  const int k = (int)(ctx->folded % EV_RING);
  hipEvent_t b = ctx->ev[2 * k], e = ctx->ev[2 * k + 1];
  if (blocking) (void)hipEventSynchronize(e);
  else if (hipEventQuery(e) != hipSuccess) return false;
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, b, e) != hipSuccess) ms = 0.0f;
  ctx->msTotal += ms;
  ctx->msLast = ms;
  const int slot = ctx->evProbe[k];
  if (slot >= 0 && ctx->evGen[k] == ctx->probeGen) {
    ctx->probeMs[slot] += ms;
    ctx->probeN[slot]++;
  }
  ctx->folded++;
  return true;
}

// fold every launch up to launch number `upto` (inclusive), waiting for them
static void foldUpTo(pt_ctx* ctx, long long upto) {
  while (ctx->folded <= upto && foldOne(ctx, true)) {
  }
}

// begin/end events for the next launch (launch number ctx->issued)
static int launchEvents(pt_ctx* ctx, hipEvent_t* b, hipEvent_t* e) {
  while (foldOne(ctx, false)) {
  }
  if (ctx->issued - ctx->folded >= EV_RING) foldOne(ctx, true);
  const int k = (int)(ctx->issued % EV_RING);
  for (int j = 2 * k; j < 2 * k + 2; j++)
    if (!ctx->ev[j]) CK(hipEventCreate(&ctx->ev[j]));
  *b = ctx->ev[2 * k];
  *e = ctx->ev[2 * k + 1];
  return PT_OK;
}

// the launch whose events launchEvents handed out has been enqueued (it renders `frames` frames)
static void commitLaunch(pt_ctx* ctx, int frames = 1) {
  ctx->frames += frames;
  const int k = (int)(ctx->issued % EV_RING);
  ctx->evProbe[k] = ctx->tagSlot;
  ctx->evGen[k] = ctx->probeGen;
  if (ctx->tagSlot >= 0) ctx->probeLast[ctx->tagSlot] = ctx->issued;
  ctx->tagSlot = -1;
  ctx->issued++;
  ctx->launches++;
}

// the RNG / Sobol sample index of frame frameCounter: sample-parallel ranks
// interleave their sample streams (rank r renders samples r, r+W, r+2W, ...)
static uint32_t sampleIndex(const pt_config& c, uint32_t frameCounter) {
  const uint32_t w = c.sample_world > 0 ? (uint32_t)c.sample_world : 1u;
  return frameCounter * w + (uint32_t)c.sample_rank;
}

static SceneView sceneView(const pt_ctx* ctx) {
  SceneView s;
  s.geo = ctx->d_geo;
  s.pairs = ctx->d_pairs;
  s.hitRec = ctx->d_hit;
  s.mats = ctx->d_mats;
  s.nMats = ctx->nMats;
  s.bvh = ctx->d_bvh;
  s.nTop = std::min(LDS_NODES, ctx->nDevNodes);
  s.rootRef = ctx->rootRef;
  s.nTri = ctx->nTri;
  s.fast = 0;  // set per launch (renderFrame)
  s.fbvh = ctx->d_fbvh;
  s.fpairs = ctx->d_fpairs;
  s.fastTri = ctx->d_fastTri;
  s.fRoot = ctx->fRoot;
  s.fnTop = std::min(LDS_NODES, ctx->fnDev);
  s.fbvh4 = ctx->d_fbvh4;
  s.f4Root = ctx->f4Root;
  s.f4nTop = std::min(LDS_NODES * 4 / W4_F4, ctx->f4nDev);  // the LDS copy holds LDS_NODES * 4 float4
  s.refParent = ctx->d_refParent;
  s.refBox = ctx->d_refBox;
  s.leafBox = ctx->d_leafBox;
  return s;
}

// make sure the overflow stack covers `threads` threads of a kernel keeping `ldsDepth` entries in LDS
static int ensureOverflow(pt_ctx* ctx, size_t threads, int* ovfDepth, int ldsDepth = LDS_STACK, int slots = 1) {
  // pt_trace.h StackT: at most maxStack - ldsDepth/2 - 1 entries are ever in HBM
  *ovfDepth = ctx->maxStack > ldsDepth ? ctx->maxStack - ldsDepth / 2 : 0;
  if (*ovfDepth == 0) return PT_OK;
  size_t need = threads * (size_t)(*ovfDepth) * (size_t)slots;  // slots: one region per frame in flight
  if (need > ctx->ovfInts) {
    dfree(ctx->d_ovf);
    CK(hipMalloc(&ctx->d_ovf, need * sizeof(int)));
    ctx->ovfInts = need;
  }
  return PT_OK;
}

// Two policies are chosen by measurement, since results are identical either
// way and which is faster depends on the scene and the integrator:
//  * the tree: the runtime's own (binned SAH; results checked against the
//    uploaded tree) pays off when the uploaded tree is poor -- the reference's
//    SAH with its z-typo: c2 0.57 -> 0.47 ms, c4 0.99 -> 0.80 -- and costs its
//    checks when the uploaded tree is already good (c5: +2 %);
//  * tile splitting (reorderKernel) pays off when the SIMDs have issue slots to
//    spare (the MIS integrator, latency-bound) and costs when they do not (the
//    Lambert megakernel is VALU-bound: a split item's idle lanes still take
//    issue cycles);
// (Longest-first tile order -- per-tile cost atomics, the order lookup of every
// claim, the reorder kernel -- was probed as well until round 5: it cost on the
// Lambert megakernel, c2 0.347 ms in band order vs 0.372, but Lambert frames run
// on the regen kernel now, and for the integrators left on the megakernel it
// never lost: c4 at N = 1 0.268 vs 0.267 ms, c4's 1/8 share in a 20-frame batch
// 0.072 vs 0.088, while the probe's noisy single-frame choice gave 0.069-0.087.)
// After a restart of the running mean (frameCounter 0, as on every camera move
// in the reference): frames 1-2 run the runtime's tree and 3-4 the uploaded
// one, unsplit; frame 5 runs the runtime's tree while the host, at frame 6,
// waits for frame 4 (frame 5 is already queued, so the GPU never drains) and
// keeps the faster tree; frames 6-10 split (the per-tile split state
// converges), 11-12 are timed, and at frame 14 -- waiting for frame 12 with 13
// queued -- the faster split policy is kept. No frame waits for its own
// predecessor. The decisions are kept across later restarts until the scene or
// the env is uploaded again (a camera move changes neither tree's merit nor,
// measurably, the split policy's), so only the first restart after an upload
// pays for the probe's slower trial frames; every restart still clears the
// per-tile split state and cost estimates. Sets *useFast; returns the split
// percentage for this frame's reorder (0 = off).
static int probePolicy(pt_ctx* ctx, uint32_t frameCounter, bool ordered, bool fastAllowed, bool* useFast, int slot,
                       hipStream_t S) {
  *useFast = fastAllowed;
  ctx->tagSlot = -1;
  if (!ordered) return 0;
  if (!PT_SPLIT_AUTO) return PT_SPLIT_PCT;
  if (frameCounter == 0) {
    ctx->probeGen++;
    ctx->probeFrame = 0;
    for (int k = 0; k < 4; k++) {
      ctx->probeN[k] = 0;
      ctx->probeMs[k] = 0.0;
      ctx->probeLast[k] = -1;
    }
    const bool keep = ctx->treeDecided >= 0 && ctx->splitDecided >= 0 && ctx->probedKey == ctx->policyKey;
    if (!keep) ctx->treeDecided = ctx->splitDecided = -1;
    // Frames batched per launch (pipelined, RenderParams::nFrames) are not split. A batch's launch
    // holds each tile once per frame, so a costly tile's frames already run side by side, and split
    // items' idle lanes only cost issue slots: c4 without splitting 0.262 -> 0.251 ms at N = 1, its
    // 1/8 share 0.075 -> 0.070 ms (20 frames) and 0.054 -> 0.048 (200 frames, split at 50 %). A launch
    // of one frame (a display() call) is split when the probe found it faster.
    // (launchReorder applies the split only to launches of one frame, renderOne)
#if PT_NO_BATCH_SPLIT_PROBE
    if (ctx->pipe && ctx->batchCap > 1) ctx->splitDecided = 0;
#endif
    ctx->probedKey = ctx->policyKey;
    // split state and cost estimates start over (the camera or scene changed), in every slot's
    // stream order (after its last reorder, before its next frame): this launch's slot on the stream
    // S it runs on (which may be the caller's, renderOne's solo launch), every other slot on its own
    // stream, with that slot's kernelDone recorded after the reset so that a later launch of the
    // slot issued solo on the caller's stream (only once every kernelDone has completed) follows it
    if (ctx->d_cost)
      for (int k = 0; k < (ctx->pipe ? ctx->pipeDepth : 1); k++) {
        const bool own = k == slot || !ctx->pipe;
        hipStream_t sk = own ? S : ctx->slotStream[k];
        (void)hipMemsetAsync(ctx->d_cost + (size_t)k * 4 * ctx->numItems + 2 * (size_t)ctx->numItems, 0,
                             2 * (size_t)ctx->numItems * sizeof(int), sk);
        if (!own && ctx->kernelDone[k]) {
          (void)hipEventRecord(ctx->kernelDone[k], sk);
          ctx->slotBusy[k] = true;
        }
      }
  }
  const int f = ctx->probeFrame < 1000 ? ctx->probeFrame++ : 1000;
  auto avg = [&](int k) { return ctx->probeN[k] ? ctx->probeMs[k] / ctx->probeN[k] : 1e30; };
  if (f == 6 && ctx->treeDecided < 0) {
    foldUpTo(ctx, std::max(ctx->probeLast[0], ctx->probeLast[1]));
    ctx->treeDecided = fastAllowed && avg(0) <= avg(1) ? 1 : 0;
  }
  if (f == 14 && ctx->splitDecided < 0) {
    foldUpTo(ctx, ctx->probeLast[2]);
    ctx->splitDecided = PT_SPLIT_PCT > 0 && avg(2) < avg(ctx->treeDecided ? 0 : 1) ? 1 : 0;
  }
  // this frame's tree, and the probe slot its time goes to
  if (ctx->treeDecided >= 0) {
    *useFast = fastAllowed && ctx->treeDecided;
  } else {
    *useFast = fastAllowed && (f <= 2 || f == 5);
    ctx->tagSlot = (f == 1 || f == 2) ? 0 : (f == 3 || f == 4) ? 1 : -1;
  }
  // this frame's split policy (for the next frame's items)
  if (ctx->splitDecided >= 0) return ctx->splitDecided ? PT_SPLIT_PCT : 0;
  if (f == 11 || f == 12) ctx->tagSlot = 2;
  return f >= 6 && f < 15 ? PT_SPLIT_PCT : 0;
}

static PackParams packParams(const pt_ctx* ctx, int rank, int world);

// the slot streams (and their events) of depth D
static int ensureSlots(pt_ctx* ctx, int D) {
  for (int k = 0; k < D; k++) {
    if (!ctx->slotStream[k]) CK(hipStreamCreateWithFlags(&ctx->slotStream[k], hipStreamNonBlocking));
    if (!ctx->kernelDone[k]) CK(hipEventCreateWithFlags(&ctx->kernelDone[k], hipEventDisableTiming));
  }
  return PT_OK;
}

// One launch: frame frameCounter, or -- pipelined, with no policy probe running and the batch
// not starting a running mean -- up to `want` consecutive frames of the same camera
// (RenderParams::nFrames, at most ctx->batchCap). *done = the frames rendered.
static int renderOne(pt_ctx* ctx, const float eye[3], const float cameraRotate[16], uint32_t frameCounter,
                     int want = 1, int* done = nullptr) {
  if (!ctx) return PT_E_INVALID;
  if (done) *done = 1;
  CK(hipSetDevice(ctx->cfg.device_id));
  const pt_config& c = ctx->cfg;
  unsigned long long* stats = reinterpret_cast<unsigned long long*>(ctx->d_ctl + CTL_STATS);
  hipEvent_t evb, eve;
  if (c.integrator == PT_BASIC_CPU_COMPAT) {
    if (!ctx->d_shapes) return fail(ctx, PT_E_NOSCENE, "no BASIC shapes uploaded");
    const int maxDepth = c.max_bounce >= 0 ? c.max_bounce : 8;  // B:254
    if (maxDepth > BASIC_MAX_DEPTH) return fail(ctx, PT_E_INVALID, "BASIC max_bounce > 31");
    if (int rc = ensureBasicImage(ctx)) return rc;
    if (!ctx->d_overruns) {
      CK(hipMalloc(&ctx->d_overruns, sizeof(unsigned long long)));
      CK(hipMemsetAsync(ctx->d_overruns, 0, sizeof(unsigned long long), ctx->stream));
    }
    int erc = launchEvents(ctx, &evb, &eve);
    if (erc) return erc;
    BasicParams p;
    p.shapes = ctx->d_shapes;
    p.nShapes = ctx->nShapes;
    p.width = c.width;
    p.height = c.height;
    p.sample = sampleIndex(c, frameCounter);
    p.seed = c.basic_seed;
    p.maxDepth = maxDepth;
    p.reset = frameCounter == 0;
    p.brightness = (float)((double)(2.0f * 3.1415926f) * (1.0 / (double)c.basic_samples));  // B:20
    p.accum = ctx->d_accum;
    p.image = ctx->d_basicImg;
    p.stream = ctx->d_stream;
    p.offsets = ctx->d_offsets;
    p.streamN = ctx->streamN;
    p.nOffsets = ctx->nOffsets;
    p.stats = stats;
    p.overruns = ctx->d_overruns;
    CK(hipEventRecord(evb, ctx->stream));
    CK(launchBasic(p, ctx->stream));
    CK(hipEventRecord(eve, ctx->stream));
    commitLaunch(ctx);
    return PT_OK;
  }
  if (!ctx->d_bvh || !eye || !cameraRotate) return fail(ctx, ctx->d_bvh ? PT_E_INVALID : PT_E_NOSCENE, "no scene");
  const bool count = (c.flags & PT_FLAG_COUNT_FETCHES) != 0;
  const bool cull = !count && !(c.flags & PT_FLAG_NO_CULL);
  // default: the lock-step persistent megakernel (also the fetch-counting
  // variant); the path-regeneration kernel on request, and by default for the
  // Disney/MIS integrators on large scenes (pt_kernels.h PT_WIDE_SCENE_MB,
  // WIDE_REGEN_WAVES), whose walks are memory-latency bound and whose long paths
  // leave a lock-step wave's lanes idle
  const size_t sceneBytes = (size_t)ctx->nTri * (PAIR_F4 * 16 + 64 + HIT_F4 * 16) + (size_t)ctx->nDevNodes * 64;
  const bool wideScene = !count && cull && c.integrator != 0 && sceneBytes > ((size_t)PT_WIDE_SCENE_MB << 20);
  // ... and the MIS integrator at its shader's own 2 bounces (IS:861): c3 at 4 hardware queues 0.1443 ->
  // 0.1331 ms per frame on the regen kernel (round 5); deeper MIS paths keep the megakernel (c4, 8
  // bounces: 0.270 vs 0.370)
  const int mbounce = c.max_bounce >= 0 ? c.max_bounce : defaultBounce(c.integrator);
  const bool regenAll = !count && cull &&
                        (ctx->regenWide > 0 ||
                         (ctx->regenWide < 0 && (c.integrator == 0 || (c.integrator == 2 && mbounce <= 2))));
  // this frame's stream and per-frame buffers: slot frameNo % depth, colour buffer
  // frameNo % (depth + 1) when pipelined
  const bool piped = ctx->pipe && !count;
  if (piped) {
    if (int e = ensureSlots(ctx, ctx->pipeDepth)) return e;
  }
  const int D = piped ? ctx->pipeDepth : 1;
  const int slot = piped ? (int)(ctx->frameNo % (unsigned)D) : 0;
  const int nCol = 2 * D + 1;
  const int colIdx = piped ? (int)(ctx->frameNo % (unsigned)nCol) : 0;
  // A launch issued while no other is in flight runs on the caller's stream itself: its camera-ray
  // pass, frame kernel and running-mean update -- and the caller's next work (the gather's pack) --
  // then follow one another in one queue instead of across queues (an event wait between hardware
  // queues costs ~15-18 us per hop; c2's 1/8 share of a 20-frame window is one launch)
  bool solo = piped && ctx->solo;
  if (solo) {
    for (int k = 0; k < D; k++)
      if (ctx->slotBusy[k] && hipEventQuery(ctx->kernelDone[k]) == hipErrorNotReady) solo = false;
    (void)hipGetLastError();  // hipEventQuery's not-ready status is not an error
  }
  // The frame kernel. A single frame issued while nothing else is in flight -- a synchronous
  // display() call (pt_render_frame), SURVEY 8(d)'s per-call time -- runs on the lock-step megakernel,
  // which splits its long tiles and orders its work longest first, where the regen kernel's launch
  // ends in its waves' last paths at falling lane counts: per call c3 0.585 -> 0.373 ms, c2 0.449 ->
  // 0.439 (c4 is on the megakernel already: 0.78; its regen kernel 1.32). Streams of frames keep
  // the regen kernel (c2's batches 0.17 ms per frame). PT_FLAG_REGEN pins the regen kernel.
  const bool oneCall = piped && solo && want == 1 && sceneBytes <= ((size_t)PT_WIDE_SCENE_MB << 20) &&
                       ctx->regenWide <= 0 && PT_CALL_MEGAKERNEL;
  const bool regen = !count && ((c.flags & PT_FLAG_REGEN) ||
                                ((wideScene || (regenAll && !oneCall)) && !(c.flags & PT_FLAG_MEGAKERNEL)));
  hipStream_t S = piped && !solo ? ctx->slotStream[slot] : ctx->stream;
  // every other slot's frame in flight has ended on S (the frames that read buffers
  // rebuilt below)
  auto waitOthers = [&]() -> int {
    for (int k = 0; k < D; k++)
      if (k != slot && ctx->slotBusy[k]) CK(hipStreamWaitEvent(S, ctx->kernelDone[k], 0));
    return PT_OK;
  };
  int nb = 0;
  // the more-waves variant of either kernel (the regen kernel's with its 4-wide walk, dynamic ray
  // fetch and camera-ray pass; on small trees with the whole tree in LDS)
  const bool wide = wideScene || (regen && regenAll);
  const bool walk4 = wide && ctx->fast4Ready && !(c.flags & PT_FLAG_REFERENCE_TREE);
  RegenShape rs;
  if (regen) {
    CK(regenShape(c.integrator, cull, wide, walk4 ? ctx->f4nDev : 0, !wideScene, &rs));
    nb = rs.blocksPerCU;
  } else {
    CK(renderBlocksPerCU(c.integrator, cull, count, wide, &nb));
  }
  if (nb < 1) nb = 1;
  const int bs = regen ? rs.block : BLOCK;  // threads per block
  ctx->lastWaves = nb * bs / 64 / 4;  // 4 SIMDs per CU
  ctx->lastRegen = regen;
  // Frames in flight share the GPU by space, not by time: a frame's persistent grid is
  // residency / (frames in flight), so the frames' waves are all resident together and a
  // frame whose long paths keep a few waves busy leaves the rest of the machine to the
  // others (and to the running-mean updates). A persistent grid sized to all of residency
  // keeps the next frame's waves -- and every other launch -- waiting for its tail: c4
  // 0.48 -> 0.34 ms per frame at 8 frames in flight, c2's 1/8 screen share 0.096 -> 0.072.
  // A caller that waits for every frame gets the whole machine for each.
  const int fullGrid = ctx->numCU * nb;
  int grid = fullGrid;
  // While other frames are in flight, each frame's grid is PT_GRID_PCT % of its equal share: a frame
  // finishing early leaves waves of the others ready to take its place (round 4, against 100 /
  // 200 / 300 % with the bench line as the driver runs it, 20 frames from an idle GPU: c2 0.285 /
  // 0.262 / 0.266 / 0.289 ms per frame at 100 / 150 / 200 / 300, c4 0.413 / 0.360 / 0.367 / 0.385;
  // round 5's batched launches prefer 125, PT_GRID_PCT).
  // The share follows the launches actually in flight, PT_GRID_PCT % / (1 + the others running):
  // a launch issued into a filling pipeline (the first batches after an idle GPU) takes the
  // machine the earlier ones leave as they drain, and a full pipeline gets PT_GRID_PCT % / D each.
  // 20 frames from an idle GPU, one rank's share of an N-way split (profiles/r4/shard_time_h20.jsonl,
  // 2 runs each): c2 N = 4 0.129-0.130 -> 0.072 ms per frame, N = 8 0.061 -> 0.046-0.048, c4 N = 4
  // 0.137 -> 0.109-0.113; N = 1, 2 and 200-frame runs within run-to-run spread.
#ifndef PT_GRID_PCT
#define PT_GRID_PCT 125  // round 5, final kernels: c4 0.2571 -> 0.2463 ms at 150 -> 125, its 1/8 share 0.0721 -> 0.0688, c2's 0.0332 -> 0.0325; 175: c2 +3 %
#endif
#ifndef PT_GRID_PCT_WIDE
#define PT_GRID_PCT_WIDE 150  // large scenes (c5: two frames per launch, ~8 ms launches): 4.44 ms at 125
#endif
  const int GRID_PCT = wideScene ? PT_GRID_PCT_WIDE : PT_GRID_PCT;
  if (piped && D > 1) {
    int others = 0;  // other launches still in flight: the caller streams frames
    for (int k = 0; k < D; k++)
      others += k != slot && ctx->slotBusy[k] && hipEventQuery(ctx->kernelDone[k]) == hipErrorNotReady;
    (void)hipGetLastError();  // hipEventQuery's not-ready status is not an error
    if (others > 0) grid = std::min(fullGrid, std::max(NUM_QUEUES, fullGrid * GRID_PCT / (100 * (others + 1))));
  }
  int ovfDepth = 0;
  int rc = ensureOverflow(ctx, (size_t)fullGrid * bs, &ovfDepth, regen ? regenLdsStack() : LDS_STACK, D);
  if (rc) return rc;
  // the colour buffer's previous launch (nCol back) has been mixed (the slot's queue counters,
  // order list and camera-ray results belong to its previous launch on this same stream)
  if (piped && ctx->frameNo >= (unsigned long long)nCol && !(S == ctx->stream && ctx->lastMixStream == S))
    CK(hipStreamWaitEvent(S, ctx->mixDone[colIdx], 0));
  int* queue = reinterpret_cast<int*>(ctx->d_ctl + CTL_QUEUES) + (size_t)slot * NUM_QUEUES * CTL_LINE_INTS;
  RenderParams p;
  std::memset(&p, 0, sizeof(p));
  p.scene = sceneView(ctx);
  p.env.hdr = ctx->d_hdr;
  p.env.cache = ctx->d_cache;
  p.env.hdr8 = ctx->d_hdr8;
  p.env.cache4 = ctx->d_cache4;
  // the table by rows for the megakernel's frames when the table outgrows an XCD's L2 share: c4's
  // frame kernel 216 -> 147 MB DRAM-side per frame, time unchanged (0.2914 / 0.2927 ms); its extra
  // dependent load costs the regen kernels more than their misses (c5 4.20 -> 4.31 ms, c3 0.1083 -> 0.111)
#ifndef PT_ROW_TABLE
#define PT_ROW_TABLE 1  // 0: never, 1: the megakernel's frames, 2: every frame (when the table outgrows 4 MB)
#endif
  const bool rowTable = PT_ROW_TABLE > 0 && (PT_ROW_TABLE == 2 || !regen) &&
                        (size_t)ctx->hdrW * ctx->hdrH * sizeof(uint32_t) > ((size_t)4 << 20);
  p.env.cacheRow = rowTable ? ctx->d_cacheRow : nullptr;
  p.env.cacheY = rowTable ? ctx->d_cacheY : nullptr;
  p.env.trig = ctx->d_trig;
  p.env.light = ctx->d_light;  // every scene: c5 too (4.25 vs 4.49 ms without the table, round 6)
  p.env.w = ctx->hdrW;
  p.env.h = ctx->hdrH;
  p.env.res = ctx->hdrW;
  p.env.nt = sceneBytes > ((size_t)PT_WIDE_SCENE_MB << 20) ? 1 : 0;
  p.width = c.width;
  p.height = c.height;
  p.frameCounter = frameCounter;
  p.sampleIndex = sampleIndex(c, frameCounter);
  p.maxBounce = c.max_bounce >= 0 ? c.max_bounce : defaultBounce(c.integrator);
  std::memcpy(p.eye, eye, sizeof(p.eye));
  std::memcpy(p.cam, cameraRotate, sizeof(p.cam));
  p.accum = ctx->d_accum;
  p.queue = queue;
  p.perQueue = ctx->perQueue;
  p.numItems = ctx->numItems;
  p.shardSize = ctx->shardSize;
  p.shardTiles = (ctx->shardSize / 8) * (ctx->shardSize / 8);
  p.shardsX = ctx->shardsX;
  p.rank = c.tile_rank;
  p.world = c.tile_world;
  p.ovf = ovfDepth ? ctx->d_ovf + (size_t)slot * fullGrid * bs * ovfDepth : nullptr;
  p.ovfDepth = ovfDepth;
  p.scene.fast = 0;  // probePolicy below

  p.stats = stats;
  p.rayShards = reinterpret_cast<unsigned long long*>(ctx->d_ctl + CTL_RAYS);
  // longest-tiles-first: each band's tiles in the order of the previous frame's cost
  const int group = std::max(1, PT_TILE_GROUP);
  const bool ordered = !regen && !count && !(c.flags & PT_FLAG_NO_TILE_ORDER) &&
                       (ctx->perQueue + group - 1) / group <= REORDER_MAX && ctx->numItems < (1 << 22);
  const int orderCap = 4 * ctx->perQueue + 64;  // room for the items of split tiles
  const size_t orderInts = (size_t)NUM_QUEUES * orderCap + NUM_QUEUES;
  ctx->orderCap = orderCap;
  if (ordered && !ctx->d_cost) {
    // per slot and tile: summed item cost, longest item, split state, cost estimate
    // (reorderKernel reads and zeroes the costs)
    const size_t n = (size_t)PIPE * ctx->numItems * 4;
    CK(hipMalloc(&ctx->d_cost, n * sizeof(int)));
    CK(hipMemset(ctx->d_cost, 0, n * sizeof(int)));
    // per slot and band: orderCap work items, then the NUM_QUEUES item counts (reorderKernel)
    CK(hipMalloc(&ctx->d_order, (size_t)PIPE * orderInts * sizeof(int)));
    for (int k = 0; k < PIPE; k++) ctx->orderValid[k] = false;
  }
  int* cost = ordered ? ctx->d_cost + (size_t)slot * 4 * ctx->numItems : nullptr;
  int* order = ordered ? ctx->d_order + (size_t)slot * orderInts : nullptr;
  // the tree (the runtime's own, checked against the uploaded one, unless asked
  // not to) and the split policy: probePolicy
  bool useFast = false;
  const int splitPct = probePolicy(ctx, frameCounter, ordered,
                                   !count && !regen && ctx->fastReady && !(c.flags & PT_FLAG_REFERENCE_TREE), &useFast,
                                   slot, S);
  // the large-scene regen kernel walks the 4-wide runtime tree (checked against the uploaded one)
  if (regen && walk4) useFast = true;
  if (regen && wide)  // its own LDS copy's size: the top of the tree, or all of it
    p.scene.f4nTop = rs.fullTree ? ctx->f4nDev : std::min(regenTop4(rs, c.integrator), ctx->f4nDev);
  p.scene.fast = useFast ? 1 : 0;
  ctx->lastFast = useFast;
  // While the policy probe times frames (PT_SPLIT_AUTO, 20 frames after a restart) a pipelined
  // frame starts only after the previous one has ended, and each launch is one frame.
  const bool probing = ordered && PT_SPLIT_AUTO &&
                       (ctx->treeDecided < 0 || ctx->splitDecided < 0);
  const int nF = piped && !probing ? std::max(1, std::min(want, ctx->batchCap)) : 1;
  if (done) *done = nF;
  p.nFrames = nF;
  // One megakernel frame issued while no other launch is in flight (a display() call, SURVEY 8(d)'s
  // per-call time): the kernel mixes each pixel's sample into the running mean itself (IS:868-871;
  // one writer per pixel, the previous frame's update is ordered before it on the caller's stream)
  // -- no colour buffer round trip and no running-mean update launch: c4 per call 0.785 -> 0.772 ms.
  // The regen kernel keeps the update launch: the read of the running mean at each path's end stalls
  // its lock-step waves (c2 0.455 either way, c3 0.578 -> 0.587 ms)
  const bool direct = piped && solo && nF == 1 && !regen && PT_DIRECT_SOLO;
  if (direct && ctx->mixPending && ctx->lastMixStream != S) CK(hipStreamWaitEvent(S, ctx->mixDone[ctx->lastCol], 0));
  p.sampleStride = c.sample_world > 0 ? (uint32_t)c.sample_world : 1u;
  // per-frame buffers indexed by the pixel's slot in this context's share (shareIndex): a 1/N share's
  // colour and camera-ray buffers are 1/N of a frame (c5 at N = 8, 16 frames per launch: ~2.4 GB of
  // colour buffers instead of ~19 GB)
  const size_t shareN = (size_t)ctx->numItems * 64;
  p.colStride = shareN;
  // every colour buffer (and below, every slot's camera-ray results) allocated at the first launch that
  // uses any, so no later launch -- a timed one -- waits for an allocation (c2's 1/8 share: a 19 us
  // hipMalloc before the sixth launch's first kernel)
  if (piped)
    for (int k = 0; k < nCol; k++)
      if (!ctx->d_col[k]) {
        const int cap = std::max(nF, ctx->batchCap);
        CK(hipMalloc(&ctx->d_col[k], (size_t)cap * shareN * COL_F * sizeof(float)));
        ctx->colCap[k] = cap;
      }
  if (piped && ctx->colCap[colIdx] < nF) {  // room for the launch's frames (each buffer grows once, to batchCap)
    if (ctx->d_col[colIdx]) {
      CK(hipEventSynchronize(ctx->mixDone[colIdx]));  // its last frames' running-mean update has read it
      dfree(ctx->d_col[colIdx]);
    }
    const int cap = std::max(nF, ctx->batchCap);
    CK(hipMalloc(&ctx->d_col[colIdx], (size_t)cap * shareN * COL_F * sizeof(float)));
    ctx->colCap[colIdx] = cap;
  }
  p.col = piped && !direct ? ctx->d_col[colIdx] : nullptr;
  p.packets = PT_PACKETS && (p.scene.fast ? ctx->fDepth : ctx->depth) + 1 <= PKT_DEPTH;
  // camera-ray bins, rebuilt when the camera or the scene changed (the previous frame
  // has ended first: it may still read the old bins); they need the reference facts
  // refReachable checks a bin's winner against
  // The camera-ray pass (primaryKernel) traces the camera rays ahead of the frame kernel: on
  // request, and by default for the large-scene regen kernel (c5 7.52 -> 6.86 ms), whose lanes
  // then start from the camera ray's hit; the megakernel is faster with its camera rays inside
  // (c2 0.372 vs 0.383 ms with the pass)
  const bool pass = (c.flags & PT_FLAG_PRIMARY_PASS) || (regen && wide);
  const bool bins = PT_BINS && !count && ctx->fastReady && !(c.flags & PT_FLAG_NO_BINS) && (!regen || pass);
  if (bins) {
    if (!ctx->binsValid || ctx->binVersion != ctx->sceneVersion || std::memcmp(ctx->binEye, eye, sizeof(ctx->binEye)) ||
        std::memcmp(ctx->binCam, cameraRotate, sizeof(ctx->binCam))) {
      if (piped) {
        if (int e = waitOthers()) return e;
      }
      ctx->binsValid = false;
      CK(buildPrimaryBins(eye, cameraRotate, c.width, c.height, ctx->d_geo, ctx->d_leafBox, ctx->nTri, ctx->bins, S));
      std::memcpy(ctx->binEye, eye, sizeof(ctx->binEye));
      std::memcpy(ctx->binCam, cameraRotate, sizeof(ctx->binCam));
      ctx->binVersion = ctx->sceneVersion;
      ctx->binsValid = true;
      if (piped) {
        CK(hipEventRecord(ctx->binsBuilt, S));
        ctx->binGen++;
        ctx->binGenSeen[slot] = ctx->binGen;
      }
    }
    // a frame in flight on the other slot's stream must not read bins still being built
    if (piped && ctx->binGenSeen[slot] != ctx->binGen) {
      CK(hipStreamWaitEvent(S, ctx->binsBuilt, 0));
      ctx->binGenSeen[slot] = ctx->binGen;
    }
    p.binStart = ctx->bins.binStart;
    p.binTris = ctx->bins.binTris;
    p.binGeo = ctx->bins.binGeo;
    p.binBox = ctx->bins.binBox;
    p.binTilesX = ctx->bins.tilesX;
    p.binTilesY = ctx->bins.tilesY;
    if (pass) {
      // per frame: the share's entries (shareN int2, compacted per wave tile), then its numItems tile masks
      const size_t primBytes = shareN * sizeof(int2) + (size_t)ctx->numItems * sizeof(unsigned long long);
      if (piped)
        for (int k = 0; k < D; k++)
          if (!ctx->d_prim[k]) {
            const int cap = std::max(nF, ctx->batchCap);
            CK(hipMalloc(&ctx->d_prim[k], (size_t)cap * primBytes));
            ctx->primCap[k] = cap;
          }
      if (ctx->primCap[slot] < nF) {  // the slot's previous launch (on S) may still read the old results
        if (ctx->d_prim[slot]) {
          CK(hipStreamSynchronize(S));
          dfree(ctx->d_prim[slot]);
        }
        const int cap = std::max(nF, piped ? ctx->batchCap : 1);
        CK(hipMalloc(&ctx->d_prim[slot], (size_t)cap * primBytes));
        ctx->primCap[slot] = cap;
      }
      p.primHit = ctx->d_prim[slot];
      p.primMask = reinterpret_cast<unsigned long long*>(ctx->d_prim[slot] + (size_t)ctx->primCap[slot] * shareN);
    }
  }
  // a frame in band order (probePolicy) records no costs and launches no reorder; the
  // slot's last order list stays valid for its next ordered frame (any list covers every tile)
  // Batches of frames run unsplit (probePolicy) -- also on small screen-tile shares, whose launch lasts
  // about as long as its longest unsplit tile (c4's 1/8 share, 20 frames in one 1.3 ms launch: single
  // 8x8 tiles of 1.2-1.5 ms): splitting there measured c4 N = 8 0.0726 -> 0.0688 ms per frame over 20
  // frames but 0.0484 -> 0.0549 over 200, N = 4 0.0867 -> 0.0962 (round 6, not kept)
  const bool splitThis = nF == 1;
  // (a batch does not run the split items a one-frame launch's reorder listed: band order, once)
  p.tileOrder = ordered && ctx->orderValid[slot] && !(!splitThis && ctx->orderSplit[slot]) ? order : nullptr;
  p.orderCap = orderCap;
  p.tileCost = ordered ? cost : nullptr;
  p.tileCostMax = ordered ? cost + ctx->numItems : nullptr;
  if (piped && probing) {
    if (int e = waitOthers()) return e;
  }
  int erc = launchEvents(ctx, &evb, &eve);
  if (erc) return erc;
#if PT_WAVE_TRACE
  // diagnostics build: each wave's {start, end, tiles | longest tile's pixel << 32,
  // longest tile's duration, its most node-loop / leaf-loop iterations of a lane} (100 MHz wall
  // clock), appended per frame to $PT_WAVE_TRACE_FILE (tools/wave_trace.py)
  const size_t nTrace = (size_t)grid * (bs / 64) * WAVE_TRACE_WORDS;
  unsigned long long* dTrace = nullptr;
  {
    CK(hipMalloc(&dTrace, nTrace * sizeof(unsigned long long)));
    CK(hipMemsetAsync(dTrace, 0, nTrace * sizeof(unsigned long long), S));
  }
  p.waveTrace = dTrace;
#endif
  // the slot's work-queue counters zeroed for this launch: by the camera-ray pass (block 0), else by a memset
  p.zeroQueue = p.primHit != nullptr;
  if (!p.primHit) CK(hipMemsetAsync(queue, 0, (size_t)NUM_QUEUES * CTL_LINE_INTS * sizeof(int), S));
  CK(hipEventRecord(evb, S));
  if (p.primHit) CK(launchPrimary(p, S));
  if (regen) CK(launchRegen(p, c.integrator, grid, S, cull, rs));
  else CK(launchRender(p, c.integrator, grid, S, cull, count, wide));
#if PT_WAVE_TRACE
  if (dTrace) {
    std::vector<unsigned long long> tr(nTrace);
    CK(hipMemcpyAsync(tr.data(), dTrace, nTrace * sizeof(unsigned long long), hipMemcpyDeviceToHost, S));
    CK(hipStreamSynchronize(S));
    (void)hipFree(dTrace);
    if (const char* fn = std::getenv("PT_WAVE_TRACE_FILE")) {
      if (FILE* f = std::fopen(fn, "ab")) {
        std::fwrite(tr.data(), sizeof(unsigned long long), nTrace, f);
        std::fclose(f);
      }
    }
  }
#endif
  if (ordered) {
    CK(launchReorder(cost, cost + ctx->numItems, cost + 2 * (size_t)ctx->numItems, cost + 3 * (size_t)ctx->numItems,
                     order, ctx->perQueue, orderCap, ctx->numItems, group, grid * (BLOCK / 64), splitThis ? splitPct : 0, S));
    ctx->orderValid[slot] = true;
    ctx->orderSplit[slot] = splitThis && splitPct > 0;
  }
  // kernel_ms: the frame's own kernels (camera-ray pass, frame kernel, reorder), so the
  // policy probe weighs the order's cost too; the running-mean update below is not in it
  CK(hipEventRecord(eve, S));
  if (piped) {
    // the running-mean updates on the caller's stream, in frame order, after this launch's kernel
    CK(hipEventRecord(ctx->kernelDone[slot], S));
    ctx->slotBusy[slot] = true;
    if (S != ctx->slotStream[slot])  // the slot's resources: its stream's later work follows this launch
      CK(hipStreamWaitEvent(ctx->slotStream[slot], ctx->kernelDone[slot], 0));
    if (S != ctx->stream) CK(hipStreamWaitEvent(ctx->stream, ctx->kernelDone[slot], 0));
    if (ctx->mixPending && ctx->lastMixStream != ctx->stream)  // the caller switched streams: keep frame order
      CK(hipStreamWaitEvent(ctx->stream, ctx->mixDone[ctx->lastCol], 0));
    ctx->lastMixStream = ctx->stream;
    if (!direct)
      CK(launchMix(packParams(ctx, c.tile_rank, c.tile_world), ctx->d_accum, ctx->d_col[colIdx], shareN, nF,
                   frameCounter, ctx->stream));
    CK(hipEventRecord(ctx->mixDone[colIdx], ctx->stream));  // direct: the frame's kernels updated it
    ctx->lastSlot = slot;
    ctx->lastCol = colIdx;
    ctx->mixPending = true;
    ctx->frameNo++;
  }
  commitLaunch(ctx, nF);
  return PT_OK;
}

// the caller's stream waits for the last pipelined frame's running-mean update
static int joinPipe(pt_ctx* ctx) {
  if (!ctx->mixPending) return PT_OK;
  CK(hipSetDevice(ctx->cfg.device_id));
  CK(hipStreamWaitEvent(ctx->stream, ctx->mixDone[ctx->lastCol], 0));
  return PT_OK;
}

// every stream the context renders on, then its own: all work done
static int syncStreams(pt_ctx* ctx) {
  CK(hipSetDevice(ctx->cfg.device_id));
  for (int k = 0; k < PIPE; k++) {
    if (ctx->slotStream[k]) CK(hipStreamSynchronize(ctx->slotStream[k]));
    ctx->slotBusy[k] = false;
  }
  CK(hipStreamSynchronize(ctx->stream));
  ctx->mixPending = false;
  return PT_OK;
}

static int groupGather(pt_ctx* ctx);

int pt_render_frame_async(pt_ctx* ctx, const float eye[3], const float cameraRotate[16], uint32_t frameCounter) {
  return pt_render_frames_async(ctx, eye, cameraRotate, frameCounter, 1);
}

int pt_render_frames_async(pt_ctx* ctx, const float eye[3], const float cameraRotate[16], uint32_t frameCounter,
                           int nFrames) {
  if (!ctx || nFrames < 0) return PT_E_INVALID;
  while (nFrames > 0) {
    int done = 1;
    if (ctx->peers.empty()) {
      if (int rc = renderOne(ctx, eye, cameraRotate, frameCounter, nFrames, &done)) return rc;
    } else {
      // a device group: every device renders its tiles of the frame on its own stream; then the
      // gather (GroupGather), frame by frame
      for (pt_ctx* m : members(ctx))
        if (int rc = renderOne(m, eye, cameraRotate, frameCounter)) return fromPeer(ctx, m, rc);
      if (int rc = groupGather(ctx)) return rc;
    }
    frameCounter += (uint32_t)done;
    nFrames -= done;
  }
  return PT_OK;
}

int pt_render_frame(pt_ctx* ctx, const float eye[3], const float cameraRotate[16], uint32_t frameCounter,
                    float* accum_rgba) {
  int rc = pt_render_frame_async(ctx, eye, cameraRotate, frameCounter);
  if (rc) return rc;
  if (accum_rgba) return pt_download_accum(ctx, accum_rgba);
  return pt_synchronize(ctx);
}

int pt_trace_closest(pt_ctx* ctx, const float* rays, int n, float* t_out, int* tri_out) {
  if (!ctx || n < 0 || (n > 0 && (!rays || !t_out || !tri_out))) return PT_E_INVALID;
  if (!ctx->d_bvh) return fail(ctx, PT_E_NOSCENE, "no scene");
  if (n == 0) return PT_OK;
  // frames in flight read the overflow stack this query reuses (and ensureOverflow may
  // reallocate): the query runs after every frame issued before it
  if (int rc = syncStreams(ctx)) return rc;
  if ((size_t)n > ctx->traceCap) {
    dfree(ctx->d_rays); dfree(ctx->d_t); dfree(ctx->d_tri);
    CK(hipMalloc(&ctx->d_rays, (size_t)n * 6 * sizeof(float)));
    CK(hipMalloc(&ctx->d_t, (size_t)n * sizeof(float)));
    CK(hipMalloc(&ctx->d_tri, (size_t)n * sizeof(int)));
    ctx->traceCap = n;
  }
  const bool cull = !(ctx->cfg.flags & (PT_FLAG_NO_CULL | PT_FLAG_COUNT_FETCHES));
  int grid = (int)std::min<long>(((long)n + BLOCK - 1) / BLOCK, (long)ctx->numCU * 8);
  int ovfDepth = 0;
  int rc = ensureOverflow(ctx, (size_t)grid * BLOCK, &ovfDepth);
  if (rc) return rc;
  CK(hipMemcpyAsync(ctx->d_rays, rays, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
  TraceParams p;
  p.scene = sceneView(ctx);
  // the runtime's own tree, results reference-exact (pt_trace.h refReachable)
  p.scene.fast = ctx->fastReady && !(ctx->cfg.flags & (PT_FLAG_REFERENCE_TREE | PT_FLAG_COUNT_FETCHES)) ? 1 : 0;
  p.rays = ctx->d_rays;
  p.n = n;
  p.t = ctx->d_t;
  p.tri = ctx->d_tri;
  p.ovf = ovfDepth ? ctx->d_ovf : nullptr;
  p.ovfDepth = ovfDepth;
  CK(launchTrace(p, grid, ctx->stream, cull));
  CK(hipMemcpyAsync(t_out, ctx->d_t, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipMemcpyAsync(tri_out, ctx->d_tri, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return PT_OK;
}

// a device group's rank-0 stream waits for the last gather (the whole image is in its accumulation)
static int joinGather(pt_ctx* ctx) {
  GroupGather* g = ctx->gather;
  if (!g || !g->pending) return PT_OK;
  CK(hipSetDevice(ctx->cfg.device_id));
  CK(hipStreamWaitEvent(ctx->stream, g->done, 0));
  return PT_OK;
}

int pt_download_accum(pt_ctx* ctx, float* accum) {
  if (!ctx || !accum) return PT_E_INVALID;
  if (int rc = joinGather(ctx)) return rc;
  if (int rc = joinPipe(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  const size_t bytes = (size_t)ctx->cfg.width * ctx->cfg.height * sizeof(float4);
  CK(hipMemcpyAsync(accum, ctx->d_accum, bytes, hipMemcpyDefault, ctx->stream));  // host or device
  CK(hipStreamSynchronize(ctx->stream));
  return PT_OK;
}

// the BASIC double image (basicKernel adds each sample to it), allocated and zeroed on first use
static int ensureBasicImage(pt_ctx* ctx) {
  if (ctx->d_basicImg) return PT_OK;
  const size_t n = (size_t)ctx->cfg.width * ctx->cfg.height * 3;
  CK(hipMalloc(&ctx->d_basicImg, n * sizeof(double)));
  CK(hipMemsetAsync(ctx->d_basicImg, 0, n * sizeof(double), ctx->stream));
  return PT_OK;
}

static int uploadAccumOne(pt_ctx* ctx, const float* accum) {
  if (int rc = joinPipe(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  const size_t npix = (size_t)ctx->cfg.width * ctx->cfg.height;
  CK(hipMemcpyAsync(ctx->d_accum, accum, npix * sizeof(float4), hipMemcpyDefault, ctx->stream));  // host or device
  if (ctx->cfg.integrator == PT_BASIC_CPU_COMPAT) {  // basicKernel continues from its double image: the sums, widened
    if (int rc = ensureBasicImage(ctx)) return rc;
    CK(launchBasicWiden(ctx->d_accum, ctx->d_basicImg, (long)npix, ctx->stream));
  }
  CK(hipStreamSynchronize(ctx->stream));
  return PT_OK;
}

int pt_upload_basic_image(pt_ctx* ctx, const double* rgb) {
  if (!ctx || !rgb) return PT_E_INVALID;
  if (ctx->cfg.integrator != PT_BASIC_CPU_COMPAT) return fail(ctx, PT_E_INVALID, "not a BASIC context");
  if (int rc = syncStreams(ctx)) return rc;
  if (int rc = ensureBasicImage(ctx)) return rc;
  const size_t npix = (size_t)ctx->cfg.width * ctx->cfg.height;
  CK(hipMemcpyAsync(ctx->d_basicImg, rgb, npix * 3 * sizeof(double), hipMemcpyDefault, ctx->stream));
  CK(launchBasicNarrow(ctx->d_basicImg, ctx->d_accum, (long)npix, ctx->stream));  // the f32 sums, as a frame leaves them
  CK(hipStreamSynchronize(ctx->stream));
  return PT_OK;
}

// (every device of a group takes the whole image: each continues the running mean of its own tiles)
int pt_upload_accum(pt_ctx* ctx, const float* accum) {
  if (!ctx || !accum) return PT_E_INVALID;
  if (int rc = joinGather(ctx)) return rc;
  for (pt_ctx* m : members(ctx))
    if (int rc = uploadAccumOne(m, accum)) return fromPeer(ctx, m, rc);
  return PT_OK;
}

int pt_clear_accum(pt_ctx* ctx) {
  if (!ctx) return PT_E_INVALID;
  if (int rc = joinGather(ctx)) return rc;
  for (pt_ctx* m : members(ctx)) {
    if (int rc = joinPipe(m)) return fromPeer(ctx, m, rc);
    if (hipSetDevice(m->cfg.device_id) != hipSuccess ||
        hipMemsetAsync(m->d_accum, 0, (size_t)m->cfg.width * m->cfg.height * sizeof(float4), m->stream) != hipSuccess)
      return fail(ctx, PT_E_HIP, "pt_clear_accum on device " + std::to_string(m->cfg.device_id));
    if (m->d_basicImg &&
        hipMemsetAsync(m->d_basicImg, 0, (size_t)m->cfg.width * m->cfg.height * 3 * sizeof(double), m->stream) != hipSuccess)
      return fail(ctx, PT_E_HIP, "pt_clear_accum (BASIC image)");
  }
  // a group's next gather unpacks into rank 0's accumulation on the gather stream, which
  // is not ordered after rank 0's stream: the clear completes first
  if (ctx->gather) {
    CK(hipSetDevice(ctx->cfg.device_id));
    CK(hipStreamSynchronize(ctx->stream));
  }
  return PT_OK;
}

int pt_accum_device_ptr(pt_ctx* ctx, void** dptr) {
  if (!ctx || !dptr) return PT_E_INVALID;
  *dptr = ctx->d_accum;
  return PT_OK;
}

int pt_tonemap(pt_ctx* ctx, float limit, float gamma, float* rgb_out) {
  if (!ctx || !rgb_out || !(limit > 0.0f)) return PT_E_INVALID;
  if (int rc = joinGather(ctx)) return rc;
  if (int rc = joinPipe(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  const int n = ctx->cfg.width * ctx->cfg.height;
  if (!ctx->d_rgb) CK(hipMalloc(&ctx->d_rgb, (size_t)n * 3 * sizeof(float)));
  CK(launchTonemap(ctx->d_accum, ctx->d_rgb, n, limit, gamma, ctx->stream));
  CK(hipMemcpyAsync(rgb_out, ctx->d_rgb, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  return PT_OK;
}

static PackParams packParams(const pt_ctx* ctx, int rank, int world) {
  PackParams p;
  p.width = ctx->cfg.width;
  p.height = ctx->cfg.height;
  p.shardSize = ctx->shardSize;
  p.shardsX = ctx->shardsX;
  p.rank = rank;
  p.world = world;
  const int numShards = ctx->shardsX * ctx->shardsY;
  const long owned = (numShards - rank + world - 1) / world;
  p.count = owned * (long)ctx->shardSize * ctx->shardSize;
  return p;
}

int pt_owned_pixel_count(pt_ctx* ctx, int rank, int world, int64_t* count) {
  if (!ctx || !count || world < 1 || rank < 0 || rank >= world) return PT_E_INVALID;
  if (!ctx->peers.empty()) return fail(ctx, PT_E_INVALID, "device groups gather inside pt_render_frame");
  *count = packParams(ctx, rank, world).count;
  return PT_OK;
}

int pt_pack_owned(pt_ctx* ctx, void* dpacked) {
  if (!ctx || !dpacked) return PT_E_INVALID;
  if (!ctx->peers.empty()) return fail(ctx, PT_E_INVALID, "device groups gather inside pt_render_frame");
  if (int rc = joinPipe(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  PackParams p = packParams(ctx, ctx->cfg.tile_rank, ctx->cfg.tile_world);
  CK(launchPack(p, ctx->d_accum, reinterpret_cast<float*>(dpacked), ctx->stream));
  return PT_OK;
}

int pt_display_pack(pt_ctx* ctx, float limit, float gamma, void* dpacked) {
  if (!ctx || !dpacked || !(limit > 0.0f)) return PT_E_INVALID;
  if (!ctx->peers.empty()) return fail(ctx, PT_E_INVALID, "device groups gather inside pt_render_frame");
  if (int rc = joinPipe(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  PackParams p = packParams(ctx, ctx->cfg.tile_rank, ctx->cfg.tile_world);
  CK(launchDisplayPack(p, ctx->d_accum, limit, gamma, reinterpret_cast<uint8_t*>(dpacked), ctx->stream));
  return PT_OK;
}

int pt_display_own(pt_ctx* ctx, float limit, float gamma, void* dimage) {
  if (!ctx || !dimage || !(limit > 0.0f)) return PT_E_INVALID;
  if (!ctx->peers.empty()) return fail(ctx, PT_E_INVALID, "device groups gather inside pt_render_frame");
  if (int rc = joinPipe(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  PackParams p = packParams(ctx, ctx->cfg.tile_rank, ctx->cfg.tile_world);
  CK(launchDisplayOwn(p, ctx->d_accum, limit, gamma, reinterpret_cast<uchar4*>(dimage), ctx->stream));
  return PT_OK;
}

int pt_display_unpack(pt_ctx* ctx, int world, const void* const* dpacked, void* dimage) {
  if (!ctx || !dpacked || !dimage || world < 1 || world > DISPLAY_MAX_WORLD) return PT_E_INVALID;
  if (!ctx->peers.empty()) return fail(ctx, PT_E_INVALID, "device groups gather inside pt_render_frame");
  CK(hipSetDevice(ctx->cfg.device_id));
  RanksUnpack d;
  std::memset(&d, 0, sizeof(d));
  d.base = packParams(ctx, 0, world);
  for (int k = 1; k < world; k++) {
    d.src[k] = dpacked[k];
    d.count[k] = packParams(ctx, k, world).count;
  }
  CK(launchDisplayUnpack(d, world, reinterpret_cast<uchar4*>(dimage), ctx->stream));
  return PT_OK;
}

int pt_unpack_ranks(pt_ctx* ctx, int world, const void* const* dpacked) {
  if (!ctx || !dpacked || world < 1 || world > DISPLAY_MAX_WORLD) return PT_E_INVALID;
  if (!ctx->peers.empty()) return fail(ctx, PT_E_INVALID, "device groups gather inside pt_render_frame");
  if (int rc = joinPipe(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  RanksUnpack d;
  std::memset(&d, 0, sizeof(d));
  d.base = packParams(ctx, 0, world);
  for (int k = 1; k < world; k++) {
    d.src[k] = dpacked[k];
    d.count[k] = packParams(ctx, k, world).count;
  }
  CK(launchUnpackRanks(d, world, ctx->d_accum, ctx->stream));
  return PT_OK;
}

int pt_unpack_rank(pt_ctx* ctx, int rank, int world, const void* dpacked) {
  if (!ctx || !dpacked || world < 1 || rank < 0 || rank >= world) return PT_E_INVALID;
  if (!ctx->peers.empty()) return fail(ctx, PT_E_INVALID, "device groups gather inside pt_render_frame");
  if (int rc = joinPipe(ctx)) return rc;
  CK(hipSetDevice(ctx->cfg.device_id));
  PackParams p = packParams(ctx, rank, world);
  CK(launchUnpack(p, ctx->d_accum, reinterpret_cast<const float*>(dpacked), ctx->stream));
  return PT_OK;
}

int pt_set_stream(pt_ctx* ctx, void* s) {
  if (!ctx) return PT_E_INVALID;
  ctx->stream = s ? reinterpret_cast<hipStream_t>(s) : ctx->own;
  return PT_OK;
}

static int syncOne(pt_ctx* ctx) { return syncStreams(ctx); }

// a group: every device's render stream, the gather's streams, then rank 0's stream
static int syncGroup(pt_ctx* ctx) {
  for (pt_ctx* p : ctx->peers)
    if (int rc = syncOne(p)) return fromPeer(ctx, p, rc);
  if (GroupGather* g = ctx->gather) {
    for (auto& P : g->peer)
      if (P.mstream) {
        CK(hipSetDevice(P.dev));
        CK(hipStreamSynchronize(P.mstream));
      }
    CK(hipSetDevice(ctx->cfg.device_id));
    CK(hipStreamSynchronize(g->cstream));
    g->pending = false;
  }
  return syncOne(ctx);
}

int pt_synchronize(pt_ctx* ctx) {
  if (!ctx) return PT_E_INVALID;
  return ctx->peers.empty() ? syncOne(ctx) : syncGroup(ctx);
}

static int statsOne(pt_ctx* ctx, pt_frame_stats* st);

// A group: rays and fetches summed over the devices, kernel times the slowest device's,
// launches / policies rank 0's.
int pt_get_stats(pt_ctx* ctx, pt_frame_stats* st) {
  if (!ctx || !st) return PT_E_INVALID;
  if (ctx->peers.empty()) return statsOne(ctx, st);
  if (int rc = syncGroup(ctx)) return rc;
  if (int rc = statsOne(ctx, st)) return rc;
  for (pt_ctx* p : ctx->peers) {
    pt_frame_stats q;
    if (int rc = statsOne(p, &q)) return fromPeer(ctx, p, rc);
    st->rays += q.rays;
    st->node_fetch += q.node_fetch;
    st->tri_fetch += q.tri_fetch;
    st->mat_fetch += q.mat_fetch;
    st->tex_fetch += q.tex_fetch;
    st->kernel_ms = std::max(st->kernel_ms, q.kernel_ms);
    st->kernel_ms_total = std::max(st->kernel_ms_total, q.kernel_ms_total);
    st->max_stack = std::max(st->max_stack, q.max_stack);
    st->split_items += q.split_items;
  }
  st->devices = 1 + (int)ctx->peers.size();
  st->gather = ctx->gather ? ctx->gather->mode : 0;
  return PT_OK;
}

static int statsOne(pt_ctx* ctx, pt_frame_stats* st) {
  if (int rc = syncStreams(ctx)) return rc;
  unsigned long long h[5];
  std::vector<unsigned long long> shards((size_t)RAY_SHARDS * RAY_SHARD_STRIDE);
  CK(hipMemcpy(h, ctx->d_ctl + CTL_STATS, sizeof(h), hipMemcpyDeviceToHost));
  CK(hipMemcpy(shards.data(), ctx->d_ctl + CTL_RAYS, shards.size() * sizeof(unsigned long long),
               hipMemcpyDeviceToHost));
  std::memset(st, 0, sizeof(*st));
  st->rays = h[0];
  for (int k = 0; k < RAY_SHARDS; k++) st->rays += shards[(size_t)k * RAY_SHARD_STRIDE];
  st->node_fetch = h[1];
  st->tri_fetch = h[2];
  st->mat_fetch = h[3];
  st->tex_fetch = h[4];
  while (foldOne(ctx, true)) {
  }
  st->kernel_ms = ctx->launches > 0 ? ctx->msLast : 0.0f;
  st->kernel_ms_total = (float)ctx->msTotal;
  st->launches = ctx->launches;
  st->frames = ctx->frames;
  st->frame_batch = ctx->batchCap;
  st->env_compact = ctx->d_hdr8 ? (ctx->d_cacheRow ? 2 : 1) : 0;
  st->tree4_nodes = ctx->fast4Ready ? ctx->f4nDev : 0;
  st->max_stack = ctx->maxStack;
  st->split_items = 0;
  st->runtime_tree = ctx->lastFast ? 1 : 0;
  st->waves_per_simd = ctx->lastWaves;
  st->regen = ctx->lastRegen ? 1 : 0;
  st->devices = 1;
  st->gather = 0;
  st->frames_in_flight = ctx->pipe ? ctx->pipeDepth : 1;
  st->upload_ms = ctx->uploadMs;
  st->accel_build_ms = ctx->accelMs;
  st->accel_device = ctx->accelDevice;
  st->accel_nodes = ctx->accelNodes;
  st->accel_depth = ctx->accelDepth;
  const int ls = ctx->pipe && ctx->frameNo > 0 ? ctx->lastSlot : 0;  // the last frame's slot
  if (ctx->d_order && ctx->orderValid[ls]) {
    int counts[NUM_QUEUES];
    const int* ord = ctx->d_order + (size_t)ls * ((size_t)NUM_QUEUES * ctx->orderCap + NUM_QUEUES);
    CK(hipMemcpy(counts, ord + (size_t)NUM_QUEUES * ctx->orderCap, sizeof(counts), hipMemcpyDeviceToHost));
    long items = 0;
    for (int q = 0; q < NUM_QUEUES; q++) items += counts[q];
    st->split_items = (int)std::max(0L, items - (long)ctx->numItems);
  }
  return PT_OK;
}

static float fmathHost(int fn, float x, float y) {
  switch (fn) {
    case 0: return ptm_sinf(x);
    case 1: return ptm_cosf(x);
    case 2: return ptm_atan2f(x, y);
    case 3: return ptm_asinf(x);
    case 4: return ptm_logf(x);
    case 5: return ptm_expf(x);
    default: return ptm_powf(x, y);
  }
}

int pt_fmath_host(int fn, const float* x, const float* y, int n, float* out) {
  if (fn < 0 || fn > 6 || n < 0 || (n > 0 && (!x || !out))) return PT_E_INVALID;
  for (int i = 0; i < n; i++) out[i] = fmathHost(fn, x[i], y ? y[i] : 0.0f);
  return PT_OK;
}

int pt_fmath_device(pt_ctx* ctx, int fn, const float* x, const float* y, int n, float* out) {
  if (!ctx || fn < 0 || fn > 6 || n < 0 || (n > 0 && (!x || !out))) return PT_E_INVALID;
  if (n == 0) return PT_OK;
  CK(hipSetDevice(ctx->cfg.device_id));
  float *dx = nullptr, *dy = nullptr, *dout = nullptr;
  const size_t b = (size_t)n * sizeof(float);
  CK(hipMalloc(&dx, b));
  CK(hipMalloc(&dy, b));
  CK(hipMalloc(&dout, b));
  CK(hipMemcpy(dx, x, b, hipMemcpyHostToDevice));
  if (y) CK(hipMemcpy(dy, y, b, hipMemcpyHostToDevice));
  else CK(hipMemset(dy, 0, b));
  CK(launchFmath(fn, dx, dy, n, dout, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  CK(hipMemcpy(out, dout, b, hipMemcpyDeviceToHost));
  CK(hipFree(dx));
  CK(hipFree(dy));
  CK(hipFree(dout));
  return PT_OK;
}

static int resetOne(pt_ctx* ctx);

int pt_reset_stats(pt_ctx* ctx) {
  if (!ctx) return PT_E_INVALID;
  for (pt_ctx* p : ctx->peers)
    if (int rc = resetOne(p)) return fromPeer(ctx, p, rc);
  return resetOne(ctx);
}

static int resetOne(pt_ctx* ctx) {
  if (int rc = syncStreams(ctx)) return rc;
  CK(hipMemset(ctx->d_ctl + CTL_STATS, 0, CTL_BYTES - CTL_STATS));
  while (foldOne(ctx, true)) {
  }
  ctx->launches = 0;
  ctx->frames = 0;
  ctx->msTotal = 0.0;
  ctx->msLast = 0.0f;
  return PT_OK;
}

// ------------------------------------------------------------ device groups
static int createGroup(pt_ctx* ctx) {
  const int n = 1 + (int)ctx->peers.size();
  GroupGather* g = new (std::nothrow) GroupGather();
  if (!g) return fail(ctx, PT_E_NOMEM, "group gather");
  ctx->gather = g;
  g->n = n;
  std::vector<int> devs{ctx->cfg.device_id};
  for (pt_ctx* p : ctx->peers) devs.push_back(p->cfg.device_id);
  bool distinct = true;
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++) distinct = distinct && devs[a] != devs[b];
  const int want = ctx->cfg.gather;
  const Rccl& R = rccl();
  if (want == PT_GATHER_RCCL && (!distinct || !R.ok))
    return fail(ctx, PT_E_INVALID, distinct ? R.err : "PT_GATHER_RCCL needs distinct devices");
  g->mode = (want == PT_GATHER_RCCL || (want == PT_GATHER_AUTO && distinct && R.ok)) ? PT_GATHER_RCCL : PT_GATHER_COPY;
  // peer access lets hipMemcpyPeerAsync go device to device over xGMI (best effort)
  for (int k = 1; k < n; k++)
    if (devs[k] != devs[0]) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devs[0], devs[k]) == hipSuccess && can) {
        (void)hipSetDevice(devs[0]);
        (void)hipDeviceEnablePeerAccess(devs[k], 0);
        (void)hipGetLastError();  // "already enabled" is fine
      }
    }
  CK(hipSetDevice(devs[0]));
  CK(hipStreamCreateWithFlags(&g->cstream, hipStreamNonBlocking));
  CK(hipEventCreateWithFlags(&g->done, hipEventDisableTiming));
  g->peer.resize(n - 1);
  for (int k = 1; k < n; k++) {
    GroupGather::Peer& P = g->peer[k - 1];
    pt_ctx* m = ctx->peers[k - 1];
    P.dev = devs[k];
    P.count = (size_t)packParams(m, k, n).count;
    CK(hipSetDevice(devs[0]));
    if (P.count) CK(hipMalloc(&P.recv, P.count * PACK_F * sizeof(float)));
    // copy mode: the transfer (and its completion event) runs on rank 0's device
    for (int i = 0; i < 2; i++)
      if (g->mode == PT_GATHER_COPY) CK(hipEventCreateWithFlags(&P.sent[i], hipEventDisableTiming));
    CK(hipSetDevice(P.dev));
    for (int i = 0; i < 2; i++) {
      if (P.count) CK(hipMalloc(&P.send[i], P.count * PACK_F * sizeof(float)));
      CK(hipEventCreateWithFlags(&P.packed[i], hipEventDisableTiming));
      if (g->mode == PT_GATHER_RCCL) CK(hipEventCreateWithFlags(&P.sent[i], hipEventDisableTiming));
    }
    if (g->mode == PT_GATHER_RCCL) CK(hipStreamCreateWithFlags(&P.mstream, hipStreamNonBlocking));
  }
  if (g->mode == PT_GATHER_RCCL) {
    ncclResult_t e = R.commInitAll(g->comms, n, devs.data());
    if (e != ncclSuccess) return fail(ctx, PT_E_HIP, std::string("ncclCommInitAll: ") + R.errorString(e));
    g->commsReady = true;
  }
  CK(hipSetDevice(devs[0]));
  return PT_OK;
}

static int groupGather(pt_ctx* ctx) {
  GroupGather& g = *ctx->gather;
  const int i = (int)(g.frame++ & 1u);
  const int n = g.n;
  const int dev0 = ctx->cfg.device_id;
  // each rank's tiles of this frame, packed on its render stream behind the frame
  for (int k = 1; k < n; k++) {
    GroupGather::Peer& P = g.peer[k - 1];
    pt_ctx* m = ctx->peers[k - 1];
    if (!P.count) continue;
    if (int rc = joinPipe(m)) return fromPeer(ctx, m, rc);
    CK(hipSetDevice(P.dev));
    if (P.sentValid[i]) CK(hipStreamWaitEvent(m->stream, P.sent[i], 0));
    CK(launchPack(packParams(m, k, n), m->d_accum, P.send[i], m->stream));
    CK(hipEventRecord(P.packed[i], m->stream));
  }
  if (g.mode == PT_GATHER_RCCL) {
    const Rccl& R = rccl();
    for (auto& P : g.peer)
      if (P.count) {
        CK(hipSetDevice(P.dev));
        CK(hipStreamWaitEvent(P.mstream, P.packed[i], 0));
      }
    ncclResult_t e = R.groupStart();
    for (int k = 1; k < n && e == ncclSuccess; k++) {
      GroupGather::Peer& P = g.peer[k - 1];
      if (!P.count) continue;
      e = R.send(P.send[i], P.count * PACK_F, ncclFloat32, 0, g.comms[k], P.mstream);
      if (e == ncclSuccess) e = R.recv(P.recv, P.count * PACK_F, ncclFloat32, k, g.comms[0], g.cstream);
    }
    ncclResult_t e2 = R.groupEnd();
    if (e == ncclSuccess) e = e2;
    if (e != ncclSuccess) return fail(ctx, PT_E_HIP, std::string("RCCL gather: ") + R.errorString(e));
    for (auto& P : g.peer)
      if (P.count) {
        CK(hipSetDevice(P.dev));
        CK(hipEventRecord(P.sent[i], P.mstream));
      }
  } else {
    CK(hipSetDevice(dev0));
    for (auto& P : g.peer) {
      if (!P.count) continue;
      CK(hipStreamWaitEvent(g.cstream, P.packed[i], 0));
      CK(hipMemcpyPeerAsync(P.recv, dev0, P.send[i], P.dev, P.count * PACK_F * sizeof(float), g.cstream));
      CK(hipEventRecord(P.sent[i], g.cstream));
    }
  }
  CK(hipSetDevice(dev0));
  for (int k = 1; k < n; k++) {
    GroupGather::Peer& P = g.peer[k - 1];
    if (P.count) CK(launchUnpack(packParams(ctx, k, n), ctx->d_accum, P.recv, g.cstream));
    P.sentValid[i] = P.count > 0;
  }
  CK(hipEventRecord(g.done, g.cstream));
  g.pending = true;
  return PT_OK;
}

static void destroyGroup(pt_ctx* ctx) {
  GroupGather* g = ctx->gather;
  if (g) {
    if (g->cstream) {
      (void)hipSetDevice(ctx->cfg.device_id);
      (void)hipStreamSynchronize(g->cstream);
    }
    for (auto& P : g->peer) {
      (void)hipSetDevice(P.dev);
      if (P.mstream) (void)hipStreamSynchronize(P.mstream);
    }
    if (g->commsReady)
      for (int k = 0; k < g->n; k++)
        if (g->comms[k]) (void)rccl().commDestroy(g->comms[k]);
    for (auto& P : g->peer) {
      (void)hipSetDevice(P.dev);
      for (int i = 0; i < 2; i++) {
        dfree(P.send[i]);
        if (P.packed[i]) (void)hipEventDestroy(P.packed[i]);
        if (g->mode == PT_GATHER_RCCL && P.sent[i]) (void)hipEventDestroy(P.sent[i]);
      }
      if (P.mstream) (void)hipStreamDestroy(P.mstream);
      (void)hipSetDevice(ctx->cfg.device_id);
      dfree(P.recv);
      for (int i = 0; i < 2; i++)
        if (g->mode == PT_GATHER_COPY && P.sent[i]) (void)hipEventDestroy(P.sent[i]);
    }
    (void)hipSetDevice(ctx->cfg.device_id);
    if (g->done) (void)hipEventDestroy(g->done);
    if (g->cstream) (void)hipStreamDestroy(g->cstream);
    delete g;
    ctx->gather = nullptr;
  }
  for (pt_ctx* p : ctx->peers) pt_destroy(p);
  ctx->peers.clear();
}

int pt_abi_version(void) { return PT_ABI_VERSION; }

}  // extern "C"
