// pt_kernels.h -- kernel parameter blocks and launchers shared by
// pt_kernels.hip (device) and pt_runtime.cpp (host).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pt {

#ifndef PT_BLOCK
#define PT_BLOCK 256  // 64 and 128 measured: c2 +18 % / +8 %, c4 -6 % / -2 %
#endif
constexpr int BLOCK = PT_BLOCK;   // threads per block (256 = 4 waves of 64)
#ifndef PT_LDS_STACK
#define PT_LDS_STACK 32
#endif
#ifndef PT_MIN_WAVES_LAMBERT
#define PT_MIN_WAVES_LAMBERT 3    // Lambert megakernel: keep 3 waves/SIMD (<= 168 VGPRs, no spills)
#endif
// Scenes whose geometry outgrows the L2s by far (> PT_WIDE_SCENE_MB of records)
// walk memory-latency bound: their Disney/MIS megakernels run the variant
// compiled for WIDE_WAVES waves per SIMD (some VGPRs spilled), which keeps more
// node fetches in flight (c5: 13.4 -> 10.5 ms; c3/c4, L2-resident: 1-5 % slower).
#ifndef PT_COST_EMA
#define PT_COST_EMA 2  // order tiles by a running estimate of their cost, this frame's weighted 2^-PT_COST_EMA (0 = off)
#endif
#ifndef PT_WIDE_SCENE_MB
#define PT_WIDE_SCENE_MB 48  // 240 B of records per triangle (pairs, geometry, shading) + 64 per node: ~200k triangles
#endif
constexpr int WIDE_WAVES = 3;
// ... and the Disney/MIS path-regeneration kernel (pt_regen.hip) compiled for 4 waves
// per SIMD (128 VGPRs, 18 spilled) is their default frame kernel: with long paths
// (c5: 16 bounces) a lane that takes a new pixel when its path ends beats the
// lock-step megakernel, whose waves last as long as their longest path (c5: 10.0
// -> 9.2 ms; on the L2-resident c4 the regen kernel is 3.6x slower)
#ifndef PT_WIDE_REGEN_WAVES
#define PT_WIDE_REGEN_WAVES 4  // MIS
#endif
// the uniform integrators' (Lambert, Disney) variant: 4 waves per SIMD since round 4's scalar pair
// test (128 VGPRs, 3 spilled; 3 waves 135 unspilled): c2 0.1938 -> 0.1884 ms per frame (5 rounds,
// profiles/r4/ab/aj_*). Before it, 3 waves (163 VGPRs) against 4 (59 spilled): 0.235 vs 0.241 ms.
#ifndef PT_WIDE_REGEN_WAVES_U
#define PT_WIDE_REGEN_WAVES_U 4
#endif
constexpr int WIDE_REGEN_WAVES = PT_WIDE_REGEN_WAVES;
constexpr int wideRegenWaves(int integrator) { return integrator == 2 ? PT_WIDE_REGEN_WAVES : PT_WIDE_REGEN_WAVES_U; }
// the MIS wide kernel on scenes that fit the L2s (c3): 3 waves per SIMD, no spills (143 VGPRs), against 4
// with 9 spilled -- c3 0.1262 -> 0.1216 ms per frame; large scenes keep 4 (c5 4.44 vs 4.79 ms at 3)
#ifndef PT_WIDE_REGEN_WAVES_SMALL
#define PT_WIDE_REGEN_WAVES_SMALL 3
#endif
#ifndef PT_MIN_WAVES
#define PT_MIN_WAVES 1            // __launch_bounds__ minimum waves per SIMD of the render kernels
#endif
// the MIS megakernel at 3 waves per SIMD (168 VGPRs; 208 uncapped, so ~30 spill): c4 0.321 ->
// 0.291 ms per frame (tools/tune.py, 3 rounds; round 3's kernel, 231 VGPRs with 142 spilled at 3
// waves, had measured no gain)
#ifndef PT_MIN_WAVES_MIS
#define PT_MIN_WAVES_MIS 3
#endif
constexpr int LDS_STACK = PT_LDS_STACK;
#ifndef PT_LDS_NODES
#define PT_LDS_NODES 128
#endif
// top-of-tree nodes (breadth-first from the root) the megakernel keeps in LDS, 64 B each
constexpr int LDS_NODES = PT_LDS_NODES;
#ifndef PT_SPLIT_PCT
#define PT_SPLIT_PCT 25  // megakernel: split a tile whose longest item costs more than this % of a wave's share
#endif
#ifndef PT_SPLIT_AUTO
#define PT_SPLIT_AUTO 1  // the runtime measures its tree and split policies after each running-mean restart (probePolicy)
#endif
#ifndef PT_WAVE_TRACE
#define PT_WAVE_TRACE 0  // diagnostics build: record each megakernel wave's lifetime (tools/wave_trace.py)
#endif
#ifndef PT_PHASE_STATS
// diagnostics build (with PT_WAVE_TRACE): the regen kernel's per-wave time and lanes per phase
// (refill, walk, reference check, shading; node and leaf iterations) -- tools/wave_trace.py --phases
#define PT_PHASE_STATS 0
#endif
constexpr int PHASE_WORDS = 24;  // PT_PHASE_STATS record (pt_regen.hip)
constexpr int WAVE_TRACE_WORDS = PT_PHASE_STATS ? PHASE_WORDS : 6;  // u64 per wave in RenderParams::waveTrace
 // traversal stack entries per lane kept in LDS (4 B x 256 lanes each)
#ifndef PT_NUM_QUEUES
#define PT_NUM_QUEUES 32
#endif
// Device-scope atomics are serialised per cache line at the memory side (~88
// same-line ops/us), so every hot counter lives on its own 256-byte line.
constexpr int CTL_LINE_INTS = 64;
constexpr int NUM_QUEUES = PT_NUM_QUEUES;  // work counters, queue q owned by blocks with blockIdx % NUM_QUEUES == q
static_assert((NUM_QUEUES & (NUM_QUEUES - 1)) == 0 && NUM_QUEUES <= 64, "NUM_QUEUES: power of two <= 64");
constexpr int RAY_SHARDS = 64;     // sharded ray counters (u64, one per 256-byte line)
constexpr int RAY_SHARD_STRIDE = CTL_LINE_INTS / 2;  // in u64
// control block layout (bytes)
constexpr int MAX_SLOTS = 16;  // frames in flight the control block has queue counters for (pt_runtime.cpp PIPE)
constexpr size_t CTL_QUEUES = 0;  // MAX_SLOTS x NUM_QUEUES padded int counters
constexpr size_t CTL_STATS = (size_t)MAX_SLOTS * 64 * 256;            // 5 u64 cumulative fetch counters
constexpr size_t CTL_RAYS = CTL_STATS + 256;                          // RAY_SHARDS padded u64 counters
constexpr size_t CTL_BYTES = CTL_RAYS + (size_t)RAY_SHARDS * 256;
#ifndef PT_FAST_TREE
#define PT_FAST_TREE 1  // build and traverse the runtime's own tree (results checked against the reference's)
#endif
#ifndef PT_WIDE4
// the megakernel's traced rays walk the runtime tree collapsed to 4-wide nodes (pt_trace.h
// traceRay4; camera rays keep their bins and the binary tree's packets): 2 = with the 4-wide
// tree's top 64 nodes in LDS (c2 0.408 -> 0.376 ms, c4 0.498 -> 0.477, c3 0.273 -> 0.262),
// 1 = without (c3 0.257, c2 0.380), 0 = the binary runtime tree
#define PT_WIDE4 2
#endif
#ifndef PT_FUSED_SLABS
#define PT_FUSED_SLABS 1  // the runtime tree's slab tests as packed FMAs (pt_trace.h visitNodeF)
#endif
#ifndef PT_ACCEL_LEAF
#define PT_ACCEL_LEAF 4  // most triangles per leaf of the runtime's tree
#endif
#ifndef PT_PACKETS
#define PT_PACKETS 1  // megakernel: camera rays as wave packets (pt_trace.h tracePacket)
#endif
constexpr int PKT_DEPTH = 128;    // camera-ray packet stack entries per wave (LDS); deeper trees trace per ray
constexpr int PAIR_F4 = 7;        // float4 per pair record (26 floats: p1, p2, p3, Ng, w of two triangles)
constexpr int HIT_F4 = 4;         // float4 per hit record (SceneView::hitRec)
constexpr int MAT_F4 = 5;         // float4 per material (SceneView::mats)
constexpr int W4_F4 = 8;          // float4 per 4-wide node as built (collapseWide4Device, encodeWide4), one 128-byte line
constexpr int LEAF_CNT_BITS = 5;  // leaf refs: ~(start << 5 | (count - 1)), count <= 32
constexpr int REF_NONE = (int)0x80000000;
constexpr int MAX_LEAF = 1 << LEAF_CNT_BITS;
constexpr int MAX_TRIS = (1 << (31 - LEAF_CNT_BITS)) - 1;

// Device-resident scene (relaid out at upload, see pt_runtime.cpp)
struct SceneView {
  const float4* geo;   // 4 float4 per triangle: (p1, w=dot(Ng,p1)), (p2, 0), (p3, 0), (Ng, 0)
  const float4* pairs; // PAIR_F4 float4 per triangle i: triangles i and i+1 component-interleaved (pt_trace.h pairTest)
  // Shading data of a hit, read once per closest hit (finishHit): per triangle one
  // 64-byte record {n1.xyz, n2.x}, {n2.yz, n3.xy}, {n3.z, material id, -, -} (the
  // Triangle_encoded normals, floats 9..17), and the scene's distinct materials,
  // MAT_F4 float4 each laid out as Triangle_encoded floats 16..35 (emissive at
  // floats 18..20, IS:207-232). 64 + ~0 bytes per triangle instead of 144.
  const float4* hitRec;
  const float4* mats;
  int nMats;           // materials in mats
  const float4* bvh;   // 4 float4 per device node id (pt_runtime.cpp: top of the tree first, breadth-first)
  int nTop;            // device ids [0, nTop) are the top of the tree, staged in LDS by the megakernel
  int rootRef;         // encoded reference to node 1
  int nTri;
  // The runtime's own tree over the same triangles (pt_runtime.cpp uploadAccel;
  // pt_trace.h "Reference-exact results through the runtime's tree"): wide
  // nodes with conservative boxes, pair records in its leaf order, and for
  // every position the uploaded triangle index. fast = 0: not used this launch.
  int fast;
  const float4* fbvh;
  const float4* fpairs;
  const int* fastTri;
  int fRoot, fnTop;
  // the same tree collapsed to 4-wide nodes (pt_runtime.cpp encodeWide4; pt_trace.h
  // traceRay4): W4_F4 float4 per node, breadth-first ids, leaves as in fbvh; null = none
  const float4* fbvh4;
  int f4Root, f4nTop;
  // reference facts: each triangle's reference leaf's box (lo, hi; lo.w = the leaf's node id as
  // int bits, -1 = in no leaf), every reference node's parent and box (lo, hi)
  const int* refParent;
  const float4* refBox;
  const float4* leafBox;
};

// HDR environment (hdrMap + hdrCache textures, IS main.cpp:843-853), float4 texels
// Render layout: one 16-byte texel serves hdrColor and hdrPdf of a direction
// together (every MIS lookup pairs them), so a miss costs one line, not two.
struct Env {
  const float4* hdr;    // w x h: (r, g, b, calculateHdrCache pdf) (row 0 = first scanline); null = black
  const float2* cache;  // calculateHdrCache sample table (x, y); null exactly when hdr is null
  // The same texels in half the bytes, used when non-null (pt_runtime.cpp envOne builds them when
  // every texel round-trips bit for bit, pt_envcache.hip envCompactKernel): hdr8 = {r | g << 8 |
  // b << 16 | E << 24, pdf bits}, each channel m * 2^(E - 136) -- the Radiance RGBE form the
  // reference's decoder expands (hdrloader.cpp:99-104) -- and cache4 = x | y << 16, the sample
  // table's float(x) / w and float(y) / h (IS main.cpp:630-631)
  const uint2* hdr8;
  const uint32_t* cache4;
  // The sample table by rows, used when non-null: calculateHdrCache's entry (row i, column j) is
  // (x(i) / w, y(x(i), j) / h) -- x from the marginal CDF at xi_1 = i / h, y from column x's
  // conditional CDF at xi_2 = j / w (IS main.cpp:621-634) -- so all rows of one x are equal.
  // cacheRow[i] = x(i) | (its distinct row's id) << 16, cacheY[id * w + j] = y; c4's 8 MB of uniformly
  // read 4-byte entries become 639 distinct rows of 2-byte ones (2.6 MB) and a 4 KB row table
  const uint32_t* cacheRow;
  const unsigned short* cacheY;
  // With the compact table: SampleHdr's (sin, cos) of theta for each y integer 0..h, then of phi
  // for each x integer 0..w (launchEnvTrig: the device functions of the same floats), null = computed
  const float2* trig;
  // With the compact texels too: per sample-table entry (y, x) (index y * (w + 1) + x, x <= w, y <= h)
  // the light sample's hdrColor and hdrPdf (IS:647-666) of SampleHdr's direction: {the texel's RGBE,
  // the pdf's bits} (launchEnvLight: the device functions of the same floats), null = computed
  const uint2* light;
  int w, h, res;        // res = hdrResolution
  // texels read as streaming (non-temporal) loads, so they leave L2 before the scene's lines: on
  // scenes larger than L2 (c5 4.15 vs 4.32 ms per frame with plain loads); on small scenes plain
  // loads let neighbouring rays share env lines (c2 0.1722 -> 0.1684, c3 0.1097 -> 0.1068, c4
  // 0.2969 -> 0.290 ms)
  int nt;
};

// One frame of a launch as a work item sees it: its sample index (RNG seeds, Sobol
// index) and its colour buffer (null: the running mean is updated in place).
constexpr int COL_F = 3;  // floats per pixel of a pipelined frame's colour buffer (r, g, b)
struct FrameRef {
  float* col;  // COL_F floats per pixel of the share
  uint32_t sampleIndex;
};

struct RenderParams {
  SceneView scene;
  Env env;
  int width, height;
  uint32_t frameCounter;  // running-mean count: weight 1/(frameCounter+1) (IS:868-871)
  uint32_t sampleIndex;   // RNG / Sobol sample index: frameCounter*sample_world + sample_rank
  int maxBounce;
  float eye[3];
  float cam[16];
  float4* accum;
  // Pipelined frames (pt_runtime.cpp "frames in flight"): non-null = write each pixel's
  // sample colour here (float4, w unused) and leave the running mean to mixKernel, which
  // runs in frame order; null = mix into accum in place (IS:868-871)
  float* col;  // COL_F floats per slot of the share
  // A batch of nFrames consecutive frames of one camera in this launch (pt_render_frames_async):
  // frame f draws sample index sampleIndex + f * sampleStride and writes its colours to
  // col + f * colStride and its camera-ray results to primHit + f * colStride, each indexed by the
  // pixel's slot in this context's screen-tile share (shareIndex: the packed order of
  // pt_pack_owned; colStride = the share's slots), so a 1/N share's buffers are 1/N of a frame. Work
  // item k of the launch is item k / nFrames of frame k % nFrames, so the frames of one tile
  // run side by side (the same camera rays, the same nodes). nFrames 1: a single frame.
  int nFrames;
  uint32_t sampleStride;
  size_t colStride;
  // camera-ray bins (pt_primary.hip): per 8x8 tile of the whole image, binStart[t] ..
  // binStart[t+1] index binTris; null = every camera ray walks the BVH
  const int* binStart;
  const int* binTris;
  // per bin entry: its triangle's geometry record (4 float4) and reference leaf box (2 float4),
  // gathered at bin build so the camera-ray pass stages a tile's bin in one round trip
  const float4* binGeo;
  const float4* binBox;
  int binTilesX, binTilesY;
  // camera-ray pass (primaryKernel): per pixel (py * width + px) the camera ray's result,
  // {tri, t bits}: tri >= 0 a hit, PRIM_MISS (finished: sky colour written), PRIM_RETRACE
  // (a tie or an unreachable winner: the megakernel traces it in the reference order),
  // PRIM_TILE (the tile's bin is over PT_BIN_CAP: the megakernel traces the tile's
  // packet); null = the megakernel traces its camera rays itself
  int2* primHit;
  // ... compacted per 8x8 wave tile (round 6): tile w of frame f has a 64-bit mask of the slots that
  // need a path (primMask[f * numItems + w]: not sky, inside the image) and their results in slot
  // order at primHit + (f * numItems + w) * 64 (primOfSlot); sky slots cost no bytes
  unsigned long long* primMask;
  int zeroQueue;  // the camera-ray pass zeroes `queue` for the frame kernel after it (no memset)
  int* queue;           // NUM_QUEUES counters (stride CTL_LINE_INTS), zeroed before each launch
  int perQueue;         // items per queue (band), claimed once per frame of the launch
  int numItems;         // 8x8 wave tiles owned by this rank
  int shardSize;        // shard tile edge (multiple of 8)
  int shardTiles;       // (shardSize/8)^2
  int shardsX;          // shard tiles per row
  int rank, world;
  int* ovf;             // traversal stack overflow (per thread ovfDepth ints), may be null
  int ovfDepth;
  int packets;          // camera rays traced as wave packets (tree depth fits PKT_DEPTH)
  unsigned long long* stats;  // [rays, nodes, tris, mats, texels]
  unsigned long long* rayShards;  // RAY_SHARDS ray counters (stride RAY_SHARD_STRIDE)
  const int* tileOrder; // per-band work items (null = one per tile, in id order), then NUM_QUEUES item
                        // counts; see TileCursor / reorderKernel
  int orderCap;         // entries per band in tileOrder
  int* tileCost;        // per tile: summed cost of its items this frame (shader cycles), null = not recorded
  int* tileCostMax;     // per tile: its longest item this frame
  unsigned long long* waveTrace;  // PT_WAVE_TRACE builds only: WAVE_TRACE_WORDS u64 per wave (pt_runtime.cpp, tools/wave_trace.py)
};

struct TraceParams {
  SceneView scene;
  const float* rays;
  int n;
  float* t;
  int* tri;
  int* ovf;
  int ovfDepth;
};

// BasicRayTracingWithC++ (pt_kernels.hip basicKernel): one sample k of every pixel
constexpr int BASIC_MAX_DEPTH = 31;  // pathTracing vertices kept for the fold (the reference's cutoff is 8)
struct BasicParams {
  const double* shapes;         // nShapes x PT_SHAPE_DOUBLES
  int nShapes;
  int width, height;
  uint32_t sample, seed;        // k, and the counter RNG's run seed
  int maxDepth;
  int reset;                    // frameCounter == 0: this sample starts the image
  float brightness;             // BRIGHTNESS (B:20) as glm's operator*= casts it
  float4* accum;                // the image as f32 (pt_download_accum)
  double* image;                // the reference's double image, width x height x 3 (B:356)
  const double* stream;         // replayed randf() stream (nullable: counter RNG)
  const long long* offsets;     // replay: start of each sample's draws, (k * height + i) * width + j
  long long streamN, nOffsets;
  unsigned long long* stats;    // ray counter
  unsigned long long* overruns; // replay: pixel samples that read past their draws
};

struct PackParams {
  int width, height, shardSize, shardsX, rank, world;
  long count;
};
// rank 0's unpack of ranks 1..world-1's packed buffers in one launch (pt_display_unpack: RGB8
// display values; pt_unpack_ranks: f32 running means); null buffers are skipped; base's rank /
// count are per rank
constexpr int DISPLAY_MAX_WORLD = 16;
struct RanksUnpack {
  PackParams base;
  const void* src[DISPLAY_MAX_WORLD];
  long count[DISPLAY_MAX_WORLD];
};

// camera-ray bins of one camera (pt_primary.hip), device buffers owned by the context
#ifndef PT_BIN_CAP
#define PT_BIN_CAP 32  // a tile whose bin holds more triangles traces its camera rays through the BVH
#endif
#ifndef PT_PASS_BIN_CAP
#define PT_PASS_BIN_CAP 64  // the camera-ray pass (primaryKernel), staged per one-wave block: c5 32 6.84, 64 6.77, 128 6.79, 256 7.08 ms
#endif
#ifndef PT_BINS
#define PT_BINS 1      // 0: no camera-ray bins
#endif
struct PrimaryBins {
  int4* rect = nullptr;      // per triangle: its tile rectangle
  int* triCount = nullptr;   // per triangle: its tiles (+1: the scan total)
  int* triOffset = nullptr;
  int* tileCount = nullptr;  // per tile: its triangles, then the fill cursors
  int* binStart = nullptr;   // per tile (+1)
  int* binTris = nullptr;
  float4* binGeo = nullptr;  // per entry: geo[4 tri .. 4 tri + 3] (RenderParams::binGeo)
  float4* binBox = nullptr;  // per entry: leafBox[2 tri], [2 tri + 1]
  void* tmp = nullptr;       // hipcub scan scratch
  size_t rectCap = 0, triCountCap = 0, triOffsetCap = 0, tileCountCap = 0, binStartCap = 0, binTrisCap = 0,
         binGeoCap = 0, binBoxCap = 0, tmpBytes = 0;
  int tilesX = 0, tilesY = 0, entries = 0;
};
hipError_t buildPrimaryBins(const float eye[3], const float cam[16], int width, int height, const float4* geo,
                            const float4* leafBox, int nTri, PrimaryBins& b, hipStream_t s);
void freePrimaryBins(PrimaryBins& b);

// The runtime's own tree built on the device (pt_build.hip): a binned-SAH tree
// over the triangles of geo (SceneView::geo layout), its wide records with
// every box widened by inflate of its own magnitude plus inflateRelAbs x the
// scene's largest coordinate (pt_runtime.cpp encodeWideTree), the pair records
// in its leaf order and that order. Device buffers owned by the caller
// (freeAccelBuild); the stream is synchronised on return.
struct BuildNode {  // 64 B, breadth-first ids (root 0)
  float4 lo;        // triangle box lo; w: first position (int bits)
  float4 hi;        // triangle box hi; w: triangle count (int bits)
  float4 clo;       // centroid bounds lo; w: left child id (int bits, -1 = leaf)
  float4 chi;       // centroid bounds hi; w: right child id
};
struct AccelBuild {
  float4* bvh = nullptr;    // nDev wide records (4 float4 each)
  float4* pairs = nullptr;  // nTri pair records (PAIR_F4 float4 each), leaf order
  int* order = nullptr;     // position -> uploaded triangle index
  BuildNode* nodes = nullptr;  // the nNodes build nodes (leaves: count <= leafSize)
  int rootRef = REF_NONE, nDev = 0, depth = 0, nNodes = 0;
};
hipError_t buildAccelDevice(const float4* geo, int nTri, int leafSize, float inflate, float inflateRelAbs,
                            AccelBuild& out, hipStream_t s);
void freeAccelBuild(AccelBuild& a);
// the build nodes collapsed to 4-wide records (SceneView::fbvh4, pt_runtime.cpp encodeWide4's
// layout, ids and widening) on the device; *out allocated here (W4_F4 float4 per wide node)
hipError_t collapseWide4Device(const BuildNode* nodes, int nNodes, int leafSize, float inflate, float inflateRelAbs,
                               float4** out, int* rootRef, int* nDev, int* depth, hipStream_t s);

// calculateHdrCache on the device (pt_envcache.hip); scratch: 2*w*h + 2*w + 1 floats
hipError_t launchHdrCache(const float* hdr, int w, int h, float4* cache, float* scratch, hipStream_t s);
// hdr[k].w = cache[k].z, samp[k] = cache[k].xy (the Env render layout)
hipError_t launchEnvCompact(const float4* hdr, const float2* cache, int w, int h, uint2* hdr8, uint32_t* cache4,
                            int* bad, hipStream_t s);
hipError_t launchEnvPack(float4* hdr, const float4* cache, float2* samp, int n, hipStream_t s);
// Env::trig: (h + 1) + (w + 1) entries
hipError_t launchEnvTrig(float2* trig, int w, int h, hipStream_t s);
// Env::light: (w + 1) * (h + 1) entries, from e's compact texels and trig table
hipError_t launchEnvLight(const Env& e, uint2* light, hipStream_t s);
hipError_t launchRender(const RenderParams& p, int integrator, int grid, hipStream_t s, bool cull, bool count,
                        bool wide = false);
// tile order of the next frame: each queue band's groups of `group` consecutive
// tiles sorted by this frame's summed cost, descending (tiles inside a group keep
// their order, which keeps neighbouring tiles together for the caches)
constexpr int REORDER_MAX = 4096;  // most groups per band the one-block LDS sort handles
// order: NUM_QUEUES * orderCap items, then NUM_QUEUES item counts; cost / costMax are read
// and zeroed; splitLg (one per tile) is the split state carried from frame to frame
hipError_t launchReorder(int* cost, int* costMax, int* splitLg, int* ema, int* order, int perQueue, int orderCap,
                         int numItems, int group, int numWaves, int splitPct, hipStream_t s);
hipError_t renderBlocksPerCU(int integrator, bool cull, bool count, bool wide, int* nb);
// the camera-ray pass: one wave per 8x8 tile of the rank's tiles, results in p.primHit
constexpr int PRIM_MISS = -1, PRIM_RETRACE = -2, PRIM_TILE = -3;
hipError_t launchPrimary(const RenderParams& p, hipStream_t s);
// the path-regeneration kernel (pt_regen.hip): the variant and launch shape of a frame
struct RegenShape {
  bool wide = false;      // the large-scene variant (WIDE_REGEN_WAVES, 4-wide walk, dynamic ray fetch)
  bool fullTree = false;  // ... with the whole 4-wide tree in LDS (small trees, uniform integrators)
  bool small = false;     // the MIS variant at PT_WIDE_REGEN_WAVES_SMALL waves per SIMD (scenes that fit the L2s)
  int block = BLOCK;      // threads per block
  int blocksPerCU = 0;    // resident blocks per CU
  size_t dynLds = 0;      // dynamic LDS bytes per block (the tree)
};
// f4nDev: nodes of the 4-wide runtime tree the frame walks (0: it walks none)
// smallScene: the scene's records fit the L2s (not a PT_WIDE_SCENE_MB scene)
hipError_t regenShape(int integrator, bool cull, bool wide, int f4nDev, bool smallScene, RegenShape* out);
hipError_t launchRegen(const RenderParams& p, int integrator, int grid, hipStream_t s, bool cull, const RegenShape& r);
int regenLdsStack();
int regenTop4(const RegenShape& r, int integrator);  // 4-wide nodes the wide regen kernel stages in LDS (PT_REGEN_TOP4[_3])
hipError_t launchTrace(const TraceParams& p, int grid, hipStream_t s, bool cull);
hipError_t launchBasic(const BasicParams& p, hipStream_t s);
// BASIC checkpoints: the double image from the f32 sums (widened), or the f32 sums from the double image
hipError_t launchBasicWiden(const float4* accum, double* image, long n, hipStream_t s);
hipError_t launchBasicNarrow(const double* image, float4* accum, long n, hipStream_t s);
hipError_t launchTonemap(const float4* accum, float* rgb, int n, float limit, float gamma, hipStream_t s);
// PACK_F floats (r, g, b) per packed slot
constexpr int PACK_F = 3;
hipError_t launchPack(const PackParams& p, const float4* accum, float* packed, hipStream_t s);
hipError_t launchFmath(int fn, const float* x, const float* y, int n, float* out, hipStream_t s);
hipError_t launchDisplayPack(const PackParams& p, const float4* accum, float limit, float gamma, uint8_t* packed,
                             hipStream_t s);
hipError_t launchDisplayOwn(const PackParams& p, const float4* accum, float limit, float gamma, uchar4* image,
                            hipStream_t s);
hipError_t launchDisplayUnpack(const RanksUnpack& d, int world, uchar4* image, hipStream_t s);
hipError_t launchUnpackRanks(const RanksUnpack& d, int world, float4* accum, hipStream_t s);
hipError_t launchUnpack(const PackParams& p, float4* accum, const float* packed, hipStream_t s);
// the running-mean updates of nFrames pipelined frames over the rank's owned pixels (PackParams
// mapping), in frame order: for f = 0 .. nFrames-1, accum = mix(accum, col + f * colStride,
// 1 / (frameCounter + f + 1)) (IS:868-871, pass2.fsh:15) -- each pixel read and written once
hipError_t launchMix(const PackParams& p, float4* accum, const float* col, size_t colStride, int nFrames,
                     uint32_t frameCounter, hipStream_t s);

}  // namespace pt
