// pt_wavefront.h -- parameter blocks of the wavefront pipeline (pt_wavefront.hip),
// shared with the host orchestration in pt_runtime.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_kernels.h"

namespace pt {

#ifndef PT_WF_LDS_STACK
#define PT_WF_LDS_STACK 16
#endif
constexpr int WF_LDS_STACK = PT_WF_LDS_STACK;  // LDS stack entries per lane in the trace kernels

// Queues are split into WF_NSEG segments, each with its own append counter, so
// appends never pile onto one address (one same-address atomic stream sustains
// only ~88 ops/us on MI355X). Producer and consumer blocks own segment
// blockIdx % WF_NSEG; grids are multiples of WF_NSEG.
constexpr int WF_NSEG = 64;

// per-pixel flags
constexpr uint32_t WF_BOUNCE_MASK = 0xffu;  // bounce index of the ray(s) in flight
constexpr uint32_t WF_PRIMARY = 1u << 8;    // the closest-hit ray in flight is the camera ray
constexpr uint32_t WF_CLS = 1u << 9;        // a closest-hit ray was cast
constexpr uint32_t WF_SHD = 1u << 10;       // an env shadow ray was cast

// counters, each on its own 256-byte line (CTL_LINE_INTS):
// cnt[(((stage * WF_CNT_TYPES) + type) * WF_NSEG + segment) * CTL_LINE_INTS]
constexpr int WF_CNT_ACT = 0, WF_CNT_CLS = 1, WF_CNT_SHD = 2, WF_CNT_TYPES = 3;
__host__ __device__ constexpr size_t wfCnt(int stage, int type, int seg = 0) {
  return ((size_t)(stage * WF_CNT_TYPES + type) * WF_NSEG + seg) * CTL_LINE_INTS;
}

// path state, structure of arrays indexed by pixel id
struct WFState {
  float4* rayO;    // origin of the ray(s) in flight (camera eye or hit point)
  float4* rayD;    // closest-hit ray direction
  float4* shD;     // env shadow ray direction (MIS)
  int2* hit;       // closest-hit result (triangle, t bits)
  int* occ;        // shadow result (1 = occluded)
  uint32_t* seed;  // rand() state (IS:73-89)
  uint32_t* flags;
  float4* hist;    // history (throughput)
  float4* Lo;      // accumulated radiance of the bounces
  float4* Le0;     // emissive of the primary hit
  float4* pend;    // f_r (xyz) and cos / NdotL (w) of the bounce in flight
  float4* shC;     // unoccluded env contribution (xyz), pdf_brdf (w) (MIS)
};

struct WFQueues {
  int* act[2];  // pixels to shade next
  int* cls[2];  // closest-hit rays to trace
  int* shd[2];  // shadow rays to trace
  int* cnt;     // counters (see wfCnt), zeroed per frame
  int segCap;   // capacity of one segment
};

struct WFParams {
  SceneView scene;
  Env env;
  WFState st;
  WFQueues q;
  float4* accum;
  int width, height;
  uint32_t frameCounter;  // running-mean count
  uint32_t sampleIndex;   // RNG / Sobol sample index
  int maxBounce;
  float eye[3];
  float cam[16];
  int numOwned;  // owned pixel slots (8x8 wave tiles x 64)
  int shardSize, shardsX, rank, world;
};

struct WFTraceParams {
  SceneView scene;
  const int* queue;   // segment s at queue + s * segCap
  const int* count;   // WF_NSEG counters, stride CTL_LINE_INTS
  int segCap;
  const float4* rayO;
  const float4* rayD;
  int2* hit;
  int* occ;
  int* ovf;
  int ovfDepth;
  unsigned long long* rays;  // RAY_SHARDS padded ray counters
  // wfTrace4Kernel: the env shadow rays (MIS), traced by the same launch after the closest-hit
  // rays (null queue = none); directions rayDS, results occ
  const int* queueS;
  const int* countS;
  const float4* rayDS;
};

hipError_t wfLaunchGen(const WFParams& p, hipStream_t s);
hipError_t wfLaunchTrace(const WFTraceParams& p, bool anyhit, bool cull, int grid, hipStream_t s);
hipError_t wfTraceBlocksPerCU(bool anyhit, bool cull, int* nb);
hipError_t wfLaunchShade(const WFParams& p, int integrator, int stage, int grid, hipStream_t s);
// the 4-wide runtime tree's trace kernel (p.scene.fast, p.scene.f4nTop <= wfTrace4Top())
hipError_t wfLaunchTrace4(const WFTraceParams& p, bool cull, int grid, hipStream_t s);
hipError_t wfTrace4Shape(bool cull, int* blockSize, int* blocksPerCU);
int wfTrace4Top();

}  // namespace pt
