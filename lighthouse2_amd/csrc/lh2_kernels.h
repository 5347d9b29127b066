/* lh2_kernels.h - kernel parameter blocks shared by the host driver and lh2_kernels.hip. */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/lh2_core_types.h"

struct DevInstance;
struct Counters;

struct CameraParams   /* camera.h:39-43 arguments (pos, right, up, p1, aperture, distortion, screenParams) */
{
	lh2_float3 pos, p1, right, up;
	float aperture, distortion, geometryEpsilon;
	int w, h, pass;
	uint32_t R0;
	/* tile of the frame owned by this launch: local row lr maps to frame row
	   y0 + (lr / band) * bandStride + lr % band  (contiguous tile: band = rows) */
	int y0, band, bandStride, tileRows;
	int tiled;   /* store rays in 8x8 pixel blocks per wave (coherent traversal); 0 = row-major */
	int primeRef;  /* RenderCore_PrimeRef camera: uniform random numbers, no distortion (camera.h:57-60) */
	/* folded into the camera launch (no launches of their own): the frame's counter / work-queue
	   reset (initC non-null: what k_init_counters does), and the accumulator reset of a restart
	   (clearAcc non-null: each pixel's first sample zeroes it; the memset of rendercore.cpp:465) */
	Counters* initC; uint32_t* cursors; int cursorWords; uint32_t pathCount, segStride;
	int keepCursor;   /* the fused primary launch (initC non-null): the first of the LH2_CURSOR_WORDS words it uses itself,
	                     left alone by its reset */
	float4* clearAcc;
	uint32_t* hvZero; uint32_t hvZeroWords;   /* heavy-first packets: the block this frame records into (TraceArgs::hvWrite) */
	/* set by the launchers (lh2_camera_derive), not by callers: right / w and up / h (IEEE division on the host: the
	   device's correctly rounded quotients), and division by the invariant divisors tileRows x w, w and band as
	   multiply-high + shifts (lh2_udiv) */
	lh2_float3 rightW, upH;
	uint32_t divTile[3], divW[3], divBand[3];
};

struct SceneDev       /* everything the traversal and shading kernels read, by value (kernarg) */
{
	const float4* nodes;
	const float4* tris;
	const DevInstance* inst;
	int tlasRoot, instCount;
	const float4* nodes4;            /* BVH4 of the same scene (traceVersion 4; null when not built) */
	const uint4* nodes4q;            /* the same BVH4 with quantized child boxes, 64 B per node (lh2_box4.inc, box4q) */
	float qBound;                    /* >= |coordinate| of every node origin, world and mesh space (slab_offsets) */
	int tlasRoot4;
	int root40;                      /* tlasRoot4 ~0 (single-instance start): the instance's BVH4 root, a kernel argument so that a
	                                    ray's first node needs no load */
	const lh2_CoreInstanceDesc* instDesc;
	const float4* tris0;             /* the single instance's shading triangles (tlasRoot4 ~0), else null: a hit's triangle
	                                    address then needs no instance-record load (HitInstance) */
	const uint4* materials;          /* 128 B CUDAMaterial records (core_settings.h:94-104) */
	const lh2_CoreLightTri* areaLights;
	const lh2_CorePointLight* pointLights;
	const lh2_CoreSpotLight* spotLights;
	const lh2_CoreDirectionalLight* dirLights;
	int nArea, nPoint, nSpot, nDir;
	const float* sky;
	int skyW, skyH;
	const uint8_t* blueNoise;
	float geometryEpsilon, clampValue;
	const int* sceneError;           /* nonzero: the scene is unsafe to traverse (TLAS too deep); trace kernels exit */
	const uint32_t* argb32;          /* texel storage (rendercore.cpp:296-336): ARGB32 / NRM32 u32 texels */
	const uint32_t* nrm32;
	uint32_t argb32Count, nrm32Count;
};

struct BounceAdvance  /* the hand-off to the next bounce (advance_bounce, lh2_kernels.hip) */
{
	const uint32_t* segNext;         /* the extension rays' segment counts: the next bounce's paths */
	const uint32_t* segNextBack;     /* ... and those at the segments' ends (two-ended segments) */
	uint32_t* segRetire;             /* this bounce's path counts, zeroed for the next shade launch's extensions */
	uint32_t* segRetireBack;
	uint32_t* rayCountLog;           /* [pathLength] = rays of the next bounce */
	uint32_t* hostActiveLog;         /* pinned host copy of the same (the host's early exit), or null */
	int zeroLog;                     /* nonzero: also zero rayCountLog past pathLength (the path tail counts into it) */
	/* shadow overlap (RenderCore setting "shadowOverlap"): the shadow rays queued so far, per segment, into
	   shadowSnap (the side launch's segment counts) and into the final shadow launch's work-queue heads
	   (shadowCursor, LH2_CURSOR_STRIDE apart), which then start behind them; null: off */
	uint32_t* shadowSnap;
	uint32_t* shadowCursor;
};

struct ShadeParams    /* shadeKernel arguments (pathtracer.h:54-59), SoA path state */
{
	const uint32_t* segCounts; uint32_t segStride;     /* input paths: a segmented stream (see LH2_SEGS) */
	const uint32_t* segBack;                           /* ... with records at the segments' ends (null: none) */
	uint32_t* segOut; uint32_t* segOutBack;            /* extension rays: segment counts (Counters::segPath / segBack) */
	/* extension rays whose chord through the scene box (chordLo, chordHi) is at most chordCut go to the
	   end of their segment (segOutBack): the next trace launch takes them last, so the rays left in
	   flight when its work queues run dry are short ones (longest-first scheduling); 0: all at the start */
	float chordLo[3], chordHi[3], chordCut;
	int advance; BounceAdvance adv;                    /* nonzero: the launch's last block hands off to the next bounce */
	uint32_t shadowStride;                             /* shadow-ray segments: capacity of each */
	const float4* rayO; const float4* rayD; const float4* T4; const float4* Q4; const uint4* hits;
	float4* rayOut; float4* rayDOut; float4* T4Out; float4* Q4Out;
	float4* shO; float4* shD; float4* shP;
	float4* acc;
	Counters* counters;
	int w, h, pass, pathLength, maxPathLength, probePixel;
	uint32_t R0;
	float spreadAngle;               /* ViewPyramid::spreadAngle: ray cone width per unit distance (texture LOD) */
	int primeRef;                    /* RenderCore_PrimeRef shading (k_shade_ref) */
	/* no lights, no material that can emit (colour > 1, colour maps) or cut out, pathLength > 1: a hit
	   on a path that cannot extend (ENOUGH_BOUNCES or the last vertex) adds and emits nothing, so
	   k_shade<true> drops it after reading its hit and flags (misses still sample the sky) */
	int terminal;
	/* the camera fused into the primary packet launch (RenderCore::Render): the first shade launch zeroes the first
	   hvZeroWords words of the heavy-packet block the frame read, the block the next frame records into */
	uint32_t* hvZero; uint32_t hvZeroWords;
};

struct TraceArgs      /* one ray stream: rays in, hits (closest) or occlusion (any) out */
{
	const float4* rayO; const float4* rayD;
	/* the rays: a segmented stream (see LH2_SEGS), counts from device memory (segCounts), or, with
	   segCounts null, countFixed rays stored densely (segments of segStride) */
	const uint32_t* segCounts; uint32_t segStride; uint32_t countFixed;
	const uint32_t* segBack;                          /* two-ended segments: rays at the segments' ends (null: none) */
	uint32_t* cursor;                                 /* LH2_SEGS zeroed work-queue heads, LH2_CURSOR_STRIDE apart */
	uint4* hits;                                      /* closest: {t, triid, instid, uv16} */
	uint32_t* mask;                                   /* any, mode 0: occlusion bits */
	const float4* potentials; float4* acc;            /* any, mode 1: fused finalizeConnection */
	int* gstack;                                      /* stack entries past LH2_STACK_LDS */
	uint32_t refill;                                  /* refill idle lanes once >= refill are idle (1..64) */
	uint32_t leafBatch;                               /* run triangle tests once >= leafBatch lanes parked a leaf */
	int version;                                      /* traversal loop: 7 (BVH4, lh2_trace4d.inc) or 1 (BVH2, trace_stream) */
	int packet;                                       /* nonzero: wave-uniform packet traversal (coherent rays, lh2_trace_packet.inc) */
	unsigned long long* stats;                        /* LH2_TRACE_STATS / LH2_TRACE_TIMES builds: per-launch counters */
	uint32_t shadeBatch;                              /* path tail (k_trace_path4d): shade once >= shadeBatch lanes finished a query */
	uint32_t tailWaves;                               /* path tail (lh2_launch_trace_path): the kernel variant for 4 waves per SIMD (4) or 3 */
	uint32_t traceWaves;                              /* BVH4 closest hit: the kernel variant for 8 waves per SIMD (8) or 7 */
	/* heavy-first packets (packet kernel, hvWrite non-null): the previous frame's packets that took more
	   than hvFactor x its mean node steps (hvRead: per-segment counts, step sums, a bit per packet and the
	   lists of packet bits) are taken first, the rest in order; this frame's are recorded into hvWrite.
	   A packet bit is segment x hvCap + its batch in the segment; hvTiles: packets of the launch */
	const uint32_t* hvRead; uint32_t* hvWrite; uint32_t hvCap, hvMaskWords, hvTiles; float hvFactor;
};
/* layout of a heavy-packet block: counts, step sums (LH2_SEGS x LH2_SEGCOUNT_STRIDE words each), the bit
   mask (hvMaskWords), then LH2_SEGS lists of hvCap packet bits; the camera launch zeroes the first
   LH2_HV_MASK + hvMaskWords words of the block the frame writes */
#define LH2_HV_CNT 0
#define LH2_HV_SUM (8 * 32)
#define LH2_HV_MASK (2 * 8 * 32)
/* traversal-loop statistics (diagnostic builds with -DLH2_TRACE_STATS; tools/trace_stats.py):
   wave-iterations, active-lane sum, leaf-phase iterations / lanes, walk iterations / lanes,
   triangle-test lane sum, triangle-loop iterations, refill events / lanes, iterations / active-lane
   sum once the queue is exhausted, wave time before / after exhaustion (100 MHz ticks) */
#define LH2_TSTAT_N 14

/* start / stop events of one launch, recorded by the dispatch itself (hipExtLaunchKernelGGL); null: none */
struct LaunchEvents { hipEvent_t start, stop; };

/* where k_finalize delivers the frame's statistics: the device counters / ray-count log / scene error,
   and the host's pinned FrameStats fields (hostCounters null: nothing is delivered) */
struct FrameStatsDev
{
	const Counters* counters; const uint32_t* rayLog;
	Counters* hostCounters; uint32_t* hostRayCount;
	const int* sceneError; int* hostSceneError;
	uint32_t* zeroHeads;    /* LH2_CURSOR_WORDS work-queue heads zeroed by the finalize (the primary launch's slot of the frame
	                           parity's block: its next user's launch may reset the rest while it runs, never its own) */
	float4* delta;          /* early shade: the frame's first-vertex contributions, added into the accumulator (and zeroed) by
	                           the finalize, so the previous frame's finalize never sees them */
};

extern "C" {
void lh2_launch_init_counters( Counters* c, uint32_t pathCount, uint32_t segStride, uint32_t* cursors, int cursorWords, LaunchEvents ev, hipStream_t st,
	int keepCursor = -1 );
void lh2_launch_counters_next( Counters* c, const BounceAdvance* a, int pathLength, int resetShadow, LaunchEvents ev, hipStream_t st );
void lh2_launch_camera( const CameraParams* p, const uint8_t* bn, float4* rayO, float4* rayD, float4* T4, float4* Q4, int jobCount, LaunchEvents ev, hipStream_t st );
void lh2_launch_trace_closest( const SceneDev* s, const TraceArgs* a, int grid, LaunchEvents ev, hipStream_t st );
/* the camera (k_camera's rays and path state) fused into the primary packet launch: a->rayO / rayD and T4 / Q4 are
   written, a->segCounts must be null (the paths are dense: countFixed); the frame's counters and work-queue heads are
   reset by k_init_counters on the core stream (the launch itself may run beside the previous frame's tail) */
void lh2_launch_trace_primary( const SceneDev* s, const TraceArgs* a, const CameraParams* cp, float4* T4, float4* Q4, int grid, LaunchEvents ev, hipStream_t st );
void lh2_launch_trace_any( const SceneDev* s, const TraceArgs* a, int grid, int fused, LaunchEvents ev, hipStream_t st );
int lh2_trace_blocks_per_cu( int waves );
int lh2_packet_blocks_per_cu( void );
void lh2_launch_shade( const SceneDev* s, const ShadeParams* p, int grid, LaunchEvents ev, hipStream_t st );
void lh2_launch_trace_path( const SceneDev* s, const TraceArgs* a, const ShadeParams* p, int grid, LaunchEvents ev, hipStream_t st );
int lh2_path_blocks_per_cu( int waves );
void lh2_touch_set( uint32_t* bitmap, uint32_t triWord, uint32_t words );   /* LH2_TOUCH builds only (lh2_trace4d.inc) */
void lh2_launch_spin( unsigned long long ticks, hipStream_t st );
void lh2_launch_pack_rows( const float4* acc, float4* dst, int w, int y0, int band, int bandStride, int rows, LaunchEvents ev, hipStream_t st );
void lh2_launch_unpack_rows( const float4* src, float4* acc, int w, int y0, int band, int bandStride, int rows, LaunchEvents ev, hipStream_t st );
/* the rows of a band partition (k_pack_rows' mapping); rows 0: every pixel */
struct RowMap { int w, y0, band, bandStride, rows; };
void lh2_launch_finalize( float4* acc, float4* out, int n, float scale, const FrameStatsDev* fs, LaunchEvents ev, hipStream_t st,
	const RowMap* rm = nullptr );
}

/* Segmented ray streams.  A stream of paths or rays lives in LH2_SEGS segments of one buffer:
   segment c holds count[c] records from index c * segStride (counters LH2_SEGCOUNT_STRIDE words
   apart, each on its own 128-B line).  Producers (the camera: densely; shade: extension and shadow
   rays) and consumers (trace, shade) take segment blockIdx % LH2_SEGS first - blocks go round-robin
   over the 8 XCDs, so that is the XCD's own segment - and every segment has its own work-queue head
   and its own compaction counter: the per-wave atomics of a launch spread over 8 words, where one
   word sustains only ~88 returning atomics per microsecond (MI355X_MICROARCH.md, 'dequeue'). */
#ifndef LH2_CHUNKS
#define LH2_CHUNKS 8
#endif
#define LH2_SEGS LH2_CHUNKS
#define LH2_SEGCOUNT_STRIDE 32
#define LH2_CURSOR_STRIDE 32
/* per trace launch: the segment heads, then the heavy-first packets' list heads (lh2_trace_packet.inc) */
#define LH2_CURSOR_WORDS (2 * LH2_CHUNKS * LH2_CURSOR_STRIDE)
#define LH2_HEAVY_CURSOR (LH2_CHUNKS * LH2_CURSOR_STRIDE)
#define LH2_MAX_BOUNCES 64                                   /* RenderCore_PrimeRef MAXPATHLENGTH (core_settings.h:25) */
#define LH2_CURSOR_SLOTS (2 * LH2_MAX_BOUNCES + 5)           /* launches per frame: [L] bounce L, [64 + L] shadow after bounce L, [130] shadow, [131] side shadow */
#define LH2_SHADOW_SLOT (2 * LH2_MAX_BOUNCES + 2)
/* traversal stacks: LH2_STACK_LDS entries per lane in LDS (16 x 256 x 4 B = 16 KiB per block), the rest in global memory */
#ifndef LH2_STACK_LDS
#define LH2_STACK_LDS 16
#endif
#define LH2_STACK_TOTAL 96
#define LH2_RAYLOG (LH2_MAX_BOUNCES + 8)   /* ray-count log words per frame parity (RenderCore::FrameRayLog) */
/* bits of the scene error flag (SceneDev::sceneError; any bit set: the trace kernels exit and the host raises FatalError) */
#define LH2_SCENE_ERR_DEPTH 1    /* BVH depth exceeds the traversal stack */
#define LH2_SCENE_ERR_QRANGE 2   /* a BVH4 node beyond the quantized grid's range (k_quantize4) */
