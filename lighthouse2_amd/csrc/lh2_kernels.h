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
	int spp;     /* > 1 (tiled, one launch for every slot): the samples of an 8x8 block in consecutive waves */
	int slotBase;  /* this launch writes slots [slotBase, slotBase + jobCount) of the tile, at 0.. (path groups) */
	int primeRef;  /* RenderCore_PrimeRef camera: uniform random numbers, no distortion (camera.h:57-60) */
	/* folded into the camera launch (no launches of their own): the frame's counter / work-queue
	   reset (initC non-null: what k_init_counters does), and the accumulator reset of a restart
	   (clearAcc non-null: each pixel's first sample zeroes it; the memset of rendercore.cpp:465) */
	Counters* initC; uint32_t* cursors; int cursorWords; uint32_t pathCount, segStride;
	float4* clearAcc;
	/* two-ended primary segments (camAlloc non-null; whole 8x8 tiles, segStride a multiple of 64): a tile
	   whose centre ray's length inside the scene box (chordLo, chordHi) is at most chordCut is written at
	   the end of its segment, so the primary trace takes the long (costly) tiles first.  camAlloc: this
	   frame's per-segment front counts (LH2_SEGS x LH2_SEGCOUNT_STRIDE words) then back counts, zeroed by
	   the previous frame's camera launch, which zeroes camZero (the other frame's block) for the next */
	uint32_t* camAlloc; uint32_t* camZero;
	uint32_t* hvZero; uint32_t hvZeroWords;   /* heavy-first packets: the block this frame records into (TraceArgs::hvWrite) */
	float chordLo[3], chordHi[3], chordCut;
};
#define LH2_CAM_ALLOC_WORDS (2 * 8 * 32)   /* front + back counts of the LH2_SEGS segments */

struct SceneDev       /* everything the traversal and shading kernels read, by value (kernarg) */
{
	const float4* nodes;
	const float4* tris;
	const DevInstance* inst;
	int tlasRoot, instCount;
	const float4* nodes4;            /* BVH4 of the same scene (traceVersion 4; null when not built) */
	int tlasRoot4;
	const lh2_CoreInstanceDesc* instDesc;
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
	uint32_t* shadowSnap; uint32_t* shadowCursor;   /* the shadow split's snapshot, or null */
	int zeroLog;                     /* nonzero: also zero rayCountLog past pathLength (the path tail counts into it) */
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
	float shadowCut;                                   /* shadow rays at most this long go to the end of their segment (0: none) */
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
	int version;                                      /* traversal loop: 1 (trace_stream), 2 (lh2_trace2.inc), 4 (BVH4, lh2_trace4.inc) */
	int packet;                                       /* wave-uniform packet traversal (coherent rays): 1 over the BVH2, 4 over the BVH4 */
	unsigned long long* stats;                        /* LH2_TRACE_STATS builds: LH2_TSTAT_N per-launch counters */
	/* tail hand-off (lh2_trace2.inc): once the queue is exhausted, a wave with fewer than tailLanes
	   active rays appends them to tailOut / tailOutUV {idx, bits(tbest), tri, inst} {u, v} - segment
	   blockIdx % LH2_SEGS, counters tailCounts (LH2_SEGCOUNT_STRIDE apart), tailStride records per
	   segment - and exits; a second launch of the same kernel (tail_args) continues them densely
	   from those records (tailIn) with the closest hit found so far as tmax, which gives the ray the
	   same closest hit (the hit does not depend on the visiting order) */
	uint4* tailOut; float2* tailOutUV; uint32_t* tailCounts; uint32_t tailStride, tailLanes;
	const uint4* tailIn; const float2* tailInUV;
	/* tail pool (lh2_trace2.inc): once the queue is exhausted, a wave holding at most `pool` rays
	   hands them, with their traversal state and stack, to another wave of its workgroup through
	   LDS and exits (0: off) */
	uint32_t pool;
	uint32_t shadeBatch;                              /* path tail (k_trace_path4d): shade once >= shadeBatch lanes finished a query */
	/* terminal trace (k_trace_term4d): the last bounce of a scene whose hits there add nothing (ShadeParams::
	   terminal); a ray that misses adds its sky sample to acc[pixel] as k_shade_last does (pathT4 / pathQ4:
	   the path state, wh: pixels per frame) and no hit record is written */
	const float4* pathT4; const float4* pathQ4; uint32_t wh;
	/* heavy-first packets (packet kernel, hvWrite non-null): the previous frame's packets that took more
	   than hvFactor x its mean node steps (hvRead: per-segment counts, step sums, a bit per packet and the
	   lists of packet bits) are taken first, the rest in order; this frame's are recorded into hvWrite.
	   A packet bit is segment x hvCap + its batch in the segment; hvTiles: packets of the launch */
	const uint32_t* hvRead; uint32_t* hvWrite; uint32_t hvCap, hvMaskWords, hvTiles; float hvFactor;
	/* shadow backfill (closest-hit launches, traceVersion 5-7, bfO non-null): once this launch's own queues
	   are dry and while any of its waves still walks a closest-hit ray, idle lanes take shadow rays queued
	   by earlier bounces - the stream bfO / bfD, front counts bfCounts (stable during the launch),
	   bfStride per segment - from the final shadow launch's work-queue heads bfCursor, claimed with a
	   bounded compare-and-swap so the final launch continues exactly behind them; an unoccluded one adds
	   its potential (potentials, acc) as that launch would */
	const float4* bfO; const float4* bfD; const uint32_t* bfCounts; uint32_t bfStride; uint32_t* bfCursor;
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
#define LH2_FS_GROUPS 4
struct FrameStatsDev
{
	int groups;
	const Counters* counters[LH2_FS_GROUPS]; const uint32_t* rayLog[LH2_FS_GROUPS];
	Counters* hostCounters[LH2_FS_GROUPS]; uint32_t* hostRayCount[LH2_FS_GROUPS];
	const int* sceneError; int* hostSceneError;
};

extern "C" {
void lh2_launch_init_counters( Counters* c, uint32_t pathCount, uint32_t segStride, uint32_t* cursors, int cursorWords, LaunchEvents ev, hipStream_t st );
void lh2_launch_counters_next( Counters* c, const BounceAdvance* a, int pathLength, int resetShadow, LaunchEvents ev, hipStream_t st );
void lh2_launch_camera( const CameraParams* p, const uint8_t* bn, float4* rayO, float4* rayD, float4* T4, float4* Q4, int jobCount, LaunchEvents ev, hipStream_t st );
void lh2_launch_trace_closest( const SceneDev* s, const TraceArgs* a, int grid, LaunchEvents ev, hipStream_t st );
void lh2_launch_trace_any( const SceneDev* s, const TraceArgs* a, int grid, int fused, LaunchEvents ev, hipStream_t st );
int lh2_trace_blocks_per_cu( void );
int lh2_any4d_blocks_per_cu( void );
int lh2_packet_blocks_per_cu( void );
void lh2_launch_shade( const SceneDev* s, const ShadeParams* p, int grid, LaunchEvents ev, hipStream_t st );
void lh2_launch_trace_path( const SceneDev* s, const TraceArgs* a, const ShadeParams* p, int grid, LaunchEvents ev, hipStream_t st );
void lh2_launch_trace_term( const SceneDev* s, const TraceArgs* a, int grid, LaunchEvents ev, hipStream_t st );
int lh2_path_blocks_per_cu( void );
void lh2_launch_spin( unsigned long long ticks, hipStream_t st );
void lh2_launch_pack_rows( const float4* acc, float4* dst, int w, int y0, int band, int bandStride, int rows, LaunchEvents ev, hipStream_t st );
void lh2_launch_unpack_rows( const float4* src, float4* acc, int w, int y0, int band, int bandStride, int rows, LaunchEvents ev, hipStream_t st );
/* the rows of a band partition (k_pack_rows' mapping); rows 0: every pixel */
struct RowMap { int w, y0, band, bandStride, rows; };
void lh2_launch_finalize( const float4* acc, float4* out, int n, float scale, const FrameStatsDev* fs, LaunchEvents ev, hipStream_t st,
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
/* per trace launch: the segment heads, the heads of its tail launch, the tail segment counts */
#define LH2_CURSOR_WORDS (3 * LH2_CHUNKS * LH2_CURSOR_STRIDE)
#define LH2_TAIL_CURSOR (LH2_CHUNKS * LH2_CURSOR_STRIDE)
#define LH2_TAIL_COUNT (2 * LH2_CHUNKS * LH2_CURSOR_STRIDE)
#define LH2_MAX_BOUNCES 64                                   /* RenderCore_PrimeRef MAXPATHLENGTH (core_settings.h:25) */
#define LH2_CURSOR_SLOTS (2 * LH2_MAX_BOUNCES + 4)           /* launches per frame: [L] bounce L, [64 + L] shadow after bounce L, [130] shadow */
#define LH2_SHADOW_SLOT (2 * LH2_MAX_BOUNCES + 2)
/* the BVH4 loops' LDS stack (lh2_trace4d.inc): LH2_STACK_TCULL 1 keeps each entry's entry distance (16 bits) beside
   it, in 12 LDS entries instead of 16 (the same LDS per block), and closest-hit walks pop the entries beyond their
   closest hit without a node step; the global part is sized for the smaller one.  Parity-exact, measured no faster
   (config-2 bounce 0.579 vs 0.576 ms, profiles/r02zm_ab_stack_tcull.txt): off */
#ifndef LH2_STACK_TCULL
#define LH2_STACK_TCULL 0
#endif
#define LH2_STACK4_LDS (LH2_STACK_TCULL ? 12 : LH2_STACK_LDS)
#define LH2_STACK4_LDS_INTS (LH2_STACK4_LDS * 256 + (LH2_STACK_TCULL ? LH2_STACK4_LDS * 128 : 0))
#ifndef LH2_STACK_LDS
#define LH2_STACK_LDS 16
#endif
#define LH2_STACK_TOTAL 96
