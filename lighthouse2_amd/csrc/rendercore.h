/* rendercore.h - host side of the MI355X render core (counterpart of
   RenderCore_OptixPrime_B/rendercore.h:48-142; same method names and call contract). */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lh2_core_types.h"
#include "bvh_build.h"
#include "bvh_gpu.h"
#include "lh2_kernels.h"
#include "lh2_device.h"

namespace lh2 {

void FatalError( const char* fmt, ... );

template <class T> struct DevBuf
{
	T* ptr = nullptr;
	size_t count = 0;
	DevBuf() = default;
	DevBuf( const DevBuf& ) = delete;
	DevBuf& operator=( const DevBuf& ) = delete;
	~DevBuf() { free(); }
	void free() { if (ptr) (void)hipFree( ptr ); ptr = nullptr; count = 0; }
	void resize( size_t n )   /* discards contents */
	{
		if (n <= count && ptr) return;
		free();
		if (n == 0) n = 1;
		if (hipMalloc( (void**)&ptr, n * sizeof( T ) ) != hipSuccess) FatalError( "hipMalloc of %zu bytes failed", n * sizeof( T ) );
		count = n;
	}
	void adopt( T* p, size_t n ) { free(); ptr = p, count = n; }   /* takes ownership of a hipMalloc'ed block */
	void upload( const T* src, size_t n, hipStream_t st )
	{
		resize( n );
		if (n) if (hipMemcpyAsync( ptr, src, n * sizeof( T ), hipMemcpyHostToDevice, st ) != hipSuccess) FatalError( "upload failed" );
	}
};

/* a deferred CPU BLAS build (RenderCore::FlushBuilds) and its host results.  Shared by the sub-cores of a MultiDevice:
   the first core to flush runs it (once, std::call_once), every core uploads the results to its own device, and the last
   reference frees them (round 6, VERDICT r5 #7: no N-fold build at deviceCount N) */
struct HostBlas
{
	std::once_flag once;
	std::function<void( HostBlas&, int )> job;   /* its argument: host threads for the build */
	std::vector<float> nodes2, tris48, nodes4;
	int leafTris = 0, nodeCount = 0, maxDepth = 0, depth4 = 0;
	void Run( int threads );
};

struct CoreMeshHost   /* RenderCore always copies what it needs (rendercore.h:57): all of it on the device */
{
	int triCount = 0;
	int leafTris = 0;                    /* triangle records of the BLAS leaves (> triCount with spatial splits) */
	float aabbLo[3], aabbHi[3];          /* lo.x > hi.x: empty mesh */
	DevBuf<float4> shadeTris;            /* CoreTri4[] in original order, for shading */
	DevBuf<float4> bvhNodes, bvhTris;    /* BLAS with mesh-local refs; relocated into the scene arrays by UpdateToplevel */
	int nodeCount = 0, maxDepth = 0;
	DevBuf<float4> bvh4Nodes;            /* the same BLAS collapsed to BVH4 (CollapseBvh4), mesh-local refs */
	int node4Count = 0, depth4 = 0;
	std::shared_ptr<HostBlas> build;     /* a deferred CPU build not uploaded yet (null: none) */
};

struct CoreInstanceHost { int mesh; float T[16]; float inv[16]; };

/* the frame's path and ray streams (segmented, lh2_kernels.h) with their counters, work-queue heads,
   traversal stacks and the events that time the frame's launches */
struct PathStreams
{
	size_t cap = 0;                      /* paths the buffers hold */
	DevBuf<float4> rayO[2], rayD[2], T4[2], Q4[2];
	DevBuf<uint4> hits;
	/* the primary rays, path state and hits of a fused frame (k_trace_primary_packet writes them, its first shade
	   launch reads them): apart from the bounce ping-pong, so the next frame's primary launch can run beside this
	   frame's later bounces */
	DevBuf<float4> rayOP[2], rayDP[2], T4P[2], Q4P[2];   /* per frame parity */
	DevBuf<uint4> hitsP[2];
	DevBuf<float4> shO, shD, shP;        /* 2 x shCap (frame parity) */
	DevBuf<uint32_t> shMask;             /* 2 x shMaskWords */
	size_t shCap = 0, shMaskWords = 0;
	DevBuf<int> gstack;
	DevBuf<int> sideStack;               /* the side shadow launch's global stack (shadowOverlap) */
	DevBuf<int> aheadStack;              /* a per-ray primary launch beside the previous frame (RenderCore::kCamAhead) */
	DevBuf<uint32_t> shSnap;             /* the shadow rays queued before the path tail, per segment (advance_bounce), per frame parity */
	/* per frame parity (fp): two consecutive frames' counters, work-queue heads, shadow streams and ray-count logs are
	   apart, so the next frame's first launches can run beside this frame's last ones (frame overlap, early shade) */
	DevBuf<Counters> counters;           /* 2 */
	DevBuf<uint32_t> cursors;            /* 2 x LH2_CURSOR_SLOTS x LH2_CURSOR_WORDS work-queue heads */
	DevBuf<uint32_t> rayLog;             /* 2 x LH2_RAYLOG */
	DevBuf<uint32_t> hv;                 /* heavy-first packets: two blocks (TraceArgs::hvRead / hvWrite), the frame parity picks */
	uint32_t hvCap = 0, hvMaskWords = 0, hvBlock = 0, hvParity = 0;
	uint32_t* activeLog = nullptr;       /* pinned: extension rays after each bounce (advance_bounce) */
	/* a launch carries only a stop event (a start event costs its dispatch ~5 us of idle GPU); a timed
	   interval runs from the previous launch's stop event, so it includes the launch gap */
	hipEvent_t evTrace[LH2_MAX_BOUNCES + 1] = {}, evShade[LH2_MAX_BOUNCES + 1] = {}, evShadowB[LH2_MAX_BOUNCES + 1] = {};
	hipEvent_t evCount[LH2_MAX_BOUNCES + 2] = {}, evCamera = nullptr, evShadow = nullptr;
	hipEvent_t evSide = nullptr, fromSide = nullptr;   /* shadowOverlap: the side launch */
	bool sideOn = false;                 /* this frame traced its early shadow rays on the side stream */
	hipEvent_t countReady[LH2_MAX_BOUNCES + 2] = {};   /* [L]: the event after which bounce L's hand-off is done (evShade or evCount, not owned) */
	hipEvent_t fromTrace[LH2_MAX_BOUNCES + 1] = {}, fromShade[LH2_MAX_BOUNCES + 1] = {}, fromShadowB[LH2_MAX_BOUNCES + 1] = {}, fromShadow = nullptr;
	/* this frame */
	uint32_t count = 0, segStride = 0, shadowStride = 0;
	int in = 0, pl = 0;
	int tailL = 0;                       /* this frame's path-tail launch (pathLength), 0: none */
	bool hvOn = false;                   /* this frame's primary packets run heavy-first (TraceArgs::hvRead) */
	/* the camera fused into the primary packet launch (setting "cameraFused"): the heavy-packet block the next frame
	   records into is zeroed by the frame's first shade launch (hvNextZeroed: it was) */
	bool hvNextZeroed = false;
	/* frame overlap (setting "frameOverlap"): the primary launch of a fused frame runs on the ahead stream after the
	   previous frame's first shade launch, unless something since then needs it to wait for the whole previous frame */
	bool lastFused = false, relaid = true;
	uint64_t lastSceneVersion = 0;
	hipEvent_t overlapEv = nullptr;      /* the last frame's shade launch the next primary launch waits for (not owned) */
	hipEvent_t evEarlyEnd = nullptr;     /* an early frame that ended before its path tail: overlapEv on the core stream (owned) */
	hipEvent_t prevStop = nullptr;
	int fp = 0;                          /* this (the last) frame's parity */
	/* early shade (setting "earlyShade"): the next frame's first shade launch also runs beside this frame's launches
	   after overlapEv.  Those use one ping-pong buffer (busy: the path tail's, or the last bounce's rays) and write
	   neither (earlyOk), so the next frame's first shade writes the other one */
	int busy = 0;
	bool earlyOk = false, early = false;
};

struct FrameStats   /* per-frame values delivered by k_finalize into pinned host memory */
{
	uint32_t rayCount[LH2_MAX_BOUNCES + 1];
	Counters counters;
	int sceneError;
};

class RenderCore
{
public:
	void Init();
	void SetProbePos( int x, int y ) { probeX = x, probeY = y; }
	void SetTarget( uint32_t w, uint32_t h, uint32_t spp );
	void SetInteropTexture( uint32_t glTextureId );   /* 0: headless (frame stays in the device buffer) */
	void Setting( const char* name, float value );
	bool GetSetting( const char* name, float& value ) const;
	void Render( const lh2_ViewPyramid& view, int converge );
	void Shutdown();
	void SetTextures( const lh2_CoreTexDesc* tex, int textureCount );
	void SetMaterials( const lh2_CoreMaterial* mat, int materialCount );
	void SetLights( const lh2_CoreLightTri* areaLights, int areaLightCount, const lh2_CorePointLight* pointLights, int pointLightCount,
		const lh2_CoreSpotLight* spotLights, int spotLightCount, const lh2_CoreDirectionalLight* directionalLights, int directionalLightCount );
	void SetSkyData( const float* pixels, uint32_t width, uint32_t height );
	void SetGeometry( int meshIdx, const float* vertexData, int vertexCount, int triangleCount, const lh2_CoreTri* triangles, const uint32_t* alphaFlags );
	/* MultiDevice: the same mesh as SetGeometry, sharing src's deferred CPU BLAS build (built once, uploaded here too) */
	void AdoptGeometry( int meshIdx, int triangleCount, const lh2_CoreTri* triangles, const RenderCore& src );
	void FlushPendingBuilds() { FlushBuilds(); }
	static int BlasBuildCount();         /* CPU BLAS builds run in this process (the build-once check) */
	void SetInstance( int instanceIdx, int meshIdx, const float* matrix16 );
	void UpdateToplevel();
	lh2_CoreStats GetCoreStats();

	/* extensions beyond the reference ABI (tile partition, headless output, unit-level kernels) */
	void SetTile( int y0, int y1 ) { tileY0 = y0, tileY1 = y1, tileBand = 0, tileStride = 0, tileChanged = true; }
	/* rank r of n owns the row bands [r*band + k*n*band, +band): balanced multi-GPU partition */
	void SetTileBands( int rank, int nranks, int band ) { tileY0 = rank * band, tileY1 = -1, tileBand = band, tileStride = nranks * band, tileChanged = true; }
	int TileRows() const;
	void Synchronize();
	void GetAccumulator( float* hostOut4 );                /* full frame, raw accumulator */
	void CopyAccumulatorRows( void* devDst, int y0, int y1 ); /* D2D copy of rows [y0,y1) */
	void PackTile( void* devDst, bool ordered = false, void* consumer = nullptr );   /* owned rows, local order (async); ordered: with the stream consumer (null: the null stream) both ways */
	hipEvent_t evConsumer = nullptr, evPacked = nullptr;
	void GetFrame( float* hostOut4 );                      /* finalizeRender output: acc / samplesTaken */
	/* in-process multi-device gather (multidevice.cpp): rows packed by the core of rank `rank` of a
	   band partition, already on this device, into this accumulator (async); then the frame output
	   of the whole accumulator again (finalizeRender + display copy, no statistics) */
	void UnpackTile( const void* devSrc, int rank, int nranks, int band );
	void FinalizeFrame();
	bool displayAtFinalize = false;   /* rank 0 of MultiDevice: the display copy follows the gather (FinalizeFrame) */
	void CopyFrameAsync( void* devDst );   /* the last finalized frame, D2D on the core stream */
	hipStream_t Stream() const { return stream; }
	int Device() const { return device; }
	int SamplesTaken() const { return samplesTaken; }
	void GetRayCounts( uint32_t* out17 );
	/* diagnostics: the last frame's queued shadow rays {O, tmin} {D, tmax} {potential rgb, pixel bits}, segment by segment */
	int DebugShadowRays( float* o4, float* d4, float* p4, int cap );
	int DebugBvh4( float* f32Nodes, uint32_t* qNodes, int cap );   /* the BVH4 nodes, f32 (32 floats) and quantized (16 words) */
	void DebugPoisonTlas( float value );   /* test hook: both TLAS slots' node regions filled with value */
	void TraceClosest( const float* orgTmin4, const float* dirTmax4, int n, uint32_t* hits4 );   /* host in/out */
	void TraceAny( const float* orgTmin4, const float* dirTmax4, int n, uint32_t* occluded );
	void TraceClosestDevice( const void* rayO, const void* rayD, int n, void* hits, int iterations, float* msOut );
	void GenerateEyeRays( const lh2_ViewPyramid& view, uint32_t R0, int pass, float* orgTmin4, float* dirTmax4, float* state8 );
	void SceneInfo( int* nodeCount, int* triCount, int* maxDepth, int* instCount );
	float lastKernelMs[8] = {};  /* traceTime of the last frame per bounce (diagnostics) */

	lh2_CoreStats coreStats{};
	hipStream_t stream = nullptr;
	hipStream_t sideStream = nullptr;    /* shadowOverlap: the device's least priority (the default level on MI355X) */
	hipStream_t aheadStream = nullptr;   /* frameOverlap: the fused primary launch */

private:
	void EnsureBuffers();
	void ConcatenateBlas( int instanceCount );
	void BuildBlas4( CoreMeshHost& m, const float* nodes2 );
	void FlushBuilds();
	bool pendingBuilds = false;
#ifdef LH2_TOUCH
	DevBuf<uint32_t> touchMap;           /* diagnostic build: the touched-record bitmap (lh2_trace4d.inc) */
	uint32_t touchNodeWords = 0;
	void TouchBegin();
	void TouchReport( int pathLength );
#endif
	int buildThreads = 0;                /* host threads of the deferred BLAS builds (setting "buildThreads"; 0: LH2_BUILD_THREADS,
	                                        OMP_NUM_THREADS or min(16, cores)) */
	void EnsurePaths( uint32_t paths );
	void EnsureStack();
	void CheckSceneError();
	bool UsePackets() const;
	SceneDev MakeSceneDev();             /* the latest TLAS slot's scene; the core stream waits for its update (SyncTlas) */
	void SyncTlas();
	Counters* FrameCounters() const { return ps.counters.ptr + ps.fp; }
	uint32_t* FrameCursors() const { return ps.cursors.ptr + (size_t)ps.fp * LH2_CURSOR_SLOTS * LH2_CURSOR_WORDS; }
	uint32_t* FrameRayLog() const { return ps.rayLog.ptr + (size_t)ps.fp * LH2_RAYLOG; }
	TraceArgs StreamArgs( const float4* o, const float4* d, const uint32_t* segCounts, uint32_t segStride, uint32_t* cursor, bool coherent ) const;
	int TraceGrid() const { return smCount * blocksPerCU; }
	int UnitGrid() const { return smCount * std::min( blocksPerCU, unitTraceWaves == 8 ? traceBlocksPerCU8 : traceBlocksPerCU7 ); }
	int PacketGrid() const { return smCount * packetBlocksPerCU; }   /* packet kernel: its own occupancy */
	int PathGrid() const { return smCount * std::min( blocksPerCU, pathBlocksPerCU ); }   /* path tail: its occupancy, within the stack's */

	int device = 0, smCount = 256, blocksPerCU = 8, maxBlocksPerCU = 8, packetBlocksPerCU = 8, pathBlocksPerCU = 3, pathBlocksPerCU4 = 4;
	int traceBlocksPerCU7 = 7, traceBlocksPerCU8 = 8;   /* occupancy of the closest-hit kernel's 7- and 8-wave variants */
	/* closest-hit launches with the chip alone: 0, the 7-wave variant (72 VGPRs); 7 or 8: that variant.  8 for every scene won
	   in round 4; with the early node loads (round 5: single-instance loops only) the single-instance 8-wave loop spills, and 7
	   there is config 3 -3.4 %, 4K -3 %, the N = 8 share -2.9 % (profiles/r05f_ab_trace_waves.txt); round 6 gave the instanced
	   loops the early loads too, at 7 waves (config 5 9.31-9.32 -> 9.19-9.21 ms; at 8 they spill: 13.2 ms,
	   profiles/r06l_ab_instanced_early.txt) */
	int traceWaves = 0;
	int userBlocksPerCU = 0;             /* setting "traceBlocksPerCU" (0: not set) */
	/* the closest-hit kernel variant a per-ray launch with the chip alone takes (traceWaves 0: 7), and its grid's
	   blocks per CU: the variant's occupancy, or the user's setting within it */
	int ScenePicksWaves() const { return traceWaves ? traceWaves : 7; }
	int ClosestBlocksPerCU( int waves ) const
	{
		const int occ = waves == 7 ? traceBlocksPerCU7 : traceBlocksPerCU8;
		return userBlocksPerCU ? std::min( userBlocksPerCU, occ ) : occ;
	}
	int unitTraceWaves = 7;              /* the unit queries' variant: 7 (the config-2 bounce rays alone: 0.481 vs 0.515 ms, r04ag) */
	bool initialized = false;
	/* scene */
	std::vector<CoreMeshHost*> meshes;
	std::vector<CoreInstanceHost> instances;
	bool geometryDirty = true, instancesDirty = true;
	DevBuf<float4> dNodes, dTris;
	DevBuf<float4> dNodes4;              /* BVH4: all BLAS (relocated), then the TLAS as two-child nodes */
	DevBuf<uint4> dNodes4q;              /* the same nodes with quantized child boxes (GpuBvhBuilder::Quantize4) */
	DevBuf<uint8_t> dInst[2];            /* DevInstance[], per TLAS slot */
	DevBuf<lh2_CoreInstanceDesc> dInstDesc[2];
	int tlasRoot = 0, blasNodeCount = 0, blasTriCount = 0, blasMeshTris = 0, sceneMaxDepth = 0;   /* blasTriCount: leaf triangle records; blasMeshTris: triangles */
	std::vector<int> meshNodeBase, meshTriBase, meshNode4Base;
	int tlasCapacity = 0, maxBlasDepth = 0;
	int blasNode4Count = 0, maxBlas4Depth = 0;
	int bvh4 = 1;                        /* build BVH4 copies of the BLAS (the default traversal loop needs them) */
	/* the 8-wide compressed BVH of round 5 (W8, Ylitie et al. 2017) measured slower in every configuration (its node step
	   issued 1.8x the BVH4 step's VALU for 0.72x the steps: profiles/r05_ab_w8.txt) and was removed in round 6 (commit
	   22e0032 holds it) */
	/* stack entries a ray may need: the BVH2 loop's BLAS depth, the BVH4 loop's 3 per level */
	int StackDepthBound() const { return bvh4 ? std::max( maxBlasDepth, 3 * maxBlas4Depth ) : maxBlasDepth; }
	bool tlasOnDevice = false;           /* TLAS of the last UpdateToplevel built by the GPU (depth in dTlasDepth) */
	GpuBvhBuilder gpuBvh;
	DevBuf<float> dMeshBounds;           /* 6 per mesh */
	DevBuf<float> dInstT;                /* 16 per instance */
	DevBuf<int> dInstMesh;
	DevBuf<int> dSceneError, dTlasDepth; /* dSceneError: one flag per TLAS slot */
	DevBuf<int> dBlasQError;             /* the BLAS quantizer's range flag (LH2_SCENE_ERR_QRANGE), copied into dSceneError per TLAS update */
	uint8_t* stage[2] = {};              /* pinned staging of UpdateToplevel (double-buffered) */
	size_t stageBytes[2] = {};
	hipEvent_t evStage[2] = {};
	int stageSlot = 0;
	/* TLAS slots (round 4): an instance-only UpdateToplevel writes the instance tables, the TLAS (the BVH2 and BVH4 regions
	   after the BLAS, tlasCapacity nodes per slot) and the scene-error flag of the slot no frame in flight reads, on the ahead
	   stream behind the last frame that read that slot (evTlasFree), so an animated frame's primary launch can still run
	   beside the previous frame; the core stream waits for the update (evTlasReady) before its next launch */
	int tlasSlot = 0;
	int tlasNodeCount[2] = { 1, 1 };     /* the nodes of each slot's TLAS (UpdateToplevel) */
	bool tlasPending = false, tlasFreeValid[2] = {};
	hipEvent_t evTlasReady = nullptr, evTlasFree[2] = {};
	int TlasBase2( int s ) const { return blasNodeCount + s * tlasCapacity; }
	int TlasBase4( int s ) const { return blasNode4Count + s * tlasCapacity; }
	int* SceneErr( int s ) const { return dSceneError.ptr + s; }
	hipGraphicsResource_t glResource = nullptr;   /* registered GL_RGBA32F target texture */
	uint32_t glTexture = 0;
	DevBuf<uint4> dMaterials;
	std::vector<lh2_CoreTexDesc> texDescs;   /* copies, firstPixel assigned per storage (rendercore.cpp:276-292) */
	DevBuf<uint32_t> dArgb32, dNrm32;        /* continuous texel arrays (rendercore.cpp:299-336) */
	DevBuf<float4> dArgb128;
	DevBuf<lh2_CoreLightTri> dArea; DevBuf<lh2_CorePointLight> dPoint; DevBuf<lh2_CoreSpotLight> dSpot; DevBuf<lh2_CoreDirectionalLight> dDir;
	int nArea = 0, nPoint = 0, nSpot = 0, nDir = 0;
	DevBuf<float> dSky; int skyW = 0, skyH = 0;
	DevBuf<uint8_t> dBlueNoise;
	/* settings (rendercore.h DeviceVars; constant-memory defaults: .cuda.cu:38-39) */
	float geometryEpsilon = 0.0f, clampValue = 10.0f;
	int maxPathLength = 16;
	bool diffuseOnly = false;            /* SetMaterials: no material can continue a path past its second vertex */
	bool canEmit = true;                 /* SetMaterials: some material may shade as emissive (colour > 1 or colour maps) or cut out */
	int primeRef = 0;                    /* RenderCore_PrimeRef validation mode (setting "primeRef") */
	int probeX = 0, probeY = 0;
	/* target + frame buffers */
	int scrwidth = 0, scrheight = 0, scrspp = 1;
	int tileY0 = 0, tileY1 = -1, tileBand = 0, tileStride = 0;
	DevBuf<float4> accumulator, frame;
	DevBuf<float4> delta;                /* early shade: the first shade launch's accumulator additions (FrameStatsDev::delta), per frame parity */
	PathStreams ps;                      /* on `stream`; also serves the unit-level trace calls */
	bool tileChanged = false;            /* the next restart clears the whole accumulator, not only the tile's pixels */
	bool frameShadows = true;            /* the last frame queued shadow-ray launches (the scene has lights) */
	bool singleInstanceStart = true;     /* one instance of a non-empty mesh: rays start at its TLAS leaf (SceneDev::tlasRoot) */
	bool terminalShade = true;           /* k_shade<true> for shade passes whose hits cannot contribute (ShadeParams::terminal) */
	FrameStats* hostStats = nullptr;     /* pinned */
	bool statsPending = false;
	hipEvent_t evFrame[3] = {};          /* the frame's start marker, its end (finalize), the previous frame's end */
	bool frameEndRecorded = false, prevFrameEndValid = false, frameWasOverlapped = false;
	int tiledRays = 1;                   /* primary rays stored in 8x8 pixel blocks per wave (coherent packets) */
	int cameraFused = 1;                 /* primary rays made by the packet launch itself (k_trace_primary_packet), no camera launch */
	/* a fused frame's primary launch beside the previous frame's later bounces (aheadStream): 1, after its shade launch
	   before the path tail (its first without one); 2, after its first shade launch; 0: off.  Right after the previous
	   frame's primary launch, beside its first shade launch too, measured slower (profiles/r05_ab_frame_overlap_chain.txt) */
	int frameOverlap = 1;
	/* with frameOverlap 1: the next frame's first shade launch follows its primary launch on the ahead stream, beside this
	   frame's path tail and shadow launches, instead of after them on the core stream (frames whose later launches use one
	   ping-pong buffer: PathStreams::earlyOk).  Accumulator additions of the two frames then interleave: the sum matches
	   the sequential one within float rounding, not bit for bit (the first-vertex depths, w, stay exact) */
	int earlyShade = 1;
	/* fixed policy constants (round 5: the knobs behind them were pruned; the values are the measured winners).
	   Small frames (at most kSmallFramePaths paths: the N = 8 rank share, config 3) take the early shade (beside a large frame's
	   tail it gains nothing and its fold costs: config-4 N = 1 1 % slower, r04e_ab.txt) and the path tail at 3 blocks per CU
	   beside the side shadow launch (large frames 2: the 4K frame 6.54 vs 6.64-6.69 ms, r04p_ab.txt, r04r_ab.txt) */
	static constexpr float kSmallFramePaths = 2.5e6f;
	/* the shade launches' grid: about kShadePathsPerThread paths per thread, between the trace grid and kShadeMaxBlocks per CU
	   (the N = 8 share 12 blocks per CU, config 3 24: -1.5 / -1.5 %, r04al_ab.txt, r04am_ab.txt, r04av_ab.txt) */
	static constexpr float kShadePathsPerThread = 1.3f;
	static constexpr int kShadeMaxBlocks = 24;
	/* blocks per CU of a closest-hit launch that the next frame's primary launch runs beside (an overlapped frame's later
	   bounces, no path tail): the packets' latency-bound waves get slots from the start (config 2 +4 %, r03q_ab_trace_blocks.txt) */
#ifndef LH2_OVERLAP_TRACE_BLOCKS
#define LH2_OVERLAP_TRACE_BLOCKS 5
#endif
	static constexpr int kOverlapTraceBlocks = LH2_OVERLAP_TRACE_BLOCKS;
	/* packets while the BVH + triangles fit the 256 MB Infinity Cache (a packet's node and triangle records come through
	   the scalar cache, one at a time: beyond the cache each is a DRAM round trip).  Config 3 (134 MB): primary 0.29 ->
	   0.24 ms with packets; config 5 (1.4 GB): 5.3 -> 7.8 ms (profiles/r02zc_ab_packets_configs.txt) */
	static constexpr double kPacketMaxBytes = 256.0 * 1048576.0;
	uint64_t sceneVersion = 0;           /* incremented by every change of device-resident scene data or buffers */
	/* dynamic ray fetch: refill a wave's idle lanes once this many are idle; BLAS leaves parked until this many
	   lanes hold one (lh2_trace4d.inc).  Primary rays: coherent 8x8-tiled batches (profiles/r01c_sweep_bvh4.jsonl,
	   r02y_ab_v7.txt); leafBatch 8 with the quantized nodes (bounce 0.492 -> 0.488 ms, N = 8 share 1.35 -> 1.32 ms,
	   r03k_ab_leafbatch.txt) */
	int refillOther = 48, leafBatch = 8;   /* primary rays traced per ray (no packets) take the same (profiles/r04ag_refill_sweep.txt;
	                                          round 5: 32 / 40 / 56 no better, r05f_ab_refill.txt, r05f_ab_beside_refill.txt) */
	/* the shadow launches park BLAS leaves until 16 lanes hold one (the closest-hit launches: leafBatch): config 3 -0.4 %, the
	   4K frame -0.9 %, the N = 8 share -0.3 % against 8; 2 and 4 slower, 24 no better; their refill stays refillOther (32 and
	   60 slower) (profiles/r05f_ab_lazy_frame_shadow_sweep.txt, r05f_ab_shadow_leafbatch.txt) */
	static constexpr int kShadowLeafBatch = 16;
#ifndef LH2_PRIMARY_RESETS
#define LH2_PRIMARY_RESETS 1
#endif
	/* an overlapped frame's counter and work-queue resets done by its primary launch (as behind the previous frame), not by
	   a k_init_counters launch before it on the ahead stream */
	static constexpr bool kPrimaryResets = LH2_PRIMARY_RESETS != 0;
#ifndef LH2_CAM_AHEAD
#define LH2_CAM_AHEAD 1
#endif
	/* frames traced per ray (no packets) overlap like packet frames: camera + per-ray primary launch on the ahead stream
	   (config 5 9.70-9.73 -> 9.48-9.51 ms, profiles/r06b_ab_cam_ahead.txt); the touch build counts one closest-hit launch at a
	   time (TouchReport), so it keeps them behind the previous frame */
#ifdef LH2_TOUCH
	static constexpr bool kCamAhead = false;
#else
	static constexpr bool kCamAhead = LH2_CAM_AHEAD != 0;
#endif
	int bvhMaxLeaf = 1;
	/* spatial splits (SBVH): overlap threshold x root area; 0 = off.  1e-3 (round 4; 1e-5 before): the same node steps and
	   triangle tests per ray (tools/bvh_quality.cpp: config 2 26.62 / 6.78 vs 26.64 / 6.68, the room 14.58 / 1.83 both)
	   at a third of the build time (config 2 0.39 vs 1.44 s, the room 1.26 vs 2.88 s; profiles/r04d_sbvh_alpha.txt) */
	float bvhSpatial = 1e-3f;
	float bvhSpatialBudget = 1.0f;       /* ... adding at most this many references per triangle */
	/* ... in nodes of at least this many references (0: every node): 64 builds config 5's 100 meshes 17-20 % faster
	   (setup 4.55 -> 3.64-3.76 s on one box) for 0.3 % more node steps (config-5 frame +0.4 %; config 2 and 3 within the
	   noise), profiles/r04g_sbvh_build.txt, r04u_config5_setup.jsonl */
	int bvhSpatialMinRefs = 64;
	int bvh4Collapse = 1;                /* BVH4 collapse: 0 greedy (CollapseBvh4), 1 dynamic programming (CollapseBvh4Sah) */
	float chordSplit = 0.35f;            /* extension rays with a chord through the scene box below this x its extent are traced last */
	float sceneLo[3] = { 0, 0, 0 }, sceneHi[3] = { 0, 0, 0 };   /* world box of the instanced meshes (UpdateToplevel) */
	float qBound = 0;                    /* |coordinate| bound of the world box and every mesh box, with slack (SceneDev::qBound) */
	/* the path tail (k_trace_path4d): bounces pathTail .. maxPathLength traced and shaded in one launch,
	   a wave shading its finished queries once pathTailBatch lanes hold one (or none walks); 0: a launch
	   pair per bounce.  Config 3 (profiles/r02zb_ab_path_tail.txt): 2.542 -> 2.389 ms per frame at 3 / 56 */
	int pathTail = 3, pathTailBatch = 56;
	/* shadow overlap: the shadow rays queued before the path tail are traced on a side stream
	   while the path tail runs (latency bound, it leaves much of the chip idle); the final shadow launch
	   traces only the path tail's.  Config 3 2.29 -> 2.235 ms, config-4 rank share at N = 8 1.431 -> 1.363
	   ms with the tail at 2 blocks per CU (profiles/r03g_overlap_sweep.txt); a side launch after every
	   shade launch slows the bounces it overlaps (2.344 / 1.426 ms) */
	bool shadowOverlap = true;
	int pathTailBlocks = 0;              /* the path tail's blocks per CU; 0: with the overlap 3 for frames of at most
	                                        kSmallFramePaths paths, else 2 (without: its occupancy limit) */
	/* the path tail kernel's variant: 0, by frame size (3 waves per SIMD for small frames, 4 for larger ones); 3 or 4 */
	int pathTailWaves = 0;
	/* blocks per CU of the frame's last shadow launch (0: the trace grid's): fewer leave the next frame's primary and early
	   shade launches room beside it: 6 against the trace grid's 8, config 3 and the N = 8 share -0.5 % (profiles/r04aj_ab.txt,
	   r04ak_ab.txt); round 5, with the shorter shade launches, 4 against 6: the N = 8 share -0.9 %, config 3 -0.3 %, 8 slower
	   (r05f_ab_final_shadow_blocks.txt) */
	int finalShadowBlocks = 4;
	int shadeBlocks = 0;                 /* blocks per CU of the frame's shade launches (0: by path count, Render) */
	/* blocks per CU of the side shadow launch beside the path tail (0: the trace grid's; -1: by frame size): 4 leaves the next
	   frame's primary and early shade launches room: config 3 -0.5 %, the N = 8 share -0.8 to -1.5 % (profiles/r04m_ab.txt,
	   r04n_ab.txt); round 6, with the lighter 4-wave path tail, small frames (<= kSmallFramePaths) 3: config 3 -1.2 %, the N = 8
	   share -1.8 %, while the 4K frame stays at 4 (3 there: +2 %, profiles/r06y_ab_side_blocks.txt) */
	int sideBlocks = -1;
	/* heavy-first primary packets (TraceArgs::hvRead): the packets of the previous frame that took more than
	   packetHeavy x its mean node steps are taken first; 0: off; -1 (default, round 6): 3 for frames with a path tail, whose
	   primary launch runs beside the previous frame's tail (config 3 -1.2 %, the 4K frame -0.8 %), 2 otherwise (config 2: 3
	   is 1.5 % slower), profiles/r06zg_ab_overlap_heavy.txt */
	float packetHeavy = -1.0f;
	int traceVersion = 0;                /* 0: auto (TraceVersion) */
	int TraceVersion() const;
	int unitCoherent = 0;
	int packetPrimary = -1;              /* wave-uniform packet traversal for 8x8-tiled primary rays (-1: by scene size) */
	int gpuBuild = 0, gpuTlas = 1;       /* BLAS builder (1: GPU PLOC, 0: CPU binned SAH); TLAS on the GPU */
	int framePathLengths = 0, framePrimeRef = 0;
	double frameHostMs = 0;
	int samplesTaken = 0;
	bool firstConvergingFrame = false;
	uint32_t camRNGseed = 0x12345678;
};

}  // namespace lh2
