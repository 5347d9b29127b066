/* rendercore.cpp - host driver of the MI355X wavefront path tracer.

   Counterpart of RenderCore_OptixPrime_B/rendercore.cpp (method-for-method, same semantics),
   re-designed for MI355X:
     - the acceleration structure is our own binned-SAH BVH2 (bvh_build.cpp) instead of the
       closed OptiX Prime BLAS/TLAS (core_mesh.cpp:53-66, rendercore.cpp:250-270);
     - path / ray / hit buffers are SoA float4 planes (coalesced 16-B lane accesses);
     - per-bounce path counts stay on the device (wave-compacted counters), so a frame is one
       stream of launches with no blocking counter copy per bounce (rendercore.cpp:547);
     - shadow rays never overflow (<= 2 per path with ENOUGH_BOUNCES = S_BOUNCED) and are traced
       once per frame with finalizeConnection fused into the any-hit kernel.
*/
#include "rendercore.h"

#include <hip/hip_gl_interop.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "../../include/lh2_detmath.h"
#include "lh2_device.h"

namespace lh2 {

void FatalError( const char* fmt, ... )
{
	char buf[1024];
	va_list args;
	va_start( args, fmt );
	vsnprintf( buf, sizeof( buf ), fmt, args );
	va_end( args );
	throw std::runtime_error( buf );
}

#define CHK_HIP( stmt ) do { hipError_t e_ = (stmt); if (e_ != hipSuccess) FatalError( "%s failed: %s (%s:%d)", #stmt, hipGetErrorString( e_ ), __FILE__, __LINE__ ); } while (0)

static std::string LibraryDir()
{
	Dl_info info;
	if (dladdr( (void*)&LibraryDir, &info ) && info.dli_fname)
	{
		std::string p( info.dli_fname );
		const size_t s = p.find_last_of( '/' );
		return s == std::string::npos ? std::string( "." ) : p.substr( 0, s );
	}
	return ".";
}

/* mat4::Inverted (RenderSystem/common_types.h:586-628); same formula as the oracle */
static void Mat4Inverse( const float* c, float* out )
{
	const float inv[16] = {
		c[5] * c[10] * c[15] - c[5] * c[11] * c[14] - c[9] * c[6] * c[15] + c[9] * c[7] * c[14] + c[13] * c[6] * c[11] - c[13] * c[7] * c[10],
		-c[1] * c[10] * c[15] + c[1] * c[11] * c[14] + c[9] * c[2] * c[15] - c[9] * c[3] * c[14] - c[13] * c[2] * c[11] + c[13] * c[3] * c[10],
		c[1] * c[6] * c[15] - c[1] * c[7] * c[14] - c[5] * c[2] * c[15] + c[5] * c[3] * c[14] + c[13] * c[2] * c[7] - c[13] * c[3] * c[6],
		-c[1] * c[6] * c[11] + c[1] * c[7] * c[10] + c[5] * c[2] * c[11] - c[5] * c[3] * c[10] - c[9] * c[2] * c[7] + c[9] * c[3] * c[6],
		-c[4] * c[10] * c[15] + c[4] * c[11] * c[14] + c[8] * c[6] * c[15] - c[8] * c[7] * c[14] - c[12] * c[6] * c[11] + c[12] * c[7] * c[10],
		c[0] * c[10] * c[15] - c[0] * c[11] * c[14] - c[8] * c[2] * c[15] + c[8] * c[3] * c[14] + c[12] * c[2] * c[11] - c[12] * c[3] * c[10],
		-c[0] * c[6] * c[15] + c[0] * c[7] * c[14] + c[4] * c[2] * c[15] - c[4] * c[3] * c[14] - c[12] * c[2] * c[7] + c[12] * c[3] * c[6],
		c[0] * c[6] * c[11] - c[0] * c[7] * c[10] - c[4] * c[2] * c[11] + c[4] * c[3] * c[10] + c[8] * c[2] * c[7] - c[8] * c[3] * c[6],
		c[4] * c[9] * c[15] - c[4] * c[11] * c[13] - c[8] * c[5] * c[15] + c[8] * c[7] * c[13] + c[12] * c[5] * c[11] - c[12] * c[7] * c[9],
		-c[0] * c[9] * c[15] + c[0] * c[11] * c[13] + c[8] * c[1] * c[15] - c[8] * c[3] * c[13] - c[12] * c[1] * c[11] + c[12] * c[3] * c[9],
		c[0] * c[5] * c[15] - c[0] * c[7] * c[13] - c[4] * c[1] * c[15] + c[4] * c[3] * c[13] + c[12] * c[1] * c[7] - c[12] * c[3] * c[5],
		-c[0] * c[5] * c[11] + c[0] * c[7] * c[9] + c[4] * c[1] * c[11] - c[4] * c[3] * c[9] - c[8] * c[1] * c[7] + c[8] * c[3] * c[5],
		-c[4] * c[9] * c[14] + c[4] * c[10] * c[13] + c[8] * c[5] * c[14] - c[8] * c[6] * c[13] - c[12] * c[5] * c[10] + c[12] * c[6] * c[9],
		c[0] * c[9] * c[14] - c[0] * c[10] * c[13] - c[8] * c[1] * c[14] + c[8] * c[2] * c[13] + c[12] * c[1] * c[10] - c[12] * c[2] * c[9],
		-c[0] * c[5] * c[14] + c[0] * c[6] * c[13] + c[4] * c[1] * c[14] - c[4] * c[2] * c[13] - c[12] * c[1] * c[6] + c[12] * c[2] * c[5],
		c[0] * c[5] * c[10] - c[0] * c[6] * c[9] - c[4] * c[1] * c[10] + c[4] * c[2] * c[9] + c[8] * c[1] * c[6] - c[8] * c[2] * c[5] };
	const float det = c[0] * inv[0] + c[1] * inv[4] + c[2] * inv[8] + c[3] * inv[12];
	if (det != 0) { const float invdet = 1.0f / det; for (int i = 0; i < 16; i++) out[i] = inv[i] * invdet; }
	else for (int i = 0; i < 16; i++) out[i] = (i % 5 == 0) ? 1.0f : 0.0f;
}

/* ------------------------------------------------------------------------------------------ */
void RenderCore::Init()   /* rendercore.cpp:96-143 */
{
	if (initialized) return;
	CHK_HIP( hipGetDevice( &device ) );
	hipDeviceProp_t props;
	CHK_HIP( hipGetDeviceProperties( &props, device ) );
	smCount = props.multiProcessorCount;
	coreStats.SMcount = (uint32_t)smCount;
	coreStats.ccMajor = (uint32_t)props.major, coreStats.ccMinor = (uint32_t)props.minor;
	coreStats.VRAM = (uint32_t)(props.totalGlobalMem >> 20);
	const char* name = props.gcnArchName[0] ? props.gcnArchName : props.name;
	coreStats.deviceName = new char[strlen( name ) + 1];   /* owned (and leaked) by the core: core_api_base.h:33 */
	memcpy( coreStats.deviceName, name, strlen( name ) + 1 );
	CHK_HIP( hipStreamCreateWithFlags( &stream, hipStreamNonBlocking ) );
	/* blue noise sampler tables (rendercore.cpp:125-134), shipped as data/bluenoise.bin */
	std::string path = getenv( "LH2_BLUENOISE" ) ? getenv( "LH2_BLUENOISE" ) : LibraryDir() + "/data/bluenoise.bin";
	FILE* f = fopen( path.c_str(), "rb" );
	if (!f) FatalError( "blue noise table not found: %s", path.c_str() );
	/* +256 zero bytes: tools_shared.h:343 reads past the table for dimensions > 7 at pixel (127,127)
	   (undefined in the reference; defined as 0 here and in the oracle) */
	std::vector<uint8_t> bn( 65536 * 5 + 256, 0 );
	const size_t got = fread( bn.data(), 1, 65536 * 5, f );
	fclose( f );
	if (got != 65536 * 5) FatalError( "blue noise table truncated: %s", path.c_str() );
	dBlueNoise.upload( bn.data(), bn.size(), stream );
	blocksPerCU = maxBlocksPerCU = std::max( 1, std::min( 8, lh2_trace_blocks_per_cu() ) );
	packetBlocksPerCU = std::max( 1, std::min( 8, lh2_packet_blocks_per_cu() ) );
	pathBlocksPerCU = std::max( 1, std::min( 8, lh2_path_blocks_per_cu() ) );
	anyBlocksPerCU = std::max( 1, std::min( 8, lh2_any4d_blocks_per_cu() ) );
	for (int gi = 0; gi < LH2_MAX_GROUPS; gi++)
	{
		PathGroup& g = grp[gi];
		if (gi == 0) g.st = stream;
		else
		{
			CHK_HIP( hipStreamCreateWithFlags( &g.st, hipStreamNonBlocking ) );
			g.ownStream = true;
		}
		g.counters.resize( 1 );
		g.cursors.resize( (size_t)LH2_CURSOR_SLOTS * LH2_CURSOR_WORDS );
		g.rayLog.resize( LH2_MAX_BOUNCES + 8 );
		g.camAlloc.resize( 2 * LH2_CAM_ALLOC_WORDS );
		CHK_HIP( hipMemsetAsync( g.camAlloc.ptr, 0, sizeof( uint32_t ) * 2 * LH2_CAM_ALLOC_WORDS, stream ) );
		CHK_HIP( hipMemsetAsync( g.rayLog.ptr, 0, sizeof( uint32_t ) * (LH2_MAX_BOUNCES + 8), stream ) );
		/* indexed by pathLength; written by k_counters_next (system scope) */
		CHK_HIP( hipHostMalloc( (void**)&g.activeLog, sizeof( uint32_t ) * (LH2_MAX_BOUNCES + 8), hipHostMallocCoherent ) );
		for (auto& e : g.evTrace) CHK_HIP( hipEventCreate( &e ) );
		for (auto& e : g.evShade) CHK_HIP( hipEventCreate( &e ) );
		for (auto& e : g.evShadowB) CHK_HIP( hipEventCreate( &e ) );
		for (auto& e : g.evCount) CHK_HIP( hipEventCreate( &e ) );   /* stop events of launches (LaunchEvents) */
		CHK_HIP( hipEventCreate( &g.evCamera ) );
		CHK_HIP( hipEventCreate( &g.evShadow ) );
		CHK_HIP( hipEventCreateWithFlags( &g.evDone, hipEventDisableTiming ) );
	}
	CHK_HIP( hipEventCreateWithFlags( &evFork, hipEventDisableTiming ) );
	CHK_HIP( hipStreamCreateWithFlags( &sideStream, hipStreamNonBlocking ) );
	CHK_HIP( hipEventCreate( &evSideStart ) );
	CHK_HIP( hipEventCreate( &evSideStop ) );
	shadowSnap.resize( LH2_SEGS * LH2_SEGCOUNT_STRIDE );
	CHK_HIP( hipHostMalloc( (void**)&hostStats, sizeof( FrameStats ), hipHostMallocCoherent ) );   /* written by k_finalize (system scope) */
	memset( hostStats, 0, sizeof( FrameStats ) );
	for (auto& e : evFrame) CHK_HIP( hipEventCreate( &e ) );
	for (auto& e : evStage) CHK_HIP( hipEventCreateWithFlags( &e, hipEventDisableTiming ) );
	dSceneError.resize( 1 ), dTlasDepth.resize( 1 );
	CHK_HIP( hipMemsetAsync( dSceneError.ptr, 0, sizeof( int ), stream ) );
	CHK_HIP( hipMemsetAsync( dTlasDepth.ptr, 0, sizeof( int ), stream ) );
	dInstDesc.resize( 1 );   /* shading reads record 0 for a miss (HitInstance): it always exists */
	CHK_HIP( hipMemsetAsync( dInstDesc.ptr, 0, sizeof( lh2_CoreInstanceDesc ), stream ) );
	if (const char* tv = getenv( "LH2_TRACE_VERSION" )) traceVersion = std::min( 7, std::max( 0, atoi( tv ) ) );   /* A/B runs */
	CHK_HIP( hipStreamSynchronize( stream ) );
	initialized = true;
}

void RenderCore::SetTarget( uint32_t w, uint32_t h, uint32_t spp )  /* rendercore.cpp:149-209 */
{
	if (spp < 1) spp = 1;
	if ((uint64_t)w * h * spp > (1u << 24)) FatalError( "path index exceeds 24 bits (camera.h:92): %ux%u x %u spp", w, h, spp );
	scrwidth = (int)w, scrheight = (int)h, scrspp = (int)spp;
	EnsureBuffers();
	CHK_HIP( hipMemsetAsync( accumulator.ptr, 0, sizeof( float4 ) * (size_t)w * h, stream ) );
	samplesTaken = 0;
}

/* display output (interoptexture.cpp:25-71): register the app's GL_RGBA32F texture with HIP once per
   SetTarget; Render copies the finalized frame into it.  Needs the app's GL context to be current,
   as the reference's interop does; ID 0 (headless RenderSystem, tests, bench) skips it. */
void RenderCore::SetInteropTexture( uint32_t glTextureId )
{
	if (glTextureId == glTexture && (glResource || !glTextureId)) return;
	if (glResource) { CHK_HIP( hipStreamSynchronize( stream ) ); (void)hipGraphicsUnregisterResource( glResource ); glResource = nullptr; }
	glTexture = glTextureId;
	if (!glTextureId) return;
	const unsigned GL_TEXTURE_2D_ = 0x0DE1;
	CHK_HIP( hipGraphicsGLRegisterImage( &glResource, glTextureId, GL_TEXTURE_2D_, hipGraphicsRegisterFlagsWriteDiscard ) );
}

/* Packets share one node fetch per wave (scalar loads, one path for 64 rays): a win while the BVH
   and triangles stay in L2 / Infinity Cache, a loss when node fetches go to DRAM, where the
   per-ray loop's 64 independent loads per wave hide latency better (config 2: 8.6 MB, packets
   1.6x faster; 1M-tri room 81 MB: 12 % slower; 10M-tri instanced 1 GB: 1.5x slower;
   profiles/r01b_ab_packets.jsonl) */
bool RenderCore::UsePackets() const
{
	if (packetPrimary >= 0) return packetPrimary != 0;
	const double bytes = ((double)blasNodeCount + tlasCapacity) * 64.0 + (double)blasTriCount * 48.0;
	return bytes <= (double)packetMaxMB * 1048576.0;
}

/* traversal loop of the per-ray launches (setting "traceVersion", 0: auto).  Auto: lh2_trace4d.inc (BVH4,
   packed-FMA slabs, LDS child references, rcp box reciprocals, the single instance entered at ray
   set-up).  While the BVH4 + triangles fit the 256 MB Infinity Cache each branch fetches its own record
   and every reached leaf is tested at once (6: config-2 bounce rays 0.86 ms vs 0.88 for the v4 loop,
   config 3 2.68 vs 2.77 ms per frame); beyond it leaves are parked in a one-entry slot and tested in
   batches of leafBatch (default 16) lanes (7: config 5, 1 GB, 12.89 ms per frame vs 13.31 for the one-fetch
   loop 5 and 13.68 for 6; profiles/r02j_ab_versions.txt, r02l_ab_slot.txt) */
int RenderCore::TraceVersion() const
{
	if (traceVersion) return (traceVersion >= 4 && !bvh4) ? 2 : traceVersion;
	if (!bvh4) return 2;
	/* the leaf-slot loop with small leaf batches: config-2 bounce rays 0.64 -> 0.60 ms, config 5 (DRAM-resident)
	   13.25 -> 13.1 ms, config 3 unchanged (profiles/r02y_ab_v7.txt); traceFetchMB no longer decides */
	return 7;
}

void RenderCore::EnsureBuffers()
{
	accumulator.resize( (size_t)scrwidth * scrheight );
	frame.resize( (size_t)scrwidth * scrheight );
}

/* path buffers of a group for `paths` paths (a bit extra, as the reference reserves, and room for
   LH2_SEGS segments of ceil(paths / LH2_SEGS)); shadow rays: 2 per path */
void RenderCore::EnsureGroup( PathGroup& g, uint32_t paths )
{
	if ((size_t)paths + 64 > g.cap)
	{
		g.cap = (size_t)paths + (paths >> 4) + 64;
		for (int i = 0; i < 2; i++) g.rayO[i].resize( g.cap ), g.rayD[i].resize( g.cap ), g.T4[i].resize( g.cap ), g.Q4[i].resize( g.cap );
		g.hits.resize( g.cap );
		g.shO.resize( 2 * g.cap ), g.shD.resize( 2 * g.cap ), g.shP.resize( 2 * g.cap );
		g.shMask.resize( (2 * g.cap + 63) / 32 + 2 );
	}
	EnsureStack( g );
}

void RenderCore::EnsureStack( PathGroup& g )
{
	const size_t need = (size_t)(LH2_STACK_TOTAL - std::min( LH2_STACK_LDS, LH2_STACK4_LDS )) * std::max( TraceGrid(), ShadowGrid() ) * 256;
	if (g.gstack.count < need) g.gstack.resize( need );
	if (&g == &grp[0] && sideStack.count < need) sideStack.resize( need );
}

void RenderCore::Setting( const char* name, float value )  /* rendercore.cpp:439-457 */
{
	if (!strcmp( name, "epsilon" )) geometryEpsilon = value;
	else if (!strcmp( name, "clampValue" )) clampValue = value;
	else if (!strcmp( name, "maxPathLength" )) maxPathLength = std::min( 16, std::max( 1, (int)value ) );
	/* PrimeRef validation mode: the RenderCore_PrimeRef path tracer (uniform random numbers, Lambert
	   BSDF, NEE without MIS, Russian roulette, MAXPATHLENGTH 64) on the same scene data */
	else if (!strcmp( name, "primeRef" )) primeRef = value != 0;
	else if (!strcmp( name, "tiledRays" )) tiledRays = value != 0;
	/* dynamic ray fetch: refill a wave's idle lanes once this many are idle (64 = whole batches);
	   coherent 8x8-tiled primary rays trace best in batches, incoherent bounce rays with refills */
	else if (!strcmp( name, "refillPrimary" )) refillPrimary = std::min( 64, std::max( 1, (int)value ) );
	else if (!strcmp( name, "refill" )) refillOther = std::min( 64, std::max( 1, (int)value ) );
	/* traversal: test parked BLAS leaves once this many lanes of a wave hold one (0 = every step) */
	else if (!strcmp( name, "leafBatch" )) leafBatch = std::min( 64, std::max( 0, (int)value ) );
	else if (!strcmp( name, "leafBatchPrimary" )) leafBatchPrimary = std::min( 64, std::max( 0, (int)value ) );
	/* the shadow launches' own loop (5, 6, 7 over the BVH4; 0: traceVersion), leaf batch (-1: leafBatch) and refill (0: refill) */
	else if (!strcmp( name, "shadowVersion" )) shadowVersion = (int)value >= 5 && (int)value <= 7 ? (int)value : 0;
	else if (!strcmp( name, "leafBatchShadow" )) leafBatchShadow = std::min( 64, std::max( -1, (int)value ) );
	else if (!strcmp( name, "refillShadow" )) refillShadow = std::min( 64, std::max( 0, (int)value ) );
	else if (!strcmp( name, "sampleInterleave" )) sampleInterleave = value != 0;   /* the samples of an 8x8 block in consecutive waves */
	else if (!strcmp( name, "shadowGridOwn" )) { shadowGridOwn = value != 0; if (scrwidth) EnsureBuffers(); }   /* final shadow launch at the any-hit kernels' occupancy */
	else if (!strcmp( name, "shadowBackfill" )) shadowBackfill = value != 0;   /* shadow rays in the closest-hit launches' tails */
	/* BLAS build parameters, used by later SetGeometry calls */
	else if (!strcmp( name, "bvhMaxLeaf" )) bvhMaxLeaf = std::min( 16, std::max( 1, (int)value ) );
	else if (!strcmp( name, "bvhTraversalCost" )) bvhTraversalCost = std::max( 0.01f, value );
	else if (!strcmp( name, "bvhSweep" )) bvhSweep = std::max( 0, (int)value );   /* exact SAH sweep for nodes of <= this many triangles */
	else if (!strcmp( name, "bvhSpatial" )) bvhSpatial = std::max( 0.0f, value );   /* SBVH overlap threshold (x root area); 0: off */
	else if (!strcmp( name, "bvhSpatialBudget" )) bvhSpatialBudget = std::min( 4.0f, std::max( 0.0f, value ) );
	else if (!strcmp( name, "bvh4Collapse" )) bvh4Collapse = value != 0;
	else if (!strcmp( name, "chordSplit" )) chordSplit = std::max( 0.0f, value );   /* two-ended path segments (longest first); 0: off */
	else if (!strcmp( name, "chordSplitShadow" )) chordSplitShadow = std::max( 0.0f, value );   /* two-ended shadow segments; 0: off */
	else if (!strcmp( name, "packetHeavy" )) packetHeavy = std::max( 0.0f, value );   /* heavy-first primary packets; 0: off */
	else if (!strcmp( name, "terminalTrace" )) terminalTrace = value != 0;   /* the last terminal bounce's sky samples in its trace launch */
	else if (!strcmp( name, "pathTail" )) pathTail = std::max( 0, (int)value );   /* bounces from this one in one trace-and-shade launch; 0: off */
	else if (!strcmp( name, "pathTailBatch" )) pathTailBatch = std::min( 64, std::max( 1, (int)value ) );
	else if (!strcmp( name, "chordSplitPrimary" )) chordSplitPrimary = std::min( 1.0f, std::max( 0.0f, value ) );   /* two-ended primary segments; 0: off */
	else if (!strcmp( name, "bvh4LeafTris" )) bvh4LeafTris = std::min( 16, std::max( 1, (int)value ) );
	else if (!strcmp( name, "bvh4LeafCost" )) bvh4LeafCost = std::max( 0.0f, value );
	else if (!strcmp( name, "bvh4TriCost" )) bvh4TriCost = std::max( 0.0f, value );
	/* packet traversal of tiled primary rays: 1 on, 0 off, -1 when the BVH + triangles fit in packetMaxMB */
	else if (!strcmp( name, "packetPrimary" )) packetPrimary = value < 0 ? -1 : value != 0;
	else if (!strcmp( name, "packetMaxMB" )) packetMaxMB = std::max( 0.0f, value );
	else if (!strcmp( name, "packetWidth" )) packetWidth = value >= 4 ? 4 : 2;   /* packets over the BVH2 / BVH4 */
	else if (!strcmp( name, "shadowSplit" )) shadowSplit = std::min( LH2_MAX_BOUNCES, std::max( 0, (int)value ) );   /* early shadow launch after this bounce (0: off) */
	else if (!strcmp( name, "pathGroups" )) pathGroups = std::min( LH2_MAX_GROUPS, std::max( 1, (int)value ) );   /* pipelined path groups per frame */
	else if (!strcmp( name, "singleInstanceStart" )) singleInstanceStart = value != 0;   /* one instance: rays start at its TLAS leaf */
	else if (!strcmp( name, "terminalShade" )) terminalShade = value != 0;   /* drop hits that cannot contribute before shading them (ShadeParams::terminal) */
	else if (!strcmp( name, "tailPool" )) tailPool = std::min( 64, std::max( 0, (int)value ) );   /* hand a dry wave's rays to another wave of its workgroup (0: off) */
	else if (!strcmp( name, "tailLanes" )) tailLanes = std::min( 64, std::max( 0, (int)value ) );   /* traversal tail hand-off (0: off) */
	else if (!strcmp( name, "traceBlocksPerCU" ))   /* persistent trace grid: blocks per CU (default: occupancy limit) */
	{
		blocksPerCU = value > 0 ? std::min( maxBlocksPerCU, std::max( 1, (int)value ) ) : maxBlocksPerCU;
	}
	else if (!strcmp( name, "packetShadow" )) packetShadow = value != 0;     /* packet traversal of the shadow rays */
	else if (!strcmp( name, "unitCoherent" )) unitCoherent = value != 0;   /* TraceClosestDevice uses the primary-ray launch */
	else if (!strcmp( name, "traceVersion" )) traceVersion = std::min( 7, std::max( 0, (int)value ) );   /* traversal loop: 1, 2 (BVH2), 4 (BVH4), 5 / 6 (BVH4, lh2_trace4d.inc: one fetch per iteration / per branch), 0 auto */
	else if (!strcmp( name, "traceFetchMB" )) traceFetchMB = std::max( 0.0f, value );
	else if (!strcmp( name, "bvh4" )) { bvh4 = value != 0; if (!bvh4 && traceVersion >= 4) traceVersion = 2; }   /* before SetGeometry */
	else if (!strcmp( name, "gpuBuild" )) gpuBuild = value != 0;          /* BLAS builder of later SetGeometry calls */
	else if (!strcmp( name, "gpuTlas" )) { gpuTlas = value != 0; instancesDirty = true; }
	else if (!strcmp( name, "plocRadius" )) gpuBvh.radius = std::min( 32, std::max( 1, (int)value ) );
	else if (!strcmp( name, "blocksPerCU" )) { blocksPerCU = std::min( 16, std::max( 1, (int)value ) ); if (scrwidth) EnsureBuffers(); }
	/* other names ("clampDirect", "filter", "TAA", ...) are ignored, as in the reference */
}

/* the current value of a setting (extension: the reference has no getter); false for unknown names */
bool RenderCore::GetSetting( const char* name, float& value ) const
{
	struct { const char* n; float v; } t[] = {
		{ "epsilon", geometryEpsilon }, { "clampValue", clampValue }, { "maxPathLength", (float)maxPathLength },
		{ "primeRef", (float)primeRef }, { "tiledRays", (float)tiledRays }, { "refillPrimary", (float)refillPrimary },
		{ "refill", (float)refillOther }, { "leafBatch", (float)leafBatch }, { "leafBatchPrimary", (float)leafBatchPrimary },
		{ "shadowVersion", (float)ShadowVersion() }, { "leafBatchShadow", (float)ShadowLeafBatch() }, { "refillShadow", (float)ShadowRefill() }, { "shadowBackfill", (float)shadowBackfill }, { "sampleInterleave", (float)sampleInterleave }, { "shadowGridOwn", (float)shadowGridOwn },
		{ "bvhMaxLeaf", (float)bvhMaxLeaf }, { "bvhSweep", (float)bvhSweep }, { "bvhSpatial", bvhSpatial }, { "bvhSpatialBudget", bvhSpatialBudget }, { "bvh4Collapse", (float)bvh4Collapse },
		{ "bvh4LeafTris", (float)bvh4LeafTris }, { "chordSplit", chordSplit }, { "chordSplitPrimary", chordSplitPrimary }, { "pathTail", (float)pathTail }, { "terminalTrace", (float)terminalTrace }, { "packetHeavy", packetHeavy }, { "chordSplitShadow", chordSplitShadow }, { "pathTailBatch", (float)pathTailBatch }, { "bvh4LeafCost", bvh4LeafCost }, { "bvh4TriCost", bvh4TriCost }, { "packetPrimary", (float)packetPrimary }, { "packetWidth", (float)packetWidth },
		{ "pathGroups", (float)pathGroups }, { "shadowSplit", (float)shadowSplit }, { "singleInstanceStart", (float)singleInstanceStart },
		{ "terminalShade", (float)terminalShade }, { "traceVersion", (float)TraceVersion() }, { "traceFetchMB", traceFetchMB }, { "bvh4", (float)bvh4 },
		{ "gpuBuild", (float)gpuBuild }, { "gpuTlas", (float)gpuTlas }, { "blocksPerCU", (float)blocksPerCU },
		{ "packetShadow", (float)packetShadow }, { "usePackets", (float)UsePackets() } };
	for (const auto& e : t) if (!strcmp( name, e.n )) { value = e.v; return true; }
	return false;
}

void RenderCore::SetTextures( const lh2_CoreTexDesc* tex, int textureCount )   /* rendercore.cpp:276-292 */
{
	texDescs.assign( tex, tex + std::max( 0, textureCount ) );
	/* SyncStorageType (rendercore.cpp:299-336) for ARGB32, ARGB128 and NRM32: one continuous array per
	   storage type, textures in descriptor order, at least 16 texels.  ARGB128 texels are copied whole
	   (the reference copies pixelCount * 4 bytes of each 16-byte texel there; this core never reads
	   ARGB128 texels while shading, so only CoreStats sees the difference). */
	for (int storage = 0; storage < 3; storage++)
	{
		uint32_t total = 0;
		for (auto& t : texDescs) if (t.storage == storage) total += t.pixelCount;
		const uint32_t alloc = std::max( 16u, total );
		if (storage == 1)
		{
			std::vector<float4> buf( alloc, make_float4( 0, 0, 0, 0 ) );
			uint32_t at = 0;
			for (auto& t : texDescs) if (t.storage == storage) { memcpy( buf.data() + at, t.idata, (size_t)t.pixelCount * 16 ); t.firstPixel = at; at += t.pixelCount; }
			dArgb128.upload( buf.data(), buf.size(), stream );
			coreStats.argb128TexelCount = alloc;
		}
		else
		{
			std::vector<uint32_t> buf( alloc, 0u );
			uint32_t at = 0;
			for (auto& t : texDescs) if (t.storage == storage) { memcpy( buf.data() + at, t.idata, (size_t)t.pixelCount * 4 ); t.firstPixel = at; at += t.pixelCount; }
			(storage == 0 ? dArgb32 : dNrm32).upload( buf.data(), buf.size(), stream );
			(storage == 0 ? coreStats.argb32TexelCount : coreStats.nrm32TexelCount) = alloc;
		}
	}
	CHK_HIP( hipStreamSynchronize( stream ) );   /* texel pointers are borrowed for this call only */
}

#define TOCHAR(a) lh2_f2u( (a) * 255.0f )
#define TOUINT4(a,b,c,d) (TOCHAR(a)+(TOCHAR(b)<<8)+(TOCHAR(c)<<16)+(TOCHAR(d)<<24))
void RenderCore::SetMaterials( const lh2_CoreMaterial* mat, int n )   /* rendercore.cpp:353-399 */
{
	std::vector<uint4> recs( (size_t)std::max( n, 1 ) * 8 );
	memset( recs.data(), 0, recs.size() * sizeof( uint4 ) );
	diffuseOnly = true, canEmit = false;
	for (int i = 0; i < n; i++)
	{
		const lh2_CoreMaterial& m = mat[i];
		/* IsEmissive (colour > 1 after the fp16 round, which keeps x <= 1 at or below 1; NaN counts as
		   emissive here), colour and detail maps (texels can exceed 1) and alpha cut-outs */
		if (!(m.color.value.x <= 1.0f && m.color.value.y <= 1.0f && m.color.value.z <= 1.0f) || m.color.textureID != -1 ||
			m.detailColor.textureID != -1 || (m.flags & 2))
			canEmit = true;
		/* a path can only continue past its second vertex through a specular event (ROUGHNESS <= 0.001,
		   a transmission sample) or an alpha cut-out (ENOUGH_BOUNCES = S_BOUNCED, pathtracer.h:33,211) */
		if (TOCHAR( m.roughness.value ) == 0 || TOCHAR( m.transmission.value ) != 0 || (m.flags & 2) || m.roughness.textureID != -1)
			diffuseOnly = false;
		const uint32_t r = lh2_f2h( m.color.value.x ), g = lh2_f2h( m.color.value.y ), b = lh2_f2h( m.color.value.z );
		const uint32_t tr = lh2_f2h( 1 - m.absorption.value.x ), tg = lh2_f2h( 1 - m.absorption.value.y ), tb = lh2_f2h( 1 - m.absorption.value.z );
		const uint32_t flags = (m.eta.value < 1 ? 1u : 0u) + ((m.flags & 1) ? (1u << 11) : 0u) + ((m.flags & 2) ? (1u << 12) : 0u);
		recs[i * 8 + 0] = make_uint4( r | (g << 16), b | (tr << 16), tg | (tb << 16), flags );
		recs[i * 8 + 1] = make_uint4( TOUINT4( m.metallic.value, m.subsurface.value, m.specular.value, m.roughness.value ),
			TOUINT4( m.specularTint.value, m.anisotropic.value, m.sheen.value, m.sheenTint.value ),
			TOUINT4( m.clearcoat.value, m.clearcoatGloss.value, m.transmission.value, 0 ), lh2_f2b( m.eta.value ) );
		/* texture / normal map records (rendercore.cpp:379-384, RenderCore::Map rendercore.h:79-86):
		   x = width | height << 16 (shorts), y / z = uvscale / uvoffset (halves), w = first texel */
		auto map = [&]( int tid, lh2_float2 uvscale, lh2_float2 uvoffs ) {
			if (tid < 0 || tid >= (int)texDescs.size()) FatalError( "SetMaterials: material %d uses texture %d of %d (call SetTextures first)", i, tid, (int)texDescs.size() );
			const lh2_CoreTexDesc& t = texDescs[tid];
			return make_uint4( (t.width & 0xffffu) | ((t.height & 0xffffu) << 16), lh2_f2h( uvscale.x ) | ((uint32_t)lh2_f2h( uvscale.y ) << 16),
				lh2_f2h( uvoffs.x ) | ((uint32_t)lh2_f2h( uvoffs.y ) << 16), t.firstPixel );
		};
		uint32_t texFlags = 0;
		if (m.color.textureID != -1) recs[i * 8 + 2] = map( m.color.textureID, m.color.uvscale, m.color.uvoffset ), texFlags |= 1u << 2;
		if (m.detailColor.textureID != -1) recs[i * 8 + 3] = map( m.detailColor.textureID, m.detailColor.uvscale, m.detailColor.uvoffset ), texFlags |= 1u << 9;
		if (m.normals.textureID != -1) recs[i * 8 + 4] = map( m.normals.textureID, m.normals.uvscale, m.normals.uvoffset ), texFlags |= 1u << 3;
		if (m.detailNormals.textureID != -1) recs[i * 8 + 5] = map( m.detailNormals.textureID, m.detailNormals.uvscale, m.detailNormals.uvoffset ), texFlags |= 1u << 7;
		if (m.specular.textureID != -1) recs[i * 8 + 6] = map( m.specular.textureID, m.specular.uvscale, m.specular.uvoffset ), texFlags |= 1u << 4;
		if (m.roughness.textureID != -1) recs[i * 8 + 7] = map( m.roughness.textureID, m.roughness.uvscale, m.roughness.uvoffset ), texFlags |= 1u << 5;
		/* DIFFUSEMAPISHDR: the reference tests textureID != 1 and so reads texDescs[-1] for untextured
		   materials (rendercore.cpp:386); here only a valid diffuse map can set it.  Not read by shading. */
		if (m.color.textureID >= 0 && (texDescs[m.color.textureID].flags & 8)) texFlags |= 1u << 1;
		recs[i * 8 + 0].w |= texFlags;
	}
	dMaterials.upload( recs.data(), recs.size(), stream );
	CHK_HIP( hipStreamSynchronize( stream ) );
}

void RenderCore::SetLights( const lh2_CoreLightTri* a, int na, const lh2_CorePointLight* p, int np, const lh2_CoreSpotLight* s, int ns,
	const lh2_CoreDirectionalLight* d, int nd )   /* rendercore.cpp:405-419 */
{
	dArea.upload( a, na, stream ), dPoint.upload( p, np, stream ), dSpot.upload( s, ns, stream ), dDir.upload( d, nd, stream );
	dArea.resize( 1 ), dPoint.resize( 1 ), dSpot.resize( 1 ), dDir.resize( 1 );
	nArea = na, nPoint = np, nSpot = ns, nDir = nd;
	CHK_HIP( hipStreamSynchronize( stream ) );
}

void RenderCore::SetSkyData( const float* pixels, uint32_t width, uint32_t height )   /* rendercore.cpp:425-433 */
{
	dSky.upload( pixels, (size_t)width * height * 3, stream );
	dSky.resize( 1 );
	skyW = (int)width, skyH = (int)height;
	CHK_HIP( hipStreamSynchronize( stream ) );
}

void RenderCore::SetGeometry( int meshIdx, const float*, int, int triangleCount, const lh2_CoreTri* tris, const uint32_t* )
{
	/* rendercore.cpp:215-223 + core_mesh.cpp:36-67: meshes arrive first-time in sequential order */
	if (meshIdx < 0 || meshIdx > (int)meshes.size()) FatalError( "SetGeometry: mesh index %d out of sequence", meshIdx );
	if (meshIdx == (int)meshes.size()) meshes.push_back( new CoreMeshHost() );
	CoreMeshHost& m = *meshes[meshIdx];
	const auto t0 = std::chrono::high_resolution_clock::now();
	m.triCount = triangleCount;
	m.shadeTris.upload( (const float4*)tris, (size_t)triangleCount * 11, stream );
	m.shadeTris.resize( 11 );
	bool cpuBuild = !(gpuBuild && triangleCount >= 2);
	if (!cpuBuild)
	{
		/* GPU PLOC build straight from the uploaded CoreTri records (bvh_gpu.h) */
		float4 *nodes = nullptr, *tris48 = nullptr;
		GpuBuildResult r;
		gpuBvh.BuildBlas( m.shadeTris.ptr, triangleCount, bvhMaxLeaf, bvhTraversalCost, &nodes, &tris48, r, stream );
		m.bvhNodes.adopt( nodes, (size_t)r.nodeCount * 4 );
		m.bvhTris.adopt( tris48, (size_t)triangleCount * 3 );
		m.leafTris = triangleCount;
		m.nodeCount = r.nodeCount, m.maxDepth = r.maxDepth;
		for (int k = 0; k < 3; k++) m.aabbLo[k] = r.lo[k], m.aabbHi[k] = r.hi[k];
		/* pathological inputs (e.g. long runs of nearly coincident triangles) can make a clustered tree
		   deep; the top-down SAH build bounds the depth by splitting such ranges in the middle */
		if (r.maxDepth > LH2_STACK_TOTAL / 2) cpuBuild = true;
	}
	if (cpuBuild)
	{
		/* CPU binned-SAH build (bvh_build.cpp) */
		std::vector<Aabb> prims( triangleCount );
		for (int k = 0; k < 3; k++) m.aabbLo[k] = 1e30f, m.aabbHi[k] = -1e30f;
		for (int i = 0; i < triangleCount; i++)
		{
			const lh2_CoreTri& t = tris[i];
			const float v[3][3] = { { t.vertex0.x, t.vertex0.y, t.vertex0.z }, { t.vertex1.x, t.vertex1.y, t.vertex1.z }, { t.vertex2.x, t.vertex2.y, t.vertex2.z } };
			for (int k = 0; k < 3; k++)
			{
				prims[i].lo[k] = std::min( std::min( v[0][k], v[1][k] ), v[2][k] );
				prims[i].hi[k] = std::max( std::max( v[0][k], v[1][k] ), v[2][k] );
				m.aabbLo[k] = std::min( m.aabbLo[k], prims[i].lo[k] ), m.aabbHi[k] = std::max( m.aabbHi[k], prims[i].hi[k] );
			}
		}
		/* spatial splits (bvhSpatial > 0) clip triangles: the builder gets their vertices */
		std::vector<float> verts;
		if (bvhSpatial > 0)
		{
			verts.resize( (size_t)triangleCount * 9 );
			for (int i = 0; i < triangleCount; i++)
			{
				const lh2_CoreTri& t = tris[i];
				const float v[9] = { t.vertex0.x, t.vertex0.y, t.vertex0.z, t.vertex1.x, t.vertex1.y, t.vertex1.z, t.vertex2.x, t.vertex2.y, t.vertex2.z };
				memcpy( &verts[(size_t)i * 9], v, sizeof( v ) );
			}
		}
		BvhOutput bvh;
		BuildBvh2( prims, bvhMaxLeaf, 0, bvh, bvhTraversalCost, bvhSweep, verts.empty() ? nullptr : verts.data(), bvhSpatial, bvhSpatialBudget );
		/* one triangle record per leaf slot (a spatial split can reference a triangle from several leaves) */
		std::vector<float> tris48( std::max<size_t>( bvh.perm.size(), 1 ) * 12, 0.0f );
		for (size_t j = 0; j < bvh.perm.size(); j++)
		{
			const uint32_t ti = bvh.perm[j];
			const lh2_CoreTri& t = tris[ti];
			float* o = &tris48[j * 12];
			/* v0, e1 = v1 - v0, e2 = v2 - v0 in fp32, exactly as the oracle's intersect_tri */
			o[0] = t.vertex0.x, o[1] = t.vertex0.y, o[2] = t.vertex0.z; memcpy( &o[3], &ti, 4 );
			o[4] = t.vertex1.x - t.vertex0.x, o[5] = t.vertex1.y - t.vertex0.y, o[6] = t.vertex1.z - t.vertex0.z, o[7] = 0;
			o[8] = t.vertex2.x - t.vertex0.x, o[9] = t.vertex2.y - t.vertex0.y, o[10] = t.vertex2.z - t.vertex0.z, o[11] = 0;
		}
		m.bvhNodes.upload( (const float4*)bvh.nodes.data(), bvh.nodes.size() / 4, stream );
		m.bvhTris.upload( (const float4*)tris48.data(), tris48.size() / 4, stream );
		m.leafTris = (int)bvh.perm.size();
		m.nodeCount = (int)(bvh.nodes.size() / 16), m.maxDepth = bvh.maxDepth;
		if (bvh4) BuildBlas4( m, bvh.nodes.data() );
	}
	else if (bvh4)
	{
		/* GPU-built BLAS: collapse on the host (one download of the BVH2) */
		std::vector<float> n2( (size_t)m.nodeCount * 16 );
		CHK_HIP( hipMemcpyAsync( n2.data(), m.bvhNodes.ptr, n2.size() * sizeof( float ), hipMemcpyDeviceToHost, stream ) );
		CHK_HIP( hipStreamSynchronize( stream ) );
		BuildBlas4( m, n2.data() );
	}
	CHK_HIP( hipStreamSynchronize( stream ) );   /* the caller's triangle array is borrowed for this call only */
	geometryDirty = true;
	coreStats.bvhBuildTime += std::chrono::duration<float>( std::chrono::high_resolution_clock::now() - t0 ).count();
}

void RenderCore::SetTail( TraceArgs& ta, PathGroup& g )
{
	ta.pool = ta.packet ? 0u : (uint32_t)tailPool;
#ifndef LH2_TAIL_HANDOFF
	(void)ta, (void)g;
	return;   /* the traversal loop is compiled without the hand-off (lh2_trace2.inc) */
#endif
	if (!tailLanes || ta.packet) return;
	const size_t threads = (size_t)TraceGrid() * 256;
	if (g.tailRec.count < threads) g.tailRec.resize( threads ), g.tailUV.resize( threads );
	ta.tailOut = g.tailRec.ptr, ta.tailOutUV = g.tailUV.ptr;
	ta.tailCounts = ta.cursor + LH2_TAIL_COUNT;
	ta.tailStride = (uint32_t)(((TraceGrid() + LH2_SEGS - 1) / LH2_SEGS) * 256);   /* one record per thread of the segment's blocks */
	ta.tailLanes = (uint32_t)tailLanes;
}

void RenderCore::BuildBlas4( CoreMeshHost& m, const float* nodes2 )
{
	std::vector<float> n4;
	/* bvh4Collapse 1: dynamic-programming collapse (surface-area costs, optional leaf merging); 0: greedy */
	m.depth4 = bvh4Collapse ? CollapseBvh4Sah( nodes2, (size_t)m.nodeCount, n4, bvh4LeafCost, bvh4TriCost, bvh4LeafTris )
		: CollapseBvh4( nodes2, (size_t)m.nodeCount, n4 );
	m.bvh4Nodes.upload( (const float4*)n4.data(), n4.size() / 4, stream );
	m.node4Count = (int)(n4.size() / 32);
}

void RenderCore::SetInstance( int instanceIdx, int meshIdx, const float* M )   /* rendercore.cpp:229-243 */
{
	if (meshIdx == -1) { if ((int)instances.size() > instanceIdx) instances.resize( instanceIdx ); instancesDirty = true; return; }
	if (meshIdx < 0 || meshIdx >= (int)meshes.size()) FatalError( "SetInstance: unknown mesh %d", meshIdx );
	if (instanceIdx >= (int)instances.size()) instances.resize( instanceIdx + 1 );
	instances[instanceIdx].mesh = meshIdx;
	memcpy( instances[instanceIdx].T, M, 64 );
	instancesDirty = true;
}

/* scene node array = all BLAS (relocated, device to device) followed by room for the TLAS */
void RenderCore::ConcatenateBlas( int ni )
{
	meshNodeBase.assign( meshes.size(), 0 ), meshTriBase.assign( meshes.size(), 0 ), meshNode4Base.assign( meshes.size(), 0 );
	int nodeTotal = 0, triTotal = 0, node4Total = 0, meshTris = 0;
	maxBlasDepth = 0, maxBlas4Depth = 0;
	std::vector<float> bounds( std::max<size_t>( meshes.size(), 1 ) * 6, 0.0f );
	for (size_t mi = 0; mi < meshes.size(); mi++)
	{
		const CoreMeshHost& m = *meshes[mi];
		meshNodeBase[mi] = nodeTotal, meshTriBase[mi] = triTotal, meshNode4Base[mi] = node4Total;
		nodeTotal += m.nodeCount, triTotal += m.leafTris, node4Total += m.node4Count, meshTris += m.triCount;
		maxBlasDepth = std::max( maxBlasDepth, m.maxDepth ), maxBlas4Depth = std::max( maxBlas4Depth, m.depth4 );
		for (int k = 0; k < 3; k++) bounds[mi * 6 + k] = m.aabbLo[k], bounds[mi * 6 + 3 + k] = m.aabbHi[k];
		if (m.triCount == 0) bounds[mi * 6] = 1.0f, bounds[mi * 6 + 3] = 0.0f;   /* empty-mesh marker */
	}
	tlasCapacity = std::max( 64, 2 * ni + 16 );
	CHK_HIP( hipStreamSynchronize( stream ) );   /* frames in flight may still read the old arrays */
	dNodes.free(), dTris.free(), dNodes4.free();
	dNodes.resize( ((size_t)nodeTotal + tlasCapacity) * 4 );
	/* the BVH4 loops address nodes with 32-bit buffer offsets (lh2_trace4d.inc): the array stays below 2 GiB */
	if (bvh4 && ((size_t)node4Total + tlasCapacity) * 128 > 0x7fffffffull)
		FatalError( "BVH4 of %zu nodes exceeds the 2 GiB the traversal addresses", (size_t)node4Total + tlasCapacity );
	if (bvh4) dNodes4.resize( ((size_t)node4Total + tlasCapacity) * 8 );
	dTris.resize( (size_t)std::max( triTotal, 1 ) * 3 );
	for (size_t mi = 0; mi < meshes.size(); mi++)
	{
		const CoreMeshHost& m = *meshes[mi];
		GpuBvhBuilder::Relocate( m.bvhNodes.ptr, m.nodeCount, meshNodeBase[mi], (uint32_t)meshTriBase[mi], dNodes.ptr, stream );
		if (bvh4) GpuBvhBuilder::Relocate4( m.bvh4Nodes.ptr, m.node4Count, meshNode4Base[mi], (uint32_t)meshTriBase[mi], dNodes4.ptr, stream );
		if (m.leafTris) CHK_HIP( hipMemcpyAsync( dTris.ptr + (size_t)meshTriBase[mi] * 3, m.bvhTris.ptr, sizeof( float4 ) * 3 * (size_t)m.leafTris, hipMemcpyDeviceToDevice, stream ) );
	}
	dMeshBounds.upload( bounds.data(), bounds.size(), stream );
	CHK_HIP( hipStreamSynchronize( stream ) );
	blasNodeCount = nodeTotal, blasTriCount = triTotal, blasNode4Count = node4Total, blasMeshTris = meshTris;
	geometryDirty = false;
}

void RenderCore::UpdateToplevel()   /* rendercore.cpp:250-270 (TLAS) + :481-505 (instance descriptors) */
{
	const int ni = (int)instances.size();
	if (geometryDirty || ni + 1 > tlasCapacity) ConcatenateBlas( ni );
	tlasRoot = blasNodeCount;
	/* host part: inverse transforms and instance records, written to pinned staging (double-buffered)
	   and copied asynchronously; no host-device round trip per frame */
	const int slot = stageSlot;
	stageSlot ^= 1;
	const size_t nRec = (size_t)std::max( ni, 1 );
	const size_t offInst = 0, offDesc = offInst + nRec * sizeof( DevInstance ), offT = offDesc + nRec * sizeof( lh2_CoreInstanceDesc );
	const size_t offMesh = offT + nRec * 64, offNodes = offMesh + nRec * 4, need = offNodes + 4 * 64 * nRec + 64;
	CHK_HIP( hipEventSynchronize( evStage[slot] ) );   /* the copies from this slot two updates ago are done */
	if (need > stageBytes[slot])
	{
		if (stage[slot]) CHK_HIP( hipHostFree( stage[slot] ) );
		stageBytes[slot] = need + need / 2;
		CHK_HIP( hipHostMalloc( (void**)&stage[slot], stageBytes[slot], hipHostMallocDefault ) );
	}
	uint8_t* sb = stage[slot];
	DevInstance* di = (DevInstance*)(sb + offInst);
	lh2_CoreInstanceDesc* desc = (lh2_CoreInstanceDesc*)(sb + offDesc);
	float* Ts = (float*)(sb + offT);
	int* meshIds = (int*)(sb + offMesh);
	memset( sb, 0, offMesh + nRec * 4 );
	for (int i = 0; i < ni; i++)
	{
		CoreInstanceHost& in = instances[i];
		Mat4Inverse( in.T, in.inv );
		di[i].inv0 = make_float4( in.inv[0], in.inv[1], in.inv[2], in.inv[3] );
		di[i].inv1 = make_float4( in.inv[4], in.inv[5], in.inv[6], in.inv[7] );
		di[i].inv2 = make_float4( in.inv[8], in.inv[9], in.inv[10], in.inv[11] );
		di[i].root = meshNodeBase[in.mesh], di[i].triBase = meshTriBase[in.mesh], di[i].mesh = in.mesh;
		di[i].root4 = bvh4 ? meshNode4Base[in.mesh] : 0;
		desc[i].triangles = meshes[in.mesh]->shadeTris.ptr;
		desc[i].A = { in.inv[0], in.inv[1], in.inv[2], in.inv[3] };
		desc[i].B = { in.inv[4], in.inv[5], in.inv[6], in.inv[7] };
		desc[i].C = { in.inv[8], in.inv[9], in.inv[10], in.inv[11] };
		desc[i].D = { in.inv[12], in.inv[13], in.inv[14], in.inv[15] };
		memcpy( Ts + (size_t)i * 16, in.T, 64 );
		meshIds[i] = in.mesh;
	}
	/* the scene's world box (instance transforms of the mesh boxes): the shade launches order extension
	   rays by their chord through it (ShadeParams::chordCut) */
	for (int k = 0; k < 3; k++) sceneLo[k] = 1e30f, sceneHi[k] = -1e30f;
	for (int i = 0; i < ni; i++)
	{
		const CoreInstanceHost& in = instances[i];
		const CoreMeshHost& m = *meshes[in.mesh];
		if (m.triCount == 0) continue;
		for (int c = 0; c < 8; c++)
		{
			const float x = c & 1 ? m.aabbHi[0] : m.aabbLo[0], y = c & 2 ? m.aabbHi[1] : m.aabbLo[1], z = c & 4 ? m.aabbHi[2] : m.aabbLo[2];
			for (int k = 0; k < 3; k++)
			{
				const float w = in.T[k * 4 + 0] * x + in.T[k * 4 + 1] * y + in.T[k * 4 + 2] * z + in.T[k * 4 + 3];
				sceneLo[k] = std::min( sceneLo[k], w ), sceneHi[k] = std::max( sceneHi[k], w );
			}
		}
	}
	dInst.resize( nRec * sizeof( DevInstance ) ), dInstDesc.resize( nRec ), dInstT.resize( nRec * 16 ), dInstMesh.resize( nRec );
	dSceneError.resize( 1 ), dTlasDepth.resize( 1 );
	CHK_HIP( hipMemcpyAsync( dInst.ptr, di, nRec * sizeof( DevInstance ), hipMemcpyHostToDevice, stream ) );
	CHK_HIP( hipMemcpyAsync( dInstDesc.ptr, desc, nRec * sizeof( lh2_CoreInstanceDesc ), hipMemcpyHostToDevice, stream ) );
	CHK_HIP( hipMemsetAsync( dSceneError.ptr, 0, sizeof( int ), stream ) );
	if (ni >= 2 && gpuTlas)
	{
		/* TLAS built on the device from the instance transforms (bvh_gpu.h) */
		CHK_HIP( hipMemcpyAsync( dInstT.ptr, Ts, nRec * 64, hipMemcpyHostToDevice, stream ) );
		CHK_HIP( hipMemcpyAsync( dInstMesh.ptr, meshIds, nRec * 4, hipMemcpyHostToDevice, stream ) );
		GpuTlasArgs ta;
		ta.T = dInstT.ptr, ta.instMesh = dInstMesh.ptr, ta.meshBounds = dMeshBounds.ptr, ta.count = ni;
		ta.nodeBase = blasNodeCount, ta.nodes = dNodes.ptr, ta.maxBlasDepth = StackDepthBound();
		ta.sceneError = dSceneError.ptr, ta.tlasDepth = dTlasDepth.ptr;
		gpuBvh.BuildTlas( ta, stream );
		tlasOnDevice = true;
		sceneMaxDepth = -1;   /* known on the device; SceneInfo reads it */
	}
	else
	{
		/* host TLAS (binned SAH) over instance world bounds, 1 instance per leaf */
		std::vector<Aabb> prims;
		std::vector<int> primInst;
		for (int i = 0; i < ni; i++)
		{
			const CoreInstanceHost& in = instances[i];
			const CoreMeshHost& m = *meshes[in.mesh];
			if (m.triCount == 0) continue;
			Aabb b;
			for (int k = 0; k < 3; k++) b.lo[k] = 1e30f, b.hi[k] = -1e30f;
			for (int c = 0; c < 8; c++)
			{
				const float p[3] = { (c & 1) ? m.aabbHi[0] : m.aabbLo[0], (c & 2) ? m.aabbHi[1] : m.aabbLo[1], (c & 4) ? m.aabbHi[2] : m.aabbLo[2] };
				for (int k = 0; k < 3; k++)
				{
					const float* r = in.T + k * 4;
					const float v = r[0] * p[0] + r[1] * p[1] + r[2] * p[2] + r[3];
					b.lo[k] = std::min( b.lo[k], v ), b.hi[k] = std::max( b.hi[k], v );
				}
			}
			/* pad by a relative epsilon: the ray is transformed in fp32 on the device */
			for (int k = 0; k < 3; k++)
			{
				const float e = 1e-5f * std::max( std::fabs( b.lo[k] ), std::fabs( b.hi[k] ) ) + 1e-30f;
				b.lo[k] -= e, b.hi[k] += e;
			}
			prims.push_back( b ), primInst.push_back( i );
		}
		BvhOutput tlas;
		BuildBvh2( prims, 1, 1, tlas );
		const size_t tn = tlas.nodes.size() / 16;
		if (tn > (size_t)tlasCapacity) FatalError( "TLAS of %zu nodes exceeds its capacity %d", tn, tlasCapacity );
		for (size_t k = 0; k < tn; k++)
		{
			int* refs = (int*)&tlas.nodes[k * 16 + 12];
			for (int c = 0; c < 2; c++)
			{
				if (refs[c] >= 0) refs[c] += blasNodeCount;
				else if (!prims.empty())
				{
					if (LEAF_COUNT( refs[c] ) != 1) FatalError( "TLAS leaf with %d instances", LEAF_COUNT( refs[c] ) );
					refs[c] = MAKE_LEAF( (uint32_t)primInst[tlas.perm[LEAF_FIRST( refs[c] )]], 1 );
				}
			}
		}
		if (tlas.nodes.size() * sizeof( float ) > need - offNodes) FatalError( "TLAS staging overflow" );
		memcpy( sb + offNodes, tlas.nodes.data(), tlas.nodes.size() * sizeof( float ) );
		CHK_HIP( hipMemcpyAsync( dNodes.ptr + (size_t)blasNodeCount * 4, sb + offNodes, tlas.nodes.size() * sizeof( float ), hipMemcpyHostToDevice, stream ) );
		sceneMaxDepth = tlas.maxDepth + StackDepthBound();
		tlasOnDevice = false;
		if (sceneMaxDepth >= LH2_STACK_TOTAL - 1) FatalError( "BVH depth %d exceeds the traversal stack (%d)", sceneMaxDepth, LH2_STACK_TOTAL );
	}
	/* the TLAS in the BVH4 array: its BVH2 nodes as two-child BVH4 nodes (one short launch) */
	if (bvh4) GpuBvhBuilder::TlasToBvh4( dNodes.ptr, blasNodeCount, tlasCapacity, blasNode4Count, dNodes4.ptr, stream );
	CHK_HIP( hipEventRecord( evStage[slot], stream ) );
	instancesDirty = false;
}

/* device-side scene errors (TLAS deeper than the traversal stack): the trace kernels skip the
   frame, and the host reports it here */
void RenderCore::CheckSceneError()
{
	if (!dSceneError.ptr) return;
	int e = 0;
	CHK_HIP( hipMemcpyAsync( &hostStats->sceneError, dSceneError.ptr, sizeof( int ), hipMemcpyDeviceToHost, stream ) );
	CHK_HIP( hipStreamSynchronize( stream ) );
	e = hostStats->sceneError;
	if (e) FatalError( "BVH depth exceeds the traversal stack (%d levels)", LH2_STACK_TOTAL );
}

SceneDev RenderCore::MakeSceneDev() const
{
	SceneDev s;
	s.nodes = dNodes.ptr, s.tris = dTris.ptr, s.inst = (const DevInstance*)dInst.ptr;
	s.sceneError = dSceneError.ptr;
	s.argb32 = dArgb32.ptr, s.nrm32 = dNrm32.ptr;
	s.argb32Count = (uint32_t)dArgb32.count, s.nrm32Count = (uint32_t)dNrm32.count;
	s.tlasRoot = tlasRoot, s.instCount = (int)instances.size();
	s.nodes4 = dNodes4.ptr, s.tlasRoot4 = blasNode4Count;
	/* one instance of a non-empty mesh: rays start at its TLAS leaf (MAKE_LEAF( 0, 1 ) = ~0) and skip
	   the TLAS root's box test, which can only cull (TopLevelBVH::Traverse bvh.cpp:594-649); the
	   instance transform runs as at the leaf, so the hits are unchanged: one loop iteration less per ray */
	if (singleInstanceStart && instances.size() == 1 && instances[0].mesh >= 0 && instances[0].mesh < (int)meshes.size() &&
		meshes[instances[0].mesh]->triCount > 0)
		s.tlasRoot = s.tlasRoot4 = ~0;
	s.instDesc = dInstDesc.ptr, s.materials = dMaterials.ptr;
	s.areaLights = dArea.ptr, s.pointLights = dPoint.ptr, s.spotLights = dSpot.ptr, s.dirLights = dDir.ptr;
	s.nArea = nArea, s.nPoint = nPoint, s.nSpot = nSpot, s.nDir = nDir;
	s.sky = dSky.ptr, s.skyW = skyW, s.skyH = skyH;
	s.blueNoise = dBlueNoise.ptr;
	s.geometryEpsilon = geometryEpsilon, s.clampValue = clampValue;
	return s;
}

static inline uint32_t XorShift( uint32_t& s ) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }  /* platform/system.cpp:48 */

void RenderCore::Render( const lh2_ViewPyramid& view, int converge )   /* rendercore.cpp:463-609 */
{
	if (!initialized) FatalError( "Render before Init" );
	if (!scrwidth) FatalError( "Render before SetTarget" );
	if (geometryDirty || instancesDirty) UpdateToplevel();
	if (!dMaterials.ptr) FatalError( "Render before SetMaterials" );
	const auto t0 = std::chrono::high_resolution_clock::now();
	/* CoreStats timings come from the stop events recorded by the launches themselves (LaunchEvents):
	   no hipEventRecord between kernels */
	const bool restart = converge == LH2_RESTART || firstConvergingFrame;
	if (restart)
	{
		samplesTaken = 0;
		firstConvergingFrame = true;
		camRNGseed = 0x12345678;
	}
	if (converge == LH2_CONVERGE) firstConvergingFrame = false;
	const int tileRows = TileRows();
	const int tilePix = tileRows * scrwidth;
	const uint32_t pathCount = (uint32_t)tilePix * (uint32_t)scrspp;
	const SceneDev sd = MakeSceneDev();
	/* path groups (PathGroup): contiguous shares of the tile's paths with their boundaries on whole
	   waves (64 slots: an 8x8 pixel block stays in one group), each on its own stream; small frames
	   run as one group */
	const int G = pathCount >= 4096u * (uint32_t)pathGroups ? pathGroups : 1;
	frameGroups = G;
	/* the accumulator reset of a restart: one frame-wide memset when path groups run concurrently,
	   else folded into the camera launch (each pixel's first sample zeroes it; rows outside this
	   rank's tile stay zero from SetTarget / SetTileBands) */
	if (restart && (G > 1 || tileChanged)) CHK_HIP( hipMemsetAsync( accumulator.ptr, 0, sizeof( float4 ) * (size_t)scrwidth * scrheight, stream ) );
	/* primary rays (camera.h) for every sample of the tile */
	CameraParams cp{};
	cp.pos = view.pos, cp.p1 = view.p1;
	cp.right = { view.p2.x - view.p1.x, view.p2.y - view.p1.y, view.p2.z - view.p1.z };
	cp.up = { view.p3.x - view.p1.x, view.p3.y - view.p1.y, view.p3.z - view.p1.z };
	cp.aperture = view.aperture, cp.distortion = view.distortion, cp.geometryEpsilon = geometryEpsilon;
	cp.w = scrwidth, cp.h = scrheight, cp.pass = samplesTaken;
	cp.R0 = XorShift( camRNGseed );
	cp.y0 = std::max( 0, tileY0 ), cp.tileRows = tileRows;
	cp.band = tileBand > 0 ? tileBand : std::max( 1, tileRows ), cp.bandStride = tileBand > 0 ? tileStride : std::max( 1, tileRows );
	cp.tiled = tiledRays;
	cp.spp = G == 1 && sampleInterleave ? scrspp : 0;
	cp.primeRef = primeRef;
	const bool twoEndedPrimary = chordSplitPrimary > 0 && tiledRays && !primeRef && scrwidth % 8 == 0 && tileRows % 8 == 0;
	const float primaryCut = twoEndedPrimary ? PrimaryChordCut( view ) : 0.0f;
	const int grid = TraceGrid();
	int maxPL = primeRef ? LH2_MAX_BOUNCES : maxPathLength;
	/* no specular event and no alpha cut-out in any material: every path ends at its second vertex,
	   so the bounce after it would be empty; not launching it saves three launches (~25 us) */
	if (!primeRef && diffuseOnly) maxPL = std::min( maxPL, 2 );
	/* the frame's start: a marker before the camera launch (~4 us of idle GPU), not the launch's own start
	   event (hipExtLaunchKernelGGL start events cost ~8 us: tools/launch_gap.hip, profiles/r02q_launch_gap.txt) */
	CHK_HIP( hipEventRecord( evFrame[0], stream ) );
	if (G > 1) CHK_HIP( hipEventRecord( evFork, stream ) );   /* the other groups start after the accumulator reset */
	for (int gi = 0; gi < G; gi++)
	{
		PathGroup& g = grp[gi];
		const uint32_t b0 = (uint32_t)(((uint64_t)pathCount * gi / G) & ~63ull);
		const uint32_t b1 = gi + 1 == G ? pathCount : (uint32_t)(((uint64_t)pathCount * (gi + 1) / G) & ~63ull);
		g.base = b0, g.count = b1 - b0;
		EnsureGroup( g, g.count );
		/* segmented path / ray streams (lh2_kernels.h): LH2_SEGS segments of segStride records; shadow
		   rays in segments of shadowStride */
		g.segStride = (g.count + LH2_SEGS - 1) / LH2_SEGS;
		g.shadowStride = (uint32_t)(g.shO.count / LH2_SEGS);
		g.in = 0, g.pl = 0, g.done = false, g.tailL = 0;
		if (gi) CHK_HIP( hipStreamWaitEvent( g.st, evFork, 0 ) );
		/* the camera launch also resets the group's counters and work-queue heads (k_init_counters) */
		CameraParams cg = cp;
		cg.slotBase = (int)g.base;
		cg.initC = g.counters.ptr, cg.cursors = g.cursors.ptr, cg.cursorWords = LH2_CURSOR_SLOTS * LH2_CURSOR_WORDS;
		cg.pathCount = g.count, cg.segStride = g.segStride;
		cg.clearAcc = restart && G == 1 && !tileChanged ? accumulator.ptr : nullptr;
		/* two-ended primary segments: whole 8x8 tiles in whole segments only */
		g.twoEnded = twoEndedPrimary && g.segStride % 64 == 0 && g.count % 64 == 0;
		/* heavy-first primary packets: this frame reads the block the previous one recorded, and records
		   into the other one, which the camera launch zeroes (a new layout zeroes both) */
		const bool heavy = packetHeavy > 0 && tiledRays && UsePackets() && !primeRef;
		if (heavy)
		{
			const uint32_t cap = (g.segStride + 63) / 64, maskWords = (LH2_SEGS * cap + 31) / 32;
			if (cap != g.hvCap)
			{
				g.hvCap = cap, g.hvMaskWords = maskWords, g.hvBlock = LH2_HV_MASK + maskWords + LH2_SEGS * cap, g.hvParity = 0;
				g.hv.resize( 2 * (size_t)g.hvBlock );
				CHK_HIP( hipMemsetAsync( g.hv.ptr, 0, sizeof( uint32_t ) * 2 * g.hvBlock, g.st ) );
			}
			cg.hvZero = g.hv.ptr + (size_t)(1 - g.hvParity) * g.hvBlock, cg.hvZeroWords = LH2_HV_MASK + g.hvMaskWords;
		}
		g.hvOn = heavy;
		if (g.twoEnded)
		{
			cg.camAlloc = g.camAlloc.ptr + (g.camFrame & 1) * LH2_CAM_ALLOC_WORDS;
			cg.camZero = g.camAlloc.ptr + ((g.camFrame + 1) & 1) * LH2_CAM_ALLOC_WORDS;
			g.camFrame++;
			for (int k = 0; k < 3; k++) cg.chordLo[k] = sceneLo[k], cg.chordHi[k] = sceneHi[k];
			cg.chordCut = primaryCut;
		}
		lh2_launch_camera( &cg, dBlueNoise.ptr, g.rayO[0].ptr, g.rayD[0].ptr, g.T4[0].ptr, g.Q4[0].ptr, (int)g.count, { nullptr, g.evCamera }, g.st );
		g.prevStop = g.evCamera;
	}
	if (restart) tileChanged = false;
	/* without lights no path samples one (RandomPointOnLight: lightPdf 0), so there are no shadow
	   rays and their launches are not queued */
	const bool shadows = nArea + nPoint + nSpot + nDir > 0;
	frameShadows = shadows;
	const int splitL = (shadows && !primeRef && G == 1 && shadowSplit > 0 && shadowSplit < maxPL) ? shadowSplit : 0;
	frameSplit = false;
	/* two-ended shadow segments (setting "chordSplitShadow"): shadow rays shorter than it x the scene's
	   extent are traced last; not with the shadow split or PrimeRef's per-bounce shadow launches */
	float shadowCut = -3.0e38f;   /* off: no shadow ray is that short */
	if (!splitL && !primeRef && chordSplitShadow > 0)
		shadowCut = chordSplitShadow * std::max( std::max( sceneHi[0] - sceneLo[0], sceneHi[1] - sceneLo[1] ), sceneHi[2] - sceneLo[2] );
	/* the path tail (setting "pathTail"): bounces pathTail .. maxPL in one launch of k_trace_path4d */
	const int tailL = (!primeRef && G == 1 && !splitL && pathTail >= 2 && pathTail <= maxPL && TraceVersion() == 7 && dNodes4.ptr) ? pathTail : 0;
	/* the bounce loop, the groups' launches interleaved */
	for (int pathLength = 1; pathLength <= maxPL; pathLength++)
	{
		bool any = false;
		for (int gi = 0; gi < G; gi++)
		{
			PathGroup& g = grp[gi];
			if (g.done) continue;
			any = true;
			g.pl = pathLength;
			Counters* c = g.counters.ptr;
			TraceArgs ta{};
			ta.version = TraceVersion();
			/* the path counts ping-pong (Counters::segPath): this bounce's paths, and its extension rays */
			uint32_t* segIn = c->segPath[(pathLength - 1) & 1];
			uint32_t* segNext = c->segPath[pathLength & 1];
			uint32_t* segInBack = c->segBack[(pathLength - 1) & 1];
			if (pathLength == 1 && g.twoEnded)
			{
				/* the camera's two-ended segments (zeroed when retired at the hand-off, as segPath[0] is) */
				segIn = g.camAlloc.ptr + ((g.camFrame - 1) & 1) * LH2_CAM_ALLOC_WORDS;
				segInBack = segIn + LH2_SEGS * LH2_SEGCOUNT_STRIDE;
			}
			uint32_t* segNextBack = c->segBack[pathLength & 1];
			ta.rayO = g.rayO[g.in].ptr, ta.rayD = g.rayD[g.in].ptr, ta.segCounts = segIn, ta.segStride = g.segStride;
			ta.segBack = segInBack;
			ta.cursor = g.cursors.ptr + (size_t)pathLength * LH2_CURSOR_WORDS;
			ta.refill = (uint32_t)(pathLength == 1 && tiledRays ? refillPrimary : refillOther);
			ta.packet = pathLength == 1 && tiledRays && UsePackets() ? PacketMode() : 0;
			ta.leafBatch = (uint32_t)(pathLength == 1 && tiledRays ? leafBatchPrimary : leafBatch);
			if (pathLength == 1 && ta.packet && g.hvOn)
			{
				ta.hvRead = g.hv.ptr + (size_t)g.hvParity * g.hvBlock, ta.hvWrite = g.hv.ptr + (size_t)(1 - g.hvParity) * g.hvBlock;
				ta.hvCap = g.hvCap, ta.hvMaskWords = g.hvMaskWords, ta.hvFactor = packetHeavy;
				ta.hvTiles = 0;
				for (int k = 0; k < LH2_SEGS; k++)
				{
					const uint32_t lo = (uint32_t)k * g.segStride, n = g.count > lo ? std::min( g.count - lo, g.segStride ) : 0u;
					ta.hvTiles += (n + 63) / 64;
				}
				g.hvParity = 1 - g.hvParity;
			}
			ta.hits = g.hits.ptr, ta.gstack = g.gstack.ptr;
			SetTail( ta, g );
			if (pathLength == tailL)
			{
				/* the path tail: trace and shade every remaining bounce in one launch; each path's records
				   are updated in place, its shadow rays queued for the shadow launch, and rayLog counted */
				ShadeParams sp{};
				sp.shadowStride = g.shadowStride;
				sp.rayO = g.rayO[g.in].ptr, sp.rayD = g.rayD[g.in].ptr, sp.T4 = g.T4[g.in].ptr, sp.Q4 = g.Q4[g.in].ptr;
				sp.rayOut = g.rayO[g.in].ptr, sp.rayDOut = g.rayD[g.in].ptr, sp.T4Out = g.T4[g.in].ptr, sp.Q4Out = g.Q4[g.in].ptr;
				sp.shO = g.shO.ptr, sp.shD = g.shD.ptr, sp.shP = g.shP.ptr;
				sp.acc = accumulator.ptr, sp.counters = c;
				sp.w = scrwidth, sp.h = scrheight, sp.pass = samplesTaken, sp.pathLength = pathLength, sp.maxPathLength = maxPL;
				sp.probePixel = probeX + scrwidth * probeY;
				sp.spreadAngle = view.spreadAngle;
				sp.adv.rayCountLog = g.rayLog.ptr;
				ta.shadeBatch = (uint32_t)pathTailBatch;
				sp.shadowCut = shadowCut;
				lh2_launch_trace_path( &sd, &ta, &sp, PathGrid(), { nullptr, g.evTrace[pathLength] }, g.st );
				g.fromTrace[pathLength] = g.prevStop, g.prevStop = g.evTrace[pathLength];
				g.tailL = pathLength;   /* no shade interval of its own (Synchronize) */
				g.done = true;
				continue;
			}
			/* the last bounce of a terminal frame (no lights, nothing that emits or cuts out: its hits add
			   nothing, ShadeParams::terminal): the trace launch adds the misses' sky samples itself, so there
			   is no hit record to write and no k_shade_last launch (setting "terminalTrace") */
			if (pathLength == maxPL && pathLength > 1 && !primeRef && !shadows && !canEmit && terminalShade && terminalTrace &&
				!ta.packet && TraceVersion() == 7 && dNodes4.ptr)
			{
				ta.pathT4 = g.T4[g.in].ptr, ta.pathQ4 = g.Q4[g.in].ptr, ta.acc = accumulator.ptr, ta.wh = (uint32_t)(scrwidth * scrheight);
				lh2_launch_trace_term( &sd, &ta, grid, { nullptr, g.evTrace[pathLength] }, g.st );
				g.fromTrace[pathLength] = g.prevStop, g.prevStop = g.evTrace[pathLength];
				g.tailL = pathLength;   /* no shade interval of its own (Synchronize) */
				g.done = true;
				continue;
			}
			/* shadow backfill: the shadow rays of the bounces before this one (their counts no longer change
			   during this launch) are the final shadow launch's work; this launch's idle lanes take them in its
			   tail, from that launch's work-queue heads (one-ended shadow segments only) */
			if (shadowBackfill && shadows && !primeRef && !splitL && !ta.packet && pathLength >= 2 && TraceVersion() == 7 &&
				dNodes4.ptr && !(shadowCut > 0.0f))
			{
				ta.bfO = g.shO.ptr, ta.bfD = g.shD.ptr, ta.bfCounts = c->segShadow, ta.bfStride = g.shadowStride;
				ta.bfCursor = g.cursors.ptr + (size_t)LH2_SHADOW_SLOT * LH2_CURSOR_WORDS;
				ta.potentials = g.shP.ptr, ta.acc = accumulator.ptr;
			}
			lh2_launch_trace_closest( &sd, &ta, ta.packet ? PacketGrid() : grid, { nullptr, g.evTrace[pathLength] }, g.st );
			g.fromTrace[pathLength] = g.prevStop, g.prevStop = g.evTrace[pathLength];
			ShadeParams sp{};
			sp.segCounts = segIn, sp.segOut = segNext, sp.segStride = g.segStride, sp.shadowStride = g.shadowStride;
			sp.segBack = segInBack, sp.segOutBack = segNextBack;
			/* two-ended path segments: rays with a chord through the scene box below chordSplit x its
			   largest extent go last (setting "chordSplit"; 0: off) */
			{
				const float ext = std::max( std::max( sceneHi[0] - sceneLo[0], sceneHi[1] - sceneLo[1] ), sceneHi[2] - sceneLo[2] );
				for (int k = 0; k < 3; k++) sp.chordLo[k] = sceneLo[k], sp.chordHi[k] = sceneHi[k];
				sp.chordCut = ext > 0 ? chordSplit * ext : 0.0f;
			}
			/* the hand-off to the next bounce: the shade launch's last block (no launch of its own), except
			   in PrimeRef mode, where the bounce's shadow rays are traced (and their counts reset) first */
			const bool split = pathLength == splitL;
			const BounceAdvance adv{ segNext, segNextBack, segIn, segInBack, g.rayLog.ptr, g.activeLog, split ? shadowSnap.ptr : nullptr,
				split ? g.cursors.ptr + (size_t)LH2_SHADOW_SLOT * LH2_CURSOR_WORDS : nullptr, pathLength + 1 == tailL };
			sp.advance = pathLength < maxPL && !primeRef;
			sp.shadowCut = shadowCut;
			sp.adv = adv;
			sp.rayO = g.rayO[g.in].ptr, sp.rayD = g.rayD[g.in].ptr, sp.T4 = g.T4[g.in].ptr, sp.Q4 = g.Q4[g.in].ptr, sp.hits = g.hits.ptr;
			sp.rayOut = g.rayO[1 - g.in].ptr, sp.rayDOut = g.rayD[1 - g.in].ptr, sp.T4Out = g.T4[1 - g.in].ptr, sp.Q4Out = g.Q4[1 - g.in].ptr;
			sp.shO = g.shO.ptr, sp.shD = g.shD.ptr, sp.shP = g.shP.ptr;
			sp.acc = accumulator.ptr, sp.counters = c;
			sp.w = scrwidth, sp.h = scrheight, sp.pass = samplesTaken, sp.pathLength = pathLength, sp.maxPathLength = maxPL;
			sp.primeRef = primeRef;
			sp.terminal = !primeRef && !shadows && !canEmit && pathLength > 1 && terminalShade;
			sp.probePixel = probeX + scrwidth * probeY;
			sp.R0 = (uint32_t)samplesTaken * 7907u + (uint32_t)pathLength * 91771u;
			sp.spreadAngle = view.spreadAngle;
			lh2_launch_shade( &sd, &sp, grid, { nullptr, g.evShade[pathLength] }, g.st );
			g.fromShade[pathLength] = g.prevStop, g.prevStop = g.evShade[pathLength];
			if (pathLength == maxPL) { g.done = true; continue; }
			if (primeRef && shadows)
			{
				/* RenderCore_PrimeRef traces the shadow rays of every bounce right after it
				   (rendercore.cpp connect step), fused with finalizeConnections */
				TraceArgs ts{};
				ts.version = ShadowVersion();
				ts.rayO = g.shO.ptr, ts.rayD = g.shD.ptr, ts.segCounts = c->segShadow, ts.segStride = g.shadowStride;
				ts.cursor = g.cursors.ptr + (size_t)(LH2_MAX_BOUNCES + pathLength) * LH2_CURSOR_WORDS;
				ts.refill = ShadowRefill(), ts.leafBatch = ShadowLeafBatch();
				ts.mask = g.shMask.ptr, ts.potentials = g.shP.ptr, ts.acc = accumulator.ptr, ts.gstack = g.gstack.ptr;
				ts.packet = packetShadow ? PacketMode() : 0;
				SetTail( ts, g );
				lh2_launch_trace_any( &sd, &ts, grid, 1, { nullptr, g.evShadowB[pathLength] }, g.st );
				g.fromShadowB[pathLength] = g.prevStop, g.prevStop = g.evShadowB[pathLength];
			}
			/* the hand-off writes this bounce's extension-ray count into the pinned activeLog itself */
			g.countReady[pathLength] = g.evShade[pathLength];
			if (primeRef)
			{
				lh2_launch_counters_next( c, &adv, pathLength, 1, { nullptr, g.evCount[pathLength] }, g.st );
				g.prevStop = g.countReady[pathLength] = g.evCount[pathLength];
			}
			if (split)
			{
				/* the shadow rays queued so far, on the side stream, beside the later bounces; the final
				   shadow launch's work queues start behind them (advance_bounce) */
				CHK_HIP( hipStreamWaitEvent( sideStream, g.countReady[pathLength], 0 ) );
				TraceArgs ta{};
				ta.version = ShadowVersion();
				ta.rayO = g.shO.ptr, ta.rayD = g.shD.ptr, ta.segCounts = shadowSnap.ptr, ta.segStride = g.shadowStride;
				ta.cursor = g.cursors.ptr + (size_t)(LH2_MAX_BOUNCES + pathLength) * LH2_CURSOR_WORDS, ta.refill = ShadowRefill(), ta.leafBatch = ShadowLeafBatch();
				ta.mask = g.shMask.ptr, ta.potentials = g.shP.ptr, ta.acc = accumulator.ptr, ta.gstack = sideStack.ptr;
				ta.packet = packetShadow ? PacketMode() : 0;
				lh2_launch_trace_any( &sd, &ta, grid, 1, { evSideStart, evSideStop }, sideStream );
				frameSplit = true;
			}
		}
		if (!any) break;
		/* early exit without stalling the GPU: wait for the count of a group's previous bounce while
		   this bounce is queued; when it was 0, this bounce is empty and so is everything after it */
		for (int gi = 0; gi < G; gi++)
		{
			PathGroup& g = grp[gi];
			if (g.done) continue;
			if (pathLength >= 2)
			{
				CHK_HIP( hipEventSynchronize( g.countReady[pathLength - 1] ) );
				if (g.activeLog[pathLength - 1] == 0) { g.done = true; continue; }
			}
			g.in = 1 - g.in;
		}
	}
	/* shadow rays + fused finalizeConnections (rendercore.cpp:575-592); then the groups join */
	for (int gi = 0; gi < G; gi++)
	{
		PathGroup& g = grp[gi];
		if (!primeRef && shadows)
		{
			TraceArgs ta{};
			ta.version = ShadowVersion();
			ta.rayO = g.shO.ptr, ta.rayD = g.shD.ptr, ta.segCounts = g.counters.ptr->segShadow, ta.segStride = g.shadowStride;
			ta.segBack = g.counters.ptr->segShadowBack;
			ta.cursor = g.cursors.ptr + (size_t)LH2_SHADOW_SLOT * LH2_CURSOR_WORDS, ta.refill = ShadowRefill(), ta.leafBatch = ShadowLeafBatch();
			ta.mask = g.shMask.ptr, ta.potentials = g.shP.ptr, ta.acc = accumulator.ptr, ta.gstack = g.gstack.ptr;
			ta.packet = packetShadow ? PacketMode() : 0;
			SetTail( ta, g );
			lh2_launch_trace_any( &sd, &ta, ta.version >= 5 && !ta.packet ? ShadowGrid() : grid, 1, { nullptr, g.evShadow }, g.st );
			g.fromShadow = g.prevStop;
		}
		if (gi == 0 && frameSplit) CHK_HIP( hipStreamWaitEvent( stream, evSideStop, 0 ) );   /* join the side stream's shadow launch */
		if (gi)
		{
			CHK_HIP( hipEventRecord( g.evDone, g.st ) );
			CHK_HIP( hipStreamWaitEvent( stream, g.evDone, 0 ) );
		}
	}
	samplesTaken += scrspp;
	/* finalize also delivers every group's counters and ray-count log, and the scene error, to hostStats */
	FrameStatsDev fs{};
	fs.groups = G;
	for (int gi = 0; gi < G; gi++)
	{
		fs.counters[gi] = grp[gi].counters.ptr, fs.rayLog[gi] = grp[gi].rayLog.ptr + 1;
		fs.hostCounters[gi] = &hostStats->counters[gi], fs.hostRayCount[gi] = hostStats->rayCount[gi] + 1;
	}
	fs.sceneError = dSceneError.ptr, fs.hostSceneError = &hostStats->sceneError;
	/* a tile finalizes its own rows only (a rank of the band partition: the gathered frame is finalized
	   where it is assembled, MultiDevice / FinalizeFrame) */
	RowMap rm{};
	if (tileRows < scrheight) rm = { scrwidth, cp.y0, cp.band, cp.bandStride, tileRows };
	lh2_launch_finalize( accumulator.ptr, frame.ptr, scrwidth * scrheight, 1.0f / (float)samplesTaken, &fs, { nullptr, evFrame[1] }, stream, &rm );
	if (glResource && !displayAtFinalize)
	{
		hipArray_t arr = nullptr;
		CHK_HIP( hipGraphicsMapResources( 1, &glResource, stream ) );
		CHK_HIP( hipGraphicsSubResourceGetMappedArray( &arr, glResource, 0, 0 ) );
		CHK_HIP( hipMemcpy2DToArrayAsync( arr, 0, 0, frame.ptr, sizeof( float4 ) * scrwidth, sizeof( float4 ) * scrwidth, scrheight, hipMemcpyDeviceToDevice, stream ) );
		CHK_HIP( hipGraphicsUnmapResources( 1, &glResource, stream ) );
	}
	framePathLengths = 0;
	for (int gi = 0; gi < G; gi++) hostStats->rayCount[gi][0] = grp[gi].count, framePathLengths = std::max( framePathLengths, grp[gi].tailL ? maxPL : grp[gi].pl );
	framePrimeRef = primeRef;
	statsPending = true;
	frameHostMs = std::chrono::duration<double, std::milli>( std::chrono::high_resolution_clock::now() - t0 ).count();
}

/* the chordSplitPrimary quantile of the frame's 8x8 tile centre rays' lengths inside the scene box (pinhole
   rays through the tile centres, at most ~4096 of them; box_chord in lh2_kernels.hip is the device side),
   recomputed when the view or the box changes */
float RenderCore::PrimaryChordCut( const lh2_ViewPyramid& view )
{
	const float box[7] = { sceneLo[0], sceneLo[1], sceneLo[2], sceneHi[0], sceneHi[1], sceneHi[2], chordSplitPrimary };
	if (cutValid && !memcmp( &view, &cutView, sizeof( view ) ) && !memcmp( box, cutBox, sizeof( box ) )) return cutValue;
	const int tw = scrwidth / 8, th = std::max( 1, scrheight / 8 );
	const int step = std::max( 1, (int)std::ceil( std::sqrt( (double)tw * th / 4096.0 ) ) );
	std::vector<float> len;
	for (int ty = 0; ty < th; ty += step)
		for (int tx = 0; tx < tw; tx += step)
		{
			const float fx = (tx * 8 + 4.5f) / scrwidth, fy = (ty * 8 + 4.5f) / scrheight;
			float d[3], o[3] = { view.pos.x, view.pos.y, view.pos.z };
			const float p1[3] = { view.p1.x, view.p1.y, view.p1.z }, p2[3] = { view.p2.x, view.p2.y, view.p2.z }, p3[3] = { view.p3.x, view.p3.y, view.p3.z };
			for (int k = 0; k < 3; k++) d[k] = p1[k] + fx * (p2[k] - p1[k]) + fy * (p3[k] - p1[k]) - o[k];
			float tn = 0, tf = 1e30f;
			for (int k = 0; k < 3; k++)
			{
				const float inv = 1.0f / d[k], a = (sceneLo[k] - o[k]) * inv, b = (sceneHi[k] - o[k]) * inv;
				if (a == a && b == b) tn = std::max( tn, std::min( a, b ) ), tf = std::min( tf, std::max( a, b ) );
			}
			const float n = std::sqrt( d[0] * d[0] + d[1] * d[1] + d[2] * d[2] );
			len.push_back( (tf - tn) * n );   /* d is not normalised: scale t to distance */
		}
	const size_t q = std::min( len.size() - 1, (size_t)(chordSplitPrimary * (len.size() - 1)) );
	std::nth_element( len.begin(), len.begin() + q, len.end() );
	cutValue = len[q], cutView = view, cutValid = true;
	memcpy( cutBox, box, sizeof( box ) );
	return cutValue;
}

void RenderCore::UnpackTile( const void* devSrc, int rank, int nranks, int band )
{
	int rows = 0;
	for (int y = rank * band; y < scrheight; y += nranks * band) rows += std::min( band, scrheight - y );
	lh2_launch_unpack_rows( (const float4*)devSrc, accumulator.ptr, scrwidth, rank * band, band, nranks * band, rows, {}, stream );
}

void RenderCore::FinalizeFrame()
{
	if (!samplesTaken) return;
	lh2_launch_finalize( accumulator.ptr, frame.ptr, scrwidth * scrheight, 1.0f / (float)samplesTaken, nullptr, {}, stream );
	if (glResource)
	{
		hipArray_t arr = nullptr;
		CHK_HIP( hipGraphicsMapResources( 1, &glResource, stream ) );
		CHK_HIP( hipGraphicsSubResourceGetMappedArray( &arr, glResource, 0, 0 ) );
		CHK_HIP( hipMemcpy2DToArrayAsync( arr, 0, 0, frame.ptr, sizeof( float4 ) * scrwidth, sizeof( float4 ) * scrwidth, scrheight, hipMemcpyDeviceToDevice, stream ) );
		CHK_HIP( hipGraphicsUnmapResources( 1, &glResource, stream ) );
	}
}

void RenderCore::CopyFrameAsync( void* devDst )
{
	CHK_HIP( hipMemcpyAsync( devDst, frame.ptr, sizeof( float4 ) * (size_t)scrwidth * scrheight, hipMemcpyDeviceToDevice, stream ) );
}

int RenderCore::TileRows() const
{
	if (tileBand > 0)
	{
		int rows = 0;
		for (int y = tileY0; y < scrheight; y += tileStride) rows += std::min( tileBand, scrheight - y );
		return rows;
	}
	const int y0 = std::max( 0, tileY0 ), y1 = tileY1 < 0 ? scrheight : std::min( scrheight, tileY1 );
	return std::max( 0, y1 - y0 );
}

/* shadow rays queued in the segments of the shadow stream (the final shadow pass traces them all) */
static uint32_t QueuedShadowRays( const Counters& c )
{
	uint32_t n = 0;
	for (int k = 0; k < LH2_SEGS; k++) n += c.segShadow[k * LH2_SEGCOUNT_STRIDE] + c.segShadowBack[k * LH2_SEGCOUNT_STRIDE];
	return n;
}

void RenderCore::Synchronize()
{
	CHK_HIP( hipStreamSynchronize( stream ) );   /* the other groups' streams joined into `stream` */
	if (statsPending)
	{
		statsPending = false;
		for (int gi = 0; gi < frameGroups; gi++)
		{
			const Counters& cn = hostStats->counters[gi];
			bool full = cn.shadowOverflow != 0;   /* a segment's two ends met: same failure */
			for (int k = 0; k < LH2_SEGS; k++) full = full || cn.segShadow[k * LH2_SEGCOUNT_STRIDE] + cn.segShadowBack[k * LH2_SEGCOUNT_STRIDE] > grp[gi].shadowStride;
			if (full) FatalError( "shadow ray buffer overflow" );
		}
		if (hostStats->sceneError) FatalError( "BVH depth exceeds the traversal stack (%d levels): frame skipped", LH2_STACK_TOTAL );
		uint32_t rc[LH2_MAX_BOUNCES + 1] = {};   /* rc[0] = primary; rc[L] = rays traced at pathLength L+1 */
		for (int gi = 0; gi < frameGroups; gi++) for (int L = 0; L <= LH2_MAX_BOUNCES; L++) rc[L] += hostStats->rayCount[gi][L];
		auto ms = [&]( hipEvent_t a, hipEvent_t b ) { float t = 0; (void)hipEventElapsedTime( &t, a, b ); return t * 1e-3f; };
		/* each interval: a group's previous launch's stop event -> this launch's stop event (kernel +
		   launch gap); with overlapping groups, a pass takes the longest of the groups' intervals */
		auto trace = [&]( int L ) {
			float t = 0;
			for (int gi = 0; gi < frameGroups; gi++) if (L <= grp[gi].pl) t = std::max( t, ms( grp[gi].fromTrace[L], grp[gi].evTrace[L] ) );
			return t;
		};
		coreStats.primaryRayCount = rc[0];
		coreStats.traceTime0 = trace( 1 );
		coreStats.bounce1RayCount = framePathLengths >= 2 ? rc[1] : 0;
		coreStats.traceTime1 = framePathLengths >= 2 ? trace( 2 ) : 0;
		coreStats.deepRayCount = 0, coreStats.traceTimeX = 0;
		/* (a path tail's bounces past its first have no launch of their own: their time is in its launch) */
		for (int L = 3; L <= framePathLengths; L++)
		{
			coreStats.deepRayCount = rc[L - 1];
			if (std::any_of( grp, grp + frameGroups, [L]( const PathGroup& g ) { return L <= g.pl; } )) coreStats.traceTimeX = trace( L );
		}
		float shadow = 0, shade = 0;
		for (int gi = 0; gi < frameGroups; gi++)
		{
			const PathGroup& g = grp[gi];
			float sh = 0, sd = 0;
			if (!frameShadows) sh = 0;
			else if (!framePrimeRef) sh = ms( g.fromShadow, g.evShadow );
			else for (int L = 1; L < g.pl; L++) sh += ms( g.fromShadowB[L], g.evShadowB[L] );
			for (int L = 1; L <= g.pl; L++) if (L != g.tailL) sd += ms( g.fromShade[L], g.evShade[L] );
			shadow = std::max( shadow, sh ), shade = std::max( shade, sd );
		}
		coreStats.shadowTraceTime = shadow;
		coreStats.shadeTime = shade;
		for (int L = 1; L <= framePathLengths && L <= 8; L++) lastKernelMs[L - 1] = trace( L ) * 1e3f;
		uint32_t shadowRays = 0, extRays = 0;
		int probe = 0;
		for (int gi = 0; gi < frameGroups; gi++)
		{
			const Counters& cnt = hostStats->counters[gi];
			shadowRays += framePrimeRef ? cnt.totalShadowRays : QueuedShadowRays( cnt );
			extRays += cnt.totalExtensionRays;
			if (cnt.probedInstid != -1 || cnt.probedTriid != -1) probe = gi;
		}
		coreStats.totalShadowRays = shadowRays;
		coreStats.totalExtensionRays = extRays;
		coreStats.totalRays = coreStats.totalExtensionRays + coreStats.totalShadowRays;
		coreStats.renderTime = ms( evFrame[0], evFrame[1] );   /* device time of the whole frame (the reference's Render blocks) */
		const Counters& pc = hostStats->counters[probe];
		coreStats.probedInstid = pc.probedInstid, coreStats.probedTriid = pc.probedTriid, coreStats.probedDist = pc.probedDist;
	}
}

lh2_CoreStats RenderCore::GetCoreStats()
{
	Synchronize();
	return coreStats;
}

void RenderCore::GetRayCounts( uint32_t* out17 )
{
	Synchronize();
	for (int i = 0; i < 17; i++)
	{
		out17[i] = 0;
		if (i < framePathLengths) for (int gi = 0; gi < frameGroups; gi++) out17[i] += hostStats->rayCount[gi][i];
	}
	out17[16] = 0;
	for (int gi = 0; gi < frameGroups; gi++)
		out17[16] += framePrimeRef ? hostStats->counters[gi].totalShadowRays : QueuedShadowRays( hostStats->counters[gi] );
}

void RenderCore::GetAccumulator( float* hostOut4 )
{
	Synchronize();
	CHK_HIP( hipMemcpy( hostOut4, accumulator.ptr, sizeof( float4 ) * (size_t)scrwidth * scrheight, hipMemcpyDeviceToHost ) );
}

void RenderCore::CopyAccumulatorRows( void* devDst, int y0, int y1 )
{
	CHK_HIP( hipMemcpyAsync( devDst, accumulator.ptr + (size_t)y0 * scrwidth, sizeof( float4 ) * (size_t)(y1 - y0) * scrwidth, hipMemcpyDeviceToDevice, stream ) );
	CHK_HIP( hipStreamSynchronize( stream ) );
}

void RenderCore::PackTile( void* devDst, bool ordered, void* consumer )
{
	const int rows = TileRows();
	const int band = tileBand > 0 ? tileBand : std::max( 1, rows ), stride = tileBand > 0 ? tileStride : std::max( 1, rows );
	/* asynchronous: consumers on other streams order themselves after the core stream (lh2_core_stream),
	   so the host can queue the next frame while this one finishes */
	if (!ordered)
	{
		lh2_launch_pack_rows( accumulator.ptr, (float4*)devDst, scrwidth, std::max( 0, tileY0 ), band, stride, rows, {}, stream );
		return;
	}
	/* ordered with a consumer stream (torch's, whose gather reads devDst): the pack waits for the
	   consumer's earlier work on devDst, and the consumer for the pack, through a marker on the
	   consumer stream and the pack launch's own stop event (no marker between the core's kernels);
	   consumer may be the null stream */
	if (!evConsumer) CHK_HIP( hipEventCreateWithFlags( &evConsumer, hipEventDisableTiming ) );
	if (!evPacked) CHK_HIP( hipEventCreate( &evPacked ) );
	CHK_HIP( hipEventRecord( evConsumer, (hipStream_t)consumer ) );
	/* the consumer's earlier work is usually long done (the previous frame's gather): then no wait
	   (a wait packet costs the core stream ~9 us even when its event has completed) */
	if (hipEventQuery( evConsumer ) != hipSuccess) CHK_HIP( hipStreamWaitEvent( stream, evConsumer, 0 ) );
	lh2_launch_pack_rows( accumulator.ptr, (float4*)devDst, scrwidth, std::max( 0, tileY0 ), band, stride, rows, { nullptr, evPacked }, stream );
	CHK_HIP( hipStreamWaitEvent( (hipStream_t)consumer, evPacked, 0 ) );
}

void RenderCore::GetFrame( float* hostOut4 )
{
	Synchronize();
	CHK_HIP( hipMemcpy( hostOut4, frame.ptr, sizeof( float4 ) * (size_t)scrwidth * scrheight, hipMemcpyDeviceToHost ) );
}

void RenderCore::TraceClosest( const float* ot, const float* dt, int n, uint32_t* hits4 )
{
	if (geometryDirty || instancesDirty) UpdateToplevel();
	DevBuf<float4> o, d; DevBuf<uint4> h; DevBuf<int> gs; DevBuf<uint32_t> ovf;
	o.upload( (const float4*)ot, n, stream ), d.upload( (const float4*)dt, n, stream );
	h.resize( n ), ovf.resize( LH2_CURSOR_WORDS );
	gs.resize( (size_t)(LH2_STACK_TOTAL - LH2_STACK_LDS) * TraceGrid() * 256 );
	CHK_HIP( hipMemsetAsync( ovf.ptr, 0, sizeof( uint32_t ) * LH2_CURSOR_WORDS, stream ) );
	const SceneDev sd = MakeSceneDev();
	TraceArgs ta{};
	ta.version = TraceVersion();
	ta.rayO = o.ptr, ta.rayD = d.ptr, ta.countFixed = (uint32_t)n, ta.segStride = (uint32_t)((n + LH2_SEGS - 1) / LH2_SEGS), ta.cursor = ovf.ptr, ta.hits = h.ptr, ta.gstack = gs.ptr;
	ta.refill = (uint32_t)(unitCoherent ? refillPrimary : refillOther), ta.leafBatch = (uint32_t)(unitCoherent ? leafBatchPrimary : leafBatch);
	ta.packet = unitCoherent && UsePackets() ? PacketMode() : 0;
	SetTail( ta, grp[0] );
	lh2_launch_trace_closest( &sd, &ta, ta.packet ? PacketGrid() : TraceGrid(), {}, stream );
	CHK_HIP( hipMemcpyAsync( hits4, h.ptr, sizeof( uint4 ) * (size_t)n, hipMemcpyDeviceToHost, stream ) );
	CHK_HIP( hipStreamSynchronize( stream ) );
	CheckSceneError();
}

void RenderCore::TraceAny( const float* ot, const float* dt, int n, uint32_t* occluded )
{
	if (geometryDirty || instancesDirty) UpdateToplevel();
	DevBuf<float4> o, d; DevBuf<uint32_t> m; DevBuf<int> gs; DevBuf<uint32_t> ovf;
	o.upload( (const float4*)ot, n, stream ), d.upload( (const float4*)dt, n, stream );
	const size_t words = ((size_t)n + 63) / 64 * 2;
	m.resize( words ), ovf.resize( LH2_CURSOR_WORDS );
	gs.resize( (size_t)(LH2_STACK_TOTAL - LH2_STACK_LDS) * TraceGrid() * 256 );
	CHK_HIP( hipMemsetAsync( ovf.ptr, 0, sizeof( uint32_t ) * LH2_CURSOR_WORDS, stream ) );
	CHK_HIP( hipMemsetAsync( m.ptr, 0, words * 4, stream ) );
	const SceneDev sd = MakeSceneDev();
	TraceArgs ta{};
	ta.version = TraceVersion();
	ta.rayO = o.ptr, ta.rayD = d.ptr, ta.countFixed = (uint32_t)n, ta.segStride = (uint32_t)((n + LH2_SEGS - 1) / LH2_SEGS), ta.cursor = ovf.ptr, ta.mask = m.ptr, ta.gstack = gs.ptr, ta.refill = (uint32_t)refillOther, ta.leafBatch = (uint32_t)leafBatch;
	ta.packet = unitCoherent && packetShadow ? PacketMode() : 0;
	SetTail( ta, grp[0] );
	lh2_launch_trace_any( &sd, &ta, TraceGrid(), 0, {}, stream );
	std::vector<uint32_t> tmp( words );
	CHK_HIP( hipMemcpyAsync( tmp.data(), m.ptr, words * 4, hipMemcpyDeviceToHost, stream ) );
	CHK_HIP( hipStreamSynchronize( stream ) );
	memcpy( occluded, tmp.data(), ((size_t)n + 31) / 32 * 4 );
	CheckSceneError();
}

void RenderCore::TraceClosestDevice( const void* ro, const void* rd, int n, void* hitsOut, int iterations, float* msOut )
{
	if (geometryDirty || instancesDirty) UpdateToplevel();
	EnsureStack( grp[0] );
	const SceneDev sd = MakeSceneDev();
	DevBuf<uint32_t> cursors;
	cursors.resize( (size_t)std::max( 1, iterations ) * LH2_CURSOR_WORDS );
	CHK_HIP( hipMemsetAsync( cursors.ptr, 0, sizeof( uint32_t ) * (size_t)std::max( 1, iterations ) * LH2_CURSOR_WORDS, stream ) );
#ifdef LH2_TRACE_STATS
	DevBuf<unsigned long long> tstats;
	tstats.resize( LH2_TSTAT_N );
	CHK_HIP( hipMemsetAsync( tstats.ptr, 0, sizeof( unsigned long long ) * LH2_TSTAT_N, stream ) );
#endif
#ifdef LH2_TRACE_TIMES
	DevBuf<unsigned long long> ttimes;
	ttimes.resize( (size_t)std::max( TraceGrid(), PacketGrid() ) * 4 * 4 );
#endif
	/* each launch timed by its own dispatch-recorded start / stop events: msOut is the mean kernel
	   duration, launch gaps excluded (as rocprofv3 --kernel-trace reports it) */
	std::vector<hipEvent_t> ev( 2 * (size_t)std::max( 1, iterations ) );
	for (auto& e : ev) CHK_HIP( hipEventCreate( &e ) );
	for (int i = 0; i < iterations; i++)
	{
		TraceArgs ta{};
		ta.version = TraceVersion();
		ta.rayO = (const float4*)ro, ta.rayD = (const float4*)rd, ta.countFixed = (uint32_t)n, ta.segStride = (uint32_t)((n + LH2_SEGS - 1) / LH2_SEGS), ta.cursor = cursors.ptr + (size_t)i * LH2_CURSOR_WORDS;
		ta.hits = (uint4*)hitsOut, ta.gstack = grp[0].gstack.ptr;
		/* unitCoherent: trace as the frame traces its (tiled) primary rays */
		ta.refill = (uint32_t)(unitCoherent ? refillPrimary : refillOther), ta.leafBatch = (uint32_t)(unitCoherent ? leafBatchPrimary : leafBatch);
		ta.packet = unitCoherent && UsePackets() ? PacketMode() : 0;
#ifdef LH2_TRACE_STATS
		ta.stats = tstats.ptr;
#endif
#ifdef LH2_TRACE_TIMES
		ta.stats = ttimes.ptr;
#endif
		SetTail( ta, grp[0] );
		lh2_launch_trace_closest( &sd, &ta, ta.packet ? PacketGrid() : TraceGrid(), { ev[2 * i], ev[2 * i + 1] }, stream );
	}
	CHK_HIP( hipStreamSynchronize( stream ) );
#ifdef LH2_TRACE_TIMES
	{
		/* the last launch's per-wave times: tools/trace_times.py reads this binary dump */
		std::vector<unsigned long long> h( ttimes.count );
		CHK_HIP( hipMemcpy( h.data(), ttimes.ptr, h.size() * 8, hipMemcpyDeviceToHost ) );
		if (const char* path = getenv( "LH2_TRACE_TIMES_OUT" ))
			if (FILE* f = fopen( path, "wb" )) { fwrite( h.data(), 8, h.size(), f ); fclose( f ); }
	}
#endif
#ifdef LH2_TRACE_STATS
	{
		unsigned long long h[LH2_TSTAT_N];
		CHK_HIP( hipMemcpy( h, tstats.ptr, sizeof( h ), hipMemcpyDeviceToHost ) );
		fprintf( stderr, "LH2_TRACE_STATS {\"rays\": %d, \"launches\": %d, \"c\": [", n, iterations );
		for (int i = 0; i < LH2_TSTAT_N; i++) fprintf( stderr, "%s%llu", i ? ", " : "", h[i] );
		fprintf( stderr, "]}\n" );
	}
#endif
	double total = 0;
	for (int i = 0; i < iterations; i++) { float t = 0; CHK_HIP( hipEventElapsedTime( &t, ev[2 * i], ev[2 * i + 1] ) ); total += t; }
	if (msOut) *msOut = (float)(total / std::max( 1, iterations ));
	CheckSceneError();
	for (auto& e : ev) (void)hipEventDestroy( e );
}

void RenderCore::GenerateEyeRays( const lh2_ViewPyramid& view, uint32_t R0, int pass, float* ot, float* dt, float* st )
{
	const int n = scrwidth * scrheight * scrspp;
	DevBuf<float4> o, d, t4, q4;
	o.resize( n ), d.resize( n ), t4.resize( n ), q4.resize( n );
	CameraParams cp{};
	cp.pos = view.pos, cp.p1 = view.p1;
	cp.right = { view.p2.x - view.p1.x, view.p2.y - view.p1.y, view.p2.z - view.p1.z };
	cp.up = { view.p3.x - view.p1.x, view.p3.y - view.p1.y, view.p3.z - view.p1.z };
	cp.aperture = view.aperture, cp.distortion = view.distortion, cp.geometryEpsilon = geometryEpsilon;
	cp.w = scrwidth, cp.h = scrheight, cp.pass = pass, cp.R0 = R0;
	cp.y0 = 0, cp.tileRows = scrheight, cp.band = scrheight, cp.bandStride = scrheight, cp.tiled = 0, cp.primeRef = primeRef;
	lh2_launch_camera( &cp, dBlueNoise.ptr, o.ptr, d.ptr, t4.ptr, q4.ptr, n, {}, stream );
	std::vector<float4> T( n ), Q( n );
	CHK_HIP( hipMemcpyAsync( ot, o.ptr, sizeof( float4 ) * n, hipMemcpyDeviceToHost, stream ) );
	CHK_HIP( hipMemcpyAsync( dt, d.ptr, sizeof( float4 ) * n, hipMemcpyDeviceToHost, stream ) );
	CHK_HIP( hipMemcpyAsync( T.data(), t4.ptr, sizeof( float4 ) * n, hipMemcpyDeviceToHost, stream ) );
	CHK_HIP( hipMemcpyAsync( Q.data(), q4.ptr, sizeof( float4 ) * n, hipMemcpyDeviceToHost, stream ) );
	CHK_HIP( hipStreamSynchronize( stream ) );
	for (int i = 0; i < n; i++) memcpy( st + i * 8, &T[i], 16 ), memcpy( st + i * 8 + 4, &Q[i], 16 );
}

void RenderCore::SceneInfo( int* nodeCount, int* triCount, int* maxDepth, int* instCount )
{
	if (geometryDirty || instancesDirty) UpdateToplevel();
	if (nodeCount) *nodeCount = blasNodeCount;
	if (triCount) *triCount = blasMeshTris;
	if (tlasOnDevice)
	{
		int d = 0;
		CHK_HIP( hipMemcpyAsync( &d, dTlasDepth.ptr, sizeof( int ), hipMemcpyDeviceToHost, stream ) );
		CHK_HIP( hipStreamSynchronize( stream ) );
		sceneMaxDepth = d + maxBlasDepth;
	}
	if (maxDepth) *maxDepth = sceneMaxDepth;
	if (instCount) *instCount = (int)instances.size();
}

void RenderCore::Shutdown()   /* rendercore.cpp:615-650 */
{
	if (!initialized) return;
	(void)hipStreamSynchronize( stream );
	for (auto* m : meshes) delete m;
	meshes.clear();
	instances.clear();
	for (int gi = 0; gi < LH2_MAX_GROUPS; gi++)
	{
		PathGroup& g = grp[gi];
		if (g.ownStream) (void)hipStreamSynchronize( g.st );
		for (auto& e : g.evTrace) (void)hipEventDestroy( e ), e = nullptr;
		for (auto& e : g.evShade) (void)hipEventDestroy( e ), e = nullptr;
		for (auto& e : g.evShadowB) (void)hipEventDestroy( e ), e = nullptr;
		for (auto& e : g.evCount) (void)hipEventDestroy( e ), e = nullptr;
		for (hipEvent_t* e : { &g.evCamera, &g.evShadow, &g.evDone }) { if (*e) (void)hipEventDestroy( *e ); *e = nullptr; }
		if (g.activeLog) (void)hipHostFree( g.activeLog );
		g.activeLog = nullptr;
		if (g.ownStream) (void)hipStreamDestroy( g.st );
		g.st = nullptr, g.ownStream = false;
	}
	if (evFork) (void)hipEventDestroy( evFork );
	evFork = nullptr;
	for (hipEvent_t* e : { &evConsumer, &evPacked }) { if (*e) (void)hipEventDestroy( *e ); *e = nullptr; }
	for (auto& e : evFrame) (void)hipEventDestroy( e );
	for (auto& e : evStage) (void)hipEventDestroy( e );
	for (int i = 0; i < 2; i++) { if (stage[i]) (void)hipHostFree( stage[i] ); stage[i] = nullptr, stageBytes[i] = 0; }
	if (glResource) (void)hipGraphicsUnregisterResource( glResource );
	glResource = nullptr, glTexture = 0;
	if (hostStats) (void)hipHostFree( hostStats );
	hostStats = nullptr;
	(void)hipStreamDestroy( stream );
	stream = nullptr;
	initialized = false;
}

}  // namespace lh2
