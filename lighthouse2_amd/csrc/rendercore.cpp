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
#include <atomic>
#include <functional>
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
	/* the core, side and ahead streams at the device's least priority, which on MI355X (range 0 .. -1) is the default level:
	   the high level for the ahead stream or the core stream measured no faster (profiles/r04k_ab.txt, r04l_ab.txt) */
	{
		int least = 0, greatest = 0;
		CHK_HIP( hipDeviceGetStreamPriorityRange( &least, &greatest ) );
		CHK_HIP( hipStreamCreateWithPriority( &stream, hipStreamNonBlocking, least ) );
		CHK_HIP( hipStreamCreateWithPriority( &sideStream, hipStreamNonBlocking, least ) );
		CHK_HIP( hipStreamCreateWithPriority( &aheadStream, hipStreamNonBlocking, least ) );
	}
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
	traceBlocksPerCU7 = std::max( 1, std::min( 8, lh2_trace_blocks_per_cu( 7 ) ) );
	traceBlocksPerCU8 = std::max( 1, std::min( 8, lh2_trace_blocks_per_cu( 8 ) ) );
	maxBlocksPerCU = std::max( traceBlocksPerCU7, traceBlocksPerCU8 );
	blocksPerCU = traceWaves == 7 ? traceBlocksPerCU7 : traceBlocksPerCU8;
	packetBlocksPerCU = std::max( 1, std::min( 8, lh2_packet_blocks_per_cu() ) );
	pathBlocksPerCU = std::max( 1, std::min( 8, lh2_path_blocks_per_cu( 3 ) ) );
	pathBlocksPerCU4 = std::max( 1, std::min( 8, lh2_path_blocks_per_cu( 4 ) ) );
	ps.counters.resize( 2 );
	CHK_HIP( hipMemsetAsync( ps.counters.ptr, 0, sizeof( Counters ) * 2, stream ) );
	ps.cursors.resize( 2 * (size_t)LH2_CURSOR_SLOTS * LH2_CURSOR_WORDS );
	CHK_HIP( hipMemsetAsync( ps.cursors.ptr, 0, sizeof( uint32_t ) * 2 * (size_t)LH2_CURSOR_SLOTS * LH2_CURSOR_WORDS, stream ) );
	ps.rayLog.resize( 2 * LH2_RAYLOG );
	CHK_HIP( hipMemsetAsync( ps.rayLog.ptr, 0, sizeof( uint32_t ) * 2 * LH2_RAYLOG, stream ) );
	/* indexed by pathLength; written by advance_bounce (system scope) */
	CHK_HIP( hipHostMalloc( (void**)&ps.activeLog, sizeof( uint32_t ) * (LH2_MAX_BOUNCES + 8), hipHostMallocCoherent ) );
	for (auto& e : ps.evTrace) CHK_HIP( hipEventCreate( &e ) );
	for (auto& e : ps.evShade) CHK_HIP( hipEventCreate( &e ) );
	for (auto& e : ps.evShadowB) CHK_HIP( hipEventCreate( &e ) );
	for (auto& e : ps.evCount) CHK_HIP( hipEventCreate( &e ) );   /* stop events of launches (LaunchEvents) */
	CHK_HIP( hipEventCreate( &ps.evCamera ) );
	CHK_HIP( hipEventCreate( &ps.evShadow ) );
	CHK_HIP( hipEventCreate( &ps.evSide ) );
	CHK_HIP( hipEventCreateWithFlags( &ps.evEarlyEnd, hipEventDisableTiming ) );
	ps.shSnap.resize( 2 * LH2_SEGS * LH2_SEGCOUNT_STRIDE );
	CHK_HIP( hipHostMalloc( (void**)&hostStats, sizeof( FrameStats ), hipHostMallocCoherent ) );   /* written by k_finalize (system scope) */
	memset( hostStats, 0, sizeof( FrameStats ) );
	for (auto& e : evFrame) CHK_HIP( hipEventCreate( &e ) );
	for (auto& e : evStage) CHK_HIP( hipEventCreateWithFlags( &e, hipEventDisableTiming ) );
	dSceneError.resize( 2 ), dTlasDepth.resize( 1 ), dBlasQError.resize( 1 );
	CHK_HIP( hipMemsetAsync( dSceneError.ptr, 0, sizeof( int ) * 2, stream ) );
	CHK_HIP( hipEventCreateWithFlags( &evTlasReady, hipEventDisableTiming ) );
	for (auto& e : evTlasFree) CHK_HIP( hipEventCreateWithFlags( &e, hipEventDisableTiming ) );
	CHK_HIP( hipMemsetAsync( dTlasDepth.ptr, 0, sizeof( int ), stream ) );
	CHK_HIP( hipMemsetAsync( dBlasQError.ptr, 0, sizeof( int ), stream ) );
	for (auto& d : dInstDesc)   /* shading reads record 0 for a miss (HitInstance): it always exists */
	{
		d.resize( 1 );
		CHK_HIP( hipMemsetAsync( d.ptr, 0, sizeof( lh2_CoreInstanceDesc ), stream ) );
	}
	CHK_HIP( hipStreamSynchronize( stream ) );
	initialized = true;
}

void RenderCore::SetTarget( uint32_t w, uint32_t h, uint32_t spp )  /* rendercore.cpp:149-209 */
{
	if (spp < 1) spp = 1;
	if ((uint64_t)w * h * spp > (1u << 24)) FatalError( "path index exceeds 24 bits (camera.h:92): %ux%u x %u spp", w, h, spp );
	scrwidth = (int)w, scrheight = (int)h, scrspp = (int)spp;
	sceneVersion++;
	EnsureBuffers();
	CHK_HIP( hipMemsetAsync( accumulator.ptr, 0, sizeof( float4 ) * (size_t)w * h, stream ) );
	CHK_HIP( hipMemsetAsync( delta.ptr, 0, sizeof( float4 ) * 2 * (size_t)w * h, stream ) );
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
	return bytes <= kPacketMaxBytes;
}

/* traversal loop of the per-ray launches (setting "traceVersion"): 7, the BVH4 loop (lh2_trace4d.inc), unless
   the BVH4 is not built (setting "bvh4" 0) or the reference BVH2 loop is asked for (1) */
int RenderCore::TraceVersion() const { return (traceVersion == 1 || !bvh4) ? 1 : 7; }

void RenderCore::EnsureBuffers()
{
	accumulator.resize( (size_t)scrwidth * scrheight );
	frame.resize( (size_t)scrwidth * scrheight );
	delta.resize( 2 * (size_t)scrwidth * scrheight );   /* per frame parity: the next frame's first shade may run beside this finalize */
}

/* path buffers for `paths` paths (a bit extra, as the reference reserves, and room for LH2_SEGS segments
   of ceil(paths / LH2_SEGS)); shadow rays: 2 per path */
void RenderCore::EnsurePaths( uint32_t paths )
{
	if ((size_t)paths + 64 > ps.cap)
	{
		ps.cap = (size_t)paths + (paths >> 4) + 64;
		for (int i = 0; i < 2; i++) ps.rayO[i].resize( ps.cap ), ps.rayD[i].resize( ps.cap ), ps.T4[i].resize( ps.cap ), ps.Q4[i].resize( ps.cap );
		ps.hits.resize( ps.cap );
		for (int i = 0; i < 2; i++) ps.rayOP[i].resize( ps.cap ), ps.rayDP[i].resize( ps.cap ), ps.T4P[i].resize( ps.cap ), ps.Q4P[i].resize( ps.cap ), ps.hitsP[i].resize( ps.cap );
		ps.relaid = true;
		/* shadow rays: 2 per path, per frame parity */
		ps.shCap = 2 * ps.cap, ps.shMaskWords = (ps.shCap + 63) / 32 + 2;
		ps.shO.resize( 2 * ps.shCap ), ps.shD.resize( 2 * ps.shCap ), ps.shP.resize( 2 * ps.shCap );
		ps.shMask.resize( 2 * ps.shMaskWords );
	}
	EnsureStack();
}

void RenderCore::EnsureStack()
{
	/* sized for the largest grid traceBlocksPerCU / traceWaves may select later */
	const size_t need = (size_t)(LH2_STACK_TOTAL - LH2_STACK_LDS) * smCount * maxBlocksPerCU * 256;
	if (ps.gstack.count < need) ps.gstack.resize( need );
	if (shadowOverlap && ps.sideStack.count < need) ps.sideStack.resize( need );
	if (cameraFused && kCamAhead && ps.aheadStack.count < need) ps.aheadStack.resize( need );
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
	else if (!strcmp( name, "refill" )) refillOther = std::min( 64, std::max( 1, (int)value ) );
	/* traversal: test parked BLAS leaves once this many lanes of a wave hold one (0 = every step) */
	else if (!strcmp( name, "leafBatch" )) leafBatch = std::min( 64, std::max( 0, (int)value ) );
	/* BLAS build parameters, used by later SetGeometry calls */
	else if (!strcmp( name, "bvhMaxLeaf" )) bvhMaxLeaf = std::min( 16, std::max( 1, (int)value ) );
	else if (!strcmp( name, "bvhSpatial" )) bvhSpatial = std::max( 0.0f, value );   /* SBVH overlap threshold (x root area); 0: off */
	else if (!strcmp( name, "bvhSpatialBudget" )) bvhSpatialBudget = std::min( 4.0f, std::max( 0.0f, value ) );
	else if (!strcmp( name, "bvhSpatialMinRefs" )) bvhSpatialMinRefs = std::max( 0, (int)value );
	else if (!strcmp( name, "bvh4Collapse" )) bvh4Collapse = value != 0;
	else if (!strcmp( name, "bvh4" )) { bvh4 = value != 0; }   /* before SetGeometry */
	else if (!strcmp( name, "gpuBuild" )) gpuBuild = value != 0;          /* BLAS builder of later SetGeometry calls */
	else if (!strcmp( name, "buildThreads" )) buildThreads = std::max( 0, (int)value );   /* host threads of the deferred CPU builds */
	else if (!strcmp( name, "gpuTlas" )) { gpuTlas = value != 0; instancesDirty = true; }
	else if (!strcmp( name, "chordSplit" )) chordSplit = std::max( 0.0f, value );   /* two-ended path segments (longest first); 0: off */
	else if (!strcmp( name, "packetHeavy" )) packetHeavy = value < 0 ? -1.0f : value;   /* heavy-first primary packets; 0: off; -1: by frame */
	else if (!strcmp( name, "pathTail" )) pathTail = std::max( 0, (int)value );   /* bounces from this one in one trace-and-shade launch; 0: off */
	else if (!strcmp( name, "pathTailBatch" )) pathTailBatch = std::min( 64, std::max( 1, (int)value ) );
	else if (!strcmp( name, "shadowOverlap" )) shadowOverlap = value != 0;
	else if (!strcmp( name, "cameraFused" )) cameraFused = value != 0;
	else if (!strcmp( name, "frameOverlap" )) frameOverlap = (int)value;
	else if (!strcmp( name, "earlyShade" )) earlyShade = value != 0;
	else if (!strcmp( name, "sideBlocks" )) sideBlocks = std::min( 8, std::max( -1, (int)value ) );
	else if (!strcmp( name, "pathTailBlocks" )) pathTailBlocks = std::min( 8, std::max( 0, (int)value ) );
	else if (!strcmp( name, "shadeBlocks" )) shadeBlocks = std::min( 64, std::max( 0, (int)value ) );
	else if (!strcmp( name, "finalShadowBlocks" )) finalShadowBlocks = std::min( 8, std::max( 0, (int)value ) );
	else if (!strcmp( name, "pathTailWaves" )) pathTailWaves = std::min( 4, std::max( 0, (int)value ) );
	/* packet traversal of tiled primary rays: 1 on, 0 off, -1 when the BVH + triangles fit in packetMaxMB */
	else if (!strcmp( name, "packetPrimary" )) packetPrimary = value < 0 ? -1 : value != 0;
	else if (!strcmp( name, "singleInstanceStart" )) singleInstanceStart = value != 0;   /* one instance: rays start at its TLAS leaf */
	else if (!strcmp( name, "terminalShade" )) terminalShade = value != 0;   /* drop hits that cannot contribute before shading them (ShadeParams::terminal) */
	else if (!strcmp( name, "traceBlocksPerCU" ))   /* persistent trace grid: blocks per CU (0: the launched variant's occupancy) */
	{
		userBlocksPerCU = value > 0 ? std::min( maxBlocksPerCU, std::max( 1, (int)value ) ) : 0;
		blocksPerCU = userBlocksPerCU ? userBlocksPerCU : traceWaves == 7 ? traceBlocksPerCU7 : traceBlocksPerCU8;
	}
	else if (!strcmp( name, "unitTraceWaves" )) unitTraceWaves = (int)value == 8 ? 8 : 7;   /* the same for the unit queries (TraceClosest*) */
	else if (!strcmp( name, "traceWaves" ))   /* closest-hit kernel variant (7 or 8 waves per SIMD; 0: by scene); resets traceBlocksPerCU */
	{
		traceWaves = (int)value == 7 ? 7 : (int)value == 8 ? 8 : 0;
		userBlocksPerCU = 0;
		blocksPerCU = traceWaves == 7 ? traceBlocksPerCU7 : traceBlocksPerCU8;
	}
	else if (!strcmp( name, "unitCoherent" )) unitCoherent = value != 0;   /* TraceClosestDevice traces as the frame traces primary rays */
	else if (!strcmp( name, "traceVersion" )) traceVersion = (int)value == 1 ? 1 : 0;   /* 1: the reference BVH2 loop; else the BVH4 loop */
	/* other names ("clampDirect", "filter", "TAA", ...) are ignored, as in the reference */
}

/* the current value of a setting (extension: the reference has no getter); false for unknown names */
bool RenderCore::GetSetting( const char* name, float& value ) const
{
	struct { const char* n; float v; } t[] = {
		{ "epsilon", geometryEpsilon }, { "clampValue", clampValue }, { "maxPathLength", (float)maxPathLength },
		{ "primeRef", (float)primeRef }, { "tiledRays", (float)tiledRays }, { "refill", (float)refillOther }, { "leafBatch", (float)leafBatch },
		{ "bvhMaxLeaf", (float)bvhMaxLeaf }, { "bvhSpatial", bvhSpatial }, { "bvhSpatialBudget", bvhSpatialBudget }, { "bvhSpatialMinRefs", (float)bvhSpatialMinRefs },
		{ "bvh4Collapse", (float)bvh4Collapse }, { "bvh4", (float)bvh4 }, { "gpuBuild", (float)gpuBuild }, { "buildThreads", (float)buildThreads }, { "gpuTlas", (float)gpuTlas },
		{ "chordSplit", chordSplit }, { "packetHeavy", packetHeavy }, { "pathTail", (float)pathTail }, { "pathTailBatch", (float)pathTailBatch },
		{ "shadowOverlap", (float)shadowOverlap }, { "cameraFused", (float)cameraFused }, { "frameOverlap", (float)frameOverlap }, { "earlyShade", (float)earlyShade },
		{ "sideBlocks", (float)sideBlocks }, { "pathTailBlocks", (float)pathTailBlocks }, { "shadeBlocks", (float)shadeBlocks }, { "finalShadowBlocks", (float)finalShadowBlocks },
		{ "pathTailWaves", (float)pathTailWaves }, { "packetPrimary", (float)packetPrimary }, { "singleInstanceStart", (float)singleInstanceStart },
		{ "terminalShade", (float)terminalShade }, { "traceBlocksPerCU", (float)ClosestBlocksPerCU( ScenePicksWaves() ) }, { "unitTraceWaves", (float)unitTraceWaves }, { "traceWaves", (float)traceWaves },
		{ "unitCoherent", (float)unitCoherent }, { "traceVersion", (float)TraceVersion() },
		{ "usePackets", (float)UsePackets() }, { "blasBuilds", (float)BlasBuildCount() } };
	for (const auto& e : t) if (!strcmp( name, e.n )) { value = e.v; return true; }
	return false;
}

void RenderCore::SetTextures( const lh2_CoreTexDesc* tex, int textureCount )   /* rendercore.cpp:276-292 */
{
	sceneVersion++;   /* device-resident scene data: the next fused frame's primary launch waits for the previous frame */
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
	sceneVersion++;   /* device-resident scene data: the next fused frame's primary launch waits for the previous frame */
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
	sceneVersion++;
	dArea.upload( a, na, stream ), dPoint.upload( p, np, stream ), dSpot.upload( s, ns, stream ), dDir.upload( d, nd, stream );
	dArea.resize( 1 ), dPoint.resize( 1 ), dSpot.resize( 1 ), dDir.resize( 1 );
	nArea = na, nPoint = np, nSpot = ns, nDir = nd;
	CHK_HIP( hipStreamSynchronize( stream ) );
}

void RenderCore::SetSkyData( const float* pixels, uint32_t width, uint32_t height )   /* rendercore.cpp:425-433 */
{
	sceneVersion++;   /* device-resident scene data: the next fused frame's primary launch waits for the previous frame */
	dSky.upload( pixels, (size_t)width * height * 3, stream );
	dSky.resize( 1 );
	skyW = (int)width, skyH = (int)height;
	CHK_HIP( hipStreamSynchronize( stream ) );
}

static std::atomic<int> gBlasBuilds{ 0 };
int RenderCore::BlasBuildCount() { return gBlasBuilds.load(); }
void HostBlas::Run( int threads )
{
	std::call_once( once, [&] { job( *this, threads ); job = nullptr; gBlasBuilds++; } );
}

void RenderCore::SetGeometry( int meshIdx, const float*, int, int triangleCount, const lh2_CoreTri* tris, const uint32_t* )
{
	sceneVersion++;
	/* rendercore.cpp:215-223 + core_mesh.cpp:36-67: meshes arrive first-time in sequential order */
	if (meshIdx < 0 || meshIdx > (int)meshes.size()) FatalError( "SetGeometry: mesh index %d out of sequence", meshIdx );
	if (meshIdx == (int)meshes.size()) meshes.push_back( new CoreMeshHost() );
	CoreMeshHost& m = *meshes[meshIdx];
	m.build = nullptr;   /* a build of earlier data not run yet is superseded */
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
		SyncTlas();   /* a TLAS build queued on the ahead stream uses the same builder scratch: this build follows it */
		gpuBvh.BuildBlas( m.shadeTris.ptr, triangleCount, bvhMaxLeaf, 1.0f, &nodes, &tris48, r, stream );
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
		/* CPU binned-SAH build (bvh_build.cpp), deferred: the inputs are copied now (the caller's triangle
		   array is borrowed for this call only) and the builds of all meshes set since the last one run in
		   parallel over the meshes when the scene is first needed (FlushBuilds) */
		std::vector<Aabb> prims( triangleCount );
		std::vector<float> verts( (size_t)triangleCount * 9 );
		for (int k = 0; k < 3; k++) m.aabbLo[k] = 1e30f, m.aabbHi[k] = -1e30f;
		for (int i = 0; i < triangleCount; i++)
		{
			const lh2_CoreTri& t = tris[i];
			const float v[9] = { t.vertex0.x, t.vertex0.y, t.vertex0.z, t.vertex1.x, t.vertex1.y, t.vertex1.z, t.vertex2.x, t.vertex2.y, t.vertex2.z };
			memcpy( &verts[(size_t)i * 9], v, sizeof( v ) );
			for (int k = 0; k < 3; k++)
			{
				prims[i].lo[k] = std::min( std::min( v[k], v[3 + k] ), v[6 + k] );
				prims[i].hi[k] = std::max( std::max( v[k], v[3 + k] ), v[6 + k] );
				m.aabbLo[k] = std::min( m.aabbLo[k], prims[i].lo[k] ), m.aabbHi[k] = std::max( m.aabbHi[k], prims[i].hi[k] );
			}
		}
		const int maxLeaf = bvhMaxLeaf, collapse = bvh4Collapse, wide = bvh4;
		const float cost = 1.0f, spatial = bvhSpatial, budget = bvhSpatialBudget;
		const int minRefs = bvhSpatialMinRefs;
		m.build = std::make_shared<HostBlas>();
		m.build->job = [prims = std::move( prims ), verts = std::move( verts ), maxLeaf, collapse, wide, cost, spatial, budget, minRefs]( HostBlas& r, int threads ) {
			BvhOutput bvh;
			BuildBvh2( prims, maxLeaf, threads, bvh, cost, 0, spatial > 0 ? verts.data() : nullptr, spatial, budget, minRefs );
			/* one triangle record per leaf slot (a spatial split can reference a triangle from several leaves):
			   v0, e1 = v1 - v0, e2 = v2 - v0 in fp32, exactly as the oracle's intersect_tri */
			std::vector<float>& t48 = r.tris48;
			t48.assign( std::max<size_t>( bvh.perm.size(), 1 ) * 12, 0.0f );
			for (size_t j = 0; j < bvh.perm.size(); j++)
			{
				const uint32_t ti = bvh.perm[j];
				const float* v = &verts[(size_t)ti * 9];
				float* o = &t48[j * 12];
				o[0] = v[0], o[1] = v[1], o[2] = v[2]; memcpy( &o[3], &ti, 4 );
				o[4] = v[3] - v[0], o[5] = v[4] - v[1], o[6] = v[5] - v[2], o[7] = 0;
				o[8] = v[6] - v[0], o[9] = v[7] - v[1], o[10] = v[8] - v[2], o[11] = 0;
			}
			r.leafTris = (int)bvh.perm.size();
			r.nodeCount = (int)(bvh.nodes.size() / 16), r.maxDepth = bvh.maxDepth;
			r.nodes4.clear(), r.depth4 = 0;
			/* BVH4 collapse: dynamic programming (surface-area costs: node step 1, leaf visit 0.4, triangle test 0.5,
			   one triangle per leaf; merged leaves run the leaf loop divergent: slower, r02s) or greedy */
			if (wide) r.depth4 = collapse ? CollapseBvh4Sah( bvh.nodes.data(), (size_t)r.nodeCount, r.nodes4, 0.4f, 0.5f, 1 )
				: CollapseBvh4( bvh.nodes.data(), (size_t)r.nodeCount, r.nodes4 );
			r.nodes2 = std::move( bvh.nodes );
		};
		pendingBuilds = true;
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

/* the deferred CPU BLAS builds (SetGeometry), in parallel over the meshes on up to `buildThreads` host threads
   (a mesh's own build gets the threads left over when there are fewer meshes than threads), then their upload */
void RenderCore::FlushBuilds()
{
	if (!pendingBuilds) return;
	pendingBuilds = false;
	const auto t0 = std::chrono::high_resolution_clock::now();
	std::vector<CoreMeshHost*> jobs;
	for (auto* m : meshes) if (m->build) jobs.push_back( m );
	int workers = buildThreads;
	if (workers <= 0)
	{
		const char* e = getenv( "LH2_BUILD_THREADS" );
		if (!e) e = getenv( "OMP_NUM_THREADS" );
		const unsigned hw = std::thread::hardware_concurrency();
		workers = e && atoi( e ) > 0 ? atoi( e ) : (int)std::min( 16u, hw ? hw : 4u );
	}
	const int nthreads = std::max( 1, std::min( workers, (int)jobs.size() ) );
	const int perJob = std::max( 1, workers / std::max( 1, (int)jobs.size() ) );
	std::atomic<int> next{ 0 }, inUse{ 0 };
	std::vector<std::string> errors( nthreads );
	/* the last jobs, fewer than the workers, get the idle workers' share as threads of their own build (SBVH subtrees):
	   a job is granted threads only out of those no running build holds, so the total stays near `workers` */
	auto work = [&]( int w ) {
		try
		{
			for (int j; (j = next.fetch_add( 1 )) < (int)jobs.size();)
			{
				const int remaining = (int)jobs.size() - j;
				const int want = std::max( perJob, std::min( 8, workers / std::max( 1, remaining ) ) );
				/* reserve the grant atomically out of the threads no running build holds (one at least: this worker's own) */
				int held = inUse.load(), grant = 1;
				do grant = std::max( 1, std::min( want, workers - held ) );
				while (!inUse.compare_exchange_weak( held, held + grant ));
				jobs[j]->build->Run( grant );
				inUse -= grant;
			}
		}
		catch (const std::exception& e) { errors[w] = e.what(); }
	};
	std::vector<std::thread> pool;
	for (int w = 1; w < nthreads; w++) pool.emplace_back( work, w );
	work( 0 );
	for (auto& t : pool) t.join();
	for (auto& e : errors) if (!e.empty()) FatalError( "BLAS build: %s", e.c_str() );
	for (auto* m : jobs)
	{
		const HostBlas& r = *m->build;
		m->leafTris = r.leafTris, m->nodeCount = r.nodeCount, m->maxDepth = r.maxDepth, m->depth4 = r.depth4;
		m->bvhNodes.upload( (const float4*)r.nodes2.data(), r.nodes2.size() / 4, stream );
		m->bvhTris.upload( (const float4*)r.tris48.data(), r.tris48.size() / 4, stream );
		if (bvh4) m->bvh4Nodes.upload( (const float4*)r.nodes4.data(), r.nodes4.size() / 4, stream ), m->node4Count = (int)(r.nodes4.size() / 32);
		CHK_HIP( hipStreamSynchronize( stream ) );
		m->build.reset();   /* the last core to upload a shared build frees its host arrays */
	}
	coreStats.bvhBuildTime += std::chrono::duration<float>( std::chrono::high_resolution_clock::now() - t0 ).count();
}

/* MultiDevice's sub-cores: the mesh of src (core 0, which has just taken it through SetGeometry), its shading triangles
   uploaded to this device, its deferred CPU build shared (run once by the first core to flush, uploaded by each).  A GPU
   build (gpuBuild), or a mesh src has already uploaded, is built here as SetGeometry builds it */
void RenderCore::AdoptGeometry( int meshIdx, int triangleCount, const lh2_CoreTri* tris, const RenderCore& src )
{
	const CoreMeshHost* sm = meshIdx >= 0 && meshIdx < (int)src.meshes.size() ? src.meshes[meshIdx] : nullptr;
	if (!sm || !sm->build || sm->triCount != triangleCount || bvh4 != src.bvh4)
	{
		SetGeometry( meshIdx, nullptr, 0, triangleCount, tris, nullptr );
		return;
	}
	sceneVersion++;
	if (meshIdx < 0 || meshIdx > (int)meshes.size()) FatalError( "SetGeometry: mesh index %d out of sequence", meshIdx );
	if (meshIdx == (int)meshes.size()) meshes.push_back( new CoreMeshHost() );
	CoreMeshHost& m = *meshes[meshIdx];
	const auto t0 = std::chrono::high_resolution_clock::now();
	m.triCount = triangleCount;
	m.shadeTris.upload( (const float4*)tris, (size_t)triangleCount * 11, stream );
	m.shadeTris.resize( 11 );
	for (int k = 0; k < 3; k++) m.aabbLo[k] = sm->aabbLo[k], m.aabbHi[k] = sm->aabbHi[k];
	m.build = sm->build;
	pendingBuilds = true;
	CHK_HIP( hipStreamSynchronize( stream ) );   /* the caller's triangle array is borrowed for this call only */
	geometryDirty = true;
	coreStats.bvhBuildTime += std::chrono::duration<float>( std::chrono::high_resolution_clock::now() - t0 ).count();
}

#ifdef LH2_TOUCH
/* the unique records one closest-hit launch reads (diagnostic build): quantized BVH4 nodes (64 B) and leaf triangle records
   (48 B), one bit each, counted after the launch; one JSON line per launch on stderr.  The launch is serialised with the
   count (the build is for this count, not for timing) */
void RenderCore::TouchBegin()
{
	CHK_HIP( hipDeviceSynchronize() );   /* nothing in flight reads the bitmap pointer while it changes */
	const uint32_t nodeWords = (uint32_t)(((size_t)blasNode4Count + 2 * tlasCapacity + 31) / 32), triWords = (uint32_t)(((size_t)blasTriCount + 31) / 32);
	touchMap.resize( (size_t)nodeWords + triWords );
	CHK_HIP( hipMemsetAsync( touchMap.ptr, 0, sizeof( uint32_t ) * ((size_t)nodeWords + triWords), stream ) );
	lh2_touch_set( touchMap.ptr, nodeWords, nodeWords + triWords );
	touchNodeWords = nodeWords;
}
void RenderCore::TouchReport( int pathLength )
{
	CHK_HIP( hipDeviceSynchronize() );
	std::vector<uint32_t> h( touchMap.count );
	CHK_HIP( hipMemcpy( h.data(), touchMap.ptr, sizeof( uint32_t ) * h.size(), hipMemcpyDeviceToHost ) );
	uint64_t nodes = 0, tris = 0;
	for (size_t i = 0; i < h.size(); i++) (i < touchNodeWords ? nodes : tris) += (uint64_t)__builtin_popcount( h[i] );
	fprintf( stderr, "LH2_TOUCH {\"pathLength\": %d, \"unique_nodes\": %llu, \"unique_tri_records\": %llu, \"node_bytes\": %llu, "
		"\"tri_bytes\": %llu, \"scene_nodes\": %d, \"scene_tri_records\": %d, \"paths\": %u}\n", pathLength, (unsigned long long)nodes,
		(unsigned long long)tris, (unsigned long long)nodes * 64ull, (unsigned long long)tris * 48ull, blasNode4Count, blasTriCount, ps.count );
	lh2_touch_set( nullptr, 0, 0 );   /* later closest-hit launches (unit queries) record nothing */
}
#endif

void RenderCore::BuildBlas4( CoreMeshHost& m, const float* nodes2 )
{
	std::vector<float> n4;
	/* bvh4Collapse 1: dynamic-programming collapse (surface-area costs, optional leaf merging); 0: greedy */
	/* node step = 1, leaf visit 0.4, triangle test 0.5; one triangle per leaf (merged leaves run the leaf loop
	   divergent: slower, profiles/r02s_ab_collapse_shade4.txt) */
	m.depth4 = bvh4Collapse ? CollapseBvh4Sah( nodes2, (size_t)m.nodeCount, n4, 0.4f, 0.5f, 1 )
		: CollapseBvh4( nodes2, (size_t)m.nodeCount, n4 );
	m.bvh4Nodes.upload( (const float4*)n4.data(), n4.size() / 4, stream );
	m.node4Count = (int)(n4.size() / 32);
}

void RenderCore::SetInstance( int instanceIdx, int meshIdx, const float* M )   /* rendercore.cpp:229-243 */
{
	/* host state only: UpdateToplevel writes it into the TLAS slot no frame in flight reads */
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
	FlushBuilds();
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
	/* frames in flight may still read the old arrays, and a TLAS update may be queued on the ahead stream */
	CHK_HIP( hipStreamSynchronize( stream ) );
	CHK_HIP( hipStreamSynchronize( aheadStream ) );
	dNodes.free(), dTris.free(), dNodes4.free(), dNodes4q.free();
	/* after the BLAS: two TLAS slots of tlasCapacity nodes each (UpdateToplevel) */
	dNodes.resize( ((size_t)nodeTotal + 2 * tlasCapacity) * 4 );
	/* the BVH4 loops address nodes with 32-bit buffer offsets (lh2_trace4d.inc): the array stays below 2 GiB */
	if (bvh4 && ((size_t)node4Total + 2 * tlasCapacity) * 128 > 0x7fffffffull)
		FatalError( "BVH4 of %zu nodes exceeds the 2 GiB the traversal addresses", (size_t)node4Total + 2 * tlasCapacity );
	if (bvh4) dNodes4.resize( ((size_t)node4Total + 2 * tlasCapacity) * 8 ), dNodes4q.resize( ((size_t)node4Total + 2 * tlasCapacity) * 4 );
	dTris.resize( (size_t)std::max( triTotal, 1 ) * 3 );
	/* the TLAS region starts as NaN boxes: a TLAS of fewer nodes than the capacity leaves no uninitialised (possibly huge,
	   finite) boxes behind it for the quantizer's range check (k_quantize4) */
	CHK_HIP( hipMemsetAsync( dNodes.ptr + (size_t)nodeTotal * 4, 0xff, sizeof( float4 ) * 4 * 2 * (size_t)tlasCapacity, stream ) );
	dBlasQError.resize( 1 );
	CHK_HIP( hipMemsetAsync( dBlasQError.ptr, 0, sizeof( int ), stream ) );
	for (size_t mi = 0; mi < meshes.size(); mi++)
	{
		const CoreMeshHost& m = *meshes[mi];
		GpuBvhBuilder::Relocate( m.bvhNodes.ptr, m.nodeCount, meshNodeBase[mi], (uint32_t)meshTriBase[mi], dNodes.ptr, stream );
		if (bvh4) GpuBvhBuilder::Relocate4( m.bvh4Nodes.ptr, m.node4Count, meshNode4Base[mi], (uint32_t)meshTriBase[mi], dNodes4.ptr, stream );
		if (m.leafTris) CHK_HIP( hipMemcpyAsync( dTris.ptr + (size_t)meshTriBase[mi] * 3, m.bvhTris.ptr, sizeof( float4 ) * 3 * (size_t)m.leafTris, hipMemcpyDeviceToDevice, stream ) );
	}
	if (bvh4) GpuBvhBuilder::Quantize4( dNodes4.ptr, 0, node4Total, dNodes4q.ptr, dBlasQError.ptr, stream );
	dMeshBounds.upload( bounds.data(), bounds.size(), stream );
	CHK_HIP( hipStreamSynchronize( stream ) );
	blasNodeCount = nodeTotal, blasTriCount = triTotal, blasNode4Count = node4Total, blasMeshTris = meshTris;
	geometryDirty = false;
}

void RenderCore::UpdateToplevel()   /* rendercore.cpp:250-270 (TLAS) + :481-505 (instance descriptors) */
{
	const int ni = (int)instances.size();
	if (geometryDirty || ni + 1 > tlasCapacity)
	{
		sceneVersion++;   /* new BLAS arrays: the next fused frame's primary launch waits for the previous frame */
		ConcatenateBlas( ni );
	}
	/* the TLAS slot no frame in flight reads (the other one is the last frame's), written on the ahead stream behind the
	   last frame that read it; instance-only updates leave sceneVersion alone, so the next frame may still overlap */
	const int ts = tlasSlot ^ 1;
	hipStream_t us = aheadStream;
	if (tlasFreeValid[ts]) CHK_HIP( hipStreamWaitEvent( us, evTlasFree[ts], 0 ) );
	tlasRoot = TlasBase2( ts );
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
	/* the quantized nodes' origins lie in these boxes (TLAS: world; BLAS: mesh space); 1 % slack for the
	   device-side TLAS bounds' own rounding */
	qBound = 0;
	for (int k = 0; k < 3; k++) qBound = std::max( qBound, std::max( fabsf( sceneLo[k] ), fabsf( sceneHi[k] ) ) );
	for (const auto& m : meshes)
		if (m->triCount) for (int k = 0; k < 3; k++) qBound = std::max( qBound, std::max( fabsf( m->aabbLo[k] ), fabsf( m->aabbHi[k] ) ) );
	qBound = qBound * 1.01f + 1e-30f;
	/* a slot's tables grow only with the work that may read them drained (DevBuf::resize frees the old buffer) */
	if (dInst[ts].count < nRec * sizeof( DevInstance ) || dInstDesc[ts].count < nRec || dInstT.count < nRec * 16 || dInstMesh.count < nRec)
	{
		CHK_HIP( hipStreamSynchronize( stream ) );
		CHK_HIP( hipStreamSynchronize( us ) );
		dInst[ts].resize( nRec * sizeof( DevInstance ) ), dInstDesc[ts].resize( nRec ), dInstT.resize( nRec * 16 ), dInstMesh.resize( nRec );
	}
	CHK_HIP( hipMemcpyAsync( dInst[ts].ptr, di, nRec * sizeof( DevInstance ), hipMemcpyHostToDevice, us ) );
	CHK_HIP( hipMemcpyAsync( dInstDesc[ts].ptr, desc, nRec * sizeof( lh2_CoreInstanceDesc ), hipMemcpyHostToDevice, us ) );
	/* the scene error starts as the BLAS quantizer's (ConcatenateBlas), the TLAS checks add to it */
	CHK_HIP( hipMemcpyAsync( SceneErr( ts ), dBlasQError.ptr, sizeof( int ), hipMemcpyDeviceToDevice, us ) );
	int tlasNodes = 1;   /* the nodes this TLAS has (the slot holds tlasCapacity): the BVH4 copy and the quantizer touch no others */
	if (ni >= 2 && gpuTlas)
	{
		/* TLAS built on the device from the instance transforms (bvh_gpu.h) */
		CHK_HIP( hipMemcpyAsync( dInstT.ptr, Ts, nRec * 64, hipMemcpyHostToDevice, us ) );
		CHK_HIP( hipMemcpyAsync( dInstMesh.ptr, meshIds, nRec * 4, hipMemcpyHostToDevice, us ) );
		GpuTlasArgs ta;
		ta.T = dInstT.ptr, ta.instMesh = dInstMesh.ptr, ta.meshBounds = dMeshBounds.ptr, ta.count = ni;
		ta.nodeBase = TlasBase2( ts ), ta.nodes = dNodes.ptr, ta.maxBlasDepth = StackDepthBound();
		ta.sceneError = SceneErr( ts ), ta.tlasDepth = dTlasDepth.ptr;
		ta.tlasFactor = 1;
		gpuBvh.BuildTlas( ta, us );
		tlasNodes = ni - 1;   /* one instance per leaf: ni - 1 child-pair nodes, dense in preorder (bvh_gpu.hip emit_node) */
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
		tlasNodes = std::max( 1, (int)tn );
		for (size_t k = 0; k < tn; k++)
		{
			int* refs = (int*)&tlas.nodes[k * 16 + 12];
			for (int c = 0; c < 2; c++)
			{
				if (refs[c] >= 0) refs[c] += TlasBase2( ts );
				else if (!prims.empty())
				{
					if (LEAF_COUNT( refs[c] ) != 1) FatalError( "TLAS leaf with %d instances", LEAF_COUNT( refs[c] ) );
					refs[c] = MAKE_LEAF( (uint32_t)primInst[tlas.perm[LEAF_FIRST( refs[c] )]], 1 );
				}
			}
		}
		if (tlas.nodes.size() * sizeof( float ) > need - offNodes) FatalError( "TLAS staging overflow" );
		memcpy( sb + offNodes, tlas.nodes.data(), tlas.nodes.size() * sizeof( float ) );
		CHK_HIP( hipMemcpyAsync( dNodes.ptr + (size_t)TlasBase2( ts ) * 4, sb + offNodes, tlas.nodes.size() * sizeof( float ), hipMemcpyHostToDevice, us ) );
		sceneMaxDepth = tlas.maxDepth + StackDepthBound();
		tlasOnDevice = false;
		if (sceneMaxDepth >= LH2_STACK_TOTAL - 1) FatalError( "BVH depth %d exceeds the traversal stack (%d)", sceneMaxDepth, LH2_STACK_TOTAL );
	}
	/* the TLAS in the BVH4 array: its BVH2 nodes as two-child BVH4 nodes (one short launch), quantized.  Only the nodes this
	   TLAS has: the slot's nodes beyond them hold an earlier, larger TLAS or memory never written, whose boxes (possibly huge,
	   finite) would set the quantizer's range error (round 4 fixed that by NaN-filling the region, 651cce0; no traversal ever
	   reaches such a node, so it is not read at all now; test_gpu_parity.py::test_stale_tlas_region_is_not_quantized) */
	if (bvh4)
	{
		GpuBvhBuilder::TlasToBvh4( dNodes.ptr, TlasBase2( ts ), tlasNodes, TlasBase4( ts ), dNodes4.ptr, us );
		GpuBvhBuilder::Quantize4( dNodes4.ptr, TlasBase4( ts ), tlasNodes, dNodes4q.ptr, SceneErr( ts ), us );
	}
	tlasNodeCount[ts] = tlasNodes;
	CHK_HIP( hipEventRecord( evStage[slot], us ) );
	CHK_HIP( hipEventRecord( evTlasReady, us ) );
	tlasSlot = ts, tlasPending = true;
	instancesDirty = false;
}

/* device-side scene errors (TLAS deeper than the traversal stack): the trace kernels skip the
   frame, and the host reports it here */
#define LH2_STR_( x ) #x
#define LH2_XSTR( x ) LH2_STR_( x )
static const char* SceneErrorText( int e )
{
	if (e & LH2_SCENE_ERR_QRANGE) return "scene extent beyond the quantized BVH4 grid (a node wider than 255 * 2^27 or coordinates beyond 2^55)";
	return "BVH depth exceeds the traversal stack (" LH2_XSTR( LH2_STACK_TOTAL ) " levels)";
}

void RenderCore::CheckSceneError()
{
	if (!dSceneError.ptr) return;
	int e = 0;
	SyncTlas();
	CHK_HIP( hipMemcpyAsync( &hostStats->sceneError, SceneErr( tlasSlot ), sizeof( int ), hipMemcpyDeviceToHost, stream ) );
	CHK_HIP( hipStreamSynchronize( stream ) );
	e = hostStats->sceneError;
	if (e) FatalError( "%s", SceneErrorText( e ) );
}

/* the core stream's next launch reads the TLAS slot the last UpdateToplevel wrote on the ahead stream */
void RenderCore::SyncTlas()
{
	if (!tlasPending) return;
	CHK_HIP( hipStreamWaitEvent( stream, evTlasReady, 0 ) );
	tlasPending = false;
}

SceneDev RenderCore::MakeSceneDev()
{
	SyncTlas();
	SceneDev s;
	s.nodes = dNodes.ptr, s.tris = dTris.ptr, s.inst = (const DevInstance*)dInst[tlasSlot].ptr;
	s.sceneError = SceneErr( tlasSlot );
	s.argb32 = dArgb32.ptr, s.nrm32 = dNrm32.ptr;
	s.argb32Count = (uint32_t)dArgb32.count, s.nrm32Count = (uint32_t)dNrm32.count;
	s.tlasRoot = tlasRoot, s.instCount = (int)instances.size();
	s.nodes4 = dNodes4.ptr, s.nodes4q = dNodes4q.ptr, s.qBound = qBound, s.tlasRoot4 = TlasBase4( tlasSlot );
	/* one instance of a non-empty mesh: rays start at its TLAS leaf (MAKE_LEAF( 0, 1 ) = ~0) and skip
	   the TLAS root's box test, which can only cull (TopLevelBVH::Traverse bvh.cpp:594-649); the
	   instance transform runs as at the leaf, so the hits are unchanged: one loop iteration less per ray */
	s.root40 = 0, s.tris0 = nullptr;
	if (singleInstanceStart && instances.size() == 1 && instances[0].mesh >= 0 && instances[0].mesh < (int)meshes.size() &&
		meshes[instances[0].mesh]->triCount > 0)
	{
		s.tlasRoot = s.tlasRoot4 = ~0;
		s.root40 = bvh4 ? meshNode4Base[instances[0].mesh] : 0;   /* DevInstance::root4 of instance 0 (UpdateToplevel) */
		s.tris0 = meshes[instances[0].mesh]->shadeTris.ptr;       /* lh2_CoreInstanceDesc::triangles of instance 0 */
	}
	s.instDesc = dInstDesc[tlasSlot].ptr, s.materials = dMaterials.ptr;
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
	const uint32_t pathCount = (uint32_t)tileRows * (uint32_t)scrwidth * (uint32_t)scrspp;
	const SceneDev sd = MakeSceneDev();
	const int frameTlas = tlasSlot;   /* the TLAS slot this frame reads (evTlasFree after its finalize) */
	/* the accumulator reset of a restart is folded into the camera launch (each pixel's first sample zeroes
	   it; rows outside this rank's tile stay zero from SetTarget); a changed tile clears the whole frame */
	if (restart && tileChanged) CHK_HIP( hipMemsetAsync( accumulator.ptr, 0, sizeof( float4 ) * (size_t)scrwidth * scrheight, stream ) );
	EnsurePaths( pathCount );
	/* segmented path / ray streams (lh2_kernels.h): LH2_SEGS segments of segStride records; shadow rays in
	   segments of shadowStride */
	ps.count = pathCount;
	ps.segStride = (pathCount + LH2_SEGS - 1) / LH2_SEGS;
	ps.shadowStride = (uint32_t)(ps.shCap / LH2_SEGS);
	ps.pl = 0, ps.tailL = 0;
	/* this frame's parity: its counters, work-queue heads, shadow stream and ray-count log (PathStreams) */
	ps.fp ^= 1;
	Counters* const c = FrameCounters();
	uint32_t* const cursors = FrameCursors();
	uint32_t* const rayLog = FrameRayLog();
	float4* const shO = ps.shO.ptr + (size_t)ps.fp * ps.shCap;
	float4* const shD = ps.shD.ptr + (size_t)ps.fp * ps.shCap;
	float4* const shP = ps.shP.ptr + (size_t)ps.fp * ps.shCap;
	uint32_t* const shMask = ps.shMask.ptr + (size_t)ps.fp * ps.shMaskWords;
	uint32_t* const shSnap = ps.shSnap.ptr + (size_t)ps.fp * LH2_SEGS * LH2_SEGCOUNT_STRIDE;   /* the rays queued before the tail */
	float4* const frameDelta = delta.ptr + (size_t)ps.fp * scrwidth * scrheight;
	/* primary rays (camera.h) for every sample of the tile; the camera launch also resets the frame's
	   counters and work-queue heads (k_init_counters) */
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
	cp.primeRef = primeRef;
	cp.initC = c, cp.cursors = cursors, cp.cursorWords = LH2_CURSOR_SLOTS * LH2_CURSOR_WORDS;
	cp.pathCount = pathCount, cp.segStride = ps.segStride;
	cp.clearAcc = restart && !tileChanged ? accumulator.ptr : nullptr;
	/* heavy-first primary packets: this frame reads the block the previous one recorded, and records into the
	   other one, which the camera launch zeroes (a new layout zeroes both) */
	ps.hvOn = packetHeavy != 0 && tiledRays && UsePackets() && !primeRef;
	if (ps.hvOn)
	{
		const uint32_t cap = (ps.segStride + 63) / 64, maskWords = (LH2_SEGS * cap + 31) / 32;
		if (cap != ps.hvCap)
		{
			ps.hvCap = cap, ps.hvMaskWords = maskWords, ps.hvBlock = LH2_HV_MASK + maskWords + LH2_SEGS * cap, ps.hvParity = 0;
			ps.hv.resize( 2 * (size_t)ps.hvBlock );
			CHK_HIP( hipMemsetAsync( ps.hv.ptr, 0, sizeof( uint32_t ) * 2 * ps.hvBlock, stream ) );
			ps.relaid = true;
		}
		cp.hvZero = ps.hv.ptr + (size_t)(1 - ps.hvParity) * ps.hvBlock, cp.hvZeroWords = LH2_HV_MASK + ps.hvMaskWords;
	}
	const int grid = TraceGrid();
	/* the shade launches walk their segment with a static block stride: blocks beyond the resident ones start as others
	   end, so more, smaller block shares balance the launch's end.  shadeBlocks 0: about shadePathsPerThread paths per
	   thread, between the trace grid and shadeMaxBlocks per CU (the N = 8 share 12 per CU, config 3 24: -1.5 / -1.5 %,
	   profiles/r04al_ab.txt, r04am_ab.txt) */
	const int shadeGrid = shadeBlocks > 0 ? smCount * shadeBlocks : std::max( grid, std::min( smCount * kShadeMaxBlocks,
		(int)((double)pathCount / (256.0 * kShadePathsPerThread)) ) );
	/* the camera fused into the primary packet launch: the heavy-packet block it records into must be zero (the previous
	   fused frame's first shade launch zeroed it) */
	const bool fusedCam = cameraFused && tiledRays && UsePackets() && !primeRef;
	/* round 6: a frame whose primary rays are traced per ray (no packets: a scene beyond the Infinity Cache,
	   config 5) takes the same frame overlap.  Its camera launch (with the frame's resets) and its per-ray primary launch
	   write the frame parity's primary buffers on the ahead stream, the primary launch with a global stack of its own
	   (PathStreams::aheadStack: the previous frame's bounce launch still uses gstack) */
	const bool camAhead = kCamAhead && !fusedCam && cameraFused && !primeRef && TraceVersion() == 7;
	const bool pFrame = fusedCam || camAhead;   /* the frame's primary stage may run beside the previous frame */
	/* the primary stage beside the previous frame (frame overlap), or behind it on the core stream: on a restart (the
	   launch zeroes accumulator pixels), after a change of scene data, buffers or tile, or when the previous frame had no
	   such primary stage */
	const bool serialize = !frameOverlap || !ps.lastFused || ps.relaid || tileChanged || sceneVersion != ps.lastSceneVersion;
	/* a restart beside the previous frame: the accumulator is zeroed on the core stream, behind the previous frame's finalize
	   and before this frame's first addition there (the early shade adds into the delta), not by the primary launch */
	if (pFrame && !serialize && cp.clearAcc)
	{
		CHK_HIP( hipMemsetAsync( accumulator.ptr, 0, sizeof( float4 ) * (size_t)scrwidth * scrheight, stream ) );
		cp.clearAcc = nullptr;
	}
	hipStream_t primStream = stream;
	/* the primary launch's work-queue heads: slot 1 of the frame parity's block, zeroed by the finalize of the frame before
	   the previous one (FrameStatsDev::zeroHeads) */
	const uint32_t primSlot = 1u;
	cp.keepCursor = -1;   /* a camera launch behind the previous frame resets every work-queue head */
	if (pFrame)
	{
		/* beside the previous frame (on the ahead stream, after the previous frame's shade launch before its path tail, or
		   its first without one: the last reader of the primary buffers and of the heavy-packet block this frame records
		   into) or behind it (core stream), the primary launch does the frame's resets itself (kPrimaryResets: this frame
		   parity's counters and heads, whose last user, the frame before the previous one, is done); only an
		   LH2_PRIMARY_RESETS=0 build queues a k_init_counters launch before it on the ahead stream instead.  Its own
		   work-queue heads (slot primSlot, zeroed by the finalize two frames back) are left alone */
		primStream = serialize ? stream : aheadStream;
		cp.keepCursor = (int)(primSlot * LH2_CURSOR_WORDS);
		if (serialize) cp.initC = c;
		else
		{
			CHK_HIP( hipStreamWaitEvent( aheadStream, ps.overlapEv, 0 ) );
			if (kPrimaryResets) cp.initC = c;   /* the primary launch resets them itself: no launch (and its gap) before it */
			else
			{
				lh2_launch_init_counters( c, pathCount, ps.segStride, cursors, LH2_CURSOR_SLOTS * LH2_CURSOR_WORDS, {}, aheadStream, -LH2_CURSOR_WORDS );
				cp.initC = nullptr;
			}
		}
		if (ps.hvOn && !ps.hvNextZeroed) CHK_HIP( hipMemsetAsync( cp.hvZero, 0, sizeof( uint32_t ) * cp.hvZeroWords, primStream ) );
		cp.hvZero = nullptr, cp.hvZeroWords = 0;
		ps.relaid = false;
	}
	ps.hvNextZeroed = false;
	uint32_t* hvReadBlock = nullptr;
	int maxPL = primeRef ? LH2_MAX_BOUNCES : maxPathLength;
	/* no specular event and no alpha cut-out in any material: every path ends at its second vertex,
	   so the bounce after it would be empty; not launching it saves three launches (~25 us) */
	if (!primeRef && diffuseOnly) maxPL = std::min( maxPL, 2 );
	/* the path tail (setting "pathTail"): bounces pathTail .. maxPL in one launch of k_trace_path4d */
	const int tailL = (!primeRef && pathTail >= 2 && pathTail <= maxPL && TraceVersion() == 7) ? pathTail : 0;
	/* early shade: the first shade launch follows the primary launch on the ahead stream and writes the ping-pong buffer
	   the previous frame's launches after its overlap event do not use (PathStreams::busy / earlyOk).  Only when this
	   frame has a path tail from bounce 3 on: else its first shade launch is its overlap event (and, with the tail from
	   bounce 2, its shadow snapshot), and on the ahead stream neither would follow the previous frame's finalize (the
	   side shadow launch and the next frames' early shades would add into the accumulator and the delta before the
	   previous frame is finalized) */
	const bool early = pFrame && !serialize && earlyShade && frameOverlap == 1 && ps.earlyOk && (float)pathCount <= kSmallFramePaths &&
		tailL >= 3;
	ps.early = early;
	ps.in = early ? ps.busy : 0;
	ps.earlyOk = false;
	/* the frame's start: a marker before the camera launch (~4 us of idle GPU), not the launch's own start
	   event (hipExtLaunchKernelGGL start events cost ~8 us: tools/launch_gap.hip, profiles/r02q_launch_gap.txt) */
	CHK_HIP( hipEventRecord( evFrame[0], pFrame ? primStream : stream ) );
	if (fusedCam) ps.prevStop = evFrame[0];
	else if (camAhead)
	{
		lh2_launch_camera( &cp, dBlueNoise.ptr, ps.rayOP[ps.fp].ptr, ps.rayDP[ps.fp].ptr, ps.T4P[ps.fp].ptr, ps.Q4P[ps.fp].ptr, (int)pathCount,
			{ nullptr, ps.evCamera }, primStream );
		ps.prevStop = ps.evCamera;
	}
	else
	{
		lh2_launch_camera( &cp, dBlueNoise.ptr, ps.rayO[0].ptr, ps.rayD[0].ptr, ps.T4[0].ptr, ps.Q4[0].ptr, (int)pathCount, { nullptr, ps.evCamera }, stream );
		ps.prevStop = ps.evCamera;
	}
	if (restart) tileChanged = false;
	/* without lights no path samples one (RandomPointOnLight: lightPdf 0), so there are no shadow
	   rays and their launches are not queued */
	const bool shadows = nArea + nPoint + nSpot + nDir > 0;
	frameShadows = shadows;
	/* shadow overlap: the shade launch before the tail snapshots the queued shadow rays (advance_bounce) */
	const bool overlap = shadows && tailL && shadowOverlap;
	bool snapped = false;
	bool besideNext = false;   /* the next frame's primary launch may run beside the launches from here on */
	ps.sideOn = false;
	/* the bounce loop */
	for (int pathLength = 1; pathLength <= maxPL; pathLength++)
	{
		ps.pl = pathLength;
		/* the path counts ping-pong (Counters::segPath): this bounce's paths, and its extension rays */
		uint32_t* const segIn = c->segPath[(pathLength - 1) & 1];
		uint32_t* const segNext = c->segPath[pathLength & 1];
		uint32_t* const segInBack = c->segBack[(pathLength - 1) & 1];
		uint32_t* const segNextBack = c->segBack[pathLength & 1];
		const bool primary = pathLength == 1 && tiledRays;
		TraceArgs ta{};
		ta.version = TraceVersion();
		ta.rayO = ps.rayO[ps.in].ptr, ta.rayD = ps.rayD[ps.in].ptr, ta.segCounts = segIn, ta.segStride = ps.segStride, ta.segBack = segInBack;
		ta.cursor = cursors + (size_t)(pathLength == 1 ? primSlot : (uint32_t)pathLength) * LH2_CURSOR_WORDS;
		ta.refill = (uint32_t)refillOther;
		ta.packet = primary && UsePackets() ? 1 : 0;
		ta.leafBatch = (uint32_t)leafBatch;
		ta.hits = ps.hits.ptr, ta.gstack = ps.gstack.ptr;
		const bool fusedPrimary = pathLength == 1 && pFrame;   /* the primary buffers (PathStreams::rayOP ..) */
		if (fusedPrimary) ta.rayO = ps.rayOP[ps.fp].ptr, ta.rayD = ps.rayDP[ps.fp].ptr, ta.hits = ps.hitsP[ps.fp].ptr;
		if (pathLength == 1 && ta.packet && ps.hvOn)
		{
			ta.hvRead = ps.hv.ptr + (size_t)ps.hvParity * ps.hvBlock, ta.hvWrite = ps.hv.ptr + (size_t)(1 - ps.hvParity) * ps.hvBlock;
			ta.hvCap = ps.hvCap, ta.hvMaskWords = ps.hvMaskWords, ta.hvFactor = packetHeavy > 0 ? packetHeavy : tailL ? 3.0f : 2.0f;
			hvReadBlock = (uint32_t*)ta.hvRead;
			ta.hvTiles = 0;
			for (int k = 0; k < LH2_SEGS; k++)
			{
				const uint32_t lo = (uint32_t)k * ps.segStride, n = ps.count > lo ? std::min( ps.count - lo, ps.segStride ) : 0u;
				ta.hvTiles += (n + 63) / 64;
			}
			ps.hvParity = 1 - ps.hvParity;
		}
		ShadeParams sp{};
		sp.shadowStride = ps.shadowStride;
		sp.shO = shO, sp.shD = shD, sp.shP = shP;
		sp.acc = accumulator.ptr, sp.counters = c;
		sp.w = scrwidth, sp.h = scrheight, sp.pass = samplesTaken, sp.pathLength = pathLength, sp.maxPathLength = maxPL;
		sp.probePixel = probeX + scrwidth * probeY;
		sp.spreadAngle = view.spreadAngle;
		if (pathLength == tailL)
		{
			/* the path tail: trace and shade every remaining bounce in one launch; each path's records are
			   updated in place, its shadow rays queued for the shadow launch, and rayLog counted */
			sp.rayO = ps.rayO[ps.in].ptr, sp.rayD = ps.rayD[ps.in].ptr, sp.T4 = ps.T4[ps.in].ptr, sp.Q4 = ps.Q4[ps.in].ptr;
			sp.rayOut = ps.rayO[ps.in].ptr, sp.rayDOut = ps.rayD[ps.in].ptr, sp.T4Out = ps.T4[ps.in].ptr, sp.Q4Out = ps.Q4[ps.in].ptr;
			sp.adv.rayCountLog = rayLog;
			ta.shadeBatch = (uint32_t)pathTailBatch;
			/* with the overlap the path tail runs fewer blocks per CU and leaves registers for the side launch's waves
			   (pathTailBlocks; 0: 3 for small frames, whose tail phase is the frame's longest, else 2) */
			const bool side = overlap && snapped;
			const bool small = (float)pathCount <= kSmallFramePaths;
			/* the kernel variant (pathTailWaves 0): 4 waves per SIMD (128 VGPRs) for every frame since the shade batches write their
			   shadow rays at once (its spills 68 -> 40 VGPRs; small frames: config 3 -0.8 %, profiles/r06s_ab_tail_waves.txt); 3
			   (no spills) was the small frames' variant before */
			ta.tailWaves = pathTailWaves == 3 || pathTailWaves == 4 ? (uint32_t)pathTailWaves : 4u;
			const int occ = ta.tailWaves == 4 ? pathBlocksPerCU4 : pathBlocksPerCU;
			const int ptBlocks = pathTailBlocks > 0 ? pathTailBlocks : side ? (small ? 3 : 2) : occ;
			lh2_launch_trace_path( &sd, &ta, &sp, smCount * std::min( std::min( blocksPerCU, occ ), ptBlocks ), { nullptr, ps.evTrace[pathLength] }, stream );
			if (side)
			{
				/* the shadow rays of the bounces before the tail, beside it on the side stream (segment counts:
				   the snapshot; the final launch's work-queue heads start behind them) */
				CHK_HIP( hipStreamWaitEvent( sideStream, ps.prevStop, 0 ) );
				TraceArgs ts{};
				ts.version = TraceVersion();
				ts.rayO = shO, ts.rayD = shD, ts.segCounts = shSnap, ts.segStride = ps.shadowStride;
				ts.cursor = cursors + (size_t)(LH2_SHADOW_SLOT + 1) * LH2_CURSOR_WORDS;
				ts.refill = (uint32_t)refillOther, ts.leafBatch = (uint32_t)kShadowLeafBatch;
				ts.mask = shMask, ts.potentials = shP, ts.acc = accumulator.ptr, ts.gstack = ps.sideStack.ptr;
				/* the global stack (sideStack) is sized for maxBlocksPerCU blocks per CU: the grid stays within it */
				const int sb = sideBlocks >= 0 ? sideBlocks : small ? 3 : 4;
				lh2_launch_trace_any( &sd, &ts, sb > 0 ? smCount * std::min( sb, maxBlocksPerCU ) : grid, 1, { nullptr, ps.evSide }, sideStream );
				ps.fromSide = ps.prevStop;
				ps.sideOn = true;
			}
			ps.fromTrace[pathLength] = ps.prevStop, ps.prevStop = ps.evTrace[pathLength];
			ps.tailL = pathLength;   /* no shade interval of its own (Synchronize) */
			break;
		}
		if (fusedPrimary && camAhead)
		{
			/* the per-ray primary launch after its camera launch (the camera's resets set the dense segment counts); beside the
			   previous frame it walks with a global stack of its own; the core stream waits for it */
			const int waves = traceWaves ? traceWaves : 7;
			ta.traceWaves = (uint32_t)waves;
			if (primStream != stream) ta.gstack = ps.aheadStack.ptr;
			lh2_launch_trace_closest( &sd, &ta, smCount * ClosestBlocksPerCU( waves ), { nullptr, ps.evTrace[pathLength] }, primStream );
			if (primStream != stream && !early) CHK_HIP( hipStreamWaitEvent( stream, ps.evTrace[pathLength], 0 ) );
		}
		else if (fusedPrimary)
		{
			/* the paths are dense (camera order): fixed counts, no segment counters; the core stream waits for it */
			ta.segCounts = nullptr, ta.segBack = nullptr, ta.countFixed = pathCount;
			lh2_launch_trace_primary( &sd, &ta, &cp, ps.T4P[ps.fp].ptr, ps.Q4P[ps.fp].ptr, PacketGrid(), { nullptr, ps.evTrace[pathLength] }, primStream );
			if (primStream != stream && !early) CHK_HIP( hipStreamWaitEvent( stream, ps.evTrace[pathLength], 0 ) );
		}
		else
		{
			/* a bounce launch the next frame's primary launch will likely run beside (this frame overlapped: the next one
			   probably does too): fewer blocks per CU, so the packets' latency-bound waves get slots from the start instead
			   of the bounce launch's tail (config 2: 4262-4296 -> 4437-4442 Mrays/s at 5, r03q_ab_trace_blocks.txt) */
			const bool beside = besideNext && !ta.packet;
			/* traceWaves 0: the 7-wave variant for every scene (round 6: instanced scenes too, with the early node loads), on its occupancy's grid */
			const int waves = traceWaves ? traceWaves : 7;
			const int g = ta.packet ? PacketGrid() : beside ? smCount * std::min( blocksPerCU, kOverlapTraceBlocks ) : smCount * ClosestBlocksPerCU( waves );
			ta.traceWaves = beside ? 7u : (uint32_t)waves;   /* 8 waves slow the packets beside the launch (r04ad) */
#ifdef LH2_TOUCH
			TouchBegin();
#endif
			lh2_launch_trace_closest( &sd, &ta, g, { nullptr, ps.evTrace[pathLength] }, stream );
#ifdef LH2_TOUCH
			TouchReport( pathLength );
#endif
		}
		ps.fromTrace[pathLength] = ps.prevStop, ps.prevStop = ps.evTrace[pathLength];
		sp.segCounts = segIn, sp.segOut = segNext, sp.segStride = ps.segStride;
		sp.segBack = segInBack, sp.segOutBack = segNextBack;
		/* two-ended path segments: rays with a chord through the scene box below chordSplit x its largest
		   extent go last (setting "chordSplit"; 0: off) */
		{
			const float ext = std::max( std::max( sceneHi[0] - sceneLo[0], sceneHi[1] - sceneLo[1] ), sceneHi[2] - sceneLo[2] );
			for (int k = 0; k < 3; k++) sp.chordLo[k] = sceneLo[k], sp.chordHi[k] = sceneHi[k];
			sp.chordCut = ext > 0 ? chordSplit * ext : 0.0f;
		}
		/* the hand-off to the next bounce: the shade launch's last block (no launch of its own), except
		   in PrimeRef mode, where the bounce's shadow rays are traced (and their counts reset) first */
		const bool snap = overlap && pathLength + 1 == tailL;
		const BounceAdvance adv{ segNext, segNextBack, segIn, segInBack, rayLog, ps.activeLog, pathLength + 1 == tailL,
			snap ? shSnap : nullptr, snap ? cursors + (size_t)LH2_SHADOW_SLOT * LH2_CURSOR_WORDS : nullptr };
		snapped = snapped || snap;
		sp.advance = pathLength < maxPL && !primeRef;
		sp.adv = adv;
		sp.rayO = ps.rayO[ps.in].ptr, sp.rayD = ps.rayD[ps.in].ptr, sp.T4 = ps.T4[ps.in].ptr, sp.Q4 = ps.Q4[ps.in].ptr, sp.hits = ps.hits.ptr;
		if (fusedPrimary) sp.rayO = ps.rayOP[ps.fp].ptr, sp.rayD = ps.rayDP[ps.fp].ptr, sp.T4 = ps.T4P[ps.fp].ptr, sp.Q4 = ps.Q4P[ps.fp].ptr, sp.hits = ps.hitsP[ps.fp].ptr;
		sp.rayOut = ps.rayO[1 - ps.in].ptr, sp.rayDOut = ps.rayD[1 - ps.in].ptr, sp.T4Out = ps.T4[1 - ps.in].ptr, sp.Q4Out = ps.Q4[1 - ps.in].ptr;
		sp.primeRef = primeRef;
		sp.terminal = !primeRef && !shadows && !canEmit && pathLength > 1 && terminalShade;
		sp.R0 = (uint32_t)samplesTaken * 7907u + (uint32_t)pathLength * 91771u;
		if (pathLength == 1 && fusedCam && hvReadBlock)
		{
			/* the block this frame's packets read is the one the next frame records into */
			sp.hvZero = hvReadBlock, sp.hvZeroWords = LH2_HV_MASK + ps.hvMaskWords;
			ps.hvNextZeroed = true;
		}
		const bool earlyHere = early && pathLength == 1;
		if (earlyHere) sp.acc = frameDelta;   /* the previous frame's finalize may not have read the accumulator yet */
		lh2_launch_shade( &sd, &sp, shadeGrid, { nullptr, ps.evShade[pathLength] }, earlyHere ? aheadStream : stream );
		if (earlyHere) CHK_HIP( hipStreamWaitEvent( stream, ps.evShade[pathLength], 0 ) );
		ps.fromShade[pathLength] = ps.prevStop, ps.prevStop = ps.evShade[pathLength];
		/* the next frame's primary launch starts after this frame's first shade launch (the last reader of the primary
		   buffers), or (frameOverlap 1) after the shade launch before the path tail: beside the latency-bound tail */
		if (pathLength == 1 || (frameOverlap == 1 && tailL && pathLength == tailL - 1))
		{
			ps.overlapEv = ps.evShade[pathLength];
			besideNext = !serialize && fusedCam && !(frameOverlap == 1 && tailL && pathLength + 1 < tailL);   /* the final overlapEv */
			/* after this launch only the path tail (in place) or the last bounce (no extension rays) runs: both use the
			   buffer this launch writes, 1 - ps.in */
			ps.busy = 1 - ps.in;
			ps.earlyOk = tailL && pathLength == tailL - 1;   /* config 2 (no tail): no gain, and the fold costs (r04b) */
		}

		if (pathLength == maxPL) break;
		if (primeRef && shadows)
		{
			/* RenderCore_PrimeRef traces the shadow rays of every bounce right after it (rendercore.cpp
			   connect step), fused with finalizeConnections */
			TraceArgs ts{};
			ts.version = TraceVersion();
			ts.rayO = shO, ts.rayD = shD, ts.segCounts = c->segShadow, ts.segStride = ps.shadowStride;
			ts.cursor = cursors + (size_t)(LH2_MAX_BOUNCES + pathLength) * LH2_CURSOR_WORDS;
			ts.refill = (uint32_t)refillOther, ts.leafBatch = (uint32_t)leafBatch;
			ts.mask = shMask, ts.potentials = shP, ts.acc = accumulator.ptr, ts.gstack = ps.gstack.ptr;
			lh2_launch_trace_any( &sd, &ts, grid, 1, { nullptr, ps.evShadowB[pathLength] }, stream );
			ps.fromShadowB[pathLength] = ps.prevStop, ps.prevStop = ps.evShadowB[pathLength];
		}
		/* the hand-off writes this bounce's extension-ray count into the pinned activeLog itself */
		ps.countReady[pathLength] = ps.evShade[pathLength];
		if (primeRef)
		{
			lh2_launch_counters_next( c, &adv, pathLength, 1, { nullptr, ps.evCount[pathLength] }, stream );
			ps.prevStop = ps.countReady[pathLength] = ps.evCount[pathLength];
		}
		/* early exit without stalling the GPU: wait for the count of the previous bounce while this one is
		   queued; when it was 0, this bounce is empty and so is everything after it */
		if (pathLength >= 2)
		{
			CHK_HIP( hipEventSynchronize( ps.countReady[pathLength - 1] ) );
			if (ps.activeLog[pathLength - 1] == 0) break;
		}
		ps.in = 1 - ps.in;
	}
	/* an early frame whose paths all ended before the shade launch before its path tail (pathTail >= 4, e.g. every primary
	   ray misses): its overlap event is still its first shade launch, on the ahead stream, which never waited for the
	   previous frame's finalize; the next frame's counter resets on this parity's block two frames on order themselves after
	   overlapEv only.  So it moves to the core stream, behind the previous frame's finalize */
	if (early && ps.overlapEv == ps.evShade[1])
	{
		CHK_HIP( hipEventRecord( ps.evEarlyEnd, stream ) );
		ps.overlapEv = ps.evEarlyEnd;
	}
	/* a snapshot whose side launch did not happen (the frame ended before its path tail): the final launch
	   traces every shadow ray, from the first */
	if (snapped && !ps.sideOn)
		CHK_HIP( hipMemsetAsync( cursors + (size_t)LH2_SHADOW_SLOT * LH2_CURSOR_WORDS, 0, sizeof( uint32_t ) * LH2_CURSOR_WORDS, stream ) );
	/* shadow rays + fused finalizeConnections (rendercore.cpp:575-592) */
	if (!primeRef && shadows)
	{
		TraceArgs ta{};
		ta.version = TraceVersion();
		ta.rayO = shO, ta.rayD = shD, ta.segCounts = c->segShadow, ta.segStride = ps.shadowStride;
		ta.cursor = cursors + (size_t)LH2_SHADOW_SLOT * LH2_CURSOR_WORDS;
		ta.refill = (uint32_t)refillOther, ta.leafBatch = (uint32_t)kShadowLeafBatch;
		ta.mask = shMask, ta.potentials = shP, ta.acc = accumulator.ptr, ta.gstack = ps.gstack.ptr;
		/* the global stack (gstack) is sized for maxBlocksPerCU blocks per CU: the grid stays within it */
		lh2_launch_trace_any( &sd, &ta, finalShadowBlocks > 0 ? smCount * std::min( finalShadowBlocks, maxBlocksPerCU ) : grid, 1, { nullptr, ps.evShadow }, stream );
		ps.fromShadow = ps.prevStop;
	}
	/* the side launch's contributions are in the accumulator before the frame is finalized */
	if (ps.sideOn) CHK_HIP( hipStreamWaitEvent( stream, ps.evSide, 0 ) );
	samplesTaken += scrspp;
	/* finalize also delivers the frame's counters and ray-count log, and the scene error, to hostStats */
	const FrameStatsDev fs{ c, rayLog + 1, &hostStats->counters, hostStats->rayCount + 1, SceneErr( frameTlas ), &hostStats->sceneError,
		cursors + (size_t)primSlot * LH2_CURSOR_WORDS, early ? frameDelta : nullptr };
	/* a tile finalizes its own rows only (a rank of the band partition: the gathered frame is finalized
	   where it is assembled, MultiDevice / FinalizeFrame) */
	RowMap rm{};
	if (tileRows < scrheight) rm = { scrwidth, cp.y0, cp.band, cp.bandStride, tileRows };
	/* the previous frame's end stays recorded (evFrame[2]): an overlapped frame's render time starts at the later of
	   its primary launch's start and the previous frame's end (Synchronize), so per-frame times sum to wall time */
	std::swap( evFrame[1], evFrame[2] );
	prevFrameEndValid = frameEndRecorded, frameWasOverlapped = pFrame && !serialize;
	lh2_launch_finalize( accumulator.ptr, frame.ptr, scrwidth * scrheight, 1.0f / (float)samplesTaken, &fs, { nullptr, evFrame[1] }, stream, &rm );
	frameEndRecorded = true;
	CHK_HIP( hipEventRecord( evTlasFree[frameTlas], stream ) );   /* the next update of this TLAS slot waits for it */
	tlasFreeValid[frameTlas] = true;
	if (glResource && !displayAtFinalize)
	{
		hipArray_t arr = nullptr;
		CHK_HIP( hipGraphicsMapResources( 1, &glResource, stream ) );
		CHK_HIP( hipGraphicsSubResourceGetMappedArray( &arr, glResource, 0, 0 ) );
		CHK_HIP( hipMemcpy2DToArrayAsync( arr, 0, 0, frame.ptr, sizeof( float4 ) * scrwidth, sizeof( float4 ) * scrwidth, scrheight, hipMemcpyDeviceToDevice, stream ) );
		CHK_HIP( hipGraphicsUnmapResources( 1, &glResource, stream ) );
	}
	hostStats->rayCount[0] = ps.count;
	ps.lastFused = pFrame, ps.lastSceneVersion = sceneVersion;
	framePathLengths = ps.tailL ? maxPL : ps.pl;
	framePrimeRef = primeRef;
	statsPending = true;
	frameHostMs = std::chrono::duration<double, std::milli>( std::chrono::high_resolution_clock::now() - t0 ).count();
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
	for (int k = 0; k < LH2_SEGS; k++) n += c.segShadow[k * LH2_SEGCOUNT_STRIDE];
	return n;
}

void RenderCore::Synchronize()
{
	CHK_HIP( hipStreamSynchronize( aheadStream ) );
	CHK_HIP( hipStreamSynchronize( stream ) );
	if (!statsPending) return;
	statsPending = false;
	const Counters& cn = hostStats->counters;
	bool full = cn.shadowOverflow != 0;
	for (int k = 0; k < LH2_SEGS; k++) full = full || cn.segShadow[k * LH2_SEGCOUNT_STRIDE] > ps.shadowStride;
	if (full) FatalError( "shadow ray buffer overflow" );
	if (hostStats->sceneError) FatalError( "%s: frame skipped", SceneErrorText( hostStats->sceneError ) );
	const uint32_t* rc = hostStats->rayCount;   /* rc[0] = primary; rc[L] = rays traced at pathLength L+1 */
	auto ms = [&]( hipEvent_t a, hipEvent_t b ) { float t = 0; (void)hipEventElapsedTime( &t, a, b ); return t * 1e-3f; };
	/* each interval: the previous launch's stop event -> this launch's stop event (kernel + launch gap) */
	auto trace = [&]( int L ) {
		if (L > ps.pl) return 0.0f;
		float t = ms( ps.fromTrace[L], ps.evTrace[L] );
		/* early shade: the second bounce's interval starts at the first shade launch's stop (ahead stream); the part
		   before the previous frame's end is the previous frame's */
		if (L == 2 && ps.early && prevFrameEndValid)
		{
			const float shared = ms( ps.fromTrace[L], evFrame[2] );
			if (shared > 0) t = std::max( 0.0f, t - shared );
		}
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
		if (L <= ps.pl) coreStats.traceTimeX = trace( L );
	}
	float shadow = 0, shade = 0;
	if (frameShadows && !framePrimeRef)
		shadow = ms( ps.fromShadow, ps.evShadow ) + (ps.sideOn ? ms( ps.fromSide, ps.evSide ) : 0.0f);
	else if (frameShadows) for (int L = 1; L < ps.pl; L++) shadow += ms( ps.fromShadowB[L], ps.evShadowB[L] );
	for (int L = 1; L <= ps.pl; L++) if (L != ps.tailL) shade += ms( ps.fromShade[L], ps.evShade[L] );
	coreStats.shadowTraceTime = shadow;
	coreStats.shadeTime = shade;
	for (int L = 1; L <= framePathLengths && L <= 8; L++) lastKernelMs[L - 1] = trace( L ) * 1e3f;
	coreStats.totalShadowRays = framePrimeRef ? cn.totalShadowRays : QueuedShadowRays( cn );
	coreStats.totalExtensionRays = cn.totalExtensionRays;
	coreStats.totalRays = coreStats.totalExtensionRays + coreStats.totalShadowRays;
	/* device time of the whole frame (the reference's Render blocks).  Under frameOverlap the frame's primary launch
	   starts beside the previous frame's tail: the part before the previous frame's end is the previous frame's
	   (ADVICE r3).  traceTime0 stays the primary launch's own duration, stretched by what ran beside it */
	coreStats.renderTime = ms( evFrame[0], evFrame[1] );
	if (frameWasOverlapped && prevFrameEndValid)
	{
		const float shared = ms( evFrame[0], evFrame[2] );
		if (shared > 0) coreStats.renderTime = std::max( 0.0f, coreStats.renderTime - shared );
	}
	coreStats.probedInstid = cn.probedInstid, coreStats.probedTriid = cn.probedTriid, coreStats.probedDist = cn.probedDist;
}

lh2_CoreStats RenderCore::GetCoreStats()
{
	Synchronize();
	return coreStats;
}

void RenderCore::GetRayCounts( uint32_t* out17 )
{
	Synchronize();
	for (int i = 0; i < 16; i++) out17[i] = i < framePathLengths ? hostStats->rayCount[i] : 0u;
	out17[16] = framePrimeRef ? hostStats->counters.totalShadowRays : QueuedShadowRays( hostStats->counters );
}

int RenderCore::DebugShadowRays( float* o4, float* d4, float* p4, int cap )
{
	Synchronize();
	int n = 0;
	for (int k = 0; k < LH2_SEGS; k++)
	{
		const uint32_t cnt = std::min( hostStats->counters.segShadow[k * LH2_SEGCOUNT_STRIDE], ps.shadowStride );
		const int m = std::min( (int)cnt, cap - n );
		if (m <= 0) break;
		const size_t at = (size_t)ps.fp * ps.shCap + (size_t)k * ps.shadowStride;   /* the last frame's parity */
		CHK_HIP( hipMemcpy( o4 + 4 * (size_t)n, ps.shO.ptr + at, 16 * (size_t)m, hipMemcpyDeviceToHost ) );
		CHK_HIP( hipMemcpy( d4 + 4 * (size_t)n, ps.shD.ptr + at, 16 * (size_t)m, hipMemcpyDeviceToHost ) );
		CHK_HIP( hipMemcpy( p4 + 4 * (size_t)n, ps.shP.ptr + at, 16 * (size_t)m, hipMemcpyDeviceToHost ) );
		n += m;
	}
	return n;
}

int RenderCore::DebugBvh4( float* f32Nodes, uint32_t* qNodes, int cap )
{
	if (geometryDirty || instancesDirty) UpdateToplevel();
	Synchronize();
	SyncTlas();
	CHK_HIP( hipStreamSynchronize( stream ) );
	if (!dNodes4.ptr || !dNodes4q.ptr) return 0;
	const int tn = tlasNodeCount[tlasSlot];   /* the current TLAS's own nodes (the slot's others are never written, §3) */
	if (cap <= 0 || !f32Nodes || !qNodes) return blasNode4Count + tn;   /* a count-only call */
	/* the BLAS nodes, then the current TLAS slot's */
	const int n = std::min( cap, blasNode4Count + tn ), nb = std::min( n, blasNode4Count ), nt = n - nb;
	CHK_HIP( hipMemcpy( f32Nodes, dNodes4.ptr, 128 * (size_t)nb, hipMemcpyDeviceToHost ) );
	CHK_HIP( hipMemcpy( qNodes, dNodes4q.ptr, 64 * (size_t)nb, hipMemcpyDeviceToHost ) );
	if (nt > 0)
	{
		CHK_HIP( hipMemcpy( f32Nodes + 32 * (size_t)nb, dNodes4.ptr + 8 * (size_t)TlasBase4( tlasSlot ), 128 * (size_t)nt, hipMemcpyDeviceToHost ) );
		CHK_HIP( hipMemcpy( qNodes + 16 * (size_t)nb, dNodes4q.ptr + 4 * (size_t)TlasBase4( tlasSlot ), 64 * (size_t)nt, hipMemcpyDeviceToHost ) );
	}
	return n;
}

/* diagnostics (test hook): fill both TLAS slots' node regions (BVH2 and BVH4, f32 and quantized) with `value`, as memory an
   earlier, larger TLAS or an uninitialised allocation leaves behind the nodes a TLAS update writes */
void RenderCore::DebugPoisonTlas( float value )
{
	if (geometryDirty || instancesDirty) UpdateToplevel();
	Synchronize();
	SyncTlas();
	CHK_HIP( hipStreamSynchronize( stream ) );
	CHK_HIP( hipStreamSynchronize( aheadStream ) );
	std::vector<float> fill( (size_t)2 * tlasCapacity * 32, value );
	CHK_HIP( hipMemcpy( dNodes.ptr + (size_t)blasNodeCount * 4, fill.data(), sizeof( float4 ) * 4 * 2 * (size_t)tlasCapacity, hipMemcpyHostToDevice ) );
	if (bvh4)
	{
		CHK_HIP( hipMemcpy( dNodes4.ptr + (size_t)blasNode4Count * 8, fill.data(), sizeof( float4 ) * 8 * 2 * (size_t)tlasCapacity, hipMemcpyHostToDevice ) );
		CHK_HIP( hipMemcpy( dNodes4q.ptr + (size_t)blasNode4Count * 4, fill.data(), sizeof( uint4 ) * 4 * 2 * (size_t)tlasCapacity, hipMemcpyHostToDevice ) );
	}
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
	ta.refill = (uint32_t)refillOther, ta.leafBatch = (uint32_t)leafBatch;
	ta.packet = unitCoherent && UsePackets() ? 1 : 0;
	ta.traceWaves = (uint32_t)unitTraceWaves;
	lh2_launch_trace_closest( &sd, &ta, ta.packet ? PacketGrid() : UnitGrid(), {}, stream );
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
	EnsureStack();
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
		ta.hits = (uint4*)hitsOut, ta.gstack = ps.gstack.ptr;
			/* unitCoherent: trace as the frame traces its (tiled) primary rays */
		ta.refill = (uint32_t)refillOther, ta.leafBatch = (uint32_t)leafBatch;
		ta.packet = unitCoherent && UsePackets() ? 1 : 0;
#ifdef LH2_TRACE_STATS
		ta.stats = tstats.ptr;
#endif
#ifdef LH2_TRACE_TIMES
		ta.stats = ttimes.ptr;
#endif
		ta.traceWaves = (uint32_t)unitTraceWaves;
		lh2_launch_trace_closest( &sd, &ta, ta.packet ? PacketGrid() : UnitGrid(), { ev[2 * i], ev[2 * i + 1] }, stream );
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
		SyncTlas();
		CHK_HIP( hipMemcpyAsync( &d, dTlasDepth.ptr, sizeof( int ), hipMemcpyDeviceToHost, stream ) );
		CHK_HIP( hipStreamSynchronize( stream ) );
		sceneMaxDepth = d + maxBlasDepth;
	}
	if (maxDepth) *maxDepth = sceneMaxDepth;
	if (instCount) *instCount = (int)instances.size();
}

#ifdef LH2_SHADE_TIMES
extern "C" void lh2_shade_times( unsigned long long out[16] );
#endif
void RenderCore::Shutdown()   /* rendercore.cpp:615-650 */
{
	if (!initialized) return;
	(void)hipStreamSynchronize( stream );
#ifdef LH2_SHADE_TIMES
	{
		unsigned long long t[16];
		lh2_shade_times( t );
		fprintf( stderr, "LH2_SHADE_TIMES [" );
		for (int i = 0; i < 16; i++) fprintf( stderr, "%s%llu", i ? ", " : "", t[i] );
		fprintf( stderr, "]\n" );
	}
#endif
	if (aheadStream) (void)hipStreamSynchronize( aheadStream );   /* a TLAS update nothing waited for */
	for (auto* m : meshes) delete m;
	meshes.clear();
	instances.clear();
	for (auto& e : ps.evTrace) (void)hipEventDestroy( e ), e = nullptr;
	for (auto& e : ps.evShade) (void)hipEventDestroy( e ), e = nullptr;
	for (auto& e : ps.evShadowB) (void)hipEventDestroy( e ), e = nullptr;
	for (auto& e : ps.evCount) (void)hipEventDestroy( e ), e = nullptr;
	for (hipEvent_t* e : { &ps.evCamera, &ps.evShadow, &ps.evSide, &ps.evEarlyEnd }) { if (*e) (void)hipEventDestroy( *e ); *e = nullptr; }
	if (ps.activeLog) (void)hipHostFree( ps.activeLog );
	ps.activeLog = nullptr;
	for (hipEvent_t* e : { &evConsumer, &evPacked }) { if (*e) (void)hipEventDestroy( *e ); *e = nullptr; }
	for (auto& e : evFrame) (void)hipEventDestroy( e );
	for (auto& e : evStage) (void)hipEventDestroy( e );
	for (hipEvent_t* e : { &evTlasReady, &evTlasFree[0], &evTlasFree[1] }) { if (*e) (void)hipEventDestroy( *e ); *e = nullptr; }
	for (int i = 0; i < 2; i++) { if (stage[i]) (void)hipHostFree( stage[i] ); stage[i] = nullptr, stageBytes[i] = 0; }
	if (glResource) (void)hipGraphicsUnregisterResource( glResource );
	glResource = nullptr, glTexture = 0;
	if (hostStats) (void)hipHostFree( hostStats );
	hostStats = nullptr;
	(void)hipStreamDestroy( stream );
	if (sideStream) (void)hipStreamDestroy( sideStream ), sideStream = nullptr;
	if (aheadStream) (void)hipStreamDestroy( aheadStream ), aheadStream = nullptr;
	stream = nullptr;
	initialized = false;
}

}  // namespace lh2
