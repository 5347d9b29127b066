/* lh2_kernels.hip - hand-written gfx950 kernels of the MI355X wavefront path tracer.

   Hot path:
     k_camera        primary rays          reference: kernels/camera.h:39-111
     k_trace<CLOSEST> BVH2 + Möller–Trumbore closest hit (replaces rtpQueryExecute CLOSEST,
                     rendercore.cpp:516-528), LDS-resident traversal stack
     k_shade         shade / extend / NEE  reference: kernels/pathtracer.h:54-265
     k_trace<ANY>    shadow rays, fused with finalizeConnection (connections.h:22-44)
     k_finalize      accumulator / spp     reference: finalize_shared.h:29-45
   Stream compaction is per wave: __ballot + mbcnt + one atomicAdd per wave (replaces the
   per-thread atomicAdd of pathtracer.h:114,202,237).  Path counts are read from device
   counters, so a frame needs no host round trip between bounces (rendercore.cpp:547).

   Numerics: compiled with -ffp-contract=off and correctly rounded div/sqrt; every expression
   keeps the reference's evaluation order so results are bit-comparable with oracle/pt_oracle.c.
*/
#include <algorithm>
#include <hip/hip_ext.h>
#include "lh2_device.h"
#include "../../include/lh2_core_types.h"
#include "lh2_kernels.h"
#include "lh2_bary.h"

#define S_SPECULAR 1
#define S_BOUNCED 2
#define S_VIASPECULAR 4
#define S_BOUNCEDTWICE 8
#define ENOUGH_BOUNCES S_BOUNCED
#define NOHIT -1
#define EPSILON 0.0001f
#define INVPI LH2_INVPI
#define PI LH2_PI
#define TWOPI LH2_TWOPI

LH2_DEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi( ~0u, __builtin_amdgcn_mbcnt_lo( ~0u, 0u ) ); }
LH2_DEV uint32_t lanes_below( uint64_t m ) { return __builtin_amdgcn_mbcnt_hi( (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo( (uint32_t)m, 0u ) ); }

/* wave-level stream compaction: one atomicAdd per wave, slots in lane order */
LH2_DEV uint32_t wave_alloc( bool want, uint32_t* counter )
{
	const uint64_t m = __ballot( want );
	if (m == 0) return 0xffffffffu;
	const uint32_t leader = (uint32_t)__ffsll( (unsigned long long)m ) - 1u;
	uint32_t base = 0;
	if (lane_id() == leader) base = atomicAdd( counter, (uint32_t)__popcll( m ) );
	base = __builtin_amdgcn_readlane( base, leader );
	return want ? base + lanes_below( m ) : 0xffffffffu;
}

/* three wave-level compactions in one atomic instruction: lane k < 3 adds the count of mask k to counter k (a null
   counter only with an empty mask), so the three slot bases cost one round trip instead of three.  The whole wave must
   be active (k_shade's compaction, after its per-lane branch has reconverged) */
LH2_DEV void wave_alloc3( const uint64_t m0, const uint64_t m1, const uint64_t m2, uint32_t* c0, uint32_t* c1, uint32_t* c2,
	uint32_t& b0, uint32_t& b1, uint32_t& b2 )
{
	b0 = b1 = b2 = 0;
	if ((m0 | m1 | m2) == 0) return;
	const uint32_t lane = lane_id();
	const uint64_t m = lane == 0 ? m0 : lane == 1 ? m1 : m2;
	uint32_t base = 0;
	if (lane < 3 && m != 0) base = atomicAdd( lane == 0 ? c0 : lane == 1 ? c1 : c2, (uint32_t)__popcll( m ) );
	b0 = (uint32_t)__builtin_amdgcn_readlane( (int)base, 0 );
	b1 = (uint32_t)__builtin_amdgcn_readlane( (int)base, 1 );
	b2 = (uint32_t)__builtin_amdgcn_readlane( (int)base, 2 );
}

static_assert( sizeof( ((Counters*)0)->segShadow ) == LH2_SEGS * LH2_SEGCOUNT_STRIDE * 4, "Counters segment layout" );

/* [lo, hi): segment c of a trace launch's ray stream (lh2_kernels.h, LH2_SEGS).  Wave-uniform, and
   said so (readfirstlane): kept in SGPRs, they cost the traversal loop no VGPRs (which it has none
   to spare: with two more live VGPRs the compiler spilled the stack pointers next to the LDS push) */
LH2_DEV void seg_range( const TraceArgs& a, uint32_t c, uint32_t& lo, uint32_t& hi, uint32_t& split, uint32_t& gap )
{
	c = __builtin_amdgcn_readfirstlane( c );
	uint32_t n, nb = 0;
	lo = c * a.segStride;
	if (a.segCounts) n = a.segCounts[c * LH2_SEGCOUNT_STRIDE], nb = a.segBack ? a.segBack[c * LH2_SEGCOUNT_STRIDE] : 0u;
	else n = a.countFixed > lo ? min( a.countFixed - lo, a.segStride ) : 0u;
	lo = __builtin_amdgcn_readfirstlane( lo );
	hi = __builtin_amdgcn_readfirstlane( lo + n + nb );
	/* two-ended segment: queue positions [lo, split) are records lo.., the rest sit at the segment's end */
	split = __builtin_amdgcn_readfirstlane( lo + n );
	gap = __builtin_amdgcn_readfirstlane( nb ? a.segStride - n - nb : 0u );
}
/* the record of queue position j of a two-ended segment */
LH2_DEV uint32_t seg_index( const uint32_t j, const uint32_t split, const uint32_t gap ) { return j < split ? j : j + gap; }

/* no rays in any segment: the launch returns at once (a bounce after the last one, or no shadow rays) */
LH2_DEV bool stream_empty( const TraceArgs& a )
{
	if (!a.segCounts) return a.countFixed == 0;
	uint32_t any = 0;
#pragma unroll
	for (int k = 0; k < LH2_SEGS; k++) any |= a.segCounts[k * LH2_SEGCOUNT_STRIDE] | (a.segBack ? a.segBack[k * LH2_SEGCOUNT_STRIDE] : 0u);
	return any == 0;
}

LH2_DEV void acc_add( float4* acc, uint32_t px, v3 c )
{
	float* a = (float*)(acc + px);
	unsafeAtomicAdd( a + 0, c.x );
	unsafeAtomicAdd( a + 1, c.y );
	unsafeAtomicAdd( a + 2, c.z );
}

/* =====================================================================================
   camera: kernels/camera.h:22-94
   ===================================================================================== */
LH2_DEV float blueNoiseSampler( const uint8_t* bn, int x, int y, int sampleIndex, int sampleDimension ) /* tools_shared.h:336-350 */
{
	x &= 127, y &= 127, sampleIndex &= 255, sampleDimension &= 255;
	int rankedSampleIndex = (sampleIndex ^ (int)bn[sampleDimension + (x + y * 128) * 8 + 65536 * 3]) & 255;
	int value = (int)bn[sampleDimension + rankedSampleIndex * 256];
	value ^= (int)bn[(sampleDimension & 7) + (x + y * 128) * 8 + 65536];
	return (0.5f + (float)value) * (1.0f / 256.0f);
}
/* blueNoiseSampler for the four dimensions dim0 .. dim0 + 3 (dim0 a multiple of 4, as every caller's
   4 + 4 * pathLength), in two steps so that callers can put other loads between them: the four ranking
   bytes and the four scrambling bytes of a pixel are adjacent and 4-aligned (one dword each), then the
   four sample bytes; the values are those of four blueNoiseSampler calls */
struct BlueNoise4 { uint32_t rank, scr; int d0, sampleIndex; };
LH2_DEV BlueNoise4 blueNoiseFetch4( const uint8_t* bn, int x, int y, const int sampleIndex, const int dim0 )
{
	x &= 127, y &= 127;
	BlueNoise4 q;
	q.d0 = dim0 & 255, q.sampleIndex = sampleIndex & 255;
	const int pix = (x + y * 128) * 8;
	q.rank = *(const uint32_t*)(bn + q.d0 + pix + 65536 * 3);
	q.scr = *(const uint32_t*)(bn + (q.d0 & 7) + pix + 65536);
	return q;
}
LH2_DEV void blueNoiseFinish4( const uint8_t* bn, const BlueNoise4& q, float r[4] )
{
	/* the four sample-byte loads issued together (one round trip): the scheduler otherwise interleaved them with their uses
	   in the primary launch's camera code, a round trip each */
	int v[4];
#pragma unroll
	for (int k = 0; k < 4; k++) v[k] = (int)bn[q.d0 + k + ((q.sampleIndex ^ (int)((q.rank >> (8 * k)) & 255)) & 255) * 256];
	__builtin_amdgcn_sched_barrier( 0 );
#pragma unroll
	for (int k = 0; k < 4; k++) r[k] = (0.5f + (float)(v[k] ^ (int)((q.scr >> (8 * k)) & 255))) * (1.0f / 256.0f);
}
LH2_DEV uint32_t WangHash( uint32_t s ) { s = (s ^ 61) ^ (s >> 16), s *= 9, s = s ^ (s >> 4), s *= 0x27d4eb2d, s = s ^ (s >> 15); return s; }
LH2_DEV uint32_t RandomInt( uint32_t& s ) { s ^= s << 13, s ^= s >> 17, s ^= s << 5; return s; }
LH2_DEV float RandomFloat( uint32_t& s ) { return (float)RandomInt( s ) * 2.3283064365387e-10f; }

LH2_DEV v3 RandomPointOnLens( const float r0, float r1, const v3 pos, const float aperture, const v3 right, const v3 up )
{
	const float blade = (float)(int)(r0 * 9);
	float r2 = (r0 - blade * (1.0f / 9.0f)) * 9.0f;
	float x1, y1, x2, y2;
	lh2_sincosf( blade * PI / 4.5f, &x1, &y1 );
	lh2_sincosf( (blade + 1.0f) * PI / 4.5f, &x2, &y2 );
	if ((r1 + r2) > 1) r1 = 1.0f - r1, r2 = 1.0f - r2;
	const float xr = x1 * r1 + x2 * r2;
	const float yr = y1 * r1 + y2 * r2;
	return add3( pos, smul( aperture, add3( muls( right, xr ), muls( up, yr ) ) ) );
}

/* InitCountersForExtend (.cuda.cu:64-74) plus the frame's work-queue heads; thread i of the launch */
LH2_DEV void init_counters( Counters* c, const uint32_t pathCount, const uint32_t segStride, uint32_t* cursors, const int cursorWords, const int i,
	const int keep = -1 )
{
	if (i < cursorWords && (i < keep || i >= keep + LH2_CURSOR_WORDS)) cursors[i] = 0;
	if (i < LH2_SEGS)
	{
		/* the camera writes the paths densely: segment i is [i * segStride, (i + 1) * segStride) */
		const uint32_t lo = (uint32_t)i * segStride;
		c->segPath[0][i * LH2_SEGCOUNT_STRIDE] = pathCount > lo ? min( pathCount - lo, segStride ) : 0u;
		c->segPath[1][i * LH2_SEGCOUNT_STRIDE] = 0, c->segShadow[i * LH2_SEGCOUNT_STRIDE] = 0;
		c->segBack[0][i * LH2_SEGCOUNT_STRIDE] = 0, c->segBack[1][i * LH2_SEGCOUNT_STRIDE] = 0;
	}
	if (i != 0) return;
	c->activePaths = pathCount, c->extensionRays = 0, c->shadowRays = 0;
	c->totalExtensionRays = pathCount, c->totalShadowRays = 0;
	c->probedInstid = -1, c->probedTriid = -1, c->probedDist = 0;
	c->reserved0 = 0, c->shadowOverflow = 0, c->shadeDone = 0;
}

/* n / d for a divisor fixed for the launch (Granlund & Montgomery 1994, the round-up multiplier with the add step):
   exact for every 32-bit n.  dv = { m, a, s } from lh2_div_magic; d == 1 is m = 0, a = 0, s = 0 */
LH2_DEV uint32_t lh2_udiv( const uint32_t n, const uint32_t dv[3] )
{
	const uint32_t t = __umulhi( n, dv[0] );
	return (t + ((n - t) >> dv[1])) >> dv[2];
}

/* the primary ray and path state of path slot `slot` (generateEyeRays, camera.h:39-111): rayO / rayD / T4 / Q4[slot]
   written, the accumulator pixel of a restart's first sample zeroed; O, D: the ray */
LH2_DEV void camera_path( const CameraParams& p, const uint8_t* __restrict__ bn, const uint32_t slot, float4* __restrict__ rayO,
	float4* __restrict__ rayD, float4* __restrict__ T4, float4* __restrict__ Q4, float4& O, float4& D )
{
	/* slot -> (sample, tile row, x) -> global jobIndex = x + (y + s * h) * w, as camera.h:48-53 */
	const uint32_t w = (uint32_t)p.w, h = (uint32_t)p.h;
	const uint32_t tilePix = (uint32_t)p.tileRows * w;
	const uint32_t s = lh2_udiv( slot, p.divTile ), r = slot - s * tilePix;
	uint32_t lr = lh2_udiv( r, p.divW ), x = r - lr * w;
	if (p.tiled && (w & 7u) == 0)
	{
		/* storage order only: each wave (64 slots) holds an 8x8 pixel block, so a wave's rays are
		   coherent; the path index (and therefore every random number) is unchanged */
		const uint32_t rb = lr >> 3;   /* r / (8 w) */
		if (rb < (uint32_t)p.tileRows / 8u)
		{
			const uint32_t q = r - rb * 8u * w, k = q & 63u;
			x = (q >> 6) * 8u + (k & 7u), lr = rb * 8u + (k >> 3);
		}
	}
	const uint32_t lb = lh2_udiv( lr, p.divBand );
	const uint32_t gy = (uint32_t)p.y0 + lb * (uint32_t)p.bandStride + (lr - lb * (uint32_t)p.band);
	const uint32_t jobIndex = x + (gy + s * h) * w;
	/* jobIndex / w = gy + s h (x < w), so the sample is s + gy / h and the row gy % h (gy < h but for odd tilings) */
	uint32_t y = gy, sampleIndex = (uint32_t)p.pass + s;
	if (gy >= h) sampleIndex += gy / h, y = gy % h;
	float r0, r1, r2, r3;
	if (sampleIndex < 256 && !p.primeRef)
	{
		/* dimensions 0..3: blueNoiseSampler's values, the four ranking and scrambling bytes in one dword each */
		float bnv[4];
		blueNoiseFinish4( bn, blueNoiseFetch4( bn, (int)x, (int)y, (int)sampleIndex, 0 ), bnv );
		r0 = bnv[0], r1 = bnv[1], r2 = bnv[2], r3 = bnv[3];
	}
	else
	{
		uint32_t seed = WangHash( (uint32_t)jobIndex + p.R0 );
		r0 = RandomFloat( seed ), r1 = RandomFloat( seed );
		r2 = RandomFloat( seed ), r3 = RandomFloat( seed );
	}
	const v3 p1 = mk3( p.p1.x, p.p1.y, p.p1.z ), right = mk3( p.right.x, p.right.y, p.right.z ), up = mk3( p.up.x, p.up.y, p.up.z );
	const v3 rightW = mk3( p.rightW.x, p.rightW.y, p.rightW.z ), upH = mk3( p.upH.x, p.upH.y, p.upH.z );   /* divs( right, w ), divs( up, h ) */
	v3 posOnPixel;
	if (p.distortion == 0 || p.primeRef)
	{
		posOnPixel = add3( add3( p1, smul( (float)x + r0, rightW ) ), smul( (float)y + r1, upH ) );
	}
	else
	{
		const float sx = (float)x / (float)w - 0.5f, sy = (float)y / (float)h - 0.5f;
		const float rr = sx * sx + sy * sy;
		const float rq = sqrtf( rr ) * (1.0f + p.distortion * rr + p.distortion * rr * rr);
		const float theta = lh2_atan2f( sx, sy );
		float st, ct;
		lh2_sincosf( theta, &st, &ct );
		const float bx = (st * rq + 0.5f) * (float)w;
		const float by = (ct * rq + 0.5f) * (float)h;
		posOnPixel = add3( add3( p1, smul( bx + r0, rightW ) ), smul( by + r1, upH ) );
	}
	const v3 posOnLens = RandomPointOnLens( r2, r3, mk3( p.pos.x, p.pos.y, p.pos.z ), p.aperture, right, up );
	const v3 rayDir = normalize3( sub3( posOnPixel, posOnLens ) );
	const uint32_t out = slot;
	O = make_float4( posOnLens.x, posOnLens.y, posOnLens.z, p.geometryEpsilon );
	D = make_float4( rayDir.x, rayDir.y, rayDir.z, 1e34f );
	rayO[out] = O, rayD[out] = D;
	T4[out] = make_float4( 1, 1, 1, bitsf( ((x + (y + (sampleIndex - (uint32_t)p.pass) * h) * w) << 8) + 1 /* S_SPECULAR */ ) );
	Q4[out] = make_float4( 1, 0, 0, 0 );
	if (p.clearAcc && sampleIndex == (uint32_t)p.pass) p.clearAcc[x + y * w] = make_float4( 0, 0, 0, 0 );
}

__global__ __launch_bounds__( 256 ) void k_camera( const CameraParams p, const uint8_t* __restrict__ bn, float4* __restrict__ rayO,
	float4* __restrict__ rayD, float4* __restrict__ T4, float4* __restrict__ Q4, const int jobCount )
{
	const int local = threadIdx.x + blockIdx.x * blockDim.x;
	if (p.initC) init_counters( p.initC, p.pathCount, p.segStride, p.cursors, p.cursorWords, local, p.keepCursor );
	if (p.hvZero && (uint32_t)local < p.hvZeroWords) p.hvZero[local] = 0;
	if (local >= jobCount) return;
	float4 O, D;
	camera_path( p, bn, (uint32_t)local, rayO, rayD, T4, Q4, O, D );
}

/* =====================================================================================
   traversal: two-level BVH2, ordered, t-culled, LDS short stack + global spill
   ===================================================================================== */
#ifndef LH2_TRACE_MINWAVES
#define LH2_TRACE_MINWAVES 7   /* min waves per SIMD the traversal kernels are compiled for (VGPR cap 72) */
#endif
#define STACK_LDS LH2_STACK_LDS   /* entries per lane kept in LDS: 16 x 256 x 4 B = 16 KB / block */
#define STACK_TOTAL LH2_STACK_TOTAL /* + global spill; the host checks the tree depth against it */

LH2_DEV float safe_inv( float d ) { return (d > -1e-30f && d < 1e-30f) ? (d < 0 ? -1e30f : 1e30f) : 1.0f / d; }

/* oinv = -O / D; oerr: its rounding per axis (|oinv| 2^-22, lh2_box4.inc slab_offsets), subtracted from the entry
   and added to the exit slab of that axis */
struct TRay { v3 O, D, invD, oinv, oerr; };
LH2_DEV void setup_ray( TRay& r, v3 O, v3 D )
{
	r.O = O, r.D = D;
	r.invD = mk3( safe_inv( D.x ), safe_inv( D.y ), safe_inv( D.z ) );
	r.oinv = mk3( -O.x * r.invD.x, -O.y * r.invD.y, -O.z * r.invD.z );
	r.oerr = mk3( fabsf( r.oinv.x ) * 0x1p-22f, fabsf( r.oinv.y ) * 0x1p-22f, fabsf( r.oinv.z ) * 0x1p-22f );
}

/* conservative slab test of one child box; culling only (padded, FMA allowed) */
LH2_DEV bool box_test( float lox, float hix, float loy, float hiy, float loz, float hiz, const TRay& r, float tmin, float tmax, float& tn )
{
#pragma clang fp contract(fast)
	const float t1x = __builtin_fmaf( lox, r.invD.x, r.oinv.x ), t2x = __builtin_fmaf( hix, r.invD.x, r.oinv.x );
	const float t1y = __builtin_fmaf( loy, r.invD.y, r.oinv.y ), t2y = __builtin_fmaf( hiy, r.invD.y, r.oinv.y );
	const float t1z = __builtin_fmaf( loz, r.invD.z, r.oinv.z ), t2z = __builtin_fmaf( hiz, r.invD.z, r.oinv.z );
	tn = fmaxf( fmaxf( fminf( t1x, t2x ) - r.oerr.x, fminf( t1y, t2y ) - r.oerr.y ), fminf( t1z, t2z ) - r.oerr.z );
	const float tf = fminf( fminf( fmaxf( t1x, t2x ) + r.oerr.x, fmaxf( t1y, t2y ) + r.oerr.y ), fmaxf( t1z, t2z ) + r.oerr.z );
	const float tfp = tf * 1.00001f + 1e-30f;
	return tn <= tfp && tfp >= tmin && tn <= tmax * 1.00001f + 1e-30f;
}

struct HitRec { float t; int tri, inst; float u, v; };

/* Möller–Trumbore, same arithmetic as oracle intersect_tri (RenderCore_Bart/common.h:19-50,
   open interval, det == 0 rejected); returns t via tOut */
LH2_DEV bool mt_test( const float4 a, const float4 b, const float4 c, const TRay& r, float& tOut, float& uOut, float& vOut )
{
	const v3 v0 = xyz( a ), e1 = xyz( b ), e2 = xyz( c );
	const v3 h = cross3( r.D, e2 );
	const float det = dot3( e1, h );
	if (det == 0.0f) return false;
	const float f = 1.0f / det;
	const v3 s = sub3( r.O, v0 );
	const float u = f * dot3( s, h );
	if (u < 0.0f || u > 1.0f) return false;
	const v3 q = cross3( s, e1 );
	const float v = f * dot3( r.D, q );
	if (v < 0.0f || u + v > 1.0f) return false;
	tOut = f * dot3( e2, q );
	uOut = u, vOut = v;
	return true;
}

#define LH2_POP INT_MIN   /* "pop the stack next" marker in cur (no valid node or leaf ref) */
#define LH2_FIN (INT_MIN + 1)   /* the BVH4 loop: "this ray is done" (no leaf ref is this: it would start at triangle 2^27 - 1) */

/* Ray-stream traversal with dynamic ray fetch (persistent waves, Aila & Laine 2009 "speculative
   fetch").  Each lane carries one ray's traversal state across loop iterations.  Every iteration
   runs one step: a node visit, an instance entry, or one leaf's triangle tests, and then a pop when
   the step ends a subtree.  A lane whose ray is finished writes its result and goes idle.  Once at
   least a.refill lanes of the wave are idle (64: whole batches), they take new rays from the device work queue: one
   merged atomicAdd per wave, with consecutive indices in lane order.  So the long rays of a batch
   no longer hold up 63 finished lanes.
     KIND 0: closest hit -> hits[idx] = {t, triid, instid, uv16} (uv quantised as pathtracer.h:71,
             OptiX Prime barycentric convention, converted at the end)
     KIND 1: any hit -> occlusion bit (RTP_BUFFER_FORMAT_HIT_BITMASK; mask zeroed by the caller)
     KIND 2: any hit fused with finalizeConnection (connections.h:22-34): unoccluded rays add their
             potential to the accumulator
   The world-space ray is re-read from the ray buffer on the rare instance entry / exit instead of
   being kept in registers.  Termination: the builder emits children after their parent
   (bvh_build.cpp flatten), so descending strictly increases the node index, and every pop undoes
   one push.  The stack depth stays within the tree depth, which UpdateToplevel checks against
   LH2_STACK_TOTAL. */
/* per-lane traversal state of one ray */
struct TraceState
{
	TRay r;
	float tmin;
	HitRec best;
	uint32_t idx;
	int sp, blasSp, cur, curInst, leaf;   /* leaf: parked BLAS leaf (0 = none) */
};

/* interior node: test both child boxes, descend into the nearer hit child, push the farther one */
LH2_DEV void visit_node( const SceneDev& s, TraceState& q, int* __restrict__ lst, int* __restrict__ gst, const uint32_t gstride )
{
	const float4* n = s.nodes + (size_t)q.cur * 4;
	const float4 n0 = n[0], n1 = n[1], n2 = n[2];
	const int4 n3 = *(const int4*)(n + 3);
	float tn0, tn1;
	const bool h0 = box_test( n0.x, n0.y, n0.z, n0.w, n2.x, n2.y, q.r, q.tmin, q.best.t, tn0 );
	const bool h1 = box_test( n1.x, n1.y, n1.z, n1.w, n2.z, n2.w, q.r, q.tmin, q.best.t, tn1 );
	if (h0 && h1)
	{
		const bool swap = tn1 < tn0;
		const int farc = swap ? n3.x : n3.y;
		q.cur = swap ? n3.y : n3.x;
		/* depth <= LH2_STACK_TOTAL is guaranteed by the host (UpdateToplevel) */
		if (q.sp < STACK_LDS) lst[q.sp * 256] = farc;
		else gst[(size_t)(q.sp - STACK_LDS) * gstride] = farc;
		q.sp++;
	}
	else q.cur = h0 ? n3.x : h1 ? n3.y : LH2_POP;
}

/* TLAS leaf (one instance): object-space ray, not renormalised, so t stays in world units (SURVEY §7
   step 3); the world ray is re-read from the ray buffer instead of being kept in registers */
LH2_DEV void enter_instance( const SceneDev& s, const TraceArgs& a, TraceState& q )
{
	const int ii = (int)LEAF_FIRST( q.cur );
	const DevInstance in = s.inst[ii];
	const float4 o4 = a.rayO[q.idx], d4 = a.rayD[q.idx];
	const v3 O = mk3( in.inv0.x * o4.x + in.inv0.y * o4.y + in.inv0.z * o4.z + in.inv0.w,
		in.inv1.x * o4.x + in.inv1.y * o4.y + in.inv1.z * o4.z + in.inv1.w,
		in.inv2.x * o4.x + in.inv2.y * o4.y + in.inv2.z * o4.z + in.inv2.w );
	const v3 D = mk3( in.inv0.x * d4.x + in.inv0.y * d4.y + in.inv0.z * d4.z,
		in.inv1.x * d4.x + in.inv1.y * d4.y + in.inv1.z * d4.z,
		in.inv2.x * d4.x + in.inv2.y * d4.y + in.inv2.z * d4.z );
	setup_ray( q.r, O, D );
	q.blasSp = q.sp, q.curInst = ii;
	q.cur = in.root;
}

/* the triangles of one BLAS leaf; any hit: returns true on the first occluder */
template <bool ANY>
LH2_DEV bool test_leaf( const SceneDev& s, TraceState& q, const int leafRef )
{
	const uint32_t first = LEAF_FIRST( leafRef );
	const int cnt = LEAF_COUNT( leafRef );
	for (int k = 0; k < cnt; k++)
	{
		const float4* tp = s.tris + (size_t)(first + k) * 3;
		const float4 ta = tp[0], tb = tp[1], tc = tp[2];
		float t, u, v;
		if (mt_test( ta, tb, tc, q.r, t, u, v ) && t > q.tmin)
		{
			if (ANY) { if (t < q.best.t) return true; }
			else
			{
				const int tri = __float_as_int( ta.w );
				if (t < q.best.t || (t == q.best.t && (q.curInst < q.best.inst || (q.curInst == q.best.inst && tri < q.best.tri))))
					q.best.t = t, q.best.tri = tri, q.best.inst = q.curInst, q.best.u = u, q.best.v = v;
			}
		}
	}
	return false;
}

/* cur == LH2_POP: leave the BLAS when its subtree is done (not while a leaf of it is parked),
   then pop the next subtree; returns true when the ray is finished */
LH2_DEV bool pop_next( const TraceArgs& a, TraceState& q, int* __restrict__ lst, int* __restrict__ gst, const uint32_t gstride )
{
	if (q.sp == q.blasSp && q.leaf == 0)
	{
		q.blasSp = -1;
		const float4 o4 = a.rayO[q.idx], d4 = a.rayD[q.idx];
		setup_ray( q.r, mk3( o4.x, o4.y, o4.z ), mk3( d4.x, d4.y, d4.z ) );
	}
	if (q.sp == q.blasSp) return false;            /* waiting for the parked leaf */
	if (q.sp == 0) return q.leaf == 0;
	--q.sp;
	q.cur = q.sp < STACK_LDS ? lst[q.sp * 256] : gst[(size_t)(q.sp - STACK_LDS) * gstride];
	return false;
}

/* Ray-stream traversal with dynamic ray fetch (persistent waves, Aila & Laine 2009 "speculative
   fetch").  Each lane carries one ray's traversal state across loop iterations.  A lane whose ray
   is finished writes its result and goes idle.  Once at least a.refill lanes of the wave are idle
   (64: whole batches), they take new rays from the device work queue: one merged atomicAdd per
   wave, with consecutive indices in lane order.  So the long rays of a batch no longer hold up 63
   finished lanes.
   PARK false (coherent primary rays): every iteration runs one step per lane: a node visit, an
   instance entry, or one leaf's triangle tests, then a pop when the step ends a subtree.
   PARK true (incoherent rays): lanes that reach a BLAS leaf park it and keep walking.  The
   triangle tests run for the whole wave at once when at least a.leafBatch lanes hold a parked
   leaf, or when no lane can take a node step.  Node visits and triangle tests then each run with
   most lanes busy, instead of both paths serialising in every iteration.
     KIND 0: closest hit -> hits[idx] = {t, triid, instid, uv16} (uv quantised as pathtracer.h:71,
             OptiX Prime barycentric convention, converted at the end)
     KIND 1: any hit -> occlusion bit (RTP_BUFFER_FORMAT_HIT_BITMASK; mask zeroed by the caller)
     KIND 2: any hit fused with finalizeConnection (connections.h:22-34): unoccluded rays add their
             potential to the accumulator
   Termination: the builder emits children after their parent (bvh_build.cpp flatten), so
   descending strictly increases the node index, and every pop undoes one push.  The stack depth
   stays within the tree depth, which UpdateToplevel checks against LH2_STACK_TOTAL. */
template <int KIND, bool PARK>
LH2_DEV void trace_stream( const SceneDev& s, const TraceArgs& a, int* __restrict__ lst, int* __restrict__ gst, const uint32_t gstride )
{
	constexpr bool ANY = KIND != 0;
	if (stream_empty( a ) || *s.sceneError) return;
	const uint32_t refill = a.refill ? a.refill : 64u;
	const uint32_t leafBatch = a.leafBatch ? a.leafBatch : 1u;
	bool active = false, exhausted = false;
	/* this wave's segment of the ray stream: blocks go round-robin over the 8 XCDs, so blockIdx % 8
	   gives each XCD its own segment and cursor; a dry segment moves the wave on to the next one */
	uint32_t chunk = blockIdx.x % LH2_CHUNKS, tried = 0, lo, hi, split, gap;
	seg_range( a, chunk, lo, hi, split, gap );
	TraceState q;
	q.idx = 0, q.tmin = 0, q.sp = 0, q.blasSp = -1, q.cur = 0, q.curInst = -1, q.leaf = 0;
	while (true)
	{
		/* ---- refill idle lanes (wave-uniform decision) ---- */
		if (!exhausted && __popcll( __ballot( !active ) ) >= refill)
		{
			bool dry = false;
			if (!active)
			{
				/* uniform address (readfirstlane): the compiler then merges the idle lanes' adds into
				   one atomic per wave, handing out consecutive indices in lane order */
				const uint32_t j = lo + atomicAdd( a.cursor + __builtin_amdgcn_readfirstlane( chunk ) * LH2_CURSOR_STRIDE, 1u );
				if (j < hi)
				{
					q.idx = seg_index( j, split, gap );
					const float4 o4 = a.rayO[q.idx], d4 = a.rayD[q.idx];
					setup_ray( q.r, mk3( o4.x, o4.y, o4.z ), mk3( d4.x, d4.y, d4.z ) );
					q.tmin = o4.w;
					q.best.t = d4.w, q.best.tri = -1, q.best.inst = -1, q.best.u = 0, q.best.v = 0;
					q.sp = 0, q.blasSp = -1, q.cur = s.tlasRoot, q.leaf = 0;
					active = true;
				}
				else dry = true;
			}
			if (__ballot( dry ) != 0)   /* cursors only grow: a dry chunk stays dry */
			{
				if (++tried == LH2_CHUNKS) exhausted = true;
				chunk = (chunk + 1) % LH2_CHUNKS;
				seg_range( a, chunk, lo, hi, split, gap );
			}
		}
		if (__ballot( active ) == 0)
		{
			if (exhausted) break;
			continue;
		}
		bool fin = false, occluded = false;
		if (!PARK)
		{
			if (!active) continue;
			if (q.cur >= 0) visit_node( s, q, lst, gst, gstride );
			else if (q.cur != LH2_POP)
			{
				if (q.blasSp < 0) enter_instance( s, a, q );
				else
				{
					occluded = fin = test_leaf<ANY>( s, q, q.cur );
					q.cur = LH2_POP;
				}
			}
			if (!fin && q.cur == LH2_POP) fin = pop_next( a, q, lst, gst, gstride );
		}
		else
		{
			const uint32_t parked = (uint32_t)__popcll( __ballot( active && q.leaf != 0 ) );
			const bool walkers = __ballot( active && q.leaf == 0 ) != 0;
			if (parked >= leafBatch || !walkers)
			{
				/* a lane whose leaf was parked at the BLAS exit or with an empty stack resumes with
				   cur == LH2_POP, and its next node step pops / leaves the BLAS */
				if (q.leaf != 0)
				{
					occluded = fin = test_leaf<ANY>( s, q, q.leaf );
					q.leaf = 0;
				}
			}
			else if (active && q.leaf == 0)
			{
				if (q.cur >= 0) visit_node( s, q, lst, gst, gstride );
				else if (q.cur != LH2_POP)
				{
					if (q.blasSp < 0) enter_instance( s, a, q );
					else { q.leaf = q.cur; q.cur = LH2_POP; }   /* park the BLAS leaf; keep walking */
				}
				if (q.cur == LH2_POP) fin = pop_next( a, q, lst, gst, gstride );
			}
		}
		if (fin)
		{
			active = false;
			if (KIND == 0)
			{
				uint4 out;
				if (q.best.tri < 0) out = make_uint4( fbits( -1.0f ), 0xffffffffu, 0xffffffffu, 0u );
				else
				{
					/* OptiX Prime barycentric convention (u = weight of vertex0, v = weight of vertex1),
					   the one material_shared.h:77-78 interpolates with; MT gave the weights of v1, v2 */
					const float bu = 1.0f - (q.best.u + q.best.v), bv = q.best.u;
					out = make_uint4( fbits( q.best.t ), (uint32_t)q.best.tri, (uint32_t)q.best.inst, lh2_f2u( 65535.0f * bu ) + (lh2_f2u( 65535.0f * bv ) << 16) );
				}
				a.hits[q.idx] = out;
			}
			else if (KIND == 1) { if (occluded) atomicOr( a.mask + (q.idx >> 5), 1u << (q.idx & 31u) ); }
			else if (!occluded)
			{
				const float4 E = a.potentials[q.idx];
				acc_add( a.acc, __float_as_uint( E.w ), mk3( E.x, E.y, E.z ) );
			}
		}
	}
}

#include "lh2_box4.inc"
/* the path-tail mode of lh2_trace4d.inc shades with k_shade's code (defined with the shading code below) */
struct ShadeOut { bool ext, shadow; float4 eO, eD, eT, eQ, sO, sD, sP; uint32_t seg; /* in: EMIT's shadow segment */ };
/* -DLH2_SHADE_TIMES (diagnostic builds only): k_shade's wave time split over the stages of shade_path, summed over every
   launch of the process into lh2_shade_tt (time since the lane's previous mark, recorded by the wave's first active lane;
   the counts of marks in [8 + k]), printed by RenderCore::Shutdown (tools/shade_times.sh) */
#ifdef LH2_SHADE_TIMES
__device__ unsigned long long lh2_shade_tt[16];
#define LH2_STT( k ) if (sttp) { __builtin_amdgcn_sched_barrier( 0 ); const uint64_t n_ = __builtin_amdgcn_s_memtime(); \
	if (lane_id() == (uint32_t)__builtin_ctzll( __ballot( true ) )) atomicAdd( &lh2_shade_tt[k], n_ - *sttp ), atomicAdd( &lh2_shade_tt[8 + (k)], 1ull ); \
	*sttp = n_; __builtin_amdgcn_sched_barrier( 0 ); }
#define LH2_STT_PARAM , uint64_t* sttp
#define LH2_STT_PARAM_DEFAULT , uint64_t* sttp = nullptr
#else
#define LH2_STT( k )
#define LH2_STT_PARAM
#define LH2_STT_PARAM_DEFAULT
#endif
template <bool NL, bool SINGLE, bool EMIT = false>
LH2_DEV void shade_path( const SceneDev& s, const ShadeParams& p, const uint4 hd, const float4 T4, const float4 O4, const float4 D4, const float4 Q4,
	const int pathLength, const uint32_t R0, ShadeOut& o LH2_STT_PARAM_DEFAULT );
#include "lh2_trace4d.inc"
#include "lh2_trace_packet.inc"

/* packet traversal of coherent (8x8-tiled primary) rays: wave-uniform, no LDS stack */
/* 8 waves per SIMD (64 VGPRs, ~32 spilled outside the node loop): the packet loop is bound by the
   latency of its dependent node fetches, and 8 waves hide more of it than the unbounded 94-VGPR
   build's 5: 0.481 -> 0.437 ms on the config-2 primary rays (A/B 5/6/7/8 waves, r01c) */
#ifndef LH2_PACKET_MINWAVES
#define LH2_PACKET_MINWAVES 8
#endif
__global__ __launch_bounds__( 256, LH2_PACKET_MINWAVES ) void k_trace_closest_packet( const SceneDev s, const TraceArgs a ) { trace_packet<false>( s, a ); }
#ifndef LH2_PRIMARY_MINWAVES
#define LH2_PRIMARY_MINWAVES 7
#endif
/* the camera fused into the primary packet launch: each lane makes its path's primary ray (camera_path) and traces it;
   no camera launch, no ray round trip through HBM.  The launch also does the frame's counter and work-queue resets
   (cp.initC), behind the previous frame on the core stream and beside it on the ahead stream alike (RenderCore::
   kPrimaryResets): the resets touch only this frame parity's block, and the launch's own work-queue heads (a fixed slot
   the finalize two frames back zeroes) are left alone */
__global__ __launch_bounds__( 256, LH2_PRIMARY_MINWAVES ) void k_trace_primary_packet( const CameraParams cp, const SceneDev s,
	const TraceArgs a, float4* T4, float4* Q4 )
{
	/* the frame's resets, the camera launch's (every work-queue head but the launch's own); initC is null only in an
	   LH2_PRIMARY_RESETS=0 build, where a k_init_counters launch before this one on the ahead stream does them */
	if (cp.initC)
		for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < (uint32_t)max( cp.cursorWords, LH2_SEGS ); i += gridDim.x * 256u)
			init_counters( cp.initC, cp.pathCount, cp.segStride, cp.cursors, cp.cursorWords, (int)i, cp.keepCursor );
	/* cp first: trace_packet<true> reloads it from the start of the kernel arguments for each packet */
	trace_packet<true>( s, a, T4, Q4 );
}

/* the reference BVH2 loop (traceVersion 1; the BVH4 is not built with setting "bvh4" 0) */
template <bool PARK>
__global__ __launch_bounds__( 256, LH2_TRACE_MINWAVES ) void k_trace_closest( const SceneDev s, const TraceArgs a )
{
	__shared__ int lstack[STACK_LDS * 256];
	trace_stream<0, PARK>( s, a, lstack + threadIdx.x, a.gstack + blockIdx.x * 256 + threadIdx.x, gridDim.x * 256u );
}
template <int MODE>
__global__ __launch_bounds__( 256, LH2_TRACE_MINWAVES ) void k_trace_any( const SceneDev s, const TraceArgs a )
{
	__shared__ int lstack[STACK_LDS * 256];
	trace_stream<MODE == 0 ? 1 : 2, true>( s, a, lstack + threadIdx.x, a.gstack + blockIdx.x * 256 + threadIdx.x, gridDim.x * 256u );
}

/* =====================================================================================
   shading: material_shared.h, lights_shared.h, disney.h, ggxmdf.h, pathtracer.h
   ===================================================================================== */
struct ShadingData
{
	v3 color; int flags;
	v3 transmittance; int matID;
	float4 tint;
	uint4 params;
};
#define CHAR2FLT(a,s) (((float)(((a)>>s)&255))*(1.0f/255.0f))
#define METALLIC CHAR2FLT( sd.params.x, 0 )
#define SUBSURFACE CHAR2FLT( sd.params.x, 8 )
#define SPECULAR CHAR2FLT( sd.params.x, 16 )
#define ROUGHNESS (fmaxf( 0.001f, CHAR2FLT( sd.params.x, 24 ) ))
#define SPECTINT CHAR2FLT( sd.params.y, 0 )
#define ANISOTROPIC CHAR2FLT( sd.params.y, 8 )
#define SHEEN CHAR2FLT( sd.params.y, 16 )
#define SHEENTINT CHAR2FLT( sd.params.y, 24 )
#define CLEARCOAT CHAR2FLT( sd.params.z, 0 )
#define CLEARCOATGLOSS CHAR2FLT( sd.params.z, 8 )
#define TRANSMISSION CHAR2FLT( sd.params.z, 16 )
#define TINT xyz( sd.tint )
#define LUMINANCE sd.tint.w
#define ETA bitsf( sd.params.w )
#define HASSMOOTHNORMALS (1 << 11)

LH2_DEV v3 linear_rgb_to_ciexyz( const v3 rgb )
{
	return mk3( fmaxf( 0.0f, 0.412453f * rgb.x + 0.357580f * rgb.y + 0.180423f * rgb.z ),
		fmaxf( 0.0f, 0.212671f * rgb.x + 0.715160f * rgb.y + 0.072169f * rgb.z ),
		fmaxf( 0.0f, 0.019334f * rgb.x + 0.119193f * rgb.y + 0.950227f * rgb.z ) );
}
LH2_DEV v3 ciexyz_to_linear_rgb( const v3 x )
{
	return mk3( fmaxf( 0.0f, 3.240479f * x.x - 1.537150f * x.y - 0.498535f * x.z ),
		fmaxf( 0.0f, -0.969256f * x.x + 1.875992f * x.y + 0.041556f * x.z ),
		fmaxf( 0.0f, 0.055648f * x.x - 0.204043f * x.y + 1.057311f * x.z ) );
}
/* half -> float is exact for every non-NaN half (lh2_h2f, the host restatement): one v_cvt_f32_f16 */
LH2_DEV float h2f( uint32_t bits16 ) { return (float)__builtin_bit_cast( _Float16, (uint16_t)bits16 ); }

LH2_DEV v3 ConsistentNormal( const v3 D, const v3 iN, const float alpha ) /* tools_shared.h:296-310 */
{
	const float t = PI - 2 * alpha, q = (t * t) / (PI * (PI + (2 * PI - 4) * alpha));
	const float b = dot3( D, iN ), g = 1 + q * (b - 1), rho = sqrtf( q * (1 + g) / (1 + b) );
	const v3 Rc = sub3( muls( iN, g + rho * b ), smul( rho, D ) );
	return normalize3( add3( D, Rc ) );
}

/* ---- texture maps: sampling_shared.h:35-86 (BILINEAR), MIPLEVELCOUNT 5 (common_settings.h:49) ----
   Texels are u32 in HBM (one gather per tap).  Defined where the reference is undefined: float->int
   conversions saturate (lh2_f2i), MIP levels narrower than one texel count as one texel (the
   reference divides by zero there), and indices are clamped to the texel array. */
#define MIPLEVELCOUNT 5
#define HASDIFFUSEMAP (1 << 2)
#define HASNORMALMAP (1 << 3)
#define HASSPECULARITYMAP (1 << 4)
#define HASROUGHNESSMAP (1 << 5)
#define HAS2NDNORMALMAP (1 << 7)
#define HAS2NDDIFFUSEMAP (1 << 9)
#define HASALPHA (1 << 12)
LH2_DEV float4 uchar4_to_float4( const uint32_t v )
{
	const float r = 1.0f / 256.0f;
	return make_float4( (float)(v & 255u) * r, (float)((v >> 8) & 255u) * r, (float)((v >> 16) & 255u) * r, (float)(v >> 24) * r );
}
LH2_DEV float4 FetchTexel( const uint32_t* __restrict__ tex, const uint32_t count, const float tcu, const float tcv, const int o, int w, int h )
{
	w = max( w, 1 ), h = max( h, 1 );
	const float tcx = (fmaxf( tcu + 1000, 0.0f ) * (float)w) - 0.5f, tcy = (fmaxf( tcv + 1000, 0.0f ) * (float)h) - 0.5f;
	const int iu = lh2_f2i( tcx ) % w, iv = lh2_f2i( tcy ) % h;
	const float fu = tcx - floorf( tcx ), fv = tcy - floorf( tcy );
	const float w0 = (1 - fu) * (1 - fv), w1 = fu * (1 - fv), w2 = (1 - fu) * fv, w3 = 1 - (w0 + w1 + w2);
	const uint32_t iu1 = (uint32_t)((iu + 1) % w), iv1 = (uint32_t)((iv + 1) % h);
	const uint32_t last = count - 1;
	const float4 p0 = uchar4_to_float4( tex[min( (uint32_t)o + (uint32_t)iu + (uint32_t)iv * (uint32_t)w, last )] );
	const float4 p1 = uchar4_to_float4( tex[min( (uint32_t)o + iu1 + (uint32_t)iv * (uint32_t)w, last )] );
	const float4 p2 = uchar4_to_float4( tex[min( (uint32_t)o + (uint32_t)iu + iv1 * (uint32_t)w, last )] );
	const float4 p3 = uchar4_to_float4( tex[min( (uint32_t)o + iu1 + iv1 * (uint32_t)w, last )] );
	return make_float4( p0.x * w0 + p1.x * w1 + p2.x * w2 + p3.x * w3, p0.y * w0 + p1.y * w1 + p2.y * w2 + p3.y * w3,
		p0.z * w0 + p1.z * w1 + p2.z * w2 + p3.z * w3, p0.w * w0 + p1.w * w1 + p2.w * w2 + p3.w * w3 );
}
LH2_DEV float4 FetchTexelTrilinear( const uint32_t* __restrict__ tex, const uint32_t count, const float lambda, const float tcu, const float tcv,
	const int offset, const int width, const int height )
{
	const int level0 = min( MIPLEVELCOUNT - 1, lh2_f2i( lambda ) );
	const int level1 = min( MIPLEVELCOUNT - 1, level0 + 1 );
	const float f = lambda - floorf( lambda );
	int o0 = offset, w0 = width, h0 = height;
	for (int i = 0; i < level0; i++) o0 += w0 * h0, w0 >>= 1, h0 >>= 1;
	int o1 = offset, w1 = width, h1 = height;
	for (int i = 0; i < level1; i++) o1 += w1 * h1, w1 >>= 1, h1 >>= 1;
	const float4 p0 = FetchTexel( tex, count, tcu, tcv, o0, w0, h0 );
	const float4 p1 = FetchTexel( tex, count, tcu, tcv, o1, w1, h1 );
	return make_float4( (1 - f) * p0.x + f * p1.x, (1 - f) * p0.y + f * p1.y, (1 - f) * p0.z + f * p1.z, (1 - f) * p0.w + f * p1.w );
}
/* texture coordinate of a map record: uvscale * (uvoffs + (tu, tv)), halves in y / z (CUDAMaterial::Map) */
LH2_DEV void map_coord( const uint4 data, const float tu, const float tv, float& cu, float& cv )
{
	cu = h2f( data.y & 0xffff ) * (h2f( data.z & 0xffff ) + tu);
	cv = h2f( data.y >> 16 ) * (h2f( data.z >> 16 ) + tv);
}
LH2_DEV float normal_scale( const uint32_t byte, const bool absArg )   /* material_shared.h:135, :142 */
{
	const float b = (float)byte - 128.0f;
	return copysignf( -0.0001f + 0.0001f * lh2_expf( 0.1f * (absArg ? fabsf( b ) : b) ), b );
}

/* GetShadingData, material_shared.h:35-178 (OPTIXPRIMEBUILD, CONSISTENTNORMALS, BILINEAR) */
/* the hit triangle's records GetShadingData reads first (CoreTri4: 1 .. 5 and 7), loaded by the caller where the loads can
   go out early (shade_path: beside the instance record's for a single instance) */
struct TriShade { float4 t1, t2, t3, t4, t5, t7; };
LH2_DEV TriShade tri_shade_load( const float4* __restrict__ tri ) { return { tri[1], tri[2], tri[3], tri[4], tri[5], tri[7] }; }
/* the hit material's record (CUDAMaterial, 128 B) and its first two quads, read first; the caller may load them early */
struct MatShade { const uint4* mat; uint4 m0, m1; };
LH2_DEV MatShade mat_shade_load( const SceneDev& s, const TriShade& tq )
{
	const uint4* mat = s.materials + (size_t)__float_as_int( tq.t1.w ) * 8;
	return { mat, mat[0], mat[1] };
}
LH2_DEV void GetShadingData( const SceneDev& s, const v3 D, const float u, const float v, const float coneWidth, const float4* __restrict__ tri,
	const TriShade& tq, const MatShade& mq, const v3 A, const v3 B, const v3 C, ShadingData& sd, v3& N, v3& iN, v3& fN, v3& T )
{

	const float4 tdata1 = tq.t1, tdata2 = tq.t2, tdata3 = tq.t3, tdata4 = tq.t4, tdata5 = tq.t5, alpha4 = tq.t7;
	const uint4* mat = mq.mat;
	const uint4 baseData = mq.m0;
	sd.params = mq.m1;
	sd.color = mk3( h2f( baseData.x & 0xffff ), h2f( baseData.x >> 16 ), h2f( baseData.y & 0xffff ) );
	sd.flags = 0;
	sd.transmittance = mk3( h2f( baseData.y >> 16 ), h2f( baseData.z & 0xffff ), h2f( baseData.z >> 16 ) );
	sd.matID = 0;
	const uint32_t flags = baseData.w;
	const v3 tint_xyz = linear_rgb_to_ciexyz( sd.color );
	const v3 tnt = tint_xyz.y > 0 ? ciexyz_to_linear_rgb( muls( tint_xyz, 1.0f / tint_xyz.y ) ) : s3( 1 );
	sd.tint = make_float4( tnt.x, tnt.y, tnt.z, tint_xyz.y );
	N = iN = fN = mk3( tdata2.w, tdata3.w, tdata4.w );
	T = xyz( tdata5 );
	const float w = 1 - (u + v);
	if (flags & HASSMOOTHNORMALS) iN = normalize3( add3( add3( smul( u, xyz( tdata2 ) ), smul( v, xyz( tdata3 ) ) ), smul( w, xyz( tdata4 ) ) ) );
	/* A, B, C: rows of the instance's inverse transform (lh2_CoreInstanceDesc, fetched by the caller) */
	const v3 n0 = N, i0 = iN;
	N = add3( add3( smul( n0.x, A ), smul( n0.y, B ) ), smul( n0.z, C ) );
	iN = add3( add3( smul( i0.x, A ), smul( i0.y, B ) ), smul( i0.z, C ) );
	const bool backSide = dot3( D, N ) > 0;
	const float alpha = u * alpha4.x + v * alpha4.y + w * alpha4.z;
	iN = smul( backSide ? -1.0f : 1.0f, ConsistentNormal( muls( D, -1.0f ), backSide ? muls( iN, -1.0f ) : iN, alpha ) );
	fN = iN;
	if (!(flags & (HASDIFFUSEMAP | HAS2NDDIFFUSEMAP | HASSPECULARITYMAP | HASNORMALMAP | HAS2NDNORMALMAP | HASROUGHNESSMAP))) return;
	/* texturing (material_shared.h:99-171) */
	const float4 tdata0 = tri[0];
	const float tu = u * tdata0.x + v * tdata0.y + w * tdata0.z;
	const float tv = u * tdata1.x + v * tdata1.y + w * tdata1.z;
	float cu, cv;
	if (flags & HASDIFFUSEMAP)
	{
		const float lambda = alpha4.w + lh2_log2f( coneWidth * (1.0f / fabsf( dot3( D, N ) )) );   /* eq. 26 */
		const uint4 data = mat[2];
		map_coord( data, tu, tv, cu, cv );
		const float4 texel = FetchTexelTrilinear( s.argb32, s.argb32Count, lambda, cu, cv, (int)data.w, (int)(data.x & 0xffff), (int)(data.x >> 16) );
		if ((flags & HASALPHA) && texel.w < 0.5f)
		{
			sd.flags |= 1;
			return;
		}
		sd.color = mul3( sd.color, mk3( texel.x, texel.y, texel.z ) );
		if (flags & HAS2NDDIFFUSEMAP)
		{
			const uint4 d1 = mat[3];
			map_coord( d1, tu, tv, cu, cv );
			const float4 t1 = FetchTexel( s.argb32, s.argb32Count, cu, cv, (int)d1.w, (int)(d1.x & 0xffff), (int)(d1.x >> 16) );
			sd.color = add3( sd.color, sub3( mk3( t1.x, t1.y, t1.z ), s3( 0.5f ) ) );
		}
	}
	if (flags & HASNORMALMAP)
	{
		const v3 Bt = xyz( tri[6] );
		const uint4 data = mat[4];
		const uint32_t part3 = baseData.z;
		const float n0scale = normal_scale( (part3 >> 8) & 255, true );
		map_coord( data, tu, tv, cu, cv );
		const float4 t0 = FetchTexel( s.nrm32, s.nrm32Count, cu, cv, (int)data.w, (int)(data.x & 0xffff), (int)(data.x >> 16) );
		v3 sN = mk3( (t0.x - 0.5f) * 2.0f, (t0.y - 0.5f) * 2.0f, (t0.z - 0.5f) * 2.0f );
		sN.x *= n0scale, sN.y *= n0scale;
		if (flags & HAS2NDNORMALMAP)
		{
			const uint4 d1 = mat[5];
			const float n1scale = normal_scale( (part3 >> 16) & 255, false );
			map_coord( d1, tu, tv, cu, cv );
			const float4 t1 = FetchTexel( s.nrm32, s.nrm32Count, cu, cv, (int)d1.w, (int)(d1.x & 0xffff), (int)(d1.x >> 16) );
			v3 l1 = mk3( (t1.x - 0.5f) * 2.0f, (t1.y - 0.5f) * 2.0f, (t1.z - 0.5f) * 2.0f );
			l1.x *= n1scale, l1.y *= n1scale;
			sN = add3( sN, l1 );
		}
		sN = normalize3( sN );
		fN = normalize3( add3( add3( smul( sN.x, T ), smul( sN.y, Bt ) ), smul( sN.z, iN ) ) );
	}
	if (flags & HASROUGHNESSMAP)
	{
		const uint4 data = mat[7];
		map_coord( data, tu, tv, cu, cv );
		const float4 t = FetchTexel( s.argb32, s.argb32Count, cu, cv, (int)data.w, (int)(data.x & 0xffff), (int)(data.x >> 16) );
		sd.params.x = (sd.params.x & 0xffffff) + (lh2_f2u( t.x * 255.0f ) << 24);
	}
}


/* ---- lights (lights_shared.h:36-261) ------------------------------------------------------ */
/* the light records are read through the constant address space: with a wave-uniform index (the potentials' loops) the
   loads are scalar loads through the scalar cache, issued together, instead of a vector-load round trip per light (the
   light arrays are written only by the host between frames) */
#define LH2_AS4 __attribute__( (address_space( 4 )) )
template <class T> LH2_DEV const LH2_AS4 T* kc( const T* p ) { return (const LH2_AS4 T*)p; }
/* field f of light record i (a lane's own index) of the n records at arr: with few (wave-uniform: at most four lights in the
   scene) selected from the n records' scalar loads, so the sampled light costs no vector-load round trip; else loaded */
template <class T, class F> LH2_DEV float light_field( const T* arr, const int n, const int i, const bool few, F f )
{
	const LH2_AS4 T* a = kc( arr );
	if (!few) return f( a[i] );
	float r = f( a[0] );
	if (n > 1) r = i == 1 ? f( a[1] ) : r;
	if (n > 2) r = i == 2 ? f( a[2] ) : r;
	if (n > 3) r = i == 3 ? f( a[3] ) : r;
	return r;
}
LH2_DEV float PotentialArea( const SceneDev& s, int idx, v3 O, v3 N, v3 I, v3 bary )
{
	const LH2_AS4 lh2_CoreLightTri& l = kc( s.areaLights )[idx];
	v3 L = I;
	if (bary.x >= 0)
	{
		const v3 V0 = mk3( l.vertex0.x, l.vertex0.y, l.vertex0.z ), V1 = mk3( l.vertex1.x, l.vertex1.y, l.vertex1.z ), V2 = mk3( l.vertex2.x, l.vertex2.y, l.vertex2.z );
		L = add3( add3( smul( bary.x, V0 ), smul( bary.y, V1 ) ), smul( bary.z, V2 ) );
	}
	L = sub3( L, O );
	const float att = 1.0f / dot3( L, L );
	L = normalize3( L );
	const float LNdotL = fmaxf( 0.0f, -dot3( mk3( l.N.x, l.N.y, l.N.z ), L ) );
	const float NdotL = fmaxf( 0.0f, dot3( N, L ) );
	return l.energy * LNdotL * NdotL * att;
}
LH2_DEV float PotentialPoint( const SceneDev& s, int idx, v3 I, v3 N )
{
	const LH2_AS4 lh2_CorePointLight& l = kc( s.pointLights )[idx];
	const v3 L = sub3( mk3( l.position.x, l.position.y, l.position.z ), I );
	const float NdotL = fmaxf( 0.0f, dot3( N, L ) );
	const float att = 1.0f / dot3( L, L );
	return l.energy * NdotL * att;
}
LH2_DEV float PotentialSpot( const SceneDev& s, int idx, v3 I, v3 N )
{
	const LH2_AS4 lh2_CoreSpotLight& l = kc( s.spotLights )[idx];
	v3 L = sub3( mk3( l.position.x, l.position.y, l.position.z ), I );
	const float att = 1.0f / dot3( L, L );
	L = normalize3( L );
	const float d = (fmaxf( 0.0f, -dot3( L, mk3( l.direction.x, l.direction.y, l.direction.z ) ) ) - l.cosOuter) / (l.cosInner - l.cosOuter);
	const float NdotL = fmaxf( 0.0f, dot3( N, L ) );
	const float LNdotL = fmaxf( 0.0f, fminf( 1.0f, d ) );
	return (l.radiance.x + l.radiance.y + l.radiance.z) * LNdotL * NdotL * att;
}
LH2_DEV float PotentialDir( const SceneDev& s, int idx, v3 N )
{
	const LH2_AS4 lh2_CoreDirectionalLight& l = kc( s.dirLights )[idx];
	const float LNdotL = fmaxf( 0.0f, -(l.direction.x * N.x + l.direction.y * N.y + l.direction.z * N.z) );
	return l.energy * LNdotL;
}
LH2_DEV float potential_i( const SceneDev& s, int i, v3 I, v3 N, v3 bary, v3 areaI )
{
	if (i < s.nArea) return PotentialArea( s, i, I, N, areaI, bary );
	i -= s.nArea;
	if (i < s.nPoint) return PotentialPoint( s, i, I, N );
	i -= s.nPoint;
	if (i < s.nSpot) return PotentialSpot( s, i, I, N );
	i -= s.nSpot;
	return PotentialDir( s, i, N );
}
LH2_DEV float LightPickProb( const SceneDev& s, int idx, v3 O, v3 N, v3 I )
{
	const int nl = s.nArea + s.nPoint + s.nSpot + s.nDir;
	float sum = 0, pidx = 0;
	for (int i = 0; i < nl; i++)
	{
		const float c = potential_i( s, i, O, N, s3( -1 ), I );
		if (i == idx) pidx = c;
		sum += c;
	}
	if (sum <= 0) return 0;
	if (idx < 0 || idx >= s.nArea) return 0;
	return pidx / sum;
}
/* RandomBarycentrics (lights_shared.h:145-164): the reference's 16-level triangle subdivision in closed form (lh2_bary.h),
   bit-identical for every digit string (tools/bary_check.cpp sweeps all 2^32, tests/test_bary.py a sample) */
LH2_DEV v3 RandomBarycentrics( const float r0 )
{
	const uint32_t uf = lh2_f2u( r0 * 4294967296.0f );
	float sx, sy;
	lh2_bary_sums( uf, sx, sy );
	const float rx = sx * 0.3333333f, ry = sy * 0.3333333f;
	return mk3( rx, ry, 1 - rx - ry );
}
LH2_DEV v3 RandomPointOnLight( const SceneDev& s, float r0, float r1, const v3 I, const v3 N, float& pickProb, float& lightPdf, v3& lightColor )
{
	const int nl = s.nArea + s.nPoint + s.nSpot + s.nDir;
	const float lightCount = (float)nl;
	const v3 bary = RandomBarycentrics( r0 );
	float sum = 0, total = 0;
	int lightIdx = 0;
	if (nl <= 4)
	{
		/* up to four lights: each potential evaluated once (the reference evaluates it in the sum, again in the pick walk and
		   once more for the pick probability; the same arithmetic on the same inputs, so the same values) */
		float pot[4] = { 0, 0, 0, 0 };
#pragma unroll
		for (int i = 0; i < 4; i++) if (i < nl) pot[i] = potential_i( s, i, I, N, bary, s3( 0 ) );
#pragma unroll
		for (int i = 0; i < 4; i++) if (i < nl) sum += pot[i];
		if (sum <= 0) { lightPdf = 0; return s3( 1 ); }
		r1 *= sum;
		bool found = false;
#pragma unroll
		for (int i = 0; i < 4; i++)
			if (i < nl && !found)
			{
				total += pot[i];
				if (total >= r1) lightIdx = i, found = true;
			}
		pickProb = (lightIdx == 0 ? pot[0] : lightIdx == 1 ? pot[1] : lightIdx == 2 ? pot[2] : pot[3]) / sum;
	}
	else
	{
		for (int i = 0; i < nl; i++) sum += potential_i( s, i, I, N, bary, s3( 0 ) );
		if (sum <= 0) { lightPdf = 0; return s3( 1 ); }
		r1 *= sum;
		for (int i = 0; i < nl; i++)
		{
			total += potential_i( s, i, I, N, bary, s3( 0 ) );
			if (total >= r1) { lightIdx = i; break; }
		}
		pickProb = potential_i( s, lightIdx, I, N, bary, s3( 0 ) ) / sum;
	}
	{ const int hi = (int)lightCount - 1; lightIdx = lightIdx < 0 ? 0 : lightIdx > hi ? hi : lightIdx; }
	const bool few = nl <= 4;
	if (lightIdx < s.nArea)
	{
#define LF( fld_ ) light_field( s.areaLights, s.nArea, lightIdx, few, []( const auto& l ) { return l.fld_; } )
		lightColor = mk3( LF( radiance.x ), LF( radiance.y ), LF( radiance.z ) );
		const v3 P = add3( add3( smul( bary.x, mk3( LF( vertex0.x ), LF( vertex0.y ), LF( vertex0.z ) ) ), smul( bary.y, mk3( LF( vertex1.x ), LF( vertex1.y ), LF( vertex1.z ) ) ) ),
			smul( bary.z, mk3( LF( vertex2.x ), LF( vertex2.y ), LF( vertex2.z ) ) ) );
		v3 L = sub3( I, P );
		const float sqDist = dot3( L, L );
		L = normalize3( L );
		const float LNdotL = L.x * LF( N.x ) + L.y * LF( N.y ) + L.z * LF( N.z );
		const float reciSolidAngle = sqDist / (LF( area ) * LNdotL);
		lightPdf = (LNdotL > 0 && dot3( L, N ) < 0) ? reciSolidAngle : 0;
		return P;
#undef LF
	}
	else if (lightIdx < s.nArea + s.nPoint)
	{
		const int li = lightIdx - s.nArea;
#define LF( fld_ ) light_field( s.pointLights, s.nPoint, li, few, []( const auto& l ) { return l.fld_; } )
		const v3 pos = mk3( LF( position.x ), LF( position.y ), LF( position.z ) );
		lightColor = mk3( LF( radiance.x ), LF( radiance.y ), LF( radiance.z ) );
		const v3 L = sub3( I, pos );
		const float sqDist = dot3( L, L );
		lightPdf = dot3( L, N ) < 0 ? sqDist : 0;
		return pos;
#undef LF
	}
	else if (lightIdx < s.nArea + s.nPoint + s.nSpot)
	{
		const int li = lightIdx - (s.nArea + s.nPoint);
#define LF( fld_ ) light_field( s.spotLights, s.nSpot, li, few, []( const auto& l ) { return l.fld_; } )
		const v3 pos = mk3( LF( position.x ), LF( position.y ), LF( position.z ) );
		v3 L = sub3( I, pos );
		const float sqDist = dot3( L, L );
		L = normalize3( L );
		const float cosOuter = LF( cosOuter );
		const float d = (fmaxf( 0.0f, L.x * LF( direction.x ) + L.y * LF( direction.y ) + L.z * LF( direction.z ) ) - cosOuter) / (LF( cosInner ) - cosOuter);
		const float LNdotL = fminf( 1.0f, d );
		lightPdf = (LNdotL > 0 && dot3( L, N ) < 0) ? (sqDist / LNdotL) : 0;
		lightColor = mk3( LF( radiance.x ), LF( radiance.y ), LF( radiance.z ) );
		return pos;
#undef LF
	}
	else
	{
		const int li = lightIdx - (s.nArea + s.nPoint + s.nSpot);
#define LF( fld_ ) light_field( s.dirLights, s.nDir, li, few, []( const auto& l ) { return l.fld_; } )
		const v3 L = mk3( LF( direction.x ), LF( direction.y ), LF( direction.z ) );
		lightColor = mk3( LF( radiance.x ), LF( radiance.y ), LF( radiance.z ) );
		const float NdotL = dot3( L, N );
		lightPdf = NdotL < 0 ? 1 : 0;
		return sub3( I, smul( 1000.0f, L ) );
#undef LF
	}
}

/* ---- Disney BSDF (disney.h:33-333, ggxmdf.h:23-243) -------------------------------------- */
LH2_DEV float schlick_fresnel( float u ) { const float m = saturatef_( 1.0f - u ), m2 = sqrf( m ), m4 = sqrf( m2 ); return m4 * m; }
LH2_DEV v3 mix_spectra( v3 a, v3 b, float t ) { return add3( smul( 1.0f - t, a ), smul( t, b ) ); }
LH2_DEV v3 mix_one_with_spectra( v3 b, float t ) { return sadd( 1.0f - t, smul( t, b ) ); }
LH2_DEV v3 mix_spectra_with_one( v3 a, float t ) { return adds( smul( 1.0f - t, a ), t ); }
LH2_DEV void microfacet_alpha_from_roughness( float roughness, float anisotropy, float& ax, float& ay )
{
	const float square_roughness = roughness * roughness;
	const float aspect = sqrtf( 1.0f + anisotropy * (anisotropy < 0 ? 0.9f : -0.9f) );
	ax = fmaxf( 0.001f, square_roughness / aspect );
	ay = fmaxf( 0.001f, square_roughness * aspect );
}
LH2_DEV float clearcoat_roughness( const ShadingData& sd ) { return mixf( 0.1f, 0.001f, CLEARCOATGLOSS ); }
LH2_DEV v3 DisneySpecularFresnel( const ShadingData& sd, v3 o, v3 h )
{
	v3 value = mix_one_with_spectra( TINT, SPECTINT );
	value = muls( value, SPECULAR * 0.08f );
	value = mix_spectra( value, sd.color, METALLIC );
	const float cos_oh = fabsf( dot3( o, h ) );
	return mix_spectra_with_one( value, schlick_fresnel( cos_oh ) );
}
LH2_DEV v3 DisneyClearcoatFresnel( const ShadingData& sd, v3 o, v3 h )
{
	const float cos_oh = fabsf( dot3( o, h ) );
	return s3( mixf( 0.04f, 1.0f, schlick_fresnel( cos_oh ) ) * 0.25f * CLEARCOAT );
}
LH2_DEV bool force_above_surface( v3& direction, const v3 normal )
{
	const float Eps = 1.0e-4f;
	const float cos_theta = dot3( direction, normal );
	const float correction = Eps - cos_theta;
	if (correction <= 0) return false;
	direction = normalize3( add3( direction, smul( correction, normal ) ) );
	return true;
}
LH2_DEV float Fr_L( float VDotN, float eio )
{
	if (VDotN < 0.0f) eio = 1.0f / eio, VDotN = fabsf( VDotN );
	const float SinThetaT2 = sqrf( eio ) * (1.0f - VDotN * VDotN);
	if (SinThetaT2 > 1.0f) return 1.0f;
	const float LDotN = sqrtf( 1.0f - SinThetaT2 );
	const float r1 = (VDotN - eio * LDotN) / (VDotN + eio * LDotN);
	const float r2 = (LDotN - eio * VDotN) / (LDotN + eio * VDotN);
	return 0.5f * (sqrf( r1 ) + sqrf( r2 ));
}
LH2_DEV bool Refract_L( const v3 wi, const v3 n, const float eta, v3& wt )
{
	const float cosThetaI = fabsf( dot3( n, wi ) );
	const float sin2ThetaI = fmaxf( 0.0f, 1.0f - cosThetaI * cosThetaI );
	const float sin2ThetaT = eta * eta * sin2ThetaI;
	if (sin2ThetaT >= 1) return false;
	const float cosThetaT = sqrtf( 1.0f - sin2ThetaT );
	wt = add3( smul( eta, muls( wi, -1.0f ) ), smul( eta * cosThetaI - cosThetaT, n ) );
	return true;
}
LH2_DEV float stretched_roughness( v3 m, float sin_theta, float ax, float ay )
{
	if (ax == ay || sin_theta == 0.0f) return 1.0f / sqrf( ax );
	const float c = sqrf( m.x / (sin_theta * ax) ), s = sqrf( m.y / (sin_theta * ay) );
	return c + s;
}
LH2_DEV float projected_roughness( v3 m, float sin_theta, float ax, float ay )
{
	if (ax == ay || sin_theta == 0.0f) return ax;
	const float c = sqrf( (m.x * ax) / sin_theta ), s = sqrf( (m.y * ay) / sin_theta );
	return sqrtf( c + s );
}
LH2_DEV float GGXMDF_D( v3 m, float ax, float ay )
{
	const float cos_theta = m.z;
	if (cos_theta == 0.0f) return sqrf( ax ) * INVPI;
	const float cos_theta_2 = sqrf( cos_theta );
	const float sin_theta = sqrtf( fmaxf( 0.0f, 1.0f - cos_theta_2 ) );
	const float cos_theta_4 = sqrf( cos_theta_2 );
	const float tan_theta_2 = (1.0f - cos_theta_2) / cos_theta_2;
	const float A = stretched_roughness( m, sin_theta, ax, ay );
	const float tmp = 1.0f + tan_theta_2 * A;
	return 1.0f / (PI * ax * ay * cos_theta_4 * sqrf( tmp ));
}
LH2_DEV float GGXMDF_lambda( v3 v, float ax, float ay )
{
	const float cos_theta = v.z;
	if (cos_theta == 0.0f) return 0.0f;
	const float cos_theta_2 = sqrf( cos_theta );
	const float sin_theta = sqrtf( fmaxf( 0.0f, 1.0f - cos_theta_2 ) );
	const float alpha = projected_roughness( v, sin_theta, ax, ay );
	const float tan_theta_2 = sqrf( sin_theta ) / cos_theta_2;
	const float a2_rcp = sqrf( alpha ) * tan_theta_2;
	return (-1.0f + sqrtf( 1.0f + a2_rcp )) * 0.5f;
}
LH2_DEV float GGXMDF_G( v3 wi, v3 wo, float ax, float ay ) { return 1.0f / (1.0f + GGXMDF_lambda( wo, ax, ay ) + GGXMDF_lambda( wi, ax, ay )); }
LH2_DEV float GGXMDF_G1( v3 v, float ax, float ay ) { return 1.0f / (1.0f + GGXMDF_lambda( v, ax, ay )); }
LH2_DEV v3 GGXMDF_sample( v3 v, float r0, float r1, float ax, float ay )
{
	const float sign_cos_vn = v.z < 0.0f ? -1.0f : 1.0f;
	v3 stretched = mk3( sign_cos_vn * v.x * ax, sign_cos_vn * v.y * ay, sign_cos_vn * v.z );
	stretched = normalize3( stretched );
	const v3 t1 = v.z < 0.9999f ? normalize3( cross3( stretched, mk3( 0, 0, 1 ) ) ) : mk3( 1, 0, 0 );
	const v3 t2 = cross3( t1, stretched );
	const float a = 1.0f / (1.0f + stretched.z);
	const float r = sqrtf( r0 );
	const float phi = r1 < a ? r1 / a * PI : PI + (r1 - a) / (1.0f - a) * PI;
	float sp, cp;
	lh2_sincosf( phi, &sp, &cp );
	const float p1 = r * cp;
	const float p2 = r * sp * (r1 < a ? 1.0f : stretched.z);
	const v3 h = add3( add3( smul( p1, t1 ), smul( p2, t2 ) ), smul( sqrtf( fmaxf( 0.0f, 1.0f - p1 * p1 - p2 * p2 ) ), stretched ) );
	const v3 m = mk3( h.x * ax, h.y * ay, fmaxf( 0.0f, h.z ) );
	return normalize3( m );
}
LH2_DEV float GGXMDF_pdf( v3 v, v3 m, float ax, float ay )
{
	const float cos_theta_v = v.z;
	if (cos_theta_v == 0.0f) return 0;
	return GGXMDF_G1( v, ax, ay ) * fabsf( dot3( v, m ) ) * GGXMDF_D( m, ax, ay ) / fabsf( cos_theta_v );
}
LH2_DEV float GTR1MDF_D( v3 m, float ax )
{
	const float alpha = clampf_( ax, 0.001f, 0.999f );
	const float alpha_x_2 = sqrf( alpha );
	const float cos_theta_2 = sqrf( m.z );
	const float a = (alpha_x_2 - 1.0f) / (PI * lh2_logf( alpha_x_2 ));
	const float b = (1 / (1 + (alpha_x_2 - 1) * cos_theta_2));
	return a * b;
}
LH2_DEV float GTR1MDF_lambda( v3 v, float ax )
{
	const float cos_theta = v.z;
	if (cos_theta == 0) return 0;
	const float cos_theta_2 = sqrf( cos_theta );
	const float sin_theta = sqrtf( fmaxf( 0.0f, 1.0f - cos_theta_2 ) );
	if (sin_theta == 0.0f) return 0.0f;
	const float cot_theta_2 = cos_theta_2 / sqrf( sin_theta );
	const float cot_theta = sqrtf( cot_theta_2 );
	const float alpha = clampf_( ax, 0.001f, 0.999f );
	const float alpha_2 = sqrf( alpha );
	const float a = sqrtf( cot_theta_2 + alpha_2 );
	const float b = sqrtf( cot_theta_2 + 1.0f );
	const float c = lh2_logf( cot_theta + b );
	const float d = lh2_logf( cot_theta + a );
	return (a - b + cot_theta * (c - d)) / (cot_theta * lh2_logf( alpha_2 ));
}
LH2_DEV float GTR1MDF_G( v3 wi, v3 wo, float ax ) { return 1.0f / (1.0f + GTR1MDF_lambda( wo, ax ) + GTR1MDF_lambda( wi, ax )); }
LH2_DEV v3 GTR1MDF_sample( float r0, float r1, float ax )
{
	const float alpha = clampf_( ax, 0.001f, 0.999f );
	const float alpha_2 = sqrf( alpha );
	const float a = 1.0f - lh2_powf( alpha_2, 1.0f - r0 );
	const float cos_theta_2 = a / (1.0f - alpha_2);
	const float cos_theta = sqrtf( cos_theta_2 );
	const float sin_theta = sqrtf( fmaxf( 0.0f, 1.0f - cos_theta_2 ) );
	float sin_phi, cos_phi;
	lh2_sincosf( TWOPI * r1, &sin_phi, &cos_phi );
	return mk3( cos_phi * sin_theta, sin_phi * sin_theta, cos_theta );
}
LH2_DEV float GTR1MDF_pdf( v3 m, float ax ) { return GTR1MDF_D( m, ax ) * fabsf( m.z ); }
LH2_DEV v3 World2Tangent( v3 V, v3 N, v3 T, v3 B ) { return mk3( dot3( V, T ), dot3( V, B ), dot3( V, N ) ); }
LH2_DEV v3 Tangent2World( v3 V, v3 N, v3 T, v3 B ) { return add3( add3( smul( V.x, T ), smul( V.y, B ) ), smul( V.z, N ) ); }
LH2_DEV v3 DiffuseReflectionCosWeighted( float r0, float r1 )
{
	const float term1 = TWOPI * r0, term2 = sqrtf( 1 - r1 );
	float s, c;
	lh2_sincosf( term1, &s, &c );
	return mk3( c * term2, s * term2, sqrtf( r1 ) );
}

template <bool GGX>
LH2_DEV void sample_mf( const ShadingData& sd, float r0, float r1, float ax, float ay, v3 N, v3 T, v3 B, v3 gN, v3 wow, v3& wiw, float& pdf, v3& value )
{
	v3 wo = World2Tangent( wow, N, T, B );
	if (wo.z == 0) return;
	v3 m = GGX ? GGXMDF_sample( wo, r0, r1, ax, ay ) : GTR1MDF_sample( r0, r1, ax );
	v3 wi = reflect3( muls( wo, -1.0f ), m );
	const v3 ng = World2Tangent( gN, N, T, B );
	if (force_above_surface( wi, ng )) m = normalize3( add3( wo, wi ) );
	if (wi.z == 0) return;
	const float cos_oh = dot3( wo, m );
	pdf = (GGX ? GGXMDF_pdf( wo, m, ax, ay ) : GTR1MDF_pdf( m, ax )) / fabsf( 4.0f * cos_oh );
	if (pdf < 1.0e-6f) return;
	const float D = GGX ? GGXMDF_D( m, ax, ay ) : GTR1MDF_D( m, ax );
	const float G = GGX ? GGXMDF_G( wi, wo, ax, ay ) : GTR1MDF_G( wi, wo, ax );
	value = GGX ? DisneySpecularFresnel( sd, wo, m ) : DisneyClearcoatFresnel( sd, wo, m );
	value = muls( value, D * G / fabsf( 4.0f * wo.z * wi.z ) );
	wiw = Tangent2World( wi, N, T, B );
}
template <bool GGX>
LH2_DEV float evaluate_mf( const ShadingData& sd, float ax, float ay, v3 N, v3 T, v3 B, v3 wow, v3 wiw, v3& bsdf )
{
	const v3 wo = World2Tangent( wow, N, T, B );
	const v3 wi = World2Tangent( wiw, N, T, B );
	if (wo.z == 0 || wi.z == 0) return 0;
	const v3 m = normalize3( add3( wi, wo ) );
	const float cos_oh = dot3( wo, m );
	if (cos_oh == 0) return 0;
	const float D = GGX ? GGXMDF_D( m, ax, ay ) : GTR1MDF_D( m, ax );
	const float G = GGX ? GGXMDF_G( wi, wo, ax, ay ) : GTR1MDF_G( wi, wo, ax );
	bsdf = GGX ? DisneySpecularFresnel( sd, wo, m ) : DisneyClearcoatFresnel( sd, wo, m );
	bsdf = muls( bsdf, D * G / fabsf( 4.0f * wo.z * wi.z ) );
	return (GGX ? GGXMDF_pdf( wo, m, ax, ay ) : GTR1MDF_pdf( m, ax )) / fabsf( 4.0f * cos_oh );
}
LH2_DEV float evaluate_diffuse( const ShadingData& sd, v3 iN, v3 wow, v3 wiw, v3& value )
{
	const v3 n = iN;
	const v3 h = normalize3( add3( wiw, wow ) );
	const float cos_on = dot3( n, wow );
	const float cos_in = dot3( n, wiw );
	const float cos_ih = dot3( wiw, h );
	const float fl = schlick_fresnel( cos_in );
	const float fv = schlick_fresnel( cos_on );
	float fd = 0;
	if (SUBSURFACE != 1.0f)
	{
		const float fd90 = 0.5f + 2.0f * sqrf( cos_ih ) * ROUGHNESS;
		fd = mixf( 1.0f, fd90, fl ) * mixf( 1.0f, fd90, fv );
	}
	if (SUBSURFACE > 0)
	{
		const float fss90 = sqrf( cos_ih ) * ROUGHNESS;
		const float fss = mixf( 1.0f, fss90, fl ) * mixf( 1.0f, fss90, fv );
		const float ss = 1.25f * (fss * (1.0f / (fabsf( cos_on ) + fabsf( cos_in )) - 0.5f) + 0.5f);
		fd = mixf( fd, ss, SUBSURFACE );
	}
	value = muls( muls( muls( sd.color, fd ), INVPI ), 1.0f - METALLIC );
	return fabsf( cos_in ) * INVPI;
}
LH2_DEV float evaluate_sheen( const ShadingData& sd, v3 wow, v3 wiw, v3& value )
{
	const v3 h = normalize3( add3( wow, wow ) );
	const float cos_ih = dot3( wiw, h );
	const float fh = schlick_fresnel( cos_ih );
	value = mix_one_with_spectra( TINT, SHEENTINT );
	value = muls( value, fh * SHEEN * (1.0f - METALLIC) );
	return 1.0f / (2 * PI);
}
LH2_DEV v3 SampleBSDF( const ShadingData& sd, v3 iN, const v3 N, const v3 iT, const v3 wow, const float distance, const float r0, const float r1,
	v3& wiw, float& pdf, bool& specular )
{
	const float flip = (dot3( wow, N ) < 0) ? -1 : 1;
	iN = muls( iN, flip );
	if (r0 < TRANSMISSION)
	{
		specular = true, pdf = 1;
		const float eio = flip < 0 ? (1.0f / ETA) : ETA, F = Fr_L( dot3( iN, wow ), eio );
		v3 beer;
		beer.x = lh2_expf( -sd.transmittance.x * distance * 2.0f );
		beer.y = lh2_expf( -sd.transmittance.y * distance * 2.0f );
		beer.z = lh2_expf( -sd.transmittance.z * distance * 2.0f );
		if (r1 < F)
		{
			wiw = reflect3( muls( wow, -1.0f ), iN );
			if (dot3( muls( N, flip ), wiw ) <= 0) pdf = 0;
			return muls( mul3( sd.color, beer ), 1 / fabsf( dot3( iN, wiw ) ) );
		}
		else
		{
			if (!Refract_L( wow, iN, eio, wiw )) return s3( 0 );
			const float ajointCorrection = 1.0f;
			return muls( muls( mul3( sd.color, beer ), ajointCorrection ), 1 / fabsf( dot3( iN, wiw ) ) );
		}
	}
	const float r3 = (r0 - TRANSMISSION) / (1 - TRANSMISSION);
	const v3 B = normalize3( cross3( iN, iT ) );
	const v3 T = normalize3( cross3( iN, B ) );
	float wx = lerpf_( LUMINANCE, 0, METALLIC ), wy = lerpf_( SHEEN, 0, METALLIC ), wz = lerpf_( SPECULAR, 1, METALLIC ), ww = CLEARCOAT * 0.25f;
	const float wsum = 1.0f / (wx + wy + wz + ww);
	wx *= wsum, wy *= wsum, wz *= wsum, ww *= wsum;
	const float cdfx = wx, cdfy = wx + wy, cdfz = wx + wy + wz;
	float probability, component_pdf = 0;
	v3 contrib = s3( 0 ), value = s3( 0 );
	if (r3 < cdfx)
	{
		const float r2 = r3 / cdfx;
		const v3 wi = DiffuseReflectionCosWeighted( r2, r1 );
		wiw = normalize3( Tangent2World( wi, iN, T, B ) );
		component_pdf = evaluate_diffuse( sd, iN, wow, wiw, value );
		probability = wx * component_pdf, wx = 0;
	}
	else if (r3 < cdfy)
	{
		const float r2 = (r3 - cdfx) / (cdfy - cdfx);
		const v3 wi = DiffuseReflectionCosWeighted( r2, r1 );
		wiw = normalize3( Tangent2World( wi, iN, T, B ) );
		component_pdf = evaluate_sheen( sd, wow, wiw, value );
		probability = wy * component_pdf, wy = 0;
	}
	else if (r3 < cdfz)
	{
		const float r2 = (r3 - cdfy) / (cdfz - cdfy);
		float ax, ay;
		microfacet_alpha_from_roughness( ROUGHNESS, ANISOTROPIC, ax, ay );
		sample_mf<true>( sd, r2, r1, ax, ay, iN, T, B, muls( N, flip ), wow, wiw, component_pdf, value );
		probability = wz * component_pdf, wz = 0;
	}
	else
	{
		const float r2 = (r3 - cdfz) / (1 - cdfz);
		const float alpha = clearcoat_roughness( sd );
		sample_mf<false>( sd, r2, r1, alpha, alpha, iN, T, B, muls( N, flip ), wow, wiw, component_pdf, value );
		probability = ww * component_pdf, ww = 0;
	}
	if (wx > 0) probability += wx * evaluate_diffuse( sd, iN, wow, wiw, contrib ), value = add3( value, contrib );
	if (wy > 0) probability += wy * evaluate_sheen( sd, wow, wiw, contrib ), value = add3( value, contrib );
	if (wz > 0)
	{
		float ax, ay;
		microfacet_alpha_from_roughness( ROUGHNESS, ANISOTROPIC, ax, ay );
		probability += wz * evaluate_mf<true>( sd, ax, ay, iN, T, B, wow, wiw, contrib );
		value = add3( value, contrib );
	}
	if (ww > 0)
	{
		const float alpha = clearcoat_roughness( sd );
		probability += ww * evaluate_mf<false>( sd, alpha, alpha, iN, T, B, wow, wiw, contrib );
		value = add3( value, contrib );
	}
	if (probability > 1.0e-6f) pdf = probability; else pdf = 0;
	return value;
}
LH2_DEV v3 EvaluateBSDF( const ShadingData& sd, const v3 iN, const v3 iT, const v3 wow, const v3 wiw, float& pdf )
{
	if (TRANSMISSION > 0.999f || ROUGHNESS <= 0.001f) { pdf = 0; return s3( 0 ); }
	float wx = lerpf_( LUMINANCE, 0, METALLIC ), wy = lerpf_( SHEEN, 0, METALLIC ), wz = lerpf_( SPECULAR, 1, METALLIC ), ww = CLEARCOAT * 0.25f;
	const float wsum = 1.0f / (wx + wy + wz + ww);
	wx *= wsum, wy *= wsum, wz *= wsum, ww *= wsum;
	pdf = 0;
	v3 value = s3( 0 );
	if (wx > 0) pdf += wx * evaluate_diffuse( sd, iN, wow, wiw, value );
	if (wy > 0) pdf += wy * evaluate_sheen( sd, wow, wiw, value );
	/* the tangent frame only for the microfacet lobes (a wave whose lanes have neither skips it: the same values when made) */
	v3 B = s3( 0 ), T = s3( 0 );
	if (wz > 0 || ww > 0) B = normalize3( cross3( iN, iT ) ), T = normalize3( cross3( iN, B ) );
	if (wz > 0)
	{
		float ax, ay;
		microfacet_alpha_from_roughness( ROUGHNESS, ANISOTROPIC, ax, ay );
		v3 contrib = s3( 0 );
		const float spec_pdf = evaluate_mf<true>( sd, ax, ay, iN, T, B, wow, wiw, contrib );
		if (spec_pdf > 0) pdf += wz * spec_pdf, value = add3( value, contrib );
	}
	if (ww > 0)
	{
		const float alpha = clearcoat_roughness( sd );
		v3 contrib = s3( 0 );
		const float clearcoat_pdf = evaluate_mf<false>( sd, alpha, alpha, iN, T, B, wow, wiw, contrib );
		if (clearcoat_pdf > 0) pdf += ww * clearcoat_pdf, value = add3( value, contrib );
	}
	return value;
}

/* ---- tools --------------------------------------------------------------------------------- */
LH2_DEV uint32_t PackNormal( const v3 N )
{
	const float f = 65535.0f / fmaxf( sqrtf( 8.0f * N.z + 8.0f ), 0.0001f );
	return lh2_f2u( N.x * f + 32767.0f ) + (lh2_f2u( N.y * f + 32767.0f ) << 16);
}
LH2_DEV v3 UnpackNormal( const uint32_t p )
{
	float nx = (float)(p & 65535) * (2.0f / 65535.0f), ny = (float)(p >> 16) * (2.0f / 65535.0f), nz = 0, nw = 0;
	nx = nx + -1.0f, ny = ny + -1.0f, nz = nz + 1.0f, nw = nw + -1.0f;
	float l = nx * -nx + ny * -ny + nz * -nw;
	nz = l, l = sqrtf( l ), nx *= l, ny *= l;
	return mk3( nx * 2.0f + 0.0f, ny * 2.0f + 0.0f, nz * 2.0f + -1.0f );
}
LH2_DEV v3 SampleSkydome( const SceneDev& s, const v3 D )
{
	const uint32_t u = lh2_f2u( (float)s.skyW * 0.5f * (1.0f + lh2_atan2f( D.x, -D.z ) * INVPI) );
	const uint32_t v = lh2_f2u( (float)s.skyH * lh2_acosf( D.y ) * INVPI );
	const uint32_t idx = u + v * (uint32_t)s.skyW;
	if (idx < (uint32_t)(s.skyW * s.skyH)) return mk3( s.sky[idx * 3], s.sky[idx * 3 + 1], s.sky[idx * 3 + 2] );
	return s3( 0 );
}
LH2_DEV v3 SafeOrigin( const v3 O, const v3 R, const v3 N, const float eps )
{
	const float parallel = 1 - fabsf( dot3( N, R ) );
	const float v = parallel * parallel;
	const float side = 1.0f;
	return add3( add3( O, muls( muls( R, eps ), 1 - v ) ), muls( muls( muls( N, side ), eps ), v ) );
}
LH2_DEV v3 clampintensity( const float clampValue, v3 c )
{
	const float v = fmaxf( c.x, fmaxf( c.y, c.z ) );
	if (v > clampValue) { const float m = clampValue / v; c.x *= m; c.y *= m; c.z *= m; }
	return c;
}
LH2_DEV v3 fixnan( v3 a ) { if (!isfinite_( a.x + a.y + a.z )) a = s3( 0 ); return a; }
LH2_DEV float SurvivalProbability( const v3 a ) { return fminf( 1.0f, fmaxf( fmaxf( a.x, a.y ), a.z ) ); }

/* the hit's instance record (lh2_CoreInstanceDesc: triangle pointer, inverse-transform rows A, B, C),
   read in one step of the dependent load chain right after the hit record; none for a miss */
template <bool SINGLE = false>
LH2_DEV const float4* HitInstance( const SceneDev& s, const int primIdx, const int instIdx, v3& A, v3& B, v3& C )
{
	/* branch-free (a miss reads record 0, which always exists: RenderCore::Init allocates it), so the
	   loads stay in flight with the caller's other loads instead of being waited for inside a branch */
	const lh2_CoreInstanceDesc* id = s.instDesc + (primIdx == NOHIT ? 0 : instIdx);
	const float4 a = *(const float4*)&id->A, b = *(const float4*)&id->B, c = *(const float4*)&id->C;
	A = xyz( a ), B = xyz( b ), C = xyz( c );
	/* SINGLE (SceneDev::tris0 set): the triangle's address needs no load, its loads go out beside the instance record's */
	return (SINGLE ? s.tris0 : (const float4*)id->triangles) + (size_t)primIdx * 11;
}

/* a shade launch's input segment: its records (front + back), the front records, and the gap between
   the two ends (two-ended segments, ShadeParams::chordCut) */
LH2_DEV void shade_segment( const ShadeParams& p, const uint32_t seg, uint32_t& count, uint32_t& front, uint32_t& gap )
{
	front = p.segCounts[seg * LH2_SEGCOUNT_STRIDE];
	const uint32_t back = p.segBack ? p.segBack[seg * LH2_SEGCOUNT_STRIDE] : 0u;
	count = front + back;
	gap = back ? p.segStride - count : 0u;
}
/* the record of position i of such a segment (relative to its start) */
LH2_DEV uint32_t seg_pos( const uint32_t i, const uint32_t front, const uint32_t gap ) { return i < front ? i : i + gap; }
/* the distance along the ray from its origin to where it leaves the scene box (a lower bound of what
   it can traverse; ordering only, so a fast reciprocal is fine) */
LH2_DEV float scene_chord( const ShadeParams& p, const float4 o, const float4 d )
{
	const float ix = __builtin_amdgcn_rcpf( d.x ), iy = __builtin_amdgcn_rcpf( d.y ), iz = __builtin_amdgcn_rcpf( d.z );
	const float tx = fmaxf( (p.chordLo[0] - o.x) * ix, (p.chordHi[0] - o.x) * ix );
	const float ty = fmaxf( (p.chordLo[1] - o.y) * iy, (p.chordHi[1] - o.y) * iy );
	const float tz = fmaxf( (p.chordLo[2] - o.z) * iz, (p.chordHi[2] - o.z) * iz );
	return fminf( fminf( tx, ty ), tz );
}
/* one path vertex of shadeKernel (pathtracer.h:54-245): the hit record, ray and path state of a path at
   pathLength in; its extension ray (o.ext) and shadow ray (o.shadow) out.  Shared by k_shade (one launch
   per bounce) and the path-tail kernel (k_trace_path4d: trace and shade in one loop per lane) */
template <bool NL, bool SINGLE, bool EMIT>
LH2_DEV void shade_path( const SceneDev& s, const ShadeParams& p, const uint4 hd, const float4 T4, const float4 O4, const float4 D4, const float4 Q4,
	const int pathLength, const uint32_t R0, ShadeOut& o LH2_STT_PARAM )
{
	const int w = p.w, h = p.h;
	const float HIT_T = __uint_as_float( hd.x );
	const int PRIMIDX = (int)hd.y;
	const int INSTANCEIDX = PRIMIDX == -1 ? 0 : (int)hd.z;
	const float HIT_U = (float)(hd.w & 65535) * (1.0f / 65535.0f);
	const float HIT_V = (float)(hd.w >> 16) * (1.0f / 65535.0f);
	uint32_t data = fbits( T4.w );
	const float bsdfPdf = Q4.x;
	const v3 D = xyz( D4 ), RAY_O = xyz( O4 );
	v3 throughput = xyz( T4 );
	const uint32_t pathIdx = data >> 8;
	const uint32_t pixelIdx = pathIdx % (uint32_t)(w * h);
	const uint32_t sampleIdx = pathIdx / (uint32_t)(w * h) + (uint32_t)p.pass;
	/* this vertex's blue-noise samples (dimensions 4..7 + 4 pathLength: r0, r1 for the light, r3, r4
	   for the BSDF) and the hit's instance record are fetched together, and the sample bytes with
	   the triangle: the dependent chain is inputs -> (ranking bytes, instance) -> (samples,
	   triangle) -> material, instead of the table lookups following the material */
	const BlueNoise4 bnq = blueNoiseFetch4( s.blueNoise, (int)(pixelIdx % (uint32_t)w), (int)(pixelIdx / (uint32_t)w), (int)sampleIdx, 4 + 4 * pathLength );
	v3 instA, instB, instC;
	const float4* tri = HitInstance<SINGLE>( s, PRIMIDX, INSTANCEIDX, instA, instB, instC );
	/* SINGLE: the triangle's records with them (a miss reads the blue-noise table instead: always there, and large
	   enough); else after the instance record, in GetShadingData */
	TriShade tq;
	MatShade mq;
	if (SINGLE) tq = tri_shade_load( PRIMIDX == NOHIT ? (const float4*)s.blueNoise : tri );
	__builtin_amdgcn_sched_barrier( 0 );
	/* SINGLE: the material's loads go out with the blue-noise sample bytes (both wait for the previous step's loads), not
	   after them (a miss reads the blue-noise table again) */
	if (SINGLE)
	{
		mq.mat = PRIMIDX == NOHIT ? (const uint4*)s.blueNoise : s.materials + (size_t)__float_as_int( tq.t1.w ) * 8;
		mq.m0 = mq.mat[0], mq.m1 = mq.mat[1];
	}
	float bnv[4];
	blueNoiseFinish4( s.blueNoise, bnq, bnv );
	LH2_STT( 0 )
	if (pathLength == 1) unsafeAtomicAdd( &p.acc[pixelIdx].w, PRIMIDX == NOHIT ? 10000.0f : HIT_T );
	if (PRIMIDX == NOHIT)
	{
		v3 contribution = muls( mul3( throughput, SampleSkydome( s, D ) ), 1.0f / bsdfPdf );
		contribution = clampintensity( s.clampValue, contribution );
		contribution = fixnan( contribution );
		acc_add( p.acc, pixelIdx, contribution );
		return;
	}
	if ((int)pixelIdx == p.probePixel && pathLength == 1 && sampleIdx == 0)
		p.counters->probedInstid = INSTANCEIDX, p.counters->probedTriid = PRIMIDX, p.counters->probedDist = HIT_T;
	{
		ShadingData sd;
		v3 N, iN, fN, T;
		const v3 I = add3( RAY_O, smul( HIT_T, D ) );
		if (!SINGLE) tq = tri_shade_load( tri ), mq = mat_shade_load( s, tq );
		GetShadingData( s, D, HIT_U, HIT_V, p.spreadAngle * HIT_T, tri, tq, mq, instA, instB, instC, sd, N, iN, fN, T );
		LH2_STT( 1 )
		if (sd.flags & 1)
		{
			if (pathLength < p.maxPathLength)
			{
				throughput = fixnan( throughput );
				o.ext = true;
				o.eO = make_float4( I.x, I.y, I.z, EPSILON ), o.eD = make_float4( D.x, D.y, D.z, 1e34f );
				o.eT = make_float4( throughput.x, throughput.y, throughput.z, bitsf( data ) ), o.eQ = make_float4( bsdfPdf, 0, 0, 0 );
			}
			return;
		}
		if (sd.color.x > 1.0f || sd.color.y > 1.0f || sd.color.z > 1.0f)
		{
			const float DdotNL = -dot3( D, N );
			v3 contribution = s3( 0 );
			if (DdotNL > 0)
			{
				if (pathLength == 1 || (data & S_SPECULAR) > 0) contribution = sd.color;
				else
				{
					const v3 lastN = UnpackNormal( fbits( Q4.y ) );
					const float4 tdata0 = tri[0], tdata5 = tq.t5;
					const float lightPdf = (HIT_T * HIT_T) / (-dot3( D, N ) * tdata5.w);     /* CalculateLightPDF, tri.area */
					const float pickProb = LightPickProb( s, __float_as_int( tdata0.w ), RAY_O, lastN, I );
					if ((bsdfPdf + lightPdf * pickProb) > 0) contribution = muls( mul3( throughput, sd.color ), 1.0f / (bsdfPdf + lightPdf * pickProb) );
				}
				contribution = clampintensity( s.clampValue, contribution );
				contribution = fixnan( contribution );
				acc_add( p.acc, pixelIdx, contribution );
			}
			return;
		}
		if (ROUGHNESS <= 0.001f || TRANSMISSION > 0.999f) data |= S_SPECULAR; else data &= ~S_SPECULAR;
		uint32_t seed = WangHash( pathIdx * 17 + R0 );
		const float faceDir = (dot3( D, N ) > 0) ? -1 : 1;
		if (faceDir == 1) sd.transmittance = s3( 0 );
		throughput = muls( throughput, 1.0f / bsdfPdf );
		if (NL && !(data & S_SPECULAR) && sampleIdx >= 2) (void)RandomFloat( seed ), (void)RandomFloat( seed );
		LH2_STT( 2 )
		if (!NL && !(data & S_SPECULAR))
		{
			float r0, r1, pickProb = 0, lightPdf = 0;
			if (sampleIdx < 2) r0 = bnv[0], r1 = bnv[1];
			else
			{
				r0 = RandomFloat( seed );
				r1 = RandomFloat( seed );
			}
			v3 lightColor = s3( 0 );
			v3 L = sub3( RandomPointOnLight( s, r0, r1, I, muls( fN, faceDir ), pickProb, lightPdf, lightColor ), I );
			LH2_STT( 3 )
			const float dist = length3( L );
			L = muls( L, 1.0f / dist );
			const float NdotL = dot3( L, muls( fN, faceDir ) );
			if (NdotL > 0 && lightPdf > 0)
			{
				float bsdfPdf2;
				const v3 sampledBSDF = EvaluateBSDF( sd, fN, T, muls( D, -1.0f ), L, bsdfPdf2 );
				if (bsdfPdf2 > 0)
				{
					v3 contribution = muls( mul3( mul3( throughput, sampledBSDF ), lightColor ), NdotL / (pickProb * lightPdf + bsdfPdf2) );
					contribution = fixnan( contribution );
					contribution = clampintensity( s.clampValue, contribution );
					const v3 so = SafeOrigin( I, L, muls( N, faceDir ), s.geometryEpsilon );
					const float4 sO = make_float4( so.x, so.y, so.z, 0 ), sD = make_float4( L.x, L.y, L.z, dist - 2 * s.geometryEpsilon );
					const float4 sP = make_float4( contribution.x, contribution.y, contribution.z, __uint_as_float( pixelIdx ) );
					if (EMIT)
					{
						/* k_shade (round 6): the shadow ray goes into the block's shadow segment here, one atomic for the lanes
						   that reach this point, so its twelve registers are not live across SampleBSDF */
						uint64_t rem = __ballot( true );
						while (rem)   /* k_shade: one segment per wave; the path tail: each lane its path's segment */
						{
							const uint32_t l0 = (uint32_t)__builtin_ctzll( rem );
							const uint32_t segv = (uint32_t)__builtin_amdgcn_readlane( (int)o.seg, l0 );
							const uint64_t mm = __ballot( o.seg == segv ) & rem;
							uint32_t b = 0;
							if (lane_id() == l0) b = atomicAdd( &p.counters->segShadow[segv * LH2_SEGCOUNT_STRIDE], (uint32_t)__popcll( mm ) );
							b = (uint32_t)__builtin_amdgcn_readlane( (int)b, l0 );
							if ((mm >> lane_id()) & 1ull)
							{
								const uint32_t ss = b + lanes_below( mm );
								if (ss < p.shadowStride) { const uint32_t so2 = segv * p.shadowStride + ss; p.shO[so2] = sO; p.shD[so2] = sD; p.shP[so2] = sP; }
								else atomicOr( &p.counters->shadowOverflow, 1u );
							}
							rem &= ~mm;
						}
					}
					else o.shadow = true, o.sO = sO, o.sD = sD, o.sP = sP;
				}
			}
		}
		LH2_STT( 4 )
		if (data & ENOUGH_BOUNCES || pathLength == p.maxPathLength) return;
		{
			v3 R = s3( 0 );
			float newBsdfPdf = 0, r3, r4;
			if (sampleIdx < 256) r3 = bnv[2], r4 = bnv[3];
			else
			{
				r3 = RandomFloat( seed );
				r4 = RandomFloat( seed );
			}
			bool specular = false;
			const v3 bsdf = SampleBSDF( sd, fN, N, T, muls( D, -1.0f ), HIT_T, r3, r4, R, newBsdfPdf, specular );
			LH2_STT( 5 )
			if (newBsdfPdf < EPSILON || newBsdfPdf != newBsdfPdf) return;
			if (specular) data |= S_SPECULAR;
			const float pr = ((data & S_SPECULAR) || ((data & S_BOUNCED) == 0)) ? 1 : SurvivalProbability( bsdf );
			if (pr < RandomFloat( seed )) return;
			throughput = muls( throughput, 1 / pr );
			const uint32_t packedNormal = PackNormal( muls( fN, faceDir ) );
			if (!(data & S_SPECULAR)) data |= data & S_BOUNCED ? S_BOUNCEDTWICE : S_BOUNCED; else data |= S_VIASPECULAR;
			const v3 eo = SafeOrigin( I, R, muls( N, faceDir ), s.geometryEpsilon );
			throughput = fixnan( throughput );
			const v3 nt = muls( mul3( throughput, bsdf ), fabsf( dot3( muls( fN, faceDir ), R ) ) );
			o.ext = true;
			o.eO = make_float4( eo.x, eo.y, eo.z, 0 ), o.eD = make_float4( R.x, R.y, R.z, 1e34f );
			o.eT = make_float4( nt.x, nt.y, nt.z, bitsf( data ) ), o.eQ = make_float4( newBsdfPdf, bitsf( packedNormal ), 0, 0 );
			LH2_STT( 6 )
		}
	}
}

/* ---- shade kernel: pathtracer.h:54-245 --------------------------------------------------- */
LH2_DEV void shade_epilogue( const ShadeParams& p );   /* the bounce hand-off, below */
/* 4 waves per SIMD (<= 128 VGPRs): the kernel is load-latency bound (a dependent chain of hit ->
   instance -> triangle -> material loads per path).  Round 1: 3 waves over the unbounded 171-VGPR
   build, 0.285 -> 0.244 ms on config 2; round 2 (no SLP, 145 VGPRs unbounded): 4 waves at 128 VGPRs
   + 36 B of spills, config-3 shade 0.565 -> 0.548 ms per frame (profiles/r02s_ab_collapse_shade4.txt) */
#ifndef LH2_SHADE_MINWAVES
#define LH2_SHADE_MINWAVES 4
#endif
/* k_shade writes each shadow ray where shade_path makes it (EMIT), not in the end-of-iteration compaction */
#ifndef LH2_SHADE_EMIT
#define LH2_SHADE_EMIT 1
#endif
#ifndef LH2_SHADE_NL_MINWAVES
#define LH2_SHADE_NL_MINWAVES 4   /* 128 VGPRs, 9 spilled; 3 waves: 144, none (A/B: profiles/r01g_ab_shade_nolights.jsonl) */
#endif
/* NL: a scene without lights.  NEE (pathtracer.h:168-208) then never yields a shadow ray
   (RandomPointOnLight: lightPdf 0), so its code is compiled out, except the two random numbers it
   draws past sample 1, which later draws depend on */
template <bool TERM, bool NL, bool SINGLE>
__global__ __launch_bounds__( 256, NL ? LH2_SHADE_NL_MINWAVES : LH2_SHADE_MINWAVES ) void k_shade( const SceneDev s, const ShadeParams p )
{
	/* the block's segment of the path stream (its XCD's), and the segment's share of the grid */
	const uint32_t seg = blockIdx.x % LH2_SEGS;
	uint32_t count, front, gap;
	shade_segment( p, seg, count, front, gap );
	if (*s.sceneError) count = 0;   /* the trace kernels refused the scene (they exited): no hit record is this frame's */
	const uint32_t segBase = seg * p.segStride;
	const uint32_t gstride = ((gridDim.x - seg + LH2_SEGS - 1) / LH2_SEGS) * 256u;
	const int w = p.w, h = p.h;
	if (p.hvZero)
		for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < p.hvZeroWords; i += gridDim.x * 256u) p.hvZero[i] = 0;
	for (uint32_t base = (blockIdx.x / LH2_SEGS) * 256u; base < count; base += gstride)
	{
#ifdef LH2_SHADE_TIMES
		uint64_t stt = __builtin_amdgcn_s_memtime(), *const sttp = &stt;
#endif
		const uint32_t jobIndex = segBase + seg_pos( base + threadIdx.x, front, gap );
		bool doExt = false, doShadow = false;
		float4 eO, eD, eT, eQ, sO, sD, sP;
		if (base + threadIdx.x < count)
		{
			/* the five input records first, all in flight together (the hit starts the dependent chain) */
			const uint4 hd = p.hits[jobIndex];
			const float4 T4 = p.T4[jobIndex];
			/* ShadeParams::terminal: a hit that cannot extend ends here with no contribution (emission
			   at :127-153 needs colour > 1, NEE at :168-208 a light, :211 stops the extension) */
			if (TERM && (int)hd.y != NOHIT && ((fbits( T4.w ) & ENOUGH_BOUNCES) || p.pathLength == p.maxPathLength)) goto compact;
			const float4 O4 = p.rayO[jobIndex], D4 = p.rayD[jobIndex], Q4 = p.Q4[jobIndex];
			__builtin_amdgcn_sched_barrier( 0 );
			ShadeOut so;
			so.ext = so.shadow = false, so.seg = seg;
#ifdef LH2_SHADE_TIMES
			shade_path<NL, SINGLE, LH2_SHADE_EMIT != 0>( s, p, hd, T4, O4, D4, Q4, p.pathLength, p.R0, so, &stt );
#else
			shade_path<NL, SINGLE, LH2_SHADE_EMIT != 0>( s, p, hd, T4, O4, D4, Q4, p.pathLength, p.R0, so );
#endif
			doExt = so.ext, doShadow = so.shadow;
			eO = so.eO, eD = so.eD, eT = so.eT, eQ = so.eQ, sO = so.sO, sD = so.sD, sP = so.sP;
		}
	compact:
		/* wave-level compaction of extension and shadow rays into this block's segment of the output
		   streams (one atomicAdd per wave each, on the segment's own counter) */
		{
			/* two-ended segment: a ray with a short chord through the scene goes to the end (traced last) */
			const bool late = doExt && p.chordCut > 0 && scene_chord( p, eO, eD ) <= p.chordCut;
			const uint64_t mE = __ballot( doExt && !late ), mB = __ballot( late ), mS = __ballot( doShadow );
			uint32_t bE, bB, bS;
			wave_alloc3( mE, mB, mS, &p.segOut[seg * LH2_SEGCOUNT_STRIDE], p.segOutBack ? &p.segOutBack[seg * LH2_SEGCOUNT_STRIDE] : nullptr,
				&p.counters->segShadow[seg * LH2_SEGCOUNT_STRIDE], bE, bB, bS );
			const uint32_t es = bE + lanes_below( mE ), eb = bB + lanes_below( mB );
			if (doExt)
			{
				const uint32_t o = segBase + (late ? p.segStride - 1u - eb : es);
				p.rayOut[o] = eO; p.rayDOut[o] = eD; p.T4Out[o] = eT; p.Q4Out[o] = eQ;
			}
			/* shadow rays into the block's segment of the shadow stream */
			const uint32_t ss = bS + lanes_below( mS );
			if (doShadow)
			{
				if (ss < p.shadowStride) { const uint32_t o = seg * p.shadowStride + ss; p.shO[o] = sO; p.shD[o] = sD; p.shP[o] = sP; }
				else atomicOr( &p.counters->shadowOverflow, 1u );
			}
		}
		LH2_STT( 7 )
	}
	if (p.advance) shade_epilogue( p );
}

/* ShadeParams::terminal at the last vertex (pathLength == maxPathLength): k_shade<true> would drop
   every hit, so the pass is the misses' sky samples (pathtracer.h:87-93, the same arithmetic as
   k_shade's miss branch) and nothing else: a small kernel at full occupancy instead of the 3-wave
   shade.  An all-zero contribution (no sky) is not added: x + 0 == x for every accumulator value */
__global__ __launch_bounds__( 256 ) void k_shade_last( const SceneDev s, const ShadeParams p )
{
	const uint32_t seg = blockIdx.x % LH2_SEGS;
	uint32_t count, front, gap;
	shade_segment( p, seg, count, front, gap );
	if (*s.sceneError) count = 0;   /* the trace kernels refused the scene (they exited): no hit record is this frame's */
	const uint32_t segBase = seg * p.segStride;
	const uint32_t gstride = ((gridDim.x - seg + LH2_SEGS - 1) / LH2_SEGS) * 256u;
	const uint32_t wh = (uint32_t)(p.w * p.h);
	for (uint32_t i = (blockIdx.x / LH2_SEGS) * 256u + threadIdx.x; i < count; i += gstride)
	{
		const uint32_t jobIndex = segBase + seg_pos( i, front, gap );
		if ((int)p.hits[jobIndex].y != NOHIT) continue;
		const float4 T4 = p.T4[jobIndex], D4 = p.rayD[jobIndex], Q4 = p.Q4[jobIndex];
		const uint32_t pixelIdx = (fbits( T4.w ) >> 8) % wh;
		v3 contribution = muls( mul3( xyz( T4 ), SampleSkydome( s, xyz( D4 ) ) ), 1.0f / Q4.x );
		contribution = clampintensity( s.clampValue, contribution );
		contribution = fixnan( contribution );
		if (contribution.x != 0 || contribution.y != 0 || contribution.z != 0) acc_add( p.acc, pixelIdx, contribution );
	}
}

/* the path tail: bounces shp.pathLength .. maxPathLength in one launch (lh2_trace4d.inc, KIND 3): each
   lane traces its path's ray, shades the hit with k_shade's code in batches of shadeBatch lanes and walks
   on with the extension ray in place, so a path's later bounces do not wait for every other path's
   (the few rays of the deep bounces run latency-bound: config 3's bounces 3 and 4 took 292 + 200 us for
   ~0.6 M rays as launches of their own).  The shade code's registers set the occupancy */
/* W: the waves per SIMD the kernel is compiled for.  3: the lit variant's 168 VGPRs, no spills; 4: 128 VGPRs and ~190 B
   of spills.  Beside the side shadow launch a large frame's tail phase is 3 % faster with 4 (the 4K frame 6.58 -> 6.39 ms),
   a small frame's 3.5 % slower (the N = 8 share 1.125 -> 1.165 ms, profiles/r04w_ab.txt): TraceArgs::tailWaves picks */
template <bool NL, bool SINGLE, int W>
__global__ __launch_bounds__( 256, W ) void k_trace_path4d( const SceneDev s, const TraceArgs a, const ShadeParams p )
{
	__shared__ int lstack[LH2_STACK_LDS * 256];
	__shared__ __attribute__( (aligned( 4096 )) ) int lrefs[4 * 256];
	trace_stream4d<3, SINGLE, NL>( s, a, lstack + threadIdx.x, lrefs + threadIdx.x, blockIdx.x * 256 + threadIdx.x, gridDim.x * 256u, &p );
}

/* counters: .cuda.cu:64-84 */
/* =====================================================================================
   PrimeRef validation mode: RenderCore_PrimeRef/kernels/pathtracer.h:44-165 with its Lambert
   BSDF (kernels/bsdf.h:18-101): uniform random numbers, NEE without MIS, Russian roulette at
   every vertex, MAXPATHLENGTH 64, no clamping.  Defined where the reference is undefined: a
   total-internal-reflection sample leaves the direction (0,0,0) (bsdf.h:75 returns before
   writing wi), and alpha cut-outs are shaded as hits (this pathtracer never tests the flag).
   ===================================================================================== */
LH2_DEV float Fr_Lambert( const float VDotN, const float eio )   /* bsdf.h:18-26 */
{
	const float SinThetaT2 = sqrf( eio ) * (1.0f - VDotN * VDotN);
	if (SinThetaT2 > 1.0f) return 1.0f;
	const float LDotN = sqrtf( 1.0f - SinThetaT2 );
	const float r1 = (VDotN - eio * LDotN) / (VDotN + eio * LDotN);
	const float r2 = (LDotN - eio * VDotN) / (LDotN + eio * VDotN);
	return 0.5f * (sqrf( r1 ) + sqrf( r2 ));
}
LH2_DEV v3 Tangent2World1( const v3 V, const v3 N )   /* tools_shared.h:211-220, "Building an Orthonormal Basis, Revisited" */
{
	const float sign = copysignf( 1.0f, N.z );
	const float a = -1.0f / (sign + N.z);
	const float b = N.x * N.y * a;
	const v3 B = mk3( 1.0f + sign * N.x * N.x * a, sign * b, -sign * N.x );
	const v3 T = mk3( b, sign + N.y * N.y * a, -N.y );
	return add3( add3( smul( V.x, T ), smul( V.y, B ) ), smul( V.z, N ) );
}
LH2_DEV v3 EvaluateBSDF_Lambert( const ShadingData& sd, const v3 iN, const v3 wi, float& pdf )   /* bsdf.h:40-51 */
{
	if (TRANSMISSION > 0.999f || ROUGHNESS <= 0.001f) { pdf = 0; return s3( 0 ); }
	pdf = fabsf( dot3( wi, iN ) ) * INVPI;
	return muls( muls( sd.color, INVPI ), ROUGHNESS );
}
LH2_DEV v3 SampleBSDF_Lambert( const ShadingData& sd, v3 iN, const v3 N, const v3 wo, const float distance, const float r3, const float r4,
	v3& wi, float& pdf, bool& specular )   /* bsdf.h:53-101 */
{
	const float flip = (dot3( wo, N ) < 0) ? -1 : 1;
	iN = muls( iN, flip );
	specular = true, pdf = 1;
	v3 bsdf;
	if (r4 < TRANSMISSION)
	{
		const float eio = flip < 0 ? (1.0f / ETA) : ETA, F = Fr_Lambert( dot3( iN, wo ), eio );
		const v3 beer = mk3( lh2_expf( -sd.transmittance.x * distance * 2.0f ), lh2_expf( -sd.transmittance.y * distance * 2.0f ),
			lh2_expf( -sd.transmittance.z * distance * 2.0f ) );
		if (r3 < F)
		{
			wi = reflect3( muls( wo, -1.0f ), iN );
			bsdf = muls( mul3( sd.color, beer ), 1 / fabsf( dot3( iN, wi ) ) );
		}
		else
		{
			if (!Refract_L( wo, iN, eio, wi )) return s3( 0 );
			return muls( mul3( sd.color, beer ), 1 / fabsf( dot3( iN, wi ) ) );
		}
	}
	else
	{
		const float pReflect = 1 - ROUGHNESS;
		if (r3 < pReflect)
		{
			wi = reflect3( muls( wo, -1.0f ), iN );
			bsdf = muls( sd.color, 1.0f / fabsf( dot3( iN, wi ) ) );
		}
		else
		{
			const float r5 = (r3 - pReflect) / (1 - pReflect);
			const float r6 = (r4 - TRANSMISSION) / (1 - TRANSMISSION);
			wi = normalize3( Tangent2World1( DiffuseReflectionCosWeighted( r5, r6 ), iN ) );
			pdf = fmaxf( 0.0f, dot3( wi, iN ) ) * INVPI;
			specular = false;
			bsdf = muls( sd.color, INVPI );
		}
	}
	if (dot3( muls( N, flip ), wi ) <= 0) pdf = 0;   /* APPLYSAFENORMALS */
	return bsdf;
}

__global__ __launch_bounds__( 256, LH2_SHADE_MINWAVES ) void k_shade_ref( const SceneDev s, const ShadeParams p )
{
	/* the block's segment of the path stream (its XCD's), and the segment's share of the grid */
	const uint32_t seg = blockIdx.x % LH2_SEGS;
	uint32_t count, front, gap;
	shade_segment( p, seg, count, front, gap );
	if (*s.sceneError) count = 0;   /* the trace kernels refused the scene (they exited): no hit record is this frame's */
	const uint32_t segBase = seg * p.segStride;
	const uint32_t gstride = ((gridDim.x - seg + LH2_SEGS - 1) / LH2_SEGS) * 256u;
	const int w = p.w, h = p.h;
	for (uint32_t base = (blockIdx.x / LH2_SEGS) * 256u; base < count; base += gstride)
	{
		const uint32_t jobIndex = segBase + seg_pos( base + threadIdx.x, front, gap );
		bool doExt = false, doShadow = false;
		float4 eO, eD, eT, eQ, sO, sD, sP;
		if (base + threadIdx.x < count)
		{
			const uint4 hd = p.hits[jobIndex];
			const float4 T4 = p.T4[jobIndex], O4 = p.rayO[jobIndex], D4 = p.rayD[jobIndex];
			__builtin_amdgcn_sched_barrier( 0 );
			const float HIT_T = __uint_as_float( hd.x );
			const int PRIMIDX = (int)hd.y;
			const int INSTANCEIDX = PRIMIDX == -1 ? 0 : (int)hd.z;
			const float HIT_U = (float)(hd.w & 65535) * (1.0f / 65535.0f);
			const float HIT_V = (float)(hd.w >> 16) * (1.0f / 65535.0f);
			v3 instA, instB, instC;
			const float4* tri = HitInstance( s, PRIMIDX, INSTANCEIDX, instA, instB, instC );
			uint32_t data = fbits( T4.w );
			const v3 D = xyz( D4 ), RAY_O = xyz( O4 );
			v3 throughput = xyz( T4 );
			const uint32_t pathIdx = data >> 8;
			const uint32_t pixelIdx = pathIdx % (uint32_t)(w * h);
			const uint32_t sampleIdx = pathIdx / (uint32_t)(w * h) + (uint32_t)p.pass;
			if (p.pathLength == 1) unsafeAtomicAdd( &p.acc[pixelIdx].w, PRIMIDX == NOHIT ? 10000.0f : HIT_T );
			if (PRIMIDX == NOHIT)
			{
				acc_add( p.acc, pixelIdx, mul3( throughput, SampleSkydome( s, D ) ) );
				goto compact;
			}
			if ((int)pixelIdx == p.probePixel && p.pathLength == 1 && sampleIdx == 0)
				p.counters->probedInstid = INSTANCEIDX, p.counters->probedTriid = PRIMIDX, p.counters->probedDist = HIT_T;
			{
				ShadingData sd;
				v3 N, iN, fN, T;
				const v3 I = add3( RAY_O, smul( HIT_T, D ) );
				const TriShade tq = tri_shade_load( tri );
				GetShadingData( s, D, HIT_U, HIT_V, p.spreadAngle * HIT_T, tri, tq, mat_shade_load( s, tq ), instA, instB, instC, sd, N, iN, fN, T );
				if (sd.color.x > 1.0f || sd.color.y > 1.0f || sd.color.z > 1.0f)
				{
					if (-dot3( D, N ) > 0 && (p.pathLength == 1 || (data & S_SPECULAR))) acc_add( p.acc, pixelIdx, mul3( throughput, sd.color ) );
					goto compact;
				}
				if (ROUGHNESS <= 0.001f || TRANSMISSION > 0.999f) data |= S_SPECULAR; else data &= ~S_SPECULAR;
				uint32_t seed = WangHash( pathIdx * 17 + p.R0 );
				const float faceDir = (dot3( D, N ) > 0) ? -1 : 1;
				if (faceDir == 1) sd.transmittance = s3( 0 );
				if (!(data & S_SPECULAR))
				{
					const float r0 = RandomFloat( seed ), r1 = RandomFloat( seed );
					float pickProb = 0, lightPdf = 0;
					v3 lightColor = s3( 0 );
					v3 L = sub3( RandomPointOnLight( s, r0, r1, I, muls( fN, faceDir ), pickProb, lightPdf, lightColor ), I );
					const float dist = length3( L );
					L = muls( L, 1.0f / dist );
					const float NdotL = dot3( L, muls( fN, faceDir ) );
					if (NdotL > 0 && lightPdf > 0 && p.pathLength < p.maxPathLength)   /* the last bounce's shadow rays are never traced (rendercore.cpp loop break) */
					{
						float bsdfPdf;
						const v3 sampledBSDF = EvaluateBSDF_Lambert( sd, fN, L, bsdfPdf );
						const v3 contribution = muls( mul3( mul3( throughput, sampledBSDF ), lightColor ), NdotL / (pickProb * lightPdf) );
						const v3 so = SafeOrigin( I, L, muls( N, faceDir ), s.geometryEpsilon );
						doShadow = true;
						sO = make_float4( so.x, so.y, so.z, 0 );
						sD = make_float4( L.x, L.y, L.z, dist - 2 * s.geometryEpsilon );
						sP = make_float4( contribution.x, contribution.y, contribution.z, __uint_as_float( pixelIdx ) );
					}
				}
				const float r3 = RandomFloat( seed ), r4 = RandomFloat( seed ), r5 = RandomFloat( seed );
				v3 R = s3( 0 );
				float newBsdfPdf = 0;
				bool specular = false;
				const v3 bsdf = SampleBSDF_Lambert( sd, fN, N, muls( D, -1.0f ), HIT_T, r3, r4, R, newBsdfPdf, specular );
				if (newBsdfPdf < EPSILON || newBsdfPdf != newBsdfPdf) goto compact;
				if (specular) data |= S_SPECULAR;
				const float pr = p.pathLength == p.maxPathLength ? 0 : ((data & S_SPECULAR) ? 1 : SurvivalProbability( bsdf ));
				if (pr <= r5) goto compact;
				throughput = mul3( throughput, divs( muls( bsdf, fabsf( dot3( fN, R ) ) ), pr * newBsdfPdf ) );
				const v3 eo = SafeOrigin( I, R, muls( N, faceDir ), s.geometryEpsilon );
				doExt = true;
				eO = make_float4( eo.x, eo.y, eo.z, 0 ), eD = make_float4( R.x, R.y, R.z, 1e34f );
				eT = make_float4( throughput.x, throughput.y, throughput.z, bitsf( data ) ), eQ = make_float4( 1, 0, 0, 0 );
			}
		}
	compact:
		{
			/* two-ended segment: a ray with a short chord through the scene goes to the end (traced last) */
			const bool late = doExt && p.chordCut > 0 && scene_chord( p, eO, eD ) <= p.chordCut;
			const uint32_t es = wave_alloc( doExt && !late, &p.segOut[seg * LH2_SEGCOUNT_STRIDE] );
			const uint32_t eb = wave_alloc( late, &p.segOutBack[seg * LH2_SEGCOUNT_STRIDE] );
			if (doExt)
			{
				const uint32_t o = segBase + (late ? p.segStride - 1u - eb : es);
				p.rayOut[o] = eO; p.rayDOut[o] = eD; p.T4Out[o] = eT; p.Q4Out[o] = eQ;
			}
			const uint32_t ss = wave_alloc( doShadow, &p.counters->segShadow[seg * LH2_SEGCOUNT_STRIDE] );
			if (doShadow)
			{
				if (ss < p.shadowStride) { const uint32_t o = seg * p.shadowStride + ss; p.shO[o] = sO; p.shD[o] = sD; p.shP[o] = sP; }
				else atomicOr( &p.counters->shadowOverflow, 1u );
			}
		}
	}
}

__global__ void k_init_counters( Counters* c, uint32_t pathCount, uint32_t segStride, uint32_t* cursors, int cursorWords, int keep )
{
	init_counters( c, pathCount, segStride, cursors, cursorWords, blockIdx.x * blockDim.x + threadIdx.x, keep );
}
/* the hand-off from bounce L to bounce L + 1 (InitCountersSubsequent, .cuda.cu:76-84): the extension
   rays counted into segNext become the next bounce's paths (the counts ping-pong, Counters::segPath),
   the retired counts of bounce L are zeroed for the shade launch of L + 1; the shadow split's snapshot;
   one thread, after every block of the shade launch of bounce L has finished */
LH2_DEV void advance_bounce( Counters* c, const BounceAdvance& a, const int pathLength, const int resetShadow )
{
	uint32_t ext = 0, sh = 0;
	for (int k = 0; k < LH2_SEGS; k++)
	{
		ext += __hip_atomic_load( &a.segNext[k * LH2_SEGCOUNT_STRIDE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
		ext += __hip_atomic_load( &a.segNextBack[k * LH2_SEGCOUNT_STRIDE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
		a.segRetire[k * LH2_SEGCOUNT_STRIDE] = 0, a.segRetireBack[k * LH2_SEGCOUNT_STRIDE] = 0;
		sh += c->segShadow[k * LH2_SEGCOUNT_STRIDE];
		if (resetShadow) c->segShadow[k * LH2_SEGCOUNT_STRIDE] = 0;
	}
	if (a.shadowSnap)
		for (int k = 0; k < LH2_SEGS; k++)
		{
			const uint32_t n = __hip_atomic_load( &c->segShadow[k * LH2_SEGCOUNT_STRIDE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
			a.shadowSnap[k * LH2_SEGCOUNT_STRIDE] = n, a.shadowCursor[k * LH2_CURSOR_STRIDE] = n;
		}
	a.rayCountLog[pathLength] = ext;     /* rays traced at pathLength + 1 */
	if (a.zeroLog) for (int k = pathLength + 1; k <= LH2_MAX_BOUNCES; k++) a.rayCountLog[k] = 0;
	c->totalExtensionRays += ext;
	c->activePaths = ext;
	if (resetShadow) c->totalShadowRays += sh;
	/* the host's early exit reads this after the launch's stop event (no copy launch) */
	if (a.hostActiveLog) __hip_atomic_store( a.hostActiveLog + pathLength, ext, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
}

/* the end of a shade launch that hands off to the next bounce (ShadeParams::advance): its last block
   to finish runs advance_bounce, so the hand-off needs no launch of its own (one dependent launch,
   ~10 us, less per bounce) */
LH2_DEV void shade_epilogue( const ShadeParams& p )
{
	/* no fences: an agent-scope fence writes back the XCD's L2 (the launch's ray outputs) in every
	   block, +75 us per shade launch on config 2.  The counts are device-scope atomics that every wave
	   waited for (wave_alloc uses their return values) before the block's arrival is issued, so they
	   are performed when the last block reads them with device-scope loads */
	__shared__ uint32_t lastBlock;
	__syncthreads();
	if (threadIdx.x == 0)
		lastBlock = __hip_atomic_fetch_add( &p.counters->shadeDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ) == gridDim.x - 1;
	__syncthreads();
	if (!lastBlock || threadIdx.x != 0) return;
	__hip_atomic_store( &p.counters->shadeDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
	advance_bounce( p.counters, p.adv, p.pathLength, 0 );
}

__global__ void k_counters_next( Counters* c, const BounceAdvance a, int pathLength, int resetShadow )
{
	if (threadIdx.x == 0) advance_bounce( c, a, pathLength, resetShadow );
}
/* rm.rows > 0: only the rows a tile owns (a rank's bands, the k_pack_rows mapping): the other rows are
   other ranks' and are finalized where the frame is gathered */
__global__ void k_finalize( float4* __restrict__ acc, float4* __restrict__ out, const int n, const float scale, const FrameStatsDev fs,
	const RowMap rm )
{
	const int i = threadIdx.x + blockIdx.x * blockDim.x;
	if (blockIdx.x == 0 && fs.hostCounters)
	{
		/* block 0 also hands the frame's counters, ray-count log and scene error to the host's pinned
		   FrameStats (system-scope stores: no device-to-host copy launches at the end): the totals and the shadow
		   stream's segment counts, the words the host reads (RenderCore::Synchronize), not the whole record */
		const uint32_t* src = (const uint32_t*)fs.counters;
		uint32_t* dst = (uint32_t*)fs.hostCounters;
		constexpr int kHead = (int)(offsetof( Counters, segPath ) / 4), kShadow = (int)(offsetof( Counters, segShadow ) / 4);
		const int k = threadIdx.x < kHead ? (int)threadIdx.x : threadIdx.x < kHead + LH2_SEGS ? kShadow + ((int)threadIdx.x - kHead) * LH2_SEGCOUNT_STRIDE : -1;
		if (k >= 0) __hip_atomic_store( dst + k, src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
		for (int k = threadIdx.x; k < LH2_MAX_BOUNCES; k += blockDim.x)
			__hip_atomic_store( fs.hostRayCount + k, fs.rayLog[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
		if (threadIdx.x == 0) __hip_atomic_store( fs.hostSceneError, *fs.sceneError, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
	}
	if (blockIdx.x == 0 && fs.zeroHeads)
		for (int k = threadIdx.x; k < LH2_CURSOR_WORDS; k += blockDim.x) fs.zeroHeads[k] = 0;
	if (i >= n) return;
	int p = i;
	if (rm.rows > 0)
	{
		const int lr = i / rm.w, x = i % rm.w;
		p = (rm.y0 + (lr / rm.band) * rm.bandStride + lr % rm.band) * rm.w + x;
	}
	float4 a = acc[p];
	if (fs.delta)
	{
		/* early shade: this frame's first-vertex contributions join the accumulator now (the depth w: one addition per
		   pixel per frame, as in frame order) */
		const float4 d = fs.delta[p];
		a = make_float4( a.x + d.x, a.y + d.y, a.z + d.z, a.w + d.w );
		acc[p] = a;
		fs.delta[p] = make_float4( 0, 0, 0, 0 );
	}
	out[p] = make_float4( a.x * scale, a.y * scale, a.z * scale, a.w * scale );
}

/* copy the rows this tile owns (local row order) out of the full-frame accumulator, for the
   multi-GPU gather; same row mapping as k_camera */
__global__ void k_pack_rows( const float4* __restrict__ acc, float4* __restrict__ dst, const int w, const int y0, const int band,
	const int bandStride, const int rows )
{
	const int i = threadIdx.x + blockIdx.x * blockDim.x;
	if (i >= rows * w) return;
	const int lr = i / w, x = i % w;
	const int gy = y0 + (lr / band) * bandStride + lr % band;
	dst[i] = acc[gy * w + x];
}

/* the inverse of k_pack_rows: rows packed by another device's core (rank `rank` of the band partition)
   back into this core's accumulator (the in-process multi-device gather, csrc/multidevice.cpp) */
__global__ void k_unpack_rows( const float4* __restrict__ src, float4* __restrict__ acc, const int w, const int y0, const int band,
	const int bandStride, const int rows )
{
	const int i = threadIdx.x + blockIdx.x * blockDim.x;
	if (i >= rows * w) return;
	const int lr = i / w, x = i % w;
	const int gy = y0 + (lr / band) * bandStride + lr % band;
	acc[gy * w + x] = src[i];
}

/* a single wave that idles its stream for `ticks` of the 100 MHz real-time counter (tests of the
   multi-device gather's ordering: MultiDevice setting "gatherStallUs") */
__global__ void k_spin( const unsigned long long ticks )
{
	const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
	while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep( 8 );
}

/* ---- host-side launchers (extern "C", no torch / no HIP types beyond the stream) ---------- */
/* Launches go through hipExtLaunchKernelGGL: its start / stop events are recorded by the kernel's own
   dispatch packet, where a hipEventRecord between two launches costs a barrier packet and ~5 us of
   idle GPU per event (rocprofv3 kernel trace of the config-2 frame); null events: a plain launch. */
#define LH2_LAUNCH( kernel, grid, block, st, ev, ... ) \
	hipExtLaunchKernelGGL( kernel, dim3( grid ), dim3( block ), 0, st, (ev).start, (ev).stop, 0, __VA_ARGS__ )

/* the per-ray loops' kernels over the BVH4: a single-instance scene (tlasRoot4 < 0) takes the loop without instance state
   (lh2_trace4d.inc SINGLE) */
static void launch_closest4d( const SceneDev* s, const TraceArgs* a, int grid, LaunchEvents ev, hipStream_t st )
{
	const bool single = s->tlasRoot4 < 0;
	if (a->traceWaves == 8)
	{
		if (single) LH2_LAUNCH( (k_trace_closest4d<true, 8>), grid, 256, st, ev, *s, *a );
		else LH2_LAUNCH( (k_trace_closest4d<false, 8>), grid, 256, st, ev, *s, *a );
	}
	else if (single) LH2_LAUNCH( (k_trace_closest4d<true, LH2_TRACE_MINWAVES>), grid, 256, st, ev, *s, *a );
	else LH2_LAUNCH( (k_trace_closest4d<false, LH2_TRACE_MINWAVES>), grid, 256, st, ev, *s, *a );
}
static void launch_any4d( const SceneDev* s, const TraceArgs* a, int grid, int fused, LaunchEvents ev, hipStream_t st )
{
	const bool single = s->tlasRoot4 < 0;
	if (fused && single) LH2_LAUNCH( (k_trace_any4d<1, true>), grid, 256, st, ev, *s, *a );
	else if (fused) LH2_LAUNCH( (k_trace_any4d<1, false>), grid, 256, st, ev, *s, *a );
	else if (single) LH2_LAUNCH( (k_trace_any4d<0, true>), grid, 256, st, ev, *s, *a );
	else LH2_LAUNCH( (k_trace_any4d<0, false>), grid, 256, st, ev, *s, *a );
}
static void launch_path4d( const SceneDev* s, const TraceArgs* a, const ShadeParams* p, int grid, LaunchEvents ev, hipStream_t st )
{
	const bool nl = s->nArea + s->nPoint + s->nSpot + s->nDir == 0, single = s->tlasRoot4 < 0;
	if (a->tailWaves == 4)
	{
		if (nl && single) LH2_LAUNCH( (k_trace_path4d<true, true, 4>), grid, 256, st, ev, *s, *a, *p );
		else if (nl) LH2_LAUNCH( (k_trace_path4d<true, false, 4>), grid, 256, st, ev, *s, *a, *p );
		else if (single) LH2_LAUNCH( (k_trace_path4d<false, true, 4>), grid, 256, st, ev, *s, *a, *p );
		else LH2_LAUNCH( (k_trace_path4d<false, false, 4>), grid, 256, st, ev, *s, *a, *p );
	}
	else if (nl && single) LH2_LAUNCH( (k_trace_path4d<true, true, 3>), grid, 256, st, ev, *s, *a, *p );
	else if (nl) LH2_LAUNCH( (k_trace_path4d<true, false, 3>), grid, 256, st, ev, *s, *a, *p );
	else if (single) LH2_LAUNCH( (k_trace_path4d<false, true, 3>), grid, 256, st, ev, *s, *a, *p );
	else LH2_LAUNCH( (k_trace_path4d<false, false, 3>), grid, 256, st, ev, *s, *a, *p );
}
template <class K> static int occupancy( K kernel )
{
	int n = 0;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor( &n, kernel, 256, 0 ) != hipSuccess || n < 1) n = 4;
	return n;
}

extern "C" {
void lh2_launch_init_counters( Counters* c, uint32_t pathCount, uint32_t segStride, uint32_t* cursors, int cursorWords, LaunchEvents ev, hipStream_t st,
	int keepCursor )
{
	LH2_LAUNCH( k_init_counters, (cursorWords + 255) / 256 + 1, 256, st, ev, c, pathCount, segStride, cursors, cursorWords, keepCursor );
}
void lh2_launch_counters_next( Counters* c, const BounceAdvance* a, int pathLength, int resetShadow, LaunchEvents ev, hipStream_t st )
{
	LH2_LAUNCH( k_counters_next, 1, 64, st, ev, c, *a, pathLength, resetShadow );
}
/* lh2_udiv's { m, a, s } for divisor d >= 1: m = floor( 2^32 (2^l - d) / d ) + 1 with l = ceil( log2 d ), a = 1, s = l - 1 */
static void lh2_div_magic( const uint32_t d, uint32_t dv[3] )
{
	if (d <= 1) { dv[0] = 0, dv[1] = 0, dv[2] = 0; return; }
	const uint32_t l = 32u - (uint32_t)__builtin_clz( d - 1u );
	dv[0] = (uint32_t)((((uint64_t)1 << l) - d) * ((uint64_t)1 << 32) / d + 1u), dv[1] = 1, dv[2] = l - 1u;
}
/* the launch-invariant quantities camera_path reads (CameraParams, last fields) */
static CameraParams lh2_camera_derive( const CameraParams& in )
{
	CameraParams c = in;
	const float fw = (float)c.w, fh = (float)c.h;
	c.rightW = { c.right.x / fw, c.right.y / fw, c.right.z / fw };
	c.upH = { c.up.x / fh, c.up.y / fh, c.up.z / fh };
	lh2_div_magic( (uint32_t)c.tileRows * (uint32_t)c.w, c.divTile );
	lh2_div_magic( (uint32_t)c.w, c.divW );
	lh2_div_magic( (uint32_t)c.band, c.divBand );
	return c;
}
void lh2_launch_camera( const CameraParams* p, const uint8_t* bn, float4* rayO, float4* rayD, float4* T4, float4* Q4, int jobCount, LaunchEvents ev, hipStream_t st )
{
	const CameraParams c = lh2_camera_derive( *p );
	const int threads = std::max( std::max( jobCount, 1 ), p->initC ? std::max( p->cursorWords, LH2_SEGS ) : 0 );
	LH2_LAUNCH( k_camera, (threads + 255) / 256, 256, st, ev, c, bn, rayO, rayD, T4, Q4, jobCount );
}
void lh2_launch_trace_primary( const SceneDev* s, const TraceArgs* a, const CameraParams* cp, float4* T4, float4* Q4, int grid, LaunchEvents ev, hipStream_t st )
{
	const CameraParams c = lh2_camera_derive( *cp );
	LH2_LAUNCH( k_trace_primary_packet, grid, 256, st, ev, c, *s, *a, T4, Q4 );
}
void lh2_launch_trace_closest( const SceneDev* s, const TraceArgs* a, int grid, LaunchEvents ev, hipStream_t st )
{
	/* coherent primary rays: packets over the BVH2 (lh2_trace_packet.inc); incoherent rays: the BVH4 loop
	   (lh2_trace4d.inc), or the reference BVH2 loop (traceVersion 1, or no BVH4) */
	if (a->packet) LH2_LAUNCH( k_trace_closest_packet, grid, 256, st, ev, *s, *a );
	else if (a->version == 7 && s->nodes4) launch_closest4d( s, a, grid, ev, st );
	else if (a->leafBatch) LH2_LAUNCH( k_trace_closest<true>, grid, 256, st, ev, *s, *a );
	else LH2_LAUNCH( k_trace_closest<false>, grid, 256, st, ev, *s, *a );
}
void lh2_launch_trace_any( const SceneDev* s, const TraceArgs* a, int grid, int fused, LaunchEvents ev, hipStream_t st )
{
	if (a->version == 7 && s->nodes4) launch_any4d( s, a, grid, fused, ev, st );
	else if (fused) LH2_LAUNCH( k_trace_any<1>, grid, 256, st, ev, *s, *a );
	else LH2_LAUNCH( k_trace_any<0>, grid, 256, st, ev, *s, *a );
}
int lh2_packet_blocks_per_cu( void )
{
	int n = 0;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor( &n, k_trace_closest_packet, 256, 0 ) != hipSuccess) n = 4;
	return n;
}
/* the per-ray traversal kernels' occupancy (persistent grid: CUs x blocks per CU) */
int lh2_trace_blocks_per_cu( int waves )
{
	/* the smallest of the variants' (the global stack is sized for this grid) */
	int n = 0;
	if (waves == 8)
		n = std::min( occupancy( k_trace_closest4d<false, 8> ), occupancy( k_trace_closest4d<true, 8> ) );
	else
		n = std::min( occupancy( k_trace_closest4d<false, LH2_TRACE_MINWAVES> ), occupancy( k_trace_closest4d<true, LH2_TRACE_MINWAVES> ) );
	return n;
}
static int lh2_shade_last_grid( void )   /* k_shade_last: every CU full (occupancy x CUs), at least a block per segment */
{
	static int g = 0;
	if (!g)
	{
		int n = 0, dev = 0, cus = 0;
		if (hipOccupancyMaxActiveBlocksPerMultiprocessor( &n, k_shade_last, 256, 0 ) != hipSuccess || n < 1) n = 4;
		if (hipGetDevice( &dev ) != hipSuccess || hipDeviceGetAttribute( &cus, hipDeviceAttributeMultiprocessorCount, dev ) != hipSuccess || cus < 1) cus = 256;
		g = n * cus < LH2_SEGS ? LH2_SEGS : n * cus;
	}
	return g;
}
void lh2_launch_trace_path( const SceneDev* s, const TraceArgs* a, const ShadeParams* p, int grid, LaunchEvents ev, hipStream_t st )
{
	if (!s->nodes4) return;   /* the host selects the path tail only over a BVH4 */
	launch_path4d( s, a, p, grid, ev, st );
}
int lh2_path_blocks_per_cu( int waves )
{
	if (waves == 4)
		return std::min( occupancy( k_trace_path4d<false, false, 4> ), occupancy( k_trace_path4d<false, true, 4> ) );
	return std::min( occupancy( k_trace_path4d<false, false, 3> ), occupancy( k_trace_path4d<false, true, 3> ) );
}
void lh2_launch_shade( const SceneDev* s, const ShadeParams* p, int grid, LaunchEvents ev, hipStream_t st )
{
	grid = grid < LH2_SEGS ? LH2_SEGS : grid;   /* every segment needs a block */
	if (p->primeRef) LH2_LAUNCH( k_shade_ref, grid, 256, st, ev, *s, *p );
	else if (p->terminal && p->pathLength == p->maxPathLength) LH2_LAUNCH( k_shade_last, lh2_shade_last_grid(), 256, st, ev, *s, *p );
	else if (s->tris0)   /* one instance (SceneDev::tris0): the triangle loads need no instance record */
	{
		if (p->terminal) LH2_LAUNCH( (k_shade<true, true, true>), grid, 256, st, ev, *s, *p );
		else if (s->nArea + s->nPoint + s->nSpot + s->nDir == 0) LH2_LAUNCH( (k_shade<false, true, true>), grid, 256, st, ev, *s, *p );
		else LH2_LAUNCH( (k_shade<false, false, true>), grid, 256, st, ev, *s, *p );
	}
	else if (p->terminal) LH2_LAUNCH( (k_shade<true, true, false>), grid, 256, st, ev, *s, *p );
	else if (s->nArea + s->nPoint + s->nSpot + s->nDir == 0) LH2_LAUNCH( (k_shade<false, true, false>), grid, 256, st, ev, *s, *p );
	else LH2_LAUNCH( (k_shade<false, false, false>), grid, 256, st, ev, *s, *p );
}
void lh2_launch_pack_rows( const float4* acc, float4* dst, int w, int y0, int band, int bandStride, int rows, LaunchEvents ev, hipStream_t st )
{
	if (rows * w <= 0) { if (ev.stop) (void)hipEventRecord( ev.stop, st ); return; }
	LH2_LAUNCH( k_pack_rows, (rows * w + 255) / 256, 256, st, ev, acc, dst, w, y0, band, bandStride, rows );
}
void lh2_launch_unpack_rows( const float4* src, float4* acc, int w, int y0, int band, int bandStride, int rows, LaunchEvents ev, hipStream_t st )
{
	if (rows * w <= 0) { if (ev.stop) (void)hipEventRecord( ev.stop, st ); return; }
	LH2_LAUNCH( k_unpack_rows, (rows * w + 255) / 256, 256, st, ev, src, acc, w, y0, band, bandStride, rows );
}
#ifdef LH2_SHADE_TIMES
void lh2_shade_times( unsigned long long out[16] ) { (void)hipMemcpyFromSymbol( out, HIP_SYMBOL( lh2_shade_tt ), 16 * 8 ); }
#endif
#ifdef LH2_TOUCH
void lh2_touch_set( uint32_t* bitmap, uint32_t triWord, uint32_t words )
{
	const uint32_t bits = bitmap ? words * 32u : 0u;
	(void)hipMemcpyToSymbol( HIP_SYMBOL( lh2_touch ), &bitmap, sizeof( bitmap ) );
	(void)hipMemcpyToSymbol( HIP_SYMBOL( lh2_touchTri ), &triWord, sizeof( triWord ) );
	(void)hipMemcpyToSymbol( HIP_SYMBOL( lh2_touchBits ), &bits, sizeof( bits ) );
}
#endif
void lh2_launch_spin( unsigned long long ticks, hipStream_t st ) { hipLaunchKernelGGL( k_spin, dim3( 1 ), dim3( 64 ), 0, st, ticks ); }
void lh2_launch_finalize( float4* acc, float4* out, int n, float scale, const FrameStatsDev* fs, LaunchEvents ev, hipStream_t st, const RowMap* rm )
{
	const FrameStatsDev none{};
	const RowMap all{};
	if (rm && rm->rows > 0) n = rm->rows * rm->w;
	LH2_LAUNCH( k_finalize, n > 0 ? (n + 255) / 256 : 1, 256, st, ev, acc, out, n, scale, fs ? *fs : none, rm ? *rm : all );
}
}
