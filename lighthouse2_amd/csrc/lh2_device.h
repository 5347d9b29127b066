/* lh2_device.h - device-side data layout and helpers of the MI355X render core.

   Evaluation order of every expression follows the reference kernels (helper_math.h semantics),
   and the core is compiled with -ffp-contract=off, so values are bit-comparable with the CPU
   oracle (oracle/pt_oracle.c).  Box tests are the one exception: they only cull, are padded
   conservatively, and may use FMA (see lh2_kernels.hip, box_test).
*/
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/lh2_detmath.h"

#define LH2_DEV static __device__ __forceinline__

/* ---- scene layout in HBM (all SoA / 16-B aligned records) --------------------------------
   BVH2 node (64 B, child-pair layout): both children's boxes live in the parent, so one visit
   is four coalesced 16-B loads and tests two boxes.
     n0 = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
     n1 = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
     n2 = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
     n3 = (c0ref, c1ref, -, -)  ref >= 0: interior node index; ref < 0: leaf, ~ref = first<<4 | (count-1)
   BVH4 node (128 B, one cache line): four children as six planes of four (child 0..3 in .x...w), so a
   ray loads its near and far plane of each axis by its direction's signs (two loads per axis, no
   min / max to order them), then the four references; unused slots have NaN boxes.
     q0 = lo.x, q1 = hi.x, q2 = lo.y, q3 = hi.y, q4 = lo.z, q5 = hi.z   (children 0..3)
     q6 = (ref0, ref1, ref2, ref3), q7 = 0
   Triangle (48 B, leaf order): (v0.xyz, original index), (e1 = v1-v0, 0), (e2 = v2-v0, 0)
   Instance (64 B): inverse transform rows 0..2, (bvhRoot, triBase, mesh, bvh4Root)          */
struct alignas( 16 ) DevInstance
{
	float4 inv0, inv1, inv2;
	int root, triBase, mesh, root4;
};

#define LEAF_FIRST(ref) ((uint32_t)(~(ref)) >> 4)
#define LEAF_COUNT(ref) ((int)((uint32_t)(~(ref)) & 15u) + 1)
#define MAKE_LEAF(first, count) ((int)~(((uint32_t)(first) << 4) | (uint32_t)((count) - 1)))

struct Counters   /* core_settings.h:81-91 plus device-side error flags */
{
	/* totals kept by the camera launch and the bounce hand-off (advance_bounce: the last block of a
	   shade launch, or k_counters_next; activePaths: paths of the next bounce); the rays themselves are
	   counted per segment below, and the host sums segShadow for the statistics (extensionRays,
	   shadowRays stay 0) */
	uint32_t activePaths, extensionRays, shadowRays, totalExtensionRays;
	uint32_t totalShadowRays; int probedInstid, probedTriid; float probedDist;
	uint32_t reserved0, shadowOverflow, shadeDone, pad1;   /* shadeDone: blocks of the running shade launch that finished */
	uint32_t pad2[20];
	/* per-segment counts of the segmented streams (lh2_kernels.h, LH2_SEGS), 128 B apart.  The path
	   counts ping-pong: the paths of pathLength L are counted in segPath / segBack[(L - 1) & 1], and
	   its shade launch counts the extension rays (pathLength L + 1) into [L & 1].  A path segment is
	   two-ended: segPath[k] records from its start, segBack[k] from its end (ShadeParams::chordCut: the
	   rays with a short chord through the scene go to the end, so they are traced last); shadow rays are
	   queued per segment */
	uint32_t segPath[2][8 * 32], segBack[2][8 * 32], segShadow[8 * 32];
};

/* ---- small vector helpers with the reference's evaluation order --------------------------- */
struct v3 { float x, y, z; };
LH2_DEV v3 mk3( float x, float y, float z ) { v3 r; r.x = x, r.y = y, r.z = z; return r; }
LH2_DEV v3 s3( float s ) { return mk3( s, s, s ); }
LH2_DEV v3 add3( v3 a, v3 b ) { return mk3( a.x + b.x, a.y + b.y, a.z + b.z ); }
LH2_DEV v3 sub3( v3 a, v3 b ) { return mk3( a.x - b.x, a.y - b.y, a.z - b.z ); }
LH2_DEV v3 mul3( v3 a, v3 b ) { return mk3( a.x * b.x, a.y * b.y, a.z * b.z ); }
LH2_DEV v3 muls( v3 a, float s ) { return mk3( a.x * s, a.y * s, a.z * s ); }
LH2_DEV v3 smul( float s, v3 a ) { return mk3( s * a.x, s * a.y, s * a.z ); }
LH2_DEV v3 divs( v3 a, float s ) { return mk3( a.x / s, a.y / s, a.z / s ); }
LH2_DEV v3 adds( v3 a, float s ) { return mk3( a.x + s, a.y + s, a.z + s ); }
LH2_DEV v3 sadd( float s, v3 a ) { return mk3( s + a.x, s + a.y, s + a.z ); }
LH2_DEV float dot3( v3 a, v3 b ) { return a.x * b.x + a.y * b.y + a.z * b.z; }
LH2_DEV v3 cross3( v3 a, v3 b ) { return mk3( a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x ); }
LH2_DEV float length3( v3 v ) { return sqrtf( dot3( v, v ) ); }
LH2_DEV v3 normalize3( v3 v ) { const float invLen = 1.0f / sqrtf( dot3( v, v ) ); return muls( v, invLen ); }
LH2_DEV v3 reflect3( v3 i, v3 n ) { return sub3( i, muls( smul( 2.0f, n ), dot3( n, i ) ) ); }
LH2_DEV float lerpf_( float a, float b, float t ) { return a + t * (b - a); }
LH2_DEV float saturatef_( float x ) { return fmaxf( 0.0f, fminf( 1.0f, x ) ); }
LH2_DEV float sqrf( float x ) { return x * x; }
LH2_DEV float mixf( float a, float b, float x ) { return x <= 0 ? a : x >= 1 ? b : lerpf_( a, b, x ); }
LH2_DEV float clampf_( float f, float a, float b ) { return fmaxf( a, fminf( f, b ) ); }
LH2_DEV v3 xyz( float4 a ) { return mk3( a.x, a.y, a.z ); }
LH2_DEV uint32_t fbits( float f ) { return __float_as_uint( f ); }
LH2_DEV float bitsf( uint32_t u ) { return __uint_as_float( u ); }
LH2_DEV bool isfinite_( float x ) { return x == x && x - x == 0.0f; }
